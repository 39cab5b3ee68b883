// gol_mpi_cli.cpp -- `gol-mpi`: the reference's multi-process launch shape
// (`mpirun -np P ./life`, Parallel_Life_MPI.cpp:190-240) on top of libgol.so,
// one MPI process per GPU, for runs that span several nodes.
//
// Halo transport (--transport):
//   rccl (default): MPI only bootstraps and orders -- MPI_Init (:195), rank/size
//     (:196-197), a broadcast of the RCCL unique id from rank 0, and the barrier
//     before the timing line; halos move over RCCL inside the engine
//     (gol_create_rank: k-deep send/recv rounds over xGMI / the node
//     interconnect).  One GPU per rank (RCCL refuses two ranks on one device).
//   mpi: the engine stages each round's Hx boundary rows through host memory and
//     this launcher moves them with MPI_Sendrecv (gol_create_rank_transport) --
//     the reference's exchangeGridData (:104-145) with the receive landing in the
//     halo, Hx rows every Hx generations instead of 1 row every generation.  Any
//     number of ranks may share a GPU.
// --dry-run reads the config and prints each rank's partition and schedule
// (gol_rank_rows, gol_round_schedule) without touching a GPU.
//
// Each rank reads only its own rows of data.txt (fixed stride w+1, so a pread
// at row0*(w+1)), advances them as part of ONE global field (GOL_SEM_GLOBAL ==
// the reference at -np 1; for the reference's P-dependent output use
// `gol --ref-ranks P`), and writes them back into output.txt at the same
// offset without truncating it (:166-183).  Stdout: "Process r wrote data to
// the file." per rank (:179) and, on rank 0, "Total time = X" (:233-237).
//
// Device: rank r uses local device (local rank % visible devices); the local
// rank comes from MPI_LOCALRANKID (MPICH/hydra) or OMPI_COMM_WORLD_LOCAL_RANK.
#include <fcntl.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>
#include <mpi.h>

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/gol.h"

namespace {

int local_rank(int rank)
{
    for (const char* k : {"MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "LOCAL_RANK"})
        if (const char* v = std::getenv(k)) return std::atoi(v);
    return rank;
}

bool pread_all(int fd, char* dst, size_t len, off_t off)
{
    size_t got = 0;
    while (got < len) {
        ssize_t n = ::pread(fd, dst + got, len - got, off + (off_t)got);
        if (n <= 0) return false;
        got += (size_t)n;
    }
    return true;
}

bool pwrite_all(int fd, const char* src, size_t len, off_t off)
{
    size_t done = 0;
    while (done < len) {
        ssize_t n = ::pwrite(fd, src + done, len - done, off + (off_t)done);
        if (n <= 0) return false;
        done += (size_t)n;
    }
    return true;
}

int fail_all(int rank, const std::string& msg)
{
    std::cerr << "rank " << rank << ": " << msg << std::endl;
    MPI_Abort(MPI_COMM_WORLD, 1);
    return 1;
}

// gol_transport over MPI: boundary rows to/from rank-1 and rank+1 (Sendrecv with
// both neighbours at once, so no ordering between ranks is needed).
struct MpiXfer {
    int rank, size;
};

int mpi_exchange(void* ctx, const void* send_up, void* recv_up, const void* send_dn,
                 void* recv_dn, uint64_t bytes)
{
    const MpiXfer* x = static_cast<const MpiXfer*>(ctx);
    if (bytes > (uint64_t)INT_MAX) return 3;
    const int n = (int)bytes;
    MPI_Request req[4];
    int k = 0;
    if (send_up) {
        MPI_Irecv(recv_up, n, MPI_BYTE, x->rank - 1, 1, MPI_COMM_WORLD, &req[k++]);
        MPI_Isend(send_up, n, MPI_BYTE, x->rank - 1, 0, MPI_COMM_WORLD, &req[k++]);
    }
    if (send_dn) {
        MPI_Irecv(recv_dn, n, MPI_BYTE, x->rank + 1, 0, MPI_COMM_WORLD, &req[k++]);
        MPI_Isend(send_dn, n, MPI_BYTE, x->rank + 1, 1, MPI_COMM_WORLD, &req[k++]);
    }
    return MPI_Waitall(k, req, MPI_STATUSES_IGNORE) == MPI_SUCCESS ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv)
{
    MPI_Init(&argc, &argv);  // :195
    int rank = 0, size = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);  // :196
    MPI_Comm_size(MPI_COMM_WORLD, &size);  // :197
    const double t0 = MPI_Wtime();         // :199

    std::string dir = ".", transport = "rccl";
    bool dry_run = false;
    gol_config cfg;
    gol_config_init(&cfg);
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--dry-run") {
            dry_run = true;
            continue;
        }
        if (i + 1 >= argc && a != "-h" && a != "--help") return fail_all(rank, "missing value for " + a);
        if (a == "--dir") dir = argv[++i];
        else if (a == "--transport") {
            transport = argv[++i];
            if (transport != "rccl" && transport != "mpi")
                return fail_all(rank, "--transport must be rccl or mpi");
        }
        else if (a == "--tb-depth") cfg.tb_depth = (uint32_t)std::strtoul(argv[++i], nullptr, 10);
        else if (a == "--halo-depth") cfg.halo_depth = (uint32_t)std::strtoul(argv[++i], nullptr, 10);
        else if (a == "--rule") {
            std::string r = argv[++i];
            if (r == "conway") {
                cfg.birth_mask = GOL_CONWAY_BIRTH;
                cfg.survive_mask = GOL_CONWAY_SURVIVE;
            } else if (r != "ref") {
                return fail_all(rank, "--rule must be ref or conway");
            }
        } else {
            if (rank == 0)
                std::cerr << "usage: mpirun -np P gol-mpi [--dir DIR] [--rule ref|conway]\n"
                             "           [--tb-depth K] [--halo-depth H] [--transport rccl|mpi]\n"
                             "           [--dry-run]\n";
            MPI_Finalize();
            return (a == "-h" || a == "--help") ? 0 : 2;
        }
    }

    long long h = 0, w = 0, epochs = 0;
    {
        std::ifstream gs(dir + "/grid_size_data.txt");  // :201-209, every rank
        if (!(gs >> h >> w >> epochs)) return fail_all(rank, "Error reading integers from file.");
    }
    if (h <= 0 || w <= 0 || epochs < 0 || h < size)
        return fail_all(rank, "invalid grid size, epoch count or rank count");

    uint64_t row0 = 0, rows = 0;
    gol_rank_rows((uint64_t)h, size, rank, &row0, &rows);
    const size_t stride = (size_t)w + 1, len = (size_t)rows * stride;
    const off_t off = (off_t)(row0 * stride);

    if (dry_run) {  // partition and schedule only; no GPU, no files touched
        uint64_t nops = 0;
        uint32_t K = 0, Hx = 0;
        if (gol_round_schedule((uint64_t)h, (uint64_t)w, &cfg, rank, size, (uint64_t)epochs, 0,
                               nullptr, 0, &nops, &K, &Hx) != GOL_OK)
            return fail_all(rank, gol_last_error());
        std::printf("rank %d/%d: rows [%llu, %llu) offset %lld K %u halo %u ops %llu transport %s\n",
                    rank, size, (unsigned long long)row0, (unsigned long long)(row0 + rows),
                    (long long)off, K, Hx, (unsigned long long)nops, transport.c_str());
        std::fflush(stdout);
        MPI_Finalize();
        return 0;
    }

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail_all(rank, "no HIP device");
    cfg.device = local_rank(rank) % ndev;
    {
        // more ranks on this node than devices: ranks share GPUs, and hand-off row
        // blocks are kept to one launch per device at a time (engine.cpp
        // gol_create_group), so ranks that share one use classic blocks
        MPI_Comm node;
        int node_size = 1;
        if (MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node) ==
            MPI_SUCCESS) {
            MPI_Comm_size(node, &node_size);
            MPI_Comm_free(&node);
        }
        if (node_size > ndev) cfg.handoff = 1;
    }

    uint8_t uid[128] = {};
    if (transport == "rccl") {
        if (rank == 0 && gol_comm_unique_id(uid) != GOL_OK) return fail_all(rank, gol_last_error());
        MPI_Bcast(uid, 128, MPI_BYTE, 0, MPI_COMM_WORLD);
    }
    MpiXfer xfer{rank, size};
    const gol_transport tp{mpi_exchange, &xfer};
    std::vector<char> buf(len);
    {
        int fd = ::open((dir + "/data.txt").c_str(), O_RDONLY);
        if (fd < 0 || !pread_all(fd, buf.data(), len, off)) {
            if (fd >= 0) ::close(fd);
            return fail_all(rank, "Error reading data.txt");
        }
        ::close(fd);
    }

    if (epochs > 0) {
        gol_engine* e = nullptr;
        gol_status st = transport == "rccl"
                            ? gol_create_rank((uint64_t)h, (uint64_t)w, &cfg, rank, size, uid, &e)
                            : gol_create_rank_transport((uint64_t)h, (uint64_t)w, &cfg, rank, size,
                                                        &tp, &e);
        if (st == GOL_OK) st = gol_load_ascii(e, buf.data(), len);
        if (st == GOL_OK) st = gol_step(e, (uint64_t)epochs);  // :215-221
        if (st == GOL_OK) st = gol_sync(e);
        if (st == GOL_OK) st = gol_store_ascii(e, buf.data(), len);
        if (st != GOL_OK) {
            std::string msg = gol_last_error();
            gol_destroy(e);
            return fail_all(rank, "gol error " + std::to_string((int)st) + ": " + msg);
        }
        gol_destroy(e);
    }

    // writeDataToFile (:166-183): create if missing, never truncate
    int fd = ::open((dir + "/output.txt").c_str(), O_WRONLY | O_CREAT, 0666);
    if (fd < 0) return fail_all(rank, "Error opening the file for writing.");
    const bool ok = pwrite_all(fd, buf.data(), len, off);
    ::close(fd);
    if (!ok) return fail_all(rank, "Error writing output.txt");
    std::cout << "Process " << rank << " wrote data to the file." << std::endl;  // :179

    MPI_Barrier(MPI_COMM_WORLD);
    if (rank == 0) std::cout << "Total time = " << MPI_Wtime() - t0 << std::endl;  // :233-237
    MPI_Finalize();
    return 0;
}
