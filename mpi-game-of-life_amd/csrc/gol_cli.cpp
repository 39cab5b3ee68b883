// gol_cli.cpp -- the reference program's surface on top of libgol.so.
//
// Mirrors main() of Parallel_Life_MPI.cpp:190-240:
//   * reads `h w epochs` from grid_size_data.txt (:201-209) and the h lines of
//     data.txt (:56-102) from the working directory (or --dir);
//   * advances `epochs` generations on the GPU (:215-221);
//   * writes output.txt (:147-188) without truncating it (the reference opens it
//     with MPI_MODE_WRONLY|MPI_MODE_CREATE, :170), at the same offsets;
//   * prints "Process r wrote data to the file." per rank (:179) and
//     "Total time = X" (:236), X being wall seconds including I/O (:199, :233).
//
// --ref-ranks P reproduces `mpirun -np P` byte for byte (GOL_SEM_REF_STRIPES:
// the reference's halo exchange is a no-op, so its output depends on P).
// Without it the field evolves as one domain (== the reference at -np 1).
// --gpus G splits that domain into G row stripes on devices 0..G-1 of this
// process with k-deep halo rounds over xGMI peer copies (gol_create_group);
// --stripes S runs S stripes round-robin on the G devices (S >= G).
//
// Deviation: where the reference prints an error and continues with
// uninitialised values (:206) or an unopened file (:186), this program exits
// with status 1.
#include <fcntl.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/gol.h"

namespace {

bool parse_rule(const std::string& s, uint32_t* b, uint32_t* sv)
{
    if (s == "ref") {
        *b = GOL_REF_BIRTH;
        *sv = GOL_REF_SURVIVE;
        return true;
    }
    if (s == "conway") {
        *b = GOL_CONWAY_BIRTH;
        *sv = GOL_CONWAY_SURVIVE;
        return true;
    }
    // "B<digits>/S<digits>"
    if (s.size() < 3 || (s[0] != 'B' && s[0] != 'b')) return false;
    size_t slash = s.find('/');
    if (slash == std::string::npos || slash + 1 >= s.size() ||
        (s[slash + 1] != 'S' && s[slash + 1] != 's'))
        return false;
    uint32_t bm = 0, sm = 0;
    for (size_t i = 1; i < slash; ++i) {
        if (s[i] < '0' || s[i] > '8') return false;
        bm |= 1u << (s[i] - '0');
    }
    for (size_t i = slash + 2; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '8') return false;
        sm |= 1u << (s[i] - '0');
    }
    *b = bm;
    *sv = sm;
    return true;
}

void usage()
{
    std::cerr << "usage: gol [--dir DIR] [--ref-ranks P] [--rule ref|conway|B3/S23]\n"
                 "           [--tb-depth K] [--rows-per-wave N] [--device D]\n"
                 "           [--gpus G] [--stripes S] [--halo-depth H]\n"
                 "Reads grid_size_data.txt and data.txt, writes output.txt.\n";
}

bool read_file(const std::string& path, size_t need, std::vector<char>& out)
{
    int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    out.resize(need);
    size_t got = 0;
    while (got < need) {
        ssize_t n = ::pread(fd, out.data() + got, need - got, (off_t)got);
        if (n <= 0) break;
        got += (size_t)n;
    }
    ::close(fd);
    return got == need;
}

}  // namespace

int main(int argc, char** argv)
{
    const auto t0 = std::chrono::steady_clock::now();  // MPI_Wtime() at :199
    std::string dir = ".";
    int gpus = 0, stripes = 0;
    gol_config cfg;
    gol_config_init(&cfg);
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) {
                usage();
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "--dir") dir = next();
        else if (a == "--ref-ranks") {
            cfg.ref_ranks = (uint32_t)std::strtoul(next().c_str(), nullptr, 10);
            cfg.semantics = GOL_SEM_REF_STRIPES;
        } else if (a == "--rule") {
            if (!parse_rule(next(), &cfg.birth_mask, &cfg.survive_mask)) {
                std::cerr << "bad rule\n";
                return 2;
            }
        } else if (a == "--tb-depth") cfg.tb_depth = (uint32_t)std::strtoul(next().c_str(), nullptr, 10);
        else if (a == "--rows-per-wave") cfg.rows_per_wave = (uint32_t)std::strtoul(next().c_str(), nullptr, 10);
        else if (a == "--device") cfg.device = (int32_t)std::strtol(next().c_str(), nullptr, 10);
        else if (a == "--gpus") gpus = (int)std::strtol(next().c_str(), nullptr, 10);
        else if (a == "--stripes") stripes = (int)std::strtol(next().c_str(), nullptr, 10);
        else if (a == "--halo-depth") cfg.halo_depth = (uint32_t)std::strtoul(next().c_str(), nullptr, 10);
        else if (a == "-h" || a == "--help") {
            usage();
            return 0;
        } else {
            usage();
            return 2;
        }
    }

    long long h = 0, w = 0, epochs = 0;
    {
        std::ifstream gs(dir + "/grid_size_data.txt");
        if (!(gs >> h >> w >> epochs)) {
            std::cerr << "Error reading integers from file." << std::endl;  // :206
            return 1;
        }
    }
    if (h <= 0 || w <= 0 || epochs < 0) {
        std::cerr << "Invalid grid size or epoch count." << std::endl;
        return 1;
    }
    const uint32_t P = cfg.semantics == GOL_SEM_REF_STRIPES ? cfg.ref_ranks : 1;
    if (P == 0 || (uint64_t)h / P == 0) {
        std::cerr << "Need 1 <= ranks <= rows." << std::endl;
        return 1;
    }
    const size_t bytes = (size_t)h * (size_t)(w + 1);
    std::vector<char> data;
    if (!read_file(dir + "/data.txt", bytes, data)) {
        std::cerr << "Error reading data.txt (need " << bytes << " bytes)." << std::endl;
        return 1;
    }

    std::vector<char> out(bytes);
    if (gpus > 0 || stripes > 0) {
        if (cfg.semantics != GOL_SEM_GLOBAL) {
            std::cerr << "--gpus/--stripes evolve one global field; drop --ref-ranks" << std::endl;
            return 1;
        }
        if (gpus <= 0) gpus = 1;
        if (stripes <= 0) stripes = gpus;
        if ((uint64_t)h / (uint64_t)stripes == 0) {
            std::cerr << "Need 1 <= stripes <= rows." << std::endl;
            return 1;
        }
    }
    if (epochs == 0) {
        // zero generations: the reference writes the input bytes back (:157-164)
        out = data;
    } else if (stripes > 0) {
        std::vector<gol_engine*> es((size_t)stripes, nullptr);
        std::vector<int> devs((size_t)stripes);
        for (int r = 0; r < stripes; ++r) devs[(size_t)r] = r % gpus;
        gol_status st = gol_create_group((uint64_t)h, (uint64_t)w, &cfg, stripes, devs.data(),
                                         es.data());
        for (int r = 0; r < stripes && st == GOL_OK; ++r) {
            uint64_t r0 = 0, n = 0;
            gol_rank_rows((uint64_t)h, stripes, r, &r0, &n);
            st = gol_load_ascii(es[(size_t)r], data.data() + r0 * (uint64_t)(w + 1),
                                n * (uint64_t)(w + 1));
        }
        if (st == GOL_OK) st = gol_group_step(es.data(), stripes, (uint64_t)epochs);
        for (int r = 0; r < stripes && st == GOL_OK; ++r) {
            uint64_t r0 = 0, n = 0;
            gol_rank_rows((uint64_t)h, stripes, r, &r0, &n);
            st = gol_store_ascii(es[(size_t)r], out.data() + r0 * (uint64_t)(w + 1),
                                 n * (uint64_t)(w + 1));
        }
        if (st != GOL_OK) std::cerr << "gol error " << (int)st << ": " << gol_last_error() << std::endl;
        for (auto* e : es) gol_destroy(e);
        if (st != GOL_OK) return 1;
    } else {
        gol_engine* e = nullptr;
        gol_status st = gol_create((uint64_t)h, (uint64_t)w, &cfg, &e);
        if (st == GOL_OK) st = gol_load_ascii(e, data.data(), data.size());
        if (st == GOL_OK) st = gol_step(e, (uint64_t)epochs);
        if (st == GOL_OK) st = gol_sync(e);
        if (st == GOL_OK) st = gol_store_ascii(e, out.data(), out.size());
        if (st != GOL_OK) {
            std::cerr << "gol error " << (int)st << ": " << gol_last_error() << std::endl;
            gol_destroy(e);
            return 1;
        }
        gol_destroy(e);
    }

    // writeDataToFile (:166-183): create if missing, never truncate, each rank's
    // rows at r*(h/P)*(w+1); together they cover [0, h*(w+1)).
    int fd = ::open((dir + "/output.txt").c_str(), O_WRONLY | O_CREAT, 0666);
    if (fd < 0) {
        std::cerr << "Error opening the file for writing." << std::endl;  // :186
        return 1;
    }
    const size_t chunk = (size_t)(h / P) * (size_t)(w + 1);
    for (uint32_t r = 0; r < P; ++r) {
        const size_t off = (size_t)r * chunk;
        const size_t len = (r == P - 1) ? bytes - off : chunk;
        size_t done = 0;
        while (done < len) {
            ssize_t n = ::pwrite(fd, out.data() + off + done, len - done, (off_t)(off + done));
            if (n <= 0) {
                std::cerr << "Error writing output.txt." << std::endl;
                ::close(fd);
                return 1;
            }
            done += (size_t)n;
        }
        std::cout << "Process " << r << " wrote data to the file." << std::endl;  // :179
    }
    ::close(fd);

    const double secs =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::cout << "Total time = " << secs << std::endl;  // :236
    return 0;
}
