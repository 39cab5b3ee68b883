/*
 * gol.h -- C ABI of the MI355X Game of Life engine (libgol.so).
 *
 * Drop-in boundary for the hot path of krutovsky-danya/mpi-game-of-life,
 * Parallel_Life_MPI.cpp.  The reference has no plugin API: its hot path is
 * `void updateGrid()` (:37-54, with countNeighbours :16-35) mutating the
 * process globals `grid`/`nextGrid` (:13), driven by the loop in main
 * (:215-221) together with `exchangeGridData` (:104-145), and fed/drained by
 * readGridFromFile (:56-102) and writeDataToFile (:147-188).  This header
 * replaces main's lines :211-231 (read -> epochs x {update, exchange, barrier}
 * -> write) with an engine handle; each entry point names the reference code
 * it stands in for.
 *
 * Conventions
 *  - Cells: bit-packed, 64 per uint64, row-major; bit j of word q is column 64q+j.
 *    Columns >= w are kept 0.  Outside the field every cell is dead
 *    (Parallel_Life_MPI.cpp:21-27).
 *  - Rule: a (birth, survive) pair of 9-bit masks, bit n <=> n live neighbours.
 *    The reference's *effective* rule is birth=0, survive=1<<2 ("B/S2"): the
 *    `count == 3` store at :44-46 is always overwritten by :47-50.
 *  - Ownership: the caller owns every host buffer; the engine owns all device
 *    memory, its HIP stream and its RCCL communicator.
 *  - Errors: every call returns gol_status; it never aborts.  gol_last_error()
 *    gives a thread-local message for the last failure.
 *  - Threading: a handle is not thread-safe; use it from one host thread.
 */
#ifndef GOL_H
#define GOL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum gol_status {
    GOL_OK = 0,
    GOL_EINVAL = 1, /* bad argument (sizes, masks, lengths, malformed ASCII) */
    GOL_ENOMEM = 2, /* device or host allocation failed */
    GOL_EHIP = 3,   /* HIP runtime error */
    GOL_ERCCL = 4,  /* RCCL error */
    GOL_EIO = 5,    /* file I/O error (CLI helpers) */
    GOL_ESTATE = 6, /* call not valid in the engine's current state */
    GOL_EXFER = 7   /* halo transport callback failed (gol_create_rank_transport) */
} gol_status;

typedef enum gol_semantics {
    /* The reference's intended semantics == its `mpirun -np 1` output: one field
     * evolving with a dead border. */
    GOL_SEM_GLOBAL = 0,
    /* The reference's actual `mpirun -np P` output: its halo exchange receives
     * into copies (:110-111, :126-127) and has no effect, so each rank's
     * extended stripe (:70-81) evolves alone and the output keeps each rank's
     * own rows (:149-175).  P = gol_config.ref_ranks. */
    GOL_SEM_REF_STRIPES = 1
} gol_semantics;

/* Reference-effective rule and Conway's rule as (birth, survive) masks. */
#define GOL_REF_BIRTH 0u
#define GOL_REF_SURVIVE (1u << 2)
#define GOL_CONWAY_BIRTH (1u << 3)
#define GOL_CONWAY_SURVIVE ((1u << 2) | (1u << 3))

typedef struct gol_config {
    uint32_t birth_mask;   /* 9-bit */
    uint32_t survive_mask; /* 9-bit */
    int32_t device;        /* HIP device ordinal; -1 = current device */
    uint32_t semantics;    /* gol_semantics */
    uint32_t ref_ranks;    /* P for GOL_SEM_REF_STRIPES (must satisfy h >= P) */
    uint32_t tb_depth;     /* generations fused per kernel launch (temporal
                              blocking); 0 = auto; allowed 1,2,4,6,7,8,12,16
                              (the dev build, make dev, adds 20,24,32); with
                              resident = 2, the resident kernel's epoch length,
                              any of 1..63 */
    uint32_t halo_depth;   /* multi-rank: halo rows exchanged per round
                              (= generations between exchanges); 0 = auto */
    uint32_t rows_per_wave;/* rows each wavefront streams per launch; 0 = auto */
    uint32_t handoff;      /* row blocks of a launch: 0 = auto (= on), 1 = off
                              (every block recomputes the K(K-1) stage-steps of
                              its vertical halo), 2 = on (each block takes the
                              rows it needs beyond its own from the block below,
                              which computed them first; tb_depth >= 4) */
    uint32_t streams;      /* gol_create, GLOBAL only: split the field into this
                              many row stripes advanced on their own streams of
                              the device (k-deep halos, device copies), so one
                              stripe's launch tail overlaps the others' work;
                              0 = auto (2 when h >= 32768), 1 = one stream */
    uint32_t strip_lanes;  /* lanes per column strip of the stencil kernel: 64, 32
                              or 16 (2 of them halo, 64/L strips per wavefront);
                              0 = auto (narrow strips for short stripes) */
    uint32_t word_planes;  /* cell planes per lane: 0 = auto (= 2: one word = 64
                              columns per lane); 4 (two words per lane) exists
                              only in the dev build (make dev) */
    uint32_t resident;     /* gol_create, GLOBAL only: small fields held in
                              registers across the chip and advanced by ONE
                              launch per gol_step (tiles swap halo rows every K
                              generations inside the launch); 0 = auto (when the
                              field fits and no streaming-kernel knob --
                              tb_depth, rows_per_wave, handoff, strip_lanes,
                              word_planes -- is set), 1 = off, 2 = on if the
                              field fits (then tb_depth sets K and rows_per_wave
                              the rows each wavefront holds: 2,3,4,6,8) */
    uint32_t exchange_overlap; /* rank engines and groups: 0 = auto (rank engines
                              over RCCL time both modes at create on their
                              communicator and keep the faster, the same on
                              every rank: gol_plan_exchange; rank engines over a
                              host transport block; in-process groups overlap),
                              1 = blocking, 2 =
                              overlapped (the round's last launch splits into a
                              band launch of the rows the neighbours need and an
                              interior launch, and the exchange of the band rows
                              runs on a side stream beside the interior launch;
                              needs stripes of >= 2 halo_depth rows, else
                              blocking) */
} gol_config;

typedef struct gol_engine gol_engine;

typedef struct gol_timing {
    uint64_t launches;     /* stencil kernel launches timed (sampled) */
    double kernel_ms;      /* sum of their HIP-event durations */
    double cell_gens;      /* cell-generations those launches produced (own rows) */
    double cell_gens_computed; /* what the lanes process: including the vertical
                                  halo stage-rows of classic blocks and the
                                  strips' halo lanes */
    uint32_t streams;      /* stripe streams whose launches run concurrently */
    /* (r06; `reserved` before) in: the caller's sizeof(gol_timing).  The layout
     * grew in r05 and r06; gol_get_timing writes the whole struct only when this
     * equals the library's sizeof(gol_timing), else only the r04 fields above
     * (40 bytes), so a caller built against an older header is never overrun.
     * out: the bytes written. */
    uint32_t struct_size;
    /* (r05) while timing is on: every stencil launch issued (sampled or not) and
     * the buffer rows the sampled launches computed; rank engines also time
     * every halo exchange with HIP events on its stream (RCCL: the stream time
     * of ncclGroupStart..End, which includes waiting for the peers; host
     * transport: staging + callback) */
    uint64_t launches_issued;
    double launch_rows;
    uint64_t exchanges;
    double exchange_ms;
    /* (r06) rank engines while timing is on: `rounds` halo rounds, round_ms = the
     * sum of their compute-stream spans (HIP events before the round's first
     * launch and after its last, the band stream joined), exchange_exposed_ms =
     * the part of the exchanges outside those spans (a blocking exchange: all of
     * it; an overlapped one: what runs past the end of its round's span).  Per
     * step: round_ms + exchange_exposed_ms <= the wall time; the rest is host
     * work and launch gaps between rounds. */
    uint64_t rounds;
    double round_ms;
    double exchange_exposed_ms;
} gol_timing;
#define GOL_TIMING_R04_BYTES 40u

/* Defaults: reference-effective rule, GLOBAL semantics, auto tuning. */
void gol_config_init(gol_config* cfg);

/* Replaces the allocation in readGridFromFile (:88-89).  h rows x w columns.
 * An engine alone on its device times a few equally exact launch plans on its
 * own buffers before returning (tens of ms) and keeps the fastest. */
gol_status gol_create(uint64_t h, uint64_t w, const gol_config* cfg, gol_engine** out);

/* Replaces readGridFromFile's parse (:91-99): buf holds the data.txt bytes,
 * h lines of exactly w cell bytes followed by '\n' (len == h*(w+1)); a cell is
 * alive iff its byte is '1'.  A rank engine (gol_create_rank) takes only its
 * own rows: len == rows*(w+1). */
gol_status gol_load_ascii(gol_engine* e, const char* buf, size_t len);

/* Replaces writeDataToFile's serialisation (:157-164): writes '0'/'1' bytes and
 * '\n' per row, len == h*(w+1) (own rows for a rank engine). */
gol_status gol_store_ascii(gol_engine* e, char* buf, size_t len);

/* Packed transfer; row_stride_words >= ceil(w/64).  Rank engines: own rows. */
gol_status gol_load_packed(gol_engine* e, const uint64_t* words, uint64_t row_stride_words);
gol_status gol_store_packed(gol_engine* e, uint64_t* words, uint64_t row_stride_words);

/* Synthetic p = 0.5 field generated on the device: word (r, q) =
 * splitmix64(seed, r*ceil(w/64)+q) masked to w (identical on the CPU oracle). */
gol_status gol_init_random(gol_engine* e, uint64_t seed);

/* Replaces the epoch loop (:215-221): advances `generations` generations
 * (including the halo exchange of a rank engine).  Returns after the work is
 * enqueued; gol_sync() waits for it. */
gol_status gol_step(gol_engine* e, uint64_t generations);
gol_status gol_sync(gol_engine* e);

/* Live-cell count and an order-independent 64-bit hash of the field
 * (sum over words of splitmix64(word ^ splitmix64(0, r*ceil(w/64)+q))).
 * Rank engines return the partial sums of their own rows (add them up). */
gol_status gol_digest(gol_engine* e, uint64_t* live, uint64_t* hash);

void gol_destroy(gol_engine* e);
const char* gol_last_error(void);

/* HIP-event timing of the stencil kernel on the engine's stream: events bracket
 * every `every`-th launch (1 = all; 0 = off).  An event pair costs a few
 * microseconds of stream time, so sample short launches (bench.py uses 8).
 * gol_timing then covers the sampled launches only. */
gol_status gol_set_timing(gol_engine* e, int every);
gol_status gol_get_timing(gol_engine* e, gol_timing* out);
gol_status gol_reset_timing(gol_engine* e);

/* Engine geometry as chosen (for tools / tests); any out pointer may be NULL.
 * rows_per_wave: the rows each wavefront streams in a full-depth launch. */
gol_status gol_info(gol_engine* e, uint64_t* h, uint64_t* w, uint64_t* row0,
                    uint64_t* rows, uint32_t* tb_depth, uint32_t* halo_depth,
                    uint32_t* rows_per_wave);

/* Launch plan of a full-depth launch as chosen (strip width in lanes, rows per
 * wavefront, planes per lane); with age-skewed blocks the rows per wavefront are
 * the shorter (young) length, gol_plan_skew gives both.  A composite engine
 * reports its first stripe's plan.  Any out pointer may be NULL. */
gol_status gol_plan_info(gol_engine* e, uint32_t* strip_lanes, uint32_t* rows_per_wave,
                         uint32_t* word_planes);

/* (r06) Resident plan details: rows per wavefront, band rows per tile, epoch
 * length K (generations between the tiles' swaps through memory), and
 * *swap_every: the generations between the wavefronts' row swaps through LDS
 * inside a tile (1 = every generation, life_res_kernel; >= 2 = the wave-level
 * temporal blocking of life_resident_mb.hip).  All 0 when the engine does not run
 * the resident kernel.  Out pointers may be NULL. */
gol_status gol_plan_resident_rows(gol_engine* e, uint32_t* rows, uint32_t* band_rows,
                                  uint32_t* epoch, uint32_t* swap_every);

/* Whether full-depth launches use hand-off row blocks (gol_config.handoff, as
 * the planner resolved it): 1 = yes, 0 = every block recomputes its halo. */
gol_status gol_plan_handoff(gol_engine* e, uint32_t* handoff);

/* Age-skewed row blocks of full-depth launches (a one-round launch at 2
 * wavefronts per SIMD: the units dispatched first win their SIMD's VALU
 * arbitration and get longer blocks): *rows_old rows for the first *units_old
 * units' blocks, *rows_young for the others; all 0 when the launches use equal
 * blocks.  A composite engine reports its first stripe (which never skews: its
 * stripes share the device).  Out pointers may be NULL. */
gol_status gol_plan_skew(gol_engine* e, uint32_t* rows_old, uint32_t* rows_young,
                         uint32_t* units_old);

/* Column layout of full-depth launches: *strips wavefront strips per row block
 * and the packed half strip's units (64-lane strips of a one-segment launch: the
 * last strip ends at the field's right edge and the gap of <= 30 lane groups
 * before it runs 32 lanes wide, two row blocks per wavefront): *half_units
 * wavefronts over *half_groups lane groups (both 0 without one).  A resident or
 * composite engine reports its first stripe / 0.  Out pointers may be NULL. */
gol_status gol_plan_columns(gol_engine* e, uint32_t* strips, uint32_t* half_units,
                            uint32_t* half_groups);

/* Resident plan (gol_config.resident): *on = 1 if gol_step runs the resident
 * kernel; then *bands x *strips tiles, one workgroup each (bands, strips may be
 * NULL).  A composite engine reports 0. */
gol_status gol_plan_resident(gol_engine* e, uint32_t* on, uint32_t* bands, uint32_t* strips);

/* The plan autotuner's outcome for the first full-depth launch plan (an engine
 * alone on its device times a few variants of the cost models' plan at create
 * and keeps one only if it is >= 3% faster): *variant 0 = the models' plan, else
 * 1 + the index in {no_half_strip, skew_0.95, skew_1.05, other_block_kind};
 * *tuned_us / *model_us = the best create-time launch of the plan that runs / of
 * the models' plan (0 when nothing was timed).  Out pointers may be NULL. */
gol_status gol_plan_tuning(gol_engine* e, uint32_t* variant, float* tuned_us, float* model_us);

/* (late r06) Exchange mode of a stripe engine: *mode = 1 blocking (the exchange after
 * the round's last launch), 2 overlapped (band launch, then the exchange beside
 * the interior launch), 0 for an engine without halo exchanges.  With
 * exchange_overlap = 0 a rank engine over RCCL chooses it at create by timing
 * rounds of both modes on its communicator (a collective: every rank of the job
 * runs the same rounds); *blocking_ms / *overlapped_ms are then the max over ranks
 * of each mode's best time per round, else 0.  gol_round_schedule called with
 * exchange_overlap set to *mode lists what gol_step runs.  Out pointers may be
 * NULL. */
gol_status gol_plan_exchange(gol_engine* e, uint32_t* mode, float* blocking_ms,
                             float* overlapped_ms);

/* Passes per full-depth launch of the first full-depth plan: 1, or 2-3 for
 * multi-pass launches (each launch runs that many depth-K passes over its row
 * blocks, alternating direction; dev switch GOL_DEV_PASSES at create, read only by
 * the dev build, libgol_dev.so: the shipped library has no multi-pass kernel
 * since r06 and always reports 1). */
gol_status gol_plan_passes(gol_engine* e, uint32_t* passes);

/* gol_digest restricted to field rows [row0, row0 + rows) (for a rank engine:
 * the part of its own rows inside that range).  Lets one engine of the whole
 * field check each rank's stripe separately. */
gol_status gol_digest_rows(gol_engine* e, uint64_t row0, uint64_t rows, uint64_t* live,
                           uint64_t* hash);

/* ---- Multi-GPU, one process per GPU (replaces the MPI stripes :70-81 and the
 * halo exchange :104-145 with RCCL send/recv over xGMI) ---- */

/* Rows of global stripe `rank` of `nranks`: contiguous, ceil-balanced.
 * Host-only; needs no GPU. */
gol_status gol_rank_rows(uint64_t h, int nranks, int rank, uint64_t* row0, uint64_t* rows);

/* Generate an RCCL unique id on one rank; broadcast its 128 bytes to the
 * others by any means (torch.distributed, a file, MPI). */
gol_status gol_comm_unique_id(uint8_t id[128]);

/* Engine for stripe `rank` of `nranks` of an h x w GLOBAL field; all ranks call
 * it collectively with the same id.  cfg->semantics must be GLOBAL. */
gol_status gol_create_rank(uint64_t h, uint64_t w, const gol_config* cfg, int rank,
                           int nranks, const uint8_t id[128], gol_engine** out);

/* The RCCL communicator of a gol_create_rank engine as RCCL reports it
 * (ncclCommCount, ncclCommUserRank, ncclCommCuDevice) and the engine's up/down
 * peers (-1: no such neighbour).  Out pointers may be NULL.  GOL_ESTATE for an
 * engine without a communicator. */
gol_status gol_comm_info(gol_engine* e, int* count, int* rank, int* peer_up, int* peer_down,
                         int* device);

/* Halo transport supplied by the caller (host memory): the same rank engine,
 * partition and rounds as gol_create_rank, but each exchange stages the Hx
 * boundary rows through host buffers and calls `exchange`, which must send
 * send_up to rank-1 and send_down to rank+1 and receive recv_up from rank-1 and
 * recv_down from rank+1, `bytes` each (NULL pointers where there is no such
 * neighbour), and return 0 on success.  This is the reference's own transport
 * shape (MPI_Sendrecv of boundary rows, Parallel_Life_MPI.cpp:104-145, here with
 * the receive landing in the halo); gol-mpi --transport mpi uses it, and it lets
 * several ranks share one GPU, which RCCL refuses. */
typedef int (*gol_halo_exchange_fn)(void* ctx, const void* send_up, void* recv_up,
                                    const void* send_down, void* recv_down, uint64_t bytes);
typedef struct gol_transport {
    gol_halo_exchange_fn exchange;
    void* ctx;
} gol_transport;
gol_status gol_create_rank_transport(uint64_t h, uint64_t w, const gol_config* cfg, int rank,
                                     int nranks, const gol_transport* transport,
                                     gol_engine** out);

/* The launch/exchange schedule a rank engine (or group member) runs for one
 * gol_step(generations) call -- host-only, no GPU needed; gol_step executes
 * exactly this list.  halo_fresh: the previous call ended with an overlapped
 * exchange still to be waited for (0 after create/load).  Launch ops name the
 * local buffer rows they write (local row i = field row row0 - Hx + i).
 * Computed is not valid: since r04 every full-depth launch of a round writes
 * the first launch's region, so after a launch only the rows inside
 * [shrink, buf_rows - shrink) (buf_rows = own rows + 2 Hx, shrink = this op's
 * field) hold that generation; rows of [out_lo, out_hi) outside that range were
 * computed from rows that were no longer valid and must not be read (an external
 * transport moves only [Hx, 2 Hx) and [R, R + Hx) after a round's last launch,
 * which are always valid). */
typedef enum gol_sched_kind {
    GOL_OP_EXCHANGE = 0,       /* blocking halo exchange on the compute stream */
    GOL_OP_WAIT_EXCHANGE = 1,  /* compute waits for the overlapped exchange */
    GOL_OP_LAUNCH = 2,         /* stencil launch over the valid region */
    GOL_OP_BAND = 3,           /* last launch of a round, boundary rows only */
    GOL_OP_INTERIOR = 4,       /* ... and the rest of the own rows, concurrently */
    GOL_OP_EXCHANGE_ASYNC = 5  /* exchange of the band rows, overlapping INTERIOR */
} gol_sched_kind;
typedef struct gol_sched_op {
    uint32_t kind;      /* gol_sched_kind */
    uint32_t depth;     /* fused generations of a launch (0 otherwise) */
    uint32_t shrink;    /* halo rows consumed per side once this launch is done */
    uint32_t nseg;      /* row ranges a launch writes: [out_lo[i], out_hi[i]); valid
                           only inside [shrink, buf_rows - shrink), see above */
    int64_t out_lo[2];
    int64_t out_hi[2];
} gol_sched_op;
gol_status gol_round_schedule(uint64_t h, uint64_t w, const gol_config* cfg, int rank,
                              int nranks, uint64_t generations, int halo_fresh,
                              gol_sched_op* ops, uint64_t cap, uint64_t* nops,
                              uint32_t* tb_depth, uint32_t* halo_depth);

/* Host-only planning model (no GPU needed): the launch plans gol_create
 * (nranks = 1: a single-stream engine) or gol_create_rank (rank of nranks)
 * would build on a device of `cus` compute units whose stencil kernels fit
 * occ_classic (classic blocks) / occ_hand (hand-off blocks) 256-thread
 * workgroups per CU, as the occupancy query reports them, before the autotuner
 * times its candidates.  Summarises the first full-depth launch plan: what the
 * planner's tests check (tests/test_planner.py, also run under the host
 * sanitizers) and what tools print. */
typedef struct gol_plan_summary {
    uint32_t tb_depth, halo_depth;
    uint32_t plans, distinct_plans; /* launch plans built; aliases share one */
    int64_t rows_lo, rows_hi;       /* buffer rows the plan computes */
    int64_t rows_per_wave;          /* the block length (the young one when skewed) */
    int32_t rows_old, units_old;    /* age-skewed blocks: old length and units (0: none) */
    int32_t strips, lane_shift;     /* strips per row block, strip width 64 >> lane_shift */
    int64_t total_units;            /* wavefronts of the launch */
    int64_t half_units;             /* of which run the packed half strip */
    int64_t blocks;                 /* row blocks per strip (summed over segments) */
    int32_t handoff, tail_off;      /* hand-off blocks, their kernel's tail offset (-1) */
    uint32_t candidates;            /* autotuner variants built for this plan */
    uint32_t passes;                /* passes per full-depth launch (gol_plan_passes);
                                       always 1 with the shipped library (multi-pass
                                       kernels: dev build).  The model assumes the
                                       multi-pass kernels fit the same occupancies
                                       as the single-pass ones (their real occupancy
                                       may be lower, where the engine would then
                                       fall back to single-pass launches). */
} gol_plan_summary;
gol_status gol_plan_model(uint64_t h, uint64_t w, const gol_config* cfg, int rank, int nranks,
                          int cus, int occ_classic, int occ_hand, gol_plan_summary* out);

/* ---- Multi-GPU (or multi-stripe) inside ONE process, no RCCL ----
 * `nranks` stripe engines of one GLOBAL field (the same partition and halo
 * rounds as gol_create_rank), stripe r on devices[r] (NULL = cfg->device for
 * all; repeats allowed, so several stripes can share one GPU).  Halos move by
 * device-to-device / xGMI peer copies ordered with HIP events.  Members are
 * loaded, stored and digested one by one like rank engines, advanced together
 * by gol_group_step, and destroyed with gol_destroy. */
gol_status gol_create_group(uint64_t h, uint64_t w, const gol_config* cfg, int nranks,
                            const int* devices, gol_engine** engines);
gol_status gol_group_step(gol_engine** engines, int nranks, uint64_t generations);

#ifdef __cplusplus
}
#endif

#endif /* GOL_H */
