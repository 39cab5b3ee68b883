/*
 * gol_oracle.c -- CPU restatement of krutovsky-danya/mpi-game-of-life's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libgol.so, the `gol` CLI)
 * links or calls this file.  Only tests/, __graft_entry__.smoke() and the
 * `cpu_baseline` leg of bench.py may load it, and only as the checker / the timed
 * CPU port, never as the thing measured or shipped.
 *
 * Parity pinning: the reference itself is NOT buildable in this image (it
 * includes <windows.h> at Parallel_Life_MPI.cpp:6, a header the image lacks;
 * writing a stand-in is not allowed).  This restatement is pinned instead
 * against the outputs of the reference that SURVEY.md §4 records (sha256 of
 * output.txt for the shipped data.txt at -np 1/2/3/4/8 and generations 0..5, 100),
 * committed as tests/golden/ref_outputs.json, and against the shipped input
 * fixture data.txt / grid_size_data.txt.  See tests/test_oracle.py.
 *
 * Two restatements live here:
 *  (1) the scalar, int-per-cell program restatement (oracle_ref_*) that follows
 *      the reference line by line in *semantics* (rule, boundary, stripe
 *      decomposition, no-op halo exchange, output layout);
 *  (2) a bit-packed uint64 stepper (oracle_bp_*) with the same rule/boundary,
 *      multithreaded, used as the parity oracle at sizes (1) cannot reach.
 *      It is pinned against (1) in tests/test_oracle.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define LIVE_CELL '1' /* Parallel_Life_MPI.cpp:11 */
#define DEAD_CELL '0' /* Parallel_Life_MPI.cpp:10 */

/* ------------------------------------------------------------------------- */
/* (1) scalar restatement                                                    */
/* ------------------------------------------------------------------------- */

/* countNeighbours, Parallel_Life_MPI.cpp:16-35: live cells ('1') among the 8
 * neighbours inside [0,h) x [0,w); everything outside the local field is dead. */
static int count_neighbours(int32_t* const* grid, int h, int w, int x, int y)
{
    int n = 0;
    for (int i = x - 1; i <= x + 1; i++) {
        if (i < 0 || i >= h) continue;
        for (int j = y - 1; j <= y + 1; j++) {
            if (j < 0 || j >= w) continue;
            if (i == x && j == y) continue;
            if (grid[i][j] == LIVE_CELL) n++;
        }
    }
    return n;
}

/* updateGrid, Parallel_Life_MPI.cpp:37-54, generalised to a (birth, survive)
 * neighbour-count mask pair.  The reference's *effective* rule is birth=0,
 * survive=1<<2 ("B/S2"): the `count==3` store at :44-46 is always overwritten
 * by the if/else at :47-50.  Conway B3/S23 is birth=1<<3, survive=(1<<2)|(1<<3). */
static void update_grid(int32_t** grid, int32_t** next, int h, int w,
                        uint32_t birth, uint32_t survive)
{
    for (int i = 0; i < h; i++) {
        for (int j = 0; j < w; j++) {
            int n = count_neighbours(grid, h, w, i, j);
            int alive = grid[i][j] == LIVE_CELL;
            uint32_t m = alive ? survive : birth;
            next[i][j] = ((m >> n) & 1u) ? LIVE_CELL : DEAD_CELL;
        }
    }
}

/* Stripe decomposition of readGridFromFile, Parallel_Life_MPI.cpp:70-81.
 * Rank r of P owns global rows [start, start+rows) (its own rows plus one overlap
 * row from each neighbour; the last rank also takes the h % P tail). */
int oracle_ref_stripe(int h, int P, int r, int* start, int* rows)
{
    if (P <= 0 || r < 0 || r >= P || h / P == 0) return -1;
    long chunk = h / P;
    long s = (long)r * chunk;
    if (r != 0) { s--; chunk++; }
    if (r == P - 1) chunk += h % P;
    else chunk += 1;
    *start = (int)s;
    *rows = (int)chunk;
    return 0;
}

typedef struct {
    const char* data; /* whole data.txt, h*(w+1) bytes */
    int h, w, epochs, P, r;
    uint32_t birth, survive;
    char* out;        /* whole output, h*(w+1) bytes */
} rank_job;

/* One rank's life: readGridFromFile (:56-102), `epochs` x updateGrid (:215-221;
 * exchangeGridData :104-145 receives into copies and so has no effect),
 * writeDataToFile (:147-188). */
static void* run_rank(void* arg)
{
    rank_job* j = (rank_job*)arg;
    int start, rows;
    oracle_ref_stripe(j->h, j->P, j->r, &start, &rows);
    int w = j->w;
    int32_t** grid = (int32_t**)malloc(sizeof(int32_t*) * rows);
    int32_t** next = (int32_t**)malloc(sizeof(int32_t*) * rows);
    for (int y = 0; y < rows; y++) {
        grid[y] = (int32_t*)malloc(sizeof(int32_t) * (w ? w : 1));
        next[y] = (int32_t*)calloc(w ? w : 1, sizeof(int32_t));
        const char* src = j->data + (size_t)(start + y) * (w + 1);
        for (int x = 0; x < w; x++) grid[y][x] = (unsigned char)src[x];
    }
    for (int e = 0; e < j->epochs; e++) {
        update_grid(grid, next, rows, w, j->birth, j->survive);
        int32_t** t = grid; grid = next; next = t; /* swap(grid, nextGrid) :53 */
    }
    /* writeDataToFile: drop the overlap rows, write at r*(h/P)*(w+1) */
    int begin = (j->r != 0) ? 1 : 0;
    int end = (j->r != j->P - 1) ? rows - 1 : rows;
    size_t off = (size_t)j->r * (size_t)(j->h / j->P) * (size_t)(w + 1);
    char* dst = j->out + off;
    for (int y = begin; y < end; y++) {
        for (int x = 0; x < w; x++) *dst++ = (char)grid[y][x];
        *dst++ = '\n';
    }
    for (int y = 0; y < rows; y++) { free(grid[y]); free(next[y]); }
    free(grid); free(next);
    return NULL;
}

/* The whole program (main :190-240) as run by `mpirun -np P`: returns 0 and fills
 * out[h*(w+1)] with the bytes the reference writes to output.txt.  Ranks run as
 * threads (they never communicate, see §0.2 of SURVEY.md). */
int oracle_ref_program(const char* data, size_t len, int h, int w, int epochs,
                       int P, uint32_t birth, uint32_t survive, char* out,
                       int parallel)
{
    if (h <= 0 || w < 0 || epochs < 0 || P <= 0 || h / P == 0) return -1;
    if (len != (size_t)h * (size_t)(w + 1)) return -2;
    rank_job* jobs = (rank_job*)calloc(P, sizeof(rank_job));
    pthread_t* th = (pthread_t*)calloc(P, sizeof(pthread_t));
    for (int r = 0; r < P; r++) {
        jobs[r] = (rank_job){data, h, w, epochs, P, r, birth, survive, out};
        if (parallel) pthread_create(&th[r], NULL, run_rank, &jobs[r]);
        else run_rank(&jobs[r]);
    }
    if (parallel)
        for (int r = 0; r < P; r++) pthread_join(th[r], NULL);
    free(jobs); free(th);
    return 0;
}

/* Plain single-field stepper on the int-per-cell layout, used by the
 * cpu_baseline leg of bench.py to time the reference's algorithm on a bounded
 * sample.  Runs `threads` independent stripes (the -np decomposition). */
typedef struct { int32_t** grid; int32_t** next; int rows, w, gens; uint32_t b, s; } bl_job;
static void* bl_run(void* a)
{
    bl_job* j = (bl_job*)a;
    for (int e = 0; e < j->gens; e++) {
        update_grid(j->grid, j->next, j->rows, j->w, j->b, j->s);
        int32_t** t = j->grid; j->grid = j->next; j->next = t;
    }
    return NULL;
}
static inline uint64_t splitmix64_at(uint64_t seed, uint64_t idx);

/* Times the reference's algorithm on the benchmark's own field: thread t runs
 * rows [t*rows_per_thread, (t+1)*rows_per_thread) of the w-wide synthetic field
 * (cell (r, c) alive iff bit c%64 of splitmix64(seed, r*ceil(w/64) + c/64), as
 * oracle_bp_init_random / the engine's gol_init_random) as its own stripe with a
 * dead boundary, like one `mpirun -np threads` rank each.  Returns the live-cell
 * count (keeps the work observable). */
int64_t oracle_ref_baseline(int rows_per_thread, int w, int gens, int threads,
                            uint64_t seed, uint32_t birth, uint32_t survive)
{
    bl_job* jobs = (bl_job*)calloc(threads, sizeof(bl_job));
    pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
    const uint64_t wq = ((uint64_t)w + 63) / 64;
    for (int t = 0; t < threads; t++) {
        jobs[t].rows = rows_per_thread; jobs[t].w = w; jobs[t].gens = gens;
        jobs[t].b = birth; jobs[t].s = survive;
        jobs[t].grid = (int32_t**)malloc(sizeof(int32_t*) * rows_per_thread);
        jobs[t].next = (int32_t**)malloc(sizeof(int32_t*) * rows_per_thread);
        for (int y = 0; y < rows_per_thread; y++) {
            const uint64_t r = (uint64_t)t * (uint64_t)rows_per_thread + (uint64_t)y;
            jobs[t].grid[y] = (int32_t*)malloc(sizeof(int32_t) * w);
            jobs[t].next[y] = (int32_t*)calloc(w, sizeof(int32_t));
            uint64_t word = 0;
            for (int x = 0; x < w; x++) {
                if ((x & 63) == 0) word = splitmix64_at(seed, r * wq + (uint64_t)(x >> 6));
                jobs[t].grid[y][x] = ((word >> (x & 63)) & 1) ? LIVE_CELL : DEAD_CELL;
            }
        }
    }
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, bl_run, &jobs[t]);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    int64_t live = 0;
    for (int t = 0; t < threads; t++) {
        for (int y = 0; y < rows_per_thread; y++) {
            for (int x = 0; x < w; x++) live += jobs[t].grid[y][x] == LIVE_CELL;
            free(jobs[t].grid[y]); free(jobs[t].next[y]);
        }
        free(jobs[t].grid); free(jobs[t].next);
    }
    free(jobs); free(th);
    return live;
}

/* ------------------------------------------------------------------------- */
/* (2) bit-packed restatement                                                */
/*   layout: row-major, `stride` uint64 words per row, bit j of word q is    */
/*   column 64q+j; bits at columns >= w are always 0.                        */
/* ------------------------------------------------------------------------- */

static inline uint64_t splitmix64_at(uint64_t seed, uint64_t idx)
{
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static inline uint64_t last_word_mask(int64_t w)
{
    int rem = (int)(w & 63);
    return rem ? ((1ULL << rem) - 1ULL) : ~0ULL;
}

/* Synthetic p=0.5 field: word (r,q) = splitmix64(seed, r*Wq+q), masked to w.
 * _rows: field rows [row0, row0 + h) only (a rank's stripe of a larger field). */
void oracle_bp_init_random_rows(uint64_t* g, int64_t row0, int64_t h, int64_t w, int64_t stride,
                                uint64_t seed)
{
    int64_t wq = (w + 63) / 64;
    for (int64_t r = 0; r < h; r++) {
        for (int64_t q = 0; q < stride; q++) {
            uint64_t v = 0;
            if (q < wq) {
                v = splitmix64_at(seed, (uint64_t)(row0 + r) * (uint64_t)wq + (uint64_t)q);
                if (q == wq - 1) v &= last_word_mask(w);
            }
            g[r * stride + q] = v;
        }
    }
}

void oracle_bp_init_random(uint64_t* g, int64_t h, int64_t w, int64_t stride, uint64_t seed)
{
    oracle_bp_init_random_rows(g, 0, h, w, stride, seed);
}

/* Order-independent digest: live count and sum over words of
 * splitmix64(word ^ splitmix64(0, r*Wq+q)) mod 2^64. */
void oracle_bp_digest(const uint64_t* g, int64_t h, int64_t w, int64_t stride,
                      uint64_t* live, uint64_t* hash)
{
    int64_t wq = (w + 63) / 64;
    uint64_t L = 0, H = 0;
    for (int64_t r = 0; r < h; r++)
        for (int64_t q = 0; q < wq; q++) {
            uint64_t v = g[r * stride + q];
            L += (uint64_t)__builtin_popcountll(v);
            uint64_t idx = (uint64_t)r * (uint64_t)wq + (uint64_t)q;
            H += splitmix64_at(v ^ splitmix64_at(0, idx), 0);
        }
    *live = L;
    *hash = H;
}

/* ASCII <-> bits (the data.txt / output.txt byte format, :91-99, :157-164). */
int oracle_bp_pack_ascii(const char* buf, size_t len, int64_t h, int64_t w,
                         uint64_t* g, int64_t stride)
{
    if (len != (size_t)h * (size_t)(w + 1)) return -1;
    memset(g, 0, sizeof(uint64_t) * (size_t)(h * stride));
    for (int64_t r = 0; r < h; r++) {
        const char* row = buf + r * (w + 1);
        for (int64_t c = 0; c < w; c++)
            if (row[c] == LIVE_CELL) g[r * stride + (c >> 6)] |= 1ULL << (c & 63);
    }
    return 0;
}

void oracle_bp_unpack_ascii(const uint64_t* g, int64_t h, int64_t w, int64_t stride, char* buf)
{
    for (int64_t r = 0; r < h; r++) {
        char* row = buf + r * (w + 1);
        for (int64_t c = 0; c < w; c++)
            row[c] = ((g[r * stride + (c >> 6)] >> (c & 63)) & 1ULL) ? LIVE_CELL : DEAD_CELL;
        row[w] = '\n';
    }
}

/* One generation on rows [r0, r1) of a field of h rows (dead outside).
 * Neighbour count built as bit-sliced sums: per row a 3-cell horizontal sum
 * (with centre) and a 2-cell one (without), then the vertical sum of
 * H3(r-1) + H2(r) + H3(r+1), carried to 4 bits (0..8) so any mask pair works. */
static void bp_rows(const uint64_t* in, uint64_t* out, int64_t h, int64_t w, int64_t stride,
                    uint32_t birth, uint32_t survive, int64_t r0, int64_t r1)
{
    int64_t wq = (w + 63) / 64;
    uint64_t lastm = last_word_mask(w);
    for (int64_t r = r0; r < r1; r++) {
        for (int64_t q = 0; q < wq; q++) {
            uint64_t s3[3], c3[3], s2 = 0, c2 = 0, alive = 0;
            for (int d = -1; d <= 1; d++) {
                int64_t rr = r + d;
                uint64_t C = 0, Wl = 0, Wr = 0;
                if (rr >= 0 && rr < h) {
                    C = in[rr * stride + q];
                    Wl = q > 0 ? in[rr * stride + q - 1] : 0;
                    Wr = q + 1 < wq ? in[rr * stride + q + 1] : 0;
                }
                uint64_t L = (C << 1) | (Wl >> 63); /* neighbour at column c-1 */
                uint64_t R = (C >> 1) | (Wr << 63); /* neighbour at column c+1 */
                if (d == 0) {
                    s2 = L ^ R; c2 = L & R; alive = C;
                } else {
                    s3[d + 1] = L ^ C ^ R;
                    c3[d + 1] = (L & C) | (R & (L ^ C));
                }
            }
            /* bit0 */
            uint64_t a0 = s3[0], b0 = s2, e0 = s3[2];
            uint64_t n0 = a0 ^ b0 ^ e0;
            uint64_t k0 = (a0 & b0) | (e0 & (a0 ^ b0));
            /* weight-2 inputs: c3[0], c2, c3[2], k0 */
            uint64_t a1 = c3[0], b1 = c2, e1 = c3[2];
            uint64_t p = a1 ^ b1 ^ e1;
            uint64_t m = (a1 & b1) | (e1 & (a1 ^ b1));
            uint64_t n1 = p ^ k0;
            uint64_t k1 = p & k0;
            uint64_t n2 = m ^ k1;
            uint64_t n3 = m & k1;
            uint64_t res = 0;
            for (int n = 0; n <= 8; n++) {
                if (!(((birth | survive) >> n) & 1u)) continue; /* no cell takes this count */
                uint64_t eq = ((n & 1) ? n0 : ~n0) & ((n & 2) ? n1 : ~n1) &
                              ((n & 4) ? n2 : ~n2) & ((n & 8) ? n3 : ~n3);
                uint64_t sel = (((survive >> n) & 1u) ? alive : 0) |
                               (((birth >> n) & 1u) ? ~alive : 0);
                res |= eq & sel;
            }
            if (q == wq - 1) res &= lastm;
            out[r * stride + q] = res;
        }
        for (int64_t q = wq; q < stride; q++) out[r * stride + q] = 0;
    }
}

typedef struct {
    const uint64_t* in; uint64_t* out; int64_t h, w, stride; uint32_t b, s; int64_t r0, r1;
} bp_job;
static void* bp_run(void* a)
{
    bp_job* j = (bp_job*)a;
    bp_rows(j->in, j->out, j->h, j->w, j->stride, j->b, j->s, j->r0, j->r1);
    return NULL;
}

void oracle_bp_step(const uint64_t* in, uint64_t* out, int64_t h, int64_t w, int64_t stride,
                    uint32_t birth, uint32_t survive, int threads)
{
    if (threads <= 1 || h < 64) {
        bp_rows(in, out, h, w, stride, birth, survive, 0, h);
        return;
    }
    bp_job* jobs = (bp_job*)calloc(threads, sizeof(bp_job));
    pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
    int64_t per = (h + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        int64_t r0 = t * per, r1 = r0 + per;
        if (r0 > h) r0 = h;
        if (r1 > h) r1 = h;
        jobs[t] = (bp_job){in, out, h, w, stride, birth, survive, r0, r1};
        pthread_create(&th[t], NULL, bp_run, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(jobs); free(th);
}

/* E generations in place (ping-pong through a scratch buffer). */
int oracle_bp_run(uint64_t* g, int64_t h, int64_t w, int64_t stride, int64_t gens,
                  uint32_t birth, uint32_t survive, int threads)
{
    size_t n = (size_t)(h * stride);
    uint64_t* tmp = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
    if (!tmp) return -1;
    uint64_t* a = g; uint64_t* b = tmp;
    for (int64_t e = 0; e < gens; e++) {
        oracle_bp_step(a, b, h, w, stride, birth, survive, threads);
        uint64_t* t = a; a = b; b = t;
    }
    if (a != g) memcpy(g, a, sizeof(uint64_t) * n);
    free(tmp);
    return 0;
}
