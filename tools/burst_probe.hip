// burst_probe.hip -- dev microbenchmark: the stencil launch's start burst.
//
// At the start of a life_tb_kernel launch every wavefront (about 2000, two per
// SIMD) needs the first rows of its row block at once: 32 rows x 64 lanes x 8 B
// in the warm-up (profiles/r05/wave_phases.jsonl: 5-15 us before the first warm-up
// block completes).  This probe times only that: a "writer" kernel stores the
// field the way a launch does (plain 8-B stores, so it is the previous launch's
// output), then a "burst" kernel with the launch's grid has every wavefront load
// the rows of its block start and records when they have all landed.  Variants:
//   0: 32 rows, sc1 8-B loads (the kernel's row stream: agent-scope relaxed atomics)
//   1: 32 rows, plain 8-B loads
//   2: 32 rows as 16 row pairs, one 16-B nontemporal load per lane per pair (a
//      layout with two rows interleaved per lane group)
//   3: 8 rows, sc1 8-B loads (the r04 kernel's first ring)
//   4: as 2 with plain 16-B loads
// Prints one JSON line per variant: kernel time (HIP events) and the per-wave
// median / max time from its start to all loads landed (s_memrealtime, 100 MHz).
// Build: hipcc -O3 --offload-arch=gfx950 tools/burst_probe.hip -o /tmp/burst_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

constexpr int kStrips = 16;
constexpr int kRowWords = 1024;  // 65536 columns

__global__ __launch_bounds__(256) void writer(uint64_t* buf, int64_t rows, uint64_t seed)
{
    const int64_t n = rows * kRowWords;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        buf[i] = (uint64_t)i * 0x9E3779B97F4A7C15ull ^ seed;
}

template <int V>
__global__ __launch_bounds__(256) void burst(const uint64_t* buf, int64_t rows, int rpw,
                                             int units, uint64_t* out, uint64_t* stamps)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63;
    const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (unit >= units) return;
    const int blk = unit / kStrips, s = unit % kStrips;
    const int64_t rb = (int64_t)blk * rpw;
    const int64_t q = (int64_t)s * 62 + lane;  // lane group (8 B) of this lane
    uint64_t acc = 0;
    auto row_ok = [&](int64_t r) { return r >= 0 && r < rows; };
    if constexpr (V == 0 || V == 1 || V == 3) {
        constexpr int N = V == 3 ? 8 : 32;
        uint64_t v[N];
#pragma unroll
        for (int p = 0; p < N; ++p) {
            const int64_t r = min(max(rb - 16 + p, (int64_t)0), rows - 1);
            const uint64_t* a = buf + r * kRowWords + min(q, (int64_t)kRowWords - 1);
            if constexpr (V == 1)
                v[p] = *a;
            else
                v[p] = __hip_atomic_load(const_cast<uint64_t*>(a), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int p = 0; p < N; ++p) acc ^= row_ok(rb - 16 + p) ? v[p] : 0;
    } else {
        // row pairs: pair k holds rows 2k, 2k+1 interleaved per lane group (16 B)
        uint64_t v[32];
#pragma unroll
        for (int p = 0; p < 16; ++p) {
            const int64_t pr = min(max((rb - 16) / 2 + p, (int64_t)0), rows / 2 - 1);
            const uint64_t* a = buf + pr * 2 * kRowWords + 2 * min(q, (int64_t)kRowWords - 1);
            // (compiler-tracked loads only: an inline-asm load returns asynchronously
            // into registers the compiler already considers written, and the first
            // version of this probe faulted the GPU that way)
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            const v4u r = V == 2 ? __builtin_nontemporal_load(reinterpret_cast<const v4u*>(a))
                                 : *reinterpret_cast<const v4u*>(a);
            v[2 * p] = ((uint64_t)r.y << 32) | r.x;
            v[2 * p + 1] = ((uint64_t)r.w << 32) | r.z;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int p = 0; p < 32; ++p) acc ^= v[p];
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    out[(int64_t)unit * 64 + lane] = acc;
    if (lane == 0) {
        stamps[2 * unit] = t0;
        stamps[2 * unit + 1] = t1;
    }
}

template <int V>
void run(const char* name, uint64_t* buf, uint64_t* buf2, int64_t rows, int rpw, int units,
         uint64_t* out, uint64_t* stamps)
{
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const int grid = (units + 3) / 4;
    std::vector<float> ks;
    std::vector<double> med, mx;
    std::vector<uint64_t> h(2 * (size_t)units);
    for (int rep = 0; rep < 6; ++rep) {
        // the previous launch: write the field (and a second buffer of the same
        // size, as the launch's other ping-pong buffer)
        hipLaunchKernelGGL(writer, dim3(2048), dim3(256), 0, 0, buf, rows, (uint64_t)rep);
        hipLaunchKernelGGL(writer, dim3(2048), dim3(256), 0, 0, buf2, rows, (uint64_t)rep + 7);
        CHK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((burst<V>), dim3(grid), dim3(256), 0, 0, buf, rows, rpw, units, out,
                           stamps);
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        CHK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
        std::vector<double> d(units);
        for (int u = 0; u < units; ++u) d[u] = (double)(h[2 * u + 1] - h[2 * u]) / 100.0;
        std::sort(d.begin(), d.end());
        if (rep > 0) {
            ks.push_back(ms * 1e3f);
            med.push_back(d[units / 2]);
            mx.push_back(d[units - 1]);
        }
    }
    std::sort(ks.begin(), ks.end());
    std::sort(med.begin(), med.end());
    std::sort(mx.begin(), mx.end());
    std::printf("{\"variant\": \"%s\", \"rows\": %lld, \"rows_per_wave\": %d, \"waves\": %d, "
                "\"kernel_us_median\": %.2f, \"wave_landed_us_median\": %.2f, "
                "\"wave_landed_us_max\": %.2f}\n",
                name, (long long)rows, rpw, units, ks[ks.size() / 2], med[med.size() / 2],
                mx[mx.size() / 2]);
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
}

int main(int argc, char** argv)
{
    const int64_t rows = argc > 1 ? std::atoll(argv[1]) : 8448;
    const int rpw = argc > 2 ? std::atoi(argv[2]) : 70;
    const int units = (int)((rows + rpw - 1) / rpw) * kStrips;
    uint64_t *buf, *buf2, *out, *stamps;
    CHK(hipMalloc(&buf, rows * kRowWords * 8));
    CHK(hipMalloc(&buf2, rows * kRowWords * 8));
    CHK(hipMalloc(&out, (size_t)units * 64 * 8));
    CHK(hipMalloc(&stamps, (size_t)units * 2 * 8));
    run<0>("32 rows sc1 8B", buf, buf2, rows, rpw, units, out, stamps);
    run<1>("32 rows plain 8B", buf, buf2, rows, rpw, units, out, stamps);
    run<2>("16 row pairs nt 16B", buf, buf2, rows, rpw, units, out, stamps);
    run<3>("8 rows sc1 8B", buf, buf2, rows, rpw, units, out, stamps);
    run<4>("16 row pairs plain 16B", buf, buf2, rows, rpw, units, out, stamps);
    return 0;
}
