// life_aux.hip -- memory-bound helper kernels (synthetic init, digest, ASCII
// codec) and the depth dispatch of the stencil kernel (life_stencil.h, one
// translation unit per depth: life_tb_d<K>.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bitlayout.h"
#include "life_internal.h"

namespace gol {

#define GOL_EXTERN_DEPTH(K)                                                                   \
    extern template hipError_t launch_depth<K>(const StepArgs&, RuleKind, int, bool,          \
                                               hipStream_t);                                  \
    extern template int occupancy_depth<K>(RuleKind, int, bool, bool);
GOL_EXTERN_DEPTH(1)
GOL_EXTERN_DEPTH(2)
GOL_EXTERN_DEPTH(4)
GOL_EXTERN_DEPTH(6)
GOL_EXTERN_DEPTH(7)
GOL_EXTERN_DEPTH(8)
GOL_EXTERN_DEPTH(12)
GOL_EXTERN_DEPTH(16)
#if GOL_DEV_KERNELS
GOL_EXTERN_DEPTH(20)
GOL_EXTERN_DEPTH(24)
GOL_EXTERN_DEPTH(32)
#endif
#undef GOL_EXTERN_DEPTH

hipError_t launch_life(const StepArgs& a, int depth, RuleKind rule, int planes, bool hand,
                       hipStream_t s)
{
    if (a.total_units <= 0) return hipSuccess;
    switch (depth) {
    case 1: return launch_depth<1>(a, rule, planes, hand, s);
    case 2: return launch_depth<2>(a, rule, planes, hand, s);
    case 4: return launch_depth<4>(a, rule, planes, hand, s);
    case 6: return launch_depth<6>(a, rule, planes, hand, s);
    case 7: return launch_depth<7>(a, rule, planes, hand, s);
    case 8: return launch_depth<8>(a, rule, planes, hand, s);
    case 12: return launch_depth<12>(a, rule, planes, hand, s);
    case 16: return launch_depth<16>(a, rule, planes, hand, s);
#if GOL_DEV_KERNELS
    case 20: return launch_depth<20>(a, rule, planes, hand, s);
    case 24: return launch_depth<24>(a, rule, planes, hand, s);
    case 32: return launch_depth<32>(a, rule, planes, hand, s);
#endif
    default: return hipErrorInvalidValue;
    }
}

int life_blocks_per_cu(int depth, RuleKind rule, int planes, bool hand, bool mp)
{
    switch (depth) {
    case 1: return occupancy_depth<1>(rule, planes, hand, mp);
    case 2: return occupancy_depth<2>(rule, planes, hand, mp);
    case 4: return occupancy_depth<4>(rule, planes, hand, mp);
    case 6: return occupancy_depth<6>(rule, planes, hand, mp);
    case 7: return occupancy_depth<7>(rule, planes, hand, mp);
    case 8: return occupancy_depth<8>(rule, planes, hand, mp);
    case 12: return occupancy_depth<12>(rule, planes, hand, mp);
    case 16: return occupancy_depth<16>(rule, planes, hand, mp);
#if GOL_DEV_KERNELS
    case 20: return occupancy_depth<20>(rule, planes, hand, mp);
    case 24: return occupancy_depth<24>(rule, planes, hand, mp);
    case 32: return occupancy_depth<32>(rule, planes, hand, mp);
#endif
    default: return 0;
    }
}

bool life_has_kernel(int depth, int planes)
{
    bool listed = false;
    for (int d : kDepthList) listed |= d == depth;
    if (!listed) return false;
    return planes == 2 || (kDevKernels && planes == 4 && depth <= 16);
}

namespace {

__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t idx)
{
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// The kernels below work per lane group of NP planes (NP/2 words, bitlayout.h);
// the canonical word index r*wq + c is what the synthetic field and the digest are
// defined on (gol.h), so they match the oracle's.

template <int NP>
__global__ __launch_bounds__(256) void init_random_kernel(uint64_t* buf, int64_t stride,
                                                          int64_t wq, uint64_t lastmask,
                                                          int64_t row_base, int64_t glob_row0,
                                                          int64_t nrows, uint64_t seed)
{
    constexpr int G = NP / 2;
    const int64_t gpr = stride / G;  // lane groups per buffer row
    const int64_t total = nrows * gpr;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = k / gpr, gq = k - i * gpr;
        uint64_t c[2] = {0, 0}, s[2];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int64_t idx = gq * G + j;
            if (idx < wq) {
                c[j] = splitmix64_at(seed, (uint64_t)(glob_row0 + i) * (uint64_t)wq + (uint64_t)idx);
                if (idx == wq - 1) c[j] &= lastmask;  // canonical mask
            }
        }
        gol_split_group(c, s, NP);
#pragma unroll
        for (int j = 0; j < G; ++j) buf[(row_base + i) * stride + gq * G + j] = s[j];
    }
}

template <int NP>
__global__ __launch_bounds__(256) void digest_kernel(const uint64_t* buf, int64_t stride,
                                                     int64_t wq, int64_t ng, int64_t row_base,
                                                     int64_t glob_row0, int64_t nrows,
                                                     unsigned long long* acc)
{
    constexpr int G = NP / 2;
    const int64_t total = nrows * ng;
    uint64_t live = 0, hash = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = k / ng, gq = k - i * ng;
        uint64_t s[2] = {0, 0}, c[2];
#pragma unroll
        for (int j = 0; j < G; ++j) s[j] = buf[(row_base + i) * stride + gq * G + j];
        gol_join_group(s, c, NP);
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int64_t idx = gq * G + j;
            if (idx < wq) {
                live += (uint64_t)__popcll(c[j]);
                const uint64_t h = (uint64_t)(glob_row0 + i) * (uint64_t)wq + (uint64_t)idx;
                hash += splitmix64_at(c[j] ^ splitmix64_at(0, h), 0);
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        live += __shfl_xor(live, off);
        hash += __shfl_xor(hash, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&acc[0], (unsigned long long)live);
        atomicAdd(&acc[1], (unsigned long long)hash);
    }
}

// ASCII codec (data.txt / output.txt bytes <-> stored lane groups), the
// device-side replacement of readGridFromFile's parse (:91-99) and
// writeDataToFile's serialisation (:157-164).  One wavefront per (row, lane
// group): lane j reads the byte of column 64c+j of each of the group's words
// (coalesced), __ballot forms the canonical words, lane 0 stores the group.
// Byte w of every row must be '\n'.
template <int NP>
__global__ __launch_bounds__(256) void ascii_pack_kernel(const char* src, int64_t rows, int64_t w,
                                                         int64_t ng, uint64_t* dst,
                                                         int64_t stride, int* bad)
{
    constexpr int G = NP / 2;
    const int lane = threadIdx.x & 63;
    const int64_t total = rows * ng;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t k = wave0; k < total; k += nwaves) {
        const int64_t r = k / ng, gq = k - r * ng;
        const char* line = src + r * (w + 1);
        uint64_t c[2] = {0, 0}, s[2];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int64_t col = (gq * G + j) * 64 + lane;
            c[j] = __ballot(col < w && line[col] == '1');
        }
        if (lane == 0) {
            gol_split_group(c, s, NP);
#pragma unroll
            for (int j = 0; j < G; ++j) dst[r * stride + gq * G + j] = s[j];
            if (gq == ng - 1 && line[w] != '\n') atomicOr(bad, 1);
        }
    }
}

template <int NP>
__global__ __launch_bounds__(256) void ascii_unpack_kernel(const uint64_t* src, int64_t stride,
                                                           int64_t rows, int64_t w, int64_t ng,
                                                           char* dst)
{
    constexpr int G = NP / 2;
    const int lane = threadIdx.x & 63;
    const int64_t total = rows * ng;
    const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t k = wave0; k < total; k += nwaves) {
        const int64_t r = k / ng, gq = k - r * ng;
        uint64_t s[2] = {0, 0}, c[2];
#pragma unroll
        for (int j = 0; j < G; ++j) s[j] = src[r * stride + gq * G + j];
        gol_join_group(s, c, NP);
        char* line = dst + r * (w + 1);
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int64_t col = (gq * G + j) * 64 + lane;
            if (col < w) line[col] = ((c[j] >> lane) & 1) ? '1' : '0';
        }
        if (gq == ng - 1 && lane == 0) line[w] = '\n';
    }
}

dim3 grid_for(int64_t items, int64_t per_block, int64_t cap)
{
    int64_t blocks = (items + per_block - 1) / per_block;
    if (blocks > cap) blocks = cap;
    return dim3((unsigned)blocks);
}

}  // namespace

hipError_t launch_init_random(uint64_t* buf, int64_t stride, int64_t wq, uint64_t lastmask,
                              int64_t row_base, int64_t glob_row0, int64_t nrows, uint64_t seed,
                              int planes, hipStream_t s)
{
    if (nrows <= 0) return hipSuccess;
    const dim3 grid = grid_for(nrows * stride / (planes / 2), 256, 8192);
    if (planes == 4)
        hipLaunchKernelGGL(init_random_kernel<4>, grid, dim3(256), 0, s, buf, stride, wq, lastmask,
                           row_base, glob_row0, nrows, seed);
    else
        hipLaunchKernelGGL(init_random_kernel<2>, grid, dim3(256), 0, s, buf, stride, wq, lastmask,
                           row_base, glob_row0, nrows, seed);
    return hipGetLastError();
}

hipError_t launch_ascii_pack(const char* src, int64_t rows, int64_t w, int64_t ng, uint64_t* dst,
                             int64_t stride, int* bad, int planes, hipStream_t s)
{
    if (rows <= 0) return hipSuccess;
    const dim3 grid = grid_for(rows * ng, 4, 16384);
    if (planes == 4)
        hipLaunchKernelGGL(ascii_pack_kernel<4>, grid, dim3(256), 0, s, src, rows, w, ng, dst,
                           stride, bad);
    else
        hipLaunchKernelGGL(ascii_pack_kernel<2>, grid, dim3(256), 0, s, src, rows, w, ng, dst,
                           stride, bad);
    return hipGetLastError();
}

hipError_t launch_ascii_unpack(const uint64_t* src, int64_t stride, int64_t rows, int64_t w,
                               int64_t ng, char* dst, int planes, hipStream_t s)
{
    if (rows <= 0) return hipSuccess;
    const dim3 grid = grid_for(rows * ng, 4, 16384);
    if (planes == 4)
        hipLaunchKernelGGL(ascii_unpack_kernel<4>, grid, dim3(256), 0, s, src, stride, rows, w, ng,
                           dst);
    else
        hipLaunchKernelGGL(ascii_unpack_kernel<2>, grid, dim3(256), 0, s, src, stride, rows, w, ng,
                           dst);
    return hipGetLastError();
}

hipError_t launch_digest(const uint64_t* buf, int64_t stride, int64_t wq, int64_t ng,
                         int64_t row_base, int64_t glob_row0, int64_t nrows,
                         unsigned long long* acc, int planes, hipStream_t s)
{
    if (nrows <= 0) return hipSuccess;
    const dim3 grid = grid_for(nrows * ng, 256, 8192);
    if (planes == 4)
        hipLaunchKernelGGL(digest_kernel<4>, grid, dim3(256), 0, s, buf, stride, wq, ng, row_base,
                           glob_row0, nrows, acc);
    else
        hipLaunchKernelGGL(digest_kernel<2>, grid, dim3(256), 0, s, buf, stride, wq, ng, row_base,
                           glob_row0, nrows, acc);
    return hipGetLastError();
}

}  // namespace gol
