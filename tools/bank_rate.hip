// bank_rate.hip -- dev microbenchmark: does the VGPR bank of v_bitop3_b32's three
// sources (bank = register index mod 4) change its issue rate on gfx950?  Each
// wave runs 16 independent accumulator chains v[32..47]; the two other sources
// are registers chosen per variant: distinct banks, two in the accumulator's
// bank, or all three in one bank.  2 waves per SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 tools/bank_rate.hip -o /tmp/bank_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

constexpr int kIters = 4096;

// accumulators v32..v47 (bank = i mod 4); sources: S1, S2 fixed registers
#define OP(d, s1, s2) "v_bitop3_b32 v" #d ", v" #d ", v" #s1 ", v" #s2 " bitop3:0x96\n"
#define SIXTEEN(s1, s2) OP(32, s1, s2) OP(33, s1, s2) OP(34, s1, s2) OP(35, s1, s2) \
    OP(36, s1, s2) OP(37, s1, s2) OP(38, s1, s2) OP(39, s1, s2) OP(40, s1, s2) OP(41, s1, s2) \
    OP(42, s1, s2) OP(43, s1, s2) OP(44, s1, s2) OP(45, s1, s2) OP(46, s1, s2) OP(47, s1, s2)
// per-accumulator bank-matched sources: S1 = d + 16, S2 = d + 32 (same bank as d)
#define OPM(d, s1, s2) "v_bitop3_b32 v" #d ", v" #d ", v" #s1 ", v" #s2 " bitop3:0x96\n"
#define SIXTEEN_SAME OPM(32, 48, 64) OPM(33, 49, 65) OPM(34, 50, 66) OPM(35, 51, 67) \
    OPM(36, 52, 68) OPM(37, 53, 69) OPM(38, 54, 70) OPM(39, 55, 71) OPM(40, 56, 72) \
    OPM(41, 57, 73) OPM(42, 58, 74) OPM(43, 59, 75) OPM(44, 60, 76) OPM(45, 61, 77) \
    OPM(46, 62, 78) OPM(47, 63, 79)
// sources in the two banks other than the accumulator's (d+1, d+2 mod 4)
#define SIXTEEN_DIFF OPM(32, 49, 66) OPM(33, 50, 67) OPM(34, 51, 64) OPM(35, 48, 65) \
    OPM(36, 53, 70) OPM(37, 54, 71) OPM(38, 55, 68) OPM(39, 52, 69) OPM(40, 57, 74) \
    OPM(41, 58, 75) OPM(42, 59, 72) OPM(43, 56, 73) OPM(44, 61, 78) OPM(45, 62, 79) \
    OPM(46, 63, 76) OPM(47, 60, 77)
// two sources in the accumulator's bank, one elsewhere
#define SIXTEEN_TWO OPM(32, 48, 65) OPM(33, 49, 66) OPM(34, 50, 67) OPM(35, 51, 64) \
    OPM(36, 52, 69) OPM(37, 53, 70) OPM(38, 54, 71) OPM(39, 55, 68) OPM(40, 56, 73) \
    OPM(41, 57, 74) OPM(42, 58, 75) OPM(43, 59, 72) OPM(44, 60, 77) OPM(45, 61, 78) \
    OPM(46, 62, 79) OPM(47, 63, 76)

#define CLOB                                                                              \
    "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43",   \
        "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
        "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", \
        "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79"

template <int OPK>
__global__ __launch_bounds__(256) void rate_kernel(unsigned* out)
{
    for (int it = 0; it < kIters; ++it) {
        if constexpr (OPK == 0) asm volatile(".p2align 3\n" SIXTEEN_DIFF ::: CLOB);
        if constexpr (OPK == 1) asm volatile(".p2align 3\n" SIXTEEN_TWO ::: CLOB);
        if constexpr (OPK == 2) asm volatile(".p2align 3\n" SIXTEEN_SAME ::: CLOB);
        if constexpr (OPK == 3) asm volatile(".p2align 3\ns_nop 0\n" SIXTEEN_DIFF ::: CLOB);
        if constexpr (OPK == 4) asm volatile(".p2align 3\ns_nop 0\n" SIXTEEN_TWO ::: CLOB);
        if constexpr (OPK == 5) asm volatile(".p2align 3\ns_nop 0\n" SIXTEEN_SAME ::: CLOB);
    }
    unsigned v;
    asm volatile("v_mov_b32 %0, v32" : "=v"(v));
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

template <int OPK>
double run(unsigned* d, int blocks)
{
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipLaunchKernelGGL(rate_kernel<OPK>, dim3(blocks), dim3(256), 0, 0, d);
    CHK(hipEventRecord(a));
    for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(rate_kernel<OPK>, dim3(blocks), dim3(256), 0, 0, d);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    return 5.0 * blocks * 4 * kIters * 16 / (ms * 1e-3);
}

int main()
{
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    unsigned* d;
    CHK(hipMalloc(&d, sizeof(unsigned) * cus * 4 * 256));
    const char* nm[] = {"distinct_banks", "two_in_one_bank", "three_in_one_bank"};
    std::printf("{\"unit\": \"v_bitop3 wave-instructions per SIMD per second, 2 waves/SIMD\"");
    for (int w = 1; w <= 2; ++w) {
        const int blocks = w * cus;
        double v[6] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks),
                       run<3>(d, blocks), run<4>(d, blocks), run<5>(d, blocks)};
        for (int i = 0; i < 3; ++i)
            std::printf(", \"%s_0mod8_%dw\": %.4g, \"%s_4mod8_%dw\": %.4g", nm[i], w,
                        v[i] / (4.0 * cus), nm[i], w, v[i + 3] / (4.0 * cus));
    }
    std::printf("}\n");
    return 0;
}
