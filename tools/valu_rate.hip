// valu_rate.hip -- dev microbenchmark: issue rate of the VALU instructions the
// stencil uses (v_xor_b32 VOP2, v_bitop3_b32 / v_alignbit_b32 / v_xor3 VOP3,
// v_mov_b32_dpp) on gfx950, to price the kernel against the VALU ceiling.
// Each wave runs 16 independent accumulator chains; the grid fills every SIMD
// with 4 waves.  Build: hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o /tmp/valu_rate
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

#define BODY16(INSTR)                                                                      \
    asm volatile(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)  \
                     INSTR(8) INSTR(9) INSTR(10) INSTR(11) INSTR(12) INSTR(13) INSTR(14)  \
                     INSTR(15)                                                             \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), \
                   "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), \
                   "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])                      \
                 : "v"(k1), "v"(k2))

#define XOR(i) "v_xor_b32 %" #i ", %" #i ", %16\n"
#define BITOP3(i) "v_bitop3_b32 %" #i ", %" #i ", %16, %17 bitop3:0x96\n"
#define XOR3(i) "v_add3_u32 %" #i ", %" #i ", %16, %17\n"
#define ALIGN(i) "v_alignbit_b32 %" #i ", %" #i ", %16, 31\n"
#define DPP(i) "v_mov_b32_dpp %" #i ", %" #i " wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define ANDOR(i) "v_and_or_b32 %" #i ", %" #i ", %16, %17\n"
#define ORDPP(i) "v_or_b32_dpp %" #i ", %" #i ", %16 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n"
#define ROWDPP(i) "v_mov_b32_dpp %" #i ", %" #i " row_shr:1 row_mask:0xf bank_mask:0xf\n"
#define LSHL(i) "v_lshlrev_b32 %" #i ", 1, %" #i "\n"
#define LSHLOR(i) "v_lshl_or_b32 %" #i ", %" #i ", 1, %16\n"
#define ADDC(i) "v_addc_co_u32 %" #i ", vcc, %" #i ", %" #i ", vcc\n"
#define ADDC64(i) "v_addc_co_u32_e64 %" #i ", s[60:61], %" #i ", %" #i ", s[62:63]\n"
#define CMPV(i) "v_cmp_gt_i32_e64 s[60:61], 0, %" #i "\n"
#define ORROWDPP(i) "v_or_b32_dpp %" #i ", %" #i ", %16 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n"

#define BODY16A(PRE, INSTR)                                                                \
    asm volatile(PRE INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7) \
                     INSTR(8) INSTR(9) INSTR(10) INSTR(11) INSTR(12) INSTR(13) INSTR(14)  \
                     INSTR(15)                                                             \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), \
                   "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), \
                   "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])                      \
                 : "v"(k1), "v"(k2))
#define BITOP3X(i) "v_bitop3_b32 %" #i ", %" #i ", %16, %17 bitop3:0x96\n" \
                   "v_bitop3_b32 %" #i ", %" #i ", %17, %16 bitop3:0xe8\n"

// a stage-like mix per chain: DPP move, funnel shift, 6 x bitop3 (8-byte encodings)
#define MIX(i) "v_mov_b32_dpp %" #i ", %" #i " wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
               "v_alignbit_b32 %" #i ", %" #i ", %16, 31\n"                             \
               "v_bitop3_b32 %" #i ", %" #i ", %16, %17 bitop3:0x96\n"                  \
               "v_bitop3_b32 %" #i ", %" #i ", %17, %16 bitop3:0xe8\n"                  \
               "v_bitop3_b32 %" #i ", %" #i ", %16, %17 bitop3:0x96\n"                  \
               "v_bitop3_b32 %" #i ", %" #i ", %17, %16 bitop3:0xe8\n"                  \
               "v_bitop3_b32 %" #i ", %" #i ", %16, %17 bitop3:0x96\n"                  \
               "v_bitop3_b32 %" #i ", %" #i ", %17, %16 bitop3:0xe8\n"
// interleaved chains: instruction k of chain i, then of chain i+1 (like the
// compiler's schedule of independent stage-steps)
#define MIX2(i, j) "v_mov_b32_dpp %" #i ", %" #i " wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
               "v_mov_b32_dpp %" #j ", %" #j " wave_shr:1 row_mask:0xf bank_mask:0xf\n"      \
               "v_alignbit_b32 %" #i ", %" #i ", %16, 31\n"                             \
               "v_alignbit_b32 %" #j ", %" #j ", %16, 31\n"                             \
               "v_bitop3_b32 %" #i ", %" #i ", %16, %17 bitop3:0x96\n"                  \
               "v_bitop3_b32 %" #j ", %" #j ", %16, %17 bitop3:0x96\n"                  \
               "v_bitop3_b32 %" #i ", %" #i ", %17, %16 bitop3:0xe8\n"                  \
               "v_bitop3_b32 %" #j ", %" #j ", %17, %16 bitop3:0xe8\n"                  \
               "v_bitop3_b32 %" #i ", %" #i ", %16, %17 bitop3:0x96\n"                  \
               "v_bitop3_b32 %" #j ", %" #j ", %16, %17 bitop3:0x96\n"                  \
               "v_bitop3_b32 %" #i ", %" #i ", %17, %16 bitop3:0xe8\n"                  \
               "v_bitop3_b32 %" #j ", %" #j ", %17, %16 bitop3:0xe8\n"
#define BODY8PAIRS(PRE)                                                                     \
    asm volatile(PRE MIX2(0, 1) MIX2(2, 3) MIX2(4, 5) MIX2(6, 7) MIX2(8, 9) MIX2(10, 11)      \
                 MIX2(12, 13) MIX2(14, 15)                                                   \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), \
                   "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), \
                   "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])                      \
                 : "v"(k1), "v"(k2))

#define DPPX(i) "v_mov_b32_dpp %" #i ", %" #i " wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define ALGX(i) "v_alignbit_b32 %" #i ", %" #i ", %16, 31\n"
#define DB(i) DPPX(i) "v_bitop3_b32 %" #i ", %" #i ", %16, %17 bitop3:0x96\n"
#define AB(i) ALGX(i) "v_bitop3_b32 %" #i ", %" #i ", %16, %17 bitop3:0x96\n"

#define BODY16S(INSTR)                                                                     \
    asm volatile(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)  \
                     INSTR(8) INSTR(9) INSTR(10) INSTR(11) INSTR(12) INSTR(13) INSTR(14)  \
                     INSTR(15)                                                             \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), \
                   "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), \
                   "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])                      \
                 : "v"(k1), "v"(k2)                                                        \
                 : "vcc", "s60", "s61", "s62", "s63")

template <int OP>
__global__ __launch_bounds__(256) void rate_kernel(unsigned* out, unsigned k1, unsigned k2)
{
    unsigned r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
    for (int it = 0; it < kIters; ++it) {
        if constexpr (OP == 0) BODY16(XOR);
        if constexpr (OP == 1) BODY16(BITOP3);
        if constexpr (OP == 2) BODY16(XOR3);
        if constexpr (OP == 3) BODY16(ALIGN);
        if constexpr (OP == 4) BODY16(DPP);
        if constexpr (OP == 5) BODY16(ANDOR);
        if constexpr (OP == 6) BODY16(ORDPP);
        if constexpr (OP == 7) BODY16(ROWDPP);
        if constexpr (OP == 8) BODY16(LSHL);
        if constexpr (OP == 9) BODY16(LSHLOR);
        if constexpr (OP == 10) BODY16(ORROWDPP);
        if constexpr (OP == 11) BODY16S(ADDC);
        if constexpr (OP == 12) BODY16S(CMPV);
        if constexpr (OP == 13) BODY16S(ADDC64);
        if constexpr (OP == 14) BODY16A(".p2align 3\n", BITOP3X);
        if constexpr (OP == 15) BODY16A(".p2align 3\ns_nop 0\n", BITOP3X);
        if constexpr (OP == 16) BODY16A(".p2align 3\n", MIX);
        if constexpr (OP == 17) BODY16A(".p2align 3\ns_nop 0\n", MIX);
        if constexpr (OP == 18) BODY8PAIRS(".p2align 3\n");
        if constexpr (OP == 19) BODY8PAIRS(".p2align 3\ns_nop 0\n");
        if constexpr (OP == 20) BODY16A(".p2align 3\n", DPPX);
        if constexpr (OP == 21) BODY16A(".p2align 3\ns_nop 0\n", DPPX);
        if constexpr (OP == 22) BODY16A(".p2align 3\n", ALGX);
        if constexpr (OP == 23) BODY16A(".p2align 3\ns_nop 0\n", ALGX);
        if constexpr (OP == 24) BODY16A(".p2align 3\n", DB);
        if constexpr (OP == 25) BODY16A(".p2align 3\ns_nop 0\n", DB);
        if constexpr (OP == 26) BODY16A(".p2align 3\n", AB);
        if constexpr (OP == 27) BODY16A(".p2align 3\ns_nop 0\n", AB);
    }
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
double run(unsigned* d, int blocks)
{
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipLaunchKernelGGL(rate_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u, 5u);  // warm
    CHK(hipEventRecord(a));
    for (int rep = 0; rep < 5; ++rep)
        hipLaunchKernelGGL(rate_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u, 5u);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double waves = 5.0 * blocks * 4;
    const double instr = waves * kIters * 16;  // wave-instructions
    return instr / (ms * 1e-3);                // wave-instructions per second
}

int main()
{
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 4;  // 4 blocks x 4 waves per CU = 4 waves per SIMD
    unsigned* d;
    CHK(hipMalloc(&d, sizeof(unsigned) * blocks * 256));
    const char* names[] = {"v_xor_b32", "v_bitop3_b32", "v_add3_u32", "v_alignbit_b32",
                           "v_mov_b32_dpp", "v_and_or_b32", "v_or_b32_dpp_wave_shr",
                           "v_mov_b32_dpp_row_shr", "v_lshlrev_b32", "v_lshl_or_b32",
                           "v_or_b32_dpp_row_shr", "v_addc_co_u32", "v_cmp_gt_i32_e64",
                           "v_addc_co_u32_e64"};
    constexpr int N = 14;
    double r[N] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks),
                   run<4>(d, blocks), run<5>(d, blocks), run<6>(d, blocks), run<7>(d, blocks),
                   run<8>(d, blocks), run<9>(d, blocks), run<10>(d, blocks),
                   run<11>(d, blocks), run<12>(d, blocks), run<13>(d, blocks)};
    std::printf("{\"cus\": %d, \"clock_mhz_prop\": %d", cus, p.clockRate / 1000);
    for (int i = 0; i < N; ++i)
        std::printf(", \"%s\": %.4g", names[i], r[i] / (4.0 * cus));  // per SIMD per second
    // issue rate vs resident waves per SIMD (16 independent chains per wave)
    // the same 32 v_bitop3 (8-byte encodings) starting at 0 mod 8 vs 4 mod 8
    std::printf(", \"v_bitop3_b32_at_0mod8\": %.4g", 2 * run<14>(d, blocks) / (4.0 * cus));
    std::printf(", \"v_bitop3_b32_at_4mod8\": %.4g", 2 * run<15>(d, blocks) / (4.0 * cus));
    std::printf(", \"v_bitop3_b32_at_0mod8_2waves\": %.4g", 2 * run<14>(d, 2 * cus) / (4.0 * cus));
    std::printf(", \"v_bitop3_b32_at_4mod8_2waves\": %.4g", 2 * run<15>(d, 2 * cus) / (4.0 * cus));
    {
        const char* nm[] = {"dpp", "alignbit", "dpp+bitop3", "alignbit+bitop3"};
        const int per[] = {1, 1, 2, 2};
        double v[8] = {run<20>(d, 2 * cus), run<21>(d, 2 * cus), run<22>(d, 2 * cus),
                       run<23>(d, 2 * cus), run<24>(d, 2 * cus), run<25>(d, 2 * cus),
                       run<26>(d, 2 * cus), run<27>(d, 2 * cus)};
        for (int i = 0; i < 4; ++i)
            std::printf(", \"%s_at_0mod8_2w\": %.4g, \"%s_at_4mod8_2w\": %.4g", nm[i],
                        per[i] * v[2 * i] / (4.0 * cus), nm[i], per[i] * v[2 * i + 1] / (4.0 * cus));
    }
    // stage-like mix (8 instructions per chain: 1 DPP, 1 alignbit, 6 bitop3)
    for (int w = 1; w <= 4; w *= 2) {
        std::printf(", \"mix_at_0mod8_%dw\": %.4g", w, 8 * run<16>(d, w * cus) / (4.0 * cus));
        std::printf(", \"mix_at_4mod8_%dw\": %.4g", w, 8 * run<17>(d, w * cus) / (4.0 * cus));
        std::printf(", \"mixpairs_at_0mod8_%dw\": %.4g", w, 6 * run<18>(d, w * cus) / (4.0 * cus));
        std::printf(", \"mixpairs_at_4mod8_%dw\": %.4g", w, 6 * run<19>(d, w * cus) / (4.0 * cus));
    }
    std::printf(", \"v_bitop3_b32_1wave\": %.4g", run<1>(d, cus) / (4.0 * cus));
    std::printf(", \"v_bitop3_b32_2waves\": %.4g", run<1>(d, 2 * cus) / (4.0 * cus));
    std::printf(", \"unit\": \"wave-instructions per SIMD per second\"}\n");
    return 0;
}
