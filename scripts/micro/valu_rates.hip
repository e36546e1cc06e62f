// Issue cost of the integer VALU instructions K1's token rounds use, one SIMD's view: every
// CU runs 16 waves (4 per SIMD), each a loop of 8 independent chains of one instruction, so
// the time per wave-instruction per SIMD is the instruction's issue cost, not its latency.
// Build/run (GPU box): hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o /tmp/vr && /tmp/vr
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP8(ins)                                                            \
    asm volatile(ins " %0, %0, %8\n\t" ins " %1, %1, %8\n\t" ins " %2, %2, %8\n\t" ins " %3, %3, %8\n\t" \
                 ins " %4, %4, %8\n\t" ins " %5, %5, %8\n\t" ins " %6, %6, %8\n\t" ins " %7, %7, %8"   \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k))
#define OP8_3(ins)                                                          \
    asm volatile(ins " %0, %0, %8, %0\n\t" ins " %1, %1, %8, %1\n\t" ins " %2, %2, %8, %2\n\t" ins " %3, %3, %8, %3\n\t" \
                 ins " %4, %4, %8, %4\n\t" ins " %5, %5, %8, %5\n\t" ins " %6, %6, %8, %6\n\t" ins " %7, %7, %8, %7"   \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k))

template <int OP>
__global__ __launch_bounds__(256) void k_rate(unsigned* out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned k = 0x9E3779B1u ^ blockIdx.x;
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) OP8("v_add_u32");
        if (OP == 1) OP8("v_mul_lo_u32");
        if (OP == 2) OP8("v_mul_hi_u32");
        if (OP == 3) OP8("v_mul_u32_u24");
        if (OP == 4) OP8("v_mul_hi_u32_u24");
        if (OP == 5) OP8_3("v_perm_b32");
        if (OP == 6) OP8_3("v_dot4_u32_u8");
        if (OP == 7) OP8_3("v_alignbit_b32");
        if (OP == 8) OP8("v_lshlrev_b32");
        if (OP == 9) OP8_3("v_bfe_u32");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

int main() {
    int dev = 0, ncu = 0, clk = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);   /* kHz */
    unsigned* out;
    hipMalloc(&out, (size_t)ncu * 4 * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24", "v_mul_hi_u32_u24",
                           "v_perm_b32", "v_dot4_u32_u8", "v_alignbit_b32", "v_lshlrev_b32", "v_bfe_u32"};
    const int iters = 20000;
    for (int op = 0; op < 10; ++op) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            switch (op) {
#define L(n) case n: k_rate<n><<<ncu * 4, 256>>>(out, iters); break;
                L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9)
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        /* per SIMD: 4 waves x iters x 8 wave-instructions */
        const double per_simd = 4.0 * iters * 8;
        printf("%-18s %8.3f ms  %6.2f ns per wave-instruction per SIMD (%.2f cycles at %.0f MHz)\n", names[op], best,
               best * 1e6 / per_simd, best * 1e6 / per_simd * clk / 1e6, clk / 1e3);
    }
    return 0;
}
