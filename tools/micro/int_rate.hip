// Microbenchmark: issue cost of the integer / packed-16-bit VALU ops the extraction kernels use
// on gfx950, at 1, 2, 4 and 8 waves per SIMD, 8 independent chains per lane.  Prints cycles per
// wave-instruction per SIMD (wave0's clock64 span / instructions x waves per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN8(ASM)                                                                                 \
    _Pragma("unroll") for (int i = 0; i < 8; i++) asm volatile(ASM : "+v"(x[i]) : "v"(y), "v"(z));

template <int OP>
__global__ __launch_bounds__(64) void k_rate(unsigned* out, int n, long long* cyc)
{
    unsigned x[8];
    unsigned y = threadIdx.x * 0x01010101u + 7, z = 0x05040302u ^ threadIdx.x;
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x * 3 + i;
    long long t0 = clock64();
    for (int k = 0; k < n; k++) {
        if (OP == 0) CHAIN8("v_perm_b32 %0, %1, %0, %2")
        if (OP == 1) CHAIN8("v_pk_min_u16 %0, %0, %1")
        if (OP == 2) CHAIN8("v_pk_sub_u16 %0, %0, %1 clamp")
        if (OP == 3) CHAIN8("v_add_u32 %0, %0, %1")
        if (OP == 4) CHAIN8("v_and_b32 %0, %0, %1")
        if (OP == 5) CHAIN8("v_dot2_u32_u16 %0, %1, %2, %0")
        if (OP == 6) CHAIN8("v_min3_u32 %0, %0, %1, %2")
        if (OP == 7) CHAIN8("v_alignbyte_b32 %0, %0, %1, %2")
        if (OP == 8) CHAIN8("v_fma_f32 %0, %0, %1, %2")
        if (OP == 9) CHAIN8("v_mad_u32_u24 %0, %0, %1, %2")
        if (OP == 10) CHAIN8("v_lshlrev_b32 %0, %1, %0")
        if (OP == 11) CHAIN8("v_pk_add_u16 %0, %0, %1")
        if (OP == 12) CHAIN8("v_dot4_u32_u8 %0, %1, %2, %0")
        if (OP == 13) CHAIN8("v_max_u16 %0, %0, %1")
        if (OP == 14) CHAIN8("v_mul_lo_u32 %0, %0, %1")
        if (OP == 15) CHAIN8("v_bfe_u32 %0, %0, %1, %2")
    }
    long long t1 = clock64();
    unsigned s = 0;
    for (int i = 0; i < 8; i++) s ^= x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

typedef void (*KFn)(unsigned*, int, long long*);
template <int... I> struct Tab { static constexpr KFn f[] = {k_rate<I>...}; };

int main()
{
    const int n = 2048;
    unsigned* out; long long* cyc;
    hipMalloc(&out, 4 * 64 * 16384); hipMalloc(&cyc, 8 * 16384);
    const char* names[] = {"v_perm_b32", "v_pk_min_u16", "v_pk_sub_u16 clamp", "v_add_u32", "v_and_b32",
                           "v_dot2_u32_u16", "v_min3_u32", "v_alignbyte_b32", "v_fma_f32", "v_mad_u32_u24",
                           "v_lshlrev_b32", "v_pk_add_u16", "v_dot4_u32_u8", "v_max_u16", "v_mul_lo_u32", "v_bfe_u32"};
    const KFn* fn = Tab<0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15>::f;
    for (int op = 0; op < 16; op++) {
        printf("%-20s", names[op]);
        for (int wps : {1, 2, 4, 8}) {
            const int blocks = 1024 * wps;   // 256 CUs x 4 SIMDs x wps
            hipLaunchKernelGGL(fn[op], dim3(blocks), dim3(64), 0, 0, out, n, cyc);
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(fn[op], dim3(blocks), dim3(64), 0, 0, out, n, cyc);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            const double instr = 8.0 * n;
            printf("  wps=%d: %5.2f cyc/instr/SIMD (wave0 %5.2f) chip %6.1f G/s", wps, c / instr / wps, c / instr,
                   instr * blocks / (ms * 1e-3) / 1e9);
        }
        printf("\n");
    }
    return 0;
}
