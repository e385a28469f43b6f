// Microbenchmark: chip-wide VALU throughput of single ops on gfx950 with k waves per SIMD
// (256-thread workgroups = one wave per SIMD each, k workgroups per CU, grid = CUs x k).  16
// independent chains per lane, long enough (n iterations) that dispatch ramp-up is noise.  Every
// wave records its s_memtime (shader clock) and s_memrealtime (100 MHz) span, so the output
// gives: the shader clock during the run, the fraction of the launch during which all waves ran
// together, and cycles per wave-instruction per SIMD over the launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CHAIN16(ASM)                                                                                \
    _Pragma("unroll") for (int i = 0; i < 16; i++) asm volatile(ASM : "+v"(x[i]) : "v"(y), "v"(z));

template <int OP>
__global__ __launch_bounds__(256) void k_rate(unsigned* out, int n, long long* st)
{
    unsigned x[16];
    unsigned y = threadIdx.x * 0x01010101u + 7, z = 0x05040302u ^ threadIdx.x;
    for (int i = 0; i < 16; i++) x[i] = threadIdx.x * 3 + i;
    const long long c0 = clock64(), r0 = wall_clock64();
    for (int k = 0; k < n; k++) {
        if (OP == 0) CHAIN16("v_perm_b32 %0, %1, %0, %2")
        if (OP == 1) CHAIN16("v_pk_min_u16 %0, %0, %1")
        if (OP == 2) CHAIN16("v_add_u32 %0, %0, %1")
        if (OP == 3) CHAIN16("v_fma_f32 %0, %0, %1, %2")
        if (OP == 4) CHAIN16("v_mul_u32_u24 %0, %0, %1")
        if (OP == 5) CHAIN16("v_min3_u32 %0, %0, %1, %2")
        if (OP == 6) CHAIN16("v_dot2_u32_u16 %0, %1, %2, %0")
        if (OP == 7) CHAIN16("v_max_u32 %0, %0, %1")
    }
    const long long c1 = clock64(), r1 = wall_clock64();
    unsigned s = 0;
    for (int i = 0; i < 16; i++) s ^= x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        long long* o = st + 4 * (blockIdx.x * 4 + (threadIdx.x >> 6));
        o[0] = c0; o[1] = c1; o[2] = r0; o[3] = r1;
    }
}

typedef void (*KFn)(unsigned*, int, long long*);
template <int... I> struct Tab { static constexpr KFn f[] = {k_rate<I>...}; };

int main()
{
    const int n = 16384;
    unsigned* out; long long* st;
    (void)hipMalloc(&out, 4 * 256 * 4096); (void)hipMalloc(&st, 32 * 4 * 4096);
    const char* names[] = {"v_perm_b32", "v_pk_min_u16", "v_add_u32", "v_fma_f32", "v_mul_u32_u24",
                           "v_min3_u32", "v_dot2_u32_u16", "v_max_u32"};
    const KFn* fn = Tab<0, 1, 2, 3, 4, 5, 6, 7>::f;
    hipDeviceProp_t pr; (void)hipGetDeviceProperties(&pr, 0);
    const int ncu = pr.multiProcessorCount;
    printf("CUs %d; columns per wps: cycles per wave-instr per SIMD over the launch | shader GHz | "
           "all-waves-together fraction of the launch | per-wave cycles per instr\n", ncu);
    for (int op = 0; op < 8; op++) {
        printf("%-16s", names[op]);
        for (int k : {1, 2, 4, 8}) {
            const int blocks = ncu * k, waves = blocks * 4;
            hipLaunchKernelGGL(fn[op], dim3(blocks), dim3(256), 0, 0, out, 256, st);
            hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(fn[op], dim3(blocks), dim3(256), 0, 0, out, n, st);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            std::vector<long long> h(4 * waves);
            (void)hipMemcpy(h.data(), st, 32 * waves, hipMemcpyDeviceToHost);
            long long rs = 0, re = 1LL << 62, rmin = 1LL << 62, rmax = 0;
            double cyc_sum = 0, rt_sum = 0;
            for (int w = 0; w < waves; w++) {
                rs = std::max(rs, h[4 * w + 2]); re = std::min(re, h[4 * w + 3]);
                rmin = std::min(rmin, h[4 * w + 2]); rmax = std::max(rmax, h[4 * w + 3]);
                cyc_sum += h[4 * w + 1] - h[4 * w]; rt_sum += h[4 * w + 3] - h[4 * w + 2];
            }
            const double ghz = cyc_sum / rt_sum / 10.0;        // realtime ticks at 100 MHz
            const double together = re > rs ? double(re - rs) / double(rmax - rmin) : 0.0;
            const double instr = 16.0 * n;
            const double span_cyc = double(rmax - rmin) * 10.0 * ghz;
            printf(" | wps=%d %5.2f %4.2fGHz %4.2f %5.2f", k, span_cyc / (instr * k), ghz, together,
                   cyc_sum / waves / instr);
        }
        printf("\n");
    }
    return 0;
}
