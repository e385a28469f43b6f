// Microbenchmark: per-wave issue cost of f64 / f32 VALU ops on gfx950 (one wave per SIMD and
// four waves per SIMD), 8 independent chains per lane.  Prints cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(64) void k_rate(double* out, float* outf, int n, long long* cyc)
{
    double d[8];
    float f[8];
    for (int i = 0; i < 8; i++) { d[i] = 1.0 + threadIdx.x * 1e-3 + i; f[i] = 1.f + threadIdx.x * 1e-3f + i; }
    const double m = 1.0000001, a = 1e-9;
    const float mf = 1.0000001f, af = 1e-9f;
    long long t0 = clock64();
    for (int k = 0; k < n; k++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (OP == 0) d[i] = d[i] * m;
            if (OP == 1) d[i] = d[i] + a;
            if (OP == 2) d[i] = __builtin_fma(d[i], m, a);
            if (OP == 3) f[i] = f[i] * mf;
            if (OP == 4) f[i] = __builtin_fmaf(f[i], mf, af);
            if (OP == 5) d[i] = (double)(float)d[i];
        }
    }
    long long t1 = clock64();
    double s = 0; float sf = 0;
    for (int i = 0; i < 8; i++) { s += d[i]; sf += f[i]; }
    out[blockIdx.x * 64 + threadIdx.x] = s;
    outf[blockIdx.x * 64 + threadIdx.x] = sf;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main()
{
    const int n = 4096;
    double* out; float* of; long long* cyc;
    hipMalloc(&out, 8 * 64 * 8192); hipMalloc(&of, 4 * 64 * 8192); hipMalloc(&cyc, 8 * 8192);
    const char* names[] = {"v_mul_f64", "v_add_f64", "v_fma_f64", "v_mul_f32", "v_fma_f32", "cvt f64->f32->f64 (2 ops)"};
    for (int blocks : {1024, 4096}) {
        for (int op = 0; op < 6; op++) {
            void (*kern)(double*, float*, int, long long*) =
                op == 0 ? k_rate<0> : op == 1 ? k_rate<1> : op == 2 ? k_rate<2> : op == 3 ? k_rate<3> : op == 4 ? k_rate<4> : k_rate<5>;
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, of, n, cyc);
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, of, n, cyc);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("%-28s waves=%5d  wave0 cycles/instr %.2f  chip: %.1f G wave-instr/s\n", names[op], blocks,
                   (double)c / (8.0 * n), (double)blocks * 8 * n / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
