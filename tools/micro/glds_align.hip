// Correctness probe: LDS-DMA (global_load_lds_dwordx4 / _dword) at byte-misaligned LDS
// destinations and byte-misaligned global sources on gfx950.  For every shift s in 0..15 one wave
// copies a 1 KiB piece (64 lanes x 16 B, or 64 x 4 B) into LDS and writes the LDS image back;
// the host compares with the expected bytes.  Prints one line per (form, shift): OK or the first
// mismatching byte.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef __attribute__((address_space(3))) void* lds_vp;

// form 0: 16-B lanes, LDS base = slab + 32 - s, source aligned
// form 1: 16-B lanes, LDS base aligned, source + s
// form 2: 4-B lanes, LDS base aligned, source + s
// form 3: 4-B lanes, LDS base = slab + 32 - s, source aligned
__global__ __launch_bounds__(64) void k_probe(const unsigned char* __restrict__ src, unsigned char* __restrict__ out,
                                              int form)
{
    __shared__ __attribute__((aligned(16))) unsigned char slab[2048];
    const int s = blockIdx.x;            // shift 0..15
    const int lane = threadIdx.x;
    for (int i = lane; i < 2048; i += 64) slab[i] = 0xEE;
    __syncthreads();
    if (form == 0) {
        const unsigned char* g = src + 16 * lane;
        __builtin_amdgcn_global_load_lds((const void*)g, (lds_vp)(slab + 32 - s), 16, 0, 0);
    } else if (form == 1) {
        const unsigned char* g = src + s + 16 * lane;
        __builtin_amdgcn_global_load_lds((const void*)g, (lds_vp)(slab + 32), 16, 0, 0);
    } else if (form == 2) {
        const unsigned char* g = src + s + 4 * lane;
        __builtin_amdgcn_global_load_lds((const void*)g, (lds_vp)(slab + 32), 4, 0, 0);
    } else {
        const unsigned char* g = src + 4 * lane;
        __builtin_amdgcn_global_load_lds((const void*)g, (lds_vp)(slab + 32 - s), 4, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);       // vmcnt(0) lgkmcnt(0)
    __syncthreads();
    for (int i = lane; i < 2048; i += 64) out[s * 2048 + i] = slab[i];
}

int main()
{
    const int N = 4096;
    unsigned char* h = (unsigned char*)malloc(N);
    for (int i = 0; i < N; i++) h[i] = (unsigned char)(i * 7 + 3 + (i >> 8));
    unsigned char *dsrc, *dout;
    if (hipMalloc(&dsrc, N) != hipSuccess || hipMalloc(&dout, 16 * 2048) != hipSuccess) return 2;
    hipMemcpy(dsrc, h, N, hipMemcpyHostToDevice);
    unsigned char* o = (unsigned char*)malloc(16 * 2048);
    const char* names[4] = {"dwordx4 lds-dest-misaligned", "dwordx4 src-misaligned", "dword src-misaligned",
                            "dword lds-dest-misaligned"};
    int bad_total = 0;
    for (int form = 0; form < 4; form++) {
        hipLaunchKernelGGL(k_probe, dim3(16), dim3(64), 0, 0, dsrc, dout, form);
        if (hipDeviceSynchronize() != hipSuccess) { printf("form %d: launch failed\n", form); return 3; }
        hipMemcpy(o, dout, 16 * 2048, hipMemcpyDeviceToHost);
        for (int s = 0; s < 16; s++) {
            const int bytes = (form <= 1) ? 1024 : 256;
            const int dst0 = (form == 0 || form == 3) ? 32 - s : 32;
            const int src0 = (form == 1 || form == 2) ? s : 0;
            int bad = -1;
            for (int i = 0; i < 2048 && bad < 0; i++) {
                const int k = i - dst0;
                const unsigned char want = (k >= 0 && k < bytes) ? h[src0 + k] : 0xEE;
                if (o[s * 2048 + i] != want) bad = i;
            }
            if (bad >= 0) {
                bad_total++;
                printf("%-30s s=%2d MISMATCH at lds byte %d: got %02x", names[form], s, bad, o[s * 2048 + bad]);
                // where did the first piece land?
                int found = -1;
                for (int i = 0; i + 8 <= 2048 && found < 0; i++)
                    if (!memcmp(&o[s * 2048 + i], &h[src0], 8)) found = i;
                int foundA = -1;
                for (int i = 0; i + 8 <= 2048 && foundA < 0; i++)
                    if (!memcmp(&o[s * 2048 + i], &h[src0 & ~3], 8)) foundA = i;
                printf("  (src[0..7] found at lds %d, src aligned-down at %d; expected %d)\n", found, foundA, dst0);
            } else {
                printf("%-30s s=%2d OK\n", names[form], s);
            }
        }
    }
    printf("glds_align: %d mismatching cases\n", bad_total);
    return 0;
}
