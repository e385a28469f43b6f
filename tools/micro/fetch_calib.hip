// FETCH_SIZE calibration on gfx950 for the extraction kernels' load shapes.
// Each kernel reads a 1.2 GB buffer (past the 256 MiB Infinity Cache) exactly once in the
// instruction shape of one of the product kernels, so the true HBM read bytes are the buffer size;
// rocprofv3 --pmc FETCH_SIZE of each dispatch divided by that size is the pattern's scale.
//   k_stream    : 16 B per lane, consecutive lanes consecutive (the guide's calibrated case)
//   k_fast_rows : k_fast's register staging: lane = (row lane>>2, 16-B chunk lane&3), three loads
//                 per lane at rows r, r+16, r+32 of a 64-B wide, 48-row window (4 chunks x 48 rows)
//   k_fast_dma  : k_fast's LDS-DMA staging: chunks 0..2 of each 96-B slab row from byte-granular
//                 (misaligned) rows of 48 B, 1 KiB LDS pieces (global_load_lds_dwordx4)
//   k_desc_rows : k_describe's patch staging: 37 rows x 64 B per keypoint, 4 lanes per row,
//                 16 rows per load instruction
//   k_dword     : 4 B per lane, consecutive (the pyramid/blur kernels' dword loads)
// Windows tile the buffer without overlap, so every byte is requested exactly once.
// Usage: fetch_calib  (prints the bytes each kernel requests; the FETCH_SIZE pass does the rest)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vp;

constexpr int kPitch = 4096;                // bytes per "image row"
constexpr int64_t kRows = 300 * 1024;       // 1.2 GB

__global__ __launch_bounds__(256) void k_stream(const uint8_t* __restrict__ p, int64_t n, unsigned* out)
{
    u32x4 acc = {0, 0, 0, 0};
    for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 16; i < n; i += (int64_t)gridDim.x * 256 * 16)
        acc ^= *reinterpret_cast<const u32x4*>(p + i);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

__global__ __launch_bounds__(64) void k_dword(const uint8_t* __restrict__ p, int64_t n, unsigned* out)
{
    unsigned acc = 0;
    for (int64_t i = ((int64_t)blockIdx.x * 64 + threadIdx.x) * 4; i < n; i += (int64_t)gridDim.x * 64 * 4)
        acc ^= *reinterpret_cast<const unsigned*>(p + i);
    if (acc == 0x12345678u) out[0] = 1;
}

// one wave per 64-B x 48-row window; windows tile the buffer (pitch / 64 per row band)
__global__ __launch_bounds__(256) void k_fast_rows(const uint8_t* __restrict__ p, unsigned* out)
{
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t band = w / (kPitch / 64), col = w % (kPitch / 64);
    if (band * 48 >= kRows) return;
    const uint8_t* base = p + band * 48 * kPitch + col * 64 + 16 * (lane & 3);
    const int r = lane >> 2;
    const u32x4 a = *reinterpret_cast<const u32x4*>(base + (int64_t)r * kPitch);
    const u32x4 b = *reinterpret_cast<const u32x4*>(base + (int64_t)(r + 16) * kPitch);
    const u32x4 c = *reinterpret_cast<const u32x4*>(base + (int64_t)(r + 32) * kPitch);
    const u32x4 x = a ^ b ^ c;
    if ((x.x ^ x.y ^ x.z ^ x.w) == 0x12345678u) out[0] = 1;
}

// one wave per 48-B x 48-row window starting at a byte offset s = w mod 16 inside its 64-B slot
// (the misaligned rows of the DMA staging); bytes requested = 48 x 48 per window
__global__ __launch_bounds__(256) void k_fast_dma(const uint8_t* __restrict__ p, unsigned* out)
{
    __shared__ __attribute__((aligned(16))) uint8_t slab[4][48 * 96 + 1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t w = (int64_t)blockIdx.x * 4 + wv;
    const int64_t band = w / (kPitch / 64), col = w % (kPitch / 64);
    if (band * 48 >= kRows) return;
    const uint8_t* row0 = p + band * 48 * kPitch + col * 64 + (int)(w & 15);
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const int q = 64 * i + lane;
        const int r = (q * 171) >> 10;
        const int k = q - 6 * r;
        if (q < 6 * 48 && k < 3)
            __builtin_amdgcn_global_load_lds((const void*)(row0 + (int64_t)r * kPitch + 16 * k),
                                             (lds_vp)(&slab[wv][1024 * i]), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (slab[wv][lane * 7] == 0xAB && slab[wv][lane * 7 + 1] == 0xCD) out[0] = 1;
}

// one wave per 64-B x 37-row patch; patches tile the buffer in 37-row bands
__global__ __launch_bounds__(256) void k_desc_rows(const uint8_t* __restrict__ p, unsigned* out)
{
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t band = w / (kPitch / 64), col = w % (kPitch / 64);
    if ((band + 1) * 37 > kRows) return;
    const uint8_t* base = p + band * 37 * kPitch + col * 64 + 16 * (lane & 3);
    u32x4 x = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const int r = (lane >> 2) + 16 * i;
        if (r < 37) x ^= *reinterpret_cast<const u32x4*>(base + (int64_t)r * kPitch);
    }
    if ((x.x ^ x.y ^ x.z ^ x.w) == 0x12345678u) out[0] = 1;
}

int main()
{
    const int64_t n = kRows * kPitch;
    uint8_t* p;
    unsigned* out;
    if (hipMalloc(&p, n) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) { printf("alloc failed\n"); return 2; }
    if (hipMemset(p, 1, n) != hipSuccess) return 2;
    const int64_t win48 = (kRows / 48) * (kPitch / 64), win37 = (kRows / 37) * (kPitch / 64);
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_stream, dim3(256 * 64), dim3(256), 0, 0, p, n, out);
        hipLaunchKernelGGL(k_dword, dim3(256 * 64), dim3(64), 0, 0, p, n, out);
        hipLaunchKernelGGL(k_fast_rows, dim3((unsigned)((win48 + 3) / 4)), dim3(256), 0, 0, p, out);
        hipLaunchKernelGGL(k_fast_dma, dim3((unsigned)((win48 + 3) / 4)), dim3(256), 0, 0, p, out);
        hipLaunchKernelGGL(k_desc_rows, dim3((unsigned)((win37 + 3) / 4)), dim3(256), 0, 0, p, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 3; }
    printf("requested bytes per dispatch:\n");
    printf("k_stream %lld\nk_dword %lld\nk_fast_rows %lld\nk_fast_dma %lld\nk_desc_rows %lld\n", (long long)n, (long long)n,
           (long long)(win48 * 48 * 64), (long long)(win48 * 48 * 48), (long long)(win37 * 37 * 64));
    return 0;
}
