// coeb_flow.hip -- Frame::ProcessMovingObject (src/Frame.cc:311-393), the T_M generation of the
// dynamic filter.  Built so far: the corner detector it starts with,
//   cv::goodFeaturesToTrack(imGrayPre, prepoint, 1000, 0.01, 8, Mat(), 3, true, 0.04)  (:333)
// as OpenCV 3.4 computes it (featureselect.cpp; cornerHarris in corner.cpp), in the canonical
// forms the oracle restates (oc_good_features_harris):
//   k_gf_response  per pixel: Sobel 3x3 (REFLECT_101) scaled by 1/3060, cov products, the
//                  unnormalised 3x3 box (row sums then column sum), Harris R in float with the
//                  k term in double; the image maximum by an ordered-int atomicMax
//   k_gf_candidates per pixel: threshold TOZERO at (float)(max * quality), 3x3 dilation, local
//                  maxima appended as (ordered value, index) keys
//   k_gf_select    one workgroup: bitonic sort of the keys (value desc, index desc =
//                  greaterThanPtr), then the greedy minDistance selection over an 8-px cell grid
//                  in LDS, one candidate at a time (the reference's order is sequential)
#include <hip/hip_runtime.h>

#include <cfloat>

#include "coeb_internal.hpp"

namespace {

__device__ __forceinline__ int gf_reflect(int p, int n)
{
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - p - 2;
    return p;
}

// float -> uint order-preserving (for atomicMax and descending sorts)
__device__ __forceinline__ uint32_t f2ord(float f)
{
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t o)
{
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

__global__ __launch_bounds__(256) void k_gf_response(const uint8_t* __restrict__ img, int w, int h, int stride, double k,
                                                     float* __restrict__ R, uint32_t* __restrict__ rmax)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    float r = -FLT_MAX;
    if (x < w && y < h) {
        const double scale = 1.0 / (4.0 * 3.0 * 255.0);
        float A[3][3], B[3][3], C[3][3];
        for (int j = 0; j < 3; j++) {
            const int yy = gf_reflect(y + j - 1, h);
            for (int i = 0; i < 3; i++) {
                const int xx = gf_reflect(x + i - 1, w);
                int p[3][3];
                for (int b = 0; b < 3; b++)
                    for (int a = 0; a < 3; a++)
                        p[b][a] = img[(size_t)gf_reflect(yy + b - 1, h) * stride + gf_reflect(xx + a - 1, w)];
                const int gx = (p[0][2] - p[0][0]) + 2 * (p[1][2] - p[1][0]) + (p[2][2] - p[2][0]);
                const int gy = (p[2][0] - p[0][0]) + 2 * (p[2][1] - p[0][1]) + (p[2][2] - p[0][2]);
                const float dx = (float)((double)gx * scale), dy = (float)((double)gy * scale);
                A[j][i] = dx * dx; B[j][i] = dx * dy; C[j][i] = dy * dy;
            }
        }
        float sa[3], sb[3], sc[3];
        for (int j = 0; j < 3; j++) {
            sa[j] = (A[j][0] + A[j][1]) + A[j][2];
            sb[j] = (B[j][0] + B[j][1]) + B[j][2];
            sc[j] = (C[j][0] + C[j][1]) + C[j][2];
        }
        const float a = (sa[0] + sa[1]) + sa[2], b = (sb[0] + sb[1]) + sb[2], c = (sc[0] + sc[1]) + sc[2];
        const float ac = a * c - b * b, apc = a + c;
        r = (float)((double)ac - (k * (double)apc) * (double)apc);
        R[(size_t)y * w + x] = r;
    }
    // block max, then one atomic per block
    __shared__ uint32_t s_m[4];
    uint32_t o = f2ord(r);
    for (int off = 32; off >= 1; off >>= 1) o = max(o, (uint32_t)__shfl_xor((int)o, off, 64));
    if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = o;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(rmax, max(max(s_m[0], s_m[1]), max(s_m[2], s_m[3])));
}

__global__ __launch_bounds__(256) void k_gf_candidates(const float* __restrict__ R, int w, int h, double quality,
                                                       const uint32_t* __restrict__ rmax, uint64_t* __restrict__ keys,
                                                       int* __restrict__ nkeys, int cap)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x < 1 || y < 1 || x >= w - 1 || y >= h - 1) return;
    const float thr = (float)((double)ord2f(*rmax) * quality);
    auto eig = [&](int xx, int yy) {
        const float r = R[(size_t)yy * w + xx];
        return r > thr ? r : 0.f;
    };
    const float v = eig(x, y);
    if (v == 0.f) return;
    float m = v;
    for (int dy = -1; dy <= 1; dy++)
        for (int dx = -1; dx <= 1; dx++) m = fmaxf(m, eig(x + dx, y + dy));
    if (v != m) return;
    const int pos = atomicAdd(nkeys, 1);
    if (pos < cap) keys[pos] = ((uint64_t)f2ord(v) << 32) | (uint32_t)(y * w + x);   // larger = earlier
}

constexpr int kGfThreads = 1024;
constexpr int kGfSortMax = 16384;          // keys sorted in LDS (128 KB)

__global__ __launch_bounds__(kGfThreads) void k_gf_select(const uint64_t* __restrict__ keys, const int* __restrict__ nkeys,
                                                         int w, int h, int max_corners, float min_distance, int cell,
                                                         float* __restrict__ out_xy, int* __restrict__ nout, int cap)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t* K = reinterpret_cast<uint64_t*>(smem);
    const int tid = threadIdx.x;
    const int n = *nkeys;
    if (n > kGfSortMax) {
        if (tid == 0) *nout = -1;
        return;
    }
    int np = 1;
    while (np < n) np <<= 1;
    for (int i = tid; i < np; i += kGfThreads) K[i] = i < n ? keys[i] : 0ull;
    __syncthreads();
    // bitonic sort, descending
    for (int size = 2; size <= np; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < np; i += kGfThreads) {
                const int j = i ^ stride;
                if (j > i) {
                    const uint64_t a = K[i], b = K[j];
                    const bool desc = (i & size) == 0;
                    if (desc ? (a < b) : (a > b)) { K[i] = b; K[j] = a; }
                }
            }
            __syncthreads();
        }
    // greedy selection (featureselect.cpp minDistance loop): wave 0, lanes 0..8 test the 3x3 cells
    const int gw = (w + cell - 1) / cell, gh = (h + cell - 1) / cell;
    constexpr int kSlots = 16;
    uint32_t* gcnt = reinterpret_cast<uint32_t*>(K + np);               // [gw*gh]
    float2* gpt = reinterpret_cast<float2*>(gcnt + ((gw * gh + 3) & ~3)); // [gw*gh][kSlots]
    for (int g = tid; g < gw * gh; g += kGfThreads) gcnt[g] = 0;
    __syncthreads();
    if (tid >= 64) return;
    const float md2 = min_distance * min_distance;
    int cnt = 0;
    for (int i = 0; i < n; i++) {
        if (max_corners > 0 && cnt >= max_corners) break;
        const int idx = (int)(uint32_t)(K[i] & 0xffffffffu);
        const int y = idx / w, x = idx - y * w;
        const int xc = x / cell, yc = y / cell;
        bool bad = false;
        if (tid < 9) {
            const int xx = xc - 1 + tid % 3, yy = yc - 1 + tid / 3;
            if (xx >= 0 && yy >= 0 && xx < gw && yy < gh) {
                const int g = yy * gw + xx;
                const int m = (int)gcnt[g];
                for (int j = 0; j < m; j++) {
                    const float2 p = gpt[g * kSlots + j];
                    const float ddx = (float)x - p.x, ddy = (float)y - p.y;
                    if (ddx * ddx + ddy * ddy < md2) bad = true;
                }
            }
        }
        if (__ballot(bad) == 0) {
            if (tid == 0) {
                const int g = yc * gw + xc;
                const int m = (int)gcnt[g];
                if (m < kSlots) gpt[g * kSlots + m] = make_float2((float)x, (float)y);
                gcnt[g] = m + 1;
                if (cnt < cap) { out_xy[2 * cnt] = (float)x; out_xy[2 * cnt + 1] = (float)y; }
            }
            cnt++;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    if (tid == 0) *nout = cnt;
}

}  // namespace

size_t gf_select_lds(int w, int h, int cell)
{
    const int gw = (w + cell - 1) / cell, gh = (h + cell - 1) / cell;
    return (size_t)kGfSortMax * 8 + (size_t)((gw * gh + 3) & ~3) * 4 + (size_t)gw * gh * 16 * 8;
}

int launch_good_features(const uint8_t* d_img, int w, int h, int stride, int max_corners, double quality,
                         double min_distance, double k, float* d_R, uint32_t* d_max, uint64_t* d_keys, int* d_nkeys,
                         int key_cap, float* d_out, int* d_nout, int out_cap, hipStream_t s)
{
    const int cell = (int)lrint(min_distance);
    if (cell < 1) return -2;
    const size_t lds = gf_select_lds(w, h, cell);
    if (lds > 160 * 1024) return -2;
    (void)hipMemsetAsync(d_max, 0, 4, s);
    (void)hipMemsetAsync(d_nkeys, 0, 4, s);
    const dim3 grid((w + 15) / 16, (h + 15) / 16);
    hipLaunchKernelGGL(k_gf_response, grid, dim3(256), 0, s, d_img, w, h, stride, k, d_R, d_max);
    hipLaunchKernelGGL(k_gf_candidates, grid, dim3(256), 0, s, d_R, w, h, quality, d_max, d_keys, d_nkeys, key_cap);
    (void)hipFuncSetAttribute((const void*)k_gf_select, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_gf_select, dim3(1), dim3(kGfThreads), lds, s, d_keys, d_nkeys, w, h, max_corners,
                       (float)min_distance, cell, d_out, d_nout, out_cap);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
