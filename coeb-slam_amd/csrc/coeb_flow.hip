// coeb_flow.hip -- Frame::ProcessMovingObject (src/Frame.cc:311-393), the T_M generation of the
// dynamic filter, as OpenCV 3.4 computes each call, in the canonical
// forms the oracle restates (oracle/orb_oracle.c):
//
//   goodFeaturesToTrack(imGrayPre, prepoint, 1000, 0.01, 8, Mat(), 3, true, 0.04)     (:333)
//     k_gf_response    Sobel 3x3 (REFLECT_101) / 3060, cov products, unnormalised 3x3 box, Harris R
//                      (k term in double): one wave per 60-column strip, lane = column sliding
//                      down, neighbours by DPP wave shifts; image max by ordered-int atomicMax
//     k_gf_candidates  per pixel: TOZERO at (float)(max*quality), 3x3 dilation, local maxima as
//                      (ordered value, index) keys
//     k_gf_select      one workgroup: the keys in 4096-key batches of rank order (MSB radix select
//                      + bitonic sort in LDS), walked 64 at a time by one wave against per-cell
//                      lists of accepted corners -- the sequential greedy minDistance result
//   cornerSubPix(imGrayPre, prepoint, Size(10,10), Size(-1,-1), (ITER|EPS, 20, 0.03))   (:334)
//     k_subpix         nine corner slots per wave: rolling getRectSubPix rows, per-row terms of
//                      every slot, one add instruction per term serves nine corners; the five sums
//                      in double in the reference's order
//   calcOpticalFlowPyrLK(imGrayPre, imgray, .., Size(22,22), 5, (ITER|EPS, 20, 0.01))   (:335)
//     k_pyr_down       pyrDown 5x5 [1 4 6 4 1]^2 per level, lane = output column sliding down a strip
//     k_sharr          calcSharrDeriv of every level of the previous frame in one launch
//     k_lk             one wave per point, levels coarse to fine; a 3x3 pixel tile per lane, window
//                      sums exact (int32 per lane, DPP wave reduction of the 16-bit halves)
//   SAD check (:337-365), findFundamentalMat(.., FM_RANSAC, 0.1, 0.99) (:373), epipolar
//   distance > 1 -> T_M (:375-384)
//     k_fm             one workgroup: SAD filter + ordered compaction into LDS, RANSAC in
//                      chunks of 32 hypotheses (RNG draws on lane 0, 7-point solves on 32
//                      lanes, inlier counts one wave per model, the reference's sequential
//                      best-model / niters scan on lane 0), LMeDS for 8..14 pairs, the
//                      epipolar test and ordered T_M compaction
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <array>
#include <map>
#include <mutex>

#include "../../include/coeb_front.h"
#include "coeb_internal.hpp"

extern "C" int coeb_internal_stream(coeb_ctx* c, hipStream_t* s, int* device);
extern "C" int coeb_internal_scratch(coeb_ctx* c, const char* name, size_t bytes, void** p);
extern "C" int coeb_internal_error(coeb_ctx* c, int code, const char* msg);
extern "C" ProfileHook* coeb_internal_prof(coeb_ctx* c);
extern "C" void coeb_internal_flow_forget(const coeb_ctx* c);
extern "C" int coeb_internal_flow_side(coeb_ctx* c, hipStream_t* side, hipEvent_t* fork, hipEvent_t* join);

namespace {

__device__ int g_subpix_count_dev[4];   // {cornerSubPix iterations, corners, LK iterations, points}
int* g_subpix_count = nullptr;    // device address of g_subpix_count_dev (COEB_SUBPIX_COUNT, A/B tool)

constexpr int kMaxPts = 1024;        // corners / tracked points per call (reference: 1000)
// k_gf_select's workgroup: 256 threads (a config-D pair has ~270 local maxima: its sort stages and
// barriers are cheaper with 4 waves than with 16, and four times as many pairs fit the CUs):
// 0.39 -> 0.25 ms per 1537-pair launch, config-D step 35.8 -> 35.4 ms (512: 0.235 ms, 35.4-35.5;
// profiles/r06/s7)
constexpr int kGfThreads = 256;
// local-maximum keys kept per frame: a quarter of the pixels (a 3 x 3 maximum needs its
// neighbours below it unless the response plateaus); more is reported as -1
inline int gf_key_cap(int w, int h) { return std::max(16384, w * h / 4); }
constexpr int kLkMaxLevels = 8;
constexpr int kFmThreads = 128;     // threads per pair of k_fm (COEB_FM_THREADS: 128 / 256 / 512 / 1024)
constexpr int kFmChunk = 32;         // RANSAC hypotheses per chunk

__device__ __forceinline__ int reflect101(int p, int n)
{
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - p - 2;
    return p;
}

// float -> uint order-preserving (atomicMax, descending sorts)
__device__ __forceinline__ uint32_t f2ord(float f)
{
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t o)
{
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

__device__ __forceinline__ int cv_floor(float v)
{
    const int i = (int)v;
    return i - (i > v);
}

// Batched calls (coeb_moving_object_points_batch_device): blockIdx.z = frame pair.  Every
// per-pair buffer lives in one block of `pz` bytes per pair, so a kernel reaches its pair's
// buffers by one byte offset; pair z's frames are the batch's frames z and z + 1, `iz` bytes
// apart.  Single calls pass iz = pz = 0 and one z-slice.
template <class T>
__device__ __forceinline__ T* at_pair(T* p, int64_t stride, uint32_t z)
{
    return p ? reinterpret_cast<T*>(reinterpret_cast<uintptr_t>(p) + (uint64_t)z * (uint64_t)stride) : p;
}
template <class T>
__device__ __forceinline__ T* at_pair(T* p, int64_t stride)
{
    return at_pair(p, stride, blockIdx.z);
}

// Per-point kernels of a batch (cornerSubPix, LK) run over one flattened work list instead of a
// grid of kMaxPts slots per pair: offs[z] = points before pair z (k_flow_index), offs[P] = all.
// A grid of P x 1024 one-wave slots of which ~150 per pair hold a point was bound by the rate
// at which the dispatcher retires empty waves (262,144 waves in ~1.5 ms for both kernels).
// item -> (pair, point) by a binary search over offs.
// (pair, index) of a flattened item packed in one int: index < kMaxPts = 2^kFlowIdxBits
constexpr int kFlowIdxBits = 10;
static_assert(kMaxPts <= (1 << kFlowIdxBits), "flow_code index field");
__device__ __forceinline__ int flow_code(int2 zp) { return (zp.x << kFlowIdxBits) | zp.y; }
__device__ __forceinline__ int2 flow_decode(int c) { return make_int2(c >> kFlowIdxBits, c & ((1 << kFlowIdxBits) - 1)); }

__device__ __forceinline__ int2 flow_item(const int* __restrict__ offs, int P, int item)
{
    int lo = 0, hi = P;                        // offs[lo] <= item < offs[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (offs[mid] <= item) lo = mid;
        else hi = mid;
    }
    return make_int2(lo, item - offs[lo]);
}

// offs[z] = sum over pairs < z of clamp(n_z, 0, nmax) (n_z at d_n + z * pz bytes), offs[P] = total
__global__ __launch_bounds__(1024) void k_flow_index(const int* __restrict__ d_n, int64_t pz, int P, int nmax,
                                                      int* __restrict__ offs)
{
    __shared__ int s_w[16];
    __shared__ int s_base;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    for (int c0 = 0; c0 < P; c0 += 1024) {
        const int z = c0 + (int)threadIdx.x;
        int v = 0;
        if (z < P) {
            v = *at_pair(d_n, pz, (uint32_t)z);
            v = v < 0 ? 0 : v > nmax ? nmax : v;
        }
        int incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) s_w[wv] = incl;
        __syncthreads();
        int before = s_base, total = s_base;
        for (int i = 0; i < 16; i++) {
            before += i < wv ? s_w[i] : 0;
            total += s_w[i];
        }
        if (z < P) offs[z] = before + incl - v;
        __syncthreads();
        if (threadIdx.x == 0) s_base = total;
        __syncthreads();
    }
    if (threadIdx.x == 0) offs[P] = s_base;
}

// ============================== goodFeaturesToTrack ==============================
// Harris response, one wave per strip of 60 output columns x kGfRows rows, lane = column
// (x0 - 2 + lane; lanes 2..61 produce).  Each lane slides down its column: a new pixel row
// enters, its left / right neighbours come from the adjacent lanes (DPP wave shifts), the Sobel
// products of the row above are formed, their 3-wide row sums take the neighbours' products the
// same way, and three row sums down give the box sum -- in the reference's order (left to right,
// then top to bottom).  Nothing goes through LDS.  (Round 2 staged Sobel products of 32 x 32
// tiles in LDS: ~130 VALU lane-operations per pixel, 0.47 ms per 256 pairs.)
// Borders (REFLECT_101, boxFilter over Sobel products that are themselves computed with
// reflected taps): a lane / row outside the image loads the reflected pixel, so its Sobel is the
// mirror image of the reflected position's -- gx (column -1, w) or gy (row -1, h) negated
// exactly -- and only the cross product dx*dy changes sign; it is negated back.
constexpr int kGfRows = 32;
constexpr int kGfCols = 60;
__device__ __forceinline__ int wave_shr1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, false); }  // lane i <- i-1
__device__ __forceinline__ int wave_shl1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, false); }  // lane i <- i+1
__device__ __forceinline__ float wave_shr1f(float v) { return __int_as_float(wave_shr1(__float_as_int(v))); }
__device__ __forceinline__ float wave_shl1f(float v) { return __int_as_float(wave_shl1(__float_as_int(v))); }

__global__ __launch_bounds__(256) void k_gf_response(const uint8_t* __restrict__ img, int w, int h, int stride, double k,
                                                     float* __restrict__ R, uint32_t* __restrict__ rmax, int64_t iz,
                                                     int64_t pz)
{
    img = at_pair(img, iz);
    R = at_pair(R, pz);
    rmax = at_pair(rmax, pz);
    const int lane = threadIdx.x & 63;
    const int strip = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int x0 = strip * kGfCols, y0 = blockIdx.y * kGfRows;
    if (x0 >= w) return;
    const int c = x0 - 2 + lane;                       // this lane's column
    const int cr = reflect101(c, w);
    const bool produce = lane >= 2 && lane < 2 + kGfCols && c < w;
    const float xsgn = (c == -1 || c == w) ? -1.f : 1.f;
    const double scale = 1.0 / (4.0 * 3.0 * 255.0);
    const uint8_t* col = img + cr;
    // pixel rows y-1, y of the Sobel being formed (own column, left, right)
    int pm = 0, pl_m = 0, pr_m = 0, p0 = 0, pl_0 = 0, pr_0 = 0;
    // row sums of the products of the last two product rows
    float ra0 = 0, rb0 = 0, rc0 = 0, ra1 = 0, rb1 = 0, rc1 = 0;
    float rmx = -FLT_MAX;
    const int y1 = min(h, y0 + kGfRows);
    // pixel rows y0-2 .. y1+1: product rows y0-1 .. y1, output rows y0 .. y1-1; all of the band's
    // pixel loads are issued before the first is used (one byte per lane each: a row-at-a-time
    // loop waited a memory round trip per row)
    int pvv[kGfRows + 4];
#pragma unroll
    for (int i = 0; i < kGfRows + 4; i++) {
        const int yy = y0 - 2 + i;
        pvv[i] = yy <= y1 + 1 ? (int)col[(int64_t)reflect101(yy, h) * stride] : 0;
    }
#pragma unroll
    for (int i = 0; i < kGfRows + 4; i++) {
        const int yy = y0 - 2 + i;
        if (yy > y1 + 1) break;
        const int pv = pvv[i];
        const int pl = wave_shr1(pv), pr = wave_shl1(pv);
        if (yy >= y0) {                                 // Sobel / products of row yy - 1
            const int gx = (pr_m - pl_m) + 2 * (pr_0 - pl_0) + (pr - pl);
            const int gy = (pl - pl_m) + 2 * (pv - pm) + (pr - pr_m);
            const float dx = (float)((double)gx * scale), dy = (float)((double)gy * scale);
            const int yp = yy - 1;
            const float sgn = (yp == -1 || yp == h) ? -xsgn : xsgn;
            const float A = dx * dx, B = (dx * dy) * sgn, C = dy * dy;
            const float ra = (wave_shr1f(A) + A) + wave_shl1f(A);
            const float rb = (wave_shr1f(B) + B) + wave_shl1f(B);
            const float rc = (wave_shr1f(C) + C) + wave_shl1f(C);
            if (yy >= y0 + 2) {                         // output row yy - 2
                const float a = (ra0 + ra1) + ra, b = (rb0 + rb1) + rb, cc = (rc0 + rc1) + rc;
                const float ac = a * cc - b * b, apc = a + cc;
                const float r = (float)((double)ac - (k * (double)apc) * (double)apc);
                if (produce) {
                    R[(size_t)(yy - 2) * w + c] = r;
                    rmx = fmaxf(rmx, r);
                }
            }
            ra0 = ra1; rb0 = rb1; rc0 = rc1;
            ra1 = ra; rb1 = rb; rc1 = rc;
        }
        pm = p0; pl_m = pl_0; pr_m = pr_0;
        p0 = pv; pl_0 = pl; pr_0 = pr;
    }
    uint32_t o = f2ord(rmx);
    for (int off = 32; off >= 1; off >>= 1) o = max(o, (uint32_t)__shfl_xor((int)o, off, 64));
    if (lane == 0) atomicMax(rmax, o);
}

// Candidates: TOZERO at thr, 3x3 dilation, local maxima (v != 0, v == its 3x3 max) appended as
// keys (append order is free: k_gf_select sorts them).  One wave per strip of kGcCols columns x
// kGcRows rows, lane = column (x0 - 1 + lane; lanes 1..62 produce): every thresholded value of the
// band (+1 row above and below) is loaded once, all rows up front, the vertical 3-max slides down
// the column and the horizontal one takes the neighbours' by DPP wave shifts.  max is exact, so
// the 9-value order of the per-pixel form does not matter.  (The per-pixel form read each value
// nine times: 0.44 ms per 513 pairs.)
constexpr int kGcCols = 62, kGcRows = 32;
__global__ __launch_bounds__(256) void k_gf_candidates(const float* __restrict__ R, int w, int h, double quality,
                                                       const uint32_t* __restrict__ rmax, uint64_t* __restrict__ keys,
                                                       int* __restrict__ nkeys, int cap, int64_t pz)
{
    R = at_pair(R, pz);
    rmax = at_pair(rmax, pz);
    keys = at_pair(keys, pz);
    nkeys = at_pair(nkeys, pz);
    const int lane = threadIdx.x & 63;
    const int x0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * kGcCols, y0 = blockIdx.y * kGcRows;
    if (x0 >= w) return;
    const int c = x0 - 1 + lane;
    const bool incol = c >= 0 && c < w;
    const bool produce = lane >= 1 && lane <= kGcCols && c >= 1 && c < w - 1;
    const float thr = (float)((double)ord2f(*rmax) * quality);
    float e[kGcRows + 2];                              // rows y0 - 1 .. y0 + kGcRows
#pragma unroll
    for (int i = 0; i < kGcRows + 2; i++) {
        const int yy = y0 - 1 + i;
        const float r = incol && yy >= 0 && yy < h ? R[(size_t)yy * w + c] : 0.f;
        e[i] = r > thr ? r : 0.f;
    }
#pragma unroll
    for (int i = 1; i <= kGcRows; i++) {
        const int y = y0 - 1 + i;
        const float vm = fmaxf(fmaxf(e[i - 1], e[i]), e[i + 1]);
        const float m = fmaxf(fmaxf(wave_shr1f(vm), vm), wave_shl1f(vm));
        const float v = e[i];
        if (produce && y >= 1 && y < h - 1 && v != 0.f && v == m) {
            const int pos = atomicAdd(nkeys, 1);
            if (pos < cap) keys[pos] = ((uint64_t)f2ord(v) << 32) | (uint32_t)(y * w + c);   // larger = earlier
        }
    }
}

// block-wide exclusive prefix of a per-thread count (NT threads, any counts); returns the total
template <int NT>
__device__ int block_scan_counts(int cnt, int* s_w, int& excl)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int x = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    __syncthreads();
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    int base = 0, total = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) {
        base += i < wv ? s_w[i] : 0;
        total += s_w[i];
    }
    excl = base + x - cnt;
    return total;
}

// Greedy minDistance selection (featureselect.cpp): candidates in sorted order (value desc,
// address desc); a candidate is accepted unless an accepted corner in one of the 3 x 3 grid
// cells around it lies closer than minDistance; stop at maxCorners.
//   * The keys are taken kGfBatch at a time in rank order: when more remain, an 8-bit MSB
//     radix select over the global key list finds the batch's smallest key (the kGfBatch-th
//     largest key below the previous batch's); the batch is gathered, bitonic-sorted in LDS and
//     walked before the next is taken, so any number of maxima is selected exactly with 48 KB of
//     LDS.  (Round 2 sorted up to 16384 keys in 150 KB of LDS: such a workgroup cannot share a
//     CU with the pose stream's k_pose and waited for it, 0.6-0.7 ms per 256 pairs.)
//   * The accepted corners are per-cell linked lists in LDS.  One wave walks a sorted batch 64
//     candidates at a time: each lane tests its candidate against the corners accepted before the
//     chunk, then against the earlier candidates of the chunk (a 64-bit conflict mask), and a
//     scalar pass over the chunk's lanes resolves the in-chunk dependencies in order -- the
//     sequential result.  (A block-wide Jacobi fixpoint over the whole list needed one block
//     pass per link of the longest conflict chain.)
constexpr uint16_t kGfNone = 0xFFFF;
constexpr int kGfBatch = 4096;
__global__ __launch_bounds__(kGfThreads) void k_gf_select(const uint64_t* __restrict__ keys, const int* __restrict__ nkeys,
                                                         int w, int h, int max_corners, float md2, int cell,
                                                         float* __restrict__ out_xy, int* __restrict__ nout, int cap,
                                                         int key_cap, int64_t pz)
{
    keys = at_pair(keys, pz);
    nkeys = at_pair(nkeys, pz);
    out_xy = at_pair(out_xy, pz);
    nout = at_pair(nout, pz);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t* K = reinterpret_cast<uint64_t*>(smem);                                  // [kGfBatch]
    const int gw = (w + cell - 1) / cell, gh = (h + cell - 1) / cell;
    uint16_t* head = reinterpret_cast<uint16_t*>(K + kGfBatch);    // [gw * gh] first accepted corner of the cell
    uint16_t* next = head + ((gw * gh + 1) & ~1);                   // [kMaxPts] next accepted corner of its cell
    uint32_t* axy = reinterpret_cast<uint32_t*>(next + kMaxPts);    // [kMaxPts] accepted x | y << 16
    __shared__ uint32_t s_hist[256];
    __shared__ uint64_t s_prefix;
    __shared__ int s_need, s_cnt, s_nacc, s_full;
    const int tid = threadIdx.x, lane = tid & 63;
    const int nall = *nkeys;
    if (nall > key_cap) {                          // more local maxima than the key buffer holds
        if (tid == 0) *nout = -1;
        return;
    }
    for (int g = tid; g < gw * gh; g += kGfThreads) head[g] = kGfNone;
    if (tid == 0) { s_nacc = 0; s_full = 0; }
    const int limit = min(max_corners > 0 ? max_corners : kMaxPts, min(cap, kMaxPts));
    uint64_t U = ~0ull;                            // keys of later batches are < U (keys are unique)
    bool first = true;
    __syncthreads();
    for (int done = 0; done < nall && !s_full; ) {
        const int m = min(kGfBatch, nall - done);
        uint64_t T = 0;                            // this batch: keys in [T, U)
        if (nall - done > kGfBatch) {
            if (tid == 0) { s_prefix = 0; s_need = kGfBatch; }
            for (int shift = 56; shift >= 0; shift -= 8) {
                for (int b = tid; b < 256; b += kGfThreads) s_hist[b] = 0;
                __syncthreads();
                const uint64_t pre = s_prefix;
                for (int i = tid; i < nall; i += kGfThreads) {
                    const uint64_t k = keys[i];
                    if ((first || k < U) && (shift == 56 || (k >> (shift + 8)) == (pre >> (shift + 8))))
                        atomicAdd(&s_hist[(k >> shift) & 255u], 1u);
                }
                __syncthreads();
                if (tid == 0) {
                    int need = s_need, b = 255;
                    while (b > 0 && (int)s_hist[b] < need) need -= (int)s_hist[b--];
                    s_need = need;
                    s_prefix = pre | ((uint64_t)b << shift);
                }
                __syncthreads();
            }
            T = s_prefix;                          // the kGfBatch-th largest key below U
        }
        if (tid == 0) s_cnt = 0;
        __syncthreads();
        if (first && m == nall) {
            for (int i = tid; i < nall; i += kGfThreads) K[i] = keys[i];
        } else {
            for (int i = tid; i < nall; i += kGfThreads) {
                const uint64_t k = keys[i];
                if ((first || k < U) && k >= T) K[atomicAdd(&s_cnt, 1)] = k;
            }
        }
        int np = 1;
        while (np < m) np <<= 1;
        for (int i = m + tid; i < np; i += kGfThreads) K[i] = 0ull;
        __syncthreads();
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
        if (tid < 64) {                            // the selection is one wave's
            int nacc = s_nacc;
            bool full = false;
            for (int c0 = 0; c0 < m && !full; c0 += 64) {
                const int i = c0 + lane;
                const bool valid = i < m;
                const int idx = valid ? (int)(uint32_t)K[i] : 0;
                const int y = idx / w, x = idx - y * w;
                const int xc = x / cell, yc = y / cell;
                const float fx = (float)x, fy = (float)y;
                bool hit = false;
                if (valid) {
                    for (int yy = max(yc - 1, 0); yy <= min(yc + 1, gh - 1) && !hit; yy++)
                        for (int xx = max(xc - 1, 0); xx <= min(xc + 1, gw - 1) && !hit; xx++)
                            for (int a = head[yy * gw + xx]; a != kGfNone; a = next[a]) {
                                const uint32_t q = axy[a];
                                const float ddx = fx - (float)(int)(q & 0xFFFFu), ddy = fy - (float)(int)(q >> 16);
                                if (ddx * ddx + ddy * ddy < md2) { hit = true; break; }
                            }
                }
                // earlier candidates of this chunk that would suppress this one once accepted
                uint64_t conf = 0;
                const int nc = min(64, m - c0);
                for (int j = 0; j < nc; j++) {
                    const int xj = __builtin_amdgcn_readlane(x, j), yj = __builtin_amdgcn_readlane(y, j);
                    const int dxc = __builtin_amdgcn_readlane(xc, j) - xc, dyc = __builtin_amdgcn_readlane(yc, j) - yc;
                    const float ddx = fx - (float)xj, ddy = fy - (float)yj;
                    if (j < lane && dxc >= -1 && dxc <= 1 && dyc >= -1 && dyc <= 1 && ddx * ddx + ddy * ddy < md2)
                        conf |= 1ull << j;
                }
                const uint64_t open = __ballot(valid && !hit);
                const int g = yc * gw + xc;
                uint64_t acc = 0;
                const uint32_t conf_lo = (uint32_t)conf, conf_hi = (uint32_t)(conf >> 32);
                // in order over the chunk (scalar loop): accept j unless an accepted earlier lane
                // conflicts; lane 0 links each accepted corner into its cell's list
                for (int j = 0; j < nc; j++) {
                    if (!((open >> j) & 1ull)) continue;
                    const uint64_t cj = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)conf_hi, j) << 32) |
                                        (uint32_t)__builtin_amdgcn_readlane((int)conf_lo, j);
                    if (cj & acc) continue;
                    const int r = nacc + __popcll(acc);
                    acc |= 1ull << j;
                    if (lane == 0) {
                        const int gj = __builtin_amdgcn_readlane(g, j);
                        next[r] = head[gj];
                        head[gj] = (uint16_t)r;
                    }
                    if (r + 1 == limit) { full = true; break; }
                }
                if ((acc >> lane) & 1ull) {
                    const int r = nacc + __popcll(acc & ((1ull << lane) - 1ull));
                    axy[r] = (uint32_t)x | ((uint32_t)y << 16);
                    out_xy[2 * r] = fx;
                    out_xy[2 * r + 1] = fy;
                }
                nacc += __popcll(acc);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");     // lists visible to the next chunk
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            if (lane == 0) { s_nacc = nacc; s_full = full; }
        }
        __syncthreads();
        done += m;
        U = T;
        first = false;
    }
    if (tid == 0) *nout = s_nacc;
}

// ============================== cornerSubPix ==============================
// The five double sums of an iteration are chains of 441 dependent adds in the reference's
// row-major order.  Round 2 ran one corner per wave and the sums on five lanes, so every add cost
// a whole wave instruction (1.44 ms per 256 pairs).  Here a wave carries G corner slots (0.89 ms),
// and an iteration is 21 phases, one
// per window row i: the fill lanes (slot, column pair) extend each slot's rolling four-row
// getRectSubPix patch by row i + 3, the term lanes (slot, column) form the five terms of window
// row i for every slot, and lane 5 g + t adds row i's 21 terms of term t of slot g -- one add
// instruction serves G corners.  Slots iterate independently (their own ipx / ipy / weights,
// rewritten each round by the slot's lane into `par`); a slot whose corner has converged takes the
// next one from the work queue at the start of the next round.  The two image rows a phase's fill
// needs come straight from global memory (L2-resident windows), issued at the start of the phase
// and consumed at its end, so no load is in flight across the loop's back edge.
// corner slots per wave (9: 45 summing lanes; 6 and 12 measured slower on the config-D step:
// 36.30 / 35.71-35.83 vs 35.10 ms, profiles/r06/s11)
constexpr int kSpSlots = 9;
constexpr int kSpPrPad = 1;      // row padding of the rolling patch (floats)
// Rolling patch of a slot: three rows (window row i reads patch rows i .. i + 2, and row i + 3 is
// filled into row i's place once they are read), slot stride kSpSS = 21 (mod 64) dwords so the
// term lanes of a pass -- slots g, g + 1, g + 2 at the same 21 columns -- read 63 distinct banks.
// The 4-row ring at 96 dwords per slot put slots g and g + 2 on the same banks: 2.74 vs 1.96
// conflict cycles per LDS instruction, k_subpix 3.26-3.32 vs 3.19-3.23 ms per config-D step
// (profiles/r06/s30).  Holding the term rows for half a window row at a time (8.8 KB of LDS, 4 waves
// per SIMD instead of 3) ran 3.70-3.72 vs 3.19-3.22 ms: the extra term passes and syncs cost more than
// the occupancy gives (s31).
constexpr int kSpRows = 3;
constexpr int kSpRS = 23 + kSpPrPad;                       // BW + padding
constexpr int kSpSS = 85;
static_assert(kSpSS >= kSpRows * kSpRS && kSpSS % 64 == 21, "k_subpix patch layout");
constexpr int kSpTrPad = 5;      // row padding of the term rows (doubles; >= 5: the sink slot G's terms)
static_assert(kSpTrPad >= 5, "the term rows hold the sink slot's five terms");
struct __attribute__((aligned(16))) SpSlot {      // read as three 16-byte words by the fill lanes
    const uint8_t* img;
    double sd;                          // in-image: (1 - a) / a
    float a12, a22, b1, b2, c4, c5;     // in-image: c4 = 1 - a; clamped: c4 = a11, c5 = a21
    int ipx, ipy, mode, pad;            // mode 0: idle, 1: window inside the image, 2: clamped
};

__device__ __forceinline__ void wave_order() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

template <int G>
__global__ __launch_bounds__(64) void k_subpix(const uint8_t* __restrict__ img0, int w, int h, int stride,
                                                  float* __restrict__ xy0, const int* __restrict__ offs, int P,
                                                  const int* __restrict__ order, int* __restrict__ queue,
                                                  const float* __restrict__ mexp, int iters, double eps2, int64_t iz,
                                                  int64_t pz, int* __restrict__ itcount)
{
    constexpr int WIN = 10, WW = 2 * WIN + 1, BW = WW + 2, NJ = (BW + 1) / 2;
    constexpr int NF = (G * NJ + 63) / 64, NT = (G * WW + 63) / 64, NL = 5 * G;
    static_assert(NL <= 64, "one summing lane per slot and term");
    // slot G is a sink: the fill and term lanes past the last slot read and write it, so no
    // pass needs a branch and the LDS reads of all passes issue together
    static_assert(BW + kSpPrPad == kSpRS, "k_subpix row stride");
    __shared__ __attribute__((aligned(16))) float pr[(G + 1) * kSpSS];   // rolling patch rows (kSpRows per slot)
    auto prow = [](int r) { return r % kSpRows; };
    __shared__ double tr[WW][NL + kSpTrPad];      // one window row's terms, [j][5 g + t]
    __shared__ SpSlot par[G + 1];
    __shared__ double ssum[NL];
    const int lane = threadIdx.x;
    const int total = offs[P];
    // the weights: mask(i, j) = e_i * e_j in float (cornerSubPix's vy * expf(-x * x)); e_lane here,
    // e_j of each term pass's column, e_i by readlane
    const float e_lane = mexp[min(lane, WW - 1)];
    float e_col[NT];
    int tg[NT], tj[NT];                                // term task (slot, column)
#pragma unroll
    for (int q = 0; q < NT; q++) {
        const int e = q * 64 + lane, g = e / WW;
        tj[q] = e - g * WW;
        tg[q] = min(g, G);
        e_col[q] = mexp[tj[q]];
    }
    if (lane == 0) {
        SpSlot sl;
        sl.img = img0; sl.sd = 0.; sl.a12 = sl.a22 = sl.b1 = sl.b2 = sl.c4 = sl.c5 = 0.f;
        sl.ipx = sl.ipy = 0; sl.mode = 0; sl.pad = 0;
        par[G] = sl;
    }
    // slot state on lane g < G
    int item = -1, it = 0, pidx = 0;
    int nit = 0, ncorner = 0;                          // wave totals (COEB_SUBPIX_COUNT)
    float tx = 0.f, ty = 0.f, cx = 0.f, cy = 0.f;
    float* xy = nullptr;
    const uint8_t* simg = nullptr;
    bool need = lane < G, drained = false;
    for (;;) {
        // refill the free slots from the queue, one atomic per wave
        const uint64_t nm = drained ? 0ull : __ballot(need);
        if (nm) {
            const int first = __ffsll((unsigned long long)nm) - 1;
            int base = 0;
            if (lane == first) base = atomicAdd(queue, __popcll(nm));
            base = __shfl(base, first, 64);
            if (base + __popcll(nm) >= total) drained = true;
            if (need) {
                const int q = base + __popcll(nm & ((1ull << lane) - 1ull));
                item = q < total ? q : -1;
                if (item >= 0) {
                    const int2 zp = flow_decode(order[item]);
                    xy = at_pair(xy0, pz, (uint32_t)zp.x);
                    simg = at_pair(img0, iz, (uint32_t)zp.x);
                    pidx = zp.y;
                    tx = xy[2 * pidx]; ty = xy[2 * pidx + 1];
                    cx = tx; cy = ty; it = 0;
                }
                need = false;
            }
            ncorner += __popcll(__ballot(lane < G && item >= 0) & nm);
        }
        const uint64_t am = __ballot(lane < G && item >= 0);
        if (!am) break;
        nit += __popcll(am);
        if (lane < G) {
            SpSlot sl;
            sl.img = item >= 0 ? simg : img0;           // idle slots: a valid address for the fill loads
            sl.sd = 0.;
            sl.a12 = sl.a22 = sl.b1 = sl.b2 = sl.c4 = sl.c5 = 0.f; sl.ipx = sl.ipy = 0; sl.mode = 0; sl.pad = 0;
            if (item >= 0) {
                const float ctrx = cx - (float)(BW - 1) * 0.5f, ctry = cy - (float)(BW - 1) * 0.5f;
                const int ipx = cv_floor(ctrx), ipy = cv_floor(ctry);
                const float a = ctrx - (float)ipx, b = ctry - (float)ipy;
                sl.ipx = ipx; sl.ipy = ipy; sl.b1 = 1.f - b; sl.b2 = b;
                if (ipx >= 0 && ipx + BW < w && ipy >= 0 && ipy + BW < h) {
                    const float ac = a < 0.0001f ? 0.0001f : a;      // getRectSubPix_8u32f's recurrence
                    sl.mode = 1;
                    sl.a12 = ac * (1.f - b); sl.a22 = ac * b; sl.c4 = 1.f - ac;
                    sl.sd = (1. - (double)ac) / (double)ac;
                } else {
                    sl.mode = 2;
                    sl.c4 = (1.f - a) * (1.f - b); sl.a12 = a * (1.f - b); sl.c5 = (1.f - a) * b; sl.a22 = a * b;
                }
            }
            par[lane] = sl;
        }
        wave_order();
        // fill lanes: task f = q * 64 + lane -> (slot f / NJ, patch columns j0, j0 + 1), image
        // columns c0 .. c0 + 2 clamped (the in-image window needs no clamping); the slot's weights
        // stay in registers for the round
        int fipy[NF], fd[NF], fj0[NF], fg[NF], fmode[NF];
        const uint8_t* fbase[NF];
        float fa12[NF], fa22[NF], fb1[NF], fb2[NF], fc4[NF], fc5[NF];
        double fsd[NF];
#pragma unroll
        for (int q = 0; q < NF; q++) {
            const int f = q * 64 + lane, g = min(f / NJ, G);
            fg[q] = g;
            fj0[q] = 2 * (f - (f / NJ) * NJ);
            const int4* pw = reinterpret_cast<const int4*>(&par[g]);
            const int4 w0 = pw[0], w1 = pw[1], w2 = pw[2], w3 = pw[3];
            fbase[q] = reinterpret_cast<const uint8_t*>((uint64_t)(uint32_t)w0.x | ((uint64_t)(uint32_t)w0.y << 32));
            fsd[q] = __builtin_bit_cast(double, (int64_t)(uint32_t)w0.z | ((int64_t)w0.w << 32));
            fa12[q] = __int_as_float(w1.x); fa22[q] = __int_as_float(w1.y); fb1[q] = __int_as_float(w1.z); fb2[q] = __int_as_float(w1.w);
            fc4[q] = __int_as_float(w2.x); fc5[q] = __int_as_float(w2.y);
            fipy[q] = w2.w;
            fmode[q] = w3.x;
            const int c = w2.z + fj0[q];
            fbase[q] += min(max(c, 0), w - 1);
            fd[q] = (min(max(c + 1, 0), w - 1) - min(max(c, 0), w - 1)) | ((min(max(c + 2, 0), w - 1) - min(max(c, 0), w - 1)) << 2) |
                    ((c < 0 || c >= w - 1) << 4) | ((c + 1 < 0 || c + 1 >= w - 1) << 5);
        }
        // the three bytes of image row rr (relative to ipy) under a fill task
        auto load_row = [&](int q, int rr, uint32_t* v) {
            typedef const uint8_t __attribute__((address_space(1)))* gp8;
            const gp8 r = (gp8)(fbase[q] + (size_t)min(max(fipy[q] + rr, 0), h - 1) * stride);
            v[0] = r[0]; v[1] = r[fd[q] & 3]; v[2] = r[(fd[q] >> 2) & 3];
        };
        // patch row r, columns j0 and j0 + 1, from image rows r (lo) and r + 1 (hi); both forms
        // are evaluated and selected, so the pass has no branch
        auto fill = [&](int q, int r, const uint32_t* lo, const uint32_t* hi) {
            const float l0 = (float)lo[0], l1 = (float)lo[1], l2 = (float)lo[2];
            const float h0 = (float)hi[0], h1 = (float)hi[1], h2 = (float)hi[2];
            const float a12 = fa12[q], a22 = fa22[q], b1 = fb1[q], b2 = fb2[q], c4 = fc4[q], c5 = fc5[q];
            // in-image: u_k = a12 src[k] + a22 src[k + sst], element j is prev(u_j) + u_{j + 1}
            const float u1 = a12 * l1 + a22 * h1, u2 = a12 * l2 + a22 * h2;
            const float p0 = fj0[q] == 0 ? c4 * (b1 * l0 + b2 * h0) : (float)((double)(a12 * l0 + a22 * h0) * fsd[q]);
            float v0 = p0 + u1;
            float v1 = (float)((double)u1 * fsd[q]) + u2;
            if (fmode[q] == 2) {                        // clamped (wave-uniform in practice: border corners last)
                v0 = (fd[q] & 16) ? l0 * b1 + h0 * b2 : l0 * c4 + l1 * a12 + h0 * c5 + h1 * a22;
                v1 = (fd[q] & 32) ? l1 * b1 + h1 * b2 : l1 * c4 + l2 * a12 + h1 * c5 + h2 * a22;
            }
            float* dst = &pr[fg[q] * kSpSS + prow(r) * kSpRS + fj0[q]];   // column 23: padding
            dst[0] = v0;
            dst[1] = v1;
        };
#pragma unroll
        for (int q = 0; q < NF; q++) {
            uint32_t ra[3], rb[3];
            load_row(q, 0, ra);
#pragma unroll
            for (int r = 0; r < 3; r++) {
                if (r & 1) { load_row(q, r + 1, ra); fill(q, r, rb, ra); }
                else { load_row(q, r + 1, rb); fill(q, r, ra, rb); }
            }
        }
        double acc = 0.0;
#pragma unroll 1
        for (int i = 0; i < WW; i++) {
            // image rows i + 3, i + 4 for patch row i + 3 (i + 3 < BW), used at the end of the phase
            uint32_t lo[NF][3], hi[NF][3];
            const int rr = min(i + 3, BW - 1);
#pragma unroll
            for (int q = 0; q < NF; q++) { load_row(q, rr, lo[q]); load_row(q, rr + 1, hi[q]); }
            wave_order();
            const float e_row = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, e_lane), i));
            const double py = i - WIN;
            float d[NT][4];
#pragma unroll
            for (int q = 0; q < NT; q++) {             // window row i: all passes' patch reads first
                const int g = tg[q], j = tj[q];
                const float* r0 = &pr[g * kSpSS + prow(i) * kSpRS + j];
                const float* r1 = &pr[g * kSpSS + prow(i + 1) * kSpRS + j];
                const float* r2 = &pr[g * kSpSS + prow(i + 2) * kSpRS + j];
                d[q][0] = r1[2]; d[q][1] = r1[0];
                d[q][2] = r2[1]; d[q][3] = r0[1];
            }
#pragma unroll
            for (int q = 0; q < NT; q++) {
                const double m = (double)(e_row * e_col[q]);
                const double tgx = (double)(d[q][0] - d[q][1]);
                const double tgy = (double)(d[q][2] - d[q][3]);
                const double gxx = tgx * tgx * m, gxy = tgx * tgy * m, gyy = tgy * tgy * m;
                const double px = tj[q] - WIN;
                double* o = &tr[tj[q]][5 * tg[q]];
                o[0] = gxx; o[1] = gxy; o[2] = gyy;
                o[3] = gxx * px + gxy * py;
                o[4] = gxy * px + gyy * py;
            }
            wave_order();
            if (lane < NL) {
#pragma unroll
                for (int j = 0; j < WW; j++) acc += tr[j][lane];
            }
            wave_order();
            if (i + 3 < BW) {
#pragma unroll
                for (int q = 0; q < NF; q++) fill(q, i + 3, lo[q], hi[q]);
            }
        }
        if (lane < NL) ssum[lane] = acc;
        wave_order();
        if (lane < G && item >= 0) {
            const double sa = ssum[5 * lane], sb = ssum[5 * lane + 1], sc = ssum[5 * lane + 2];
            const double bb1 = ssum[5 * lane + 3], bb2 = ssum[5 * lane + 4];
            bool fin = false;
            const double det = sa * sc - sb * sb;
            if (fabs(det) <= DBL_EPSILON * DBL_EPSILON) fin = true;
            else {
                const double scale = 1.0 / det;
                const float nx = (float)((double)cx + sc * scale * bb1 - sb * scale * bb2);
                const float ny = (float)((double)cy - sb * scale * bb1 + sa * scale * bb2);
                const double err = (double)((nx - cx) * (nx - cx) + (ny - cy) * (ny - cy));
                cx = nx; cy = ny;
                if (cx < 0 || cx >= (float)w || cy < 0 || cy >= (float)h) fin = true;
                else if (!(++it < iters && err > eps2)) fin = true;
            }
            if (fin) {
                if (fabsf(cx - tx) > (float)WIN || fabsf(cy - ty) > (float)WIN) { cx = tx; cy = ty; }
                xy[2 * pidx] = cx; xy[2 * pidx + 1] = cy;
                item = -1;
                need = true;
            }
        }
        wave_order();
    }
    if (itcount && lane == 0) { atomicAdd(itcount, nit); atomicAdd(itcount + 1, ncorner); }
}

// cornerSubPix work order: the corners whose window may leave the image (getRectSubPix's
// clamped path) last, so the waves that take the in-image path (nearly all) never execute the
// other; lane order within a wave is kept (wave-aggregated atomics), so a wave's corners stay
// mostly one frame's.  ocnt = {interior, border} counters, zeroed before the launch.
__global__ __launch_bounds__(256) void k_subpix_order(const float* __restrict__ xy0, const int* __restrict__ offs,
                                                      int P, int w, int h, int margin, int64_t pz,
                                                      int* __restrict__ order, int* __restrict__ ocnt)
{
    const int total = offs[P];
    const int lane = threadIdx.x & 63;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int base = blockIdx.x * 256 + (threadIdx.x & ~63); base < total; base += gridDim.x * 256) {
        const int item = base + lane;
        bool in = false, bd = false;
        int code = 0;
        if (item < total) {
            const int2 zp = flow_item(offs, P, item);
            // the corner as (pair, index) packed (flow_code): k_subpix's slot refill then needs no
            // binary search over offs (11 dependent global loads per corner)
            code = flow_code(zp);
            const float* xy = at_pair(xy0, pz, (uint32_t)zp.x);
            const float x = xy[2 * zp.y], y = xy[2 * zp.y + 1];
            in = x >= (float)margin && x <= (float)(w - 1 - margin) && y >= (float)margin && y <= (float)(h - 1 - margin);
            bd = !in;
        }
        const uint64_t mi = __ballot(in), mb = __ballot(bd);
        int bi = 0, bb = 0;
        if (lane == 0) {
            bi = atomicAdd(&ocnt[0], __popcll(mi));
            bb = atomicAdd(&ocnt[1], __popcll(mb));
        }
        bi = __builtin_amdgcn_readfirstlane(bi);
        bb = __builtin_amdgcn_readfirstlane(bb);
        if (in) order[bi + __popcll(mi & lt)] = code;
        if (bd) order[total - 1 - (bb + __popcll(mb & lt))] = code;
    }
}

// ============================== pyramidal Lucas-Kanade ==============================
struct LkPyr {
    const uint8_t* P[kLkMaxLevels];   // previous frame levels (level 0 = the input, pitch stride)
    const uint8_t* N[kLkMaxLevels];   // next frame levels
    const short2* D[kLkMaxLevels];    // Scharr (dx, dy) of the previous frame levels
    int pitch[kLkMaxLevels];          // image pitch per level
    int w[kLkMaxLevels], h[kLkMaxLevels];
    int L;
};

struct PyrDownArgs {
    const uint8_t* src[2];
    uint8_t* dst[2];
    int sw, sh, spitch, dw, dh;
    int src_img;                        // src = the input frames (pair stride iz), else pyramid levels (pz)
    int nfr;                            // frames per pair block: 2 (prev, next) or 1 (one pyramid per frame)
};

// pyrDown 8U (5x5 [1 4 6 4 1]^2, (sum + 128) >> 8, REFLECT_101); blockIdx.z = nfr * pair + frame.
// One wave per strip of 62 output columns x kPdRows rows, lane = output column x0 - 1 + lane
// (lanes 1..62 produce): a lane loads source columns 2x and 2x + 1 of each source row (reflected
// indices), the taps 2x - 2, 2x - 1 and 2x + 2 come from the neighbouring lanes (DPP wave shifts),
// and the five horizontal sums of an output row slide down the strip two source rows at a time.
// (Round 2 gathered all 25 taps per output pixel with a reflection per tap.)
constexpr int kPdRows = 16;
constexpr int kPdCols = 62;
__global__ __launch_bounds__(256) void k_pyr_down(PyrDownArgs a, int64_t iz, int64_t pz)
{
    const int lane = threadIdx.x & 63;
    const int strip = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int x0 = strip * kPdCols, y0 = blockIdx.y * kPdRows;
    if (x0 >= a.dw) return;
    const int fr = a.nfr == 2 ? (int)(blockIdx.z & 1) : 0;
    const uint64_t pair = a.nfr == 2 ? blockIdx.z >> 1 : blockIdx.z;
    const uint8_t* src = a.src[fr] + pair * (uint64_t)(a.src_img ? iz : pz);
    uint8_t* dst = a.dst[fr] + pair * (uint64_t)pz;
    const int c = x0 - 1 + lane;
    const int s0 = reflect101(2 * c, a.sw), s1 = reflect101(2 * c + 1, a.sw);
    const bool produce = lane >= 1 && lane <= kPdCols && c < a.dw;
    auto hsum = [&](int sr) {
        const uint8_t* row = src + (size_t)reflect101(sr, a.sh) * a.spitch;
        const int e0 = row[s0], e1 = row[s1];
        const int l0 = wave_shr1(e0), l1 = wave_shr1(e1), r0 = wave_shl1(e0);
        return l0 + 4 * l1 + 6 * e0 + 4 * e1 + r0;
    };
    const int y1 = min(a.dh, y0 + kPdRows);
    // source rows 2y - 2 .. 2y + 2 of output row y
    int h0 = hsum(2 * y0 - 2), h1 = hsum(2 * y0 - 1), h2 = hsum(2 * y0);
    for (int y = y0; y < y1; y++) {
        const int h3 = hsum(2 * y + 1), h4 = hsum(2 * y + 2);
        const int acc = h0 + 4 * h1 + 6 * h2 + 4 * h3 + h4;
        if (produce) dst[(size_t)y * a.dw + c] = (uint8_t)((acc + 128) >> 8);
        h0 = h2; h1 = h3; h2 = h4;
    }
}

// calcSharrDeriv of every previous-frame level; blockIdx.y = level, blockIdx.z = pair.  One wave
// per strip of kShCols columns x kShRows rows of a level, lane = column (x0 - 1 + lane; lanes
// 1..62 produce): the band's source bytes (+1 row above and below, the trow border rule) are all
// loaded up front, each lane forms its column's vertical terms t0 = 3 (s0 + s2) + 10 s1 and
// t1 = s2 - s0, and the neighbours' come by DPP wave shifts -- the same integer expressions as
// calcSharrDeriv, one byte load per pixel.  (The grid-stride per-pixel form read 9 bytes per pixel
// with a division per pixel, and its level-0 blocks ran 19 passes while the others idled.)
constexpr int kShCols = 62, kShRows = 32;
__global__ __launch_bounds__(256) void k_sharr(LkPyr pyr, int64_t iz, int64_t pz)
{
    const int l = blockIdx.y;
    const int w = pyr.w[l], h = pyr.h[l], pitch = pyr.pitch[l];
    const int nstrip = (w + kShCols - 1) / kShCols, nband = (h + kShRows - 1) / kShRows;
    const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (item >= nstrip * nband) return;
    const int strip = item % nstrip, band = item / nstrip;
    const uint8_t* img = at_pair(pyr.P[l], l == 0 ? iz : pz);
    short2* d = at_pair(const_cast<short2*>(pyr.D[l]), pz);
    const int lane = threadIdx.x & 63;
    const int x0 = strip * kShCols, y0 = band * kShRows, y1 = min(h, y0 + kShRows);
    const int c = x0 - 1 + lane;
    // trow border: trow[-1] = trow[1], trow[w] = trow[w-2]; columns past w are never used
    const int cc = c < 0 ? (w > 1 ? 1 : 0) : (c >= w ? (w > 1 ? w - 2 : 0) : c);
    const bool produce = lane >= 1 && lane <= kShCols && c < w;
    int px[kShRows + 2];                               // source rows y0 - 1 .. y0 + kShRows
#pragma unroll
    for (int i = 0; i < kShRows + 2; i++) {
        const int yy = y0 - 1 + i;
        const int yr = yy < 0 ? (h > 1 ? 1 : 0) : (yy >= h ? (h > 1 ? h - 2 : 0) : yy);
        px[i] = yy <= y1 ? (int)img[(size_t)yr * pitch + cc] : 0;
    }
#pragma unroll
    for (int i = 1; i <= kShRows; i++) {
        const int y = y0 - 1 + i;
        if (y >= y1) break;
        const int t0 = (px[i - 1] + px[i + 1]) * 3 + px[i] * 10, t1 = px[i + 1] - px[i - 1];
        const int t0l = wave_shr1(t0), t0r = wave_shl1(t0), t1l = wave_shr1(t1), t1r = wave_shl1(t1);
        if (produce) d[(size_t)y * w + c] = make_short2((short)(t0r - t0l), (short)((t1r + t1l) * 3 + t1 * 10));
    }
}

// Wave sum of an int32 whose total may need 34 bits: the 16-bit halves are summed separately
// (|hi| < 2^15 and lo < 2^16 per lane keep both sums inside int32 over 64 lanes) with DPP row
// shifts and row broadcasts -- no LDS round trips (an int64 __shfl_xor tree costs 12
// ds_bpermute) -- and joined in int64.  Exact: the per-lane partial sums fit int32 (<= 8
// products of < 2^27).
__device__ __forceinline__ int dpp_sum_to63(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return v;                                                          // lane 63: the total
}
__device__ __forceinline__ int64_t wave_sum_i32x(int v)
{
    const int hi = dpp_sum_to63(v >> 16), lo = dpp_sum_to63(v & 0xffff);
    return (int64_t)__builtin_amdgcn_readlane(hi, 63) * 65536 + (int64_t)__builtin_amdgcn_readlane(lo, 63);
}

__device__ __forceinline__ int refl1(int p, int n) { return p < 0 ? -p : (p >= n ? 2 * n - 2 - p : p); }

// One wave per point.  The window (win <= 24) is tiled 8 x 8 by 3 x 3 pixel tiles, lane
// (tr, tc) = (lane >> 3, lane & 7) carrying rows 3 tr .. 3 tr + 2 and columns 3 tc .. 3 tc + 2
// (a 22 x 22 window keeps 484 of the 576 slots busy, every lane has work).  A tile's four image
// rows (three pixel rows and the +1 neighbour row) are one unaligned 4-byte segment each; each
// bilinear tap pair (p[k], p[k + 1]) of a row is one v_perm into a u16x2, shared by the pixel rows
// above and below it, and weighed by v_dot2_i32_i16 against (iw00, iw01) or (iw10, iw11); the
// products with the derivatives are v_mad_i32_i24 (all operands < 2^23).  sum (J - I) * g is
// accumulated as sum J * g - sum I * g with the second term fixed per level: every per-lane
// partial stays exact in int32 (<= 9 products of < 2^26), and the window sums are joined by DPP
// wave reductions of their 16-bit halves.  Windows that reach past the level edge take the
// per-pixel reflected path of calcOpticalFlowPyrLK (REFLECT_101 images, zero derivatives).
// signed: iw11 = 16384 - iw00 - iw01 - iw10 is -1 when the three rounded weights overshoot
typedef short lk_i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int dot2s(uint32_t a, uint32_t b, int c)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(lk_i16x2, a), __builtin_bit_cast(lk_i16x2, b), c, false);
}

// the three tap pairs (p[k], p[k + 1]), k = 0, 1, 2, of a 4-byte row segment as u16x2
__device__ __forceinline__ void tap_pairs(uint32_t q, uint32_t* t)
{
    t[0] = __builtin_amdgcn_perm(0u, q, 0x0c010c00u);
    t[1] = __builtin_amdgcn_perm(0u, q, 0x0c020c01u);
    t[2] = __builtin_amdgcn_perm(0u, q, 0x0c030c02u);
}

// The four row segments of the lane's tile as tap pairs, through a buffer resource over the level image (bounds-checked: a dword past the
// image end reads as 0, so no per-row clamp), the window at scalar byte offset s_off and the
// lane's four row offsets lofs[i] = min(C0, win) + min(R0 + i, win) * pitch fixed per level:
// per row one add and two ands, two loads with a scalar base, one alignbyte (round 5's 64-bit
// addresses with a clamped second dword cost ~30 more VALU per LK iteration: k_lk 3.27 -> 2.95 ms
// per config-D step, profiles/r06/s3).  Every lane loads all four rows (no divergent waits):
// rows and columns are clamped to the window's +1 row / column, which the caller has checked lie
// inside the level, and the samples this brings in outside the tile's pixels are weighed by zero
// derivatives.
__device__ __forceinline__ void tile_pairs_buf(__amdgpu_buffer_rsrc_t r, int s_off, const int (&lofs)[4], uint32_t (*t)[3])
{
    const int s_al = s_off & ~3, s_mis = s_off & 3;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t o = (uint32_t)(lofs[i] + s_mis);
        const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(r, o & ~3u, s_al, 0);
        const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(r, (o & ~3u) + 4u, s_al, 0);
        tap_pairs(__builtin_amdgcn_alignbyte(hi, lo, o & 3u), t[i]);
    }
}

// The same taps for a window that reaches past the level edge: byte gathers at REFLECT_101
// coordinates (the taps of calcOpticalFlowPyrLK's border path), same clamping
__device__ __forceinline__ void tile_pairs_reflect(const uint8_t* img, int pitch, int lw, int lh, int x0, int y0, int win,
                                                   int C0, int R0, uint32_t (*t)[3])
{
    int cx[4];
#pragma unroll
    for (int j = 0; j < 4; j++) cx[j] = refl1(x0 + min(C0 + j, win), lw);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint8_t* r = img + (size_t)refl1(y0 + min(R0 + i, win), lh) * pitch;
        const uint32_t q = (uint32_t)r[cx[0]] | ((uint32_t)r[cx[1]] << 8) | ((uint32_t)r[cx[2]] << 16) | ((uint32_t)r[cx[3]] << 24);
        tap_pairs(q, t[i]);
    }
}

#ifndef COEB_LK_MINW
#define COEB_LK_MINW 1         // launch bound of k_lk in waves per SIMD
#endif
__global__ __launch_bounds__(256, COEB_LK_MINW) void k_lk(LkPyr pyr, const float* __restrict__ pxy0, const int* __restrict__ offs, int P,
                                            float* __restrict__ nxy0, uint8_t* __restrict__ status0, int win, int max_count,
                                            double eps2, int64_t iz, int64_t pz, int* __restrict__ itcount)
{
    const int lane = threadIdx.x & 63;
    const int R0 = (lane >> 3) * 3, C0 = (lane & 7) * 3;
    const int nr = min(3, max(0, win - R0)), nc = nr > 0 ? min(3, max(0, win - C0)) : 0;   // this lane's pixels
    const int total = offs[P];
    // points in grid-stride order (taking them from a queue, one atomic per point, measured slower:
    // 3.53 vs 3.29 ms per config-D step, profiles/r05/s43; the blocks dealt to the XCDs in
    // contiguous runs, so a pair's points share one L2, 2.97-3.00 vs 2.96-2.98 ms, r06/s27)
    for (int item = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); item < total; item += gridDim.x * 4) {
    // (the points in k_subpix_order's order, decoded from its packed codes instead of this binary
    // search: 3.01-3.04 vs 2.95-3.01 ms per config-D step, the order loses the frames' locality;
    // profiles/r06/s26)
    const int2 zp = flow_item(offs, P, item);
    const uint32_t z = (uint32_t)zp.x;
    const float* pxy = at_pair(pxy0, pz, z);
    float* nxy = at_pair(nxy0, pz, z);
    uint8_t* status = at_pair(status0, pz, z);
    const int p = zp.y;
    const float hw = (float)(win - 1) * 0.5f;
    const float FLT_SCALE = 1.f / (1 << 20);
    int st = 1;
    float nx = 0.f, ny = 0.f;
    const float px0 = pxy[2 * p], py0 = pxy[2 * p + 1];
    int gxv[9], gyv[9];
    int nit = 0;
    for (int level = pyr.L - 1; level >= 0; level--) {
        const int lw = pyr.w[level], lh = pyr.h[level], pitch = pyr.pitch[level];
        const uint8_t* I = at_pair(pyr.P[level], level == 0 ? iz : pz, z);
        const uint8_t* J = at_pair(pyr.N[level], level == 0 ? iz : pz, z);
        const short2* D = at_pair(pyr.D[level], pz, z);
        const __amdgpu_buffer_rsrc_t rI = __builtin_amdgcn_make_buffer_rsrc((void*)I, 0, pitch * lh, 0x00020000);
        const __amdgpu_buffer_rsrc_t rJ = __builtin_amdgcn_make_buffer_rsrc((void*)J, 0, pitch * lh, 0x00020000);
        int lofs[4];
#pragma unroll
        for (int i = 0; i < 4; i++) lofs[i] = min(C0, win) + min(R0 + i, win) * pitch;
        const float sc = (float)(1. / (1 << level));
        float px = px0 * sc, py = py0 * sc;
        if (level == pyr.L - 1) { nx = px; ny = py; }
        else { nx = nx * 2.f; ny = ny * 2.f; }
        px -= hw; py -= hw;
        const int ipx = cv_floor(px), ipy = cv_floor(py);
        if (ipx < -win || ipx >= lw || ipy < -win || ipy >= lh) {
            if (level == 0) st = 0;
            continue;
        }
        float a = px - (float)ipx, b = py - (float)ipy;
        int iw00 = (int)rintf((1.f - a) * (1.f - b) * 16384.f);
        int iw01 = (int)rintf(a * (1.f - b) * 16384.f);
        int iw10 = (int)rintf((1.f - a) * b * 16384.f);
        int iw11 = 16384 - iw00 - iw01 - iw10;
        int sA11 = 0, sA12 = 0, sA22 = 0;                 // per lane: <= 9 products of < 2^25
        int sIx = 0, sIy = 0;                             // per lane sum I * g: <= 9 products of < 2^26
        const int X0 = ipx + C0, Y0 = ipy + R0;
        const bool inside = ipx >= 0 && ipy >= 0 && ipx + win < lw && ipy + win < lh;
        uint32_t t[4][3];
        if (inside)
            tile_pairs_buf(rI, __builtin_amdgcn_readfirstlane(ipy * pitch + ipx), lofs, t);
        else
            tile_pairs_reflect(I, pitch, lw, lh, ipx, ipy, win, C0, R0, t);
        const uint32_t W0 = (uint32_t)iw00 | ((uint32_t)iw01 << 16), W1 = (uint32_t)iw10 | ((uint32_t)iw11 << 16);
#pragma unroll
        for (int k = 0; k < 9; k++) {
            const int i = k / 3, j = k % 3;
            gxv[k] = 0; gyv[k] = 0;
            if (i < nr && j < nc) {
                const int iv = (dot2s(t[i][j], W0, dot2s(t[i + 1][j], W1, 1 << 8)) >> 9);
                const int X = X0 + j, Y = Y0 + i;
                short2 e00, e01, e10, e11;
                if (inside) {
                    const short2* d0 = D + (size_t)Y * lw + X;
                    e00 = d0[0]; e01 = d0[1]; e10 = d0[lw]; e11 = d0[lw + 1];
                } else {
                    auto dv = [&](int xq, int yq) {
                        return (xq < 0 || yq < 0 || xq >= lw || yq >= lh) ? make_short2(0, 0) : D[(size_t)yq * lw + xq];
                    };
                    e00 = dv(X, Y); e01 = dv(X + 1, Y); e10 = dv(X, Y + 1); e11 = dv(X + 1, Y + 1);
                }
                gxv[k] = (__mul24(e00.x, iw00) + __mul24(e01.x, iw01) + __mul24(e10.x, iw10) + __mul24(e11.x, iw11) + (1 << 13)) >> 14;
                gyv[k] = (__mul24(e00.y, iw00) + __mul24(e01.y, iw01) + __mul24(e10.y, iw10) + __mul24(e11.y, iw11) + (1 << 13)) >> 14;
                sA11 += __mul24(gxv[k], gxv[k]);
                sA12 += __mul24(gxv[k], gyv[k]);
                sA22 += __mul24(gyv[k], gyv[k]);
                sIx += __mul24(iv, gxv[k]);
                sIy += __mul24(iv, gyv[k]);
            }
        }
        const int64_t tA11 = wave_sum_i32x(sA11), tA12 = wave_sum_i32x(sA12), tA22 = wave_sum_i32x(sA22);
        const float A11 = (float)tA11 * FLT_SCALE, A12 = (float)tA12 * FLT_SCALE, A22 = (float)tA22 * FLT_SCALE;
        float D2 = A11 * A22 - A12 * A12;
        const float minEig = ((A22 + A11) - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * win * win);
        if (minEig < 1e-4f || D2 < FLT_EPSILON) {
            if (level == 0) st = 0;
            continue;
        }
        D2 = 1.f / D2;
        float lx = nx - hw, ly = ny - hw;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < max_count; j++) {
            nit++;
            const int inx = cv_floor(lx), iny = cv_floor(ly);
            if (inx < -win || inx >= lw || iny < -win || iny >= lh) {
                if (level == 0) st = 0;
                break;
            }
            a = lx - (float)inx; b = ly - (float)iny;
            iw00 = (int)rintf((1.f - a) * (1.f - b) * 16384.f);
            iw01 = (int)rintf(a * (1.f - b) * 16384.f);
            iw10 = (int)rintf((1.f - a) * b * 16384.f);
            iw11 = 16384 - iw00 - iw01 - iw10;
            int ib1 = -sIx, ib2 = -sIy;               // per lane: sum (J - I) * g, exact in int32
            uint32_t t[4][3];
            if (inx >= 0 && iny >= 0 && inx + win < lw && iny + win < lh)    // the window and its +1 neighbours inside
                tile_pairs_buf(rJ, __builtin_amdgcn_readfirstlane(iny * pitch + inx), lofs, t);
            else
                tile_pairs_reflect(J, pitch, lw, lh, inx, iny, win, C0, R0, t);
            const uint32_t W0 = (uint32_t)iw00 | ((uint32_t)iw01 << 16), W1 = (uint32_t)iw10 | ((uint32_t)iw11 << 16);
#pragma unroll
            for (int k = 0; k < 9; k++) {                 // gxv = gyv = 0 outside the window
                const int jv = (dot2s(t[k / 3][k % 3], W0, dot2s(t[k / 3 + 1][k % 3], W1, 1 << 8)) >> 9);
                ib1 = __mul24(jv, gxv[k]) + ib1;
                ib2 = __mul24(jv, gyv[k]) + ib2;
            }
            const int64_t tb1 = wave_sum_i32x(ib1), tb2 = wave_sum_i32x(ib2);
            const float b1 = (float)tb1 * FLT_SCALE, b2 = (float)tb2 * FLT_SCALE;
            const float dx = (A12 * b2 - A22 * b1) * D2, dy = (A12 * b1 - A11 * b2) * D2;
            lx += dx; ly += dy;
            nx = lx + hw; ny = ly + hw;
            if ((double)dx * dx + (double)dy * dy <= eps2) break;
            if (j > 0 && fabsf(dx + pdx) < 0.01 && fabsf(dy + pdy) < 0.01) {
                nx -= dx * 0.5f; ny -= dy * 0.5f;
                break;
            }
            pdx = dx; pdy = dy;
        }
        if (level == 0 && st) {
            const float ex = nx - hw, ey = ny - hw;
            const int iex = cv_floor(ex), iey = cv_floor(ey);
            if (iex < -win || iex >= lw || iey < -win || iey >= lh) st = 0;
        }
    }
    if (lane == 0) {
        nxy[2 * p] = nx;
        nxy[2 * p + 1] = ny;
        status[p] = (uint8_t)st;
        if (itcount) { atomicAdd(itcount + 2, nit); atomicAdd(itcount + 3, 1); }
    }
    }
}

// ============================== findFundamentalMat + T_M ==============================
// canonical double acos / log / exp (fdlibm) and cos (the pose kernel's Cody-Waite series)
__constant__ double kFlSin[14] = {0x1.0000000000000p+0, -0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13,
                                  0x1.71de3a556c734p-19, -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33, -0x1.ae7f3e733b81fp-41,
                                  0x1.952c77030ad4ap-49, -0x1.2f49b46814157p-57, 0x1.71b8ef6dcf572p-66, -0x1.761b413163819p-75,
                                  0x1.3f3ccdd165fa9p-84, -0x1.d1ab1c2dccea3p-94};
__constant__ double kFlCos[14] = {0x1.0000000000000p+0, -0x1.0000000000000p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10,
                                  0x1.a01a01a01a01ap-16, -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29, -0x1.93974a8c07c9dp-37,
                                  0x1.ae7f3e733b81fp-45, -0x1.6827863b97d97p-53, 0x1.e542ba4020225p-62, -0x1.0ce396db7f853p-70,
                                  0x1.f2cf01972f578p-80, -0x1.88e85fc6a4e59p-89};

__device__ double fl_cos(double x)
{
    const double k = floor(x * 0.63661977236758134308 + 0.5);
    const double r = (x - k * 1.57079632673412561417e+00) - k * 6.07710050650619224932e-11;
    const double r2 = r * r;
    double ps = kFlSin[13], pc = kFlCos[13];
    for (int n = 12; n >= 0; n--) {
        ps = ps * r2 + kFlSin[n];
        pc = pc * r2 + kFlCos[n];
    }
    const double s0 = r * ps, c0 = pc;
    const int q = ((int)(long)k) & 3;
    return q == 0 ? c0 : q == 1 ? -s0 : q == 2 ? -c0 : s0;
}

__device__ __forceinline__ uint32_t fd_hi(double x) { return (uint32_t)((uint64_t)__double_as_longlong(x) >> 32); }
__device__ __forceinline__ uint32_t fd_lo(double x) { return (uint32_t)(uint64_t)__double_as_longlong(x); }
__device__ __forceinline__ double fd_make(uint32_t hi, uint32_t lo)
{
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ double fd_acos(double x)
{
    const double pi = 0x1.921fb54442d18p+1, pio2_hi = 0x1.921fb54442d18p+0, pio2_lo = 0x1.1a62633145c07p-54;
    const double pS0 = 0x1.5555555555555p-3, pS1 = -0x1.4d61203eb6f7dp-2, pS2 = 0x1.9c1550e884455p-3,
                 pS3 = -0x1.48228b5688f3bp-5, pS4 = 0x1.9efe07501b288p-11, pS5 = 0x1.23de10dfdf709p-15;
    const double qS1 = -0x1.33a271c8a2d4bp+1, qS2 = 0x1.02ae59c598ac8p+1, qS3 = -0x1.6066c1b8d0159p-1,
                 qS4 = 0x1.3b8c5b12e9282p-4;
    const int32_t hx = (int32_t)fd_hi(x), ix = hx & 0x7fffffff;
    if (ix >= 0x3ff00000) {
        if (((ix - 0x3ff00000) | fd_lo(x)) == 0) return hx > 0 ? 0.0 : pi + 2.0 * pio2_lo;
        return __builtin_nan("");
    }
    if (ix < 0x3fe00000) {
        if (ix <= 0x3c600000) return pio2_hi + pio2_lo;
        const double z = x * x;
        const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const double r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    } else if (hx < 0) {
        const double z = (1.0 + x) * 0.5;
        const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const double s = sqrt(z);
        const double r = p / q;
        const double w = r * s - pio2_lo;
        return pi - 2.0 * (s + w);
    }
    const double z = (1.0 - x) * 0.5;
    const double s = sqrt(z);
    const double df = fd_make(fd_hi(s), 0);
    const double c = (z - df * df) / (s + df);
    const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const double r = p / q;
    const double w = r * s + c;
    return 2.0 * (df + w);
}

__device__ double fd_log(double x)
{
    const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33, two54 = 0x1p54;
    const double Lg1 = 0x1.5555555555593p-1, Lg2 = 0x1.999999997fa04p-2, Lg3 = 0x1.2492494229359p-2,
                 Lg4 = 0x1.c71c51d8e78afp-3, Lg5 = 0x1.7466496cb03dep-3, Lg6 = 0x1.39a09d078c69fp-3,
                 Lg7 = 0x1.2f112df3e5244p-3;
    int32_t hx = (int32_t)fd_hi(x);
    const uint32_t lx = fd_lo(x);
    int32_t k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -__builtin_inf();
        if (hx < 0) return __builtin_nan("");
        k -= 54; x *= two54;
        hx = (int32_t)fd_hi(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i0 = (hx + 0x95f64) & 0x100000;
    x = fd_make((uint32_t)(hx | (i0 ^ 0x3ff00000)), fd_lo(x));
    k += (i0 >> 20);
    const double f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            const double dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        const double dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    const double dk = (double)k;
    const double z = s * s;
    int32_t i = hx - 0x6147a;
    const double w = z * z;
    const int32_t j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    const double R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

__device__ double fd_exp(double x)
{
    const double ln2HI = 0x1.62e42fee00000p-1, ln2LO = 0x1.a39ef35793c76p-33, invln2 = 0x1.71547652b82fep+0;
    const double P1 = 0x1.555555555553ep-3, P2 = -0x1.6c16c16bebd93p-9, P3 = 0x1.1566aaf25de2cp-14,
                 P4 = -0x1.bbd41c5d26bf1p-20, P5 = 0x1.6376972bea4d0p-25;
    const double o_threshold = 0x1.62e42fefa39efp+9, u_threshold = -0x1.74910d52d3051p+9;
    uint32_t hx = fd_hi(x);
    const int xsb = (hx >> 31) & 1;
    hx &= 0x7fffffff;
    if (hx >= 0x40862E42) {
        if (hx >= 0x7ff00000) {
            if (((hx & 0xfffff) | fd_lo(x)) != 0) return x + x;
            return xsb == 0 ? x : 0.0;
        }
        if (x > o_threshold) return __builtin_inf();
        if (x < u_threshold) return 0.0;
    }
    double hi = 0, lo = 0;
    int k = 0;
    if (hx > 0x3fd62e42) {
        if (hx < 0x3FF0A2B2) {
            hi = x - (xsb ? -ln2HI : ln2HI); lo = xsb ? -ln2LO : ln2LO; k = 1 - xsb - xsb;
        } else {
            k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
            const double t = k;
            hi = x - t * ln2HI;
            lo = t * ln2LO;
        }
        x = hi - lo;
    } else if (hx < 0x3e300000) {
        return 1.0 + x;
    } else k = 0;
    const double t = x * x;
    const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    if (k >= -1021) return fd_make(fd_hi(y) + ((uint32_t)k << 20), fd_lo(y));
    y = fd_make(fd_hi(y) + ((uint32_t)(k + 1000) << 20), fd_lo(y));
    return y * 0x1p-1000;
}

__device__ __forceinline__ double fd_pow_pos(double x, double y) { return x == 0.0 ? 0.0 : fd_exp(y * fd_log(x)); }

__device__ int solve_cubic(const double c[4], double r[3])
{
    double a0 = c[0], a1 = c[1], a2 = c[2], a3 = c[3], x0 = 0, x1 = 0, x2 = 0;
    int n = 0;
    if (a0 == 0) {
        if (a1 == 0) {
            if (a2 == 0) n = a3 == 0 ? -1 : 0;
            else { x0 = -a3 / a2; n = 1; }
        } else {
            double d = a2 * a2 - 4 * a1 * a3;
            if (d >= 0) {
                d = sqrt(d);
                const double q1 = (-a2 + d) * 0.5, q2 = (a2 + d) * -0.5;
                if (fabs(q1) > fabs(q2)) { x0 = q1 / a1; x1 = a3 / q1; }
                else { x0 = q2 / a1; x1 = a3 / q2; }
                n = d > 0 ? 2 : 1;
            }
        }
    } else {
        a0 = 1. / a0;
        a1 *= a0; a2 *= a0; a3 *= a0;
        const double Q = (a1 * a1 - 3 * a2) * (1. / 9);
        const double R = (2 * a1 * a1 * a1 - 9 * a1 * a2 + 27 * a3) * (1. / 54);
        const double Qcubed = Q * Q * Q;
        double d = Qcubed - R * R;
        if (d > 0) {
            const double theta = fd_acos(R / sqrt(Qcubed));
            const double sqrtQ = sqrt(Q);
            const double t0 = -2 * sqrtQ, t1 = theta * (1. / 3), t2 = a1 * (1. / 3);
            x0 = t0 * fl_cos(t1) - t2;
            x1 = t0 * fl_cos(t1 + (2. * 3.1415926535897932384626433832795 / 3)) - t2;
            x2 = t0 * fl_cos(t1 + (4. * 3.1415926535897932384626433832795 / 3)) - t2;
            n = 3;
        } else if (d == 0) {
            if (R >= 0) { x0 = -2 * fd_pow_pos(R, 1. / 3) - a1 / 3; x1 = fd_pow_pos(R, 1. / 3) - a1 / 3; }
            else { x0 = 2 * fd_pow_pos(-R, 1. / 3) - a1 / 3; x1 = -fd_pow_pos(-R, 1. / 3) - a1 / 3; }
            x2 = 0;
            n = x0 == x1 ? 1 : 2;
            x1 = x0 == x1 ? 0 : x1;
        } else {
            d = sqrt(-d);
            double e = fd_pow_pos(d + fabs(R), 0.333333333333);
            if (R > 0) e = -e;
            x0 = (e + Q / e) - a1 * (1. / 3);
            n = 1;
        }
    }
    r[0] = x0; r[1] = x1; r[2] = x2;
    return n;
}

// run7Point with the null space from complete-pivoting Gauss-Jordan (oracle oc_run7point); A is
// this thread's 7x9 scratch (LDS)
__device__ int run7point(const float2* s1, const float2* s2, double* A, int* perm, double* F)
{
    for (int i = 0; i < 7; i++) {
        const double x0 = s1[i].x, y0 = s1[i].y, x1 = s2[i].x, y1 = s2[i].y;
        double* a = A + 9 * i;
        a[0] = x1 * x0; a[1] = x1 * y0; a[2] = x1;
        a[3] = y1 * x0; a[4] = y1 * y0; a[5] = y1;
        a[6] = x0; a[7] = y0; a[8] = 1;
    }
    for (int j = 0; j < 9; j++) perm[j] = j;
    for (int r = 0; r < 7; r++) {
        int pi = r, pj = r;
        double best = -1.0;
        for (int i = r; i < 7; i++)
            for (int j = r; j < 9; j++)
                if (fabs(A[9 * i + j]) > best) { best = fabs(A[9 * i + j]); pi = i; pj = j; }
        if (!(best > 0.0)) return 0;
        if (pi != r)
            for (int j = 0; j < 9; j++) { const double t = A[9 * r + j]; A[9 * r + j] = A[9 * pi + j]; A[9 * pi + j] = t; }
        if (pj != r) {
            for (int i = 0; i < 7; i++) { const double t = A[9 * i + r]; A[9 * i + r] = A[9 * i + pj]; A[9 * i + pj] = t; }
            const int t = perm[r]; perm[r] = perm[pj]; perm[pj] = t;
        }
        const double piv = A[9 * r + r];
        for (int i = 0; i < 7; i++) {
            if (i == r) continue;
            const double f = A[9 * i + r] / piv;
            for (int j = r; j < 9; j++) A[9 * i + j] = A[9 * i + j] - f * A[9 * r + j];
        }
    }
    double f1[9], f2[9];
    // v[perm[i]] = -A[i][col] / A[i][i] (i < 7), v[perm[7]], v[perm[8]] = unit (a gather over the
    // inverse permutation keeps f1/f2 in registers)
#pragma unroll
    for (int q = 0; q < 9; q++) {
        double v1 = 0, v2 = 0;
        for (int i = 0; i < 9; i++) {
            if (perm[i] != q) continue;
            if (i < 7) { v1 = -A[9 * i + 7] / A[9 * i + i]; v2 = -A[9 * i + 8] / A[9 * i + i]; }
            else if (i == 7) { v1 = 1.0; v2 = 0.0; }
            else { v1 = 0.0; v2 = 1.0; }
        }
        f1[q] = v1; f2[q] = v2;
    }
#pragma unroll
    for (int i = 0; i < 9; i++) f1[i] -= f2[i];
    double c[4], rr[3];
    double t0 = f2[4] * f2[8] - f2[5] * f2[7];
    double t1 = f2[3] * f2[8] - f2[5] * f2[6];
    double t2 = f2[3] * f2[7] - f2[4] * f2[6];
    c[3] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2;
    c[2] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2 - f1[3] * (f2[1] * f2[8] - f2[2] * f2[7]) +
           f1[4] * (f2[0] * f2[8] - f2[2] * f2[6]) - f1[5] * (f2[0] * f2[7] - f2[1] * f2[6]) +
           f1[6] * (f2[1] * f2[5] - f2[2] * f2[4]) - f1[7] * (f2[0] * f2[5] - f2[2] * f2[3]) +
           f1[8] * (f2[0] * f2[4] - f2[1] * f2[3]);
    t0 = f1[4] * f1[8] - f1[5] * f1[7];
    t1 = f1[3] * f1[8] - f1[5] * f1[6];
    t2 = f1[3] * f1[7] - f1[4] * f1[6];
    c[1] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2 - f2[3] * (f1[1] * f1[8] - f1[2] * f1[7]) +
           f2[4] * (f1[0] * f1[8] - f1[2] * f1[6]) - f2[5] * (f1[0] * f1[7] - f1[1] * f1[6]) +
           f2[6] * (f1[1] * f1[5] - f1[2] * f1[4]) - f2[7] * (f1[0] * f1[5] - f1[2] * f1[3]) +
           f2[8] * (f1[0] * f1[4] - f1[1] * f1[3]);
    c[0] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2;
    const int n = solve_cubic(c, rr);
    if (n < 1 || n > 3) return n;
    for (int k = 0; k < n; k++) {
        double* fm = F + 9 * k;
        const double rk = k == 0 ? rr[0] : k == 1 ? rr[1] : rr[2];
        double lambda = rk, mu = 1.;
        const double s = f1[8] * rk + f2[8];
        if (fabs(s) > DBL_EPSILON) { mu = 1. / s; lambda *= mu; fm[8] = 1.; }
        else fm[8] = 0.;
#pragma unroll
        for (int i = 0; i < 8; i++) fm[i] = f1[i] * lambda + f2[i] * mu;
    }
    return n;
}

__device__ __forceinline__ float fm_error(const double* F, float x1, float y1, float x2, float y2)
{
    double a = F[0] * x1 + F[1] * y1 + F[2];
    double b = F[3] * x1 + F[4] * y1 + F[5];
    double c = F[6] * x1 + F[7] * y1 + F[8];
    const double s2 = 1. / (a * a + b * b);
    const double d2 = x2 * a + y2 * b + c;
    a = F[0] * x2 + F[3] * y2 + F[6];
    b = F[1] * x2 + F[4] * y2 + F[7];
    c = F[2] * x2 + F[5] * y2 + F[8];
    const double s1 = 1. / (a * a + b * b);
    const double d1 = x1 * a + y1 * b + c;
    const double e1 = d1 * d1 * s1, e2 = d2 * d2 * s2;
    return (float)(e1 < e2 ? e2 : e1);
}

__device__ bool fm_collinear(const float2* m)
{
    const int i = 6;
    for (int j = 0; j < i; j++) {
        const double dx1 = (double)(m[j].x - m[i].x), dy1 = (double)(m[j].y - m[i].y);
        for (int k = 0; k < j; k++) {
            const double dx2 = (double)(m[k].x - m[i].x), dy2 = (double)(m[k].y - m[i].y);
            if (fabs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return true;
        }
    }
    return false;
}

__device__ __forceinline__ unsigned rng_next(uint64_t& st)
{
    st = (uint64_t)(unsigned)st * 4164903690U + (unsigned)(st >> 32);
    return (unsigned)st;
}

// RANSACUpdateNumIters(p, ep, 7, maxIters) in the canonical forms (oracle oc_ransac_update_iters)
__device__ int ransac_update_iters(double p, double ep, int max_iters)
{
    p = p > 0. ? p : 0.; p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.; ep = ep < 1. ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    const double b = 1. - ep;
    double denom = 1. - b * b * b * b * b * b * b;
    if (denom < DBL_MIN) return 0;
    num = fd_log(num);
    denom = fd_log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)rint(num / denom);
}

struct FmOut {
    float* tm;          // T_M (x, y) pairs
    int* ntm;           // |T_M|, -1 when F is empty
    uint8_t* state;     // state after the SAD check (optional)
    double* F;          // 9 (optional)
    int* nf;            // |F_prepoint| (optional)
    int tm_cap;
    int64_t tm_z;       // batch: pair stride of tm / ntm in bytes when they are caller buffers (0: the pair block)
};

// NT threads per pair (COEB_FM_THREADS, default kFmThreads): the (hypothesis, model) scoring runs
// NT / 64 waves wide, and the pair's latency is mostly the serial draws, 7-point solves and scan.
// Per 513-pair launch (config D, profiles/r05/s25-s27): 1024 threads 0.81 ms (128 VGPRs and 208 B
// of spills per lane, one pair per CU), 512 0.78, 256 0.46, 128 0.34 (191-203 VGPRs, no spills,
// two pairs per CU in one round); config D's step 13.14-13.27 -> 12.35-12.43 ms at 128.
#ifndef COEB_FM_MINWG
#define COEB_FM_MINWG 0        // launch bound in waves per SIMD (0: the defaults below)
#endif
// The bound steers the register allocator more than the occupancy: k_fm<128> cannot reach 6 waves per
// SIMD (its 45 KB of LDS allow 3 workgroups per CU) and lands on 203 VGPRs either way, but with a
// 6-wave bound it spills 17 SGPRs instead of 74 (and 60 B of VGPRs to scratch) and runs 0.336-0.338
// ms per 513-pair launch against 0.516-0.523 at 2-4 (profiles/r05/s30).
template <int NT>
constexpr int fm_bound() { return COEB_FM_MINWG ? COEB_FM_MINWG : NT == 1024 ? 4 : NT == 128 ? 6 : 2; }
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wpass-failed"
template <int NT>
__global__ __launch_bounds__(NT, fm_bound<NT>()) void k_fm(const uint8_t* __restrict__ prev, const uint8_t* __restrict__ cur,
                                                  int w, int h, int stride, const float* __restrict__ pxy,
                                                  const float* __restrict__ nxy, const uint8_t* __restrict__ status,
                                                  const int* __restrict__ d_n, int nmax, int edge, double limit,
                                                  double thr, double conf, FmOut out, int64_t iz, int64_t pz)
{
    prev = at_pair(prev, iz);
    cur = at_pair(cur, iz);
    pxy = at_pair(pxy, pz);
    nxy = at_pair(nxy, pz);
    status = at_pair(status, pz);
    d_n = at_pair(d_n, pz);
    out.tm = at_pair(out.tm, out.tm_z ? out.tm_z : pz);
    out.ntm = at_pair(out.ntm, out.tm_z ? 4 : pz);
    out.state = at_pair(out.state, pz);
    out.F = at_pair(out.F, pz);
    out.nf = at_pair(out.nf, pz);
    __shared__ float2 s_m1[kMaxPts], s_m2[kMaxPts];
    __shared__ uint16_t s_map[kMaxPts];
    __shared__ int s_w[16];
    __shared__ double s_A[kFmChunk][63];
    __shared__ int s_perm[kFmChunk][9];
    __shared__ double s_models[kFmChunk][27];
    __shared__ int s_nm[kFmChunk];
    __shared__ float2 s_sub1[kFmChunk][7], s_sub2[kFmChunk][7];
    __shared__ int s_found[kFmChunk];
    __shared__ int s_good[kFmChunk * 3];
    __shared__ float s_med[kFmChunk * 3];
    __shared__ double s_F[9];
    __shared__ int s_ok, s_done, s_niters, s_base;
    __shared__ uint64_t s_rng;
    constexpr int E = kMaxPts / NT;     // points per thread in the ordered compactions
    static_assert(E * NT == kMaxPts && NT >= 128 && NT <= 1024, "k_fm thread count");
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int n = *d_n;
    n = n < nmax ? n : nmax;
    n = n < kMaxPts ? n : kMaxPts;
    // ---- SAD check (Frame.cc:337-365) and the ordered F_ sets: thread t takes points E t .. E t + E - 1
    //      (the E loads of a thread are independent; rounds of NT points with a block scan each
    //      measured slower, 0.38 vs 0.34 ms per 513-pair launch at 128 threads) ----
    int keep[E], cnt = 0;
    float2 p1[E], p2[E];
#pragma unroll
    for (int j = 0; j < E; j++) {
        const int i = E * tid + j;
        keep[j] = 0;
        p1[j] = make_float2(0.f, 0.f); p2[j] = p1[j];
        if (i < n) {
            uint8_t st = status[i];
            p1[j] = make_float2(pxy[2 * i], pxy[2 * i + 1]);
            p2[j] = make_float2(nxy[2 * i], nxy[2 * i + 1]);
            if (st) {
                const int x1 = (int)p1[j].x, y1 = (int)p1[j].y, x2 = (int)p2[j].x, y2 = (int)p2[j].y;
                if (x1 < edge || x1 >= w - edge || x2 < edge || x2 >= w - edge || y1 < edge || y1 >= h - edge ||
                    y2 < edge || y2 >= h - edge) {
                    st = 0;
                } else {
                    double sum = 0;
                    for (int k = 0; k < 9; k++) {
                        const int dx = k % 3 - 1, dy = k / 3 - 1;
                        sum += (double)abs((int)prev[(size_t)(y1 + dy) * stride + x1 + dx] -
                                           (int)cur[(size_t)(y2 + dy) * stride + x2 + dx]);
                    }
                    if (sum > limit) st = 0;
                }
            }
            keep[j] = st != 0;
            if (out.state) out.state[i] = (uint8_t)keep[j];
        }
        cnt += keep[j];
    }
    int pos;
    const int nf = block_scan_counts<NT>(cnt, s_w, pos);
#pragma unroll
    for (int j = 0; j < E; j++)
        if (keep[j]) { s_m1[pos] = p1[j]; s_m2[pos] = p2[j]; s_map[pos] = (uint16_t)(E * tid + j); pos++; }
    if (tid == 0) {
        s_ok = 0; s_done = 0; s_base = 0; s_rng = ~0ull;
        if (out.nf) *out.nf = nf;
    }
    __syncthreads();
    // ---- findFundamentalMat ----
    if (nf == 7) {
        if (tid == 0) {
            const int k = run7point(s_m1, s_m2, s_A[0], s_perm[0], s_models[0]);
            if (k > 0) {
                for (int q = 0; q < 9; q++) s_F[q] = s_models[0][q];
                s_ok = 1;
            }
        }
    } else if (nf >= 8) {
        const bool ransac = nf >= 15;
        const int max_attempts = ransac ? 10000 : 1000;
        const float t = (float)(thr * thr);
        int max_good = 0;           // lane 0 state
        double min_median = DBL_MAX;
        if (tid == 0) {
            if (ransac) s_niters = 1000;
            else {
                const int ni = ransac_update_iters(conf, 0.45, 1000);
                s_niters = ni > 3 ? ni : 3;
            }
        }
        __syncthreads();
        for (;;) {
            const int base = s_base, niters = s_niters;
            if (s_done || base >= niters) break;
            // draws for iterations base .. base + kFmChunk - 1 (getSubset, checkPartialSubsets = false)
            if (tid == 0) {
                uint64_t rng = s_rng;
                for (int hh = 0; hh < kFmChunk; hh++) {
                    int idx[7];
                    int iters = 0, i = 0;
                    for (; iters < max_attempts; iters++) {
                        for (i = 0; i < 7 && iters < max_attempts;) {
                            int id;
                            for (;;) {
                                id = (int)(rng_next(rng) % (unsigned)nf);
                                int j;
                                for (j = 0; j < i; j++)
                                    if (id == idx[j]) break;
                                if (j == i) break;
                            }
                            idx[i] = id;
                            s_sub1[hh][i] = s_m1[id];
                            s_sub2[hh][i] = s_m2[id];
                            i++;
                        }
                        if (i == 7 && (fm_collinear(s_sub1[hh]) || fm_collinear(s_sub2[hh]))) continue;
                        break;
                    }
                    s_found[hh] = i == 7 && iters < max_attempts;
                }
                s_rng = rng;
            }
            __syncthreads();
            if (tid < kFmChunk) s_nm[tid] = s_found[tid] ? run7point(s_sub1[tid], s_sub2[tid], s_A[tid], s_perm[tid], s_models[tid]) : 0;
            __syncthreads();
            // score every (hypothesis, model): one wave each
            for (int pr = wv; pr < kFmChunk * 3; pr += NT / 64) {
                const int hh = pr / 3, m = pr - hh * 3;
                if (m >= s_nm[hh]) continue;
                const double* F = s_models[hh] + 9 * m;
                if (ransac) {
                    int good = 0;
                    for (int i = lane; i < nf; i += 64)
                        good += fm_error(F, s_m1[i].x, s_m1[i].y, s_m2[i].x, s_m2[i].y) <= t;
                    for (int off = 32; off >= 1; off >>= 1) good += __shfl_xor(good, off, 64);
                    if (lane == 0) s_good[pr] = good;
                } else if (lane == 0) {
                    float e[16];
                    for (int i = 0; i < nf; i++) e[i] = fm_error(F, s_m1[i].x, s_m1[i].y, s_m2[i].x, s_m2[i].y);
                    for (int a = 1; a < nf; a++) {
                        const float v = e[a];
                        int b = a - 1;
                        while (b >= 0 && e[b] > v) { e[b + 1] = e[b]; b--; }
                        e[b + 1] = v;
                    }
                    s_med[pr] = e[nf / 2];
                }
            }
            __syncthreads();
            // the reference's sequential scan (ptsetreg.cpp run loops)
            if (tid == 0) {
                int ni = niters;
                for (int hh = 0; hh < kFmChunk; hh++) {
                    const int iter = base + hh;
                    if (iter >= ni) { s_done = 1; break; }
                    if (!s_found[hh]) {
                        if (iter == 0) s_ok = -1;
                        s_done = 1;
                        break;
                    }
                    for (int m = 0; m < s_nm[hh]; m++) {
                        if (ransac) {
                            const int good = s_good[hh * 3 + m];
                            if (good > (max_good > 6 ? max_good : 6)) {
                                for (int q = 0; q < 9; q++) s_F[q] = s_models[hh][9 * m + q];
                                max_good = good;
                                s_ok = 1;
                                ni = ransac_update_iters(conf, (double)(nf - good) / nf, ni);
                            }
                        } else {
                            const double med = s_med[hh * 3 + m];
                            if (med < min_median) {
                                min_median = med;
                                for (int q = 0; q < 9; q++) s_F[q] = s_models[hh][9 * m + q];
                            }
                        }
                    }
                }
                s_niters = ni;
                s_base = base + kFmChunk;
                if (!ransac && !s_done && s_base >= ni) s_done = 1;
                if (!ransac && s_done && s_ok != -1) {
                    if (min_median < DBL_MAX) {
                        double sigma = 2.5 * 1.4826 * (1 + 5. / (nf - 7)) * sqrt(min_median);
                        sigma = sigma > 0.001 ? sigma : 0.001;
                        const float tt = (float)(sigma * sigma);
                        int good = 0;
                        for (int i = 0; i < nf; i++) good += fm_error(s_F, s_m1[i].x, s_m1[i].y, s_m2[i].x, s_m2[i].y) <= tt;
                        s_ok = good >= 7 ? 1 : 0;
                    } else s_ok = 0;
                }
                if (ransac && s_ok == 1 && max_good <= 0) s_ok = 0;
            }
            __syncthreads();
        }
    }
    __syncthreads();
    // ---- epipolar distance > 1 -> T_M (Frame.cc:375-384), in point order ----
    if (s_ok != 1) {
        if (tid == 0) *out.ntm = -1;
        return;
    }
    if (tid < 9 && out.F) out.F[tid] = s_F[tid];
    int flag[E], fcnt = 0;
    float2 q2[E];
#pragma unroll
    for (int j = 0; j < E; j++) {
        const int i = E * tid + j;
        flag[j] = 0;
        q2[j] = make_float2(0.f, 0.f);
        if (i < nf) {
            const float2 q1 = s_m1[i];
            q2[j] = s_m2[i];
            const double px = q1.x, py = q1.y;
            const double A = s_F[0] * px + s_F[1] * py + s_F[2];
            const double B = s_F[3] * px + s_F[4] * py + s_F[5];
            const double Cc = s_F[6] * px + s_F[7] * py + s_F[8];
            const double dd = fabs(A * q2[j].x + B * q2[j].y + Cc) / sqrt(A * A + B * B);
            flag[j] = !(dd <= 1);
        }
        fcnt += flag[j];
    }
    int tpos;
    const int nt = block_scan_counts<NT>(fcnt, s_w, tpos);
#pragma unroll
    for (int j = 0; j < E; j++)
        if (flag[j]) {
            if (tpos < out.tm_cap) {
                out.tm[2 * tpos] = q2[j].x;
                out.tm[2 * tpos + 1] = q2[j].y;
            }
            tpos++;
        }
    if (tid == 0) *out.ntm = nt;
}

#pragma clang diagnostic pop

// ============================== host side ==============================
struct FlowDev {
    uint8_t *prev, *cur;                // packed (pitch w) copies of the two frames
    float* R;
    uint32_t* rmax;
    int* nkeys;
    uint64_t* keys;
    float *pts, *nxt;
    int* npts;
    uint8_t *status, *state;
    float* mexp;                        // cornerSubPix weight factors e_k = expf(-x_k^2), k < 21
    uint8_t* pyr;                       // levels 1.. of both frames
    short2* der;                        // Scharr of every previous-frame level
    float* tm;
    int* ntm;
    double* F;
    int* nf;
    // batch layout: every pointer above but prev / cur / mexp is pair 0's; pair z's copy is
    // pz * z bytes further on
    int npairs;
    int64_t pz;
    int* offs;                          // k_flow_index: points before each pair, [npairs] = all
    int* order;                         // k_subpix_order: corner work order (interior first)
    int* ocnt;                          // its two counters
    ProfileHook* prof = nullptr;        // the context's HIP-event profiler (coeb_profile_enable)
};

// one launch bracketed by the context profiler's event pair (a no-op unless profiling is on)
#define FLOW_LAUNCH(d, name, s, ...)                 \
    do {                                             \
        prof_begin((d)->prof, name, s);              \
        hipLaunchKernelGGL(__VA_ARGS__);             \
        prof_end((d)->prof, s);                      \
    } while (0)

int lk_levels(int w, int h, int win, int max_level)
{
    for (int level = 0; level <= max_level; level++) {
        w = (w + 1) / 2; h = (h + 1) / 2;
        if (w <= win || h <= win) return level + 1;
    }
    return max_level + 1;
}

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }
constexpr size_t kSubpixMaskBytes = sizeof(float) * 21;   // subpix_mask

int flow_alloc(coeb_ctx* c, int w, int h, FlowDev* d, int npairs = 1)
{
    size_t pyr_bytes = 0, der_px = 0;
    {
        int lw = w, lh = h;
        der_px += (size_t)lw * lh;
        for (int l = 1; l < kLkMaxLevels; l++) {
            lw = (lw + 1) / 2; lh = (lh + 1) / 2;
            pyr_bytes += 2 * align256((size_t)lw * lh);
            der_px += (size_t)lw * lh;
        }
    }
    // shared: the two frame copies of the host entry points, the subpix weights; then one block
    // per pair
    const size_t shared[] = {align256((size_t)w * h), align256((size_t)w * h), align256(kSubpixMaskBytes),
                             align256(sizeof(int) * ((size_t)npairs + 1)), align256(sizeof(int) * (size_t)npairs * kMaxPts),
                             256};
    const size_t sizes[] = {align256((size_t)w * h * 4), 256, 256, align256((size_t)gf_key_cap(w, h) * 8),
                            align256((size_t)kMaxPts * 8),
                            align256((size_t)kMaxPts * 8), 256, align256(kMaxPts), align256(kMaxPts), align256(pyr_bytes),
                            align256(der_px * 4 + 64 * kLkMaxLevels), align256((size_t)kMaxPts * 8), 256, 256, 256};
    size_t pair_bytes = 0, shared_bytes = 0;
    for (size_t v : sizes) pair_bytes += v;
    for (size_t v : shared) shared_bytes += v;
    void* base;
    // npairs + 1 blocks: a batch's pyramids are kept per frame, pair z's next frame being pair
    // z + 1's previous one (launch_lk), so frame `npairs` needs a block of its own
    const int rc = coeb_internal_scratch(c, "flow", shared_bytes + pair_bytes * (size_t)(npairs + 1), &base);
    if (rc) return rc;
    uint8_t* p = (uint8_t*)base;
    size_t o = 0;
    d->prev = p + o; o += shared[0];
    d->cur = p + o; o += shared[1];
    d->mexp = (float*)(p + o); o += shared[2];
    d->offs = (int*)(p + o); o += shared[3];
    d->order = (int*)(p + o); o += shared[4];
    d->ocnt = (int*)(p + o); o += shared[5];
    int i = 0;
    auto take = [&]() { void* r = p + o; o += sizes[i++]; return r; };
    d->R = (float*)take(); d->rmax = (uint32_t*)take(); d->nkeys = (int*)take(); d->keys = (uint64_t*)take();
    d->pts = (float*)take(); d->nxt = (float*)take(); d->npts = (int*)take();
    d->status = (uint8_t*)take(); d->state = (uint8_t*)take(); d->pyr = (uint8_t*)take(); d->der = (short2*)take();
    d->tm = (float*)take(); d->ntm = (int*)take(); d->F = (double*)take(); d->nf = (int*)take();
    d->npairs = npairs;
    d->pz = (int64_t)pair_bytes;
    d->prof = coeb_internal_prof(c);
    return COEB_OK;
}

size_t gf_select_lds(int w, int h, int cell, int np)
{
    const int gw = (w + cell - 1) / cell, gh = (h + cell - 1) / cell;
    // sorted keys, per-cell list heads (u16), per accepted corner: next (u16) and x | y << 16
    return (size_t)(np > 1 ? np : 2) * 8 + (size_t)((gw * gh + 1) & ~1) * 2 + (size_t)kMaxPts * (2 + 4);
}

// goodFeaturesToTrack into d->pts / d->npts (device count: -1 when the sort capacity is exceeded)
int launch_gf(const FlowDev* d, const uint8_t* img, int w, int h, int stride, int max_corners, double quality,
              double min_distance, double k, hipStream_t s, int64_t iz = 0)
{
    const int P = d->npairs;
    const int cell = (int)lrint(min_distance);
    if (cell < 1) return -2;
    const size_t lds = gf_select_lds(w, h, cell, kGfBatch);
    if (lds > 160 * 1024) return -2;
    (void)hipMemset2DAsync(d->rmax, (size_t)d->pz, 0, 4, P, s);      // one word per pair
    (void)hipMemset2DAsync(d->nkeys, (size_t)d->pz, 0, 4, P, s);
    FLOW_LAUNCH(d, "k_gf_response", s, k_gf_response, dim3((w + 4 * kGfCols - 1) / (4 * kGfCols), (h + kGfRows - 1) / kGfRows, P),
                dim3(256), 0, s, img, w, h,
                       stride, k, d->R, d->rmax, iz, d->pz);
    FLOW_LAUNCH(d, "k_gf_candidates", s, k_gf_candidates,
                dim3((w + 4 * kGcCols - 1) / (4 * kGcCols), (h + kGcRows - 1) / kGcRows, P), dim3(256), 0, s, d->R, w,
                h, quality, d->rmax, d->keys, d->nkeys,
                       gf_key_cap(w, h), d->pz);
    lds_limit_max((const void*)k_gf_select);
    FLOW_LAUNCH(d, "k_gf_select", s, k_gf_select, dim3(1, 1, P), dim3(kGfThreads), lds, s, d->keys, d->nkeys, w, h, max_corners,
                       (float)(min_distance * min_distance), cell, d->pts, d->npts, kMaxPts, gf_key_cap(w, h),
                       d->pz);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the flattened point list of every pair (k_flow_index) for k_subpix / k_lk: the corners of
// goodFeaturesToTrack, which both consume unchanged (cornerSubPix refines them in place)
void launch_flow_index(const FlowDev* d, hipStream_t s)
{
    hipLaunchKernelGGL(k_flow_index, dim3(1), dim3(1024), 0, s, d->npts, d->pz, d->npairs, kMaxPts, d->offs);
}

// workgroups of a persistent per-point launch (ipw points per workgroup and pass): enough to
// fill the chip several times over, never more than there can be points
int flow_grid(const FlowDev* d, int ipw)
{
    const int64_t most = (int64_t)d->npairs * kMaxPts;
    const int64_t want = 256 * 32;                   // workgroups: 32 per CU
    return (int)std::max<int64_t>(1, std::min<int64_t>((most + ipw - 1) / ipw, want));
}

// cornerSubPix's weights (cornerSubPix: mask(i, j) = vy_i * expf(-x_j^2) in float, x = (k - win) /
// win): the 2 win + 1 float factors e_k, so mask(i, j) = e_i * e_j (k_subpix forms the product)
void subpix_mask(int win, float* ex)
{
    const int n = 2 * win + 1;
    for (int k = 0; k < n; k++) {
        const float x = (float)(k - win) / (float)win;
        ex[k] = expf(-x * x);
    }
}

int launch_subpix(const FlowDev* d, const uint8_t* img, int w, int h, int stride, int max_iter, double eps,
                  hipStream_t s, int64_t iz = 0)
{
    const int iters = max_iter < 1 ? 1 : max_iter > 100 ? 100 : max_iter;
    const double e = eps > 0 ? eps : 0.;
    int* itc = nullptr;
    if (coeb_experiment("COEB_SUBPIX_COUNT")) {
        if (!g_subpix_count) (void)hipGetSymbolAddress((void**)&g_subpix_count, HIP_SYMBOL(g_subpix_count_dev));
        itc = g_subpix_count;
    }
    launch_flow_index(d, s);
    (void)hipMemsetAsync(d->ocnt, 0, 12, s);            // {interior, border, corner queue}
    // interior: the window (23 x 23 around the corner, +1 for the interpolation) stays inside the
    // image with 2 px of drift to spare
    hipLaunchKernelGGL(k_subpix_order, dim3(flow_grid(d, 256)), dim3(256), 0, s, d->pts, d->offs, d->npairs, w, h, 14,
                       d->pz, d->order, d->ocnt);
    FLOW_LAUNCH(d, "k_subpix", s, k_subpix<kSpSlots>, dim3(flow_grid(d, 8 * kSpSlots)), dim3(64), 0, s, img, w, h, stride,
                d->pts, d->offs, d->npairs, d->order, d->ocnt + 2, d->mexp, iters, e * e, iz, d->pz, itc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// LK pyramids of both frames (pyrDown levels and the Scharr derivatives of every level): they read
// only the images, so a batch builds them on a second stream beside goodFeaturesToTrack and
// cornerSubPix (coeb_internal_pmo_batch); `pyr` is filled for launch_lk_track.
int launch_lk_pyramids(const FlowDev* d, const uint8_t* prev, const uint8_t* cur, int w, int h, int stride, int win,
                       int max_level, hipStream_t s, int64_t iz, LkPyr& pyr)
{
    const int P = d->npairs;
    memset(&pyr, 0, sizeof(pyr));
    const int L = lk_levels(w, h, win, max_level);
    if (L > kLkMaxLevels) return -2;
    pyr.L = L;
    pyr.P[0] = prev; pyr.N[0] = cur; pyr.w[0] = w; pyr.h[0] = h; pyr.pitch[0] = stride;
    uint8_t* q = d->pyr;
    short2* dq = d->der;
    pyr.D[0] = dq;
    dq += (size_t)w * h;
    // consecutive frames of a batch (pair z = frames z, z + 1): one pyramid per frame, in pair
    // block z, and pair z's next-frame pyramid is pair z + 1's previous-frame one
    const bool chained = P > 1 && iz != 0 && cur == prev + iz;
    for (int l = 1; l < L; l++) {
        pyr.w[l] = (pyr.w[l - 1] + 1) / 2; pyr.h[l] = (pyr.h[l - 1] + 1) / 2; pyr.pitch[l] = pyr.w[l];
        const size_t sz = (size_t)pyr.w[l] * pyr.h[l];
        pyr.P[l] = q; q += align256(sz);
        pyr.N[l] = chained ? pyr.P[l] + d->pz : q; q += align256(sz);
        pyr.D[l] = dq; dq += sz;
        PyrDownArgs a;
        a.src[0] = pyr.P[l - 1]; a.src[1] = pyr.N[l - 1];
        a.dst[0] = const_cast<uint8_t*>(pyr.P[l]); a.dst[1] = const_cast<uint8_t*>(pyr.N[l]);
        a.sw = pyr.w[l - 1]; a.sh = pyr.h[l - 1]; a.spitch = pyr.pitch[l - 1]; a.dw = pyr.w[l]; a.dh = pyr.h[l];
        a.src_img = l == 1;
        a.nfr = chained ? 1 : 2;
        FLOW_LAUNCH(d, "k_pyr_down", s, k_pyr_down, dim3((a.dw + 4 * kPdCols - 1) / (4 * kPdCols), (a.dh + kPdRows - 1) / kPdRows,
                                                         chained ? P + 1 : 2 * P), dim3(256), 0, s, a,
                           iz, d->pz);
    }
    const int sh_items = ((w + kShCols - 1) / kShCols) * ((h + kShRows - 1) / kShRows);   // level 0 is the largest
    FLOW_LAUNCH(d, "k_sharr", s, k_sharr, dim3((sh_items + 3) / 4, L, P), dim3(256), 0, s, pyr, iz, d->pz);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The LK iterations on the pyramids launch_lk_pyramids built (ordered before this on `s`).
int launch_lk_track(const FlowDev* d, const LkPyr& pyr, int win, int max_count, double eps, hipStream_t s,
                    int64_t iz)
{
    const int P = d->npairs;
    launch_flow_index(d, s);            // the host LK entry point sets npts without cornerSubPix
    int* itc = nullptr;
    if (coeb_experiment("COEB_SUBPIX_COUNT")) {
        if (!g_subpix_count) (void)hipGetSymbolAddress((void**)&g_subpix_count, HIP_SYMBOL(g_subpix_count_dev));
        itc = g_subpix_count;
    }
    FLOW_LAUNCH(d, "k_lk", s, k_lk, dim3(flow_grid(d, 4)), dim3(256), 0, s, pyr, d->pts, d->offs, P, d->nxt,
                d->status, win, max_count, eps * eps, iz, d->pz, itc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_lk(const FlowDev* d, const uint8_t* prev, const uint8_t* cur, int w, int h, int stride, int win,
              int max_level, int max_count, double eps, hipStream_t s, int64_t iz = 0)
{
    LkPyr pyr;
    const int rc = launch_lk_pyramids(d, prev, cur, w, h, stride, win, max_level, s, iz, pyr);
    if (rc) return rc;
    return launch_lk_track(d, pyr, win, max_count, eps, s, iz);
}

int launch_fm(const FlowDev* d, const uint8_t* prev, const uint8_t* cur, int w, int h, int stride, int edge, double limit,
              hipStream_t s, int tm_cap, int64_t iz = 0, float* tm_out = nullptr, int* ntm_out = nullptr)
{
    FmOut o;
    o.tm = d->tm; o.ntm = d->ntm; o.state = d->state; o.F = d->F; o.nf = d->nf; o.tm_cap = tm_cap; o.tm_z = 0;
    const FmOut oo = tm_out ? FmOut{tm_out, ntm_out, o.state, o.F, o.nf, tm_cap, (int64_t)tm_cap * 8} : o;
    int nt = kFmThreads;
    if (const char* e = coeb_switch("COEB_FM_THREADS")) nt = atoi(e);
#define COEB_FM_GO(NT_)                                                                                          \
    FLOW_LAUNCH(d, "k_fm", s, k_fm<NT_>, dim3(1, 1, d->npairs), dim3(NT_), 0, s, prev, cur, w, h, stride, d->pts, \
                d->nxt, d->status, d->npts, kMaxPts, edge, limit, 0.1, 0.99, oo, iz, d->pz)
    if (nt == 128) COEB_FM_GO(128);
    else if (nt == 256) COEB_FM_GO(256);
    else if (nt == 512) COEB_FM_GO(512);
    else COEB_FM_GO(1024);
#undef COEB_FM_GO
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#define FL_TRY(c, x)                                                                          \
    do {                                                                                      \
        const hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) return coeb_internal_error(c, COEB_EDEVICE, hipGetErrorString(e_)); \
    } while (0)

struct FlowCall {
    hipStream_t s;
    FlowDev d;
};

int flow_begin(coeb_ctx* c, int w, int h, FlowCall* fc, const char* who)
{
    int dev;
    if (coeb_internal_stream(c, &fc->s, &dev)) return coeb_internal_error(c, COEB_EINVAL, who);
    (void)hipSetDevice(dev);
    if (w < 32 || h < 32 || (size_t)w * h > (size_t)1 << 26) return coeb_internal_error(c, COEB_EINVAL, who);
    // a single-pair call rewrites the flow scratch with npairs = 1: the last batch's geometry
    // no longer describes it, so coeb_internal_flow_counts must refuse rather than misread
    coeb_internal_flow_forget(c);
    return flow_alloc(c, w, h, &fc->d);
}

int upload_gray(coeb_ctx* c, hipStream_t s, uint8_t* dst, const uint8_t* src, int w, int h, size_t stride)
{
    FL_TRY(c, hipMemcpy2DAsync(dst, (size_t)w, src, stride, (size_t)w, h, hipMemcpyHostToDevice, s));
    return COEB_OK;
}

}  // namespace

extern "C" int coeb_good_features(coeb_ctx* c, const uint8_t* img, int w, int h, size_t stride, int max_corners,
                                  double quality, double min_distance, double k, float* xy_out, int cap, int* n_out)
{
    if (!c || !img || !n_out || (cap > 0 && !xy_out) || stride < (size_t)w || quality <= 0 || min_distance < 1)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_good_features: invalid arguments");
    if (max_corners <= 0 || max_corners > kMaxPts)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_good_features: max_corners must be in 1..1024");
    FlowCall fc;
    int rc = flow_begin(c, w, h, &fc, "coeb_good_features: invalid arguments");
    if (rc) return rc;
    if ((rc = upload_gray(c, fc.s, fc.d.prev, img, w, h, stride))) return rc;
    if (launch_gf(&fc.d, fc.d.prev, w, h, w, max_corners, quality, min_distance, k, fc.s))
        return coeb_internal_error(c, COEB_EDEVICE, "coeb_good_features: launch failed");
    int n = 0;
    FL_TRY(c, hipMemcpyAsync(&n, fc.d.npts, 4, hipMemcpyDeviceToHost, fc.s));
    FL_TRY(c, hipStreamSynchronize(fc.s));
    if (n < 0) return coeb_internal_error(c, COEB_ERANGE, "coeb_good_features: more local maxima than the exact selection covers");
    if (n > 0 && cap > 0) {
        FL_TRY(c, hipMemcpyAsync(xy_out, fc.d.pts, (size_t)(n < cap ? n : cap) * 8, hipMemcpyDeviceToHost, fc.s));
        FL_TRY(c, hipStreamSynchronize(fc.s));
    }
    *n_out = n;
    return COEB_OK;
}

extern "C" int coeb_corner_subpix(coeb_ctx* c, const uint8_t* img, int w, int h, size_t stride, float* xy, int n,
                                  int win, int max_iter, double eps)
{
    if (!c || !img || n < 0 || n > kMaxPts || (n > 0 && !xy) || stride < (size_t)w)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_corner_subpix: invalid arguments");
    if (win != 10) return coeb_internal_error(c, COEB_EINVAL, "coeb_corner_subpix: window 10 only (Frame.cc:334)");
    if (n == 0) return COEB_OK;
    FlowCall fc;
    int rc = flow_begin(c, w, h, &fc, "coeb_corner_subpix: invalid arguments");
    if (rc) return rc;
    float mask[21];
    subpix_mask(win, mask);
    if ((rc = upload_gray(c, fc.s, fc.d.prev, img, w, h, stride))) return rc;
    FL_TRY(c, hipMemcpyAsync(fc.d.mexp, mask, kSubpixMaskBytes, hipMemcpyHostToDevice, fc.s));
    FL_TRY(c, hipMemcpyAsync(fc.d.pts, xy, (size_t)n * 8, hipMemcpyHostToDevice, fc.s));
    FL_TRY(c, hipMemcpyAsync(fc.d.npts, &n, 4, hipMemcpyHostToDevice, fc.s));
    if (launch_subpix(&fc.d, fc.d.prev, w, h, w, max_iter, eps, fc.s))
        return coeb_internal_error(c, COEB_EDEVICE, "coeb_corner_subpix: launch failed");
    FL_TRY(c, hipMemcpyAsync(xy, fc.d.pts, (size_t)n * 8, hipMemcpyDeviceToHost, fc.s));
    FL_TRY(c, hipStreamSynchronize(fc.s));
    return COEB_OK;
}

extern "C" int coeb_optical_flow_pyr_lk(coeb_ctx* c, const uint8_t* prev, const uint8_t* next, int w, int h,
                                        size_t stride, const float* prev_xy, int n, int win, int max_level,
                                        int max_count, double eps, float* next_xy, uint8_t* status)
{
    if (!c || !prev || !next || n < 0 || n > kMaxPts || (n > 0 && (!prev_xy || !next_xy || !status)) ||
        stride < (size_t)w || max_level < 0 || max_count < 1)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_optical_flow_pyr_lk: invalid arguments");
    if (win < 3 || win * win > 512)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_optical_flow_pyr_lk: window must be 3..22");
    if (n == 0) return COEB_OK;
    FlowCall fc;
    int rc = flow_begin(c, w, h, &fc, "coeb_optical_flow_pyr_lk: invalid arguments");
    if (rc) return rc;
    if (lk_levels(w, h, win, max_level) > kLkMaxLevels)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_optical_flow_pyr_lk: more than 8 pyramid levels");
    if ((rc = upload_gray(c, fc.s, fc.d.prev, prev, w, h, stride)) || (rc = upload_gray(c, fc.s, fc.d.cur, next, w, h, stride)))
        return rc;
    FL_TRY(c, hipMemcpyAsync(fc.d.pts, prev_xy, (size_t)n * 8, hipMemcpyHostToDevice, fc.s));
    FL_TRY(c, hipMemcpyAsync(fc.d.npts, &n, 4, hipMemcpyHostToDevice, fc.s));
    if (launch_lk(&fc.d, fc.d.prev, fc.d.cur, w, h, w, win, max_level, max_count, eps, fc.s))
        return coeb_internal_error(c, COEB_EDEVICE, "coeb_optical_flow_pyr_lk: launch failed");
    FL_TRY(c, hipMemcpyAsync(next_xy, fc.d.nxt, (size_t)n * 8, hipMemcpyDeviceToHost, fc.s));
    FL_TRY(c, hipMemcpyAsync(status, fc.d.status, (size_t)n, hipMemcpyDeviceToHost, fc.s));
    FL_TRY(c, hipStreamSynchronize(fc.s));
    return COEB_OK;
}

extern "C" int coeb_moving_tail(coeb_ctx* c, const uint8_t* prev, const uint8_t* cur, int w, int h, size_t stride,
                                const float* prev_xy, const float* next_xy, uint8_t* state, int n, float* tm_xy,
                                int tm_cap, int* n_tm, double F_out[9], int* nf_out)
{
    if (!c || !prev || !cur || n < 0 || n > kMaxPts || (n > 0 && (!prev_xy || !next_xy || !state)) || !n_tm ||
        (tm_cap > 0 && !tm_xy) || stride < (size_t)w)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_moving_tail: invalid arguments");
    FlowCall fc;
    int rc = flow_begin(c, w, h, &fc, "coeb_moving_tail: invalid arguments");
    if (rc) return rc;
    if ((rc = upload_gray(c, fc.s, fc.d.prev, prev, w, h, stride)) || (rc = upload_gray(c, fc.s, fc.d.cur, cur, w, h, stride)))
        return rc;
    if (n > 0) {
        FL_TRY(c, hipMemcpyAsync(fc.d.pts, prev_xy, (size_t)n * 8, hipMemcpyHostToDevice, fc.s));
        FL_TRY(c, hipMemcpyAsync(fc.d.nxt, next_xy, (size_t)n * 8, hipMemcpyHostToDevice, fc.s));
        FL_TRY(c, hipMemcpyAsync(fc.d.status, state, (size_t)n, hipMemcpyHostToDevice, fc.s));
    }
    FL_TRY(c, hipMemcpyAsync(fc.d.npts, &n, 4, hipMemcpyHostToDevice, fc.s));
    if (launch_fm(&fc.d, fc.d.prev, fc.d.cur, w, h, w, 5, 2120.0, fc.s, kMaxPts))
        return coeb_internal_error(c, COEB_EDEVICE, "coeb_moving_tail: launch failed");
    int nt = 0, nf = 0;
    double F[9];
    FL_TRY(c, hipMemcpyAsync(&nt, fc.d.ntm, 4, hipMemcpyDeviceToHost, fc.s));
    FL_TRY(c, hipMemcpyAsync(&nf, fc.d.nf, 4, hipMemcpyDeviceToHost, fc.s));
    FL_TRY(c, hipMemcpyAsync(F, fc.d.F, sizeof(F), hipMemcpyDeviceToHost, fc.s));
    if (n > 0) FL_TRY(c, hipMemcpyAsync(state, fc.d.state, (size_t)n, hipMemcpyDeviceToHost, fc.s));
    FL_TRY(c, hipStreamSynchronize(fc.s));
    if (nt > 0 && tm_cap > 0) {
        FL_TRY(c, hipMemcpyAsync(tm_xy, fc.d.tm, (size_t)(nt < tm_cap ? nt : tm_cap) * 8, hipMemcpyDeviceToHost, fc.s));
        FL_TRY(c, hipStreamSynchronize(fc.s));
    }
    *n_tm = nt;
    if (nf_out) *nf_out = nf;
    if (F_out && nt >= 0) memcpy(F_out, F, sizeof(F));
    return COEB_OK;
}

extern "C" int coeb_moving_object_points(coeb_ctx* c, const uint8_t* prev, const uint8_t* cur, int w, int h,
                                         size_t stride, float* tm_xy, int tm_cap, int* n_tm, coeb_flow_debug* dbg)
{
    if (!c || !prev || !cur || !n_tm || (tm_cap > 0 && !tm_xy) || stride < (size_t)w)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_moving_object_points: invalid arguments");
    FlowCall fc;
    int rc = flow_begin(c, w, h, &fc, "coeb_moving_object_points: invalid arguments");
    if (rc) return rc;
    if (lk_levels(w, h, 22, 5) > kLkMaxLevels)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_moving_object_points: image too large");
    float mask[21];
    subpix_mask(10, mask);
    if ((rc = upload_gray(c, fc.s, fc.d.prev, prev, w, h, stride)) || (rc = upload_gray(c, fc.s, fc.d.cur, cur, w, h, stride)))
        return rc;
    FL_TRY(c, hipMemcpyAsync(fc.d.mexp, mask, kSubpixMaskBytes, hipMemcpyHostToDevice, fc.s));
    return coeb_moving_object_points_device(c, fc.d.prev, fc.d.cur, w, h, w, tm_xy, tm_cap, n_tm, dbg);
}

// Frame::ProcessMovingObject for every consecutive pair of a device-resident batch (the Frame
// constructor's T_M, Frame.cc:164-166): pair f-1 = frames (f-1, f) of d_gray (packed, w x h),
// T_M of frame f into tm_out + f * tm_cap * 2 floats, |T_M| (or -1: F empty) into ntm_out[f];
// ntm_out[0] = 0 (no previous frame).  Enqueued on the context stream, no synchronisation.
// A/B tool hook: {iterations, corners} counted by the cornerSubPix variants under
// COEB_SUBPIX_COUNT since the last read (then reset)
extern "C" int coeb_internal_subpix_count(int* out)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_subpix_count_dev), 16) != hipSuccess) return COEB_EDEVICE;
    const int z[4] = {0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_subpix_count_dev), z, 16) == hipSuccess ? COEB_OK : COEB_EDEVICE;
}

// geometry of each context's last moving-object batch, for coeb_internal_flow_counts
static std::mutex g_pmo_mu;
static std::map<const coeb_ctx*, std::array<int, 3>> g_pmo_last;

extern "C" void coeb_internal_flow_forget(const coeb_ctx* c)   // coeb_destroy
{
    std::lock_guard<std::mutex> lk(g_pmo_mu);
    g_pmo_last.erase(c);
}

// Per pair of the context's last moving-object batch: {Harris candidate keys, corners} (bench.py's
// algorithmic bytes of k_gf_select / k_subpix / k_lk / k_fm).  Synchronises the context stream.
extern "C" int coeb_internal_flow_counts(coeb_ctx* c, int* out, int cap, int* npairs)
{
    std::array<int, 3> g;
    {
        std::lock_guard<std::mutex> lk(g_pmo_mu);
        auto it = g_pmo_last.find(c);
        if (it == g_pmo_last.end()) return COEB_EINVAL;
        g = it->second;
    }
    FlowCall fc;
    int dev;
    if (coeb_internal_stream(c, &fc.s, &dev)) return COEB_EINVAL;
    (void)hipSetDevice(dev);
    int rc = flow_alloc(c, g[0], g[1], &fc.d, g[2]);
    if (rc) return rc;
    *npairs = g[2];
    FL_TRY(c, hipStreamSynchronize(fc.s));
    for (int z = 0; z < g[2] && 2 * z + 1 < cap; z++) {
        FL_TRY(c, hipMemcpy(out + 2 * z, (const uint8_t*)fc.d.nkeys + (size_t)z * fc.d.pz, 4, hipMemcpyDeviceToHost));
        FL_TRY(c, hipMemcpy(out + 2 * z + 1, (const uint8_t*)fc.d.npts + (size_t)z * fc.d.pz, 4, hipMemcpyDeviceToHost));
    }
    return COEB_OK;
}

extern "C" int coeb_internal_pmo_batch(coeb_ctx* c, const uint8_t* d_gray, int F, int w, int h, float* tm_out,
                                       int* ntm_out, int tm_cap)
{
    if (F < 1 || !d_gray || !tm_out || !ntm_out || tm_cap < 1 || tm_cap > kMaxPts)
        return coeb_internal_error(c, COEB_EINVAL, "moving-object batch: invalid arguments");
    FlowCall fc;
    int dev;
    if (coeb_internal_stream(c, &fc.s, &dev)) return COEB_EINVAL;
    (void)hipSetDevice(dev);
    FL_TRY(c, hipMemsetAsync(ntm_out, 0, 4, fc.s));
    if (F < 2) return COEB_OK;
    if (w < 32 || h < 32 || lk_levels(w, h, 22, 5) > kLkMaxLevels)
        return coeb_internal_error(c, COEB_EINVAL, "moving-object batch: frame size");
    int rc = flow_alloc(c, w, h, &fc.d, F - 1);
    if (rc) return rc;
    {
        std::lock_guard<std::mutex> lk(g_pmo_mu);
        g_pmo_last[c] = {w, h, F - 1};
    }
    float mask[21];
    subpix_mask(10, mask);
    FL_TRY(c, hipMemcpyAsync(fc.d.mexp, mask, kSubpixMaskBytes, hipMemcpyHostToDevice, fc.s));
    const int64_t iz = (int64_t)w * h;
    // COEB_FLOW_SIDE=1: the LK pyramids go to the context's side stream (idle until extraction)
    // beside the corner detection, and the context stream joins them before k_lk (measured slower)
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    const bool split = coeb_internal_flow_side(c, &side, &fork, &join) == 0;
    LkPyr pyr;
    if (split) {
        FL_TRY(c, hipEventRecord(fork, fc.s));
        FL_TRY(c, hipStreamWaitEvent(side, fork, 0));
        if (launch_lk_pyramids(&fc.d, d_gray, d_gray + iz, w, h, w, 22, 5, side, iz, pyr))
            return coeb_internal_error(c, COEB_EDEVICE, "moving-object batch: launch failed");
        FL_TRY(c, hipEventRecord(join, side));
    }
    if (launch_gf(&fc.d, d_gray, w, h, w, 1000, 0.01, 8.0, 0.04, fc.s, iz) ||
        launch_subpix(&fc.d, d_gray, w, h, w, 20, 0.03, fc.s, iz))
        return coeb_internal_error(c, COEB_EDEVICE, "moving-object batch: launch failed");
    if (split) FL_TRY(c, hipStreamWaitEvent(fc.s, join, 0));
    if ((split ? launch_lk_track(&fc.d, pyr, 22, 20, 0.01, fc.s, iz)
               : launch_lk(&fc.d, d_gray, d_gray + iz, w, h, w, 22, 5, 20, 0.01, fc.s, iz)) ||
        launch_fm(&fc.d, d_gray, d_gray + iz, w, h, w, 5, 2120.0, fc.s, tm_cap, iz, tm_out + (size_t)tm_cap * 2,
                  ntm_out + 1))
        return coeb_internal_error(c, COEB_EDEVICE, "moving-object batch: launch failed");
    return COEB_OK;
}

// device-resident frames (pitch `stride`); the subpix weight table is uploaded on first use
extern "C" int coeb_moving_object_points_device(coeb_ctx* c, const uint8_t* d_prev, const uint8_t* d_cur, int w, int h,
                                                size_t stride, float* tm_xy, int tm_cap, int* n_tm,
                                                coeb_flow_debug* dbg)
{
    if (!c || !d_prev || !d_cur || !n_tm || (tm_cap > 0 && !tm_xy) || stride < (size_t)w)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_moving_object_points_device: invalid arguments");
    FlowCall fc;
    int rc = flow_begin(c, w, h, &fc, "coeb_moving_object_points_device: invalid arguments");
    if (rc) return rc;
    if (lk_levels(w, h, 22, 5) > kLkMaxLevels)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_moving_object_points_device: image too large");
    float mask[21];
    subpix_mask(10, mask);
    FL_TRY(c, hipMemcpyAsync(fc.d.mexp, mask, kSubpixMaskBytes, hipMemcpyHostToDevice, fc.s));
    const int sp = (int)stride;
    if (launch_gf(&fc.d, d_prev, w, h, sp, 1000, 0.01, 8.0, 0.04, fc.s))
        return coeb_internal_error(c, COEB_EDEVICE, "coeb_moving_object_points: goodFeaturesToTrack launch failed");
    if (dbg && dbg->corners_raw) {
        FL_TRY(c, hipMemcpyAsync(dbg->corners_raw, fc.d.pts, (size_t)1000 * 8, hipMemcpyDeviceToHost, fc.s));
    }
    if (launch_subpix(&fc.d, d_prev, w, h, sp, 20, 0.03, fc.s) ||
        launch_lk(&fc.d, d_prev, d_cur, w, h, sp, 22, 5, 20, 0.01, fc.s) ||
        launch_fm(&fc.d, d_prev, d_cur, w, h, sp, 5, 2120.0, fc.s, kMaxPts))
        return coeb_internal_error(c, COEB_EDEVICE, "coeb_moving_object_points: launch failed");
    int nt = 0, nc = 0;
    FL_TRY(c, hipMemcpyAsync(&nt, fc.d.ntm, 4, hipMemcpyDeviceToHost, fc.s));
    FL_TRY(c, hipMemcpyAsync(&nc, fc.d.npts, 4, hipMemcpyDeviceToHost, fc.s));
    if (dbg) {
        if (dbg->corners) FL_TRY(c, hipMemcpyAsync(dbg->corners, fc.d.pts, (size_t)1000 * 8, hipMemcpyDeviceToHost, fc.s));
        if (dbg->next_pts) FL_TRY(c, hipMemcpyAsync(dbg->next_pts, fc.d.nxt, (size_t)1000 * 8, hipMemcpyDeviceToHost, fc.s));
        if (dbg->status) FL_TRY(c, hipMemcpyAsync(dbg->status, fc.d.status, 1000, hipMemcpyDeviceToHost, fc.s));
        if (dbg->state) FL_TRY(c, hipMemcpyAsync(dbg->state, fc.d.state, 1000, hipMemcpyDeviceToHost, fc.s));
        if (dbg->F) FL_TRY(c, hipMemcpyAsync(dbg->F, fc.d.F, 72, hipMemcpyDeviceToHost, fc.s));
        if (dbg->nf) FL_TRY(c, hipMemcpyAsync(dbg->nf, fc.d.nf, 4, hipMemcpyDeviceToHost, fc.s));
    }
    FL_TRY(c, hipStreamSynchronize(fc.s));
    if (nc < 0) return coeb_internal_error(c, COEB_ERANGE, "coeb_moving_object_points: more local maxima than the exact selection covers");
    if (dbg && dbg->ncorners) *dbg->ncorners = nc;
    if (nt > 0 && tm_cap > 0) {
        FL_TRY(c, hipMemcpyAsync(tm_xy, fc.d.tm, (size_t)(nt < tm_cap ? nt : tm_cap) * 8, hipMemcpyDeviceToHost, fc.s));
        FL_TRY(c, hipStreamSynchronize(fc.s));
    }
    *n_tm = nt;
    return COEB_OK;
}
