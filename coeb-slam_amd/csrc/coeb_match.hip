// coeb_match.hip -- CDNA4 kernels for the tracking-time projection searches:
//   ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)  src/ORBmatcher.cc:1329-1471  (k_match)
//   ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th)     src/ORBmatcher.cc:44-129     (k_match_local)
//   Frame::AssignFeaturesToGrid / GetFeaturesInArea                   src/Frame.cc:396-411, 503-568
//   Frame::ComputeStereoFromRGBD                                      src/Frame.cc:820-842         (k_prep)
//   ORBmatcher::DescriptorDistance                                    src/ORBmatcher.cc:1648-1664
//
// One 1024-thread workgroup per frame (pair).  Phase 0 (stage_grid) stages the current frame
// in LDS and builds the 64 x 48 keypoint grid as a CSR by a stable counting sort, so a cell
// column ix over rows [iy0, iy1] is ONE contiguous range in the reference's enumeration order
// (ix outer, iy inner, in-cell insertion order).  Phase 1: kQL lanes per query walk its
// window (level, window, stereo checks, 256-bit Hamming via popcount) and write its candidate
// list in that order.  Phase 2 resolves the sequential claim dependency (:1404-1406 / :86-88)
// as a Jacobi fixpoint, with the literal loop as fallback.  Phase 3 assigns (last writer
// wins) and, for k_match, applies the rotation-histogram top-3 filter.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "coeb_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr int HISTO_LENGTH = 30;
constexpr int TH_HIGH = 100;

struct Kp { float x, y, size, angle, response; int octave, class_id; };

__device__ __forceinline__ int hamming32(const uint32_t* a, const uint32_t* b)
{
    int d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d += __popc(a[i] ^ b[i]);
    return d;
}

// ================================ k_prep ================================
// Frame::ComputeStereoFromRGBD + the LastFrame snapshot used by the next frame's matcher:
// MapPoint world position = Frame::UnprojectStereo (src/Frame.cc:844-858) with the frame as
// world reference (Twc = I), Observations() = nobs_value.
__global__ __launch_bounds__(kThreads) void k_prep(PrepBufs b)
{
    const int f = blockIdx.y;
    const int i = blockIdx.x * kThreads + threadIdx.x;
    const int n = b.n[f];
    if (i >= n) return;
    const Kp kp = reinterpret_cast<const Kp*>(b.kps)[(int64_t)f * b.stride + i];
    const int64_t o = (int64_t)f * b.stride + i;
    const float d = b.depth[(int64_t)f * b.W * b.H + (int64_t)(int)kp.y * b.W + (int)kp.x];
    float ur = -1.f, dep = -1.f;
    if (d > 0) { dep = d; ur = kp.x - b.bf / d; }
    b.ur[o] = ur;
    b.dep[o] = dep;
    if (b.has) {
        b.has[o] = d > 0 ? 1 : 0;
        b.outl[o] = 0;
        b.nobs[o] = b.nobs_value;
        const float invfx = 1.0f / b.fx, invfy = 1.0f / b.fy;
        const float z = dep;
        const float x = (kp.x - b.cx) * z * invfx;
        const float y = (kp.y - b.cy) * z * invfy;
        b.xw[3 * o + 0] = x;
        b.xw[3 * o + 1] = y;
        b.xw[3 * o + 2] = z;
    }
}

// ================================ k_match ================================
// One workgroup per frame pair (512 threads when the pair's LDS fits half a CU, else 1024).
//   phase 0  stage CurrentFrame (x, y, uR, octave, descriptor) in LDS; build the 64 x 48
//            grid as a CSR by a stable counting sort of (cell << 12 | index): a cell column ix
//            over rows [iy0, iy1] is one contiguous range, so range order == the reference's
//            (ix outer, iy inner, insertion order) enumeration.
//   phase 1  one thread per LastFrame point: projection, window, level / window / stereo
//            filters and Hamming distance; the candidates with dist <= TH_HIGH are kept in
//            enumeration order (only they can ever be chosen).
//   phase 2  claims.  Sequentially, point q takes the first strict minimum (dist, order) among
//            its candidates not claimed by an earlier point p < q whose MapPoint has
//            Observations() > 0 (ORBmatcher.cc:1401-1429).  With res_q = F_q(res_{<q}) this is
//            a triangular system; Jacobi iteration (all q in parallel, owner[c] = min p with
//            res_p = c, nobs_p > 0) reaches its unique fixpoint -- the sequential result --
//            and stops when an iteration changes nothing.
//   phase 3  CurrentFrame.mvpMapPoints[c] = last claimer of c; rotation histogram
//            (round(rot/30)), ComputeThreeMaxima, drop the rest (ORBmatcher.cc:1432-1468).
//   retry    nmatches < retry_below -> again with 2*th (Tracking.cc:954-958).
// A pair whose candidate list overflows kCQ, or that does not converge in kMaxIter
// iterations, runs the literal sequential loop instead (exact, slower).
constexpr int kMThreads = 1024;
constexpr int kCQ = 64;

constexpr int kMaxIter = 64;
constexpr int kIdxBits = 12;
// Lanes per LastFrame query in the candidate phase: a grid column range holds a few
// candidates (10-px cells), so few lanes per query waste least (round 1: 16 -> 8 lanes, 0.171 ->
// 0.147 ms/step; round 3: 8 -> 4 lanes, lists 174k -> 160k cycles per pair, k_match 0.314 ->
// 0.309 ms per 1025-frame launch)
#ifndef COEB_MATCH_QL
#define COEB_MATCH_QL 4
#endif
constexpr int kQL = COEB_MATCH_QL;

// Up to kQL window columns, one per lane of a kQL-lane group (lane j: CSR range [lo_j, lo_j +
// len_j)), as one concatenated range in column-major order: its length, and the CSR index of
// concatenated position f.  A group scan (DPP row shifts, masked to the group) gives each
// column's end; ds_swizzle broadcasts (groups of kQL within each 32-lane half) hand every lane
// all of them.
struct GroupCols {
    int total;
    uint32_t pk[kQL];                  // column j: end in the concatenation << 16 | (lo_j - start_j + 0x8000)
    __device__ __forceinline__ int index(int f) const
    {
        uint32_t sel = pk[0];
#pragma unroll
        for (int j = 1; j < kQL; j++)
            if (f >= (int)(pk[j - 1] >> 16)) sel = pk[j];
        return f + (int)(sel & 0xFFFFu) - 0x8000;
    }
};

template <int K>
__device__ __forceinline__ void group_bcast(uint32_t v, GroupCols& g)
{
    constexpr int pat = (0x1F & ~(kQL - 1)) | (K << 5);   // lane = (lane & and_mask) | K
    g.pk[K] = (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, pat);
    if constexpr (K + 1 < kQL) group_bcast<K + 1>(v, g);
}

__device__ __forceinline__ GroupCols group_cols(int lo, int len, int gl)
{
    static_assert(kQL <= 16 && (kQL & (kQL - 1)) == 0, "group scan within one 16-lane DPP row");
    int inc = len;
    int t = __builtin_amdgcn_mov_dpp(inc, 0x111, 0xf, 0xf, true);          // row_shr:1
    if (gl >= 1) inc += t;
    if constexpr (kQL > 2) {
        t = __builtin_amdgcn_mov_dpp(inc, 0x112, 0xf, 0xf, true);          // row_shr:2
        if (gl >= 2) inc += t;
    }
    if constexpr (kQL > 4) {
        t = __builtin_amdgcn_mov_dpp(inc, 0x114, 0xf, 0xf, true);          // row_shr:4
        if (gl >= 4) inc += t;
    }
    if constexpr (kQL > 8) {
        t = __builtin_amdgcn_mov_dpp(inc, 0x118, 0xf, 0xf, true);          // row_shr:8
        if (gl >= 8) inc += t;
    }
    GroupCols g;   // candidate counts < 2^16 and |lo - start| < 2^15 (kIdxBits = 12: <= 4096 keypoints)
    group_bcast<0>(((uint32_t)inc << 16) | (uint32_t)(lo - (inc - len) + 0x8000), g);
    g.total = (int)(g.pk[kQL - 1] >> 16);
    return g;
}
#ifndef COEB_MATCH_REGLIST
#define COEB_MATCH_REGLIST 16
#endif
constexpr int kRegList = COEB_MATCH_REGLIST;        // list head kept in registers by the claim fixpoint
#ifndef COEB_MATCH_QPT1024
#define COEB_MATCH_QPT1024 2
#endif
#ifndef COEB_MATCH_RL1024
#define COEB_MATCH_RL1024 12
#endif
#ifndef COEB_LOCAL_QPT
#define COEB_LOCAL_QPT 2                           // k_match_local: points per thread with register list heads
#endif
#ifndef COEB_LOCAL_RL
#define COEB_LOCAL_RL 8                            // ... and the entries held per point
#endif

struct QueryWin {
    bool ok, chk;
    bool st = true;            // stereo (uR) check applies
    float u, v, radius, ur_q;
    int minL, maxL, x0, x1, y0, y1;
};

// Grid cell range of GetFeaturesInArea(u, v, radius, minL, maxL) (Frame.cc:507-522); false when
// the window misses the grid.
__device__ __forceinline__ bool window_cells(const MatchCam& cam, QueryWin& w)
{
    w.x0 = max(0, (int)floorf(((w.u - cam.min_x) - w.radius) * cam.grid_inv_w));
    if (w.x0 >= COEB_GRID_COLS) return false;
    w.x1 = min(COEB_GRID_COLS - 1, (int)ceilf(((w.u - cam.min_x) + w.radius) * cam.grid_inv_w));
    if (w.x1 < 0) return false;
    w.y0 = max(0, (int)floorf(((w.v - cam.min_y) - w.radius) * cam.grid_inv_h));
    if (w.y0 >= COEB_GRID_ROWS) return false;
    w.y1 = min(COEB_GRID_ROWS - 1, (int)ceilf(((w.v - cam.min_y) + w.radius) * cam.grid_inv_h));
    if (w.y1 < 0) return false;
    w.chk = (w.minL > 0) || (w.maxL >= 0);
    return true;
}

__device__ __forceinline__ QueryWin query_window(const MatchCam& cam, const float* T, const float* scale, const float* X,
                                                 int octave, float th, bool fwd, bool bwd)
{
    QueryWin w;
    w.ok = false;
    float p3[3];
    for (int k = 0; k < 3; k++) {                  // x3Dc = Rcw*x3Dw + tcw (cv::Mat small gemm)
        float t = T[k * 4 + 0] * X[0] + T[k * 4 + 1] * X[1];
        t = t + T[k * 4 + 2] * X[2];
        p3[k] = (float)((double)t + (double)T[k * 4 + 3]);
    }
    const float invzc = (float)(1.0 / (double)p3[2]);
    if (invzc < 0) return w;
    w.u = __builtin_fmaf(cam.fx * p3[0], invzc, cam.cx);   // fused in the reference binary
    w.v = __builtin_fmaf(cam.fy * p3[1], invzc, cam.cy);
    if (w.u < cam.min_x || w.u > cam.max_x) return w;
    if (w.v < cam.min_y || w.v > cam.max_y) return w;
    w.radius = th * scale[octave];
    if (fwd) { w.minL = octave; w.maxL = -1; }
    else if (bwd) { w.minL = 0; w.maxL = octave; }
    else { w.minL = octave - 1; w.maxL = octave + 1; }
    w.ur_q = __builtin_fmaf(-cam.bf, invzc, w.u);     // u - mbf*invzc (fused)
    w.ok = window_cells(cam, w);
    return w;
}

// The current frame's keypoints as candidates.  In LDS mode they are staged in CSR (grid)
// order, so candidate e of a cell range is read at position e with no indirection through
// L.sort (one LDS round trip per candidate step instead of three); the global fallback reads
// keypoint i.
template <bool kLds>
struct CurView {
    const float4* kp;         // LDS, CSR order: (x, y, uR, octave bits)
    const uint32_t* desc;     // LDS, CSR order: 8 words per keypoint
    const Kp* gkp;            // global fallbacks, keypoint order
    const float* gur;
    const uint8_t* gdesc;
    __device__ __forceinline__ void get(int e, int i, float& x, float& y, float& ur, int& oct) const
    {
        if (kLds) {
            const float4 k = kp[e];
            x = k.x; y = k.y; ur = k.z; oct = __float_as_int(k.w);
        } else {
            x = gkp[i].x; y = gkp[i].y; oct = gkp[i].octave; ur = gur ? gur[i] : -1.f;
        }
    }
    __device__ __forceinline__ int dist(int e, int i, const uint32_t* q) const
    {
        const uint32_t* d = kLds ? desc + 8 * e : reinterpret_cast<const uint32_t*>(gdesc + 32 * i);
        return hamming32(q, d);
    }
};

// Candidates of one query passing the level / window / stereo filters, in enumeration order.
template <bool kLds, class Fn>
__device__ __forceinline__ void for_candidates(const QueryWin& w, const int* s_cell, const uint32_t* s_sort,
                                               const CurView<kLds>& cv, Fn&& fn)
{
    for (int ix = w.x0; ix <= w.x1; ix++) {
        const int c0 = s_cell[ix * COEB_GRID_ROWS + w.y0];
        const int c1 = s_cell[ix * COEB_GRID_ROWS + w.y1 + 1];
        for (int q = c0; q < c1; q++) {
            const int i2 = (int)(s_sort[q] & ((1u << kIdxBits) - 1));
            float x, y, ur;
            int oct;
            cv.get(q, i2, x, y, ur, oct);
            if (w.chk) {
                if (oct < w.minL) continue;
                if (w.maxL >= 0 && oct > w.maxL) continue;
            }
            const float distx = x - w.u, disty = y - w.v;
            if (!(fabsf(distx) < w.radius && fabsf(disty) < w.radius)) continue;
            if (w.st && ur > 0) {
                const float er = fabsf(w.ur_q - ur);
                if (er > w.radius) continue;
            }
            if (!fn(q, i2)) return;
        }
    }
}

__device__ __forceinline__ int rot_bin(float a_last, float a_cur)
{
    float rot = a_last - a_cur;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / HISTO_LENGTH));
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

// ORBmatcher::ComputeThreeMaxima (ORBmatcher.cc:1602-1638) as selects.  max1 >= max2 >= max3
// holds throughout, so s > max1 implies s > max2 implies s > max3, and each branch of the
// reference's if / else-if chain is one combination of the three tests.  (Written as that chain,
// the compiler addressed the index variables through scratch memory -- a dependent scratch
// round trip per bin, ~20 k cycles of k_match's assignment phase per pair.)
__device__ __forceinline__ void three_maxima(const int* hist, int& ind1, int& ind2, int& ind3)
{
    int max1 = 0, max2 = 0, max3 = 0;
    int i1 = -1, i2 = -1, i3 = -1;
#pragma unroll 6
    for (int i = 0; i < HISTO_LENGTH; i++) {
        const int s = hist[i];
        const bool g1 = s > max1, g2 = s > max2, g3 = s > max3;
        max3 = g2 ? max2 : g3 ? s : max3;
        i3 = g2 ? i2 : g3 ? i : i3;
        max2 = g1 ? max1 : g2 ? s : max2;
        i2 = g1 ? i1 : g2 ? i : i2;
        max1 = g1 ? s : max1;
        i1 = g1 ? i : i1;
    }
    ind1 = i1; ind2 = i2; ind3 = i3;
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
}

constexpr int kHeldOct = 0x100;          // stage_grid's held-keypoint flag (octaves are < 16)

struct MatchLds {
    int* cell; uint32_t* sort; int* owner; int* res; int* qn; float4* kp; uint32_t* desc;
};

__host__ __device__ inline size_t match_lds_bytes(int nmax, int qmax, bool lds_cur, size_t* offs)
{
    const size_t n4 = (size_t)((nmax + 3) & ~3), q4 = (size_t)((qmax + 3) & ~3);
    size_t o = 0;
    size_t off[7];
    off[0] = o; o += ((COEB_GRID_CELLS + 1) * 4 + 15) & ~(size_t)15;
    off[1] = o; o += n4 * 4;
    off[2] = o; o += n4 * 4;
    off[3] = o; o += q4 * 4;
    off[4] = o; o += q4 * 4;
    off[5] = o; if (lds_cur) o += n4 * 16;
    off[6] = o; if (lds_cur) o += n4 * 32;
    if (offs) for (int i = 0; i < 7; i++) offs[i] = off[i];
    return o;
}

// Phase 0 of both matchers: stage the CurrentFrame (x, y, uR, octave, descriptor) in LDS and
// build its 64 x 48 grid (Frame::AssignFeaturesToGrid, Frame.cc:396-411) as a CSR by a stable
// counting sort: L.cell[c] = start of cell c in L.sort, L.sort = (cell << kIdxBits | index) in
// cell order, index order inside a cell.  L.owner is scratch here.
template <bool kLds, int NT = kMThreads>
__device__ __forceinline__ void stage_grid(const MatchCam& cam, const Kp* cur, const float* cur_ur, const uint8_t* cdesc,
                                           int n, const MatchLds& L, const int* cur_obs = nullptr)
{
    const int tid = threadIdx.x;
    for (int c = tid; c <= COEB_GRID_CELLS; c += NT) L.cell[c] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += NT) {
        const Kp k = cur[i];
        const int px = (int)roundf((k.x - cam.min_x) * cam.grid_inv_w);   // PosInGrid (Frame.cc:560)
        const int py = (int)roundf((k.y - cam.min_y) * cam.grid_inv_h);
        int cell = -1;
        if (px >= 0 && px < COEB_GRID_COLS && py >= 0 && py < COEB_GRID_ROWS) {
            cell = px * COEB_GRID_ROWS + py;
            atomicAdd(&L.cell[cell + 1], 1);
        }
        L.owner[i] = cell;                 // scratch until phase 2
    }
    __syncthreads();
    {                                      // prefix: L.cell[c + 1] = end of cell c (block scan)
        constexpr int CPT = COEB_GRID_CELLS / NT;
        static_assert(COEB_GRID_CELLS == CPT * NT, "whole cells per thread");
        __shared__ int s_wsum[NT / 64];
        const int lane = tid & 63, wv = tid >> 6;
        const int c0 = 1 + CPT * tid;
        int a[CPT];
        int v = 0;
#pragma unroll
        for (int k = 0; k < CPT; k++) { a[k] = L.cell[c0 + k]; v += a[k]; }
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(v, o, 64);
            if (lane >= o) v += y;
        }
        if (lane == 63) s_wsum[wv] = v;
        __syncthreads();
        int off = 0;
        for (int w = 0; w < wv; w++) off += s_wsum[w];
        int end = off + v;                                  // inclusive prefix through cell c0 + CPT - 1
#pragma unroll
        for (int k = CPT - 1; k >= 0; k--) { L.cell[c0 + k] = end; end -= a[k]; }
        if (tid == 0) L.cell[0] = 0;
    }
    __syncthreads();
    // scatter with a per-cell cursor (L.cell[c] advances to the end of cell c = start of c+1) ...
    for (int i = tid; i < n; i += NT) {
        const int cell = L.owner[i];
        if (cell >= 0) {
            const int pos = atomicAdd(&L.cell[cell], 1);
            L.sort[pos] = ((uint32_t)cell << kIdxBits) | (uint32_t)i;
        }
    }
    __syncthreads();
    // ... so shift the cursors back by one cell to get the starts again
    {
        int v[(COEB_GRID_CELLS + NT) / NT];
#pragma unroll
        for (int k = 0; k < (COEB_GRID_CELLS + NT) / NT; k++) {
            const int c = tid + k * NT;
            v[k] = (c >= 1 && c <= COEB_GRID_CELLS) ? L.cell[c - 1] : 0;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < (COEB_GRID_CELLS + NT) / NT; k++) {
            const int c = tid + k * NT;
            if (c >= 1 && c <= COEB_GRID_CELLS) L.cell[c] = v[k];
        }
        if (tid == 0) L.cell[0] = 0;
    }
    __syncthreads();
    // insertion order inside a cell = keypoint index order (Frame.cc:403-410): sort each
    // (short) cell range by index
    for (int c = tid; c < COEB_GRID_CELLS; c += NT) {
        const int a = L.cell[c], e = L.cell[c + 1];
        for (int x = a + 1; x < e; x++) {
            const uint32_t key = L.sort[x];
            int y = x - 1;
            while (y >= a && L.sort[y] > key) { L.sort[y + 1] = L.sort[y]; y--; }
            L.sort[y + 1] = key;
        }
    }
    __syncthreads();
    if (kLds) {                            // candidates in CSR order (CurView)
        const int ng = L.cell[COEB_GRID_CELLS];
        for (int e = tid; e < ng; e += NT) {
            const int i = (int)(L.sort[e] & ((1u << kIdxBits) - 1));
            const Kp k = cur[i];
            // cur_obs (k_match_local): a keypoint whose MapPoint has observations carries kHeldOct in
            // its staged octave, which puts it above every level window (it is never a candidate)
            const int oct = cur_obs && cur_obs[i] > 0 ? k.octave | kHeldOct : k.octave;
            L.kp[e] = make_float4(k.x, k.y, cur_ur ? cur_ur[i] : -1.f, __int_as_float(oct));
            const uint4* d = reinterpret_cast<const uint4*>(cdesc + 32 * i);
            const uint4 d0 = d[0], d1 = d[1];
            uint4* o = reinterpret_cast<uint4*>(L.desc + 8 * e);
            o[0] = d0;
            o[1] = d1;
        }
        __syncthreads();
    }
}

// Phase 2 of the first-minimum matchers (k_match, k_match_kf).  lists + q * stride: query q's
// candidates (dist << kIdxBits | index) in enumeration order; L.qn[q] = count (-1: none), with
// 0x10000 set when q's assignment blocks later queries.  res_q = first minimum of q's list over
// keypoints not claimed by a blocking p < q, solved as a Jacobi fixpoint (iteration k fixes
// queries 0..k-1, so it reaches the sequential answer).  L.res = the result.  Returns true when
// kMaxIter rounds did not converge (the caller then runs its literal loop).  Block-uniform.
__device__ __forceinline__ void first_min_step(const MatchLds& L, uint32_t v, int e, int q, uint32_t& bk, int& best)
{
    const int i2 = (int)(v & ((1u << kIdxBits) - 1));
    if (L.owner[i2] < q) return;                          // claimed by an earlier point
    const uint32_t key = ((v >> kIdxBits) << 16) | (uint32_t)e;
    if (key < bk) { bk = key; best = i2; }
}

template <int NT = kMThreads>
__device__ bool claims_first_min(const MatchLds& L, const uint32_t* lists, int stride, int n, int nq, int* s_flag)
{
    const int tid = threadIdx.x;
    // the thread's first QPT queries (tid, tid + NT, ...) keep the heads of their lists in
    // registers across iterations (global list reads per iteration were most of this phase's
    // time); a 512-thread workgroup splits the same register budget over two queries
    constexpr int QPT = NT >= 1024 ? COEB_MATCH_QPT1024 : 1024 / NT;
    constexpr int RL = NT >= 1024 ? COEB_MATCH_RL1024 : kRegList / QPT;
    uint32_t rl[QPT][RL];
    int rm[QPT];
#pragma unroll
    for (int u = 0; u < QPT; u++) {
        const int q = tid + u * NT;
        rm[u] = -1;
        if (q < nq) {
            const int qn = L.qn[q];
            if (qn >= 0) {
                rm[u] = qn & 0xFFFF;
                const uint32_t* lst = lists + (int64_t)q * stride;
#pragma unroll
                for (int e = 0; e < RL; e++) rl[u][e] = e < rm[u] ? lst[e] : 0u;
            }
        }
    }
    for (int it = 0;; it++) {
        for (int c = tid; c < n; c += NT) L.owner[c] = 0x7fffffff;
        if (tid == 0) s_flag[1] = 0;
        __syncthreads();
        if (it > 0) {
            for (int q = tid; q < nq; q += NT) {
                const int r = L.res[q];
                if (r >= 0 && (L.qn[q] & 0x10000)) atomicMin(&L.owner[r], q);
            }
            __syncthreads();
        }
        bool changed = false;
#pragma unroll
        for (int u = 0; u < QPT; u++) {
            const int q = tid + u * NT;
            if (q < nq) {
                int best = -1;
                uint32_t bk = 0xFFFFFFFFu;
                if (rm[u] >= 0) {
#pragma unroll
                    for (int e = 0; e < RL; e++)
                        if (e < rm[u]) first_min_step(L, rl[u][e], e, q, bk, best);
                    const uint32_t* lst = lists + (int64_t)q * stride;
                    for (int e = RL; e < rm[u]; e++) first_min_step(L, lst[e], e, q, bk, best);
                }
                if (it == 0 || best != L.res[q]) changed = true;
                L.res[q] = best;
            }
        }
        for (int q = tid + QPT * NT; q < nq; q += NT) {
            int best = -1;
            uint32_t bk = 0xFFFFFFFFu;
            const int qn = L.qn[q];
            if (qn >= 0) {
                const int m = qn & 0xFFFF;
                const uint32_t* lst = lists + (int64_t)q * stride;
                for (int e = 0; e < m; e++) first_min_step(L, lst[e], e, q, bk, best);
            }
            if (it == 0 || best != L.res[q]) changed = true;
            L.res[q] = best;
        }
        if (changed) s_flag[1] = 1;
        __syncthreads();
        if (threadIdx.x == 0) s_flag[7] = it + 1;
        if (!s_flag[1]) return false;
        if (it >= kMaxIter) return true;
        __syncthreads();
    }
}

// Phase 3 of the first-minimum matchers: CurrentFrame.mvpMapPoints[res_q] = q (the last q
// wins), then the rotation-histogram filter (ORBmatcher.cc:1446-1466 / :1580-1597) over
// rot = angle(q) - cur[res_q].angle when check_ori.  Leaves L.owner[c] = assigned query or -1
// and returns nmatches (assignments minus the ones the filter removed).  Block-uniform.
template <int NT = kMThreads, class AngleFn>
__device__ int assign_rotation(const MatchLds& L, int n, int nq, const Kp* cur, int check_ori, AngleFn qangle,
                               int* s_hist, int* s_flag)
{
    const int tid = threadIdx.x;
    for (int c = tid; c < n; c += NT) L.owner[c] = -1;
    if (tid < HISTO_LENGTH) s_hist[tid] = 0;
    if (tid == 0) { s_flag[2] = 0; s_flag[3] = 0; }
    __syncthreads();
    int mine = 0;
    for (int q = tid; q < nq; q += NT) {
        const int r = L.res[q];
        if (r >= 0) {
            atomicMax(&L.owner[r], q);
            mine++;
            if (check_ori) {
                const int bin = rot_bin(qangle(q), cur[r].angle);
                L.qn[q] = bin;
                atomicAdd(&s_hist[bin], 1);
            }
        }
    }
    if (mine) atomicAdd(&s_flag[2], mine);
    __syncthreads();
    if (check_ori) {
        if (tid == 0) {
            int i1, i2, i3;
            three_maxima(s_hist, i1, i2, i3);
            s_flag[4] = i1; s_flag[5] = i2; s_flag[6] = i3;
        }
        __syncthreads();
        const int i1 = s_flag[4], i2 = s_flag[5], i3 = s_flag[6];
        int rem = 0;
        for (int q = tid; q < nq; q += NT) {
            const int r = L.res[q];
            if (r >= 0) {
                const int bin = L.qn[q];
                if (bin != i1 && bin != i2 && bin != i3) {
                    L.owner[r] = -1;
                    rem++;
                }
            }
        }
        if (rem) atomicAdd(&s_flag[3], rem);
        __syncthreads();
    }
    return s_flag[2] - s_flag[3];
}

// Pair p's view of a batch launch: the current / last frame arrays and the pose algebra of
// SearchByProjection (ORBmatcher.cc:1339-1350): twc = -Rcw^T tcw (double accumulation), tlc.
struct PairView {
    const Kp* cur; const uint8_t* cdesc; const float* cur_ur;
    const Kp* last; const uint8_t* ldesc; const uint8_t* lhas; const uint8_t* lout; const float* lxw;
    const int* lnobs; uint32_t* lists; const float* T;
    int n, nl;
    bool fwd, bwd;
};

__device__ __forceinline__ PairView pair_view(const MatchCam& cam, const MatchBufs& b, int p, int bmono)
{
    PairView v;
    v.n = b.cur_n[p];
    v.nl = b.last_n[p];
    v.cur = reinterpret_cast<const Kp*>(b.cur_kps) + (int64_t)p * b.cur_stride;
    v.cdesc = b.cur_desc + (int64_t)p * b.cur_stride * 32;
    v.cur_ur = b.cur_ur + (int64_t)p * b.cur_stride;
    v.last = reinterpret_cast<const Kp*>(b.last_kps) + (int64_t)p * b.last_stride;
    v.ldesc = b.last_desc + (int64_t)p * b.last_stride * 32;
    v.lhas = b.last_has + (int64_t)p * b.last_stride;
    v.lout = b.last_out + (int64_t)p * b.last_stride;
    v.lxw = b.last_xw + (int64_t)p * b.last_stride * 3;
    v.lnobs = b.last_nobs + (int64_t)p * b.last_stride;
    v.lists = reinterpret_cast<uint32_t*>(b.scratch) + (int64_t)p * b.scratch_stride;
    v.T = b.Tcw_cur + (int64_t)p * 16;
    const float* T = v.T;
    const float* Tl = b.Tcw_last + (int64_t)p * 16;
    float twc[3], tlc[3];
    for (int k = 0; k < 3; k++) {
        double s = (double)T[0 * 4 + k] * T[3] + (double)T[1 * 4 + k] * T[7];
        s = s + (double)T[2 * 4 + k] * T[11];
        twc[k] = (float)(s * -1.0);
    }
    for (int k = 0; k < 3; k++) {
        float t = Tl[k * 4 + 0] * twc[0] + Tl[k * 4 + 1] * twc[1];
        t = t + Tl[k * 4 + 2] * twc[2];
        tlc[k] = (float)((double)t + (double)Tl[k * 4 + 3]);
    }
    v.fwd = tlc[2] > cam.mb && !bmono;
    v.bwd = -tlc[2] > cam.mb && !bmono;
    return v;
}

__device__ __forceinline__ bool pair_bad(const MatchBufs& b, const PairView& v)
{
    return v.n > b.cur_stride || v.nl > b.last_stride || v.n >= (1 << kIdxBits);
}

// Phase 1 of k_match for the queries q0 + grp, q0 = qbeg, qbeg + qstep, ...: candidate lists
// (static filters) -> v.lists, counts -> qn_out[q] (-1: none; 0x10000 set when q blocks later
// queries); s_flag[0] = 1 when a list overflows kCQ.  The caller zeroes s_flag[0] and syncs after.
template <bool kLds, int NT>
__device__ void build_lists(const MatchCam& cam, const PairView& v, const MatchLds& L, const CurView<kLds>& cv,
                            float th, int qbeg, int qstep, int* qn_out, int* s_flag, long long* tm)
{
    const int tid = threadIdx.x;
    const int nl = v.nl;
    const Kp* last = v.last;
    const uint8_t* ldesc = v.ldesc;
    const uint8_t* lhas = v.lhas;
    const uint8_t* lout = v.lout;
    const float* lxw = v.lxw;
    const int* lnobs = v.lnobs;
    uint32_t* lists = v.lists;
    const bool fwd = v.fwd, bwd = v.bwd;
    // the pose and the level scales every query's window reads, staged once: read from global
    // memory the compiler reloads them for every query (the list stores might alias them) and
    // waits for each load in turn
    __shared__ float s_geo[12 + COEB_MAXL];
    if (tid < 12) s_geo[tid] = v.T[tid];
    else if (tid < 12 + COEB_MAXL) s_geo[tid] = cam.scale[tid - 12];
    __syncthreads();
    const float* T = s_geo;
    const float* scale = s_geo + 12;
    // one kQL-lane group per query; lanes take the candidates of a grid column range kQL at a
    // time and ballot-compact them, so each list stays in enumeration order
    {
        const int grp = tid / kQL, gl = tid % kQL, gsh = (tid & 63) & ~(kQL - 1);
        // a query's inputs (flags, world point, octave, descriptor) are loaded one pass ahead
        // (the flags are kept raw and tested when the query is taken: as lhas[q] && !lout[q] the
        // second load waited for the first, and testing them here waits for both one pass early;
        // Observations() rides along for the count word)
        struct QIn { int has, out, oct, nobs; float X[3]; uint4 d0, d1; };
        auto load_qin = [&](int q, QIn& r) {
            r.has = 0;
            r.out = 1;
            r.nobs = 0;
            if (q < nl) {
                r.has = lhas[q];
                r.out = lout[q];
                r.nobs = lnobs[q];
                r.oct = last[q].octave;
                r.X[0] = lxw[3 * q]; r.X[1] = lxw[3 * q + 1]; r.X[2] = lxw[3 * q + 2];
                const uint4* d = reinterpret_cast<const uint4*>(ldesc + 32 * q);
                r.d0 = d[0]; r.d1 = d[1];
            }
        };
        QIn nx;
        load_qin(qbeg + grp, nx);
        const long long tw0 = tm ? clock64() : 0;
        for (int q0 = qbeg; q0 < nl; q0 += qstep) {
            const int q = q0 + grp;
            const QIn qi = nx;
            load_qin(q + qstep, nx);
            int cnt = -1;
            QueryWin w;
            w.ok = false;
            if (qi.has && !qi.out) w = query_window(cam, T, scale, qi.X, qi.oct, th, fwd, bwd);
            if (w.ok) {
                uint32_t qd[8];
                qd[0] = qi.d0.x; qd[1] = qi.d0.y; qd[2] = qi.d0.z; qd[3] = qi.d0.w;
                qd[4] = qi.d1.x; qd[5] = qi.d1.y; qd[6] = qi.d1.z; qd[7] = qi.d1.w;
                cnt = 0;
                uint32_t* lst = lists + (int64_t)q * kCQ;
                // the window's columns kQL at a time: lane gl holds column gx + gl's CSR range, a
                // group scan gives each column's offset in the concatenated (column-major) order,
                // and the group walks that concatenation kQL candidates at a time -- one pass per
                // column group instead of one per column, same enumeration order
                for (int gx = w.x0; gx <= w.x1; gx += kQL) {
                    int clo = 0, clen = 0;
                    if (gx + gl <= w.x1) {
                        clo = L.cell[(gx + gl) * COEB_GRID_ROWS + w.y0];
                        clen = L.cell[(gx + gl) * COEB_GRID_ROWS + w.y1 + 1] - clo;
                    }
                    const GroupCols gc = group_cols(clo, clen, gl);
                    for (int base = 0; base < gc.total; base += kQL) {
                        const int fi = base + gl;
                        const int e = gc.index(fi);
                        const int c1 = fi < gc.total ? e + 1 : e;      // e < c1 <=> fi < total
                        bool ok = false;
                        uint32_t ent = 0;
                        if (e < c1) {
                            const int i2 = (int)(L.sort[e] & ((1u << kIdxBits) - 1));
                            float x, y, ur;
                            int oct;
                            cv.get(e, i2, x, y, ur, oct);
                            ok = true;
                            if (w.chk) {
                                if (oct < w.minL) ok = false;
                                if (w.maxL >= 0 && oct > w.maxL) ok = false;
                            }
                            const float distx = x - w.u, disty = y - w.v;
                            if (!(fabsf(distx) < w.radius && fabsf(disty) < w.radius)) ok = false;
                            if (ur > 0 && fabsf(w.ur_q - ur) > w.radius) ok = false;
                            if (ok) {
                                const int dist = cv.dist(e, i2, qd);
                                ok = dist <= TH_HIGH;
                                ent = ((uint32_t)dist << kIdxBits) | (uint32_t)i2;
                            }
                        }
                        const uint32_t gb = (uint32_t)(__ballot(ok) >> gsh) & ((1u << kQL) - 1u);
                        if (ok) {
                            const int pos = cnt + __popc(gb & ((1u << gl) - 1u));
                            if (pos < kCQ) lst[pos] = ent;
                        }
                        cnt += __popc(gb);
                    }
                }
                if (cnt > kCQ) s_flag[0] = 1;      // overflow -> sequential path
            }
            if (q < nl && gl == 0) qn_out[q] = cnt < 0 ? -1 : (min(cnt, kCQ) | (qi.nobs > 0 ? 0x10000 : 0));
            if (tm && tid == 0) tm[15] += 1;
        }
        if (tm && (tid & 63) == 0) {           // per-wave loop time: slowest / fastest wave
            const long long dt = clock64() - tw0;
            atomicMax((unsigned long long*)&tm[13], (unsigned long long)dt);
            atomicMin((unsigned long long*)&tm[14], (unsigned long long)dt);
        }
    }
}

// Split form of phase 1 for small batches (few pairs: one workgroup per pair leaves most CUs
// idle): workgroup (p, s) stages pair p's grid and builds the lists of every S-th query group
// (s, s + S, ...), writing the counts to b.qn (pair p's row; entry last_stride + s = s's
// overflow flag).  k_match then starts at phase 2 with those lists (its own phases 0-1 run only
// for the sequential fallback or the retry).
constexpr int kMaxSplit = 8;

template <bool kLds, int NT>
__global__ __launch_bounds__(NT) void k_match_lists(MatchCam cam, MatchBufs b, float th0, int bmono)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int s_flag[8];
    const int p = blockIdx.x, sl = blockIdx.y, S = gridDim.y;
    const PairView v = pair_view(cam, b, p, bmono);
    int* qn = b.qn + (int64_t)p * b.qn_stride;
    if (pair_bad(b, v)) {
        if (threadIdx.x == 0) qn[b.last_stride + sl] = 1;        // k_match reports the error
        return;
    }
    size_t off[7];
    match_lds_bytes(b.cur_stride, 0, kLds, off);
    MatchLds L;
    L.cell = reinterpret_cast<int*>(smem + off[0]);
    L.sort = reinterpret_cast<uint32_t*>(smem + off[1]);
    L.owner = reinterpret_cast<int*>(smem + off[2]);
    L.res = nullptr;
    L.qn = nullptr;
    L.kp = reinterpret_cast<float4*>(smem + off[5]);
    L.desc = reinterpret_cast<uint32_t*>(smem + off[6]);
    CurView<kLds> cv;
    cv.kp = L.kp; cv.desc = L.desc; cv.gkp = v.cur; cv.gur = v.cur_ur; cv.gdesc = v.cdesc;
    stage_grid<kLds, NT>(cam, v.cur, v.cur_ur, v.cdesc, v.n, L);
    if (threadIdx.x == 0) s_flag[0] = 0;
    __syncthreads();
    build_lists<kLds, NT>(cam, v, L, cv, th0, sl * (NT / kQL), S * (NT / kQL), qn, s_flag, nullptr);
    __syncthreads();
    if (threadIdx.x == 0) qn[b.last_stride + sl] = s_flag[0];
}

// k_match's arguments as one struct at offset 0 of the kernarg segment (kernarg<MatchArgs>())
struct MatchArgs {
    MatchCam cam;
    MatchBufs b;
    float th0;
    int bmono, check_ori, retry_below, force_seq, nsplit;
};
template <class T>
__device__ __forceinline__ const T& kernarg()
{
    return *(const T*)__builtin_amdgcn_kernarg_segment_ptr();
}

template <bool kLds, int NT>
#ifndef COEB_MATCH_MINWG
#define COEB_MATCH_MINWG 4     // launch bound in waves per SIMD (4: two 512-thread pairs per CU)
#endif
__global__ __launch_bounds__(NT, COEB_MATCH_MINWG) void k_match(MatchArgs args)
{
    // the arguments are read where they are used, from the kernarg segment (a by-value struct is
    // loaded whole at entry and kept in SGPRs for the kernel's life: 140 spilled SGPRs)
    const MatchArgs& A = kernarg<MatchArgs>();
    const MatchCam& cam = A.cam;
    const MatchBufs& b = A.b;
    const float th0 = A.th0;
    const int bmono = A.bmono, check_ori = A.check_ori, retry_below = A.retry_below, force_seq = A.force_seq,
              nsplit = A.nsplit;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int s_hist[HISTO_LENGTH];
    __shared__ int s_flag[8];
    const int p = blockIdx.x;
    const int tid = threadIdx.x;
    const PairView v = pair_view(cam, b, p, bmono);
    const int n = v.n, nl = v.nl;
    size_t off[7];
    match_lds_bytes(b.cur_stride, b.last_stride, kLds, off);
    MatchLds L;
    L.cell = reinterpret_cast<int*>(smem + off[0]);
    L.sort = reinterpret_cast<uint32_t*>(smem + off[1]);
    L.owner = reinterpret_cast<int*>(smem + off[2]);
    L.res = reinterpret_cast<int*>(smem + off[3]);
    L.qn = reinterpret_cast<int*>(smem + off[4]);
    L.kp = reinterpret_cast<float4*>(smem + off[5]);
    L.desc = reinterpret_cast<uint32_t*>(smem + off[6]);
    const Kp* cur = v.cur;
    const uint8_t* cdesc = v.cdesc;
    const float* cur_ur = v.cur_ur;
    const Kp* last = v.last;
    const uint8_t* ldesc = v.ldesc;
    const float* lxw = v.lxw;
    const int* lnobs = v.lnobs;
    uint32_t* lists = v.lists;
    if (pair_bad(b, v)) {
        if (tid == 0) { atomicOr(b.err, 16); b.nmatch[p] = 0; }
        return;
    }
    CurView<kLds> cv;
    cv.kp = L.kp; cv.desc = L.desc; cv.gkp = cur; cv.gur = cur_ur; cv.gdesc = cdesc;

    // ---- phase 0: stage CurrentFrame, grid CSR by a stable counting sort ----
    // phase clocks: experiment builds only (-DCOEB_MATCH_CLOCK=1 with COEB_MATCH_TIMING set,
    // tools/_match_timing.py); the product build has no hook (14 SGPRs)
    long long* tm = COEB_MATCH_CLOCK && b.timing ? b.timing + (int64_t)p * 16 : nullptr;
    if (tm && tid == 0) { tm[0] = clock64(); tm[13] = 0; tm[14] = 0x7fffffffffffffffll; tm[15] = 0; }
    // with split lists (nsplit > 0) the grid is built only if the sequential path or the retry
    // needs it
    bool staged = false;
    auto ensure_grid = [&]() {
        if (!staged) stage_grid<kLds, NT>(cam, cur, cur_ur, cdesc, n, L);
        staged = true;
    };
    if (!nsplit) ensure_grid();
    if (tm && tid == 0) tm[1] = clock64();

    const float* T = v.T;
    const bool fwd = v.fwd, bwd = v.bwd;

    float th = th0;
    int nmatches = 0;
    for (int attempt = 0; attempt < 2; attempt++) {
        // ---- phase 1: candidate lists (static filters) ----
        if (tid == 0) { s_flag[0] = 0; s_flag[1] = 0; s_flag[2] = 0; s_flag[3] = 0; }
        if (attempt == 0 && nsplit) {
            // lists and counts from k_match_lists
            const int* qg = b.qn + (int64_t)p * b.qn_stride;
            for (int q = tid; q < nl; q += NT) L.qn[q] = qg[q];
            if (tid == 0) {
                int ov = 0;
                for (int k = 0; k < nsplit; k++) ov |= qg[b.last_stride + k];
                s_flag[0] = ov;
            }
        } else {
            ensure_grid();
            __syncthreads();
            build_lists<kLds, NT>(cam, v, L, cv, th, 0, NT / kQL, L.qn, s_flag, tm);
        }
        __syncthreads();
        bool seq = force_seq || s_flag[0];
        // ---- phase 2: claims by fixpoint iteration ----
        if (tm && tid == 0) tm[2 + 4 * attempt] = clock64();
        if (!seq) seq = claims_first_min<NT>(L, lists, kCQ, n, nl, s_flag);
        if (tm && tid == 0) { tm[3 + 4 * attempt] = clock64(); tm[12 + attempt] = s_flag[7]; }
        // ---- sequential path (overflow / no convergence / forced): literal loop, one thread ----
        if (seq) {
            ensure_grid();
            for (int c = tid; c < n; c += NT) L.owner[c] = -1;
            __syncthreads();
            if (tid == 0) {
                for (int q = 0; q < nl; q++) {
                    int best = -1;
                    if (L.qn[q] >= 0) {
                        const QueryWin w = query_window(cam, T, cam.scale, lxw + 3 * q, last[q].octave, th, fwd, bwd);
                        if (w.ok) {
                            uint32_t qd[8];
                            for (int k = 0; k < 8; k++) qd[k] = reinterpret_cast<const uint32_t*>(ldesc + 32 * q)[k];
                            int bestDist = 256;
                            for_candidates<kLds>(w, L.cell, L.sort, cv, [&](int e, int i2) {
                                const int own = L.owner[i2];
                                if (own >= 0 && lnobs[own] > 0) return true;
                                const int dist = cv.dist(e, i2, qd);
                                if (dist < bestDist) { bestDist = dist; best = i2; }
                                return true;
                            });
                            if (bestDist > TH_HIGH) best = -1;
                            if (best >= 0) L.owner[best] = q;
                        }
                    }
                    L.res[q] = best;
                }
            }
            __syncthreads();
        }
        // ---- phase 3: mvpMapPoints, rotation consistency ----
        if (tm && tid == 0) tm[4 + 4 * attempt] = clock64();
        nmatches = assign_rotation<NT>(L, n, nl, cur, check_ori, [&](int q) { return last[q].angle; }, s_hist, s_flag);
        if (tm && tid == 0) tm[5 + 4 * attempt] = clock64();
        __syncthreads();
        if (nmatches >= retry_below) break;
        th = 2 * th0;                                  // Tracking.cc:954-958
    }
    int* mo = b.match + (int64_t)p * b.cur_stride;
    for (int i = tid; i < n; i += NT) mo[i] = L.owner[i];
    if (tid == 0) b.nmatch[p] = nmatches;
    if (tm && tid == 0) tm[10] = clock64();
}


// ================================ k_match_local ================================
// ORBmatcher::SearchByProjection(Frame &F, const vector<MapPoint*> &vpMapPoints, th)
// (src/ORBmatcher.cc:44-129) for one frame, one 1024-thread workgroup.  The local-map points
// arrive as Frame::isInFrustum left them (projection, predicted level, viewing cosine).
//   phase 0  stage CurrentFrame + grid CSR (stage_grid)
//   phase 1  per point (kQL lanes): window r = RadiusByViewingCos(cos) * th * scale[level],
//            levels [level-1, level], keypoints whose entry MapPoint has Observations() > 0
//            dropped, stereo check; EVERY candidate kept with its distance and octave (the
//            second best feeds the ratio test, whatever its distance)
//   phase 2  claims: point q skips keypoints taken by an earlier point p < q with
//            Observations() > 0; best / second best / ratio test on what is left.  Same
//            Jacobi fixpoint as k_match (owner[c] = min such p), reaching the sequential answer
//   phase 3  the last point assigned to a keypoint wins (F.mvpMapPoints[bestIdx] = pMP)
// Overflowing lists or no convergence run the literal loop instead.
struct LocalBufs {
    const void* cur_kps; const uint8_t* cur_desc; const float* cur_ur; const int* cur_obs; int cur_n;
    const uint8_t* in_view; const float* proj_x; const float* proj_y; const float* proj_xr;
    const int* level; const float* view_cos; const uint8_t* desc; const int* nobs; int mp_n;
    int* match; int* nmatch; uint32_t* lists; int* err; int* path;
    // batch form (cur_n_arr != null): workgroup p searches frame p's arrays (LocalBufsHost)
    const int* cur_n_arr; const uint8_t* active; int cur_stride, mp_stride, mp_desc_stride;
};

// workgroup p's view of a batch launch
__device__ __forceinline__ LocalBufs local_at_pair(LocalBufs b, int p)
{
    if (!b.cur_n_arr) return b;
    const int64_t c = (int64_t)p * b.cur_stride, m = (int64_t)p * b.mp_stride;
    b.cur_n = b.cur_n_arr[p];
    b.cur_kps = reinterpret_cast<const Kp*>(b.cur_kps) + c;
    b.cur_desc += c * 32; b.cur_ur += c; b.cur_obs += c;
    b.in_view += m; b.proj_x += m; b.proj_y += m; b.proj_xr += m; b.level += m; b.view_cos += m; b.nobs += m;
    b.desc += (int64_t)p * b.mp_desc_stride * 32;
    b.match += c; b.nmatch += p; b.lists += m * kCQ; b.path += 2 * p;
    return b;
}

__device__ __forceinline__ float radius_by_viewing_cos(float c) { return c > 0.998f ? 2.5f : 4.0f; }   // ORBmatcher.cc:131-137

// window of point q (r = RadiusByViewingCos * th (if th != 1) * mvScaleFactors[level])
__device__ __forceinline__ QueryWin local_window(const MatchCam& cam, const LocalBufs& b, int q, float th)
{
    QueryWin w;
    const int level = b.level[q];
    float r = radius_by_viewing_cos(b.view_cos[q]);
    if (th != 1.0f) r *= th;
    w.u = b.proj_x[q];
    w.v = b.proj_y[q];
    w.radius = r * cam.scale[level];
    w.minL = level - 1;
    w.maxL = level;
    w.ur_q = b.proj_xr[q];
    w.ok = b.in_view[q] && window_cells(cam, w);
    return w;
}

constexpr int kLocKeyDist = 16, kLocKeyOct = 12;    // list entry: dist << 16 | octave << 12 | index

template <bool kLds, int NT>
__global__ __launch_bounds__(NT) void k_match_local(MatchCam cam, LocalBufs b0, float th, float nnratio,
                                                           int force_seq)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int s_flag[8];
    const int tid = threadIdx.x;
    const LocalBufs b = local_at_pair(b0, blockIdx.x);
    if (b0.active && !b0.active[blockIdx.x]) {                 // frame not handed to TrackLocalMap
        for (int c = tid; c < b.cur_n; c += NT) b.match[c] = -1;
        if (tid == 0) *b.nmatch = 0;
        return;
    }
    const int n = b.cur_n, nq = b.mp_n;
    size_t off[7];
    match_lds_bytes(n, nq, kLds, off);
    MatchLds L;
    L.cell = reinterpret_cast<int*>(smem + off[0]);
    L.sort = reinterpret_cast<uint32_t*>(smem + off[1]);
    L.owner = reinterpret_cast<int*>(smem + off[2]);
    L.res = reinterpret_cast<int*>(smem + off[3]);
    L.qn = reinterpret_cast<int*>(smem + off[4]);
    L.kp = reinterpret_cast<float4*>(smem + off[5]);
    L.desc = reinterpret_cast<uint32_t*>(smem + off[6]);
    const Kp* cur = reinterpret_cast<const Kp*>(b.cur_kps);
    if (n >= (1 << kIdxBits)) {
        if (tid == 0) { atomicOr(b.err, 16); *b.nmatch = 0; }
        return;
    }
    CurView<kLds> cv;
    cv.kp = L.kp; cv.desc = L.desc; cv.gkp = cur; cv.gur = b.cur_ur; cv.gdesc = b.cur_desc;
    // the level scales, read by every point's window (from the kernel arguments each read is a
    // dependent global load)
    __shared__ float s_scale[COEB_MAXL];
    if (tid < COEB_MAXL) s_scale[tid] = cam.scale[tid];
    stage_grid<kLds, NT>(cam, cur, b.cur_ur, b.cur_desc, n, L, kLds ? b.cur_obs : nullptr);
    if (tid == 0) { s_flag[0] = 0; s_flag[1] = 0; s_flag[2] = 0; }
    __syncthreads();

    // ---- phase 1: candidate lists ----
    {
        const int grp = tid / kQL, gl = tid % kQL, gsh = (tid & 63) & ~(kQL - 1);
        constexpr int qstep = NT / kQL;
        // a point's inputs (isInFrustum's outputs, Observations(), descriptor) are loaded one pass
        // ahead, as in k_match's lists
        struct LIn { int view, level, nobs; float vcos, px, py, pxr; uint4 d0, d1; };
        auto load_lin = [&](int q, LIn& r) {
            r.view = 0;
            r.nobs = 0;
            if (q < nq) {
                r.view = b.in_view[q];
                r.level = b.level[q];
                r.vcos = b.view_cos[q];
                r.px = b.proj_x[q]; r.py = b.proj_y[q]; r.pxr = b.proj_xr[q];
                r.nobs = b.nobs[q];
                const uint4* d = reinterpret_cast<const uint4*>(b.desc + 32 * q);
                r.d0 = d[0]; r.d1 = d[1];
            }
        };
        LIn nx;
        load_lin(grp, nx);
        for (int q0 = 0; q0 < nq; q0 += qstep) {
            const int q = q0 + grp;
            const LIn qi = nx;
            load_lin(q + qstep, nx);
            int cnt = -1;
            QueryWin w;                               // local_window, from the prefetched inputs
            w.ok = false;
            if (q < nq && qi.view) {
                float r = radius_by_viewing_cos(qi.vcos);
                if (th != 1.0f) r *= th;
                w.u = qi.px;
                w.v = qi.py;
                w.radius = r * s_scale[qi.level];
                w.minL = qi.level - 1;
                w.maxL = qi.level;
                w.ur_q = qi.pxr;
                w.ok = window_cells(cam, w);
            }
            if (w.ok) {
                uint32_t qd[8];
                qd[0] = qi.d0.x; qd[1] = qi.d0.y; qd[2] = qi.d0.z; qd[3] = qi.d0.w;
                qd[4] = qi.d1.x; qd[5] = qi.d1.y; qd[6] = qi.d1.z; qd[7] = qi.d1.w;
                cnt = 0;
                uint32_t* lst = b.lists + (int64_t)q * kCQ;
                for (int gx = w.x0; gx <= w.x1; gx += kQL) {        // column groups, as in k_match
                    int clo = 0, clen = 0;
                    if (gx + gl <= w.x1) {
                        clo = L.cell[(gx + gl) * COEB_GRID_ROWS + w.y0];
                        clen = L.cell[(gx + gl) * COEB_GRID_ROWS + w.y1 + 1] - clo;
                    }
                    const GroupCols gc = group_cols(clo, clen, gl);
                    for (int base = 0; base < gc.total; base += kQL) {
                        const int fi = base + gl;
                        const int e = gc.index(fi);
                        const int c1 = fi < gc.total ? e + 1 : e;
                        bool ok = false;
                        uint32_t ent = 0;
                        if (e < c1) {
                            const int i2 = (int)(L.sort[e] & ((1u << kIdxBits) - 1));
                            float x, y, ur;
                            int oct;
                            cv.get(e, i2, x, y, ur, oct);
                            ok = !(oct < w.minL || oct > w.maxL);              // chk is always set here
                            const float distx = x - w.u, disty = y - w.v;
                            if (!(fabsf(distx) < w.radius && fabsf(disty) < w.radius)) ok = false;
                            if (!kLds && b.cur_obs[i2] > 0) ok = false;  // :86-88, entry holder (LDS: kHeldOct)
                            if (ur > 0 && fabsf(w.ur_q - ur) > w.radius) ok = false;   // :90-95
                            if (ok) {
                                const int dist = cv.dist(e, i2, qd);
                                ent = ((uint32_t)dist << kLocKeyDist) | ((uint32_t)oct << kLocKeyOct) | (uint32_t)i2;
                            }
                        }
                        const uint32_t gb = (uint32_t)(__ballot(ok) >> gsh) & ((1u << kQL) - 1u);
                        if (ok) {
                            const int pos = cnt + __popc(gb & ((1u << gl) - 1u));
                            if (pos < kCQ) lst[pos] = ent;
                        }
                        cnt += __popc(gb);
                    }
                }
                if (cnt > kCQ) s_flag[0] = 1;
            }
            if (q < nq && gl == 0) L.qn[q] = cnt < 0 ? -1 : (min(cnt, kCQ) | (qi.nobs > 0 ? 0x10000 : 0));
        }
    }
    __syncthreads();
    bool seq = force_seq || s_flag[0];
    int iters = 0;
    // ---- phase 2: claims by fixpoint iteration ----
    // The thread's first LQ points (tid, tid + 1024, ...) keep the first LR entries of their
    // lists in registers across the iterations, as k_match's claims do; the rest are read from
    // the global lists in each iteration
    constexpr int LQ = COEB_LOCAL_QPT, LR = COEB_LOCAL_RL;
    auto walk = [&](uint32_t v, int q, int& bestDist, int& bestLevel, int& bestDist2, int& bestLevel2, int& bestIdx) {
        const int i2 = (int)(v & ((1u << kIdxBits) - 1));
        if (L.owner[i2] < q) return;                       // taken by an earlier point
        const int dist = (int)(v >> kLocKeyDist), oct = (int)((v >> kLocKeyOct) & 0xF);
        if (dist < bestDist) {
            bestDist2 = bestDist; bestDist = dist;
            bestLevel2 = bestLevel; bestLevel = oct; bestIdx = i2;
        } else if (dist < bestDist2) {
            bestLevel2 = oct; bestDist2 = dist;
        }
    };
    auto decide = [&](int bestDist, int bestLevel, int bestDist2, int bestLevel2, int bestIdx) {
        return bestDist <= TH_HIGH && !(bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2)
                   ? bestIdx : -1;
    };
    if (!seq) {
        uint32_t rl[LQ][LR];
        int rm[LQ];
#pragma unroll
        for (int u = 0; u < LQ; u++) {
            const int q = tid + u * NT;
            rm[u] = -1;
            if (q < nq) {
                const int qn = L.qn[q];
                if (qn >= 0) {
                    rm[u] = qn & 0xFFFF;
                    const uint32_t* lst = b.lists + (int64_t)q * kCQ;
#pragma unroll
                    for (int e = 0; e < LR; e++) rl[u][e] = e < rm[u] ? lst[e] : 0u;
                }
            }
        }
        for (int it = 0;; it++) {
            iters = it + 1;
            for (int c = tid; c < n; c += NT) L.owner[c] = 0x7fffffff;
            if (tid == 0) s_flag[1] = 0;
            __syncthreads();
            if (it > 0) {
                for (int q = tid; q < nq; q += NT) {
                    const int r = L.res[q];
                    if (r >= 0 && (L.qn[q] & 0x10000)) atomicMin(&L.owner[r], q);
                }
                __syncthreads();
            }
#pragma unroll
            for (int u = 0; u < LQ; u++) {
                const int q = tid + u * NT;
                if (q < nq) {
                    int res = -1;
                    if (rm[u] >= 0) {
                        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
#pragma unroll
                        for (int e = 0; e < LR; e++)
                            if (e < rm[u]) walk(rl[u][e], q, bestDist, bestLevel, bestDist2, bestLevel2, bestIdx);
                        const uint32_t* lst = b.lists + (int64_t)q * kCQ;
                        for (int e = LR; e < rm[u]; e++) walk(lst[e], q, bestDist, bestLevel, bestDist2, bestLevel2, bestIdx);
                        res = decide(bestDist, bestLevel, bestDist2, bestLevel2, bestIdx);
                    }
                    if (it == 0 || res != L.res[q]) s_flag[1] = 1;
                    L.res[q] = res;
                }
            }
            for (int q = tid + LQ * NT; q < nq; q += NT) {
                const int qn = L.qn[q];
                int res = -1;
                if (qn >= 0) {
                    const int m = qn & 0xFFFF;
                    const uint32_t* lst = b.lists + (int64_t)q * kCQ;
                    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                    for (int e = 0; e < m; e++) walk(lst[e], q, bestDist, bestLevel, bestDist2, bestLevel2, bestIdx);
                    res = decide(bestDist, bestLevel, bestDist2, bestLevel2, bestIdx);
                }
                if (it == 0 || res != L.res[q]) s_flag[1] = 1;
                L.res[q] = res;
            }
            __syncthreads();
            if (!s_flag[1]) break;
            if (it >= kMaxIter) { seq = true; break; }
            __syncthreads();
        }
    }
    if (seq) {
        // literal loop (ORBmatcher.cc:48-126), one thread; L.owner = Observations() of each
        // keypoint's holder
        for (int c = tid; c < n; c += NT) { L.owner[c] = b.cur_obs[c]; }
        __syncthreads();
        if (tid == 0) {
            b.path[0] = force_seq ? 1 : s_flag[0] ? 2 : 3;   // forced / list overflow / no convergence
            b.path[1] = iters;
            int nm = 0;
            for (int c = 0; c < n; c++) b.match[c] = -1;
            for (int q = 0; q < nq; q++) {
                QueryWin w = local_window(cam, b, q, th);
                if (!w.ok) continue;
                uint32_t qd[8];
                for (int k = 0; k < 8; k++) qd[k] = reinterpret_cast<const uint32_t*>(b.desc + 32 * q)[k];
                int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                for_candidates<kLds>(w, L.cell, L.sort, cv, [&](int e, int i2) {
                    if (L.owner[i2] > 0) return true;
                    const int dist = cv.dist(e, i2, qd);
                    float x, y, ur;
                    int oct;
                    cv.get(e, i2, x, y, ur, oct);
                    if (dist < bestDist) {
                        bestDist2 = bestDist; bestDist = dist;
                        bestLevel2 = bestLevel; bestLevel = oct; bestIdx = i2;
                    } else if (dist < bestDist2) {
                        bestLevel2 = oct; bestDist2 = dist;
                    }
                    return true;
                });
                if (bestDist <= TH_HIGH) {
                    if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) continue;
                    b.match[bestIdx] = q;
                    L.owner[bestIdx] = b.nobs[q];
                    nm++;
                }
            }
            *b.nmatch = nm;
        }
        return;
    }
    // ---- phase 3: the last assignment to a keypoint wins ----
    for (int c = tid; c < n; c += NT) L.owner[c] = -1;
    __syncthreads();
    int mine = 0;
    for (int q = tid; q < nq; q += NT) {
        const int r = L.res[q];
        if (r >= 0) { atomicMax(&L.owner[r], q); mine++; }
    }
    if (mine) atomicAdd(&s_flag[2], mine);
    __syncthreads();
    for (int c = tid; c < n; c += NT) b.match[c] = L.owner[c];
    if (tid == 0) { *b.nmatch = s_flag[2]; b.path[0] = 0; b.path[1] = iters; }
}


// ================================ k_match_kf ================================
// ORBmatcher::SearchByProjection(Frame &CurrentFrame, KeyFrame *pKF, const set<MapPoint*>
// &sAlreadyFound, th, ORBdist) (src/ORBmatcher.cc:1473-1600), the relocalisation search
// (calls Tracking.cc:1531, 1545), for one frame, one 1024-thread workgroup.  Per KeyFrame map
// point: project with CurrentFrame.mTcw (no depth-sign test in the reference), bounds, the
// distance-invariance range, MapPoint::PredictScale, window th * scale[level] over levels
// [level-1, level+1], no stereo check.  A keypoint holding any MapPoint (at entry or given
// earlier in this call) is skipped (:1545-1546), so every assignment blocks later points: the
// same fixpoint as k_match with every query blocking.  Then the rotation histogram.
struct KfBufs {
    const void* cur_kps; const uint8_t* cur_desc; const uint8_t* cur_has; int cur_n;
    const uint8_t* valid; const float* xw; const uint8_t* desc; const float* maxd; const float* mind;
    const float* angle; int kf_n;
    const float* Tcw;
    int* match; int* nmatch; uint32_t* lists; int* err; int* path;
};

// MapPoint::PredictScale(dist, Frame*) (MapPoint.cc:402-417); log canonical as in the oracle
__device__ __forceinline__ int predict_scale(const MatchCam& cam, float max_dist, float dist)
{
    const float ratio = max_dist / dist;
    int s = (int)ceilf((float)log((double)ratio) / cam.log_sf);
    if (s < 0) s = 0;
    else if (s >= cam.nlevels) s = cam.nlevels - 1;
    return s;
}

__device__ __forceinline__ QueryWin kf_window(const MatchCam& cam, const float* T, const float* Ow, const KfBufs& b,
                                              int q, float th)
{
    QueryWin w;
    w.ok = false;
    w.st = false;
    w.ur_q = 0.f;
    if (!b.valid[q]) return w;
    const float* X = b.xw + 3 * q;
    float p3[3];
    for (int k = 0; k < 3; k++) {                  // x3Dc = Rcw*x3Dw + tcw (as query_window)
        float t = T[k * 4 + 0] * X[0] + T[k * 4 + 1] * X[1];
        t = t + T[k * 4 + 2] * X[2];
        p3[k] = (float)((double)t + (double)T[k * 4 + 3]);
    }
    const float invzc = (float)(1.0 / (double)p3[2]);
    w.u = __builtin_fmaf(cam.fx * p3[0], invzc, cam.cx);
    w.v = __builtin_fmaf(cam.fy * p3[1], invzc, cam.cy);
    if (w.u < cam.min_x || w.u > cam.max_x) return w;
    if (w.v < cam.min_y || w.v > cam.max_y) return w;
    // dist3D = cv::norm(x3Dw - Ow): float differences, squares summed in double (normL2_32f)
    const float d0 = X[0] - Ow[0], d1 = X[1] - Ow[1], d2 = X[2] - Ow[2];
    double ss = 0.0;
    ss += (double)d0 * (double)d0;
    ss += (double)d1 * (double)d1;
    ss += (double)d2 * (double)d2;
    const float dist3D = (float)sqrt(ss);
    const float maxd = b.maxd[q], mind = b.mind[q];
    if (dist3D < 0.8f * mind || dist3D > 1.2f * maxd) return w;   // Get{Min,Max}DistanceInvariance
    const int lvl = predict_scale(cam, maxd, dist3D);
    w.radius = th * cam.scale[lvl];
    w.minL = lvl - 1;
    w.maxL = lvl + 1;
    w.ok = window_cells(cam, w);
    return w;
}

template <bool kLds>
__global__ __launch_bounds__(kMThreads) void k_match_kf(MatchCam cam, KfBufs b, float th, int orb_dist, int check_ori,
                                                        int force_seq)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int s_hist[HISTO_LENGTH];
    __shared__ int s_flag[8];
    const int tid = threadIdx.x;
    const int n = b.cur_n, nq = b.kf_n;
    size_t off[7];
    match_lds_bytes(n, nq, kLds, off);
    MatchLds L;
    L.cell = reinterpret_cast<int*>(smem + off[0]);
    L.sort = reinterpret_cast<uint32_t*>(smem + off[1]);
    L.owner = reinterpret_cast<int*>(smem + off[2]);
    L.res = reinterpret_cast<int*>(smem + off[3]);
    L.qn = reinterpret_cast<int*>(smem + off[4]);
    L.kp = reinterpret_cast<float4*>(smem + off[5]);
    L.desc = reinterpret_cast<uint32_t*>(smem + off[6]);
    const Kp* cur = reinterpret_cast<const Kp*>(b.cur_kps);
    if (n >= (1 << kIdxBits)) {
        if (tid == 0) { atomicOr(b.err, 16); *b.nmatch = 0; }
        return;
    }
    // no uR is read here: the CSR staging takes the keypoint records only
    CurView<kLds> cv;
    cv.kp = L.kp; cv.desc = L.desc; cv.gkp = cur; cv.gur = nullptr; cv.gdesc = b.cur_desc;
    stage_grid<kLds>(cam, cur, nullptr, b.cur_desc, n, L);
    const float* T = b.Tcw;
    float Ow[3];
    for (int k = 0; k < 3; k++) {                 // Ow = -Rcw^T tcw (double accumulation)
        double s = (double)T[0 * 4 + k] * T[3] + (double)T[1 * 4 + k] * T[7];
        s = s + (double)T[2 * 4 + k] * T[11];
        Ow[k] = (float)(s * -1.0);
    }
    if (tid == 0) { s_flag[0] = 0; s_flag[1] = 0; }
    __syncthreads();
    // ---- phase 1: candidate lists (window, levels, entry holders, dist <= ORBdist) ----
    {
        const int grp = tid / kQL, gl = tid % kQL, gsh = (tid & 63) & ~(kQL - 1);
        for (int q0 = 0; q0 < nq; q0 += kMThreads / kQL) {
            const int q = q0 + grp;
            int cnt = -1;
            QueryWin w;
            w.ok = false;
            if (q < nq) w = kf_window(cam, T, Ow, b, q, th);
            if (w.ok) {
                uint32_t qd[8];
                const uint4* d = reinterpret_cast<const uint4*>(b.desc + 32 * q);
                const uint4 d0 = d[0], d1 = d[1];
                qd[0] = d0.x; qd[1] = d0.y; qd[2] = d0.z; qd[3] = d0.w;
                qd[4] = d1.x; qd[5] = d1.y; qd[6] = d1.z; qd[7] = d1.w;
                cnt = 0;
                uint32_t* lst = b.lists + (int64_t)q * kCQ;
                for (int gx = w.x0; gx <= w.x1; gx += kQL) {        // column groups, as in k_match
                    int clo = 0, clen = 0;
                    if (gx + gl <= w.x1) {
                        clo = L.cell[(gx + gl) * COEB_GRID_ROWS + w.y0];
                        clen = L.cell[(gx + gl) * COEB_GRID_ROWS + w.y1 + 1] - clo;
                    }
                    const GroupCols gc = group_cols(clo, clen, gl);
                    for (int base = 0; base < gc.total; base += kQL) {
                        const int fi = base + gl;
                        const int e = gc.index(fi);
                        const int c1 = fi < gc.total ? e + 1 : e;
                        bool ok = false;
                        uint32_t ent = 0;
                        if (e < c1) {
                            const int i2 = (int)(L.sort[e] & ((1u << kIdxBits) - 1));
                            float x, y, ur;
                            int oct;
                            cv.get(e, i2, x, y, ur, oct);
                            ok = !(oct < w.minL || oct > w.maxL);            // chk always set (maxL >= 0)
                            const float distx = x - w.u, disty = y - w.v;
                            if (!(fabsf(distx) < w.radius && fabsf(disty) < w.radius)) ok = false;
                            if (b.cur_has[i2]) ok = false;                     // :1545-1546, entry holder
                            if (ok) {
                                const int dist = cv.dist(e, i2, qd);
                                ok = dist <= orb_dist;
                                ent = ((uint32_t)dist << kIdxBits) | (uint32_t)i2;
                            }
                        }
                        const uint32_t gb = (uint32_t)(__ballot(ok) >> gsh) & ((1u << kQL) - 1u);
                        if (ok) {
                            const int pos = cnt + __popc(gb & ((1u << gl) - 1u));
                            if (pos < kCQ) lst[pos] = ent;
                        }
                        cnt += __popc(gb);
                    }
                }
                if (cnt > kCQ) s_flag[0] = 1;
            }
            if (q < nq && gl == 0) L.qn[q] = cnt < 0 ? -1 : (min(cnt, kCQ) | 0x10000);
        }
    }
    __syncthreads();
    const bool overflow = s_flag[0] != 0;
    bool seq = force_seq || overflow;
    if (!seq) seq = claims_first_min(L, b.lists, kCQ, n, nq, s_flag);
    if (seq) {
        // literal loop (ORBmatcher.cc:1489-1578), one thread; L.owner[c] >= 0: c holds a MapPoint
        const int path = force_seq ? 1 : overflow ? 2 : 3;
        for (int c = tid; c < n; c += kMThreads) L.owner[c] = b.cur_has[c] ? nq : -1;
        __syncthreads();
        if (tid == 0) {
            b.path[0] = path;
            for (int q = 0; q < nq; q++) {
                int best = -1;
                const QueryWin w = kf_window(cam, T, Ow, b, q, th);
                if (w.ok) {
                    uint32_t qd[8];
                    for (int k = 0; k < 8; k++) qd[k] = reinterpret_cast<const uint32_t*>(b.desc + 32 * q)[k];
                    int bestDist = 256;
                    for_candidates<kLds>(w, L.cell, L.sort, cv, [&](int e, int i2) {
                        if (L.owner[i2] >= 0) return true;
                        const int dist = cv.dist(e, i2, qd);
                        if (dist < bestDist) { bestDist = dist; best = i2; }
                        return true;
                    });
                    if (bestDist > orb_dist) best = -1;
                    if (best >= 0) L.owner[best] = q;
                }
                L.res[q] = best;
            }
        }
        __syncthreads();
    } else if (tid == 0) {
        b.path[0] = 0;
    }
    // ---- phase 3: assignments (unique here), rotation consistency ----
    const int nm = assign_rotation(L, n, nq, cur, check_ori, [&](int q) { return b.angle[q]; }, s_hist, s_flag);
    for (int c = tid; c < n; c += kMThreads) b.match[c] = L.owner[c];
    if (tid == 0) *b.nmatch = nm;
}

}  // namespace

int launch_prep(const PrepBufs& b, int F, hipStream_t s, ProfileHook* prof)
{
    prof_begin(prof, "k_prep", s);
    hipLaunchKernelGGL(k_prep, dim3((b.stride + kThreads - 1) / kThreads, F), dim3(kThreads), 0, s, b);
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_match(const MatchCam& cam, const MatchBufs& b, int P, float th, int bmono, int check_ori,
                 int retry_below, hipStream_t s, ProfileHook* prof)
{
    if (P <= 0) return 0;
    const int force_seq = coeb_switch("COEB_MATCH_SEQUENTIAL") ? 1 : 0;   // test knob: exact literal path
    const size_t lds_full = match_lds_bytes(b.cur_stride, b.last_stride, true, nullptr) + 256;
    const size_t lds_min = match_lds_bytes(b.cur_stride, b.last_stride, false, nullptr) + 256;
    // 512-thread workgroups when a pair's LDS fits half a CU (config A: 80.6 KB), so two pairs
    // share a CU and one pair's barrier waits overlap the other's work (k_match 0.355 -> 0.335 ms
    // per 1025-frame launch, profiles/r03/s5/match_nt_ab.txt); otherwise 1024 threads per pair
    const int nt = lds_full <= 80 * 1024 ? 512 : 1024;     // (1024 always: config A 8.62-8.70 vs 8.35-8.47 ms, r06/s10)
    // Few pairs (a small shard): the candidate lists are built by k_match_lists with nsplit
    // workgroups per pair, so ~256 workgroups share the work instead of P; COEB_MATCH_SPLIT=0
    // turns this off, =N forces N
    int nsplit = 0;
    if (b.qn && b.qn_stride >= b.last_stride + kMaxSplit) {
        nsplit = std::min(kMaxSplit, 256 / std::max(P, 1));
        if (const char* e = coeb_switch("COEB_MATCH_SPLIT")) nsplit = std::max(0, std::min(kMaxSplit, atoi(e)));
        if (nsplit < 2) nsplit = 0;
    }
    // (the current frame read from global memory instead, for half the LDS: config A 8.72-8.77 vs
    // 8.39-8.46 ms per step, D 35.43-35.55 vs 35.17-35.24, profiles/r06/s14)
    bool lds_cur = lds_full <= 160 * 1024;
    if (!lds_cur && lds_min > 160 * 1024) return -2;
    if (nsplit) {
        // the lists kernel stages the current frame in LDS (COEB_MATCH_LISTS_LDS=0: reads it from
        // global memory); k_match then needs no staged frame (its phases 0-1 run only for the
        // sequential fallback / the retry, then reading the frame from global memory), so it takes
        // a fraction of the LDS and leaves the CU to the other pipeline's kernels
        // (COEB_MATCH_SPLIT_FULL=1 keeps the staged form)
        const char* le = coeb_experiment("COEB_MATCH_LISTS_LDS");
        const bool lists_lds = lds_cur && !(le && atoi(le) == 0);
        const size_t lds_l = match_lds_bytes(b.cur_stride, 0, lists_lds, nullptr);
        auto gl = [&](auto kern) {
            lds_limit_max((const void*)kern);
            hipLaunchKernelGGL(kern, dim3(P, nsplit), dim3(1024), lds_l, s, cam, b, th, bmono);
        };
        prof_begin(prof, "k_match_lists", s);
        if (lists_lds) gl(k_match_lists<true, 1024>);
        else gl(k_match_lists<false, 1024>);
        prof_end(prof, s);
        const char* fe = coeb_experiment("COEB_MATCH_SPLIT_FULL");
        if (!(fe && atoi(fe) != 0)) lds_cur = false;
    }
    auto go = [&](auto kern, size_t lds) {
        lds_limit_max((const void*)kern);
        const MatchArgs a{cam, b, th, bmono, check_ori, retry_below, force_seq, nsplit};
        hipLaunchKernelGGL(kern, dim3(P), dim3(nt), lds - 256, s, a);
    };
    prof_begin(prof, "k_match", s);
    if (lds_cur) {
        if (nt == 512) go(k_match<true, 512>, lds_full);
        else go(k_match<true, 1024>, lds_full);
    } else {
        if (nt == 512) go(k_match<false, 512>, lds_min);
        else go(k_match<false, 1024>, lds_min);
    }
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_match_local(const MatchCam& cam, const LocalBufsHost& h, float th, float nnratio, hipStream_t s, ProfileHook* prof)
{
    LocalBufs b;
    b.cur_kps = h.cur_kps; b.cur_desc = h.cur_desc; b.cur_ur = h.cur_ur; b.cur_obs = h.cur_obs; b.cur_n = h.cur_n;
    b.in_view = h.in_view; b.proj_x = h.proj_x; b.proj_y = h.proj_y; b.proj_xr = h.proj_xr; b.level = h.level;
    b.view_cos = h.view_cos; b.desc = h.desc; b.nobs = h.nobs; b.mp_n = h.mp_n;
    b.match = h.match; b.nmatch = h.nmatch; b.lists = h.lists; b.err = h.err; b.path = h.path;
    b.cur_n_arr = h.cur_n_arr; b.active = h.active;
    b.cur_stride = h.cur_stride; b.mp_stride = h.mp_n; b.mp_desc_stride = h.mp_desc_stride;
    const int P = h.cur_n_arr ? h.npairs : 1;
    if (P <= 0) return 0;
    if (h.cur_n_arr && h.cur_stride >= (1 << kIdxBits)) return -2;
    const int force_seq = coeb_switch("COEB_MATCH_SEQUENTIAL") ? 1 : 0;
    const int cs = std::max(h.cur_n_arr ? h.cur_stride : h.cur_n, 1), qs = std::max(h.mp_n, 1);
    const size_t lds_full = match_lds_bytes(cs, qs, true, nullptr) + 256;
    const size_t lds_min = match_lds_bytes(cs, qs, false, nullptr) + 256;
    prof_begin(prof, "k_match_local", s);
    // COEB_LOCAL_LDS=0: the current frame read from global memory (a third of the LDS, so the
    // workgroup finds room beside the pose and flow kernels sooner)
    const char* le = coeb_experiment("COEB_LOCAL_LDS");
    // a batch (the configs[4] loop's TrackLocalMap) takes 512 threads per frame: the kernel alone
    // runs longer (0.78 vs 0.51 ms per 1537 frames) but leaves room to the pose / flow kernels it
    // overlaps, and the config-D step is shorter (35.11 vs 35.45-35.60 ms, profiles/r06/s8); one
    // frame from host buffers keeps 1024 (its latency is all there is)
    auto go = [&](auto k1024, auto k512, size_t lds) {
        if (P > 1) {
            lds_limit_max((const void*)k512);
            hipLaunchKernelGGL(k512, dim3(P), dim3(512), lds - 256, s, cam, b, th, nnratio, force_seq);
        } else {
            lds_limit_max((const void*)k1024);
            hipLaunchKernelGGL(k1024, dim3(P), dim3(1024), lds - 256, s, cam, b, th, nnratio, force_seq);
        }
    };
    if (lds_full <= 160 * 1024 && !(le && atoi(le) == 0)) {
        go(k_match_local<true, 1024>, k_match_local<true, 512>, lds_full);
    } else if (lds_min <= 160 * 1024) {
        go(k_match_local<false, 1024>, k_match_local<false, 512>, lds_min);
    } else {
        prof_end(prof, s);
        return -2;
    }
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int match_list_cap() { return kCQ; }

int launch_match_kf(const MatchCam& cam, const KfBufsHost& h, float th, int orb_dist, int check_ori, hipStream_t s,
                    ProfileHook* prof)
{
    KfBufs b;
    b.cur_kps = h.cur_kps; b.cur_desc = h.cur_desc; b.cur_has = h.cur_has; b.cur_n = h.cur_n;
    b.valid = h.valid; b.xw = h.xw; b.desc = h.desc; b.maxd = h.maxd; b.mind = h.mind; b.angle = h.angle;
    b.kf_n = h.kf_n; b.Tcw = h.Tcw; b.match = h.match; b.nmatch = h.nmatch; b.lists = h.lists; b.err = h.err;
    b.path = h.path;
    const int force_seq = coeb_switch("COEB_MATCH_SEQUENTIAL") ? 1 : 0;
    const int cs = std::max(h.cur_n, 1), qs = std::max(h.kf_n, 1);
    const size_t lds_full = match_lds_bytes(cs, qs, true, nullptr) + 256;
    const size_t lds_min = match_lds_bytes(cs, qs, false, nullptr) + 256;
    prof_begin(prof, "k_match_kf", s);
    if (lds_full <= 160 * 1024) {
        lds_limit_max((const void*)k_match_kf<true>);
        hipLaunchKernelGGL(k_match_kf<true>, dim3(1), dim3(kMThreads), lds_full - 256, s, cam, b, th, orb_dist, check_ori,
                           force_seq);
    } else if (lds_min <= 160 * 1024) {
        lds_limit_max((const void*)k_match_kf<false>);
        hipLaunchKernelGGL(k_match_kf<false>, dim3(1), dim3(kMThreads), lds_min - 256, s, cam, b, th, orb_dist, check_ori,
                           force_seq);
    } else {
        prof_end(prof, s);
        return -2;
    }
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
