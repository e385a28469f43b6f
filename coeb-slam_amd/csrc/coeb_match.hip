// coeb_match.hip -- CDNA4 kernels for the tracking-time projection matcher:
//   ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)  src/ORBmatcher.cc:1329-1471
//   Frame::AssignFeaturesToGrid / GetFeaturesInArea                   src/Frame.cc:396-411, 503-568
//   Frame::ComputeStereoFromRGBD                                      src/Frame.cc:820-842
//   ORBmatcher::DescriptorDistance                                    src/ORBmatcher.cc:1648-1664
//
// One workgroup per (current, last) frame pair.  Phase 0 (whole workgroup) builds the
// 64 x 48 keypoint grid as a CSR: keys (cell << 13 | index) are bitonic-sorted in LDS, so a
// cell column ix over rows [iy0, iy1] is ONE contiguous range and the reference's
// enumeration order (ix outer, iy inner, in-cell insertion order) is range order.  Phase 1
// walks the LastFrame points in index order (the claim dependency of :1404-1406/1429 is
// sequential); each query's candidates are evaluated 64 at a time by one wave (window,
// level, claim, stereo check, 256-bit Hamming via popcount) and reduced to the first strict
// minimum with one wave min.  Phase 2 applies the rotation-histogram top-3 filter.
#include <hip/hip_runtime.h>

#include "coeb_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr int kCurMax = 4096;          // current keypoints per frame (host checks)
constexpr int kCellIdxBits = 13;
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

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v)
{
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(v, o, 64);
        v = y < v ? y : v;
    }
    return v;
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
__global__ __launch_bounds__(kThreads) void k_match(MatchCam cam, MatchBufs b, float th0, int bmono,
                                                     int check_ori, int retry_below)
{
    __shared__ uint32_t s_sort[kCurMax];
    __shared__ int s_cell[COEB_GRID_CELLS + 1];
    __shared__ int s_owner[kCurMax];
    const int p = blockIdx.x;
    const int tid = threadIdx.x, lane = __lane_id(), wv = tid >> 6;
    const int n = b.cur_n[p];
    const int nl = b.last_n[p];
    const Kp* cur = reinterpret_cast<const Kp*>(b.cur_kps) + (int64_t)p * b.cur_stride;
    const uint8_t* cdesc = b.cur_desc + (int64_t)p * b.cur_stride * 32;
    const float* cur_ur = b.cur_ur + (int64_t)p * b.cur_stride;
    const Kp* last = reinterpret_cast<const Kp*>(b.last_kps) + (int64_t)p * b.last_stride;
    const uint8_t* ldesc = b.last_desc + (int64_t)p * b.last_stride * 32;
    const uint8_t* lhas = b.last_has + (int64_t)p * b.last_stride;
    const uint8_t* lout = b.last_out + (int64_t)p * b.last_stride;
    const float* lxw = b.last_xw + (int64_t)p * b.last_stride * 3;
    const int* lnobs = b.last_nobs + (int64_t)p * b.last_stride;
    int* hist_i2 = b.scratch + (int64_t)p * b.scratch_stride;
    int* hist_bin = hist_i2 + b.scratch_stride / 2;
    if (n > kCurMax) {
        if (tid == 0) { atomicOr(b.err, 16); b.nmatch[p] = 0; }
        return;
    }

    // ---- phase 0: grid CSR (AssignFeaturesToGrid / PosInGrid) ----
    int np2 = 64;
    while (np2 < n) np2 <<= 1;
    for (int c = tid; c <= COEB_GRID_CELLS; c += kThreads) s_cell[c] = 0;
    __syncthreads();
    for (int i = tid; i < np2; i += kThreads) {
        uint32_t key = 0xFFFFFFFFu;
        if (i < n) {
            const int px = (int)roundf((cur[i].x - cam.min_x) * cam.grid_inv_w);
            const int py = (int)roundf((cur[i].y - cam.min_y) * cam.grid_inv_h);
            if (px >= 0 && px < COEB_GRID_COLS && py >= 0 && py < COEB_GRID_ROWS) {
                const int cell = px * COEB_GRID_ROWS + py;
                key = ((uint32_t)cell << kCellIdxBits) | (uint32_t)i;
                atomicAdd(&s_cell[cell + 1], 1);
            }
        }
        s_sort[i] = key;
    }
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < np2; i += kThreads) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t a = s_sort[i], c = s_sort[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > c) == up) { s_sort[i] = c; s_sort[ixj] = a; }
                }
            }
            __syncthreads();
        }
    }
    // inclusive scan of counts -> cell_start (single wave; 3072 cells)
    if (wv == 0) {
        int carry = 0;
        for (int base = 1; base <= COEB_GRID_CELLS; base += 64) {
            const int c = base + lane;
            int v = c <= COEB_GRID_CELLS ? s_cell[c] : 0;
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(v, o, 64);
                if (lane >= o) v += y;
            }
            if (c <= COEB_GRID_CELLS) s_cell[c] = carry + v;
            carry += __shfl(v, 63, 64);
        }
    }
    __syncthreads();

    // ---- pose algebra (ORBmatcher.cc:1339-1350) ----
    const float* T = b.Tcw_cur + (int64_t)p * 16;
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
    const bool bForward = tlc[2] > cam.mb && !bmono;
    const bool bBackward = -tlc[2] > cam.mb && !bmono;

    if (wv != 0) return;   // phases 1-2: one wave (sequential claim dependency)

    float th = th0;
    int nmatches = 0;
    for (int attempt = 0; attempt < 2; attempt++) {
        for (int i = lane; i < n; i += 64) s_owner[i] = -1;
        __builtin_amdgcn_wave_barrier();
        nmatches = 0;
        int nhist = 0;
        for (int i = 0; i < nl; i++) {
            if (!lhas[i] || lout[i]) continue;
            const float X0 = lxw[3 * i], X1 = lxw[3 * i + 1], X2 = lxw[3 * i + 2];
            float p3[3];
            for (int k = 0; k < 3; k++) {
                float t = T[k * 4 + 0] * X0 + T[k * 4 + 1] * X1;
                t = t + T[k * 4 + 2] * X2;
                p3[k] = (float)((double)t + (double)T[k * 4 + 3]);
            }
            const float invzc = (float)(1.0 / (double)p3[2]);
            if (invzc < 0) continue;
            const float u = __builtin_fmaf(cam.fx * p3[0], invzc, cam.cx);
            const float v = __builtin_fmaf(cam.fy * p3[1], invzc, cam.cy);
            if (u < cam.min_x || u > cam.max_x) continue;
            if (v < cam.min_y || v > cam.max_y) continue;
            const int nLastOctave = last[i].octave;
            const float radius = th * cam.scale[nLastOctave];
            int minLevel, maxLevel;
            if (bForward) { minLevel = nLastOctave; maxLevel = -1; }
            else if (bBackward) { minLevel = 0; maxLevel = nLastOctave; }
            else { minLevel = nLastOctave - 1; maxLevel = nLastOctave + 1; }
            // GetFeaturesInArea cell window (Frame.cc:508-522)
            const int nMinCellX = max(0, (int)floorf(((u - cam.min_x) - radius) * cam.grid_inv_w));
            if (nMinCellX >= COEB_GRID_COLS) continue;
            const int nMaxCellX = min(COEB_GRID_COLS - 1, (int)ceilf(((u - cam.min_x) + radius) * cam.grid_inv_w));
            if (nMaxCellX < 0) continue;
            const int nMinCellY = max(0, (int)floorf(((v - cam.min_y) - radius) * cam.grid_inv_h));
            if (nMinCellY >= COEB_GRID_ROWS) continue;
            const int nMaxCellY = min(COEB_GRID_ROWS - 1, (int)ceilf(((v - cam.min_y) + radius) * cam.grid_inv_h));
            if (nMaxCellY < 0) continue;
            const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
            uint32_t qd[8];
#pragma unroll
            for (int w = 0; w < 8; w++) qd[w] = reinterpret_cast<const uint32_t*>(ldesc + 32 * i)[w];
            const float ur_q = __builtin_fmaf(-cam.bf, invzc, u);     // u - mbf*invzc (fused)
            unsigned long long best = ~0ull;
            int pos = 0;
            for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
                const int c0 = s_cell[ix * COEB_GRID_ROWS + nMinCellY];
                const int c1 = s_cell[ix * COEB_GRID_ROWS + nMaxCellY + 1];
                for (int base = c0; base < c1; base += 64) {
                    const int q = base + lane;
                    unsigned long long cand = ~0ull;
                    if (q < c1) {
                        const int i2 = (int)(s_sort[q] & ((1u << kCellIdxBits) - 1));
                        const Kp kp = cur[i2];
                        bool ok = true;
                        if (bCheckLevels) {
                            if (kp.octave < minLevel) ok = false;
                            if (maxLevel >= 0 && kp.octave > maxLevel) ok = false;
                        }
                        const float distx = kp.x - u, disty = kp.y - v;
                        ok = ok && fabsf(distx) < radius && fabsf(disty) < radius;
                        if (ok) {
                            const int own = __hip_atomic_load(&s_owner[i2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            if (own >= 0 && lnobs[own] > 0) ok = false;
                        }
                        if (ok && cur_ur[i2] > 0) {
                            const float er = fabsf(ur_q - cur_ur[i2]);
                            if (er > radius) ok = false;
                        }
                        if (ok) {
                            const int dist = hamming32(qd, reinterpret_cast<const uint32_t*>(cdesc + 32 * i2));
                            if (dist < 256)
                                cand = ((unsigned long long)dist << 40) | ((unsigned long long)(pos + q - base) << 16) |
                                       (unsigned long long)i2;
                        }
                    }
                    cand = wave_min_u64(cand);
                    best = cand < best ? cand : best;
                }
                pos += c1 - c0;
            }
            if (best != ~0ull) {
                const int bestDist = (int)(best >> 40);
                const int bestIdx2 = (int)(best & 0xFFFF);
                if (bestDist <= TH_HIGH) {
                    if (lane == 0)
                        __hip_atomic_store(&s_owner[bestIdx2], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __builtin_amdgcn_wave_barrier();
                    nmatches++;
                    if (check_ori) {
                        float rot = last[i].angle - cur[bestIdx2].angle;
                        if (rot < 0.0) rot += 360.0f;
                        int bin = (int)roundf(rot * (1.0f / HISTO_LENGTH));
                        if (bin == HISTO_LENGTH) bin = 0;
                        if (lane == 0) { hist_i2[nhist] = bestIdx2; hist_bin[nhist] = bin; }
                        nhist++;
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        if (check_ori) {
            // ComputeThreeMaxima (ORBmatcher.cc:1602-1643)
            int cnt = 0;
            if (lane < HISTO_LENGTH)
                for (int e = 0; e < nhist; e++) cnt += hist_bin[e] == lane;
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int bi = 0; bi < HISTO_LENGTH; bi++) {
                const int s = __shfl(cnt, bi, 64);
                if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = bi; }
                else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = bi; }
                else if (s > max3) { max3 = s; ind3 = bi; }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
            int removed = 0;
            for (int e = lane; e < nhist; e += 64) {
                const int bn = hist_bin[e];
                if (bn != ind1 && bn != ind2 && bn != ind3) {
                    __hip_atomic_store(&s_owner[hist_i2[e]], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    removed++;
                }
            }
            for (int o = 32; o > 0; o >>= 1) removed += __shfl_xor(removed, o, 64);
            nmatches -= removed;
        }
        __builtin_amdgcn_wave_barrier();
        if (nmatches >= retry_below) break;
        th = 2 * th0;                  // Tracking.cc:954-958
    }
    int* mo = b.match + (int64_t)p * b.cur_stride;
    for (int i = lane; i < n; i += 64) mo[i] = s_owner[i];
    if (lane == 0) b.nmatch[p] = nmatches;
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
    prof_begin(prof, "k_match", s);
    hipLaunchKernelGGL(k_match, dim3(P), dim3(kThreads), 0, s, cam, b, th, bmono, check_ori, retry_below);
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
