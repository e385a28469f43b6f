// coeb_track.hip -- Tracking::TrackLocalMap on a device batch (BASELINE configs[4]):
//   TrackWithMotionModel's outlier discard          src/Tracking.cc:966-993   (k_tlm_discard)
//   SearchLocalPoints: skip matched points,         src/Tracking.cc:1222-1272 (k_tlm_frustum)
//     Frame::isInFrustum(pMP, 0.5)                  src/Frame.cc:445-501
//     MapPoint::PredictScale                        src/MapPoint.cc:402-417
//   ORBmatcher::SearchByProjection(F, vpLocalMapPoints, th)     k_match_local (coeb_match.hip)
//   second Optimizer::PoseOptimization (:1006)      k_tlm_pose_prep + k_pose (coeb_pose.hip)
//
// The local map of frame f is the MapPoints of two KeyFrames, KF2 = frame f-2 and KF1 = frame
// f-1, each keypoint with depth > 0 one MapPoint with a single observation
// (MapPoint::UpdateNormalAndDepth, MapPoint.cc:330-371).  KF1 is the world frame of the pair
// (as in the motion-model step); KF2's points are placed by KF1's motion-model pose.  The
// definition and its canonical float forms are DESIGN.md s4.3; oracle/orb_oracle.c
// (oc_local_map_build) restates them for the parity tests.
//
// Launch order: k_tlm_snapshot on the context stream (it copies every batch array the rest
// reads, so the next batch's extraction may overwrite them), then on the pose stream after
// the first k_pose: k_tlm_discard -> k_tlm_frustum -> k_match_local -> k_tlm_pose_prep -> k_pose.
#include <hip/hip_runtime.h>

#include "coeb_internal.hpp"

namespace {

constexpr int kT = 256;

struct KpT { float x, y, size, angle, response; int octave, class_id; };   // coeb_keypoint

// ---- k_tlm_snapshot: frame f's slots into the s_* arrays; seen / nmap cleared ----
__global__ __launch_bounds__(kT) void k_tlm_snapshot(TlmBufs t)
{
    const int f = blockIdx.y;
    const int i = blockIdx.x * kT + threadIdx.x;
    const int n = t.counts[f];
    const int64_t K = t.K;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        t.s_cnt[f] = n;
        t.s_nm1[f] = f ? t.nmatch1[f] : 0;
        t.nmap[f] = 0;
    }
    if (i < t.K) t.seen[f * K + i] = 0;
    if (i >= n) return;
    const int64_t o = f * K + i;
    const uint4* src = reinterpret_cast<const uint4*>(t.desc + o * 32);
    uint4* dst = reinterpret_cast<uint4*>(t.s_desc + (o + K) * 32);
    dst[0] = src[0];
    dst[1] = src[1];
    t.s_oct[o] = (int8_t)reinterpret_cast<const KpT*>(t.kps)[o].octave;
    t.s_has[o] = t.has[o];
    t.s_xw[3 * o + 0] = t.xw[3 * o + 0];
    t.s_xw[3 * o + 1] = t.xw[3 * o + 1];
    t.s_xw[3 * o + 2] = t.xw[3 * o + 2];
    t.s_m1[o] = f ? t.match1[o] : -1;
}

// ---- k_tlm_discard: Tracking.cc:966-985 ----
// A matched keypoint flagged outlier by the first PoseOptimization loses its MapPoint; the
// MapPoints the matcher assigned (inliers and outliers) get mnLastFrameSeen = current, so
// SearchLocalPoints skips them (:979, :1237, :1249).  nmatchesMap counts the kept ones with
// Observations() > 0.
__global__ __launch_bounds__(kT) void k_tlm_discard(TlmBufs t)
{
    const int f = blockIdx.y + 1;
    const int i = blockIdx.x * kT + threadIdx.x;
    const int64_t K = t.K;
    const bool go = t.s_nm1[f] >= t.min_matches;                  // PoseOptimization ran (:954-964)
    const int n = t.s_cnt[f];
    bool kept = false;
    if (i < n) {
        const int64_t o = f * K + i;
        const int m = t.s_m1[o];
        if (go && m >= 0) t.seen[f * K + m] = 1;
        const bool inl = go && t.has1[o] && !t.outl1[o];
        t.cur_obs[o] = inl ? t.nobs : -1;
        kept = inl && t.nobs > 0;
    }
    const uint64_t b = __ballot(kept);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(&t.nmap[f], (int)__popcll(b));
}

// x = R*X + t (cv::Mat R*X + t: small-matrix float products, the addend added in double)
__device__ __forceinline__ void gemm_add(const float* T, const float* X, float* out)
{
#pragma unroll
    for (int k = 0; k < 3; k++) {
        float v = T[k * 4 + 0] * X[0] + T[k * 4 + 1] * X[1];
        v = v + T[k * 4 + 2] * X[2];
        out[k] = (float)((double)v + (double)T[k * 4 + 3]);
    }
}

__device__ __forceinline__ double norm3(const float* d)
{
    double ss = 0.0;
    ss += (double)d[0] * (double)d[0];
    ss += (double)d[1] * (double)d[1];
    ss += (double)d[2] * (double)d[2];
    return sqrt(ss);
}

// ---- k_tlm_frustum: the local map of frame f through Frame::isInFrustum(pMP, 0.5) ----
__global__ __launch_bounds__(kT) void k_tlm_frustum(MatchCam cam, TlmBufs t)
{
    const int f = blockIdx.y + 1;
    const int q = blockIdx.x * kT + threadIdx.x;
    const int64_t K = t.K, M = 2 * K;
    if (q >= M) return;
    // TrackWithMotionModel's verdict (:954-961, :993): TrackLocalMap runs only when it held
    const bool ok = t.s_nm1[f] >= t.min_matches && t.nmap[f] >= t.min_map;
    if (q == 0) t.active[f] = ok ? 1 : 0;
    const int64_t o = f * M + q;
    int in = 0, lvl = 0;
    if (ok) {
        const bool kf1 = q >= K;
        const int j = kf1 ? (int)(q - K) : q;
        const int g = kf1 ? f - 1 : f - 2;
        bool exists = g >= 0 && (kf1 || t.nkf >= 2);
        if (exists) exists = j < t.s_cnt[g] && t.s_has[g * K + j] && !(kf1 && t.seen[f * K + j]);
        if (exists) {
            const float* X = t.s_xw + 3 * (g * K + j);
            float P[3], Ow[3];
            if (kf1) {
                P[0] = X[0]; P[1] = X[1]; P[2] = X[2];
                Ow[0] = Ow[1] = Ow[2] = 0.0f;
            } else {                                               // UnprojectStereo with KF2's Twc
                const float* T = t.T1 + (int64_t)(f - 1) * 16;
                const float Xl[3] = {X[0], X[1], X[2]};
                gemm_add(T, Xl, P);
                Ow[0] = T[3]; Ow[1] = T[7]; Ow[2] = T[11];
            }
            // UpdateNormalAndDepth, one observation (MapPoint.cc:348-370)
            const float d[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
            const double nd = norm3(d);
            float Pn[3];
            for (int k = 0; k < 3; k++) Pn[k] = (float)((double)d[k] / nd);
            const int oct = t.s_oct[g * K + j];
            const float maxd = (float)nd * cam.scale[oct];
            const float mind = maxd / cam.scale[cam.nlevels - 1];
            // isInFrustum (Frame.cc:445-501)
            const float* T = t.T1 + (int64_t)f * 16;
            float Pc[3];
            gemm_add(T, P, Pc);
            bool v = !(Pc[2] < 0.0f);
            float u = 0.f, vv = 0.f, invz = 0.f;
            if (v) {
                invz = 1.0f / Pc[2];
                u = __builtin_fmaf(cam.fx * Pc[0], invz, cam.cx);
                vv = __builtin_fmaf(cam.fy * Pc[1], invz, cam.cy);
                if (u < cam.min_x || u > cam.max_x) v = false;
                if (vv < cam.min_y || vv > cam.max_y) v = false;
            }
            float dist = 0.f, viewCos = 0.f;
            if (v) {
                float Oc[3];
                for (int k = 0; k < 3; k++) {                      // mOw = -mRcw.t()*mtcw (GEMM_1_T)
                    double s = (double)T[0 * 4 + k] * T[3] + (double)T[1 * 4 + k] * T[7];
                    s = s + (double)T[2 * 4 + k] * T[11];
                    Oc[k] = (float)(s * -1.0);
                }
                const float PO[3] = {P[0] - Oc[0], P[1] - Oc[1], P[2] - Oc[2]};
                dist = (float)norm3(PO);
                if (dist < 0.8f * mind || dist > 1.2f * maxd) v = false;
                if (v) {
                    double dot = 0.0;
                    dot += (double)PO[0] * (double)Pn[0];
                    dot += (double)PO[1] * (double)Pn[1];
                    dot += (double)PO[2] * (double)Pn[2];
                    viewCos = (float)(dot / (double)dist);
                    if (viewCos < 0.5f) v = false;
                }
            }
            if (v) {
                const float ratio = maxd / dist;                   // PredictScale
                int s = (int)ceilf((float)log((double)ratio) / cam.log_sf);
                lvl = s < 0 ? 0 : (s >= cam.nlevels ? cam.nlevels - 1 : s);
                in = 1;
                t.px[o] = u;
                t.py[o] = vv;
                t.pxr[o] = __builtin_fmaf(-cam.bf, invz, u);       // u - mbf*invz (fused)
                t.vcos[o] = viewCos;
                t.lm_xw[3 * o + 0] = P[0];
                t.lm_xw[3 * o + 1] = P[1];
                t.lm_xw[3 * o + 2] = P[2];
            }
        }
    }
    t.in_view[o] = (uint8_t)in;
    t.level[o] = lvl;
    t.lm_nobs[o] = t.nobs;
}

// ---- k_tlm_pose_prep: CurrentFrame.mvpMapPoints for the second PoseOptimization ----
// A keypoint holds the local-map point SearchByProjection gave it, else the motion-model
// MapPoint it kept through the discard; the pose starts at the first optimisation's result.
__global__ __launch_bounds__(kT) void k_tlm_pose_prep(TlmBufs t)
{
    const int f = blockIdx.y + 1;
    const int i = blockIdx.x * kT + threadIdx.x;
    const int64_t K = t.K;
    const bool ok = t.active[f] != 0;
    const int n = t.s_cnt[f];
    if (blockIdx.x == 0) {
        if (threadIdx.x < 16) t.T2[(int64_t)f * 16 + threadIdx.x] = t.T1[(int64_t)f * 16 + threadIdx.x];
        if (threadIdx.x == 16) t.n2[f] = ok ? n : 0;
    }
    if (i >= n) return;
    const int64_t o = f * K + i;
    if (!ok) {          // TrackLocalMap does not run: no second optimisation, nothing is an outlier
        t.has2[o] = 0;
        t.outl2[o] = 0;
        return;
    }
    const int lm = t.lmatch[o];
    t.outl2[o] = 0;
    if (lm >= 0) {
        const int64_t p = f * 2 * K + lm;
        t.has2[o] = 1;
        t.xw2[3 * o + 0] = t.lm_xw[3 * p + 0];
        t.xw2[3 * o + 1] = t.lm_xw[3 * p + 1];
        t.xw2[3 * o + 2] = t.lm_xw[3 * p + 2];
    } else if (t.cur_obs[o] >= 0) {
        t.has2[o] = 1;
        t.xw2[3 * o + 0] = t.xw1[3 * o + 0];
        t.xw2[3 * o + 1] = t.xw1[3 * o + 1];
        t.xw2[3 * o + 2] = t.xw1[3 * o + 2];
    } else {
        t.has2[o] = 0;
    }
}

}  // namespace

int launch_tlm_snapshot(const TlmBufs& t, int F, hipStream_t s, ProfileHook* prof)
{
    prof_begin(prof, "k_tlm_snapshot", s);
    hipLaunchKernelGGL(k_tlm_snapshot, dim3((t.K + kT - 1) / kT, F), dim3(kT), 0, s, t);
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_tlm_frustum(const MatchCam& cam, const TlmBufs& t, int F, hipStream_t s, ProfileHook* prof)
{
    if (F < 2) return 0;
    prof_begin(prof, "k_tlm_discard", s);
    hipLaunchKernelGGL(k_tlm_discard, dim3((t.K + kT - 1) / kT, F - 1), dim3(kT), 0, s, t);
    prof_end(prof, s);
    prof_begin(prof, "k_tlm_frustum", s);
    hipLaunchKernelGGL(k_tlm_frustum, dim3((2 * t.K + kT - 1) / kT, F - 1), dim3(kT), 0, s, cam, t);
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_tlm_pose_prep(const TlmBufs& t, int F, hipStream_t s, ProfileHook* prof)
{
    if (F < 2) return 0;
    prof_begin(prof, "k_tlm_pose_prep", s);
    hipLaunchKernelGGL(k_tlm_pose_prep, dim3((t.K + kT - 1) / kT, F - 1), dim3(kT), 0, s, t);
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
