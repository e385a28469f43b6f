// coeb_pose.hip -- Optimizer::PoseOptimization(Frame*) (src/Optimizer.cc:239-451) on the device:
// g2o's Levenberg-Marquardt (OptimizationAlgorithmLevenberg, BlockSolver_6_3 with one SE3
// vertex, LinearSolverDense) over the frame's EdgeSE3ProjectXYZOnlyPose /
// EdgeStereoSE3ProjectXYZOnlyPose edges with the Huber kernel, 4 rounds x 10 iterations with
// chi2 outlier classification.  g2o is not vendored in the reference (Thirdparty/g2o absent):
// this follows its published 2012 algorithm as restated in oracle/orb_oracle.c
// (oc_pose_optimization), operation for operation, in double precision.
//
// One 256-thread workgroup per frame.  Edge i lives with thread i % 256; per-edge sums (the
// 21 Hessian terms, 6 gradient terms, robust chi2) are reduced in the canonical order
// (per-thread sequential, 32-thread runs in thread order, the 8 runs in order) so the
// result is bit-identical to the oracle.  The 6x6 solve, the SE3 exponential and the LM
// bookkeeping run on thread 0 and are broadcast through LDS.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "coeb_internal.hpp"

namespace {

constexpr int kPT = 256;

struct Se3 { double w, x, y, z, t[3]; };
struct KpRec { float x, y, size, angle, response; int octave, class_id; };   // coeb_keypoint
struct PEdge { double X[3], obs[3], w; int stereo; };

// Eigen's Quaternion-from-rotation-matrix, t <= 0 branch with the largest diagonal entry I
// (compile-time indices: a runtime-indexed R / q would live in scratch memory).
template <int I>
__device__ __forceinline__ void pq_from_R_diag(const double R[9], double q[4])
{
    constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
    double t = sqrt(((R[I * 4] - R[J * 4]) - R[K * 4]) + 1.0);
    q[I] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (R[K * 3 + J] - R[J * 3 + K]) * t;
    q[J] = (R[J * 3 + I] + R[I * 3 + J]) * t;
    q[K] = (R[K * 3 + I] + R[I * 3 + K]) * t;
}

__device__ void pq_from_R(const double R[9], Se3& s)
{
    double t = (R[0] + R[4]) + R[8];
    double q[4];
    if (t > 0.0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (R[7] - R[5]) * t;
        q[1] = (R[2] - R[6]) * t;
        q[2] = (R[3] - R[1]) * t;
    } else {
        int i = 0;
        if (R[4] > R[0]) i = 1;
        if (R[8] > (i ? R[4] : R[0])) i = 2;
        if (i == 0) pq_from_R_diag<0>(R, q);
        else if (i == 1) pq_from_R_diag<1>(R, q);
        else pq_from_R_diag<2>(R, q);
    }
    s.x = q[0]; s.y = q[1]; s.z = q[2]; s.w = q[3];
}

__device__ __forceinline__ double rl_d(double v, int j)   // v of lane j (j wave-uniform)
{
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), j);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// kWave: called by every lane of a wave with the same (uniform) values; the four divisions run
// as one, component c on lanes c mod 4, and come back by v_readlane (the same quotients).
template <bool kWave = false>
__device__ void pq_normalize(Se3& s)
{
    if (s.w < 0) { s.w = -s.w; s.x = -s.x; s.y = -s.y; s.z = -s.z; }
    const double n = sqrt(((s.x * s.x + s.y * s.y) + s.z * s.z) + s.w * s.w);
    if constexpr (kWave) {
        const int c = __lane_id() & 3;
        const double q = (c == 0 ? s.x : c == 1 ? s.y : c == 2 ? s.z : s.w) / n;
        s.x = rl_d(q, 0); s.y = rl_d(q, 1); s.z = rl_d(q, 2); s.w = rl_d(q, 3);
    } else {
        s.x = s.x / n; s.y = s.y / n; s.z = s.z / n; s.w = s.w / n;
    }
}

__device__ __forceinline__ void pq_rotate(const Se3& s, const double v[3], double o[3])
{
    double uv[3] = {s.y * v[2] - s.z * v[1], s.z * v[0] - s.x * v[2], s.x * v[1] - s.y * v[0]};
    uv[0] = uv[0] + uv[0]; uv[1] = uv[1] + uv[1]; uv[2] = uv[2] + uv[2];
    const double c[3] = {s.y * uv[2] - s.z * uv[1], s.z * uv[0] - s.x * uv[2], s.x * uv[1] - s.y * uv[0]};
    for (int k = 0; k < 3; k++) o[k] = (v[k] + s.w * uv[k]) + c[k];
}

template <bool kWave = false>
__device__ Se3 pq_mul(const Se3& a, const Se3& b)
{
    Se3 r;
    double bt[3];
    pq_rotate(a, b.t, bt);
    for (int k = 0; k < 3; k++) r.t[k] = a.t[k] + bt[k];
    r.w = ((a.w * b.w - a.x * b.x) - a.y * b.y) - a.z * b.z;
    r.x = ((a.w * b.x + a.x * b.w) + a.y * b.z) - a.z * b.y;
    r.y = ((a.w * b.y + a.y * b.w) + a.z * b.x) - a.x * b.z;
    r.z = ((a.w * b.z + a.z * b.w) + a.x * b.y) - a.y * b.x;
    pq_normalize<kWave>(r);
    return r;
}

// canonical sin/cos (the oracle's table)
__constant__ double kPqSin[14] = {0x1.0000000000000p+0, -0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13,
                                  0x1.71de3a556c734p-19, -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33, -0x1.ae7f3e733b81fp-41,
                                  0x1.952c77030ad4ap-49, -0x1.2f49b46814157p-57, 0x1.71b8ef6dcf572p-66, -0x1.761b413163819p-75,
                                  0x1.3f3ccdd165fa9p-84, -0x1.d1ab1c2dccea3p-94};
__constant__ double kPqCos[14] = {0x1.0000000000000p+0, -0x1.0000000000000p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10,
                                  0x1.a01a01a01a01ap-16, -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29, -0x1.93974a8c07c9dp-37,
                                  0x1.ae7f3e733b81fp-45, -0x1.6827863b97d97p-53, 0x1.e542ba4020225p-62, -0x1.0ce396db7f853p-70,
                                  0x1.f2cf01972f578p-80, -0x1.88e85fc6a4e59p-89};

__device__ void pq_sincos(double x, double& sn, double& cs)
{
    const double k = floor(x * 0.63661977236758134308 + 0.5);
    const double r = (x - k * 1.57079632673412561417e+00) - k * 6.07710050650619224932e-11;
    const double r2 = r * r;
    double ps = kPqSin[13], pc = kPqCos[13];
    for (int n = 12; n >= 0; n--) {
        ps = ps * r2 + kPqSin[n];
        pc = pc * r2 + kPqCos[n];
    }
    const double s0 = r * ps, c0 = pc;
    const int q = ((int)(long)k) & 3;
    if (q == 0) { sn = s0; cs = c0; }
    else if (q == 1) { sn = c0; cs = -s0; }
    else if (q == 2) { sn = -s0; cs = -c0; }
    else { sn = -c0; cs = s0; }
}

// SE3Quat::exp(update); kWave as pq_normalize (A, B, C as one division on lanes 0..2)
template <bool kWave = false>
__device__ Se3 pq_exp(const double u[6])
{
    const double o0 = u[0], o1 = u[1], o2 = u[2];
    const double theta = sqrt((o0 * o0 + o1 * o1) + o2 * o2);
    const double Om[9] = {0.0, -o2, o1, o2, 0.0, -o0, -o1, o0, 0.0};
    double Om2[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            Om2[i * 3 + j] = (Om[i * 3] * Om[j] + Om[i * 3 + 1] * Om[3 + j]) + Om[i * 3 + 2] * Om[6 + j];
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = ((i % 4 == 0 ? 1.0 : 0.0) + Om[i]) + Om2[i];
        for (int i = 0; i < 9; i++) V[i] = R[i];
    } else {
        double sn, cs;
        pq_sincos(theta, sn, cs);
        const double th2 = theta * theta;
        double A, B, Cc;
        if constexpr (kWave) {
            const int c = __lane_id() % 3;
            const double num = c == 0 ? sn : c == 1 ? (1.0 - cs) : (theta - sn);
            const double den = c == 0 ? theta : c == 1 ? th2 : (th2 * theta);
            const double q = num / den;
            A = rl_d(q, 0); B = rl_d(q, 1); Cc = rl_d(q, 2);
        } else {
            A = sn / theta; B = (1.0 - cs) / th2; Cc = (theta - sn) / (th2 * theta);
        }
        for (int i = 0; i < 9; i++) {
            const double I = i % 4 == 0 ? 1.0 : 0.0;
            R[i] = (I + A * Om[i]) + B * Om2[i];
            V[i] = (I + B * Om[i]) + Cc * Om2[i];
        }
    }
    Se3 s;
    pq_from_R(R, s);
    for (int i = 0; i < 3; i++) s.t[i] = (V[i * 3] * u[3] + V[i * 3 + 1] * u[4]) + V[i * 3 + 2] * u[5];
    pq_normalize<kWave>(s);
    return s;
}

__device__ Se3 pq_from_Tcw(const float* T)
{
    double R[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i * 3 + j] = (double)T[i * 4 + j];
    Se3 s;
    pq_from_R(R, s);
    for (int i = 0; i < 3; i++) s.t[i] = (double)T[i * 4 + 3];
    pq_normalize(s);
    return s;
}

__device__ void pq_to_Tcw(const Se3& s, float* T)
{
    const double tx = 2.0 * s.x, ty = 2.0 * s.y, tz = 2.0 * s.z;
    const double twx = tx * s.w, twy = ty * s.w, twz = tz * s.w;
    const double txx = tx * s.x, txy = ty * s.x, txz = tz * s.x;
    const double tyy = ty * s.y, tyz = tz * s.y, tzz = tz * s.z;
    const double R[9] = {1.0 - (tyy + tzz), txy - twz, txz + twy,
                         txy + twz, 1.0 - (txx + tzz), tyz - twx,
                         txz - twy, tyz + twx, 1.0 - (txx + tyy)};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[i * 4 + j] = (float)R[i * 3 + j];
        T[i * 4 + 3] = (float)s.t[i];
    }
    T[12] = 0.f; T[13] = 0.f; T[14] = 0.f; T[15] = 1.f;
}

struct PoseCam { double fx, fy, cx, cy, bf; };

// error, raw chi2 and (J != nullptr) the error Jacobian of one edge at pose s
__device__ __forceinline__ double pq_edge_eval(const PoseCam& cm, const Se3& s, const PEdge& E, double e[3], double* J)
{
    double p[3];
    pq_rotate(s, E.X, p);
    for (int k = 0; k < 3; k++) p[k] = p[k] + s.t[k];
    if (!E.stereo) {
        const double u = (p[0] / p[2]) * cm.fx + cm.cx, v = (p[1] / p[2]) * cm.fy + cm.cy;
        e[0] = E.obs[0] - u; e[1] = E.obs[1] - v; e[2] = 0.0;
    } else {
        const float invzf = 1.0f / (float)p[2];
        const double u = (p[0] * (double)invzf) * cm.fx + cm.cx, v = (p[1] * (double)invzf) * cm.fy + cm.cy;
        const double ur = u - cm.bf * (double)invzf;
        e[0] = E.obs[0] - u; e[1] = E.obs[1] - v; e[2] = E.obs[2] - ur;
    }
    if (J) {
        const double x = p[0], y = p[1], invz = 1.0 / p[2], invz_2 = invz * invz;
        J[0] = ((x * y) * invz_2) * cm.fx;
        J[1] = -(1.0 + ((x * x) * invz_2)) * cm.fx;
        J[2] = (y * invz) * cm.fx;
        J[3] = -invz * cm.fx;
        J[4] = 0.0;
        J[5] = (x * invz_2) * cm.fx;
        J[6] = (1.0 + ((y * y) * invz_2)) * cm.fy;
        J[7] = -((x * y) * invz_2) * cm.fy;
        J[8] = -(x * invz) * cm.fy;
        J[9] = 0.0;
        J[10] = -invz * cm.fy;
        J[11] = (y * invz_2) * cm.fy;
        if (E.stereo) {
            J[12] = J[0] - (cm.bf * y) * invz_2;
            J[13] = J[1] + (cm.bf * x) * invz_2;
            J[14] = J[2];
            J[15] = J[3];
            J[16] = 0.0;
            J[17] = J[5] - cm.bf * invz_2;
        }
    }
    double c = e[0] * (E.w * e[0]) + e[1] * (E.w * e[1]);
    if (E.stereo) c = c + e[2] * (E.w * e[2]);
    return c;
}

__device__ __forceinline__ void pq_huber(double e2, double delta, double& r0, double& r1)
{
    const double dsqr = delta * delta;
    if (e2 <= dsqr) { r0 = e2; r1 = 1.0; }
    else {
        const double sq = sqrt(e2);
        r0 = (2.0 * sq) * delta - dsqr;
        r1 = delta / sq;
    }
}

// pow(2*rho - 1, 3) of g2o's LM update, as the oracle's pq_cube: the exact double-double cube
// rounded once (the correctly rounded value glibc's pow returns)
__device__ inline double pq_cube(double t)
{
    const double h = t * t, l = __builtin_fma(t, t, -h);
    const double h2 = h * t, l2 = __builtin_fma(h, t, -h2);
    return h2 + __builtin_fma(l, t, l2);
}

// Index of H(a, b), a <= b, in the 21 upper-triangle terms of buildSystem's order (a outer).
__host__ __device__ constexpr int pq_hu(int a, int b) { return a * 6 - (a * (a - 1)) / 2 + (b - a); }

// LDLT solve of (H + lambda I) x = b with H given by its 21 upper-triangle terms hu (LDS) and b by
// bv (LDS); the same operations in the same order as a dense copy Hl = H, Hl(j, j) += lambda
// (the oracle's pq_solve6).  L is kept packed (15 terms) so thread 0 holds ~40 doubles, not
// three 6x6 matrices: the kernel then fits 128 VGPRs and two workgroups share a CU.
__device__ bool pq_solve6(const double* hu, double lambda, const double* bv, double x[6])
{
    double L[15], d[6], y[6];
#define PQ_L(i, j) L[((i) * ((i) - 1)) / 2 + (j)]       // i > j
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double v = hu[pq_hu(j, j)] + lambda;
#pragma unroll
        for (int k = 0; k < j; k++) v = v - (PQ_L(j, k) * PQ_L(j, k)) * d[k];
        if (!(v > 0.0)) return false;
        d[j] = v;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            double w = hu[pq_hu(j, i)];
#pragma unroll
            for (int k = 0; k < j; k++) w = w - (PQ_L(i, k) * PQ_L(j, k)) * d[k];
            PQ_L(i, j) = w / d[j];
        }
    }
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double v = bv[i];
#pragma unroll
        for (int k = 0; k < i; k++) v = v - PQ_L(i, k) * y[k];
        y[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] = y[i] / d[i];
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double v = y[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) v = v - PQ_L(k, i) * x[k];
        x[i] = v;
    }
#undef PQ_L
    return true;
}

// pq_solve6 with the rows on lanes (all 64 lanes of one wave call it; lane i < 6 holds row i of L,
// the others compute a copy of row 5 that is never read).  Column j of the LDL^T: lane i forms
// hu(j, i) - sum_k (L(i,k) L(j,k)) d_k in the oracle's k order (lane j's value is d_j, plus
// lambda on the diagonal), and ONE division serves every row below j; the forward substitution
// runs by columns (lane i subtracts L(i,k) y_k for k = 0, 1, .. in order), the y_i / d_i
// divisions are one, and the back substitution -- whose row order (k increasing) has to be kept --
// runs on uniform values.  Row j's values reach the other lanes by v_readlane (j is a constant).
// Same operations on the same operands as pq_solve6, so x is bit-identical; x is uniform.
__device__ bool pq_solve6_wave(const double* hu, double lambda, const double* bv, double x[6])
{
    const int lane = __lane_id();
    const int i = lane < 6 ? lane : 5;
    double Lr[6];                          // Lr[k] = L(i, k), k < i (lane i's row)
    double d[6];                           // uniform pivots
    double dl = 1.0;                       // lane i's own pivot d_i
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const int ii = i > j ? i : j;      // lanes above row j recompute row j (unused)
        double v = hu[pq_hu(j, ii)];
        if (ii == j) v = v + lambda;
#pragma unroll
        for (int k = 0; k < j; k++) v = v - (Lr[k] * rl_d(Lr[k], j)) * d[k];
        const double dj = rl_d(v, j);
        if (!(dj > 0.0)) return false;
        d[j] = dj;
        if (i == j) dl = v;
        Lr[j] = v / dj;                    // L(i, j) on lanes i > j
    }
    // forward substitution by columns; lane i's y_i is final when column i is reached
    double yv = bv[i], ymine = 0.0;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        if (i == k) ymine = yv;
        const double yk = rl_d(yv, k);
        if (k < 5 && i > k) yv = yv - Lr[k] * yk;
    }
    const double yd = ymine / dl;          // y_i / d_i on lane i
    double y[6], Lu[6][6];
#pragma unroll
    for (int k = 0; k < 6; k++) y[k] = rl_d(yd, k);
#pragma unroll
    for (int a = 0; a < 6; a++)
#pragma unroll
        for (int k = a + 1; k < 6; k++) Lu[k][a] = rl_d(Lr[a], k);     // L(k, a)
#pragma unroll
    for (int a = 5; a >= 0; a--) {
        double v = y[a];
#pragma unroll
        for (int k = a + 1; k < 6; k++) v = v - Lu[k][a] * x[k];
        x[a] = v;
    }
    return true;
}

// Reduction staging, per wave: wave w holds threads 64w .. 64w + 63, i.e. the whole of runs 2w and
// 2w + 1, so each wave sums its own two runs with no workgroup barrier.  The values go through a
// wave-private LDS area kRC at a time (lane l at slot l + l / 32 of a kWRow-double row: the two runs
// 33 doubles apart), lane (k, c) of the wave sums run c of value k; one barrier publishes the 8 run
// sums of every value: two workgroup barriers per reduction instead of three (0.5 % on config D's
// step; kRC = 27, 57 KB).  Smaller chunks cut the LDS (kRC = 9: 22 KB per frame), so more frames'
// workgroups would fit a CU, but every variant that used that measured slower (profiles/r05/s22).
#ifndef COEB_POSE_RCHUNK
#define COEB_POSE_RCHUNK 27
#endif
constexpr int kRC = COEB_POSE_RCHUNK;
constexpr int kWRow = 66;

// Trials per round after the first of an iteration (see k_pose): g2o's inner loop retries a
// rejected step with lambda *= ni, ni *= 2 from the same saved estimate, so the trials that follow
// a rejection depend only on that lambda sequence and can be solved and scored together.
#ifndef COEB_POSE_TB
#define COEB_POSE_TB 4
#endif
constexpr int kTB = COEB_POSE_TB;
static_assert(kTB >= 1 && kTB <= kPT / 64, "one wave per trial of a round");
#ifndef COEB_POSE_T1
#define COEB_POSE_T1 1         // trials in an iteration's first round (speculative beyond 1)
#endif
constexpr int kT1 = COEB_POSE_T1;
static_assert(kT1 >= 1 && kT1 <= kTB, "first-round trials");

struct PoseTrial {
    Se3 s;                 // exp(x) * saved
    double x[6], lam;      // step and its lambda
    int ok;                // the LDLT succeeded
};

struct PoseLds {
    Se3 s;                 // current estimate (broadcast)
    Se3 last;              // estimate of the last chi2 evaluation (the classification's errors)
    double wpart[kPT / 64][kRC][kWRow];   // per-wave staging of kRC values (block_reduce)
    double run[28][8];     // 32-lane run sums
    double out[28];        // reduced
    double hb[27];         // this iteration's 21 Hessian + 6 gradient terms (thread 0's system)
    PoseTrial tr[kTB];     // this round's trials
    double lam, ni;        // lambda and ni at the round's first trial
    double rho;
    int qmax, stop, nbad[4], accepted;
};

__device__ __forceinline__ void pose_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// block-wide canonical reduction of nv <= NV per-thread partials (uniform call): each run of 32
// threads summed in thread order, then the 8 run sums in order (the oracle's pq_reduce)
template <int NV>
__device__ void block_reduce(PoseLds& L, const double (&v)[NV], int nv)
{
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double* wp = &L.wpart[wv][0][0];
#pragma unroll
    for (int k0 = 0; k0 < NV; k0 += kRC) {
        if (k0 < nv) {
#pragma unroll
            for (int k = 0; k < kRC; k++)
                if (k0 + k < NV && k0 + k < nv) wp[k * kWRow + lane + (lane >> 5)] = v[k0 + k];
            pose_wave_sync();
            if (lane < 2 * min(kRC, nv - k0)) {
                const int k = lane >> 1, c = lane & 1;
                const double* r = wp + k * kWRow + 33 * c;
                double p = 0.0;
#pragma unroll 8
                for (int l = 0; l < 32; l++) p = p + r[l];       // threads 64 wv + 32 c + l in order
                L.run[k0 + k][2 * wv + c] = p;
            }
            pose_wave_sync();                                   // the next chunk reuses wp
        }
    }
    __syncthreads();
    if (tid < nv) {
        double t = L.run[tid][0];
        for (int c = 1; c < 8; c++) t = t + L.run[tid][c];
        L.out[tid] = t;
    }
    __syncthreads();
}

// Edge storage of one thread: edges e = tid + kPT * j.  EPT > 0 keeps them in registers
// (records, chi2, active bits; every pass then runs without global loads), EPT == 0 reads the
// global scratch arrays (frames with more than kPT * EPT keypoints).  Both visit a thread's
// edges in increasing e, so the per-thread partial sums -- and the results -- are the same.
template <int EPT>
struct EdgeSet {
    static constexpr int R = EPT > 0 ? EPT : 1;
    PoseEdgeRec rec[R];
    uint32_t act;
};

__device__ __forceinline__ PEdge edge_of(const PoseEdgeRec& r)
{
    PEdge E;
    E.X[0] = (double)r.x; E.X[1] = (double)r.y; E.X[2] = (double)r.z;
    E.obs[0] = (double)r.u; E.obs[1] = (double)r.v; E.obs[2] = r.stereo ? (double)r.ur : 0.0;
    E.w = (double)r.w;
    E.stereo = r.stereo;
    return E;
}

// Runs the body over this thread's edges in increasing e with `rec` (the edge record) and `act`
// (its active flag; the body may change it) in scope.
#define COEB_FOR_EDGES(ES, ...)                                                                   \
    if constexpr (EPT > 0) {                                                                        \
        _Pragma("unroll") for (int j_ = 0; j_ < EPT; j_++) {                                        \
            const int e = threadIdx.x + j_ * kPT;                                                   \
            if (e < ne) {                                                                           \
                const PoseEdgeRec& rec = ES.rec[j_];                                                \
                bool act = (ES.act >> j_) & 1u;                                                     \
                __VA_ARGS__;                                                                        \
                ES.act = (ES.act & ~(1u << j_)) | ((act ? 1u : 0u) << j_);                          \
            }                                                                                       \
        }                                                                                           \
    } else {                                                                                        \
        for (int e = threadIdx.x; e < ne; e += kPT) {                                               \
            const PoseEdgeRec rec = b.edges[(int64_t)f * b.stride + e];                             \
            bool act = b.active[(int64_t)f * b.stride + e] != 0;                                    \
            __VA_ARGS__;                                                                            \
            b.active[(int64_t)f * b.stride + e] = act ? 1 : 0;                                      \
        }                                                                                           \
    }

// computeActiveErrors + activeRobustChi2 at each of the T poses (LDS): robust chi2 sums of the
// active edges -> L.out[0..T).  Each sum runs over the thread's edges in increasing e and is
// reduced in the canonical order, so pose t's sum is what a pass at that pose alone gives.
template <int EPT>
__device__ void active_chi2(PoseLds& L, const PoseBufs& b, const PoseCam& cm, int f, int ne, bool robust,
                            const double delta[2], EdgeSet<EPT>& ES, const Se3* poses, int pstride, int T)
{
    double acc[kTB];
#pragma unroll
    for (int t = 0; t < kTB; t++) {
        acc[t] = 0.0;
        if (t < T) {
            const Se3 s = *reinterpret_cast<const Se3*>(reinterpret_cast<const uint8_t*>(poses) + t * pstride);
            double a = 0.0;
            COEB_FOR_EDGES(ES, {
                if (act) {
                    const PEdge E = edge_of(rec);
                    double er[3];
                    const double c = pq_edge_eval(cm, s, E, er, nullptr);
                    double r = c, r1;
                    if (robust) pq_huber(c, delta[E.stereo], r, r1);
                    a += r;
                }
            })
            acc[t] = a;
        }
    }
    block_reduce(L, acc, T);
}

// phase clocks of thread 0 (diagnostic, COEB_POSE_TIMING): [0] chi2 passes, [1] build passes,
// [2] thread-0 solve + exp + bookkeeping, [3] classification, [4] total, [5] iterations, [6] trials
// Compiled in only with -DCOEB_POSE_CLOCK=1 (tools/_pose_timing.py's builds): the runtime checks of
// b.timing alone cost 19 SGPR and 2 VGPR spills in k_pose<5> (3.91 -> 3.85 ms per config-D step
// without them, profiles/r05/s34).
#ifndef COEB_POSE_CLOCK
#define COEB_POSE_CLOCK 0
#endif
#if COEB_POSE_CLOCK
#define PT_ON(b) ((b).timing)
#else
#define PT_ON(b) false
#endif
#define PT_MARK(var) long long var = PT_ON(b) ? (long long)clock64() : 0
#define PT_ADD(slot, t0) do { if (PT_ON(b) && threadIdx.x == 0) b.timing[(int64_t)blockIdx.x * 8 + (slot)] += (long long)clock64() - (t0); } while (0)
#define PT_INC(slot) do { if (PT_ON(b) && threadIdx.x == 0) b.timing[(int64_t)blockIdx.x * 8 + (slot)] += 1; } while (0)

#ifndef COEB_POSE_MINWG
#define COEB_POSE_MINWG 2      // launch bound: workgroups per CU the register budget must allow
#endif
#ifndef COEB_POSE_MINWG0
#define COEB_POSE_MINWG0 2     // the same for k_pose<0> (edges in global scratch)
#endif
template <int EPT>
__global__ __launch_bounds__(kPT, EPT == 0 ? COEB_POSE_MINWG0 : COEB_POSE_MINWG) void k_pose(PoseBufs b, PoseCam cm)
{
    PT_MARK(t_all);
    EdgeSet<EPT> ES;
    ES.act = 0;
    __shared__ PoseLds L;
    __shared__ int s_ne, s_cnt[4];
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = b.n[f];
    const int64_t base = (int64_t)f * b.stride;
    // ---- edges: keypoints with a MapPoint, in keypoint order (block-ordered compaction) ----
    if (tid == 0) s_ne = 0;
    __syncthreads();
    for (int i0 = 0; i0 < n; i0 += kPT) {
        const int i = i0 + tid;
        const bool has = i < n && b.has_mp[base + i];
        const uint64_t m = __ballot(has);
        if (lane == 0) s_cnt[wv] = __popcll(m);
        __syncthreads();
        int pre = s_ne;
        for (int w = 0; w < wv; w++) pre += s_cnt[w];
        if (has) {
            const int e = pre + __popcll(m & ((1ull << lane) - 1ull));
            const KpRec k = reinterpret_cast<const KpRec*>(b.kps)[base + i];
            PoseEdgeRec r;
            r.x = b.xw[(base + i) * 3 + 0]; r.y = b.xw[(base + i) * 3 + 1]; r.z = b.xw[(base + i) * 3 + 2];
            r.u = k.x; r.v = k.y;
            const float ur = b.ur[base + i];
            r.stereo = !(ur < 0);                                  // Optimizer.cc:287
            r.ur = ur;
            r.w = b.inv_sigma2[k.octave];
            r.kp = i;
            b.edges[base + e] = r;
            b.active[base + e] = 1;
            b.outlier[base + i] = 0;
        }
        __syncthreads();
        if (tid == 0) s_ne += s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        __syncthreads();
    }
    const int ne = s_ne;
    if constexpr (EPT > 0) {                                       // own edges into registers
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            const int e = tid + j * kPT;
            if (e < ne) { ES.rec[j] = b.edges[base + e]; ES.act |= 1u << j; }
        }
    }
    float* Tcw = b.Tcw + (int64_t)f * 16;
    if (ne < 3) {                                                  // :361-362
        if (tid == 0) b.result[f] = 0;
        return;
    }
    const double delta[2] = {(double)(float)sqrt(5.991), (double)(float)sqrt(7.815)};
    const double chi2th[2] = {(double)5.991f, (double)7.815f};
    Se3 s0;
    if (tid == 0) s0 = pq_from_Tcw(Tcw);
    int nBad = 0;
    for (int it = 0; it < 4; it++) {                                // its < 4 (Optimizer.cc:364)
        if (tid == 0) L.s = s0;                                    // setEstimate(toSE3Quat(mTcw))
        __syncthreads();
        const bool robust = it < 3;
        // ---- optimize(10): OptimizationAlgorithmLevenberg::solve per iteration ----
        double lambda = 0.0, ni = 2.0;                             // thread 0's copies
        double currentChi = 0.0;
        bool fresh = false;        // the last trial was accepted: errors and chi2 are already at L.s
        for (int iter = 0; iter < 10; iter++) {
            // computeActiveErrors + activeRobustChi2 at the current estimate.  After an accepted
            // trial the estimate is that trial's, so the chi2 computed for it (= tempChi, thread 0)
            // is exactly what this pass would produce: skip it.
            PT_INC(5);
            PT_MARK(t_c0);
            if (!fresh) {
                active_chi2<EPT>(L, b, cm, f, ne, robust, delta, ES, &L.s, 0, 1);
                currentChi = L.out[0];
            }
            PT_ADD(0, t_c0);
            PT_MARK(t_b0);
            // buildSystem
            double acc[27];
            for (int k = 0; k < 27; k++) acc[k] = 0.0;
            {
                const Se3 s = L.s;
                COEB_FOR_EDGES(ES, {
                    if (act) {
                    const PEdge E = edge_of(rec);
                    double er[3], J[18];
                    const double c = pq_edge_eval(cm, s, E, er, J);
                    double r0, rho1 = 1.0;
                    if (robust) pq_huber(c, delta[E.stereo], r0, rho1);
                    const double wgt = rho1 * E.w;
                    int k = 0;
                    for (int a = 0; a < 6; a++)
                        for (int bb = a; bb < 6; bb++) {
                            double c2 = J[a] * J[bb] + J[6 + a] * J[6 + bb];
                            if (E.stereo) c2 = c2 + J[12 + a] * J[12 + bb];
                            acc[k++] += wgt * c2;
                        }
                    for (int a = 0; a < 6; a++) {
                        double c1 = J[a] * er[0] + J[6 + a] * er[1];
                        if (E.stereo) c1 = c1 + J[12 + a] * er[2];
                        acc[21 + a] += -(wgt * c1);
                    }
                    }
                })
            }
            block_reduce(L, acc, 27);
            PT_ADD(1, t_b0);
            PT_MARK(t_s0);
            if (tid == 0) {
                for (int k = 0; k < 27; k++) L.hb[k] = L.out[k];
                if (iter == 0) {
                    double m = 0.0;
                    for (int j = 0; j < 6; j++) m = fmax(fabs(L.out[pq_hu(j, j)]), m);
                    lambda = 1e-5 * m;
                    ni = 2.0;
                }
                L.qmax = 0;
            }
            // The trial loop (do { ... } while (rho < 0 && qmax < 10)) in rounds of T trials: the
            // first round of an iteration tries one step; after a rejection, a round solves and
            // scores the next T steps of the rejection sequence (lambda_t+1 = lambda_t * ni_t,
            // ni_t+1 = 2 ni_t, all from the same saved estimate) at once -- wave t solves step t,
            // one chi2 pass scores all T, and thread 0 then walks them in order exactly as
            // the sequential loop would, stopping where it stops.  Steps past that point were never
            // taken: their results are dropped.
            int qmax = 0;                                          // uniform copy of L.qmax
            for (;;) {
                const int T = qmax == 0 ? kT1 : min(kTB, 10 - qmax);
                if (tid == 0) { L.lam = lambda; L.ni = ni; }
                __syncthreads();
                if (wv < T) {
                    // trial wv of the round on wave wv (kTB <= the 4 waves): its LDL^T solve on the
                    // wave's lanes, the SE3 exponential and product as uniform values
                    double lam = L.lam, nu = L.ni;
                    for (int k = 0; k < wv; k++) { lam = lam * nu; nu = nu * 2.0; }
                    double x[6];
                    for (int j = 0; j < 6; j++) x[j] = 0.0;
                    const int ok2 = pq_solve6_wave(L.hb, lam, L.hb + 21, x) ? 1 : 0;
                    if (!ok2) for (int j = 0; j < 6; j++) x[j] = 0.0;
                    const Se3 saved = L.s;
                    const Se3 up = pq_exp<true>(x);
                    const Se3 ns = pq_mul<true>(up, saved);
                    if (lane == 0) {
                        PoseTrial& tr = L.tr[wv];
                        tr.s = ns;
                        for (int j = 0; j < 6; j++) tr.x[j] = x[j];
                        tr.lam = lam;
                        tr.ok = ok2;
                    }
                }
                __syncthreads();
                PT_ADD(2, t_s0);
                PT_INC(6);
                PT_MARK(t_c1);
                active_chi2<EPT>(L, b, cm, f, ne, robust, delta, ES, &L.tr[0].s, (int)sizeof(PoseTrial), T);
                PT_ADD(0, t_c1);
                t_s0 = PT_ON(b) ? (long long)clock64() : 0;
                if (tid == 0) {
                    int q = L.qmax, stop = 0;
                    double rho = 0.0;
                    for (int t = 0; t < T; t++) {
                        const PoseTrial& tr = L.tr[t];
                        double tempChi = L.out[t];
                        if (!tr.ok) tempChi = DBL_MAX;
                        double scale = 0.0;
                        for (int j = 0; j < 6; j++) scale = scale + tr.x[j] * (lambda * tr.x[j] + L.hb[21 + j]);
                        scale = scale + 1e-3;   // g2o OptimizationAlgorithmLevenberg::solve: "make sure it's non-zero"
                        rho = (currentChi - tempChi) / scale;
                        L.last = tr.s;          // the errors computeActiveErrors left behind
                        if (rho > 0 && isfinite(tempChi)) {
                            double alpha = 1.0 - pq_cube(2.0 * rho - 1.0);
                            alpha = fmin(alpha, 2.0 / 3.0);
                            const double sf = fmax(1.0 / 3.0, alpha);
                            lambda = lambda * sf;
                            ni = 2.0;
                            currentChi = tempChi;
                            L.s = tr.s;
                            L.accepted = 1;
                        } else {
                            lambda = lambda * ni;
                            ni = ni * 2.0;
                            L.accepted = 0;
                        }
                        q = q + 1;
                        if (!(rho < 0 && q < 10)) { stop = 1; break; }
                    }
                    L.qmax = q;
                    L.rho = rho;
                    L.stop = stop;
                }
                __syncthreads();
                qmax = L.qmax;
                const int stop = L.stop;
                // no barrier after these reads: thread 0 next writes L.qmax / L.stop only after
                // barriers every thread reaches after reading them
                if (stop) break;
            }
            const double rho = L.rho;
            PT_ADD(2, t_s0);
            fresh = L.accepted != 0;
            if (qmax == 10 || rho == 0) break;                     // Terminate
        }
        // ---- classification (Optimizer.cc:381-437): the chi2 of an active edge is the one its
        //      last computeActiveErrors left (at L.last, possibly a rejected trial's estimate), an
        //      inactive edge's is computed at the final estimate (e->computeError()) ----
        PT_MARK(t_k0);
        const Se3 s = L.s, sl = L.last;
        int bad = 0;
        COEB_FOR_EDGES(ES, {
            const PEdge E = edge_of(rec);
            double er[3];
            const double c = pq_edge_eval(cm, act ? sl : s, E, er, nullptr);
            const int kp = rec.kp;
            if (c > chi2th[E.stereo]) { b.outlier[base + kp] = 1; act = false; bad++; }
            else { b.outlier[base + kp] = 0; act = true; }
        })
        for (int off = 32; off >= 1; off >>= 1) bad += __shfl_xor(bad, off, 64);
        if (lane == 0) L.nbad[wv] = bad;
        __syncthreads();
        nBad = (L.nbad[0] + L.nbad[1]) + (L.nbad[2] + L.nbad[3]);
        __syncthreads();
        PT_ADD(3, t_k0);
        if (ne < 10) break;                                        // optimizer.edges().size() < 10
    }
    if (tid == 0) {
        pq_to_Tcw(L.s, Tcw);
        b.result[f] = ne - nBad;
    }
    PT_ADD(4, t_all);
}

// ================================ k_track_prep ================================
// Tracking::TrackWithMotionModel between SearchByProjection and PoseOptimization
// (src/Tracking.cc:947-964): CurrentFrame.mvpMapPoints[i] = the LastFrame MapPoint the
// matcher assigned to keypoint i (its position: the LastFrame snapshot k_prep wrote), and
// `if (nmatches < 20) return false` (:954-958) -- such a frame reaches the optimiser with no
// keypoints, so k_pose leaves its pose at the prediction and reports 0.
__global__ __launch_bounds__(kPT) void k_track_prep(TrackPrepBufs t)
{
    const int f = blockIdx.y + 1;
    const int i = blockIdx.x * kPT + threadIdx.x;
    const bool go = t.nmatch[f] >= t.min_matches;
    const int n = t.counts[f];
    if (blockIdx.x == 0) {
        if (threadIdx.x < 16) t.Tout[(int64_t)f * 16 + threadIdx.x] = t.Tin[(int64_t)f * 16 + threadIdx.x];
        if (threadIdx.x == 16) t.n[f] = go ? n : 0;
        if (f == 1 && threadIdx.x >= 32 && threadIdx.x < 32 + COEB_MAXL) t.isg_out[threadIdx.x - 32] = t.isg[threadIdx.x - 32];
    }
    if (!go || i >= n) return;
    const int64_t o = (int64_t)f * t.stride + i;
    reinterpret_cast<KpRec*>(t.kps_out)[o] = reinterpret_cast<const KpRec*>(t.kps_in)[o];   // k_pose's own copies
    t.ur_out[o] = t.ur_in[o];
    const int m = t.match[o];
    t.has[o] = m >= 0 ? 1 : 0;
    if (m >= 0) {
        const int64_t q = ((int64_t)(f - 1) * t.stride + m) * 3;
        t.xw[3 * o + 0] = t.last_xw[q + 0];
        t.xw[3 * o + 1] = t.last_xw[q + 1];
        t.xw[3 * o + 2] = t.last_xw[q + 2];
    }
}

}  // namespace

int launch_track_prep(const TrackPrepBufs& t, int F, hipStream_t s, ProfileHook* prof)
{
    if (F < 2) return 0;
    prof_begin(prof, "k_track_prep", s);
    hipLaunchKernelGGL(k_track_prep, dim3((t.stride + kPT - 1) / kPT, F - 1), dim3(kPT), 0, s, t);
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_pose(const PoseBufs& b, int F, double fx, double fy, double cx, double cy, double bf, hipStream_t s,
                ProfileHook* prof)
{
    PoseCam cm{fx, fy, cx, cy, bf};
    prof_begin(prof, "k_pose", s);
    // edges per thread by the keypoint stride: registers up to 9 x 256 edges, else global scratch
    int ept = (b.stride + kPT - 1) / kPT;
    if (ept <= 5) hipLaunchKernelGGL(k_pose<5>, dim3(F), dim3(kPT), 0, s, b, cm);
    else if (ept <= 9) hipLaunchKernelGGL(k_pose<9>, dim3(F), dim3(kPT), 0, s, b, cm);
    else hipLaunchKernelGGL(k_pose<0>, dim3(F), dim3(kPT), 0, s, b, cm);
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
