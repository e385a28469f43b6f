// coeb_extract.hip -- CDNA4 (gfx950) kernels for ORBextractor::operator()
// (src/ORBextractor.cc:1088-1342).  Integer/bitwise work: no MFMA.  Built with
// -ffp-contract=off; every fused multiply-add is an explicit __builtin_fmaf placed where the
// reference binary fused (SURVEY.md s7 hard part 3).
//
// Pipeline for F frames (one launch each, all on the context stream):
//   k_dynmask    dynamic-object rectangles + area flag           (ORBextractor.cc:1101-1195)
//   k_pyr_level  cascaded INTER_LINEAR pyramid, level l from l-1  (:1344-1367)
//   k_blur_rows  7x7 sigma-2 Gaussian of every level, 16x8 tiles  (:1317-1318)
//   k_fast       per 30-px cell FAST-9/16 + NMS + iniTh/minTh     (:811-850)
//   k_octree     per (frame, level) DistributeOctTree emulation   (:546-769, 852-890, 1204-1207)
//   k_describe   IC_Angle + rBRIEF + output assembly              (:80-156, 902-903, 1291-1337)
#include <type_traits>
#include <cmath>
#include <hip/hip_runtime.h>

#include "coeb_internal.hpp"

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ int lane_id() { return __lane_id(); }
// Wave index in the workgroup as a wave-uniform (scalar) value: derived from threadIdx the
// compiler treats it as divergent, and everything indexed by it (cell descriptors, level
// geometry) becomes per-lane vector loads and VGPR arithmetic.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
// orders one wave's LDS accesses (the compiler and the LDS queue), no workgroup barrier
__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));   // native vector: stays in VGPRs

__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

__device__ __forceinline__ int wave_sum(int v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Exclusive block scan of one int per thread (256 threads).  Returns prefix; *total = sum.
// All threads must call it.  sbuf: >= kWaves+1 ints of LDS.
template <int NW = kWaves>
__device__ __forceinline__ int block_scan_excl(int v, int* total, int* sbuf)
{
    const int lane = lane_id(), w = threadIdx.x >> 6;
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sbuf[w] = x;
    __syncthreads();
    int base = 0, tot = 0;
    for (int i = 0; i < NW; i++) {
        int t = sbuf[i];
        if (i < w) base += t;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// Exclusive block scan for a 0/1 predicate via ballots (cheaper).
template <int NW = kWaves>
__device__ __forceinline__ int block_scan_flag(bool pred, int* total, int* sbuf)
{
    const int w = threadIdx.x >> 6;
    uint64_t m = __ballot(pred);
    int pre = __popcll(m & lanemask_lt());
    if (lane_id() == 0) sbuf[w] = __popcll(m);
    __syncthreads();
    int base = 0, tot = 0;
    for (int i = 0; i < NW; i++) {
        int t = sbuf[i];
        if (i < w) base += t;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return base + pre;
}

__device__ __forceinline__ const uint8_t* level_ptr(const Plan* P, const ExtractBufs& b, int f, int l)
{
    if (l == 0) return b.gray + (int64_t)f * P->W * P->H;
    return b.pyr + (int64_t)f * P->pyr_stride + P->lv[l].pyr_off;
}

// CheckMovingKeyPoints / _finall mask lookup (ORBextractor.cc:1391-1397, 1426-1440)
__device__ __forceinline__ bool masked_out(const DynMask& m, float px, float py, float scale, int W, int H)
{
    float sx = px * scale, sy = py * scale;
    if (sx >= (float)(W - 1)) sx = (float)(W - 1);
    if (sy >= (float)(H - 1)) sy = (float)(H - 1);
    const int ix = (int)sx, iy = (int)sy;
    for (int r = 0; r < m.nrect; r++)
        if (ix >= m.rect[r][0] && ix < m.rect[r][2] && iy >= m.rect[r][1] && iy < m.rect[r][3]) return true;
    return false;
}

// ================================ k_dynmask ================================
// One thread per frame: the literal box-layer loop (tiny, <= 16 boxes x |T_M| points).
__global__ void k_dynmask(ExtractBufs b, int F, int W, int H)
{
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    DynMask m;
    m.area_flag = 0;
    m.nrect = 0;
    float area = 0.f;
    const int b0 = b.box_off ? b.box_off[f] : 0, b1 = b.box_off ? b.box_off[f + 1] : 0;
    const float* tm = b.tm;
    int t0 = b.tm_off ? b.tm_off[f] : 0, t1 = b.tm_off ? b.tm_off[f + 1] : 0;
    if (b.tmd) {                                  // T_M left on the device by ProcessMovingObject
        tm = b.tmd + (int64_t)f * b.tmd_cap * 2;
        t0 = 0;
        t1 = min(max(b.ntmd[f], 0), b.tmd_cap);
    }
    for (int bi = b0; bi < b1; bi++) {
        const float xmin = b.boxes[4 * bi + 0], ymin = b.boxes[4 * bi + 1];
        const float xmax = b.boxes[4 * bi + 2], ymax = b.boxes[4 * bi + 3];
        const int rx = (int)xmin, ry = (int)ymin, rw = (int)(xmax - xmin), rh = (int)(ymax - ymin);
        const float area_box = (xmax - xmin) * (ymax - ymin);
        bool mark = false;
        unsigned long long nin = 0;
        for (int t = t0; t < t1; t++) {
            const int px = (int)tm[2 * t], py = (int)tm[2 * t + 1];
            const bool in = px >= 0 && px < W && py >= 0 && py < H && px >= rx && px < rx + rw &&
                            py >= ry && py < ry + rh;
            if (in) nin++;
            if ((float)(nin * 10000ull) > area_box) { mark = true; break; }   // layer 1 (:1145)
        }
        const int bf = b.blurf ? b.blurf[bi] : 0;
        if (mark || (bf == 1 && nin > 0)) {                                       // layer 2 (:1168)
            area = area + area_box;
            const int x0 = max((int)xmin, 0), x1 = min((int)xmax, W);
            const int y0 = max((int)ymin, 0), y1 = min((int)ymax, H);
            if (x1 > x0 && y1 > y0) {
                if (m.nrect < COEB_MAXBOX) {
                    m.rect[m.nrect][0] = x0; m.rect[m.nrect][1] = y0;
                    m.rect[m.nrect][2] = x1; m.rect[m.nrect][3] = y1;
                    m.nrect++;
                } else {
                    atomicOr(b.err, 1);
                }
            }
        }
    }
    m.area_flag = area > 200000.f ? 1 : 0;                                      // :1192
    b.dyn[f] = m;
}

typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ us2 as_us2(uint32_t v) { return __builtin_bit_cast(us2, v); }
__device__ __forceinline__ uint32_t as_u32(us2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ us2 pk2(int lo, int hi) { us2 r; r.x = (unsigned short)lo; r.y = (unsigned short)hi; return r; }

// ================================ k_pyr_level ================================
// cv::resize INTER_LINEAR 8U, canonical rounding.  Four consecutive output
// pixels per thread (one 32-bit store); the <= 12 source bytes they need from each of the
// two source rows come from three aligned 32-bit loads.  64 x 4 threads cover 256 x 4 outputs.
__device__ __forceinline__ int byte_of(uint32_t w0, uint32_t w1, uint32_t w2, int o)
{
    const uint32_t w = o < 4 ? w0 : (o < 8 ? w1 : w2);
    return (int)((w >> ((o & 3) * 8)) & 0xFFu);
}

// VResizeLinearVec_32s8u: ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2.
// Coefficients are in [0, 2048] and h <= 255 * 2048, so h >> 4 <= 32640 (the 16-bit
// saturations of the SIMD code never trigger).  The horizontal pass produces g = h << 4 (its
// coefficients pre-shifted; g < 2^24), so ((h >> 4) * b) >> 16 = mul_hi_u24(g & ~0xFF, b << 8):
// one AND and one full-rate 24-bit multiply-high per term.  Each term is <= (32656 * b) >> 16
// and b0 + b1 <= 2049 (coefficients rounded separately), so the sum is <= 1021 and the result
// <= 255: the final saturate_cast never clips.
__device__ __forceinline__ uint32_t vresize_g(uint32_t g0, uint32_t g1, uint32_t b0s, uint32_t b1s)
{
    const uint32_t m0 = __umulhi(g0 & 0xFFFF00u, b0s & 0xFFFFFFu);   // v_mul_hi_u32_u24
    const uint32_t m1 = __umulhi(g1 & 0xFFFF00u, b1s & 0xFFFFFFu);
    return (m0 + m1 + 2u) >> 2;
}

// Output tile 128 x 32 per workgroup; the source rows/columns it touches (<= 32*scale+2 rows,
// <= 128*scale+2 columns) are staged in LDS -- 16-byte loads, each thread issuing all of its
// loads before its first LDS store -- then each thread produces 4 x 4 outputs (one 32-bit
// store per output row).  The LDS tile (pitch tsw, tsh rows) is sized per level from the
// level's scale (pyr_tile_lds): 7.2 KB at scale 1.2 instead of a fixed 20.7 KB for scale 2, so
// 12 workgroups fit a CU instead of 7.
constexpr int PT_W = 128, PT_H = 32;

// First column of VResizeLinear's scalar tail for a row of w outputs (oracle oc_resize_simd_end):
// the SSE2 loops run 16 columns while x <= w - 16, then 4 while x < w - 4.
// LDS source tile of a 128 x 32 output tile resized from sw x sh to dw x dh: columns
// xofs[ox] & ~15 .. xofs[ox + 127] + 1 (<= ceil(127 * sw / dw) + 2 + 15 bytes), rows
// yofs[oy] .. yofs[oy + 31] + 1 (<= ceil(31 * sh / dh) + 2), with a margin of one chunk / row.
void pyr_tile_lds(int sw, int sh, int dw, int dh, int* tsw, int* tsh)
{
    const int span = (int)std::ceil(127.0 * sw / dw) + 2 + 15;
    *tsw = 16 * ((span + 15) / 16 + 1);
    *tsh = (int)std::ceil(31.0 * sh / dh) + 4;
}

int resize_simd_end(int w)
{
    int x = w >= 16 ? (w / 16) * 16 : 0;
    while (x < w - 4) x += 4;
    return x;
}

// Columns >= xs (VResizeLinear's scalar tail on x86-64: the SIMD loops stop at xs, DESIGN.md
// s2.1) round exactly: (h0*b0 + h1*b1 + 2^21) >> 22 (FixedPtCast<int, uchar, 22>).
__device__ __forceinline__ uint32_t vresize_exact(uint32_t g0, uint32_t g1, uint32_t b0s, uint32_t b1s)
{
    const uint32_t v = __umul24(g0 >> 4, b0s >> 8) + __umul24(g1 >> 4, b1s >> 8) + (1u << 21);   // < 2^31
    return min(v >> 22, 255u);
}

__global__ __launch_bounds__(kThreads) void k_pyr_level(const uint8_t* __restrict__ src, int64_t src_fs, int sp,
                                                        int sw, int sh, uint8_t* __restrict__ dst, int64_t dst_fs,
                                                        int dp, int dw, int dh, const int* __restrict__ tab, int xmax,
                                                        int xs, int tsw, int tsh)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t s_src[];   // tsh x tsw
    const int f = blockIdx.z;
    const int ox = blockIdx.x * PT_W, oy = blockIdx.y * PT_H;
    const int* xofs = tab;
    const int* alpha = tab + dw;
    const int* yofs = tab + 2 * dw;
    const int* beta = tab + 2 * dw + dh;
    const int ex = min(ox + PT_W, dw) - 1, ey = min(oy + PT_H, dh) - 1;
    const int sx1 = min(xofs[ex] + 1, sw - 1);
    const int sy0 = max(yofs[oy], 0), sy1 = min(max(yofs[ey] + 1, 0), sh - 1);
    const int nrows = sy1 - sy0 + 1;
    const uint8_t* S = src + (int64_t)f * src_fs;
    const int tid = threadIdx.x;
    int sx0;                                      // source column of LDS tile column 0
    const bool vec = ((sp | (int)reinterpret_cast<uintptr_t>(S)) & 15) == 0;
    if (vec && ((sx1 - (xofs[ox] & ~15)) >> 4) + 1 <= tsw / 16 && nrows <= tsh) {
        sx0 = xofs[ox] & ~15;
        const int nch = ((sx1 - sx0) >> 4) + 1;   // 16-byte chunks per row
        const int rstep = kThreads / nch;         // rows per pass; thread = (row, chunk)
        const int r = tid / nch, k = tid - r * nch;
        if (r < rstep) {
            const uint4* base = reinterpret_cast<const uint4*>(S + (int64_t)sy0 * sp + sx0) + k;
            const int pw = sp >> 4;
            uint4 q0 = base[min(r, nrows - 1) * pw];
            uint4 q1 = base[min(r + rstep, nrows - 1) * pw];
            uint4 q2 = base[min(r + 2 * rstep, nrows - 1) * pw];
            if (r < nrows) *reinterpret_cast<uint4*>(s_src + r * tsw + 16 * k) = q0;
            if (r + rstep < nrows) *reinterpret_cast<uint4*>(s_src + (r + rstep) * tsw + 16 * k) = q1;
            if (r + 2 * rstep < nrows) *reinterpret_cast<uint4*>(s_src + (r + 2 * rstep) * tsw + 16 * k) = q2;
            for (int rr = r + 3 * rstep; rr < nrows; rr += rstep)     // tall tiles (scale > 1.5)
                *reinterpret_cast<uint4*>(s_src + rr * tsw + 16 * k) = base[rr * pw];
        }
    } else if ((sp & 3) == 0) {
        sx0 = xofs[ox] & ~3;
        const int nwords = (sx1 - sx0) / 4 + 1;
        for (int i = tid; i < nwords * nrows; i += kThreads) {
            const int r = i / nwords, k = i - r * nwords;
            *reinterpret_cast<uint32_t*>(s_src + r * tsw + 4 * k) =
                *reinterpret_cast<const uint32_t*>(S + (int64_t)(sy0 + r) * sp + sx0 + 4 * k);
        }
    } else {
        sx0 = xofs[ox];
        const int nb = sx1 - sx0 + 1;
        for (int i = tid; i < nb * nrows; i += kThreads) {
            const int r = i / nb, k = i - r * nb;
            s_src[r * tsw + k] = S[(int64_t)(sy0 + r) * sp + sx0 + k];
        }
    }
    __syncthreads();
    const int cx = ox + (threadIdx.x & 31) * 4, cy = oy + (threadIdx.x >> 5) * 4;
    if (cx >= dw) return;
    const int nk = min(4, dw - cx);
    int lx[4], a0[4], a1[4];                      // horizontal coefficients << 4 (pass gives g = h << 4)
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int d = min(cx + k, dw - 1);
        const int sx = xofs[d];
        const int a = alpha[d];
        a0[k] = ((int)(short)(a & 0xFFFF)) << 4;
        a1[k] = (a >> 16) << 4;
        if (d >= xmax) { a0[k] = 2048 << 4; a1[k] = 0; }   // HResizeLinear tail: S[sx]*ONE
        lx[k] = sx - sx0;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int dy = cy + r;
        if (dy >= dh) break;
        const int q0 = yofs[dy];
        const int r0 = (q0 >= 0 ? (q0 < sh ? q0 : sh - 1) : 0) - sy0;
        const int r1 = (q0 + 1 >= 0 ? (q0 + 1 < sh ? q0 + 1 : sh - 1) : 0) - sy0;
        const int bb = beta[dy];
        const uint32_t b0s = (uint32_t)((int)(short)(bb & 0xFFFF)) << 8, b1s = (uint32_t)(bb >> 16) << 8;
        const uint8_t* R0 = s_src + __mul24(r0, tsw);
        const uint8_t* R1 = s_src + __mul24(r1, tsw);
        uint32_t word = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int g0 = __mul24((int)R0[lx[k]], a0[k]) + __mul24((int)R0[lx[k] + 1], a1[k]);
            const int g1 = __mul24((int)R1[lx[k]], a0[k]) + __mul24((int)R1[lx[k] + 1], a1[k]);
            const uint32_t v = cx + k < xs ? vresize_g((uint32_t)g0, (uint32_t)g1, b0s, b1s)
                                           : vresize_exact((uint32_t)g0, (uint32_t)g1, b0s, b1s);
            word |= v << (8 * k);
        }
        uint8_t* D = dst + (int64_t)f * dst_fs + (int64_t)dy * dp + cx;
        if (nk == 4 && (dp & 3) == 0) *reinterpret_cast<uint32_t*>(D) = word;
        else for (int k = 0; k < nk; k++) D[k] = (uint8_t)(word >> (8 * k));
    }
}

// k_pyr_rows: the same resize for the common case (scale <= 2, 4-byte aligned source rows),
// shaped for VALU issue, which bounds the extraction step:
//   * a wave owns 128 output columns (2 per lane) of PR_ROWS output rows; the rows are wave-
//     uniform, so yofs / beta / the row clamps / the row addresses are scalar work;
//   * each lane loads its 8-byte window of a source row (two dword loads from the row's SGPR
//     base, the second clamped inside the pitch) for all of its rows before the first use;
//   * horizontal pass as one v_dot2_u32_u16 per output and source row: a v_perm with a per-column
//     selector lifts (S[sx], S[sx+1]) into a u16 pair, dotted with the packed (a0, a1);
//   * vertical pass on h: SIMD columns ((h0 >> 4) * b0 >> 16) + ((h1 >> 4) *
//     b1 >> 16) + 2 >> 2, each term v_mul_hi_u32_u24(h & ~15, b << 12) (16 * 4096 = 2^16; both
//     operands < 2^24); tail columns (>= xs) (h0*b0 + h1*b1 + 2^21) >> 22.
// About 10.5 VALU lane-operations per output pixel against ~38 for k_pyr_level's byte form.
constexpr int PR_ROWS = 8, PR_COLS = 128;

__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }

// The output rows of a k_pyr_rows wave; kTail: the wave holds columns >= xs (exact rounding);
// kEdge: the wave holds the level's last column (per-lane store guards).  Row descriptors
// (yrow: clamped source-row offsets, beta, the output row offset) are one scalar 16-byte load
// each, and loads / stores are buffer operations with the row offset as the scalar soffset, so a
// row costs no 64-bit address arithmetic and no exec-mask juggling in interior waves.
template <bool kTail, bool kEdge>
__device__ __forceinline__ void pyr_rows_out(const uint32_t (&w)[PR_ROWS][4], const uint32_t (&sel)[2],
                                             const uint32_t (&coef)[2], const int4* __restrict__ yrow,
                                             __amdgpu_buffer_rsrc_t rd, int oy, int dh, uint32_t cx, int dw, int xs)
{
#pragma unroll
    for (int r = 0; r < PR_ROWS; r++) {
        const int dy = oy + r;
        if (dy >= dh) break;
        const int4 yr = yrow[dy];
        const uint32_t bb = (uint32_t)yr.z;
        const uint32_t b0 = bb & 0xFFFFu, b1 = bb >> 16;
        const uint32_t b0s = (bb << 12) & 0xFFF000u, b1s = (bb >> 4) & 0xFFF000u;
        uint32_t v[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const uint32_t h0 = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(w[r][1], w[r][0], sel[k])),
                                                       as_us2(coef[k]), 0u, false);
            const uint32_t h1 = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(w[r][3], w[r][2], sel[k])),
                                                       as_us2(coef[k]), 0u, false);
            v[k] = (__umulhi(h0 & 0xFFFF0u, b0s) + __umulhi(h1 & 0xFFFF0u, b1s) + 2u) >> 2;
            if (kTail && (int)cx + k >= xs)       // h < 2^20, b <= 2048: 24-bit multiplies
                v[k] = min((__umul24(h0, b0) + __umul24(h1, b1) + (1u << 21)) >> 22, 255u);
        }
        const uint32_t pr = v[0] | (v[1] << 8);
        if (!kEdge) {
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)pr, rd, cx, yr.w, 0);
        } else {
            if ((int)cx + 1 < dw) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)pr, rd, cx, yr.w, 0);
            else if ((int)cx < dw) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)pr, rd, cx, yr.w, 0);
        }
    }
}

__global__ __launch_bounds__(kThreads) void k_pyr_rows(const uint8_t* __restrict__ src, int64_t src_fs, int sp,
                                                       int sh, uint8_t* __restrict__ dst, int64_t dst_fs, int dp,
                                                       int dw, int dh, const int* __restrict__ tab, int xmax, int xs,
                                                       const int4* __restrict__ yrow)
{
    const int f = blockIdx.z;
    const int oy = (blockIdx.y * kWaves + wave_id()) * PR_ROWS;
    if (oy >= dh) return;
    const int lane = lane_id();
    const int ox = blockIdx.x * PR_COLS;
    const uint32_t cx = (uint32_t)(ox + 2 * lane);
    const int* xofs = tab;
    const int* alpha = tab + dw;
    uint32_t sel[2], coef[2];
    const int d0 = min((int)cx, dw - 1);
    const uint32_t wb = (uint32_t)(xofs[d0] & ~3);                 // the lane's window: bytes wb .. wb + 7
    const uint32_t wb1 = (uint32_t)min((int)wb + 4, sp - 4);      // (the second word stays inside the pitch)
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int d = min((int)cx + k, dw - 1);
        const int o = xofs[d] - (int)wb;          // <= 5 for scale <= 2 (make_plan's rows_ok)
        const int a = alpha[d];
        const uint32_t a0 = d >= xmax ? 2048u : (uint32_t)(a & 0xFFFF), a1 = d >= xmax ? 0u : (uint32_t)a >> 16;
        coef[k] = a0 | (a1 << 16);
        sel[k] = (uint32_t)o | 0x0c00u | ((uint32_t)(o + 1) << 16) | 0x0c000000u;
    }
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(src + (int64_t)f * src_fs), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc((void*)(dst + (int64_t)f * dst_fs), 0, 0x7fffffff, 0x00020000);
    uint32_t w[PR_ROWS][4];
    // (round 6: dealing the grid to the XCDs in contiguous runs (block_xy's mapping over
    // (strip, band, frame)) cuts this kernel's fetch 1.88x -> 1.02x its reads -- round-robin puts
    // neighbouring strips, which share 2-3 source lines per row, on different L2s -- but runs
    // 0.583 vs 0.568 ms per 7-launch pyramid, the step unchanged; a frame-major grid (a frame's
    // blocks on one XCD) fetched 1.06x and ran 0.600 ms.  The pyramid is not bound by these bytes;
    // profiles/r06/s17..s19.  Reusing the source row that consecutive output rows share, behind wave-uniform
    // branches, ran 0.669 vs 0.569 ms per 7-launch pyramid: the loads no longer issue back to
    // back; profiles/r06/s3)
#pragma unroll
    for (int r = 0; r < PR_ROWS; r++) {
        const int4 yr = yrow[min(oy + r, dh - 1)];
        w[r][0] = __builtin_amdgcn_raw_buffer_load_b32(rs, wb, yr.x, 0);
        w[r][1] = __builtin_amdgcn_raw_buffer_load_b32(rs, wb1, yr.x, 0);
        w[r][2] = __builtin_amdgcn_raw_buffer_load_b32(rs, wb, yr.y, 0);
        w[r][3] = __builtin_amdgcn_raw_buffer_load_b32(rs, wb1, yr.y, 0);
    }
    (void)dp;
    const bool edge = ox + PR_COLS > dw - 1;
    if (ox + PR_COLS > xs) {
        if (edge) pyr_rows_out<true, true>(w, sel, coef, yrow, rd, oy, dh, cx, dw, xs);
        else pyr_rows_out<true, false>(w, sel, coef, yrow, rd, oy, dh, cx, dw, xs);
    } else {
        if (edge) pyr_rows_out<false, true>(w, sel, coef, yrow, rd, oy, dh, cx, dw, xs);
        else pyr_rows_out<false, false>(w, sel, coef, yrow, rd, oy, dh, cx, dw, xs);
    }
}

// ================================ k_blur ================================
// GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101), Q8 kernel k (symmetric, sum 256), result
// (sum_ij k_i k_j p_ij + 2^15) >> 16.  OpenCV's horizontal-then-vertical
// order has no intermediate rounding, so the same integer is computed vertical-first:
//   * vertical 7-tap on packed u16 column pairs (sums <= 255*256 fit 16 bits): 7 v_pk ops
//     per 2 columns, the 7 source rows slide through registers (row loop unrolled by 7, so
//     the ring never moves);
//   * horizontal 7-tap as four v_dot2_u32_u16 per output on the packed vertical sums, the
//     3-column halo coming from the neighbouring lanes by DPP row shifts;
//   * the rounded result is byte 2 of the 24-bit accumulator: v_perm packs 4 outputs.
// Work item = one wave: 4 row groups of 16 lanes; a group covers 64 source columns (4 per
// lane) of which lanes 1..14 produce (56 output columns), and one band of rows.
constexpr int kBlurCols = 56;

__device__ __forceinline__ int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - p - 2;
    return p;
}

struct BlurWork {
    int L;
    int item0, item1;              // this launch's wave items [item0, item1)
    int item_off[COEB_MAXL + 1];   // wave items per level (prefix)
    int nstrips[COEB_MAXL];        // 56-column strips
    int bh[COEB_MAXL];             // rows per band (4 bands per item)
    int nquads[COEB_MAXL];         // k_blur_rows: groups of 4 adjacent strips per level
    int brows;                     // k_blur_rows: rows per band
};


// Logical (x, y) block of a 2-D grid with each XCD given a contiguous run of logical blocks.
// Blocks are observed to be dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, Workgroup
// dispatch & XCD placement): physical block p lands on XCD p % 8.  Mapping XCD x's k-th block
// to logical block x*q + min(x, r) + k (q, r = n / 8, n % 8) keeps the blocks of one frame
// (y) on one L2, so the patches / ROIs they share are fetched into one L2 instead of eight.
// Performance only: any placement gives the same results.  Measured (256 frames): k_describe
// 0.227 -> 0.215 ms, k_blur 0.178 -> 0.169 ms; k_fast 0.320 -> 0.324 ms, so k_fast keeps the
// round-robin order (its cells share only 3-px borders).
template <bool kRemap = true>
__device__ __forceinline__ int2 block_xy()
{
    const int gx = gridDim.x;
    if (!kRemap) return make_int2(blockIdx.x, blockIdx.y);
    const int n = gx * gridDim.y, p = blockIdx.x + gx * blockIdx.y;
    const int q = n >> 3, r = n & 7, x = p & 7, k = p >> 3;
    const int lg = x * q + min(x, r) + k;
    return make_int2(lg % gx, lg / gx);
}

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t v)   // lane i <- lane i-1 (16-lane rows)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_shl1(uint32_t v)   // lane i <- lane i+1 (16-lane rows)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x101, 0xf, 0xf, false);
}

// k_blur_rows: a wave item is 4 ADJACENT 56-column strips (one per 16-lane group) of one band of
// brows rows, so every row index, its REFLECT_101 and the row
// pointers are scalar (SGPR base + the lane's constant column offset, no per-row 64-bit address
// VALU), the band halo is 6 rows per brows instead of per 16, and the next 7-row block's loads
// are issued before the current block is filtered.
__device__ __forceinline__ int reflect_row(int r, int h)
{
    // selects, not min/max chains: uniform min3/max3 has no scalar form, and the compiler then
    // moves the whole row offset into VGPRs
    int rr = r < 0 ? -r : r;
    rr = rr >= h ? 2 * h - 2 - rr : rr;
    return rr < 0 ? 0 : rr;
}

constexpr int kBlurQuad = 4 * kBlurCols;     // columns of one k_blur_rows wave item (14 tiles of 16)
static_assert(kBlurQuad % 16 == 0, "a wave item must cover whole 16-column tiles");

__global__ __launch_bounds__(kThreads) void k_blur_rows(const Plan* __restrict__ P, ExtractBufs b, BlurWork bw)
{
    // 8 output rows of the wave item, transposed through LDS into whole 128-B tile lines
    __shared__ __attribute__((aligned(16))) uint8_t s_tile[kWaves][8 * kBlurQuad];
    const int2 bxy = block_xy();
    const int f = bxy.y;
    const int item = bw.item0 + bxy.x * kWaves + wave_id();
    if (item >= bw.item1) return;
    int l = 0;
    while (l + 1 < bw.L && item >= bw.item_off[l + 1]) l++;
    const int it = item - bw.item_off[l];
    const int nq = bw.nquads[l];
    const int quad = it % nq, band = it / nq;
    const LevelGeom& g = P->lv[l];
    const int w = g.w, h = g.h, sp = g.pitch, dp = g.bpitch;
    const int lane = lane_id(), grp = lane >> 4, gl = lane & 15;
    const int y0 = band * bw.brows, y1 = min(h, y0 + bw.brows);
    const int x = (quad * 4 + grp) * kBlurCols - 4 + gl * 4;
    const bool produce = gl >= 1 && gl <= 14 && x < w;
    const int xbase = quad * kBlurQuad;                            // first column of the item (16-aligned)
    uint8_t* tl = s_tile[wave_id()];
    // Every lane loads one dword at column a and picks its 4 columns' bytes with the u16-pair
    // perms below: a = x inside the level; at the edges a is moved so that the REFLECT_101
    // columns reflect101(x + q) all fall in [a, a + 3] (w >= 5), so no lane takes a byte path.
    int cq[4];
#pragma unroll
    for (int q = 0; q < 4; q++) cq[q] = reflect101(min(x + q, w + 2), w);
    const int a = min(min(min(cq[0], cq[1]), min(cq[2], cq[3])), w - 4);
    const uint32_t sel0 = 0x0c000c00u | (uint32_t)(cq[0] - a) | ((uint32_t)(cq[1] - a) << 16);
    const uint32_t sel1 = 0x0c000c00u | (uint32_t)(cq[2] - a) | ((uint32_t)(cq[3] - a) << 16);
    // rows through buffer resources: the row offset is a scalar (soffset), the lane's column
    // the only vector operand
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)level_ptr(P, b, f, l), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc((void*)(b.blur + (int64_t)f * P->blur_stride + g.blur_off), 0, 0x7fffffff,
                                          0x00020000);
    const int k0 = P->gauss[0], k1 = P->gauss[1], k2 = P->gauss[2], k3 = P->gauss[3];
    const us2 K0 = pk2(k0, k0), K1 = pk2(k1, k1), K2 = pk2(k2, k2), K3 = pk2(k3, k3);
    const us2 W_l01_0 = pk2(0, k0), W_l23_0 = pk2(k1, k2), W_c01_0 = pk2(k3, k2), W_c23_0 = pk2(k1, k0);
    const us2 W_l23_1 = pk2(k0, k1), W_c01_1 = pk2(k2, k3), W_c23_1 = pk2(k2, k1), W_r01_1 = pk2(k0, 0);
    const us2 W_l23_2 = pk2(0, k0), W_c01_2 = pk2(k1, k2), W_c23_2 = pk2(k3, k2), W_r01_2 = pk2(k1, k0);
    const us2 W_c01_3 = pk2(k0, k1), W_c23_3 = pk2(k2, k3), W_r01_3 = pk2(k2, k1), W_r23_3 = pk2(k0, 0);
    const uint32_t rnd = 1u << 15;
    const int n_rows = (y1 - y0) + 6;          // source rows y0-3 .. y1+2
    auto load_row = [&](int i) -> uint32_t {   // source row y0 - 3 + i (uniform), REFLECT_101
        const int so = __builtin_amdgcn_readfirstlane(reflect_row(y0 - 3 + i, h) * sp);
        return __builtin_amdgcn_raw_buffer_load_b32(rs, a, so, 0);
    };
    uint32_t nxt[7];
#pragma unroll
    for (int ph = 0; ph < 7; ph++) nxt[ph] = load_row(ph);
    uint32_t R0[7], R1[7];
    for (int i0 = 0; i0 < n_rows; i0 += 7) {
        uint32_t raw[7];
#pragma unroll
        for (int ph = 0; ph < 7; ph++) raw[ph] = nxt[ph];
        if (i0 + 7 < n_rows) {
#pragma unroll
            for (int ph = 0; ph < 7; ph++) nxt[ph] = load_row(i0 + 7 + ph);
        }
#pragma unroll
        for (int ph = 0; ph < 7; ph++) {
            const int i = i0 + ph;
            if (i >= n_rows) break;
            R0[ph] = __builtin_amdgcn_perm(0u, raw[ph], sel0);
            R1[ph] = __builtin_amdgcn_perm(0u, raw[ph], sel1);
            if (i < 6) continue;
            const int s0 = (ph + 1) % 7, s1 = (ph + 2) % 7, s2 = (ph + 3) % 7, s3 = (ph + 4) % 7,
                      s4 = (ph + 5) % 7, s5 = (ph + 6) % 7, s6 = ph;
            const us2 v01 = K3 * as_us2(R0[s3]) + K2 * (as_us2(R0[s2]) + as_us2(R0[s4])) +
                            K1 * (as_us2(R0[s1]) + as_us2(R0[s5])) + K0 * (as_us2(R0[s0]) + as_us2(R0[s6]));
            const us2 v23 = K3 * as_us2(R1[s3]) + K2 * (as_us2(R1[s2]) + as_us2(R1[s4])) +
                            K1 * (as_us2(R1[s1]) + as_us2(R1[s5])) + K0 * (as_us2(R1[s0]) + as_us2(R1[s6]));
            const uint32_t V01 = as_u32(v01), V23 = as_u32(v23);
            const us2 L01 = as_us2(dpp_shr1(V01)), L23 = as_us2(dpp_shr1(V23));
            const us2 R01 = as_us2(dpp_shl1(V01)), R23 = as_us2(dpp_shl1(V23));
            uint32_t a0 = __builtin_amdgcn_udot2(L01, W_l01_0, rnd, false);
            a0 = __builtin_amdgcn_udot2(L23, W_l23_0, a0, false);
            a0 = __builtin_amdgcn_udot2(v01, W_c01_0, a0, false);
            a0 = __builtin_amdgcn_udot2(v23, W_c23_0, a0, false);
            uint32_t a1 = __builtin_amdgcn_udot2(L23, W_l23_1, rnd, false);
            a1 = __builtin_amdgcn_udot2(v01, W_c01_1, a1, false);
            a1 = __builtin_amdgcn_udot2(v23, W_c23_1, a1, false);
            a1 = __builtin_amdgcn_udot2(R01, W_r01_1, a1, false);
            uint32_t a2 = __builtin_amdgcn_udot2(L23, W_l23_2, rnd, false);
            a2 = __builtin_amdgcn_udot2(v01, W_c01_2, a2, false);
            a2 = __builtin_amdgcn_udot2(v23, W_c23_2, a2, false);
            a2 = __builtin_amdgcn_udot2(R01, W_r01_2, a2, false);
            uint32_t a3 = __builtin_amdgcn_udot2(v01, W_c01_3, rnd, false);
            a3 = __builtin_amdgcn_udot2(v23, W_c23_3, a3, false);
            a3 = __builtin_amdgcn_udot2(R01, W_r01_3, a3, false);
            a3 = __builtin_amdgcn_udot2(R23, W_r23_3, a3, false);
            const int y = y0 - 6 + i;                                  // uniform
            // row y into the item's LDS rows; after every 8th row (tile rows start at multiples of 8:
            // y0 is) the 8 rows leave as whole tile lines, 16 B per lane, consecutive lanes
            // consecutive bytes (a tile row's tiles are adjacent), 1.75 KiB in two instructions.
            // Storing each row straight into the tiles (14 partial lines per instruction) took
            // k_blur_rows 0.487 -> 0.829 ms per 1025-frame launch (profiles/r05/s4).
            if (produce) {
                const uint32_t p01 = __builtin_amdgcn_perm(a1, a0, 0x0c0c0602u);
                const uint32_t p23 = __builtin_amdgcn_perm(a3, a2, 0x06020c0cu);
                *reinterpret_cast<uint32_t*>(tl + (y & 7) * kBlurQuad + (x - xbase)) = p01 | p23;
            }
            if ((y & 7) == 7 || y == y1 - 1) {
                wave_sync_lds();
                const int so = __builtin_amdgcn_readfirstlane((int)blur_tile_off(0, y & ~7, dp));
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const int c = lane + 64 * k;                           // chunk: tile c >> 3, row c & 7
                    if (c < kBlurQuad / 2 && xbase + 16 * (c >> 3) < dp) {
                        const u32x4 v = *reinterpret_cast<const u32x4*>(tl + (c & 7) * kBlurQuad + 16 * (c >> 3));
                        __builtin_amdgcn_raw_buffer_store_b128(v, rd, (xbase >> 4) * 128 + 16 * c, so, 0);
                    }
                }
                wave_sync_lds();
            }
        }
    }
}

// ================================ k_fast ================================
// One workgroup per (FAST cell, frame).  The cell ROI (<= 64 x 64) is staged in LDS; each
// detection pixel gets its corner strength M = max over the 16 nine-pixel arcs of
// min(|v - ring|) taken with the arc's sign.  For threshold t: corner <=> M > t, and
// OpenCV's cornerScore<16> = M - 1 (derivation: DESIGN.md s4.2).  Per-cell NMS then
// compares against neighbours' scores (0 outside the detection window), exactly as
// FAST_t's 3-row buffers do; an empty cell at iniThFAST is redone at minThFAST (:834-838).
// LDS pointers kept in their address space (a generic pointer would become flat loads)
typedef const __attribute__((address_space(3))) uint8_t* lds_cu8;
typedef const __attribute__((address_space(3))) uint32_t* lds_cu32;

__device__ __forceinline__ void ring16(const uint8_t* c, int st, int p[16])
{
    p[0] = c[3 * st];      p[1] = c[3 * st + 1];  p[2] = c[2 * st + 2];  p[3] = c[st + 3];
    p[4] = c[3];           p[5] = c[-st + 3];     p[6] = c[-2 * st + 2]; p[7] = c[-3 * st + 1];
    p[8] = c[-3 * st];     p[9] = c[-3 * st - 1]; p[10] = c[-2 * st - 2]; p[11] = c[-st - 3];
    p[12] = c[-3];         p[13] = c[st - 3];     p[14] = c[2 * st - 2]; p[15] = c[3 * st - 1];
}

// Exact corner strength M = max over the 16 nine-pixel arcs of min(v - ring) (dark) or
// min(ring - v) (bright); OpenCV cornerScore<16> = M - 1 for a corner.
// Arc minima by doubling: m2 -> m4 -> m8 -> m9.
__device__ __forceinline__ int corner_strength(const uint8_t* c, int st)
{
    int p[16];
    ring16(c, st, p);
    const int v = c[0];
    int d[16];
#pragma unroll
    for (int k = 0; k < 16; k++) d[k] = v - p[k];
    // 9-arc minima (dark) and maxima (bright) from 3-arcs: arc9(k) = arc3(k), arc3(k+3), arc3(k+6)
    int t[16];
#pragma unroll
    for (int k = 0; k < 16; k++) t[k] = min(min(d[k], d[(k + 1) & 15]), d[(k + 2) & 15]);
    int A = -1000;
#pragma unroll
    for (int k = 0; k < 16; k++) A = max(A, min(min(t[k], t[(k + 3) & 15]), t[(k + 6) & 15]));
#pragma unroll
    for (int k = 0; k < 16; k++) t[k] = max(max(d[k], d[(k + 1) & 15]), d[(k + 2) & 15]);
    int Bm = 1000;
#pragma unroll
    for (int k = 0; k < 16; k++) Bm = min(Bm, max(max(t[k], t[(k + 3) & 15]), t[(k + 6) & 15]));
    return max(A, -Bm);
}

// One wave per cell, four cells per workgroup, no workgroup barriers.
//  1. stage the cell ROI in the wave's LDS slab with aligned 32-bit loads (slab row starts at
//     the ROI's x0 & 3, so words are stored unshifted);
//  2. OpenCV's pre-test at minThFAST (ring pairs 0/8, 2/10, 4/12, 6/14 -- a necessary
//     condition of a corner) on every detection pixel; survivors (a few %) are compacted
//     (ballot) into a per-wave list, keeping row-major order;
//  3. exact strength M of the survivors; M > minThFAST <=> corner at minThFAST.  Corners go to
//     Ms (all other pixels keep M = 0: not a corner at any threshold the reference uses) and,
//     still in row-major order, to the corner list;
//  4. NMS over the corner list at iniThFAST (fallback minThFAST if the cell came out empty,
//     :834-838) with ordered (ballot) stores of the kept keys.  A cell with more corners than
//     the list holds walks the whole window instead.
constexpr int kFastRowBytes = 72;          // >= 1 + 64 + 7 (slab byte = ROI column + 1): any ROI up to 64 wide
constexpr int kFastRowBytesM = 96;         // ROIs up to 46 wide: pixels in bytes 0..47, M in bytes 48..95
// (24 dwords: the four rows a half-wave's pre-test reads land on disjoint banks, (a/4) mod 32)
constexpr int kFastGuard = 16;             // bytes before each wave's slab (unaligned staging spill)
constexpr int kFastEnt = 128;              // pre-test entries (u16: first pixel's offset / 4 | survivor mask << 12)
constexpr int kFastSurv = 4 * 64 + 8;      // survivors of one 64-entry expansion, + the odd-count pad
constexpr int kFastCorners = 256;          // corner list (more corners: NMS walks the whole window)
constexpr int kFastLists = kFastSurv;      // u16 entries before the corner list
// entry offsets / 4 fit 12 bits: ROIs are at most 64 rows (coeb_capi.hip kRoiMax)
static_assert(kFastRowBytesM * 64 <= 4 * 4096 && kFastRowBytes * 64 <= 4 * 4096, "k_fast entry offset field");


// FAST_t's first rejection stage (features2d/fast.cpp): d = tab[p0]|tab[p8]; d &= tab[p2]|tab[p10];
// d &= tab[p4]|tab[p12]; d &= tab[p6]|tab[p14]; with tab = 1 (darker than v-t) / 2 (brighter).
__device__ __forceinline__ bool fast_pretest(const uint8_t* c, int st, int t)
{
    const int v = c[0];
    const int lo = v - t, hi = v + t;
    auto cls = [&](int x) { return (x < lo ? 1 : 0) | (x > hi ? 2 : 0); };
    int d = cls(c[3 * st]) | cls(c[-3 * st]);                 // p0 | p8
    d &= cls(c[2 * st + 2]) | cls(c[-2 * st - 2]);             // p2 | p10
    d &= cls(c[3]) | cls(c[-3]);                               // p4 | p12
    d &= cls(c[-2 * st + 2]) | cls(c[2 * st - 2]);             // p6 | p14
    return d != 0;
}

// The same pre-test for 4 adjacent detection pixels at once (one lane): c points at the first
// of them, 4-byte aligned in the slab.  Ring bytes are gathered by v_perm straight into
// packed u16 pairs; per pair, with d = min/max of the opposite ring pixels,
//   dark  survives <=> max over pairs of min(a, b) <  v - t   (some of each pair darker)
//   bright survives <=> min over pairs of max(a, b) >  v + t
// Returns a 4-bit survivor mask (bit q = pixel q).
__device__ __forceinline__ uint32_t win_lo(uint32_t a, uint32_t b, int s)   // bytes s, s+1 of a:b as u16 pair
{
    return __builtin_amdgcn_perm(b, a, 0x0c000c00u | (uint32_t)s | ((uint32_t)(s + 1) << 16));
}
__device__ __forceinline__ uint32_t win_hi(uint32_t a, uint32_t b, int s)   // bytes s+2, s+3
{
    return __builtin_amdgcn_perm(b, a, 0x0c000c00u | (uint32_t)(s + 2) | ((uint32_t)(s + 3) << 16));
}

__device__ __forceinline__ us2 pk_min(us2 a, us2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ us2 pk_max(us2 a, us2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ us2 pk_subs(us2 a, us2 b) { return __builtin_elementwise_sub_sat(a, b); }

// Three-input packed max / min of u16 pixel pairs (values <= 255) as v_pk_maximum3_f16 /
// v_pk_minimum3_f16: read as f16 the patterns are positive denormals, ordered like the integers
// (f16 denormals are not flushed), so one instruction replaces two v_pk_max/min_u16
__device__ __forceinline__ us2 pk_max3(us2 a, us2 b, us2 c)
{
    uint32_t r;
    asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(as_u32(a)), "v"(as_u32(b)), "v"(as_u32(c)));
    return as_us2(r);
}
__device__ __forceinline__ us2 pk_min3(us2 a, us2 b, us2 c)
{
    uint32_t r;
    asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(as_u32(a)), "v"(as_u32(b)), "v"(as_u32(c)));
    return as_us2(r);
}

__device__ __forceinline__ uint32_t pretest_half(us2 v, us2 p0, us2 p8, us2 p2, us2 p10, us2 p4, us2 p12, us2 p6,
                                                 us2 p14, us2 T)
{
    // dark survives <=> v - md > t, bright <=> mb - v > t: one threshold test of their maximum
    const us2 md = pk_max3(pk_min(p0, p8), pk_min(p2, p10), pk_max(pk_min(p4, p12), pk_min(p6, p14)));
    const us2 mb = pk_min3(pk_max(p0, p8), pk_max(p2, p10), pk_min(pk_max(p4, p12), pk_max(p6, p14)));
    return as_u32(pk_subs(pk_max(pk_subs(v, md), pk_subs(mb, v)), T));
}

// v_pk_maximum3_f16 / v_pk_minimum3_f16 on u16 patterns (see pk_max3) with the halves of the
// second (S1) and / or third (S2) operand swapped by op_sel
template <bool kMax, bool S1, bool S2>
__device__ __forceinline__ uint32_t pk3(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
#define COEB_PK3(OP, SEL) asm(OP " %0, %1, %2, %3" SEL : "=v"(r) : "v"(a), "v"(b), "v"(c))
    if constexpr (kMax) {
        if constexpr (!S1 && !S2) COEB_PK3("v_pk_maximum3_f16", "");
        else if constexpr (!S1 && S2) COEB_PK3("v_pk_maximum3_f16", " op_sel:[0,0,1] op_sel_hi:[1,1,0]");
        else if constexpr (S1 && !S2) COEB_PK3("v_pk_maximum3_f16", " op_sel:[0,1,0] op_sel_hi:[1,0,1]");
        else COEB_PK3("v_pk_maximum3_f16", " op_sel:[0,1,1] op_sel_hi:[1,0,0]");
    } else {
        if constexpr (!S1 && !S2) COEB_PK3("v_pk_minimum3_f16", "");
        else if constexpr (!S1 && S2) COEB_PK3("v_pk_minimum3_f16", " op_sel:[0,0,1] op_sel_hi:[1,1,0]");
        else if constexpr (S1 && !S2) COEB_PK3("v_pk_minimum3_f16", " op_sel:[0,1,0] op_sel_hi:[1,0,1]");
        else COEB_PK3("v_pk_minimum3_f16", " op_sel:[0,1,1] op_sel_hi:[1,0,0]");
    }
#undef COEB_PK3
    return r;
}

// max over the 16 circular nine-pixel arcs of the arc minimum, with ring positions k and k + 8
// in the two u16 halves of Q[k] (k < 8): three-input packed min / max over both halves at once
// (8 + 8 + 4 instructions instead of 16 + 16 + 8); the wrap-around operands are the swapped
// registers (op_sel)
__device__ __forceinline__ uint32_t arc_max_min_pk(const uint32_t Q[8])
{
    uint32_t M3[8], M9[8];
#pragma unroll
    for (int k = 0; k < 6; k++) M3[k] = pk3<false, false, false>(Q[k], Q[k + 1], Q[k + 2]);
    M3[6] = pk3<false, false, true>(Q[6], Q[7], Q[0]);     // (q6, q7, q8) | (q14, q15, q0)
    M3[7] = pk3<false, true, true>(Q[7], Q[0], Q[1]);      // (q7, q8, q9) | (q15, q0, q1)
    M9[0] = pk3<false, false, false>(M3[0], M3[3], M3[6]);
    M9[1] = pk3<false, false, false>(M3[1], M3[4], M3[7]);
#pragma unroll
    for (int k = 2; k < 5; k++) M9[k] = pk3<false, false, true>(M3[k], M3[k + 3], M3[k - 2]);
#pragma unroll
    for (int k = 5; k < 8; k++) M9[k] = pk3<false, true, true>(M3[k], M3[k - 5], M3[k - 2]);
    const uint32_t A = pk3<true, false, false>(M9[0], M9[1], M9[2]);
    const uint32_t B = pk3<true, false, false>(M9[3], M9[4], M9[5]);
    return pk3<true, false, false>(M9[6], M9[7], pk3<true, false, false>(A, B, A));
}

// The same M for a pre-test survivor, computing only the arc sign(s) that passed the pre-test at
// t (the four opposite pairs 0/8, 2/10, 4/12, 6/14).  Every nine-pixel arc holds one pixel of each
// opposite pair, so a sign whose pre-test fails has arc strength <= t: it can neither make the
// pixel a corner at t nor at any larger threshold, and M only matters where M > t.  Hence
//   dark passed:   M = max_k min_arc(v - p) = X - (255 - v),  X = max_k min_arc(255 - p)
//   bright passed: M = max_k min_arc(p - v) = X - v,          X = max_k min_arc(p)
// i.e. X over q = p ^ mask (mask = 255 for dark, 0 for bright) and M = X - (v ^ mask): one arc
// pass of min3/max3 instead of two.  A pixel passing both pre-tests (rare) takes the bright pass
// as well.  The base pointer sits at the lowest ring byte (p9 = -3 rows - 1 column), so all 17
// reads take positive immediate offsets (LDS offsets are unsigned).
// The ring bytes are loaded straight into u16 halves (Q[k] = p_k | p_{k+8} << 16) and the arc is
// taken by arc_max_min_pk.
template <int st>
__device__ __forceinline__ int corner_strength_pos2(const uint8_t* c, int t)
{
    lds_cu8 b = (lds_cu8)c - (3 * st + 1);
    asm volatile("" : "+v"(b));
    constexpr int o = 3 * st + 1;                          // c[x] = b[x + o]
    constexpr int off[16] = {o + 3 * st, o + 3 * st + 1, o + 2 * st + 2, o + st + 3, o + 3, o - st + 3, o - 2 * st + 2,
                             o - 3 * st + 1, 1, 0, o - 2 * st - 2, o - st - 3, o - 3, o + st - 3, o + 2 * st - 2,
                             o + 3 * st - 1};
    us2 Qv[8];
#pragma unroll
    for (int k = 0; k < 8; k++) { Qv[k].x = b[off[k]]; Qv[k].y = b[off[k + 8]]; }
    const int v = b[o];
    uint32_t Q[8];
#pragma unroll
    for (int k = 0; k < 8; k++) Q[k] = as_u32(Qv[k]);
    auto lo = [](uint32_t x) { return (int)(x & 0xFFFFu); };
    auto hi = [](uint32_t x) { return (int)(x >> 16); };
    const int md = max(max(min(lo(Q[0]), hi(Q[0])), min(lo(Q[2]), hi(Q[2]))),
                       max(min(lo(Q[4]), hi(Q[4])), min(lo(Q[6]), hi(Q[6]))));
    const int mb = min(min(max(lo(Q[0]), hi(Q[0])), max(lo(Q[2]), hi(Q[2]))),
                       min(max(lo(Q[4]), hi(Q[4])), max(lo(Q[6]), hi(Q[6]))));
    const bool dark = md < v - t, bright = mb > v + t;
    const uint32_t mask = dark ? 0x00FF00FFu : 0u;
    uint32_t Qx[8];
#pragma unroll
    for (int k = 0; k < 8; k++) Qx[k] = Q[k] ^ mask;
    const uint32_t X = arc_max_min_pk(Qx);
    int M = max(lo(X), hi(X)) - (v ^ (int)(mask & 0xFFu));
    if (__builtin_expect(__ballot(dark && bright) != 0, 0)) {
        if (dark && bright) {
            const uint32_t Y = arc_max_min_pk(Q);
            M = max(M, max(lo(Y), hi(Y)) - v);
        }
    }
    return M;
}

// Same test, raw packed results: pixel q survives iff 16-bit half q of (lo, hi) is nonzero.
template <int RB>
__device__ __forceinline__ void fast_pretest4_raw(const uint8_t* c, int t, uint32_t& lo, uint32_t& hi)
{
    constexpr int st = RB;
    // base at the lowest word read (row -3), so every read takes a positive immediate offset
    lds_cu32 w = (lds_cu32)(c - 3 * st);
    asm volatile("" : "+v"(w));
    constexpr int o = 3 * st / 4;            // word index of c
    const uint32_t a0 = w[o - 1], b0 = w[o], c0 = w[o + 1];
    const uint32_t ap = w[o + 2 * st / 4 - 1], bp = w[o + 2 * st / 4], cp = w[o + 2 * st / 4 + 1];
    const uint32_t am = w[o - 2 * st / 4 - 1], bm = w[o - 2 * st / 4], cm = w[o - 2 * st / 4 + 1];
    const uint32_t u3 = w[o + 3 * st / 4];
    const uint32_t d3 = w[0];
    const us2 T = pk2(t, t);
    lo = pretest_half(
        as_us2(__builtin_amdgcn_perm(0u, b0, 0x0c010c00u)), as_us2(__builtin_amdgcn_perm(0u, u3, 0x0c010c00u)),
        as_us2(__builtin_amdgcn_perm(0u, d3, 0x0c010c00u)), as_us2(win_lo(bp, cp, 2)), as_us2(win_lo(am, bm, 2)),
        as_us2(win_lo(b0, c0, 3)), as_us2(win_lo(a0, b0, 1)), as_us2(win_lo(bm, cm, 2)), as_us2(win_lo(ap, bp, 2)), T);
    hi = pretest_half(
        as_us2(__builtin_amdgcn_perm(0u, b0, 0x0c030c02u)), as_us2(__builtin_amdgcn_perm(0u, u3, 0x0c030c02u)),
        as_us2(__builtin_amdgcn_perm(0u, d3, 0x0c030c02u)), as_us2(win_hi(bp, cp, 2)), as_us2(win_hi(am, bm, 2)),
        as_us2(win_hi(b0, c0, 3)), as_us2(win_hi(a0, b0, 1)), as_us2(win_hi(bm, cm, 2)), as_us2(win_hi(ap, bp, 2)), T);
}

// M of the detection window (zero around it, for the NMS neighbours):
//  * RB = kFastRowBytesM: in the right half of the pixel slab's own rows, M of the pixel at slab
//    offset o at o + 45 (columns 48.., rows 2..rh-3), pitch RB;
//  * RB = kFastRowBytes: a compact slab of its own (pitch mp = window width + 2, one zero row /
//    column around the window): detection pixel (r, c) at (r + 1) * mp + c + 1.
// Either way 5.8-6.6 KB of LDS per wave instead of 8.3 KB for two 72-byte slabs, so 6-7
// workgroups fit a CU instead of four.  The ROI slab offset o of detection pixel (r, c) is
// (r + 3) * RB + c + 4.
template <int RB>
__device__ __forceinline__ int fast_mi(int o, int mp)
{
    if constexpr (RB == kFastRowBytesM) {
        return o + 45;
    } else {
        const int yy = (int)((unsigned)o / (unsigned)RB);
        return (yy - 2) * mp + (o - yy * RB) - 3;
    }
}

__device__ __forceinline__ int nms_keep(const uint8_t* Ms, int mi, int mp, int t, int* sc_out)
{
    const int M = Ms[mi];
    if (M <= t) return 0;
    const int sc = M - 1;
    bool kept = true;
#pragma unroll
    for (int dy = -1; dy <= 1; dy++)
#pragma unroll
        for (int dx = -1; dx <= 1; dx++) {
            if (dx == 0 && dy == 0) continue;
            const int Mn = Ms[mi + dy * mp + dx];
            const int ns = Mn > t ? Mn - 1 : 0;
            kept = kept && (sc > ns);
        }
    *sc_out = sc;
    return kept ? 1 : 0;
}

// Count of set bits of a wave mask below this lane (v_mbcnt_lo/hi).
__device__ __forceinline__ int mbcnt(uint64_t m)
{
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

constexpr int kFastPass = 12;            // prefetched ROI rows / 4 (cells up to 48 rows)

// Staging of a cell ROI into the wave's slab (slab byte = ROI column + 1, so detection
// column 0 = ROI column 3 is 4-byte aligned).  The word path keeps the loads in registers
// (q0) so the next cell's loads can be issued before the current cell is processed.
struct FastCellGeom {
    const uint8_t* img;
    int pitch, x0, y0, rw, rh, nwords;
    bool vec;                          // 16-byte aligned rows, row fits 12 words, <= 48 rows
    bool words;                        // pitch % 4 == 0 and the row fits 15 words
};

// ROI prefetch registers: 16-byte path (lane = row (lane >> 2) + 16 i, chunk lane & 3) or
// word path (lane = row (lane >> 4) + 4 i, word lane & 15).
struct FastRegs {
    u32x4 v0, v1, v2;                  // 16-byte path only: the word path loads when it stages
};

__device__ __forceinline__ FastCellGeom fast_geom(const Plan* P, const ExtractBufs& b, int f, const CellDesc& c)
{
    FastCellGeom G;
    const LevelGeom& g = P->lv[c.level];
    G.img = level_ptr(P, b, f, c.level);
    G.pitch = g.pitch;
    G.x0 = c.x0; G.y0 = c.y0; G.rw = c.rw; G.rh = c.rh;
    G.nwords = (1 + c.rw + 3) >> 2;
    G.vec = ((g.pitch | (int)reinterpret_cast<uintptr_t>(G.img)) & 15) == 0 && G.nwords <= 12 && c.rh <= 48;
    G.words = (g.pitch & 3) == 0 && G.nwords <= 15 && c.rh <= 4 * kFastPass;
    return G;
}

__device__ __forceinline__ void fast_prefetch(const FastCellGeom& G, FastRegs& R)
{
    const int lane = lane_id();
    if (G.vec) {
        // three 16-byte loads per lane cover 48 rows x 64 bytes from (x0 - 1) & ~15
        const uint8_t* base = G.img + (int64_t)G.y0 * G.pitch + ((G.x0 - 1) & ~15) + 16 * (lane & 3);
        const int r = lane >> 2;
        R.v0 = *reinterpret_cast<const u32x4*>(base + (int64_t)min(r, G.rh - 1) * G.pitch);
        R.v1 = *reinterpret_cast<const u32x4*>(base + (int64_t)min(r + 16, G.rh - 1) * G.pitch);
        R.v2 = *reinterpret_cast<const u32x4*>(base + (int64_t)min(r + 32, G.rh - 1) * G.pitch);
    }
}

// Zero chunks of the LDS-DMA staging (the M columns of a 96-B slab row).
__device__ __attribute__((aligned(64))) const uint8_t g_fast_zero[64] = {0};

// LDS-DMA staging of a cell ROI into 96-B slab rows (RB = kFastRowBytesM, rh <= 48): slab row r is
// six 16-byte chunks, chunks 0..2 the image bytes x0 - 1 + 16 k .. of row y0 + r (byte-granular
// source address, so slab byte j = ROI column j - 1 with no realignment and 16-byte aligned LDS
// writes), chunks 3..5 zeros from g_fast_zero (the M columns 48..95).  A wave-instruction writes
// 64 consecutive chunks (1 KiB); chunks past row rh - 1 are masked off.  No VGPR staging, no
// ds_write: the register-staged form's unaligned ds_write_b128 stores were replayed by the LDS
// (SQ_LDS_UNALIGNED_STALL, profiles/r04/ab8).  Completion: vmcnt (fast_dma_wait).
__device__ __forceinline__ void fast_dma(const FastCellGeom& G, uint8_t* roi)
{
    typedef __attribute__((address_space(3))) void* lds_vp;
    const int lane = lane_id();
    const int nq = 6 * G.rh;
    const uint8_t* row0 = G.img + (int64_t)G.y0 * G.pitch + (G.x0 - 1);
#pragma unroll
    for (int i = 0; i < 5; i++) {
        if (64 * i < nq) {
            const int q = 64 * i + lane;
            const int r = (q * 171) >> 10;                 // q / 6 for q < 512
            const int k = q - 6 * r;
            const uint8_t* src = k < 3 ? row0 + r * G.pitch + 16 * k : g_fast_zero;
            if (q < nq) __builtin_amdgcn_global_load_lds((const void*)src, (lds_vp)(roi + 1024 * i), 16, 0, 0);
        }
    }
}
__device__ __forceinline__ void fast_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int RB>
__device__ __forceinline__ void fast_stage(const FastCellGeom& G, const FastRegs& R, uint8_t* roi)
{
    const int lane = lane_id();
    if (G.vec) {
        // the 64-byte window's chunks stored as loaded, each at its own slab offset - sh
        // (unaligned ds_write_b128: gfx950 LDS takes any byte address), so slab byte j = ROI
        // column j - 1 with no realignment in registers.  Row r's first chunk spills sh bytes
        // into the tail of row r - 1 (its M columns 81..95, zeroed by the M clear that follows)
        // and row 0's into the 16-byte guard before the slab; the last chunk's bytes past
        // column 47 land in the row's own M columns, also cleared after.
        const int sh = (G.x0 - 1) & 15;
        const int r = lane >> 2, c = lane & 3;
        uint8_t* d = roi + r * RB + 16 * c - sh;
        if (r < G.rh) __builtin_memcpy(d, &R.v0, 16);
        if (r + 16 < G.rh) __builtin_memcpy(d + 16 * RB, &R.v1, 16);
        if (r + 32 < G.rh) __builtin_memcpy(d + 32 * RB, &R.v2, 16);
        if constexpr (RB == kFastRowBytesM) {
            // then zero the rows' M columns 48..95 (after every row's data: the stores above
            // spill into them), three lanes per row.  Per lane the data and zero stores never
            // overlap, so nothing in the compiler's alias analysis keeps them in this order; the
            // spill of ANOTHER lane's data store does overlap.  The empty asm with a memory clobber
            // is a scheduling barrier: the zero stores stay after the data stores (one wave's LDS
            // instructions execute in issue order).
            asm volatile("" ::: "memory");
            uint8_t* z = roi + r * RB + 48 + 16 * c;
            const uint4 zero = make_uint4(0, 0, 0, 0);
            if (c < 3 && r < G.rh) *reinterpret_cast<uint4*>(z) = zero;
            if (c < 3 && r + 16 < G.rh) *reinterpret_cast<uint4*>(z + 16 * RB) = zero;
            if (c < 3 && r + 32 < G.rh) *reinterpret_cast<uint4*>(z + 32 * RB) = zero;
        }
    } else if (G.words) {
        const int gx = G.x0 - 1;
        const int kw = min(lane & 15, G.nwords);
        const uint32_t* wbase = reinterpret_cast<const uint32_t*>(G.img + (int64_t)G.y0 * G.pitch + (gx & ~3)) + kw;
        const int pw = G.pitch >> 2;
        const int npass = (G.rh + 3) >> 2;
        uint32_t q0[kFastPass];
#pragma unroll
        for (int i = 0; i < kFastPass; i++)
            if (i < npass) q0[i] = wbase[min((lane >> 4) + 4 * i, G.rh - 1) * pw];
        // word k of slab row = ROI columns 4k-1 .. 4k+2 = this lane's aligned word joined
        // with the next lane's (DPP row shift; one slab row = one 16-lane DPP row)
        const int al = (G.x0 - 1) & 3;
#pragma unroll
        for (int i = 0; i < kFastPass; i++) {
            if (i < npass) {
                const uint32_t q1 = dpp_shl1(q0[i]);
                const int yy = (lane >> 4) + 4 * i;
                if (yy < G.rh && (lane & 15) < G.nwords)
                    *reinterpret_cast<uint32_t*>(roi + yy * RB + 4 * (lane & 15)) =
                        __builtin_amdgcn_alignbyte(q1, q0[i], (uint32_t)al);
            }
        }
    } else if ((G.pitch & 3) == 0) {
        const int gx = G.x0 - 1;
        const int al = gx & 3;
        const uint8_t* base = G.img + (int64_t)G.y0 * G.pitch + (gx & ~3);
        for (int yy = lane >> 4; yy < G.rh; yy += 4)
            for (int k = lane & 15; k < G.nwords; k += 16) {
                const uint32_t* q = reinterpret_cast<const uint32_t*>(base + (int64_t)yy * G.pitch) + k;
                *reinterpret_cast<uint32_t*>(roi + yy * RB + 4 * k) =
                    __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)al);
            }
    } else {
        for (int yy = lane >> 4; yy < G.rh; yy += 4)
            for (int xx = lane & 15; xx < G.rw; xx += 16)
                roi[yy * RB + 1 + xx] = G.img[(int64_t)(G.y0 + yy) * G.pitch + G.x0 + xx];
    }
}

// Bytes of one per-wave ROI (or M) slab: 16-byte multiple so every slab starts 16-aligned.
// Per-wave LDS of k_fast<RB>: pixel slab (+ M slab for RB = kFastRowBytes), survivor list with
// one scratch slot per lane, corner list.  RB = kFastRowBytesM when every ROI is <= 46 wide.
__host__ __device__ inline int fast_rb(const Plan& P) { return P.max_roi_w <= 46 ? kFastRowBytesM : kFastRowBytes; }
__host__ __device__ inline int fast_slab(const Plan& P, int rb) { return (rb * P.max_roi_h + 15) & ~15; }
__host__ __device__ inline int fast_mp(const Plan& P) { return (P.max_roi_w - 6 + 2 + 3) & ~3; }
__host__ __device__ inline int fast_ms_slab(const Plan& P, int rb)
{
    return rb == kFastRowBytesM ? 0 : (fast_mp(P) * (P.max_roi_h - 4) + 15) & ~15;
}
__host__ __device__ inline int fast_wave_lds(const Plan& P, int rb)
{
    return kFastGuard + fast_slab(P, rb) + fast_ms_slab(P, rb) + 2 * (kFastLists + kFastCorners + kFastEnt);
}

#ifndef COEB_FAST_CLOCK
#define COEB_FAST_CLOCK 0      // experiment builds: per-cell k_fast phase clocks (fast_timing)
#endif
#define FC_MARK(v) long long v = COEB_FAST_CLOCK ? (long long)clock64() : 0
// per-cell slots spread over 256 copies (blockIdx.x & 255) so the counters do not contend
__device__ unsigned long long g_fast_clk[256 * 8];
#define FC_SLOT(slot) g_fast_clk[(blockIdx.x & 255) * 8 + (slot)]
#define FC_ADD(slot, t0) do { if (COEB_FAST_CLOCK && lane_id() == 0) atomicAdd(&FC_SLOT(slot), (unsigned long long)((long long)clock64() - (t0))); } while (0)

// Pre-test, exact strength, NMS and ordered output of one staged cell.
template <int RB>
__device__ __forceinline__ void fast_cell(const Plan* P, const ExtractBufs& b, int f, int cidx, const CellDesc& c,
                                          int th_ini, int th_min, const uint8_t* roi, uint8_t* Ms, uint16_t* surv,
                                          uint16_t* corn, uint16_t* ent)
{
    constexpr int sh = 1;
    const int lane = lane_id();
    const LevelGeom& g = P->lv[c.level];
    const int rw = c.rw, rh = c.rh;
    const int ww = rw - 6, wh = rh - 6;
    const int mp = RB == kFastRowBytesM ? RB : fast_mp(*P);   // M pitch
    const int npix = ww > 0 && wh > 0 ? ww * wh : 0;
    // ---- 2 + 3: pre-test 4 pixels per lane (8 or 16 lanes per row).  A lane with survivors
    //      appends ONE entry (slab offset of its first pixel / 4 | 4-bit survivor mask << 12) to the
    //      wave's entry list, in ballot (= row-major) order: one ballot per pass instead of one
    //      compaction per pixel slot.  When a pass could overflow the list, and at the end, the
    //      entries are expanded into the survivor list (a wave scan of their popcounts keeps the
    //      row-major order) and the survivors' exact strengths taken -> Ms + corner list.
    int ne = 0, nc = 0;
    const int ngrp = (ww + 3) >> 2;
    const int lpr_log = ngrp > 8 ? 4 : 3;
    const int cg = lane & ((1 << lpr_log) - 1), rsub = lane >> lpr_log;
    const int rpi = 64 >> lpr_log;
    // lanes' pixel columns inside the window (fixed for the cell)
    const uint32_t vmask4 = (1u << min(max(ww - 4 * cg, 0), 4)) - 1u;   // columns 4 cg + k < ww
    int o = (rsub + 3) * RB + 4 + 4 * cg;
    const uint32_t one2 = 0x00010001u;
    FC_MARK(t_scan);
    long long t_str = 0;
    // entries -> survivors -> exact strengths -> Ms + corner list (the list is drained when a
    // further pass could overflow it, and at the end)
    auto flush = [&]() {
        FC_MARK(t_s0);
        wave_sync_lds();
        for (int e0 = 0; e0 < ne; e0 += 64) {
            const int e = e0 + lane;
            const uint32_t en = e < ne ? (uint32_t)ent[e] : 0u;
            const uint32_t m = en >> 12;
            const int cnt = __popc(m);
            // exclusive prefix of cnt (0..4) over the lanes, by bit planes
            const uint64_t b0 = __ballot(cnt & 1), b1 = __ballot(cnt & 2), b2 = __ballot(cnt & 4);
            int q = mbcnt(b0) + 2 * mbcnt(b1) + 4 * mbcnt(b2);
            const int ns = uniform((int)__popcll(b0) + 2 * (int)__popcll(b1) + 4 * (int)__popcll(b2));
            const int ob = (int)(en & 0xFFFu) << 2;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if ((m >> k) & 1u) surv[q++] = (uint16_t)(ob + k);
            surv[ns] = surv[ns > 0 ? ns - 1 : 0];      // pad an odd count (the pair's B repeats A's pixel)
            wave_sync_lds();
            for (int s0 = 0; s0 < ns; s0 += 64) {
                const int si = s0 + lane;
                int oo = 0, M = 0;
                if (si < ns) {
                    oo = surv[si];
                    M = corner_strength_pos2<RB>(&roi[oo], th_min);
                }
                const bool isc = si < ns && M > th_min;
                if (isc) Ms[fast_mi<RB>(oo, mp)] = (uint8_t)M;
                const uint64_t mc = __ballot(isc);
                if (isc) {
                    const int qq = nc + mbcnt(mc);
                    if (qq < kFastCorners) corn[qq] = (uint16_t)oo;
                }
                nc = uniform(nc + (int)__popcll(mc));
            }
            wave_sync_lds();
        }
        ne = 0;
        if (COEB_FAST_CLOCK) t_str += (long long)clock64() - t_s0;
    };
    // (round 6: the passes' pre-tests first with the survivor masks gathered in registers, then
    // one entry append per pass -- no cross-lane step between pre-tests -- measured slower,
    // 0.857 vs 0.836 ms per 1025-frame launch, profiles/r06/fast)
    for (int r0 = 0; npix > 0 && r0 < wh; r0 += rpi, o += rpi * RB) {
        // every lane runs the test (rows past the window read slab bytes that are masked off)
        uint32_t lo, hi;
        fast_pretest4_raw<RB>(&roi[o], th_min, lo, hi);
        // survivor bits: a packed u16 half is nonzero iff its pixel survives.  min(half, 1) as an
        // opaque v_pk_min_u16: written in C the compiler turns it into per-half compares and selects
        uint32_t s01, s23;
        asm("v_pk_min_u16 %0, %1, %2" : "=v"(s01) : "v"(lo), "v"(one2));
        asm("v_pk_min_u16 %0, %1, %2" : "=v"(s23) : "v"(hi), "v"(one2));
        const uint32_t t2 = s01 | (s23 << 2);
        const uint32_t m4 = (t2 | (t2 >> 15)) & (rsub < wh - r0 ? vmask4 : 0u);   // wh - r0: scalar
        const uint64_t mk = __ballot(m4 != 0u);
        if (mk) {
            if (m4) ent[ne + mbcnt(mk)] = (uint16_t)(((uint32_t)o >> 2) | (m4 << 12));   // o = 4 mod 4: exact
            ne = uniform(ne + (int)__popcll(mk));
        }
        if (ne > kFastEnt - 64 || r0 + rpi >= wh) flush();
    }
    FC_ADD(1, t_scan + t_str);                        // pre-test passes (strength flushes excluded)
    if (COEB_FAST_CLOCK && lane_id() == 0) atomicAdd(&FC_SLOT(2), (unsigned long long)t_str);
    FC_MARK(t_nms);
    // ---- 4: NMS + ordered compaction
    uint32_t* out = b.cand + ((int64_t)f * P->ncells + cidx) * P->cell_cap;
    int nkept = 0;
    for (int pass = 0; pass < 2; pass++) {
        const int t = pass == 0 ? th_ini : th_min;
        int running = 0;
        if (nc <= kFastCorners) {
            for (int e0 = 0; e0 < nc; e0 += 64) {
                const int e = e0 + lane;
                int oo = 0, sc = 0, kept = 0;
                if (e < nc) {
                    oo = corn[e];
                    kept = nms_keep(Ms, fast_mi<RB>(oo, mp), mp, t, &sc);
                }
                const uint64_t m = __ballot(kept);
                if (kept) {
                    const int q = running + mbcnt(m);
                    const int yy = oo / RB, xx = oo - yy * RB - sh;
                    if (q < P->cell_cap) out[q] = pack_key(xx + c.j * g.wcell, yy + c.i * g.hcell, sc);
                    else atomicOr(b.err, 2);
                }
                running = uniform(running + __popcll(m));
            }
        } else {
            int row0 = 0, col0 = 0;
            for (int base = 0; base < npix; base += 64) {
                int col = col0 + lane, row = row0;
                while (col >= ww) { col -= ww; row++; }
                int sc = 0, kept = 0;
                const int mi = RB == kFastRowBytesM ? (row + 3) * RB + col + 4 + 45 : (row + 1) * mp + col + 1;
                if (base + lane < npix) kept = nms_keep(Ms, mi, mp, t, &sc);
                const uint64_t m = __ballot(kept);
                if (kept) {
                    const int q = running + mbcnt(m);
                    if (q < P->cell_cap) out[q] = pack_key(col + 3 + c.j * g.wcell, row + 3 + c.i * g.hcell, sc);
                    else atomicOr(b.err, 2);
                }
                running = uniform(running + __popcll(m));
                col0 += 64;
                while (col0 >= ww) { col0 -= ww; row0++; }
            }
        }
        nkept = running;
        if (nkept > 0) break;
    }
    if (lane == 0) b.cand_n[(int64_t)f * P->ncells + cidx] = min(nkept, P->cell_cap);
    FC_ADD(3, t_nms);
    if (COEB_FAST_CLOCK && lane == 0) { atomicAdd(&FC_SLOT(5), 1ull); atomicAdd(&FC_SLOT(6), (unsigned long long)nc); }
}

// Cell descriptor as one 16-byte scalar load (16-bit fields would become vector loads).
__device__ __forceinline__ CellDesc load_cell(const CellDesc* __restrict__ cells, int i)
{
    const int4 r = reinterpret_cast<const int4*>(cells)[i];
    CellDesc c;
    c.level = (int16_t)(r.x & 0xFFFF); c.pad = 0;
    c.x0 = (int16_t)(r.y & 0xFFFF); c.y0 = (int16_t)(r.y >> 16);
    c.rw = (int16_t)(r.z & 0xFFFF); c.rh = (int16_t)(r.z >> 16);
    c.i = (int16_t)(r.w & 0xFFFF); c.j = (int16_t)(r.w >> 16);
    return c;
}

// One wave per cell, four waves per workgroup, no workgroup barriers.  (Two cells per wave with
// the second cell's ROI loads issued before the first is processed spilled 240 B per lane and
// ran 2.7x slower.)
template <int RB>
#ifndef COEB_FAST_MINWG
#define COEB_FAST_MINWG 6      // launch bound: workgroups per CU the register budget must allow
#endif
__global__ __launch_bounds__(kThreads, COEB_FAST_MINWG) void k_fast(const Plan* __restrict__ P, ExtractBufs b,
                                                       const CellDesc* __restrict__ cells,   // read-only: scalar loads
                                                       int cell0, int cell1)                 // this launch's cells
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // A wave-uniform wave index, so the cell geometry and the per-cell bookkeeping live in
    // SGPRs on the scalar unit: the kernel is VALU-bound (SQ_INSTS_VALU x 4 cycles = 95 % of the
    // SIMDs' cycles, profiles/r04/pipes), and moving that work off the VALU took 1.026 -> 0.962 ms
    // per 1025-frame launch (profiles/r04/ab7).  (Round 2 measured the opposite, 5 % slower, when
    // the scalar unit was the busier pipe.)  A u16-pixel slab (ring operands as aligned u16
    // pairs, no byte gathers; 11 ds_read_b64 per 4-pixel group) cut VALU 7 % but ran 5 % slower
    // (twice the staging stores): the byte slab stays.
    const int wv = wave_id(), lane = lane_id();
    const int slab = fast_slab(*P, RB), ms_slab = fast_ms_slab(*P, RB);   // per-wave LDS: roi, M, lists
    uint8_t* wbase = smem + (size_t)wv * fast_wave_lds(*P, RB) + kFastGuard;
    uint8_t* roi = wbase;
    uint8_t* Ms = RB == kFastRowBytesM ? wbase : wbase + slab;
    uint16_t* surv = reinterpret_cast<uint16_t*>(wbase + slab + ms_slab);
    uint16_t* corn = surv + kFastLists;
    uint16_t* ent = corn + kFastCorners;
    const int2 bxy = block_xy<false>();
    const int f = bxy.y;
    const int cidx = cell0 + bxy.x * kWaves + wv;
    if (cidx >= cell1) return;
    const int area = b.dyn[f].area_flag;
    const int th_ini = area ? 30 : 20, th_min = area ? 10 : 7;   // ORBextractor.cc:775-784
    const CellDesc c = load_cell(cells, cidx);
    const FastCellGeom G = fast_geom(P, b, f, c);
    const bool dma = RB == kFastRowBytesM && c.rh <= 48;     // 96-B slab rows by LDS-DMA (wave-uniform)
    FastRegs R;
    if (dma) fast_dma(G, roi);
    else fast_prefetch(G, R);
    FC_MARK(t_all);
    FC_MARK(t_st);
    if (dma) fast_dma_wait();
    else fast_stage<RB>(G, R, roi);
    if (RB == kFastRowBytesM) {
        // M columns 48..95 of rows 2 .. rh-3 (the 16-byte staging and the DMA zero them themselves)
        if (!G.vec && !dma)
        for (int i = lane; i < 3 * (c.rh - 4); i += 64) {
            const int row = 2 + i / 3;
            reinterpret_cast<uint4*>(Ms + row * RB + 48)[i - 3 * (row - 2)] = make_uint4(0, 0, 0, 0);
        }
    } else {
        for (int i = lane; i < ms_slab / 16; i += 64) reinterpret_cast<uint4*>(Ms)[i] = make_uint4(0, 0, 0, 0);
    }
    wave_sync_lds();
    FC_ADD(0, t_st);                              // wait for the ROI loads + stage + M clear
    fast_cell<RB>(P, b, f, cidx, c, th_ini, th_min, roi, Ms, surv, corn, ent);
    FC_ADD(4, t_all);
}

// Workgroup barrier ordering LDS only: __syncthreads() also waits for every outstanding global
// load and store (vmcnt).  Used where waves share nothing through global memory.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ================================ k_octree ================================
// One workgroup per (level, frame): gathers the level's FAST candidates in the reference
// order (cell row-major, then FAST row-major), applies the pre-octree cull when area_flag,
// and emulates DistributeOctTree's std::list exactly (push_front order, erase, the sorted
// final phase with size ties broken by allocation order = monotonic allocator), then
// retains the best response per node (first wins ties), adds the border, and applies
// CheckMovingKeyPoints_finall when !area_flag.  Keys live in two global ping-pong buffers
// (L2-resident); a node's keys are a contiguous range and DivideNode is a stable 4-way
// partition of it done by one wave with ballots.  Node records live in two global sets and
// are compacted into list order after every pass.
struct NodeRef {
    int* start; int* cnt; int* alloc; int* buf; int4* rect;
};

// k_octree dynamic LDS: work arrays (W entries), two node-record sets (W records), and two
// key buffers of oct_kl entries used when the level has at most that many candidates.
struct OctLds {
    int* work; int4* cnt; int* base; int* rank; int* push; uint8_t* dead;
    NodeRef set[2];
    uint32_t* keys[2];
    size_t set_stride;     // bytes between set[0] and set[1] fields
};

__device__ __forceinline__ OctLds oct_lds(uint8_t* smem, int W, int KL)
{
    OctLds o;
    size_t off = 0;
    o.cnt = reinterpret_cast<int4*>(smem + off); off += (size_t)W * 16;
    o.work = reinterpret_cast<int*>(smem + off); off += (size_t)W * 4;
    o.base = reinterpret_cast<int*>(smem + off); off += (size_t)W * 4;
    o.rank = reinterpret_cast<int*>(smem + off); off += (size_t)W * 4;
    o.push = reinterpret_cast<int*>(smem + off); off += (size_t)W * 4;
    for (int s = 0; s < 2; s++) {
        o.set[s].rect = reinterpret_cast<int4*>(smem + off); off += (size_t)W * 16;
        o.set[s].start = reinterpret_cast<int*>(smem + off); off += (size_t)W * 4;
        o.set[s].cnt = reinterpret_cast<int*>(smem + off); off += (size_t)W * 4;
        o.set[s].alloc = reinterpret_cast<int*>(smem + off); off += (size_t)W * 4;
        o.set[s].buf = reinterpret_cast<int*>(smem + off); off += (size_t)W * 4;
    }
    o.set_stride = (size_t)W * 32;
    o.keys[0] = reinterpret_cast<uint32_t*>(smem + off); off += (size_t)KL * 4;
    o.keys[1] = reinterpret_cast<uint32_t*>(smem + off); off += (size_t)KL * 4;
    o.dead = smem + off;
    return o;
}

// set[s] without a dynamically indexed local array (which the compiler puts in scratch)
__device__ __forceinline__ NodeRef nref(const OctLds& O, int s)
{
    NodeRef r = O.set[0];
    const size_t d = s ? O.set_stride : 0;
    r.rect = reinterpret_cast<int4*>(reinterpret_cast<uint8_t*>(r.rect) + d);
    r.start = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(r.start) + d);
    r.cnt = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(r.cnt) + d);
    r.alloc = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(r.alloc) + d);
    r.buf = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(r.buf) + d);
    return r;
}

__device__ __forceinline__ int quadrant(uint32_t k, int sx, int sy)
{
    const int x = key_x(k), y = key_y(k);
    return x < sx ? (y < sy ? 0 : 2) : (y < sy ? 1 : 3);
}

// Count keys per quadrant of node range [s, s+n) (one wave).
__device__ __forceinline__ int4 wave_count_quadrants(const uint32_t* src, int s, int n, int sx, int sy)
{
    int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    const int lane = lane_id();
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        const bool v = i < n;
        const int q = v ? quadrant(src[s + i], sx, sy) : -1;
        c0 += __popcll(__ballot(q == 0));
        c1 += __popcll(__ballot(q == 1));
        c2 += __popcll(__ballot(q == 2));
        c3 += __popcll(__ballot(q == 3));
    }
    return make_int4(c0, c1, c2, c3);
}

// Stable scatter of keys [s, s+n) of src into dst, quadrant q's keys from position r.q on
// (one wave).
__device__ __forceinline__ void wave_scatter_quadrants_at(const uint32_t* src, uint32_t* dst, int s, int n,
                                                          int sx, int sy, int4 r)
{
    int r0 = r.x, r1 = r.y, r2 = r.z, r3 = r.w;
    const int lane = lane_id();
    const uint64_t lt = lanemask_lt();
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        const bool v = i < n;
        const uint32_t k = v ? src[s + i] : 0u;
        const int q = v ? quadrant(k, sx, sy) : -1;
        const uint64_t m0 = __ballot(q == 0), m1 = __ballot(q == 1), m2 = __ballot(q == 2), m3 = __ballot(q == 3);
        if (v) {
            const uint64_t mq = q == 0 ? m0 : q == 1 ? m1 : q == 2 ? m2 : m3;
            const int rq = q == 0 ? r0 : q == 1 ? r1 : q == 2 ? r2 : r3;
            dst[rq + __popcll(mq & lt)] = k;
        }
        r0 += __popcll(m0); r1 += __popcll(m1); r2 += __popcll(m2); r3 += __popcll(m3);
    }
}

// Stable scatter of node range [s, s+n) from src into dst at [s, s+n), quadrant order.
__device__ __forceinline__ void wave_scatter_quadrants(const uint32_t* src, uint32_t* dst, int s, int n,
                                                       int sx, int sy, int4 c)
{
    wave_scatter_quadrants_at(src, dst, s, n, sx, sy,
                              make_int4(s, s + c.x, s + c.x + c.y, s + c.x + c.y + c.z));
}

// The same two steps for one node by one lane (the final phase and the late passes divide
// many nodes of a few keys each: a wave per node would idle most of its lanes).
__device__ __forceinline__ int4 lane_count_quadrants(const uint32_t* src, int s, int n, int sx, int sy)
{
    int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int i = 0; i < n; i++) {
        const int q = quadrant(src[s + i], sx, sy);
        c0 += q == 0; c1 += q == 1; c2 += q == 2; c3 += q == 3;
    }
    return make_int4(c0, c1, c2, c3);
}

__device__ __forceinline__ void lane_scatter_quadrants(const uint32_t* src, uint32_t* dst, int s, int n, int sx,
                                                       int sy, int4 c)
{
    int r0 = s, r1 = s + c.x, r2 = s + c.x + c.y, r3 = s + c.x + c.y + c.z;
    for (int i = 0; i < n; i++) {
        const uint32_t k = src[s + i];
        const int q = quadrant(k, sx, sy);
        const int r = q == 0 ? r0++ : q == 1 ? r1++ : q == 2 ? r2++ : r3++;
        dst[r] = k;
    }
}

// The same two steps by a team of G lanes of one wave (G = 4 or 16): the team's lanes stay
// converged (same node, same trip count), so the per-lane counts are summed over the team with
// xor shuffles and the scatter ranks come from the wave's ballots masked to the team's lanes.
template <int G>
__device__ __forceinline__ int4 team_count_quadrants(const uint32_t* src, int s, int n, int sx, int sy)
{
    int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int i = lane_id() & (G - 1); i < n; i += G) {
        const int q = quadrant(src[s + i], sx, sy);
        c0 += q == 0; c1 += q == 1; c2 += q == 2; c3 += q == 3;
    }
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
        c0 += __shfl_xor(c0, o, 64); c1 += __shfl_xor(c1, o, 64);
        c2 += __shfl_xor(c2, o, 64); c3 += __shfl_xor(c3, o, 64);
    }
    return make_int4(c0, c1, c2, c3);
}

template <int G>
__device__ __forceinline__ void team_scatter_quadrants(const uint32_t* src, uint32_t* dst, int s, int n, int sx,
                                                       int sy, int4 c)
{
    int r0 = s, r1 = s + c.x, r2 = s + c.x + c.y, r3 = s + c.x + c.y + c.z;
    const int lane = lane_id(), gl = lane & (G - 1);
    const uint64_t tm = ((1ull << G) - 1ull) << (lane & ~(G - 1));   // this team's lanes
    for (int base = 0; base < n; base += G) {
        const int i = base + gl;
        const bool v = i < n;
        const uint32_t k = v ? src[s + i] : 0u;
        const int q = v ? quadrant(k, sx, sy) : -1;
        const uint64_t m0 = __ballot(q == 0) & tm, m1 = __ballot(q == 1) & tm;
        const uint64_t m2 = __ballot(q == 2) & tm, m3 = __ballot(q == 3) & tm;
        if (v) {
            const uint64_t mq = q == 0 ? m0 : q == 1 ? m1 : q == 2 ? m2 : m3;
            const int rq = q == 0 ? r0 : q == 1 ? r1 : q == 2 ? r2 : r3;
            dst[rq + mbcnt(mq)] = k;
        }
        r0 += __popcll(m0); r1 += __popcll(m1); r2 += __popcll(m2); r3 += __popcll(m3);
    }
}

// Lanes per node for dividing nd nodes of about `avg` keys with NT threads: the team size
// (1, 4, 16 or 64) with the fewest sequential key loads per lane, ceil(nd G / NT) ceil(avg / G)
// (the key loads are latency-bound, L2 when the keys are global); ties go to the larger team.
template <int NT>
__device__ __forceinline__ int oct_team(int nd, int avg)
{
    int best = 64, bc = 0x7fffffff;
#pragma unroll
    for (int gi = 0; gi < 4; gi++) {
        const int G = 64 >> (2 * gi);
        const int c = ((nd * G + NT - 1) / NT) * ((avg + G - 1) / G);
        if (c < bc) { bc = c; best = G; }
    }
    return best;
}

__device__ __forceinline__ void child_rect(const int4 p, int q, int4* out, int* sx, int* sy)
{
    const int hx = (int)ceilf((float)(p.z - p.x) / 2);   // ExtractorNode::DivideNode :491-492
    const int hy = (int)ceilf((float)(p.w - p.y) / 2);
    const int mx = p.x + hx, my = p.y + hy;
    *sx = mx; *sy = my;
    if (q == 0) *out = make_int4(p.x, p.y, mx, my);
    else if (q == 1) *out = make_int4(mx, p.y, p.z, my);
    else if (q == 2) *out = make_int4(p.x, my, mx, p.w);
    else *out = make_int4(mx, my, p.z, p.w);
}

#ifndef COEB_OCT_CLOCK
#define COEB_OCT_CLOCK 0       // experiment builds: per-workgroup k_octree clocks (oct_timing)
#endif
// [wg][6]: level, K (candidates), start (wall clock), cycles: total, gather + initial nodes, main loop
__device__ long long g_oct_clk[4096 * 6];

template <int NT>
__global__ __launch_bounds__(NT) void k_octree(const Plan* __restrict__ P, ExtractBufs b, int level0, int oct_w,
                                                int oct_kl)   // this launch's node slots / LDS key capacity
{
    const long long oc_t0 = COEB_OCT_CLOCK ? (long long)clock64() : 0;
    const long long oc_w0 = COEB_OCT_CLOCK ? (long long)wall_clock64() : 0;
    long long oc_t1 = 0, oc_t2 = 0;
    constexpr int NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int sbuf[(NW + 2 + 3) & ~3];   // 16-byte multiple: keeps the dynamic LDS base aligned
    __shared__ int4 s_wq[NW];                 // per-wave quadrant counts of a node divided by all waves
    const OctLds O = oct_lds(smem, oct_w, oct_kl);
    int* const s_work = O.work;      // slot ids of nodes divided this phase (processing order)
    int4* const s_cnt = O.cnt;       // their quadrant counts
    int* const s_base = O.base;      // exclusive prefix of nonempty children (push order)
    int* const s_rank = O.rank;      // final phase: processing rank of vPrev entry
    int* const s_push = O.push;      // final phase: push-order base per rank
    uint8_t* const s_dead = O.dead;  // final phase: slot erased this round
    const int OCT_LMAX = oct_w;

    // frame-fastest grid: every frame's level-0 list (the longest) is dispatched in the first
    // wave of workgroups, the cheap upper levels fill in behind them
    const int f = blockIdx.x, l = level0 + blockIdx.y;
    const LevelGeom& g = P->lv[l];
    const int tid = threadIdx.x, wv = wave_id(), lane = lane_id();
    const DynMask& dm = b.dyn[f];      // by reference: a local copy is indexed dynamically (scratch)
    const int area = dm.area_flag;
    const int N = area ? g.nfeat_area : g.nfeat;
    // ---- 1. gather candidates in reference order ----
    const int* cn = b.cand_n + (int64_t)f * P->ncells + g.cell0;
    const uint32_t* cand = b.cand + ((int64_t)f * P->ncells + g.cell0) * P->cell_cap;
    int K = 0;
    {
        int part = 0;
        for (int ci = tid; ci < g.ncells; ci += NT) part += cn[ci];
        int tot;
        block_scan_excl<NW>(part, &tot, sbuf);
        K = tot;
    }
    // keys in LDS when they fit, else in the level's global ping-pong buffers (L2-resident)
    uint32_t* KB0;
    int64_t kdelta;
    // global keys: barriers also wait for the key stores (an LDS-only fence leaves them in flight)
    const bool kglob = K > oct_kl;
    auto obar = [&]() { if (kglob) __syncthreads(); else lds_barrier(); };
    if (K <= oct_kl) {
        KB0 = O.keys[0];
        kdelta = O.keys[1] - O.keys[0];
    } else {
        KB0 = b.keys + (int64_t)f * 2 * P->kbuf_stride + g.kcap_off;
        kdelta = P->kbuf_stride;
    }
    auto KB = [&](int i) -> uint32_t* { return KB0 + (i ? kdelta : 0); };
    if (g.ncells < oct_kl) {
        // per-cell offsets in LDS (keys[1] is free until the pre-octree cull), then every
        // thread copies keys, finding its cell by binary search: all loads independent
        int* s_coff = reinterpret_cast<int*>(O.keys[1]);
        int carry = 0;
        for (int base = 0; base < g.ncells; base += NT) {
            const int ci = base + tid;
            const int v = ci < g.ncells ? cn[ci] : 0;
            int tot;
            const int pre = block_scan_excl<NW>(v, &tot, sbuf);
            if (ci < g.ncells) s_coff[ci] = carry + pre;
            carry += tot;
        }
        K = carry;
        obar();
        for (int i = tid; i < K; i += NT) {
            int lo = 0, hi = g.ncells - 1;            // last cell with offset <= i
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_coff[mid] <= i) lo = mid; else hi = mid - 1;
            }
            KB(0)[i] = cand[(int64_t)lo * P->cell_cap + (i - s_coff[lo])];
        }
    } else {
        int carry = 0;
        for (int base = 0; base < g.ncells; base += NT) {
            const int ci = base + tid;
            const int v = ci < g.ncells ? cn[ci] : 0;
            int tot;
            const int pre = block_scan_excl<NW>(v, &tot, sbuf);
            if (ci < g.ncells) {
                const uint32_t* src = cand + (int64_t)ci * P->cell_cap;
                uint32_t* dst = KB(0) + carry + pre;
                for (int q = 0; q < v; q++) dst[q] = src[q];
            }
            carry += tot;
        }
        K = carry;
    }
    obar();
    int kb = 0;   // buffer currently holding the candidates
    // ---- pre-octree cull (ORBextractor.cc:854-858; coordinates still relative, reference quirk)
    if (area) {
        const float scale = (l != 0) ? g.scale : 1.0f;
        int carry = 0;
        for (int base = 0; base < K; base += NT) {
            const int i = base + tid;
            uint32_t k = 0;
            bool keep = false;
            if (i < K) {
                k = KB(0)[i];
                keep = !masked_out(dm, (float)key_x(k), (float)key_y(k), scale, P->W, P->H);
            }
            int tot;
            const int pre = block_scan_flag<NW>(keep, &tot, sbuf);
            if (keep) KB(1)[carry + pre] = k;
            carry += tot;
        }
        K = carry;
        kb = 1;
        obar();
    }

    // ---- 2. initial nodes (:549-592) ----
    int n = 0;             // live list length (list order == slot order in set `cs`)
    int cs = 0;            // current node set
    int alloc_ctr = g.nini;
    {
        NodeRef S = O.set[0];
        if (g.nini == 1) {
            if (K > 0 && tid == 0) {
                S.start[0] = 0; S.cnt[0] = K; S.alloc[0] = 0; S.buf[0] = kb;
                S.rect[0] = make_int4((int)(g.hx * 0.f), 0, (int)(g.hx * 1.f), g.maxY);
            }
            n = K > 0 ? 1 : 0;
        } else {
            // stable multiway distribution by (int)(x / hX) into the other buffer
            int carry = 0;
            for (int i = 0; i < g.nini; i++) {
                const int lo = g.ini_bound[i], hi = g.ini_bound[i + 1];
                const int start = carry;
                for (int base = 0; base < K; base += NT) {
                    const int idx = base + tid;
                    uint32_t k = 0;
                    bool in = false;
                    if (idx < K) {
                        k = KB(kb)[idx];
                        in = key_x(k) >= lo && key_x(k) < hi;
                    }
                    int tot;
                    const int pre = block_scan_flag<NW>(in, &tot, sbuf);
                    if (in) KB(kb ^ 1)[carry + pre] = k;
                    carry += tot;
                }
                if (carry > start) {
                    if (tid == 0) {
                        S.start[n] = start; S.cnt[n] = carry - start; S.alloc[n] = i; S.buf[n] = kb ^ 1;
                        S.rect[n] = make_int4((int)(g.hx * (float)i), 0, (int)(g.hx * (float)(i + 1)), g.maxY);
                    }
                    n++;
                }
            }
        }
    }
    obar();

    // Quadrant work on the nodes s_work[j] of set S with teams of G lanes (oct_team): mode 0
    // counts (-> s_cnt[j]) and divides (keys KB(buf) -> KB(buf ^ 1)) nodes j < cnt; mode 1 only
    // counts; mode 2 divides the nodes j = s_base[r], r < cnt, with the counts already in s_cnt.
    auto divide_nodes = [&](int G, const NodeRef& S, int cnt, int mode) {
        auto team = [&](auto gc) {
            constexpr int TG = decltype(gc)::value;
            for (int r = tid / TG; r < cnt; r += NT / TG) {
                const int j = mode == 2 ? s_base[r] : r;
                const int k = s_work[j];
                const int s = S.start[k], c = S.cnt[k], bf = S.buf[k];
                int4 tmp; int sx, sy;
                child_rect(S.rect[k], 0, &tmp, &sx, &sy);
                int4 qc;
                if (mode == 2) {
                    qc = s_cnt[j];
                } else {
                    if constexpr (TG == 64) qc = wave_count_quadrants(KB(bf), s, c, sx, sy);
                    else if constexpr (TG == 1) qc = lane_count_quadrants(KB(bf), s, c, sx, sy);
                    else qc = team_count_quadrants<TG>(KB(bf), s, c, sx, sy);
                }
                if (mode != 1) {
                    if constexpr (TG == 64) wave_scatter_quadrants(KB(bf), KB(bf ^ 1), s, c, sx, sy, qc);
                    else if constexpr (TG == 1) lane_scatter_quadrants(KB(bf), KB(bf ^ 1), s, c, sx, sy, qc);
                    else team_scatter_quadrants<TG>(KB(bf), KB(bf ^ 1), s, c, sx, sy, qc);
                }
                if (mode != 2 && (lane & (TG - 1)) == 0) s_cnt[j] = qc;
            }
        };
        if (G == 64) team(std::integral_constant<int, 64>());
        else if (G == 16) team(std::integral_constant<int, 16>());
        else if (G == 4) team(std::integral_constant<int, 4>());
        else team(std::integral_constant<int, 1>());
    };

    if (COEB_OCT_CLOCK) oc_t1 = (long long)clock64();
    // ---- 3. main loop (:601-745) ----
    bool finish = false;
    bool final_phase = false;
    while (!finish) {
        const int prevSize = n;
        if (n > OCT_LMAX || n > g.ncap) { if (tid == 0) atomicOr(b.err, 4); finish = true; break; }
        NodeRef S = nref(O, cs), D = nref(O, cs ^ 1);
        // divided nodes = cnt > 1, in list order
        int nd = 0;
        for (int base = 0; base < n; base += NT) {
            const int k = base + tid;
            const bool dv = k < n && S.cnt[k] > 1;
            int tot;
            const int pre = block_scan_flag<NW>(dv, &tot, sbuf);
            if (dv) s_work[nd + pre] = k;
            nd += tot;
        }
        obar();
        // partition: one wave per divided node while the nodes are few and large, one lane per
        // node once there are many (then each holds a few keys)
        if (nd < NW) {
            // fewer nodes than waves: every wave on each node in turn, wave w on the w-th
            // 64-aligned slice, slices placed by a prefix of the per-wave counts
            for (int j = 0; j < nd; j++) {
                const int k = s_work[j];
                const int s = S.start[k], c = S.cnt[k], bf = S.buf[k];
                int4 tmp; int sx, sy;
                child_rect(S.rect[k], 0, &tmp, &sx, &sy);
                const int chunk = ((c + NW - 1) / NW + 63) & ~63;
                const int ws = min(c, wv * chunk), wn = min(c - ws, chunk);
                const int4 qw = wave_count_quadrants(KB(bf), s + ws, wn, sx, sy);
                if (lane == 0) s_wq[wv] = qw;
                obar();
                int4 tot = make_int4(0, 0, 0, 0), pre = tot;
                for (int w = 0; w < NW; w++) {
                    const int4 t = s_wq[w];
                    tot.x += t.x; tot.y += t.y; tot.z += t.z; tot.w += t.w;
                    if (w < wv) { pre.x += t.x; pre.y += t.y; pre.z += t.z; pre.w += t.w; }
                }
                const int4 r = make_int4(s + pre.x, s + tot.x + pre.y, s + tot.x + tot.y + pre.z,
                                         s + tot.x + tot.y + tot.z + pre.w);
                wave_scatter_quadrants_at(KB(bf), KB(bf ^ 1), s + ws, wn, sx, sy, r);
                if (tid == 0) s_cnt[j] = tot;
                obar();   // s_wq is rewritten for the next node
            }
        } else {
            // divided nodes hold every key but the single-key nodes'
            const int G = oct_team<NT>(nd, (K - (n - nd) + nd - 1) / nd);
            divide_nodes(G, S, nd, 0);
        }
        obar();
        // children alloc order = divided nodes in list order, n1..n4 nonempty
        int T = 0, nexp = 0;
        for (int base = 0; base < nd; base += NT) {
            const int j = base + tid;
            int e = 0, x = 0;
            if (j < nd) {
                const int4 q = s_cnt[j];
                e = (q.x > 0) + (q.y > 0) + (q.z > 0) + (q.w > 0);
                x = (q.x > 1) + (q.y > 1) + (q.z > 1) + (q.w > 1);
            }
            int tot, tot2;
            const int pre = block_scan_excl<NW>(e, &tot, sbuf);
            block_scan_excl<NW>(x, &tot2, sbuf);
            if (j < nd) s_base[j] = T + pre;
            T += tot;
            nexp += tot2;
        }
        obar();
        const int nnew = T + (n - nd);
        if (nnew > g.ncap) { if (tid == 0) atomicOr(b.err, 4); finish = true; break; }
        // write children (reverse push order at the front)
        for (int j = tid; j < nd; j += NT) {
            const int k = s_work[j];
            const int4 q = s_cnt[j];
            const int s = S.start[k], bf = S.buf[k];
            const int4 r = S.rect[k];
            int a = s_base[j];
            int off = s;
            const int qq[4] = {q.x, q.y, q.z, q.w};
            for (int c4 = 0; c4 < 4; c4++) {
                if (qq[c4] > 0) {
                    const int pos = T - 1 - a;
                    int4 cr; int sx, sy;
                    child_rect(r, c4, &cr, &sx, &sy);
                    D.start[pos] = off; D.cnt[pos] = qq[c4]; D.alloc[pos] = alloc_ctr + a;
                    D.buf[pos] = bf ^ 1; D.rect[pos] = cr;
                    a++;
                }
                off += qq[c4];
            }
        }
        // non-divided nodes keep their relative order after the children
        {
            int carry = 0;
            for (int base = 0; base < n; base += NT) {
                const int k = base + tid;
                const bool keep = k < n && S.cnt[k] <= 1;
                int tot;
                const int pre = block_scan_flag<NW>(keep, &tot, sbuf);
                if (keep) {
                    const int pos = T + carry + pre;
                    D.start[pos] = S.start[k]; D.cnt[pos] = S.cnt[k]; D.alloc[pos] = S.alloc[k];
                    D.buf[pos] = S.buf[k]; D.rect[pos] = S.rect[k];
                }
                carry += tot;
            }
        }
        obar();
        alloc_ctr += T;
        n = nnew;
        cs ^= 1;
        if (n >= N || n == prevSize) { finish = true; break; }
        if (n + nexp * 3 > N) { final_phase = true; break; }
    }

    // ---- 3b. final phase (:683-743) ----
    while (final_phase && !finish) {
        const int prevSize = n;
        if (n > OCT_LMAX) { if (tid == 0) atomicOr(b.err, 4); break; }
        NodeRef S = nref(O, cs), D = nref(O, cs ^ 1);
        // vPrev = list nodes with cnt > 1, i.e. vSizeAndPointerToNode of the previous round
        int m = 0;
        for (int base = 0; base < n; base += NT) {
            const int k = base + tid;
            const bool dv = k < n && S.cnt[k] > 1;
            int tot;
            const int pre = block_scan_flag<NW>(dv, &tot, sbuf);
            if (dv) s_work[m + pre] = k;
            m += tot;
        }
        for (int k = tid; k < n; k += NT) s_dead[k] = 0;
        obar();
        // quadrant counts of every vPrev node (vPrev holds every key but the single-key nodes')
        const int avg = m > 0 ? (K - (n - m) + m - 1) / m : 0;
        if (m > 0) divide_nodes(oct_team<NT>(m, avg), S, m, 1);
        // sort(vPrev) by (size, node) ascending and walk from the back: rank 0 = largest size,
        // ties -> later allocation first (pointer order of a monotonic allocator)
        // (cnt, alloc) packed as cnt << 16 | alloc (alloc < 2^16, cnt < 2^15) in s_push,
        // which is free until the push order is written
        for (int j = tid; j < m; j += NT) {
            const int k = s_work[j];
            s_push[j] = (int)(((uint32_t)S.cnt[k] << 16) | (uint32_t)S.alloc[k]);   // used when K < 2^15
        }
        obar();
        if (K < 32768 && alloc_ctr < 65536) {
            for (int j = tid; j < m; j += NT) {
                const int kj = s_push[j];
                int rank = 0;
#pragma unroll 8
                for (int i = 0; i < m; i++) rank += s_push[i] > kj;
                s_rank[j] = rank;
            }
        } else {
            for (int j = tid; j < m; j += NT) {
                const int k = s_work[j];
                const int cj = S.cnt[k], aj = S.alloc[k];
                int rank = 0;
                for (int i = 0; i < m; i++) {
                    const int ki = s_work[i];
                    const int ci = S.cnt[ki], ai = S.alloc[ki];
                    rank += (ci > cj) || (ci == cj && ai > aj);
                }
                s_rank[j] = rank;
            }
        }
        obar();
        for (int j = tid; j < m; j += NT) s_base[s_rank[j]] = j;
        obar();
        // list size after processing rank r is n + sum_{r'<=r}(e-1); the first r reaching N breaks
        int nproc = m;
        {
            int carry = 0, found = 0x7fffffff;
            for (int base = 0; base < m; base += NT) {
                const int r = base + tid;
                int d = 0;
                if (r < m) {
                    const int4 q = s_cnt[s_base[r]];
                    d = (q.x > 0) + (q.y > 0) + (q.z > 0) + (q.w > 0) - 1;
                }
                int tot;
                const int pre = block_scan_excl<NW>(d, &tot, sbuf);
                if (r < m && n + carry + pre + d >= N) found = min(found, r);
                carry += tot;
            }
            int fr = found;
            for (int o = 32; o > 0; o >>= 1) fr = min(fr, __shfl_xor(fr, o, 64));
            if (lane == 0) sbuf[wv] = fr;
            obar();
            int mn = 0x7fffffff;
            for (int i = 0; i < NW; i++) mn = min(mn, sbuf[i]);
            obar();
            if (mn != 0x7fffffff) nproc = mn + 1;
        }
        // push order = processing order, children n1..n4 nonempty
        int T = 0;
        for (int base = 0; base < nproc; base += NT) {
            const int r = base + tid;
            int e = 0;
            if (r < nproc) {
                const int4 q = s_cnt[s_base[r]];
                e = (q.x > 0) + (q.y > 0) + (q.z > 0) + (q.w > 0);
            }
            int tot;
            const int pre = block_scan_excl<NW>(e, &tot, sbuf);
            if (r < nproc) s_push[r] = T + pre;
            T += tot;
        }
        for (int j = tid; j < m; j += NT)
            if (s_rank[j] < nproc) s_dead[s_work[j]] = 1;
        obar();
        const int nnew = T + n - nproc;
        if (nnew > g.ncap) { if (tid == 0) atomicOr(b.err, 4); break; }
        // DivideNode of the processed nodes (the largest: teams sized for the mean vPrev node
        // at least), then push_front of their children (one lane per node)
        divide_nodes(oct_team<NT>(nproc, avg), S, nproc, 2);
        for (int r = tid; r < nproc; r += NT) {
            const int j = s_base[r];
            const int k = s_work[j];
            const int s = S.start[k], bf = S.buf[k];
            const int4 pr = S.rect[k];
            const int4 qc = s_cnt[j];
            {
                int a = s_push[r];
                int off = s;
                const int qq[4] = {qc.x, qc.y, qc.z, qc.w};
                for (int c4 = 0; c4 < 4; c4++) {
                    if (qq[c4] > 0) {
                        const int pos = T - 1 - a;
                        int4 cr; int ssx, ssy;
                        child_rect(pr, c4, &cr, &ssx, &ssy);
                        D.start[pos] = off; D.cnt[pos] = qq[c4]; D.alloc[pos] = alloc_ctr + a;
                        D.buf[pos] = bf ^ 1; D.rect[pos] = cr;
                        a++;
                    }
                    off += qq[c4];
                }
            }
        }
        // erase processed nodes, keep the rest in list order behind the children
        {
            int carry = 0;
            for (int base = 0; base < n; base += NT) {
                const int k = base + tid;
                const bool keep = k < n && !s_dead[k];
                int tot;
                const int pre = block_scan_flag<NW>(keep, &tot, sbuf);
                if (keep) {
                    const int pos = T + carry + pre;
                    D.start[pos] = S.start[k]; D.cnt[pos] = S.cnt[k]; D.alloc[pos] = S.alloc[k];
                    D.buf[pos] = S.buf[k]; D.rect[pos] = S.rect[k];
                }
                carry += tot;
            }
        }
        obar();
        alloc_ctr += T;
        n = nnew;
        cs ^= 1;
        if (n >= N || n == prevSize) finish = true;
    }
    if (COEB_OCT_CLOCK) oc_t2 = (long long)clock64();

    // ---- 4. retain the best response per node (:747-766), border, final cull ----
    NodeRef S = nref(O, cs);
    uint32_t* out = b.lvl_kp + (int64_t)f * P->lvl_stride + g.out_off;
    const bool cull = !area && l < 8;                  // CheckMovingKeyPoints_finall loops 8 levels
    const float scale = (l != 0) ? g.scale : 1.0f;
    int carry = 0;
    for (int base = 0; base < n; base += NT) {
        const int k = base + tid;
        uint32_t best = 0;
        bool keep = false;
        if (k < n) {
            const uint32_t* src = KB(S.buf[k]) + S.start[k];
            const int c = S.cnt[k];
            best = src[0];
            int maxr = key_s(best);
            for (int q = 1; q < c; q++) {
                const uint32_t kk = src[q];
                if (key_s(kk) > maxr) { best = kk; maxr = key_s(kk); }
            }
            const int x = key_x(best) + 16, y = key_y(best) + 16;   // :886-887 (minBorderX/Y)
            best = pack_key(x, y, key_s(best));
            keep = !(cull && masked_out(dm, (float)x, (float)y, scale, P->W, P->H));
        }
        int tot;
        const int pre = block_scan_flag<NW>(keep, &tot, sbuf);
        if (keep) {
            if (carry + pre < g.out_cap) out[carry + pre] = best;
            else atomicOr(b.err, 8);
        }
        carry += tot;
    }
    if (tid == 0) b.lvl_n[(int64_t)f * P->L + l] = min(carry, g.out_cap);
    if (COEB_OCT_CLOCK && tid == 0) {
        const int wg = blockIdx.x + gridDim.x * blockIdx.y;
        if (wg < 4096) {
            long long* r = g_oct_clk + 6 * wg;
            r[0] = l; r[1] = K; r[2] = oc_w0;
            r[3] = (long long)clock64() - oc_t0; r[4] = oc_t1 - oc_t0; r[5] = oc_t2 - oc_t1;
        }
    }
}

// ================================ k_describe ================================
// IC_Angle on the unblurred level, fastAtan2, canonical sincosf, 256 rBRIEF tests on the
// blurred level, output in cv::KeyPoint layout.
__device__ float fast_atan2_dev(float y, float x)
{
    const float p1 = 0.9997878412794807f * (float)(180 / 3.1415926535897932384626433832795);
    const float p3 = -0.3258083974640975f * (float)(180 / 3.1415926535897932384626433832795);
    const float p5 = 0.1555786518463281f * (float)(180 / 3.1415926535897932384626433832795);
    const float p7 = -0.04432655554792128f * (float)(180 / 3.1415926535897932384626433832795);
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.2204460492503131e-16);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)2.2204460492503131e-16);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// canonical sincosf, identical operation sequence to the oracle
__device__ void sincos_canon(float af, float* s, float* c)
{
    const double two_over_pi = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_1t = 6.07710050650619224932e-11;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double x = (double)af;
    const double kd = rint(x * two_over_pi);
    double r = __builtin_fma(-kd, pio2_1, x);
    r = __builtin_fma(-kd, pio2_1t, r);
    const double z = r * r;
    const double v = z * r;
    const double sr = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double sn = r + v * (S1 + z * sr);
    const double cr = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double cs = w + (((1.0 - w) - hz) + z * cr);
    const int q = ((int)kd) & 3;
    double so, co;
    if (q == 0) { so = sn; co = cs; }
    else if (q == 1) { so = cs; co = -sn; }
    else if (q == 2) { so = -sn; co = -cs; }
    else { so = -cs; co = sn; }
    *s = (float)so;
    *c = (float)co;
}

struct KeyPointOut { float x, y, size, angle, response; int octave, class_id; };

// KP keypoints of one frame per wave (KP = 8 by default), in three phases:
//   A  kDescLpk = 64/KP lanes per keypoint: IC_Angle from 16-byte row loads of the unblurred
//      level, half of the lanes taking rows -|v| and half +|v|, each lane KP/2 rows; every row is
//      realigned in registers so byte j is patch column j-15, masked with the disc row |v| (a
//      17 x 32 B table in LDS: the rows differ across lanes) and summed by two v_dot4_u32_u8
//      per 4-pixel group, then reduced over the keypoint's lanes.  fastAtan2 and the canonical
//      sincosf run on every lane of the keypoint; the cv::KeyPoint record is written here.
//   B  kDescGroup keypoints per step: their 37 x 64 B blurred patches are staged in the wave's
//      LDS slab (the next group's are loaded into registers meanwhile); lane = 4 of the 256
//      tests of each; the nibbles are OR-combined by DPP into the descriptor dwords (LDS).
//   C  the wave's descriptors (KP x 32 B) are written out with 16-byte stores.
// Few keypoints per wave so that one XCD's resident waves cover few frames: a frame's level and
// blur images (~1.4 MB of patch rows) then stay in that XCD's 4 MB L2 while its neighbouring
// patches are read.  With 32 keypoints per wave an XCD had ~20 frames in flight and refetched
// every patch row (4.6 MB per frame past L2 vs 0.95 MB when only ~2 frames were in flight,
// tools/_exp_l2.sh).
// Few wide loads per keypoint: with one byte per lane per load (lane = patch column) the
// texture-address path, not the VALU, bounded this kernel.
// The rotated pattern offsets are cvRound of |(px, py)| <= 13*sqrt(2), so |offset| <= 18.
// Patch rows are 64 source bytes at an LDS pitch of 72 (18 dwords): consecutive rows land on
// different banks, so the 64 lanes' scattered test samples rarely conflict (a 64-byte pitch put
// every other row on the same 16 banks).
constexpr int kBlRow = 72, kBlRows = 37;
constexpr int kDescGroup = 2;                                        // patches staged per step
constexpr int kDescIcBatch = 32;   // IC row-chunk loads in flight per lane (>= the tasks per lane: all at once)
#ifndef COEB_DESC_KP
// keypoints per wave: 8 is the fastest alone (0.537 vs 0.568 ms per 1025-frame launch for 16) and
// in the steps of configs B, C and D (16: -6 %, -3 %, -1 %); 16 wins only config A's step
// (+1 %, profiles/r05/s13-s17)
#define COEB_DESC_KP 8
#endif
template <int KP> constexpr int desc_slab() { return kBlRow * kBlRows * kDescGroup + 32 * KP; }
constexpr int kUmax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};   // ORBextractor.cc:461-476

// Disc mask of row |v| = av (av 16: all zero), dword d of the realigned row (patch columns
// j = 4d..4d+3, u = j - 15): byte 0xFF where |u| <= umax[av].
__device__ __forceinline__ uint32_t ic_mask(int av, int d)
{
    uint32_t w = 0;
    for (int i = 0; i < 4; i++) {
        const int u = 4 * d + i - 15;
        if (av < 16 && (u < 0 ? -u : u) <= kUmax[av]) w |= 0xFFu << (8 * i);
    }
    return w;
}

__device__ __forceinline__ uint32_t dpp_or_xor1(uint32_t v)   // quad_perm [1,0,3,2]
{
    return v | (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_or_xor2(uint32_t v)   // quad_perm [2,3,0,1]
{
    return v | (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_or_shl4(uint32_t v)   // lane i |= lane i+4 (row_shl:4)
{
    return v | (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x104, 0xf, 0xf, false);
}

// One IC row: 48 bytes from 16-byte aligned `rp` (kVec) or byte loads.
template <bool kVec>
__device__ __forceinline__ void ic_row_load(const uint8_t* rp, uint4& c0, uint4& c1, uint4& c2)
{
    if (kVec) {
        c0 = reinterpret_cast<const uint4*>(rp)[0];
        c1 = reinterpret_cast<const uint4*>(rp)[1];
        c2 = reinterpret_cast<const uint4*>(rp)[2];
    } else {
        uint32_t q[12];
#pragma unroll
        for (int k = 0; k < 12; k++)
            q[k] = (uint32_t)rp[4 * k] | ((uint32_t)rp[4 * k + 1] << 8) | ((uint32_t)rp[4 * k + 2] << 16) |
                   ((uint32_t)rp[4 * k + 3] << 24);
        c0 = make_uint4(q[0], q[1], q[2], q[3]);
        c1 = make_uint4(q[4], q[5], q[6], q[7]);
        c2 = make_uint4(q[8], q[9], q[10], q[11]);
    }
}

template <bool kVec0, int KP>
// (24 waves per CU, a launch bound of 6 blocks: 80 VGPRs, 3 spilled, measured 0.253 vs 0.212 ms/step)
__global__ __launch_bounds__(kThreads) void k_describe(const Plan* __restrict__ P, ExtractBufs b)
{
    constexpr int kLpk = 64 / KP;          // lanes per keypoint in phase A
    constexpr int kHl = kLpk / 2;          // lanes per half (rows -|v| / +|v|)
    constexpr int kNr = 16 / kHl;          // IC rows per lane
    constexpr int kNb = kNr < 4 ? kNr : 4; // rows whose loads are in flight together
    static_assert(KP >= 2 && KP <= 32 && (KP & (KP - 1)) == 0, "KP: power of two in [2, 32]");
    __shared__ __attribute__((aligned(16))) uint8_t s_slab[kWaves][desc_slab<KP>()];
    __shared__ __attribute__((aligned(16))) uint32_t s_msk[17][8];
    if (threadIdx.x < 17 * 8) s_msk[threadIdx.x >> 3][threadIdx.x & 7] = ic_mask(threadIdx.x >> 3, threadIdx.x & 7);
    __syncthreads();
    const int2 bxy = block_xy();
    const int f = bxy.y;
    const int L = P->L;
    const int lane = lane_id(), wv = wave_id();
    // per-level keypoint offsets (wave prefix over lanes 0..L-1)
    const int nl = lane < L ? b.lvl_n[(int64_t)f * L + lane] : 0;
    int incl = nl;
    for (int o = 1; o < COEB_MAXL; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const int total = __builtin_amdgcn_readlane(incl, L - 1);
    if (bxy.x == 0 && threadIdx.x == 0) b.counts[f] = total;
    const int idx0 = (bxy.x * kWaves + wv) * KP;
    if (idx0 >= total) return;
    const int nk = min(KP, total - idx0);
    // ---- phase A: lanes kq*kLpk .. +kLpk-1 = keypoint idx0 + kq (excess repeat the last one, no writes)
    const int kq = lane / kLpk, half = (lane / kHl) & 1, qi = lane % kHl;
    const int id = idx0 + min(kq, nk - 1);
    int l = 0, start = 0;
    for (int q = 0; q < L - 1; q++) {
        const int e = __builtin_amdgcn_readlane(incl, q);      // end of level q
        if (id >= e) { l = q + 1; start = e; }
    }
    const LevelGeom& g = P->lv[l];
    const uint32_t key = b.lvl_kp[(int64_t)f * P->lvl_stride + g.out_off + (id - start)];
    const int x = key_x(key), y = key_y(key), sc = key_s(key);
    const uint8_t* img = level_ptr(P, b, f, l);
    // IC_Angle (ORBextractor.cc:80-107): A = sum j*p, S = sum p over the disc, m01 = sum v*rowsum;
    // lane (half, qi) takes rows |v| = qi + kHl*i, i < kNr (row 0 in the lower half only)
    uint32_t A = 0, S = 0;
    int m01 = 0;
    const int a = (x - 15) & 15;
    const uint32_t m8 = (a & 8) ? 0xFFFFFFFFu : 0u, m4 = (a & 4) ? 0xFFFFFFFFu : 0u;
    const uint8_t* rowp = img + (int64_t)y * g.pitch + (x - 15 - a);         // row v = 0
    const int64_t spitch = half ? (int64_t)g.pitch : -(int64_t)g.pitch;      // rows +|v| / -|v|
    const bool vec = kVec0 || l != 0;
    int aoff = 15;                             // m10 = A - aoff * S
    if (vec) {
        // lane (kq, j) takes tasks r = j + kLpk i of its keypoint, r = 3 row + chunk: image row
        // y + row - 15, 16-byte chunk `chunk` of the 48 bytes from x - 15 - a.  One load
        // instruction then covers ~kLpk / 3 whole rows of each keypoint rather than one chunk of
        // kLpk rows: a third of the distinct L1 lines per instruction (the row-per-lane form kept
        // the address unit busy 77 % of the kernel, stalled on the L1 half of it).  The disc mask
        // is formed per byte from u = column - x, the column weights are u + 31 (in [1, 63], so
        // packed bytes never carry) and m01 takes v * (row sum) directly.
        constexpr int kTasks = (93 + kLpk - 1) / kLpk;
        // loads in flight per batch (kDescIcBatch: all kTasks, or fewer for fewer VGPRs)
        constexpr int kBatch = kDescIcBatch < kTasks ? kDescIcBatch : kTasks;
        constexpr uint64_t kUmaxPk = 0x3689ABCDDEEEFFFFull;     // umax[av] in nibble av (kUmax)
        const int j = lane % kLpk;
        const uint8_t* base0 = img + (int64_t)(y - 15) * g.pitch + (x - 15 - a);
#pragma unroll
        for (int i0 = 0; i0 < kTasks; i0 += kBatch) {
        uint4 cq[kBatch];
#pragma unroll
        for (int ii = 0; ii < kBatch; ii++) {
            const int i = i0 + ii;
            if (i >= kTasks) break;
            const int r = min(j + kLpk * i, 92);
            const int row = r / 3, ch = r - 3 * row;
            cq[ii] = *reinterpret_cast<const uint4*>(base0 + (int64_t)row * g.pitch + 16 * ch);
        }
#pragma unroll
        for (int ii = 0; ii < kBatch; ii++) {
            const int i = i0 + ii;
            if (i >= kTasks) break;
            const int r = j + kLpk * i;
            if (r < 93) {
                const int row = r / 3, ch = r - 3 * row;
                const int v = row - 15, av = v < 0 ? -v : v;
                const int um = (int)((kUmaxPk >> (4 * av)) & 15u);
                const uint32_t q[4] = {cq[ii].x, cq[ii].y, cq[ii].z, cq[ii].w};
                uint32_t rs = 0;
#pragma unroll
                for (int d = 0; d < 4; d++) {
                    const int u0 = 16 * ch + 4 * d - a - 15;        // u of the dword's first byte
                    const int s0 = min(max(-um - u0, 0), 4), e0 = min(max(um - u0 + 1, 0), 4);
                    const uint32_t msk = (uint32_t)((1ull << (8 * e0)) - 1ull) & ~(uint32_t)((1ull << (8 * s0)) - 1ull);
                    const uint32_t pm = q[d] & msk;
                    A = __builtin_amdgcn_udot4(pm, (uint32_t)(u0 + 31) * 0x01010101u + 0x03020100u, A, false);
                    rs = __builtin_amdgcn_udot4(pm, 0x01010101u, rs, false);
                }
                S += rs;
                m01 += v * (int)rs;
            }
        }
        }
        aoff = 31;
    } else {
#pragma unroll
    for (int i0 = 0; i0 < kNr; i0 += kNb) {
        uint4 c[kNb][3];
#pragma unroll
        for (int r = 0; r < kNb; r++) {
            const uint8_t* rp = rowp + (qi + kHl * (i0 + r)) * spitch;
            if (vec) ic_row_load<true>(rp, c[r][0], c[r][1], c[r][2]);
            else ic_row_load<false>(rp, c[r][0], c[r][1], c[r][2]);
        }
#pragma unroll
        for (int r = 0; r < kNb; r++) {
            const int av = qi + kHl * (i0 + r);
            const uint32_t* msk = s_msk[(av == 0 && half) ? 16 : av];
            const uint32_t q[12] = {c[r][0].x, c[r][0].y, c[r][0].z, c[r][0].w, c[r][1].x, c[r][1].y,
                                    c[r][1].z, c[r][1].w, c[r][2].x, c[r][2].y, c[r][2].z, c[r][2].w};
            // realign by a: bit selects, then alignbyte
            uint32_t r1[10], r2[9];
#pragma unroll
            for (int k = 0; k < 10; k++) r1[k] = (m8 & q[k + 2]) | (~m8 & q[k]);
#pragma unroll
            for (int k = 0; k < 9; k++) r2[k] = (m4 & r1[k + 1]) | (~m4 & r1[k]);
            uint32_t rs = 0;
#pragma unroll
            for (int d = 0; d < 8; d++) {
                const uint32_t pm = __builtin_amdgcn_alignbyte(r2[d + 1], r2[d], (uint32_t)(a & 3)) & msk[d];
                A = __builtin_amdgcn_udot4(pm, 0x03020100u + 0x04040404u * (uint32_t)d, A, false);
                rs = __builtin_amdgcn_udot4(pm, 0x01010101u, rs, false);
            }
            S += rs;
            m01 += av * (int)rs;
        }
    }
        if (half == 0) m01 = -m01;             // lower half: rows -|v|
    }
#pragma unroll
    for (int o = 1; o < kLpk; o <<= 1) {
        A += __shfl_xor(A, o, 64);
        S += __shfl_xor(S, o, 64);
        m01 += __shfl_xor(m01, o, 64);
    }
    const int m10 = (int)A - aoff * (int)S;
    const float angle = fast_atan2_dev((float)m01, (float)m10);
    const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
    float bs, ac;
    sincos_canon(angle * factorPI, &bs, &ac);
    if (lane % kLpk == 0 && kq < nk) {   // cv::KeyPoint {x, y, size, angle, response, octave, class_id}
        float fx = (float)x, fy = (float)y;
        if (l != 0) { fx *= g.scale; fy *= g.scale; }          // :1327-1334
        KeyPointOut o;
        o.x = fx; o.y = fy; o.size = (float)g.size_i; o.angle = angle; o.response = (float)sc;
        o.octave = l; o.class_id = -1;
        reinterpret_cast<KeyPointOut*>(b.kps)[(int64_t)f * P->kcap + idx0 + kq] = o;
    }
    // ---- phase B: descriptors (ORBextractor.cc:109-156), kDescGroup keypoints per step
    const int4 pa = reinterpret_cast<const int4*>(b.pattern)[lane];   // tests 4*lane .. 4*lane+3
    float px0[4], py0[4], px1[4], py1[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int pw = t == 0 ? pa.x : t == 1 ? pa.y : t == 2 ? pa.z : pa.w;
        px0[t] = (float)(int8_t)(pw & 0xff); py0[t] = (float)(int8_t)((pw >> 8) & 0xff);
        px1[t] = (float)(int8_t)((pw >> 16) & 0xff); py1[t] = (float)(int8_t)(pw >> 24);
    }
    uint8_t* slab = s_slab[wv];
    uint32_t* dsl = reinterpret_cast<uint32_t*>(slab + kBlRow * kBlRows * kDescGroup);
    const int xoff = x - ((x - 18) & ~15);        // patch column of the keypoint
    const uint8_t* blur_f = b.blur + (int64_t)f * P->blur_stride;
    static_assert(kDescGroup == 2, "staging below is written for 2 patches per step");
    uint4 qa0, qa1, qa2, qb0, qb1, qb2;
    // Patch = rows y-18 .. y+18 x the 64 bytes from (x-18) & ~15 of the tiled blurred level: 4 tile
    // columns x (5 or 6) tile rows of 8.  Load e (of 192, three per lane) = tile row e >> 5, tile
    // column (e >> 3) & 3, row e & 7 inside the tile: 8 consecutive lanes read one whole 128-B
    // line, so an instruction touches 8 lines (row-major: ~22 half-used ones).  Patch row =
    // 8 * tile row + (e & 7) - dy; rows outside 0..36 are loaded but not staged.
    const int ty0 = (y - 18) >> 3, dy = (y - 18) & 7, tymax = ((y + 18) >> 3) - ty0;
    const int porg = (int)g.blur_off + (int)blur_tile_off((x - 18) & ~15, ty0 * 8, g.bpitch);
    const int trs = g.bpitch * 8;                 // bytes per tile row
    const int lo = ((lane >> 3) & 3) * 128 + (lane & 7) * 16;   // the lane's tile column and row
    const int tr0 = lane >> 5;                    // tile row of load 0 (loads 1, 2: + 2, + 4)
#define COEB_LOAD_PATCH(t, q0, q1, q2)                                                          \
    {                                                                                           \
        const int tt_ = min((t), nk - 1);                                                       \
        const uint8_t* o_ = blur_f + __builtin_amdgcn_readlane(porg, tt_ * kLpk) + lo;          \
        const int trs_ = __builtin_amdgcn_readlane(trs, tt_ * kLpk);                            \
        const int tm_ = __builtin_amdgcn_readlane(tymax, tt_ * kLpk);                           \
        q0 = *reinterpret_cast<const uint4*>(o_ + min(tr0, tm_) * trs_);                        \
        q1 = *reinterpret_cast<const uint4*>(o_ + min(tr0 + 2, tm_) * trs_);                    \
        q2 = *reinterpret_cast<const uint4*>(o_ + min(tr0 + 4, tm_) * trs_);                    \
    }
    COEB_LOAD_PATCH(0, qa0, qa1, qa2)
    COEB_LOAD_PATCH(1, qb0, qb1, qb2)
    for (int t0 = 0; t0 < nk; t0 += kDescGroup) {
        {
            // a 16-byte chunk into slab row `row`, bytes 16 c .. +15 (two 8-byte stores: the pitch is
            // 8-aligned)
            auto put = [&](uint8_t* base, int row, int c, uint4 v) {
                uint2* d = reinterpret_cast<uint2*>(base + row * kBlRow + 16 * c);
                d[0] = make_uint2(v.x, v.y);
                d[1] = make_uint2(v.z, v.w);
            };
            uint8_t* pb = slab + kBlRow * kBlRows;
            const int dya = __builtin_amdgcn_readlane(dy, min(t0, nk - 1) * kLpk);
            const int dyb = __builtin_amdgcn_readlane(dy, min(t0 + 1, nk - 1) * kLpk);
            const int c = (lane >> 3) & 3, r = 8 * tr0 + (lane & 7);
            auto put_t = [&](uint8_t* base, int row, uint4 v) {
                if ((unsigned)row < (unsigned)kBlRows) put(base, row, c, v);
            };
            put_t(slab, r - dya, qa0);
            put_t(slab, r + 16 - dya, qa1);
            put_t(slab, r + 32 - dya, qa2);
            put_t(pb, r - dyb, qb0);
            put_t(pb, r + 16 - dyb, qb1);
            put_t(pb, r + 32 - dyb, qb2);
        }
        wave_sync_lds();
        if (t0 + kDescGroup < nk) {
            COEB_LOAD_PATCH(t0 + 2, qa0, qa1, qa2)
            COEB_LOAD_PATCH(t0 + 3, qb0, qb1, qb2)
        }
#pragma unroll
        for (int k = 0; k < kDescGroup; k++) {
            const int t = t0 + k;
            if (t >= nk) break;
            const float tb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bs), t * kLpk));
            const float ta = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ac), t * kLpk));
            const uint8_t* bc = slab + k * kBlRow * kBlRows + 18 * kBlRow + __builtin_amdgcn_readlane(xoff, t * kLpk);
            // (row, col) = (fma(px, b, py*a), fma(px, a, -(py*b))) as packed-f32 pairs: the same
            // two roundings per component as the reference's fused forms, half the instructions
            const f32x2 AB = {ta, tb}, BA = {tb, ta};
            uint32_t nib = 0;
#pragma unroll
            for (int tt = 0; tt < 4; tt++) {
                const f32x2 t0 = f32x2{py0[tt], py0[tt]} * AB, t1 = f32x2{py1[tt], py1[tt]} * AB;
                const f32x2 rc0 = __builtin_elementwise_fma(f32x2{px0[tt], px0[tt]}, BA, f32x2{t0.x, -t0.y});
                const f32x2 rc1 = __builtin_elementwise_fma(f32x2{px1[tt], px1[tt]}, BA, f32x2{t1.x, -t1.y});
                // cvRound, then row * pitch + col exactly in f32 (|row|, |col| <= 18)
                const int o0 = (int)__builtin_fmaf(rintf(rc0.x), (float)kBlRow, rintf(rc0.y));
                const int o1 = (int)__builtin_fmaf(rintf(rc1.x), (float)kBlRow, rintf(rc1.y));
                nib |= (uint32_t)(bc[o0] < bc[o1]) << tt;
            }
            // bit k of byte i = test 8i+k: dword d = nibbles of lanes 8d .. 8d+7
            uint32_t dw = nib << (4 * (lane & 7));
            dw = dpp_or_shl4(dpp_or_xor2(dpp_or_xor1(dw)));
            if ((lane & 7) == 0) dsl[8 * t + (lane >> 3)] = dw;
        }
        wave_sync_lds();                         // patch reads done before the next staging
    }
#undef COEB_LOAD_PATCH
    // ---- phase C: descriptors out
    uint4* gd = reinterpret_cast<uint4*>(b.desc + ((int64_t)f * P->kcap + idx0) * 32);
    if (lane < 2 * nk) gd[lane] = reinterpret_cast<const uint4*>(dsl)[lane];
}

}  // namespace

// Per-cell phase clocks of k_fast (COEB_FAST_CLOCK builds), summed over the 256 slot copies;
// read and cleared.
int fast_timing_read(unsigned long long* out)
{
    static unsigned long long h[256 * 8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_fast_clk), sizeof(h)) != hipSuccess) return -1;
    for (int k = 0; k < 8; k++) {
        out[k] = 0;
        for (int i = 0; i < 256; i++) out[k] += h[i * 8 + k];
    }
    static const unsigned long long z[256 * 8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_fast_clk), z, sizeof(z)) == hipSuccess ? 0 : -1;
}

// k_octree per-workgroup clocks (COEB_OCT_CLOCK builds): 4096 x 6 long long, see g_oct_clk
int oct_timing_read(long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_oct_clk), sizeof(long long) * 4096 * 6) == hipSuccess ? 0 : -1;
}

int launch_extract(const Plan& plan, const Plan* d_plan, const ExtractBufs& b, int F, hipStream_t s,
                   ProfileHook* prof, const SideStream* side)
{
    prof_begin(prof, "k_dynmask", s);
    hipLaunchKernelGGL(k_dynmask, dim3((F + 63) / 64), dim3(64), 0, s, b, F, plan.W, plan.H);
    prof_end(prof, s);
    BlurWork bw;
    bw.L = plan.L;
    int items = 0;
    // 32-row bands (round 4: 0.487 ms per 1025-frame launch; the strip-per-lane k_blur it replaced
    // took 0.759, and was deleted in round 6)
    const int brows = 32;
    static_assert(brows % 8 == 0, "bands start on tile rows");
    bw.brows = brows;
    for (int l = 0; l < plan.L; l++) {
        const LevelGeom& g = plan.lv[l];
        bw.nstrips[l] = (g.w + kBlurCols - 1) / kBlurCols;
        bw.item_off[l] = items;
        bw.nquads[l] = (bw.nstrips[l] + 3) / 4;
        bw.bh[l] = 0;
        items += bw.nquads[l] * ((g.h + brows - 1) / brows);
    }
    bw.item_off[plan.L] = items;
    // COEB_PYR_BYTES=1 forces k_pyr_level's byte form for every level (tests run both forms)
    const char* pb = coeb_switch("COEB_PYR_BYTES");
    const bool pyr_bytes = pb && atoi(pb) != 0;
    // COEB_FAST_RB=72 forces the general slab layout (tests run both layouts)
    const char* frb = coeb_switch("COEB_FAST_RB");
    const int fast_rbytes = frb && atoi(frb) == kFastRowBytes ? kFastRowBytes : fast_rb(plan);
    const int fast_lds = kWaves * fast_wave_lds(plan, fast_rbytes);
    constexpr int kFastPerBlock = kWaves;
    auto blur = [&](hipStream_t st, int i0, int i1) {
        if (i1 <= i0) return;
        BlurWork w = bw;
        w.item0 = i0; w.item1 = i1;
        prof_begin(prof, "k_blur", st);
        hipLaunchKernelGGL(k_blur_rows, dim3((i1 - i0 + kWaves - 1) / kWaves, F), dim3(kThreads), 0,
                           st, d_plan, b, w);
        prof_end(prof, st);
    };
    // FAST over levels [l0, l1): one wave per cell.  A band form (one LDS copy per cell-row
    // segment, each image row fetched once) measured slower and was removed.
    auto fast = [&](hipStream_t st, int l0, int l1) {
        l1 = std::min(l1, plan.L);
        if (l1 <= l0) return;
        prof_begin(prof, "k_fast", st);
        const int c0 = plan.lv[l0].cell0, c1 = l1 < plan.L ? plan.lv[l1].cell0 : plan.ncells;
        hipLaunchKernelGGL(fast_rbytes == kFastRowBytesM ? k_fast<kFastRowBytesM> : k_fast<kFastRowBytes>,
                           dim3((c1 - c0 + kFastPerBlock - 1) / kFastPerBlock, F), dim3(kThreads), fast_lds,
                           st, d_plan, b, b.cells, c0, c1);
        prof_end(prof, st);
    };
    // level 0 (the input frame itself) needs no pyramid: with a side stream its blur and FAST
    // overlap the cascaded pyramid launches, whose small late levels leave most CUs idle; levels
    // 1..m-1 follow on the side stream as soon as the pyramid has built them
    const bool split = side && side->s && plan.L > 1;
    const int m = split ? std::min(std::max(side->split, 1), plan.L) : 0;
    if (split) {
        (void)hipEventRecord(side->fork, s);                 // after k_dynmask (area_flag -> FAST thresholds)
        (void)hipStreamWaitEvent(side->s, side->fork, 0);
        blur(side->s, 0, bw.item_off[1]);
        fast(side->s, 0, 1);
    }
    for (int l = 1; l < plan.L; l++) {
        const LevelGeom& g = plan.lv[l];
        const LevelGeom& gp = plan.lv[l - 1];
        const uint8_t* src = l == 1 ? b.gray : b.pyr + gp.pyr_off;
        const int64_t src_fs = l == 1 ? (int64_t)plan.W * plan.H : plan.pyr_stride;
        prof_begin(prof, "k_pyr_level", s);
        // k_pyr_rows needs 4-byte aligned source rows and every 2-column window within 8 bytes
        // (g.rows_ok, make_plan: scale <= 2); otherwise the byte form
        const bool rows = g.rows_ok && ((gp.pitch | (int)(src_fs & 3) | (int)((uintptr_t)src & 3)) & 3) == 0;
        if (rows && !pyr_bytes) {
            hipLaunchKernelGGL(k_pyr_rows, dim3((g.w + PR_COLS - 1) / PR_COLS, (g.h + kWaves * PR_ROWS - 1) / (kWaves * PR_ROWS), F),
                               dim3(kThreads), 0, s, src, src_fs, gp.pitch, gp.h, b.pyr + g.pyr_off, plan.pyr_stride,
                               g.pitch, g.w, g.h, b.rtab + g.rtab_off, g.xmax, resize_simd_end(g.w),
                               reinterpret_cast<const int4*>(b.rtab + g.yrow_off));
        } else {
            int tsw, tsh;
            pyr_tile_lds(gp.w, gp.h, g.w, g.h, &tsw, &tsh);
            hipLaunchKernelGGL(k_pyr_level, dim3((g.w + PT_W - 1) / PT_W, (g.h + PT_H - 1) / PT_H, F), dim3(kThreads),
                               tsw * tsh, s, src, src_fs, gp.pitch, gp.w, gp.h, b.pyr + g.pyr_off, plan.pyr_stride,
                               g.pitch, g.w, g.h, b.rtab + g.rtab_off, g.xmax, resize_simd_end(g.w), tsw, tsh);
        }
        prof_end(prof, s);
        if (split && m > 1 && l == m - 1) {
            (void)hipEventRecord(side->mid, s);
            (void)hipStreamWaitEvent(side->s, side->mid, 0);
            blur(side->s, bw.item_off[1], bw.item_off[m]);
            fast(side->s, 1, m);
        }
    }
    constexpr int kOctThreads = 256;       // 512 / 1024 measured slower on large batches, 128 too (r06/s10)
    // Small batches (per-rank shards: fewer workgroups than two per CU): the key capacity in LDS
    // doubles (up to 4096 keys, within 150 KB), so a 1280x960 level 0 (~2 700 candidates) keeps
    // its keys in LDS instead of the global ping-pong buffers; large batches keep the plan's
    // capacity, which leaves more workgroups per CU.  (Level 0 as one 1024-thread workgroup and
    // the short upper levels as one-wave workgroups were both measured slower)
    // One frame (the single-frame path) with 1024 / 512 threads per workgroup: 1024 adds 5 us to
    // the frame's extract, 512 is within noise of 256 (r06/s38), so one size serves every batch.
    int oct_kl = plan.oct_kl, oct_lds = plan.oct_lds;
    if (F * plan.L <= 2 * 256) {
        int kl = oct_kl;
        while (kl < 4096 && plan.oct_w * (4 + 16 + 4 + 4 + 4 + 1 + 64) + 8 * (2 * kl) <= 150 * 1024) kl *= 2;
        oct_kl = kl;
        oct_lds = plan.oct_w * (4 + 16 + 4 + 4 + 4 + 1 + 64) + 8 * kl;
    }
    if (const char* e = coeb_experiment("COEB_OCT_KL_SMALL")) if (atoi(e) == 0) { oct_kl = plan.oct_kl; oct_lds = plan.oct_lds; }
    lds_limit_max((const void*)k_octree<kOctThreads>);
    auto octree = [&](hipStream_t st, int l0, int l1) {
        if (l1 <= l0) return;
        prof_begin(prof, "k_octree", st);
        hipLaunchKernelGGL(k_octree<kOctThreads>, dim3(F, l1 - l0), dim3(kOctThreads), oct_lds, st, d_plan, b, l0, plan.oct_w,
                           oct_kl);
        prof_end(prof, st);
    };
    // the late blur goes to the side stream (beside FAST / octree, which do not read it) and the
    // octree of the side levels follows their FAST there; s joins before the descriptors
    const bool late = split && side->blur_late;
    const bool soct = late && side->side_octree;
    if (soct) octree(side->s, 0, m);
    if (split) (void)hipEventRecord(side->join, side->s);
    if (late) {
        (void)hipEventRecord(side->pyr_done, s);
        (void)hipStreamWaitEvent(side->s, side->pyr_done, 0);
        blur(side->s, bw.item_off[m], items);
        (void)hipEventRecord(side->join2, side->s);
    } else {
        blur(s, split ? bw.item_off[m] : 0, items);
    }
    fast(s, split ? m : 0, plan.L);
    // one cross-stream wait on the critical path instead of two: each costs a ~6 us gap between
    // the launches it separates (rocprofv3 timeline), and the late blur ends well before FAST
    // does, so waiting for all of the side stream (join2) before the octree delays nothing
    if (soct) {
        octree(s, m, plan.L);
        (void)hipStreamWaitEvent(s, late ? side->join2 : side->join, 0);
    } else {
        if (split) (void)hipStreamWaitEvent(s, late ? side->join2 : side->join, 0);
        octree(s, 0, plan.L);
    }
    prof_begin(prof, "k_describe", s);
    const bool vec0 = plan.W % 16 == 0 && (reinterpret_cast<uintptr_t>(b.gray) & 15) == 0;
    // COEB_DESC_KP keypoints per wave (round 1's 32 let one XCD's resident waves span ~20 frames
    // and refetch every patch row past L2; 4 and 16 are slower alone, and 16 is slower in three of
    // the four configs' steps)
    constexpr int KP = COEB_DESC_KP;
    if (vec0)
        hipLaunchKernelGGL((k_describe<true, KP>), dim3((plan.kcap + kWaves * KP - 1) / (kWaves * KP), F), dim3(kThreads), 0,
                           s, d_plan, b);
    else
        hipLaunchKernelGGL((k_describe<false, KP>), dim3((plan.kcap + kWaves * KP - 1) / (kWaves * KP), F), dim3(kThreads), 0,
                           s, d_plan, b);
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
