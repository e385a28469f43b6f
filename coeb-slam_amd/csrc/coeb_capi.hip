// coeb_capi.hip -- context, host-side geometry plan and the C-ABI of include/coeb_front.h.
//
// Host work here is O(levels + cells) per image size (cached), plus the per-call argument
// marshalling.  All per-pixel / per-keypoint work runs in the kernels of coeb_extract.hip and
// coeb_match.hip.  There is no CPU fallback: without a usable gfx950 device coeb_create fails.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/coeb_front.h"
#include "coeb_internal.hpp"

static const int8_t kPattern[1024] = {
#include "../../data/orb_bit_pattern_31.inc"
};

// per host thread: ranks of `bench.py --gpus N` (one thread per device) and threaded adapters call
// the library concurrently; coeb_last_error(NULL) returns the calling thread's last message
static thread_local std::string g_last_error;

// coeb_flow.hip
extern "C" int coeb_internal_flow_counts(coeb_ctx* c, int* out, int cap, int* npairs);
extern "C" void coeb_internal_flow_forget(const coeb_ctx* c);

namespace {

enum { PATCH_SIZE = 31, HALF_PATCH_SIZE = 15, EDGE_THRESHOLD = 19 };
constexpr int kRoiMax = 64;
constexpr int kFrameTmCap = 1024;     // T_M points per frame kept on the device (coeb_frame_batch_device)
constexpr int kCurMax = 4095;
constexpr int kMatchCQ = 64;   // candidate list entries per LastFrame point (coeb_match.hip kCQ)

inline int cv_round(float v) { return (int)lrintf(v); }
inline int cv_round_d(double v) { return (int)lrint(v); }
inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
inline int cv_ceil_d(double v) { int i = (int)v; return i + (i < v); }
inline int64_t align256(int64_t v) { return (v + 255) & ~int64_t(255); }

struct Tables {
    int nfeatures;
    double scale_factor;   // ORBextractor.h:114 `double scaleFactor`
    int nlevels;
    float scale[COEB_MAXL], inv_scale[COEB_MAXL], sigma2[COEB_MAXL], inv_sigma2[COEB_MAXL];
    int nfeat[COEB_MAXL];
    int umax[16];
};

// ORBextractor::ORBextractor (src/ORBextractor.cc:418-477)
bool make_tables(const coeb_orb_params& prm, Tables& t)
{
    if (prm.nlevels < 1 || prm.nlevels > COEB_MAXL || prm.nfeatures < 0 || !(prm.scale_factor > 0)) return false;
    memset(&t, 0, sizeof(t));
    t.nfeatures = prm.nfeatures;
    t.scale_factor = prm.scale_factor;
    t.nlevels = prm.nlevels;
    t.scale[0] = 1.0f;
    t.sigma2[0] = 1.0f;
    for (int i = 1; i < t.nlevels; i++) {
        t.scale[i] = (float)((double)t.scale[i - 1] * t.scale_factor);
        t.sigma2[i] = t.scale[i] * t.scale[i];
    }
    for (int i = 0; i < t.nlevels; i++) {
        t.inv_scale[i] = 1.0f / t.scale[i];
        t.inv_sigma2[i] = 1.0f / t.sigma2[i];
    }
    const float factor = (float)(1.0f / t.scale_factor);
    float ndesired = t.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)t.nlevels));
    int sum = 0;
    for (int l = 0; l < t.nlevels - 1; l++) {
        t.nfeat[l] = cv_round(ndesired);
        sum += t.nfeat[l];
        ndesired *= factor;
    }
    t.nfeat[t.nlevels - 1] = std::max(t.nfeatures - sum, 0);
    int v, v0;
    const int vmax = cv_floor(HALF_PATCH_SIZE * sqrtf(2.f) / 2 + 1);
    const int vmin = cv_ceil_d(HALF_PATCH_SIZE * sqrtf(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    for (v = 0; v <= vmax; ++v) t.umax[v] = cv_round_d(std::sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
        while (t.umax[v0] == t.umax[v0 + 1]) ++v0;
        t.umax[v] = v0;
        ++v0;
    }
    return true;
}

// Gaussian 7-tap sigma 2, Q8 error-diffused
void gauss_kernel7(int k[7])
{
    const int n = 7, n2 = 3;
    const double scale2X = -0.125 / (2.0 * 2.0);
    double values[3], sum = 0.0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        const double t = std::exp((double)(x * x) * scale2X);
        values[i] = t;
        sum += t;
    }
    sum = sum * 2.0 + 1.0;
    const double mul1 = 1.0 / sum;
    double err = 0.0;
    int64_t s = 0;
    for (int i = 0; i < n2; i++) {
        const double adj = values[i] * mul1 * 256.0 + err;
        const int64_t q = cv_round_d(adj);
        err = adj - (double)q;
        k[i] = k[n - 1 - i] = (int)q;
        s += q;
    }
    k[n2] = (int)(256 - 2 * s);
}

// cv::resize INTER_LINEAR coefficient tables (imgproc resize.cpp, 8U fixed point)
int resize_tables(int sw, int sh, int dw, int dh, std::vector<int>& tab)
{
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    const size_t base = tab.size();
    tab.resize(base + 2 * dw + 2 * dh);
    int* xofs = tab.data() + base;
    int* alpha = xofs + dw;
    int* yofs = alpha + dw;
    int* beta = yofs + dh;
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        const int a0 = std::max(-32768, std::min(32767, cv_round((1.f - fx) * 2048)));
        const int a1 = std::max(-32768, std::min(32767, cv_round(fx * 2048)));
        alpha[dx] = (a0 & 0xFFFF) | (a1 << 16);
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = cv_floor(fy);
        fy -= sy;
        yofs[dy] = sy;
        const int b0 = std::max(-32768, std::min(32767, cv_round((1.f - fy) * 2048)));
        const int b1 = std::max(-32768, std::min(32767, cv_round(fy * 2048)));
        beta[dy] = (b0 & 0xFFFF) | (b1 << 16);
    }
    return xmax;
}

bool make_plan(const Tables& t, int W, int H, Plan& P, std::vector<int>& rtab, std::vector<CellDesc>& cells,
               std::string& err)
{
    memset(&P, 0, sizeof(P));
    P.W = W; P.H = H; P.L = t.nlevels;
    rtab.clear();
    cells.clear();
    if (W > 4096 || H > 4096) { err = "image larger than 4096 px is not supported (12-bit key packing)"; return false; }
    int64_t pyr = 0, blur = 0, node = 0;
    int kcap_total = 0, out_total = 0, cell_cap = 1;
    for (int l = 0; l < t.nlevels; l++) {
        LevelGeom& g = P.lv[l];
        g.w = cv_round((float)W * t.inv_scale[l]);     // ComputePyramid :1349
        g.h = cv_round((float)H * t.inv_scale[l]);
        g.scale = t.scale[l];
        g.size_i = (int)(PATCH_SIZE * t.scale[l]);
        g.pitch = l == 0 ? W : (g.w + 63) & ~63;
        g.bpitch = (g.w + 63) & ~63;
        if (l == 0) g.pyr_off = -1;
        else { g.pyr_off = pyr; pyr = align256(pyr + (int64_t)g.pitch * g.h); }
        g.blur_off = blur;
        blur = align256(blur + (int64_t)g.bpitch * ((g.h + 7) & ~7));    // whole 8-row tiles
        if (l > 0) {
            while (rtab.size() % 4) rtab.push_back(0);     // 16-byte aligned table rows
            g.rtab_off = (int)rtab.size();
            g.xmax = resize_tables(P.lv[l - 1].w, P.lv[l - 1].h, g.w, g.h, rtab);
            g.rows_ok = 1;
            for (int c = 0; c < g.w; c += 2) {
                const int* xofs = rtab.data() + g.rtab_off;
                if (xofs[std::min(c + 1, g.w - 1)] - (xofs[c] & ~3) > 5) g.rows_ok = 0;
            }
            // k_pyr_rows' row descriptors: one 16-byte scalar load per output row
            while (rtab.size() % 4) rtab.push_back(0);
            g.yrow_off = (int)rtab.size();
            const int sh = P.lv[l - 1].h, sp = P.lv[l - 1].pitch;
            for (int dy = 0; dy < g.h; dy++) {
                const int q0 = rtab[g.rtab_off + 2 * g.w + dy], bb = rtab[g.rtab_off + 2 * g.w + g.h + dy];
                const int r0 = q0 >= 0 ? (q0 < sh ? q0 : sh - 1) : 0;
                const int r1 = q0 + 1 >= 0 ? (q0 + 1 < sh ? q0 + 1 : sh - 1) : 0;
                rtab.push_back(r0 * sp);
                rtab.push_back(r1 * sp);
                rtab.push_back(bb);
                rtab.push_back(dy * g.pitch);
            }
        }
        // FAST cells (ComputeKeyPointsOctTree :795-829)
        const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
        const int maxBorderX = g.w - EDGE_THRESHOLD + 3, maxBorderY = g.h - EDGE_THRESHOLD + 3;
        const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
        const float Wc = 30;
        g.ncols = (int)(width / Wc);
        g.nrows = (int)(height / Wc);
        if (g.ncols <= 0 || g.nrows <= 0) { err = "pyramid level too small for the 30-px FAST grid"; return false; }
        g.wcell = (int)ceilf(width / g.ncols);
        g.hcell = (int)ceilf(height / g.nrows);
        g.cell0 = (int)cells.size();
        for (int i = 0; i < g.nrows; i++) {
            const float iniY = (float)(minBorderY + i * g.hcell);
            float maxY = iniY + g.hcell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = (float)maxBorderY;
            for (int j = 0; j < g.ncols; j++) {
                const float iniX = (float)(minBorderX + j * g.wcell);
                float maxX = iniX + g.wcell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = (float)maxBorderX;
                CellDesc c;
                c.level = (int16_t)l; c.pad = 0;
                c.x0 = (int16_t)(int)iniX; c.y0 = (int16_t)(int)iniY;
                c.rw = (int16_t)((int)maxX - (int)iniX); c.rh = (int16_t)((int)maxY - (int)iniY);
                c.i = (int16_t)i; c.j = (int16_t)j;
                if (c.rw > kRoiMax || c.rh > kRoiMax) { err = "FAST cell ROI exceeds 64 px"; return false; }
                const int ww = std::max(0, c.rw - 6), wh = std::max(0, c.rh - 6);
                cell_cap = std::max(cell_cap, ((ww + 1) / 2) * ((wh + 1) / 2));
                P.max_roi_w = std::max(P.max_roi_w, (int)c.rw);
                P.max_roi_h = std::max(P.max_roi_h, (int)c.rh);
                cells.push_back(c);
            }
        }
        g.ncells = (int)cells.size() - g.cell0;
        // DistributeOctTree constants (:549-552, :866-875)
        g.nfeat = t.nfeat[l];
        g.nfeat_area = (int)((double)t.nfeat[l] * 0.7);
        g.maxX = maxBorderX - minBorderX;
        g.maxY = maxBorderY - minBorderY;
        g.nini = (int)roundf((float)g.maxX / g.maxY);
        if (g.nini < 1 || g.nini > 4) { err = "aspect ratio gives an unsupported number of initial octree nodes"; return false; }
        g.hx = (float)g.maxX / g.nini;
        int b = 0;
        for (int i = 0; i <= g.nini; i++) {
            while (b <= g.maxX + 1 && (int)((float)b / g.hx) < i) b++;
            g.ini_bound[i] = b;
        }
        g.ini_bound[g.nini] = 1 << 20;
        // list size never exceeds max(N + 2, 4 * nIni)
        g.out_cap = std::max(g.nfeat + 3, 4 * g.nini) + 5;
        g.ncap = g.out_cap + 8;
        g.node_off = node;
        node += 2 * 8 * (int64_t)g.ncap;
        g.out_off = out_total;
        out_total += g.out_cap;
    }
    P.ncells = (int)cells.size();
    P.cell_cap = cell_cap;
    for (int l = 0; l < t.nlevels; l++) {
        P.lv[l].kcap_off = kcap_total;
        P.lv[l].kcap = P.lv[l].ncells * cell_cap;
        kcap_total += P.lv[l].kcap;
    }
    P.pyr_stride = std::max<int64_t>(pyr, 256);
    P.blur_stride = blur;
    P.kbuf_stride = kcap_total;
    P.node_stride = node;
    P.lvl_stride = out_total;
    P.kcap = out_total;
    P.rtab_ints = (int)rtab.size();
    P.oct_w = 0;
    for (int l = 0; l < t.nlevels; l++) P.oct_w = std::max(P.oct_w, P.lv[l].ncap);
    P.oct_w = (P.oct_w + 15) & ~15;
    // keys kept in LDS per level (more candidates: global ping-pong buffers, slower but exact):
    // the power of two >= 4.5 x the largest level's features (FAST leaves ~3.8 candidates per
    // level-0 feature on the config-A frames: 818 median, 934 max for 217), so that config A's
    // octree needs 31 KB of LDS and five workgroups share a CU (0.091 -> 0.075 ms per step; 768
    // keys pushed level 0 to the global buffers, 0.102 ms); COEB_OCT_KL overrides
    int nmax = 0;
    for (int l = 0; l < t.nlevels; l++) nmax = std::max(nmax, P.lv[l].nfeat);
    P.oct_kl = 512;
    while (P.oct_kl < 4096 && P.oct_kl < (9 * nmax + 1) / 2) P.oct_kl *= 2;
    if (const char* e = coeb_experiment("COEB_OCT_KL")) P.oct_kl = std::max(256, std::min(8192, atoi(e)));
    P.oct_lds = P.oct_w * (4 + 16 + 4 + 4 + 4 + 1 + 64) + 8 * P.oct_kl;
    if (P.oct_lds > 150 * 1024) { err = "octree LDS budget exceeded (features per level too large)"; return false; }
    memcpy(P.umax, t.umax, sizeof(P.umax));
    // k_describe folds the IC_Angle disc (umax for HALF_PATCH_SIZE 15) into constants
    static const int kUmaxDisc[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
    if (memcmp(t.umax, kUmaxDisc, sizeof(kUmaxDisc)) != 0) { err = "unexpected IC_Angle disc (umax)"; return false; }
    gauss_kernel7(P.gauss);

    return true;
}

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
};

struct ProfImpl {
    bool enabled = false;
    std::vector<std::string> names;
    std::vector<double> ms;
    std::vector<int64_t> launches;
    std::vector<hipEvent_t> pool;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
    int cur_name = -1;
    hipEvent_t cur_start = nullptr;
    hipEvent_t get()
    {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e;
        (void)hipEventCreate(&e);
        return e;
    }
    void drain()
    {
        for (auto& pe : pending) {
            float t = 0.f;
            (void)hipEventSynchronize(pe.second.second);
            (void)hipEventElapsedTime(&t, pe.second.first, pe.second.second);
            ms[pe.first] += t;
            launches[pe.first] += 1;
            pool.push_back(pe.second.first);
            pool.push_back(pe.second.second);
        }
        pending.clear();
    }
};

}  // namespace

void prof_begin(ProfileHook* p, const char* name, hipStream_t s)
{
    if (!p || !p->impl) return;
    ProfImpl* pi = static_cast<ProfImpl*>(p->impl);
    if (!pi->enabled) return;
    int id = -1;
    for (size_t i = 0; i < pi->names.size(); i++)
        if (pi->names[i] == name) id = (int)i;
    if (id < 0) {
        id = (int)pi->names.size();
        pi->names.push_back(name);
        pi->ms.push_back(0.0);
        pi->launches.push_back(0);
    }
    pi->cur_name = id;
    pi->cur_start = pi->get();
    (void)hipEventRecord(pi->cur_start, s);
}

void prof_end(ProfileHook* p, hipStream_t s)
{
    if (!p || !p->impl) return;
    ProfImpl* pi = static_cast<ProfImpl*>(p->impl);
    if (!pi->enabled || pi->cur_name < 0) return;
    hipEvent_t e = pi->get();
    (void)hipEventRecord(e, s);
    pi->pending.push_back({pi->cur_name, {pi->cur_start, e}});
    pi->cur_name = -1;
    if (pi->pending.size() > 4096) pi->drain();
}

struct coeb_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    coeb_orb_params params{};
    Tables tab{};
    int max_w = 0, max_h = 0, max_batch = 0;
    bool has_plan = false;
    Plan plan{};
    std::vector<int> rtab;
    std::vector<CellDesc> cells;
    std::map<std::string, DevBuf> bufs;
    std::string err;
    ProfImpl prof;
    ProfileHook hook;
    int batch_frames = 0;      // frames of the last extracted batch
    const uint8_t* batch_gray = nullptr;
    int ident_frames = 0;      // identity poses initialised in "b_I"
    // Batch chunking over several HIP streams (coeb_set_batch_streams): chunk k = frames
    // [chunk[k], chunk[k+1]) runs extract -> prep -> match on subs[k]; match of chunk k's first
    // frame waits for chunk k-1's prep (its LastFrame).  The context stream joins the chunk
    // streams lazily, before anything else is enqueued on it (main_stream()).
    int nstreams = 1;
    std::vector<hipStream_t> subs;
    std::vector<int> chunk;                      // chunk boundaries of the last batch
    std::vector<hipEvent_t> ev_prep, ev_mdone;   // per chunk: prep done / match done
    bool mdone_valid = false;                    // ev_mdone holds the previous batch's matches
    bool pending_join = false;
    bool extract_chunked = false;                // the last batch extract ran on the chunk streams
    hipEvent_t ev_main = nullptr, ev_join = nullptr;
    // coeb_pose_batch_device runs k_pose on its own stream, so the optimiser of batch k overlaps
    // the extraction and matching of batch k+1 (k_pose is latency bound, one workgroup per frame;
    // the extraction kernels are VALU bound).  k_track_prep copies everything k_pose reads into
    // t_* buffers; the next coeb_pose_batch_device, coeb_batch_pose_results, coeb_memcpy_d2h,
    // coeb_synchronize and coeb_destroy join it (join_pose()).
    hipStream_t pose_stream = nullptr;
    // level-0 blur + FAST beside the pyramid (launch_extract's SideStream); COEB_SIDE_STREAM=0 disables
    SideStream side{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 2, true, false};
    bool side_init = false;
    bool side_shared = false;                 // side.s is the device's shared side stream
    hipEvent_t ev_ffork = nullptr, ev_fjoin = nullptr;   // the moving-object batch's LK-pyramid fork / join
    hipEvent_t ev_tprep = nullptr, ev_pose = nullptr;
    bool pose_pending = false;
    // batch tracking state: Observations() the matcher gave the LastFrame points, the frames and
    // min_matches of the last coeb_pose_batch_device (TrackLocalMap continues that batch)
    int batch_nobs = 2, pose_frames = 0, pose_min_matches = 20;
    hipEvent_t ev_tlm = nullptr;
    int tlm_frames = 0;
    // pinned host staging of the host-buffer entry points: their inputs are packed here and
    // moved in one copy (a dozen small pageable copies cost more than the kernels)
    uint8_t* pin = nullptr;
    uint8_t* pin_dev = nullptr;        // the same page-locked bytes as the device addresses them
    size_t pin_n = 0;
};

namespace {

int set_err(coeb_ctx* c, int code, const std::string& msg)
{
    if (c) c->err = msg;
    g_last_error = msg;
    return code;
}

int hip_err(coeb_ctx* c, hipError_t e, const char* where)
{
    return set_err(c, COEB_EDEVICE, std::string(where) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(ctx, expr)                                          \
    do {                                                            \
        hipError_t _e = (expr);                                     \
        if (_e != hipSuccess) return hip_err((ctx), _e, #expr);     \
    } while (0)

int quiesce(coeb_ctx* c);

template <typename T>
int ensure(coeb_ctx* c, const char* name, size_t count, T** out)
{
    DevBuf& b = c->bufs[name];
    const size_t bytes = std::max<size_t>(count * sizeof(T), 256);
    if (b.n < bytes) {
        if (b.p) {
            int rc = quiesce(c);          // work in flight on any of the context's streams may read it
            if (rc) return rc;
            (void)hipFree(b.p);
        }
        b.p = nullptr;
        b.n = 0;
        hipError_t e = hipMalloc(&b.p, bytes);
        if (e != hipSuccess) return set_err(c, COEB_ENOMEM, std::string("hipMalloc ") + name + ": " + hipGetErrorString(e));
        b.n = bytes;
    }
    *out = static_cast<T*>(b.p);
    return 0;
}

// One frame's results written straight into the context's page-locked buffer (its device
// alias): the keypoint count and the first min(count, guess) records and descriptors, so the
// host reads them after one synchronisation with no copy operations in between (each D2H copy
// op of the single-frame path cost 5-25 us plus its launch gap, profiles/r06/sf).
__global__ __launch_bounds__(256) void k_out_pack(const int* counts, const uint32_t* kps, const uint4* desc, int guess,
                                                  int* out_n, uint32_t* out_k, uint4* out_d)
{
    const int n = min(*counts, guess);
    const int t = blockIdx.x * 256 + threadIdx.x, T = gridDim.x * 256;
    if (t == 0) *out_n = *counts;
    for (int i = t; i < 7 * n; i += T) out_k[i] = kps[i];          // 28-byte records
    for (int i = t; i < 2 * n; i += T) out_d[i] = desc[i];         // 32-byte rows
}

// Inputs of one call packed at 16-byte aligned offsets of the pinned staging buffer, moved to
// the device in one copy; fill() parts are constant bytes (absent optional arrays).
struct Pack {
    struct Part { const void* p; size_t n; int fill; };
    std::vector<Part> parts;
    size_t total = 0;
    size_t add(const void* p, size_t n) { return put(Part{p, n, -1}); }
    size_t fill(int byte, size_t n) { return put(Part{nullptr, n, byte}); }
    size_t put(Part q)
    {
        const size_t off = total;
        parts.push_back(q);
        total = (total + q.n + 15) & ~(size_t)15;
        return off;
    }
};

int pinned(coeb_ctx* c, size_t bytes)
{
    if (c->pin_n >= bytes) return 0;
    if (c->pin) (void)hipHostFree(c->pin);
    c->pin = nullptr;
    c->pin_n = 0;
    const size_t n = std::max<size_t>(bytes, (size_t)1 << 20);
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&c->pin), n, hipHostMallocDefault);
    if (e != hipSuccess) return set_err(c, COEB_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    void* dv = nullptr;
    e = hipHostGetDevicePointer(&dv, c->pin, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(c->pin);
        c->pin = nullptr;
        return set_err(c, COEB_ENOMEM, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
    }
    c->pin_dev = static_cast<uint8_t*>(dv);
    c->pin_n = n;
    return 0;
}

// pack -> pinned -> one H2D copy into the "stage" device buffer; *dbase = its device address.
// The previous call's copies have completed: every host-buffer entry point synchronises.
int stage_in(coeb_ctx* c, const Pack& pk, uint8_t** dbase, hipStream_t s)
{
    int rc;
    const size_t total = std::max<size_t>(pk.total, 16);
    if ((rc = pinned(c, total)) || (rc = ensure(c, "stage", total, dbase))) return rc;
    size_t off = 0;
    for (const Pack::Part& q : pk.parts) {
        if (q.n) {
            if (q.p) memcpy(c->pin + off, q.p, q.n);
            else memset(c->pin + off, q.fill, q.n);
        }
        off = (off + q.n + 15) & ~(size_t)15;
    }
    HIP_TRY(c, hipMemcpyAsync(*dbase, c->pin, total, hipMemcpyHostToDevice, s));
    return 0;
}

int ensure_plan(coeb_ctx* c, int W, int H)
{
    if (c->has_plan && c->plan.W == W && c->plan.H == H) return 0;
    if (W <= 0 || H <= 0 || W > c->max_w || H > c->max_h)
        return set_err(c, COEB_EINVAL, "image size outside the context limits");
    std::string err;
    Plan P;
    if (!make_plan(c->tab, W, H, P, c->rtab, c->cells, err)) return set_err(c, COEB_EINVAL, err);
    // the plan, rtab and cells are rewritten in place below: batches still in flight on the
    // context's streams (pyramid / FAST / octree / describe read them) must finish first
    int rc;
    if ((rc = quiesce(c))) return rc;
    c->plan = P;
    Plan* dplan;
    int* drtab;
    CellDesc* dcells;
    int8_t* dpat;
    if ((rc = ensure(c, "plan", 1, &dplan))) return rc;
    if ((rc = ensure(c, "rtab", std::max<size_t>(c->rtab.size(), 1), &drtab))) return rc;
    if ((rc = ensure(c, "cells", c->cells.size(), &dcells))) return rc;
    if ((rc = ensure(c, "pattern", 1024, &dpat))) return rc;
    HIP_TRY(c, hipMemcpy(dplan, &c->plan, sizeof(Plan), hipMemcpyHostToDevice));
    if (!c->rtab.empty()) HIP_TRY(c, hipMemcpy(drtab, c->rtab.data(), c->rtab.size() * sizeof(int), hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(dcells, c->cells.data(), c->cells.size() * sizeof(CellDesc), hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(dpat, kPattern, 1024, hipMemcpyHostToDevice));
    c->has_plan = true;
    return 0;
}

// Allocate per-frame buffers for F frames and fill ExtractBufs.
int extract_bufs(coeb_ctx* c, int F, ExtractBufs& b)
{
    const Plan& P = c->plan;
    memset(&b, 0, sizeof(b));
    int rc;
    uint8_t *pyr, *blur, *nodes, *desc;
    int *cand_n, *lvl_n, *counts, *err;
    uint32_t *cand, *keys, *lvl_kp;
    coeb_keypoint* kps;
    DynMask* dyn;
    if ((rc = ensure(c, "pyr", (size_t)F * P.pyr_stride + 4096, &pyr))) return rc;
    if ((rc = ensure(c, "blur", (size_t)F * P.blur_stride + 4096, &blur))) return rc;
    if ((rc = ensure(c, "cand_n", (size_t)F * P.ncells, &cand_n))) return rc;
    if ((rc = ensure(c, "cand", (size_t)F * P.ncells * P.cell_cap, &cand))) return rc;
    if ((rc = ensure(c, "keys", (size_t)F * 2 * P.kbuf_stride, &keys))) return rc;
    if ((rc = ensure(c, "nodes", (size_t)F * P.node_stride * 4, &nodes))) return rc;
    if ((rc = ensure(c, "lvl_n", (size_t)F * P.L, &lvl_n))) return rc;
    if ((rc = ensure(c, "lvl_kp", (size_t)F * P.lvl_stride, &lvl_kp))) return rc;
    if ((rc = ensure(c, "kps", (size_t)F * P.kcap, &kps))) return rc;
    if ((rc = ensure(c, "desc", (size_t)F * P.kcap * 32, &desc))) return rc;
    if ((rc = ensure(c, "counts", (size_t)F, &counts))) return rc;
    if ((rc = ensure(c, "dyn", (size_t)F, &dyn))) return rc;
    if ((rc = ensure(c, "err", 4, &err))) return rc;
    b.pyr = pyr; b.blur = blur; b.cand_n = cand_n; b.cand = cand; b.keys = keys; b.nodes = nodes;
    b.lvl_n = lvl_n; b.lvl_kp = lvl_kp; b.kps = kps; b.desc = desc; b.counts = counts; b.dyn = dyn; b.err = err;
    b.rtab = static_cast<const int*>(c->bufs["rtab"].p);
    b.cells = static_cast<const CellDesc*>(c->bufs["cells"].p);
    b.pattern = static_cast<const int8_t*>(c->bufs["pattern"].p);
    return 0;
}

// Upload per-frame boxes / T_M / blur flags (host arrays, offset layout) for F frames.
int upload_dyn(coeb_ctx* c, int F, const coeb_box* boxes, const int32_t* box_off, const float* tm_xy,
               const int32_t* tm_off, const int32_t* blur_flag, ExtractBufs& b)
{
    const int nbox = (box_off && boxes) ? box_off[F] : 0;
    const int ntm = (tm_off && tm_xy) ? tm_off[F] : 0;
    int rc;
    float *dbox, *dtm;
    int32_t *dboff, *dtoff, *dblur;
    // offsets must start at 0 and never decrease: every box then gets its frame from
    // k_box_frame, and every T_M range lies inside the uploaded array
    if (box_off && boxes && box_off[0] != 0) return set_err(c, COEB_EINVAL, "box_off[0] != 0");
    if (tm_off && tm_xy && tm_off[0] != 0) return set_err(c, COEB_EINVAL, "tm_off[0] != 0");
    for (int f = 0; f < F; f++) {
        if (box_off && boxes && box_off[f + 1] < box_off[f]) return set_err(c, COEB_EINVAL, "box_off decreases");
        if (tm_off && tm_xy && tm_off[f + 1] < tm_off[f]) return set_err(c, COEB_EINVAL, "tm_off decreases");
    }
    if (nbox > 0) {
        for (int f = 0; f < F; f++)
            if (box_off[f + 1] - box_off[f] > COEB_MAXBOX) return set_err(c, COEB_EINVAL, "more than 16 boxes in a frame");
        if ((rc = ensure(c, "boxes", (size_t)nbox * 4, &dbox))) return rc;
        if ((rc = ensure(c, "box_off", (size_t)F + 1, &dboff))) return rc;
        if ((rc = ensure(c, "blurf", (size_t)nbox, &dblur))) return rc;
        HIP_TRY(c, hipMemcpyAsync(dbox, boxes, (size_t)nbox * 16, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(dboff, box_off, (size_t)(F + 1) * 4, hipMemcpyHostToDevice, c->stream));
        if (blur_flag) {
            HIP_TRY(c, hipMemcpyAsync(dblur, blur_flag, (size_t)nbox * 4, hipMemcpyHostToDevice, c->stream));
        } else {
            HIP_TRY(c, hipMemsetAsync(dblur, 0, (size_t)nbox * 4, c->stream));
        }
        b.boxes = dbox; b.box_off = dboff; b.blurf = dblur;
    }
    if (ntm > 0) {
        if ((rc = ensure(c, "tm", (size_t)ntm * 2, &dtm))) return rc;
        if ((rc = ensure(c, "tm_off", (size_t)F + 1, &dtoff))) return rc;
        HIP_TRY(c, hipMemcpyAsync(dtm, tm_xy, (size_t)ntm * 8, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(dtoff, tm_off, (size_t)(F + 1) * 4, hipMemcpyHostToDevice, c->stream));
        b.tm = dtm; b.tm_off = dtoff;
    }
    return 0;
}

// The context stream, after it has been made to wait for every chunk stream of the last
// batch (so work enqueued on it sees the batch's results).
}  // namespace

// The product switches (coeb_internal.hpp); every one of them is set by a GPU test.
static const char* const kSwitches[] = {
    "COEB_SIDE_STREAM",        // 0: no extraction side stream     (test_sharded_batch_equals_unsharded[off])
    "COEB_SIDE_SHARED",        // 1: one side stream per device     ([shared], bench config C)
    "COEB_SIDE_EAGER",         // 1: side stream made with the ctx  ([eager], bench config A)
    "COEB_MATCH_SEQUENTIAL",   // 1: the literal sequential claims  (test_match_paths_agree, ...)
    "COEB_MATCH_SPLIT",        // N: split-list workgroups per pair (test_batch_small_split_lists...)
    "COEB_PYR_BYTES",          // 1: k_pyr_level byte form          (test_blur_pyramid_matches_oracle)
    "COEB_FAST_RB",            // 72: the general FAST slab layout  (test_fast_general_slab_layout...)
    "COEB_FM_THREADS",         // k_fm threads per pair             (tests/test_gpu_flow.py)
};

const char* coeb_switch(const char* name)
{
    for (const char* k : kSwitches)
        if (strcmp(k, name) == 0) return getenv(name);
    return nullptr;            // not a product switch: never read
}

const char* coeb_experiment(const char* name)
{
    static const bool on = [] {
        const char* e = getenv("COEB_EXPERIMENTS");
        return e && e[0] == '1';
    }();
    return on ? getenv(name) : nullptr;
}

namespace {

// The side stream of launch_extract (created on first use), or null when disabled.  Per-kernel
// profiling (coeb_profile_enable) serialises everything on the context stream, so each event
// pair brackets one whole-batch launch.
// A non-blocking stream whose priority the environment variable `env` may set ("high" / "low":
// the device's greatest / least stream priority; unset: the default).  Experiment knob for the
// multi-stream schedules (which queue the dispatcher serves first when CUs free up).
static hipError_t make_stream(hipStream_t* s, const char* env)
{
    const char* e = env ? coeb_experiment(env) : nullptr;
    if (e && (e[0] == 'h' || e[0] == 'l')) {
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
            return hipStreamCreateWithPriority(s, hipStreamNonBlocking, e[0] == 'h' ? greatest : least);
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

// The device's shared side stream (COEB_SIDE_SHARED=1): with P pipelines the P context streams
// plus one side stream fill the 4 hardware queues exactly, instead of 2P streams sharing them.
// Reference-counted over the contexts that use it.
static std::mutex g_shared_side_mu;
static std::map<int, std::pair<hipStream_t, int>> g_shared_side;

static hipError_t shared_side_acquire(int device, hipStream_t* out)
{
    std::lock_guard<std::mutex> lk(g_shared_side_mu);
    auto& e = g_shared_side[device];
    if (!e.first) {
        hipError_t r = make_stream(&e.first, "COEB_SIDE_PRIO");
        if (r != hipSuccess) { e.first = nullptr; return r; }
    }
    ++e.second;
    *out = e.first;
    return hipSuccess;
}

static void shared_side_release(int device)
{
    std::lock_guard<std::mutex> lk(g_shared_side_mu);
    auto it = g_shared_side.find(device);
    if (it == g_shared_side.end() || --it->second.second > 0) return;
    (void)hipStreamSynchronize(it->second.first);
    (void)hipStreamDestroy(it->second.first);
    g_shared_side.erase(it);
}

const SideStream* side_stream(coeb_ctx* c)
{
    if (c->prof.enabled) return nullptr;
    if (!c->side_init) {
        c->side_init = true;
        const char* e = coeb_switch("COEB_SIDE_STREAM");
        if (e && e[0] == '0') return nullptr;
        const char* sp = coeb_experiment("COEB_SIDE_SPLIT");          // first level left to the context stream
        if (sp) c->side.split = atoi(sp);
        const char* bl = coeb_experiment("COEB_SIDE_BLUR");           // 0: late levels' blur on the context stream
        if (bl) c->side.blur_late = bl[0] == '1';
        const char* so = coeb_experiment("COEB_SIDE_OCTREE");         // 1: early levels' octree on the side stream
        if (so) c->side.side_octree = so[0] == '1';
        const char* sh = coeb_switch("COEB_SIDE_SHARED");         // 1: one side stream per device
        c->side_shared = sh && sh[0] == '1';
        hipError_t se = c->side_shared ? shared_side_acquire(c->device, &c->side.s)
                                       : make_stream(&c->side.s, "COEB_SIDE_PRIO");
        hipEvent_t* evs[] = {&c->side.fork, &c->side.mid, &c->side.pyr_done, &c->side.join2, &c->side.join};
        bool ok = se == hipSuccess;
        for (hipEvent_t* e : evs) {
            *e = nullptr;
            if (ok && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
                *e = nullptr;
                ok = false;
            }
        }
        if (!ok) {
            // run without a side stream: release what was made
            for (hipEvent_t* e : evs)
                if (*e) (void)hipEventDestroy(*e), *e = nullptr;
            if (se == hipSuccess) {
                if (c->side_shared) shared_side_release(c->device);
                else (void)hipStreamDestroy(c->side.s);
            }
            c->side.s = nullptr;
            c->side_shared = false;
        }
    }
    return c->side.s ? &c->side : nullptr;
}

// The context stream waits for the last batch pose (k_pose on pose_stream).
void join_pose(coeb_ctx* c)
{
    if (c->pose_pending) {
        (void)hipStreamWaitEvent(c->stream, c->ev_pose, 0);
        c->pose_pending = false;
    }
}

hipStream_t main_stream(coeb_ctx* c)
{
    if (c->pending_join) {
        for (hipStream_t s : c->subs) {
            (void)hipEventRecord(c->ev_join, s);
            (void)hipStreamWaitEvent(c->stream, c->ev_join, 0);
        }
        c->pending_join = false;
    }
    return c->stream;
}

// Wait until nothing enqueued by this context is still running: the chunk streams and the pose
// stream are joined into the context stream (the side stream is joined there by every
// extraction), then the context stream is drained.
int quiesce(coeb_ctx* c)
{
    if (!c->stream) return 0;
    main_stream(c);
    join_pose(c);
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return 0;
}

// Chunk boundaries for F frames over the context's batch streams (>= 16 frames per chunk).
int make_chunks(coeb_ctx* c, int F)
{
    int n = std::max(1, std::min(c->nstreams, F / 16));
    if (n > 1 && (int)c->subs.size() < n) {
        while ((int)c->subs.size() < n) {
            hipStream_t s;
            hipEvent_t a, b;
            if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) break;
            (void)hipEventCreateWithFlags(&a, hipEventDisableTiming);
            (void)hipEventCreateWithFlags(&b, hipEventDisableTiming);
            c->subs.push_back(s);
            c->ev_prep.push_back(a);
            c->ev_mdone.push_back(b);
        }
        n = std::min<int>(n, (int)c->subs.size());
    }
    c->chunk.assign(n + 1, 0);
    for (int k = 0; k <= n; k++) c->chunk[k] = (int)((int64_t)F * k / n);
    return n;
}

// Per-frame buffers of frames [f0, ...): every per-frame array advanced by f0 frames.
ExtractBufs offset_bufs(const Plan& P, const ExtractBufs& b, int f0)
{
    ExtractBufs o = b;
    o.gray = b.gray + (int64_t)f0 * P.W * P.H;
    o.pyr = b.pyr + (int64_t)f0 * P.pyr_stride;
    o.blur = b.blur + (int64_t)f0 * P.blur_stride;
    o.cand_n = b.cand_n + (int64_t)f0 * P.ncells;
    o.cand = b.cand + (int64_t)f0 * P.ncells * P.cell_cap;
    o.keys = b.keys + (int64_t)f0 * 2 * P.kbuf_stride;
    o.nodes = b.nodes + (int64_t)f0 * P.node_stride * 4;
    o.lvl_n = b.lvl_n + (int64_t)f0 * P.L;
    o.lvl_kp = b.lvl_kp + (int64_t)f0 * P.lvl_stride;
    o.kps = static_cast<coeb_keypoint*>(b.kps) + (int64_t)f0 * P.kcap;
    o.desc = b.desc + (int64_t)f0 * P.kcap * 32;
    o.counts = b.counts + f0;
    o.dyn = b.dyn + f0;
    if (b.box_off) o.box_off = b.box_off + f0;   // offsets index the shared box / T_M arrays
    if (b.tm_off) o.tm_off = b.tm_off + f0;
    return o;
}

// The device error word copied behind the work of a host-buffer call into `dst` (page-locked),
// so the call's one synchronisation also brings the word back; err_word_seen checks the copy.
int err_word_async(coeb_ctx* c, uint8_t* dst)
{
    int* derr = static_cast<int*>(c->bufs["err"].p);
    if (!derr) {
        memset(dst, 0, 4);
        return 0;
    }
    HIP_TRY(c, hipMemcpyAsync(dst, derr, 4, hipMemcpyDeviceToHost, main_stream(c)));
    return 0;
}

int err_word_seen(coeb_ctx* c, const uint8_t* src)
{
    int h = 0;
    memcpy(&h, src, 4);
    if (!h) return 0;
    char msg[160];
    snprintf(msg, sizeof msg, "internal capacity exceeded (device error bits 0x%x)", h);
    HIP_TRY(c, hipMemsetAsync(c->bufs["err"].p, 0, 4, main_stream(c)));
    return set_err(c, COEB_ERANGE, msg);
}

int check_err_word(coeb_ctx* c)
{
    main_stream(c);
    int* derr = static_cast<int*>(c->bufs["err"].p);
    if (!derr) return 0;
    int h = 0;
    HIP_TRY(c, hipMemcpyAsync(&h, derr, 4, hipMemcpyDeviceToHost, main_stream(c)));
    HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
    if (h) {
        char msg[160];
        snprintf(msg, sizeof msg, "internal capacity exceeded (device error bits 0x%x)", h);
        HIP_TRY(c, hipMemsetAsync(derr, 0, 4, main_stream(c)));
        return set_err(c, COEB_ERANGE, msg);
    }
    return 0;
}

}  // namespace

extern "C" {

int coeb_abi_version(void) { return COEB_ABI_VERSION; }

int coeb_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

coeb_ctx* coeb_create(const coeb_orb_params* params, int device, int max_width, int max_height, int max_batch)
{
    if (!params || max_width <= 0 || max_height <= 0 || max_batch <= 0) {
        g_last_error = "coeb_create: invalid arguments";
        return nullptr;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) {
        g_last_error = "coeb_create: no usable HIP device (the HIP path has no CPU fallback)";
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        g_last_error = std::string("coeb_create: device is not gfx950 (") + prop.gcnArchName + ")";
        return nullptr;
    }
    coeb_ctx* c = new coeb_ctx();
    c->device = device;
    c->params = *params;
    if (!make_tables(*params, c->tab)) {
        g_last_error = "coeb_create: invalid ORB parameters";
        delete c;
        return nullptr;
    }
    c->max_w = max_width;
    c->max_h = max_height;
    c->max_batch = max_batch;
    if (hipSetDevice(device) != hipSuccess || make_stream(&c->stream, "COEB_MAIN_PRIO") != hipSuccess) {
        g_last_error = "coeb_create: stream creation failed";
        delete c;
        return nullptr;
    }
    c->hook.impl = &c->prof;
    // COEB_SIDE_EAGER=1: create the side stream now, right after the context stream, so the
    // contexts' streams take the hardware queues in (context, side) pairs (experiment knob; by
    // default it is created at the first extraction, after every context stream of the process)
    if (const char* e = coeb_switch("COEB_SIDE_EAGER"))
        if (e[0] == '1') (void)side_stream(c);
    if (hipEventCreateWithFlags(&c->ev_main, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess) {
        g_last_error = "coeb_create: event creation failed";
        coeb_destroy(c);
        return nullptr;
    }
    int* err;
    if (ensure(c, "err", 4, &err) || hipMemset(err, 0, 16) != hipSuccess) {
        g_last_error = "coeb_create: device allocation failed";
        coeb_destroy(c);
        return nullptr;
    }
    return c;
}

void coeb_destroy(coeb_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(main_stream(c));
    if (c->side.s) {
        if (c->side_shared) {
            // this context's side work ends at its join events; the other contexts' work queued on
            // the shared stream is theirs to wait for (the last release synchronises the stream)
            (void)hipEventSynchronize(c->side.join);
            (void)hipEventSynchronize(c->side.join2);
            if (c->ev_fjoin) (void)hipEventSynchronize(c->ev_fjoin);
            shared_side_release(c->device);
        } else {
            (void)hipStreamSynchronize(c->side.s);
            (void)hipStreamDestroy(c->side.s);
        }
        (void)hipEventDestroy(c->side.fork);
        (void)hipEventDestroy(c->side.mid);
        (void)hipEventDestroy(c->side.pyr_done);
        (void)hipEventDestroy(c->side.join2);
        (void)hipEventDestroy(c->side.join);
    }
    if (c->ev_ffork) (void)hipEventDestroy(c->ev_ffork);
    if (c->ev_fjoin) (void)hipEventDestroy(c->ev_fjoin);
    if (c->pose_stream) {
        (void)hipStreamSynchronize(c->pose_stream);
        (void)hipStreamDestroy(c->pose_stream);
        (void)hipEventDestroy(c->ev_tprep);
        (void)hipEventDestroy(c->ev_pose);
        if (c->ev_tlm) (void)hipEventDestroy(c->ev_tlm);
    }
    for (auto& kv : c->bufs)
        if (kv.second.p) (void)hipFree(kv.second.p);
    c->prof.drain();
    for (auto e : c->prof.pool) (void)hipEventDestroy(e);
    for (size_t k = 0; k < c->subs.size(); k++) {
        (void)hipStreamDestroy(c->subs[k]);
        (void)hipEventDestroy(c->ev_prep[k]);
        (void)hipEventDestroy(c->ev_mdone[k]);
    }
    if (c->ev_main) (void)hipEventDestroy(c->ev_main);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->pin) (void)hipHostFree(c->pin);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    coeb_internal_flow_forget(c);
    delete c;
}

const char* coeb_last_error(const coeb_ctx* c)
{
    if (c && !c->err.empty()) return c->err.c_str();
    return g_last_error.c_str();
}

int coeb_orb_tables_get(const coeb_ctx* c, coeb_orb_tables* out)
{
    if (!c || !out) return COEB_EINVAL;
    memset(out, 0, sizeof(*out));
    out->nlevels = c->tab.nlevels;
    out->scale_factor = (float)c->tab.scale_factor;
    for (int l = 0; l < c->tab.nlevels; l++) {
        out->scale[l] = c->tab.scale[l];
        out->inv_scale[l] = c->tab.inv_scale[l];
        out->sigma2[l] = c->tab.sigma2[l];
        out->inv_sigma2[l] = c->tab.inv_sigma2[l];
        out->features_per_level[l] = c->tab.nfeat[l];
    }
    memcpy(out->umax, c->tab.umax, sizeof(out->umax));
    return COEB_OK;
}

int coeb_max_keypoints(const coeb_ctx* cc, int width, int height)
{
    coeb_ctx* c = const_cast<coeb_ctx*>(cc);
    if (!c) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    int rc = ensure_plan(c, width, height);
    if (rc) return rc;
    return c->plan.kcap;
}

int coeb_extract_batch_device(coeb_ctx* c, const uint8_t* d_gray, int F, int W, int H, const coeb_box* boxes,
                              const int32_t* box_off, const float* tm_xy, const int32_t* tm_off,
                              const int32_t* blur_flag)
{
    if (!c || !d_gray || F <= 0) return set_err(c, COEB_EINVAL, "coeb_extract_batch_device: invalid arguments");
    if (F > c->max_batch) return set_err(c, COEB_EINVAL, "batch larger than max_batch");
    (void)hipSetDevice(c->device);
    int rc;
    if ((rc = ensure_plan(c, W, H))) return rc;
    ExtractBufs b;
    const std::vector<int> prev_chunk = c->chunk;
    const bool prev_mdone = c->mdone_valid;
    const int n = make_chunks(c, F);
    const bool has_dyn = (boxes && box_off) || (tm_xy && tm_off);
    // per-frame buffers may be reallocated and the box / T_M staging rewritten: let every
    // outstanding batch finish first in those cases
    const bool serial = n == 1 || has_dyn || (c->batch_frames != F);
    if (serial) main_stream(c);
    if ((rc = extract_bufs(c, F, b))) return rc;
    if ((rc = upload_dyn(c, F, boxes, box_off, tm_xy, tm_off, blur_flag, b))) return rc;
    b.gray = d_gray;
    const Plan* dplan = static_cast<const Plan*>(c->bufs["plan"].p);
    c->mdone_valid = false;
    c->extract_chunked = n > 1;
    if (n == 1) {
        if (launch_extract(c->plan, dplan, b, F, main_stream(c), &c->hook, side_stream(c)))
            return hip_err(c, hipGetLastError(), "launch_extract");
    } else {
        HIP_TRY(c, hipEventRecord(c->ev_main, c->stream));   // no join: steps overlap
        const bool cross = !serial && prev_mdone && prev_chunk == c->chunk;
        for (int k = 0; k < n; k++) {
            hipStream_t s = c->subs[k];
            HIP_TRY(c, hipStreamWaitEvent(s, c->ev_main, 0));
            // the previous batch's matcher of chunk k+1 reads chunk k's last frame
            if (cross && k + 1 < n) HIP_TRY(c, hipStreamWaitEvent(s, c->ev_mdone[k + 1], 0));
            const int f0 = c->chunk[k], f1 = c->chunk[k + 1];
            if (launch_extract(c->plan, dplan, offset_bufs(c->plan, b, f0), f1 - f0, s, &c->hook))
                return hip_err(c, hipGetLastError(), "launch_extract");
        }
        c->pending_join = true;
    }
    c->batch_frames = F;
    c->batch_gray = d_gray;
    return COEB_OK;
}

extern "C" int coeb_internal_pmo_batch(coeb_ctx* c, const uint8_t* d_gray, int F, int w, int h, float* tm_out,
                                       int* ntm_out, int tm_cap);
extern "C" int coeb_internal_blur_flags_batch(coeb_ctx* c, const uint8_t* d_gray, int W, int H, const float* d_boxes,
                                              const int* d_box_off, int F, int* d_box_frame, int nbox, int* d_out,
                                              hipStream_t s);

int coeb_frame_batch_device(coeb_ctx* c, const uint8_t* d_gray, int F, int W, int H, const coeb_box* boxes,
                            const int32_t* box_off)
{
    if (!c || !d_gray || F <= 0 || (boxes && !box_off))
        return set_err(c, COEB_EINVAL, "coeb_frame_batch_device: invalid arguments");
    if (F > c->max_batch) return set_err(c, COEB_EINVAL, "batch larger than max_batch");
    (void)hipSetDevice(c->device);
    int rc;
    if ((rc = ensure_plan(c, W, H))) return rc;
    // Everything below runs on the context stream, so stream order protects the flow scratch,
    // T_M and the box staging of the previous batch (ensure() quiesces before it reallocates);
    // the pose stream reads only its own snapshots (k_track_prep / k_tlm_snapshot).
    hipStream_t s = main_stream(c);
    const int nbox = boxes ? box_off[F] : 0;
    float* tm;
    int32_t *ntm, *bframe = nullptr, *blur = nullptr;
    if ((rc = ensure(c, "f_tm", (size_t)F * kFrameTmCap * 2, &tm)) || (rc = ensure(c, "f_ntm", (size_t)F, &ntm)))
        return rc;
    // ProcessMovingObject(frame f-1, frame f) -> T_M of frame f (Frame.cc:164-166)
    if ((rc = coeb_internal_pmo_batch(c, d_gray, F, W, H, tm, ntm, kFrameTmCap))) return rc;
    ExtractBufs b;
    if ((rc = extract_bufs(c, F, b))) return rc;
    if ((rc = upload_dyn(c, F, boxes, box_off, nullptr, nullptr, nullptr, b))) return rc;
    if (nbox > 0) {
        // detect_laplacian blur flag of every box (Frame.cc:171-202); frame 0 = the first frame.
        // The box -> frame map is built on the device from the box offsets upload_dyn staged.
        if ((rc = ensure(c, "f_bframe", (size_t)nbox, &bframe)) || (rc = ensure(c, "f_blur", (size_t)nbox, &blur)))
            return rc;
        if (coeb_internal_blur_flags_batch(c, d_gray, W, H, b.boxes, b.box_off, F, bframe, nbox, blur, s))
            return hip_err(c, hipGetLastError(), "blur flags");
        b.blurf = blur;
    }
    b.tmd = tm;
    b.ntmd = ntm;
    b.tmd_cap = kFrameTmCap;
    b.gray = d_gray;
    c->mdone_valid = false;
    c->extract_chunked = false;
    c->chunk.assign(2, 0);
    c->chunk[1] = F;
    if (launch_extract(c->plan, static_cast<const Plan*>(c->bufs["plan"].p), b, F, s, &c->hook, side_stream(c)))
        return hip_err(c, hipGetLastError(), "launch_extract");
    c->batch_frames = F;
    c->batch_gray = d_gray;
    return COEB_OK;
}

int coeb_batch_frame_results(coeb_ctx* c, const float** d_tm, const int32_t** d_ntm, int* tm_cap,
                             const int32_t** d_blur)
{
    if (!c || !c->bufs.count("f_ntm")) return set_err(c, COEB_EINVAL, "no frame batch yet");
    if (d_tm) *d_tm = static_cast<const float*>(c->bufs["f_tm"].p);
    if (d_ntm) *d_ntm = static_cast<const int32_t*>(c->bufs["f_ntm"].p);
    if (tm_cap) *tm_cap = kFrameTmCap;
    if (d_blur) *d_blur = c->bufs.count("f_blur") ? static_cast<const int32_t*>(c->bufs["f_blur"].p) : nullptr;
    return COEB_OK;
}

int coeb_set_batch_streams(coeb_ctx* c, int nstreams)
{
    if (!c || nstreams < 1 || nstreams > 16) return set_err(c, COEB_EINVAL, "coeb_set_batch_streams: 1..16 streams");
    (void)hipSetDevice(c->device);
    main_stream(c);
    c->nstreams = nstreams;
    c->mdone_valid = false;
    return COEB_OK;
}

int coeb_batch_results(coeb_ctx* c, const coeb_keypoint** d_kps, const uint8_t** d_desc, const int32_t** d_counts,
                       int* kcap)
{
    if (!c || !c->has_plan) return set_err(c, COEB_EINVAL, "no batch extracted yet");
    if (d_kps) *d_kps = static_cast<const coeb_keypoint*>(c->bufs["kps"].p);
    if (d_desc) *d_desc = static_cast<const uint8_t*>(c->bufs["desc"].p);
    if (d_counts) *d_counts = static_cast<const int32_t*>(c->bufs["counts"].p);
    if (kcap) *kcap = c->plan.kcap;
    return COEB_OK;
}

int coeb_extract(coeb_ctx* c, const uint8_t* gray, int W, int H, size_t stride, const coeb_box* boxes, int nbox,
                 const float* tm_xy, int ntm, const int32_t* blur_flag, int nblur, coeb_keypoint* kp_out,
                 uint8_t* desc_out, int cap, int* n_out)
{
    if (!c || !n_out) return set_err(c, COEB_EINVAL, "coeb_extract: invalid arguments");
    *n_out = 0;
    if (!gray || W <= 0 || H <= 0) return COEB_OK;          // _image.empty() -> return (:1096-1097)
    if (stride < (size_t)W) return set_err(c, COEB_EINVAL, "stride < width");
    if (nbox < 0 || nbox > COEB_MAXBOX || ntm < 0 || nblur < 0) return set_err(c, COEB_EINVAL, "bad box/T_M counts");
    if ((nbox && !boxes) || (ntm && !tm_xy)) return set_err(c, COEB_EINVAL, "coeb_extract: null box / T_M array");
    (void)hipSetDevice(c->device);
    int rc;
    if ((rc = ensure_plan(c, W, H))) return rc;
    uint8_t* dgray;
    if ((rc = ensure(c, "gray_stage", (size_t)W * H, &dgray))) return rc;
    // pinned staging at both ends: the image rows go through the context's page-locked buffer
    // (one DMA, no runtime pinning of the caller's pages), and the results come back into it
    // behind the kernels -- the count and the first `guess` records in one synchronisation
    // (a pageable round trip each cost 120-170 us on the box, profiles/r06/sf)
    const size_t img = ((size_t)W * H + 255) & ~(size_t)255;
    const int kcap = c->plan.kcap;
    const size_t o_n = img, o_k = img + 256, o_d = o_k + (((size_t)kcap * sizeof(coeb_keypoint) + 255) & ~(size_t)255);
    // the dynamic-mask inputs (boxes, T_M, blur flags, their offsets) staged behind the results
    const size_t o_dyn = o_d + (((size_t)kcap * 32 + 255) & ~(size_t)255);
    const size_t o_bo = o_dyn + (size_t)nbox * sizeof(coeb_box), o_bl = o_bo + 16, o_to = o_bl + (size_t)nbox * 4 + 16,
                 o_tm = o_to + 16;
    if ((rc = pinned(c, o_tm + (size_t)ntm * 8))) return rc;
    if (stride == (size_t)W) memcpy(c->pin, gray, (size_t)W * H);
    else
        for (int y = 0; y < H; y++) memcpy(c->pin + (size_t)y * W, gray + (size_t)y * stride, (size_t)W);
    HIP_TRY(c, hipMemcpyAsync(dgray, c->pin, (size_t)W * H, hipMemcpyHostToDevice, main_stream(c)));
    int32_t* box_off = reinterpret_cast<int32_t*>(c->pin + o_bo);
    int32_t* tm_off = reinterpret_cast<int32_t*>(c->pin + o_to);
    int32_t* blur = reinterpret_cast<int32_t*>(c->pin + o_bl);
    box_off[0] = 0; box_off[1] = nbox; tm_off[0] = 0; tm_off[1] = ntm;
    for (int i = 0; i < nbox; i++)                      // missing flags (or a null array) read as 0
        blur[i] = (blur_flag && i < nblur) ? blur_flag[i] : 0;
    if (nbox) memcpy(c->pin + o_dyn, boxes, (size_t)nbox * sizeof(coeb_box));
    if (ntm) memcpy(c->pin + o_tm, tm_xy, (size_t)ntm * 8);
    ExtractBufs b;
    if ((rc = extract_bufs(c, 1, b))) return rc;
    if ((rc = upload_dyn(c, 1, nbox ? reinterpret_cast<const coeb_box*>(c->pin + o_dyn) : nullptr, box_off,
                         ntm ? reinterpret_cast<const float*>(c->pin + o_tm) : nullptr, tm_off, nbox ? blur : nullptr, b)))
        return rc;
    b.gray = dgray;
    // one frame on one stream: the side stream's fork / join cost more than the overlap it buys
    // at F = 1 (0.389 vs 0.350 ms per single-frame step, profiles/r06/sf)
    if (launch_extract(c->plan, static_cast<const Plan*>(c->bufs["plan"].p), b, 1, main_stream(c), &c->hook, nullptr))
        return hip_err(c, hipGetLastError(), "launch_extract");
    c->batch_frames = 1;
    c->batch_gray = dgray;
    // the retained set is nfeatures plus at most a few per level (the final cull, ORBextractor.cc
    // :1204-1207), so nfeatures + 256 records almost always cover it; a larger count costs a
    // second round trip for the rest
    const int guess = (kp_out && desc_out) ? std::min({kcap, std::max(cap, 0), c->params.nfeatures + 256}) : 0;
    hipStream_t s = main_stream(c);
    hipLaunchKernelGGL(k_out_pack, dim3(16), dim3(256), 0, s, b.counts, static_cast<const uint32_t*>(b.kps),
                       reinterpret_cast<const uint4*>(b.desc), guess, reinterpret_cast<int*>(c->pin_dev + o_n),
                       reinterpret_cast<uint32_t*>(c->pin_dev + o_k), reinterpret_cast<uint4*>(c->pin_dev + o_d));
    HIP_TRY(c, hipGetLastError());
    if ((rc = err_word_async(c, c->pin + o_n + 16))) return rc;
    HIP_TRY(c, hipStreamSynchronize(s));
    if ((rc = err_word_seen(c, c->pin + o_n + 16))) return rc;
    int n = 0;
    memcpy(&n, c->pin + o_n, 4);
    *n_out = n;
    const int m = std::min(n, cap);
    if (m > guess) {                         // past the packed records (or one output array only)
        const size_t r = (size_t)(m - guess);
        if (kp_out)
            HIP_TRY(c, hipMemcpyAsync(c->pin + o_k + (size_t)guess * sizeof(coeb_keypoint), static_cast<const coeb_keypoint*>(b.kps) + guess,
                                      r * sizeof(coeb_keypoint), hipMemcpyDeviceToHost, s));
        if (desc_out) HIP_TRY(c, hipMemcpyAsync(c->pin + o_d + (size_t)guess * 32, b.desc + (size_t)guess * 32, r * 32,
                                                hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipStreamSynchronize(s));
    }
    if (m > 0 && kp_out) memcpy(kp_out, c->pin + o_k, (size_t)m * sizeof(coeb_keypoint));
    if (m > 0 && desc_out) memcpy(desc_out, c->pin + o_d, (size_t)m * 32);
    if (n > cap) return set_err(c, COEB_ERANGE, "keypoint output capacity too small");
    return COEB_OK;
}

static MatchCam make_cam(const coeb_ctx* c, const coeb_camera* cam)
{
    MatchCam m;
    memset(&m, 0, sizeof(m));
    m.fx = cam->fx; m.fy = cam->fy; m.cx = cam->cx; m.cy = cam->cy; m.bf = cam->bf;
    m.mb = cam->bf / cam->fx;                                       // Frame.cc:246
    m.min_x = cam->min_x; m.max_x = cam->max_x; m.min_y = cam->min_y; m.max_y = cam->max_y;
    m.grid_inv_w = (float)COEB_GRID_COLS / (cam->max_x - cam->min_x);   // Frame.cc:233-234
    m.grid_inv_h = (float)COEB_GRID_ROWS / (cam->max_y - cam->min_y);
    for (int l = 0; l < c->tab.nlevels; l++) m.scale[l] = c->tab.scale[l];
    m.nlevels = c->tab.nlevels;
    // mfLogScaleFactor = log(mfScaleFactor): std::log(float), canonical correctly rounded
    m.log_sf = (float)std::log((double)(float)c->tab.scale_factor);
    return m;
}

int coeb_match_lastframe(coeb_ctx* c, const coeb_camera* cam, const coeb_curframe* cur, const coeb_lastframe* last,
                         const float Tcw_cur[16], const float Tcw_last[16], float th, int bmono, int check_ori,
                         int32_t* match_out, int* nmatches)
{
    if (!c || !cam || !cur || !last || !Tcw_cur || !Tcw_last || !nmatches)
        return set_err(c, COEB_EINVAL, "coeb_match_lastframe: invalid arguments");
    *nmatches = 0;
    if (cur->n < 0 || last->n < 0) return set_err(c, COEB_EINVAL, "negative frame size");
    if (cur->n > kCurMax) return set_err(c, COEB_EINVAL, "more than 4095 current keypoints");
    const int n = cur->n, nl = last->n;
    if (n && (!cur->keys_un || !cur->descriptors || !cur->u_right))
        return set_err(c, COEB_EINVAL, "coeb_match_lastframe: missing current-frame arrays");
    if (nl && (!last->has_mappoint || !last->outlier || !last->world_pos || !last->mp_descriptor ||
               !last->mp_observations || !last->keys_un))
        return set_err(c, COEB_EINVAL, "coeb_match_lastframe: missing LastFrame arrays");
    // the kernel indexes mvScaleFactors[octave] of every LastFrame point with a MapPoint
    for (int i = 0; i < nl; i++)
        if (last->has_mappoint[i] && (last->keys_un[i].octave < 0 || last->keys_un[i].octave >= c->params.nlevels))
            return set_err(c, COEB_EINVAL, "coeb_match_lastframe: LastFrame keypoint octave outside the pyramid");
    (void)hipSetDevice(c->device);
    const int cs = std::max(n, 1), ls = std::max(nl, 1);
    int rc;
    int32_t *dscr, *derr, *dqn;
    uint8_t* dbase;
    if ((rc = ensure(c, "m_scr", (size_t)ls * kMatchCQ, &dscr)) || (rc = ensure(c, "m_qn", (size_t)ls + 8, &dqn)) ||
        (rc = ensure(c, "err", 4, &derr)))
        return rc;
    hipStream_t s = main_stream(c);
    // every input in one pinned staged copy (ten small pageable copies cost more than the kernel)
    const int32_t cnts[2] = {n, nl};
    Pack pk;
    const size_t o_cn = pk.add(cnts, 8), o_T = pk.add(Tcw_cur, 64), o_Tl = pk.add(Tcw_last, 64);
    const size_t o_ck = pk.add(cur->keys_un, (size_t)n * sizeof(coeb_keypoint)), o_cd = pk.add(cur->descriptors, (size_t)n * 32);
    const size_t o_ur = pk.add(cur->u_right, (size_t)n * 4);
    const size_t o_lk = pk.add(last->keys_un, (size_t)nl * sizeof(coeb_keypoint));
    const size_t o_ld = pk.add(last->mp_descriptor, (size_t)nl * 32), o_h = pk.add(last->has_mappoint, (size_t)nl);
    const size_t o_o = pk.add(last->outlier, (size_t)nl), o_xw = pk.add(last->world_pos, (size_t)nl * 12);
    const size_t o_nb = pk.add(last->mp_observations, (size_t)nl * 4);
    // k_match writes match[cs] and nmatches straight behind the staged inputs (page-locked, no
    // copy back)
    const size_t o_res = (pk.total + 255) & ~(size_t)255;
    const size_t o_err = (o_res + ((size_t)cs + 1) * 4 + 15) & ~(size_t)15;
    if ((rc = pinned(c, o_err + 16)) || (rc = stage_in(c, pk, &dbase, s))) return rc;
    int32_t* dout = reinterpret_cast<int32_t*>(c->pin_dev + o_res);
    MatchBufs mb;
    memset(&mb, 0, sizeof(mb));
    mb.cur_kps = reinterpret_cast<const coeb_keypoint*>(dbase + o_ck);
    mb.cur_desc = dbase + o_cd;
    mb.cur_n = reinterpret_cast<const int32_t*>(dbase + o_cn);
    mb.cur_ur = reinterpret_cast<const float*>(dbase + o_ur);
    mb.cur_stride = cs;
    mb.last_kps = reinterpret_cast<const coeb_keypoint*>(dbase + o_lk);
    mb.last_desc = dbase + o_ld;
    mb.last_n = reinterpret_cast<const int32_t*>(dbase + o_cn) + 1;
    mb.last_has = dbase + o_h;
    mb.last_out = dbase + o_o;
    mb.last_xw = reinterpret_cast<const float*>(dbase + o_xw);
    mb.last_nobs = reinterpret_cast<const int32_t*>(dbase + o_nb);
    mb.last_stride = ls;
    mb.Tcw_cur = reinterpret_cast<const float*>(dbase + o_T);
    mb.Tcw_last = reinterpret_cast<const float*>(dbase + o_Tl);
    mb.match = dout; mb.nmatch = dout + cs; mb.scratch = dscr; mb.scratch_stride = ls * kMatchCQ; mb.err = derr;
    // one pair: its candidate lists are built by 8 workgroups (k_match_lists), as for a small
    // batch, instead of by the pair's one workgroup
    mb.qn = dqn; mb.qn_stride = ls + 8;
    if (launch_match(make_cam(c, cam), mb, 1, th, bmono, check_ori, 0, s, &c->hook))
        return hip_err(c, hipGetLastError(), "launch_match");
    if ((rc = err_word_async(c, c->pin + o_err))) return rc;
    HIP_TRY(c, hipStreamSynchronize(s));
    if ((rc = err_word_seen(c, c->pin + o_err))) return rc;
    const int32_t* hout = reinterpret_cast<const int32_t*>(c->pin + o_res);    // written by k_match in place
    if (n && match_out) memcpy(match_out, hout, (size_t)n * 4);
    *nmatches = hout[cs];
    return COEB_OK;
}

int coeb_match_localmap(coeb_ctx* c, const coeb_camera* cam, const coeb_curframe* cur, const int32_t* cur_obs,
                        const coeb_localmap* mp, float th, float nnratio, int32_t* match_out, int* nmatches)
{
    if (!c || !cam || !cur || !mp || !nmatches) return set_err(c, COEB_EINVAL, "coeb_match_localmap: invalid arguments");
    *nmatches = 0;
    if (cur->n < 0 || mp->n < 0) return set_err(c, COEB_EINVAL, "negative frame / local map size");
    if (cur->n > kCurMax) return set_err(c, COEB_EINVAL, "more than 4095 current keypoints");
    const int n = cur->n, nq = mp->n;
    if (n && (!cur->keys_un || !cur->descriptors || !cur->u_right))
        return set_err(c, COEB_EINVAL, "coeb_match_localmap: missing current-frame arrays");
    if (nq && (!mp->in_view || !mp->proj_x || !mp->proj_y || !mp->proj_xr || !mp->level || !mp->view_cos ||
               !mp->descriptor || !mp->observations))
        return set_err(c, COEB_EINVAL, "coeb_match_localmap: missing local-map arrays");
    // the kernel indexes mvScaleFactors[level] for every point in view
    for (int q = 0; q < nq; q++)
        if (mp->in_view[q] && (mp->level[q] < 0 || mp->level[q] >= c->tab.nlevels))
            return set_err(c, COEB_EINVAL, "coeb_match_localmap: predicted level outside the pyramid");
    (void)hipSetDevice(c->device);
    const int cs = std::max(n, 1), qs = std::max(nq, 1);
    int rc;
    int32_t *dout, *derr, *dpath;
    uint32_t* dlist;
    uint8_t* dbase;
    if ((rc = ensure(c, "l_out", (size_t)cs + 1, &dout)) || (rc = ensure(c, "l_list", (size_t)qs * match_list_cap(), &dlist)) ||
        (rc = ensure(c, "err", 4, &derr)) || (rc = ensure(c, "l_path", 2, &dpath)))
        return rc;
    hipStream_t s = main_stream(c);
    Pack pk;
    const size_t o_k = pk.add(cur->keys_un, (size_t)n * sizeof(coeb_keypoint)), o_d = pk.add(cur->descriptors, (size_t)n * 32);
    const size_t o_ur = pk.add(cur->u_right, (size_t)n * 4);
    const size_t o_co = cur_obs ? pk.add(cur_obs, (size_t)n * 4) : pk.fill(0xff, (size_t)n * 4);   // -1: all NULL
    const size_t o_v = pk.add(mp->in_view, (size_t)nq), o_px = pk.add(mp->proj_x, (size_t)nq * 4);
    const size_t o_py = pk.add(mp->proj_y, (size_t)nq * 4), o_pxr = pk.add(mp->proj_xr, (size_t)nq * 4);
    const size_t o_l = pk.add(mp->level, (size_t)nq * 4), o_c = pk.add(mp->view_cos, (size_t)nq * 4);
    const size_t o_qd = pk.add(mp->descriptor, (size_t)nq * 32), o_no = pk.add(mp->observations, (size_t)nq * 4);
    if ((rc = stage_in(c, pk, &dbase, s))) return rc;
    LocalBufsHost b;
    b.cur_kps = dbase + o_k; b.cur_desc = dbase + o_d; b.cur_ur = (const float*)(dbase + o_ur);
    b.cur_obs = (const int*)(dbase + o_co); b.cur_n = n;
    b.in_view = dbase + o_v; b.proj_x = (const float*)(dbase + o_px); b.proj_y = (const float*)(dbase + o_py);
    b.proj_xr = (const float*)(dbase + o_pxr); b.level = (const int*)(dbase + o_l); b.view_cos = (const float*)(dbase + o_c);
    b.desc = dbase + o_qd; b.nobs = (const int*)(dbase + o_no); b.mp_n = nq;
    b.match = dout; b.nmatch = dout + cs; b.lists = dlist; b.err = derr; b.path = dpath;
    rc = launch_match_local(make_cam(c, cam), b, th, nnratio, s, &c->hook);
    if (rc == -2) return set_err(c, COEB_ERANGE, "coeb_match_localmap: frame and local map exceed the LDS budget");
    if (rc) return hip_err(c, hipGetLastError(), "launch_match_local");
    int32_t* hout = reinterpret_cast<int32_t*>(c->pin);          // one copy back: match[cs], nmatch
    HIP_TRY(c, hipMemcpyAsync(hout, dout, ((size_t)cs + 1) * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if ((rc = check_err_word(c))) return rc;
    if (n && match_out) memcpy(match_out, hout, (size_t)n * 4);
    *nmatches = hout[cs];
    return COEB_OK;
}

int coeb_match_keyframe(coeb_ctx* c, const coeb_camera* cam, const coeb_curframe* cur, const uint8_t* cur_has,
                        const coeb_keyframe_points* kf, const float Tcw[16], float th, int orb_dist, int check_ori,
                        int32_t* match_out, int* nmatches)
{
    if (!c || !cam || !cur || !kf || !Tcw || !nmatches) return set_err(c, COEB_EINVAL, "coeb_match_keyframe: invalid arguments");
    *nmatches = 0;
    if (cur->n < 0 || kf->n < 0) return set_err(c, COEB_EINVAL, "negative frame / keyframe size");
    if (cur->n > kCurMax) return set_err(c, COEB_EINVAL, "more than 4095 current keypoints");
    const int n = cur->n, nq = kf->n;
    if (n && (!cur->keys_un || !cur->descriptors)) return set_err(c, COEB_EINVAL, "coeb_match_keyframe: missing current-frame arrays");
    if (nq && (!kf->valid || !kf->world_pos || !kf->descriptor || !kf->max_distance || !kf->min_distance || !kf->angle))
        return set_err(c, COEB_EINVAL, "coeb_match_keyframe: missing keyframe arrays");
    (void)hipSetDevice(c->device);
    const int cs = std::max(n, 1), qs = std::max(nq, 1);
    int rc;
    int32_t *dout, *derr, *dpath;
    uint32_t* dlist;
    uint8_t* dbase;
    if ((rc = ensure(c, "l_out", (size_t)cs + 1, &dout)) || (rc = ensure(c, "l_list", (size_t)qs * match_list_cap(), &dlist)) ||
        (rc = ensure(c, "err", 4, &derr)) || (rc = ensure(c, "l_path", 2, &dpath)))
        return rc;
    hipStream_t s = main_stream(c);
    Pack pk;
    const size_t o_k = pk.add(cur->keys_un, (size_t)n * sizeof(coeb_keypoint)), o_d = pk.add(cur->descriptors, (size_t)n * 32);
    const size_t o_h = cur_has ? pk.add(cur_has, (size_t)n) : pk.fill(0, (size_t)n);
    const size_t o_v = pk.add(kf->valid, (size_t)nq), o_x = pk.add(kf->world_pos, (size_t)nq * 12);
    const size_t o_qd = pk.add(kf->descriptor, (size_t)nq * 32), o_mx = pk.add(kf->max_distance, (size_t)nq * 4);
    const size_t o_mn = pk.add(kf->min_distance, (size_t)nq * 4), o_a = pk.add(kf->angle, (size_t)nq * 4);
    const size_t o_T = pk.add(Tcw, 64);
    if ((rc = stage_in(c, pk, &dbase, s))) return rc;
    KfBufsHost b;
    b.cur_kps = dbase + o_k; b.cur_desc = dbase + o_d; b.cur_has = dbase + o_h; b.cur_n = n;
    b.valid = dbase + o_v; b.xw = (const float*)(dbase + o_x); b.desc = dbase + o_qd;
    b.maxd = (const float*)(dbase + o_mx); b.mind = (const float*)(dbase + o_mn); b.angle = (const float*)(dbase + o_a);
    b.kf_n = nq; b.Tcw = (const float*)(dbase + o_T);
    b.match = dout; b.nmatch = dout + cs; b.lists = dlist; b.err = derr; b.path = dpath;
    rc = launch_match_kf(make_cam(c, cam), b, th, orb_dist, check_ori ? 1 : 0, s, &c->hook);
    if (rc == -2) return set_err(c, COEB_ERANGE, "coeb_match_keyframe: frame and keyframe exceed the LDS budget");
    if (rc) return hip_err(c, hipGetLastError(), "launch_match_kf");
    int32_t* hout = reinterpret_cast<int32_t*>(c->pin);          // one copy back: match[cs], nmatch
    HIP_TRY(c, hipMemcpyAsync(hout, dout, ((size_t)cs + 1) * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if ((rc = check_err_word(c))) return rc;
    if (n && match_out) memcpy(match_out, hout, (size_t)n * 4);
    *nmatches = hout[cs];
    return COEB_OK;
}

int coeb_pose_optimization(coeb_ctx* c, const coeb_camera* cam, const coeb_pose_frame* fr, float Tcw[16],
                           uint8_t* outlier_out, int* ninliers)
{
    if (!c || !cam || !fr || !Tcw || !ninliers) return set_err(c, COEB_EINVAL, "coeb_pose_optimization: invalid arguments");
    *ninliers = 0;
    const int n = fr->n;
    if (n < 0) return set_err(c, COEB_EINVAL, "negative frame size");
    if (n && (!fr->has_mappoint || !fr->world_pos || !fr->keys_un || !fr->u_right))
        return set_err(c, COEB_EINVAL, "coeb_pose_optimization: missing frame arrays");
    for (int i = 0; i < n; i++)
        if (fr->has_mappoint[i] && (fr->keys_un[i].octave < 0 || fr->keys_un[i].octave >= c->tab.nlevels))
            return set_err(c, COEB_EINVAL, "coeb_pose_optimization: keypoint octave outside the pyramid");
    (void)hipSetDevice(c->device);
    const int cs = std::max(n, 1);
    int rc;
    uint8_t *dact, *dbase;
    PoseEdgeRec* dedge;
    double* dchi;
    if ((rc = ensure(c, "p_act", cs, &dact)) || (rc = ensure(c, "p_edge", cs, &dedge)) || (rc = ensure(c, "p_chi", cs, &dchi)))
        return rc;
    hipStream_t s = main_stream(c);
    // one staged region: outputs first (result, pose, outlier flags; copied back in one go), then inputs
    Pack pk;
    const size_t o_n = pk.add(&fr->n, 4), o_res = pk.fill(0, 4), o_T = pk.add(Tcw, 64), o_out = pk.fill(0, (size_t)cs);
    const size_t head = o_out + (size_t)cs;
    const size_t o_h = pk.add(fr->has_mappoint, (size_t)n), o_x = pk.add(fr->world_pos, (size_t)n * 12);
    const size_t o_k = pk.add(fr->keys_un, (size_t)n * sizeof(coeb_keypoint)), o_ur = pk.add(fr->u_right, (size_t)n * 4);
    const size_t o_is = pk.add(c->tab.inv_sigma2, sizeof(float) * COEB_MAXL);
    if ((rc = stage_in(c, pk, &dbase, s))) return rc;
    PoseBufs b;
    b.n = (const int*)(dbase + o_n); b.has_mp = dbase + o_h; b.xw = (const float*)(dbase + o_x); b.kps = dbase + o_k;
    b.ur = (const float*)(dbase + o_ur); b.inv_sigma2 = (const float*)(dbase + o_is); b.Tcw = (float*)(dbase + o_T);
    b.outlier = dbase + o_out; b.result = (int*)(dbase + o_res); b.edges = dedge; b.active = dact; b.chi2 = dchi;
    b.timing = nullptr;
    b.stride = cs;
    if (launch_pose(b, 1, cam->fx, cam->fy, cam->cx, cam->cy, cam->bf, s, &c->hook))
        return hip_err(c, hipGetLastError(), "launch_pose");
    HIP_TRY(c, hipMemcpyAsync(c->pin, dbase, head, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    int res;
    memcpy(&res, c->pin + o_res, 4);
    memcpy(Tcw, c->pin + o_T, 64);
    if (n && outlier_out)
        for (int i = 0; i < n; i++)
            if (fr->has_mappoint[i]) outlier_out[i] = c->pin[o_out + i];
    *ninliers = res;
    return COEB_OK;
}

namespace {

// Common body of the batch matchers.  dT_cur: device poses, pair p (current frame p+1) at
// dT_cur + 16 p; LastFrame poses are identities (frame p is the world frame of its pair).
int match_batch_impl(coeb_ctx* c, const float* d_depth, int F, int W, int H, const coeb_camera* cam,
                     const float* dT_cur, float th, int32_t nobs, bool wait_main)
{
    const int K = c->plan.kcap;
    if (K > kCurMax) return set_err(c, COEB_EINVAL, "keypoint capacity exceeds the matcher limit (4095)");
    int rc;
    float *ur, *dep, *xw, *dI;
    uint8_t *has, *outl;
    int32_t *nobsb, *match, *nm, *scr, *mqn, *derr;
    const int qs = K + 8;                                   // split-list counts + 8 flags per pair
    if ((rc = ensure(c, "b_mqn", (size_t)F * qs, &mqn)) || (rc = ensure(c, "b_ur", (size_t)F * K, &ur)) || (rc = ensure(c, "b_dep", (size_t)F * K, &dep)) ||
        (rc = ensure(c, "b_xw", (size_t)F * K * 3, &xw)) || (rc = ensure(c, "b_has", (size_t)F * K, &has)) ||
        (rc = ensure(c, "b_outl", (size_t)F * K, &outl)) || (rc = ensure(c, "b_nobs", (size_t)F * K, &nobsb)) ||
        (rc = ensure(c, "b_match", (size_t)F * K, &match)) || (rc = ensure(c, "b_nm", (size_t)F, &nm)) ||
        (rc = ensure(c, "b_scr", (size_t)F * K * kMatchCQ, &scr)) || (rc = ensure(c, "err", 4, &derr)))
        return rc;
    if (c->ident_frames < F || !c->bufs.count("b_I")) {
        const int n = std::max(F, c->max_batch);
        HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
        if ((rc = ensure(c, "b_I", (size_t)n * 16, &dI))) return rc;
        std::vector<float> I((size_t)n * 16, 0.f);
        for (int p = 0; p < n; p++) I[(size_t)p * 16 + 0] = I[(size_t)p * 16 + 5] = I[(size_t)p * 16 + 10] = I[(size_t)p * 16 + 15] = 1.f;
        HIP_TRY(c, hipMemcpy(dI, I.data(), I.size() * 4, hipMemcpyHostToDevice));
        c->ident_frames = n;
    }
    dI = static_cast<float*>(c->bufs["b_I"].p);
    const coeb_keypoint* kps = static_cast<const coeb_keypoint*>(c->bufs["kps"].p);
    const uint8_t* desc = static_cast<const uint8_t*>(c->bufs["desc"].p);
    const int32_t* counts = static_cast<const int32_t*>(c->bufs["counts"].p);
    const MatchCam mcam = make_cam(c, cam);
    // chunk k (frames [f0, f1)) on its stream: prep, then the pairs whose current frame is in
    // the chunk; the first of them needs chunk k-1's last frame prepared
    const bool chunked = c->extract_chunked && (int)c->chunk.size() > 2 && c->chunk.back() == F;
    const int n = chunked ? (int)c->chunk.size() - 1 : 1;
    if (!chunked) main_stream(c);
    else if (wait_main) HIP_TRY(c, hipEventRecord(c->ev_main, c->stream));
    for (int k = 0; k < n; k++) {
        const int f0 = chunked ? c->chunk[k] : 0, f1 = chunked ? c->chunk[k + 1] : F;
        hipStream_t s = chunked ? c->subs[k] : main_stream(c);
        if (chunked && wait_main) HIP_TRY(c, hipStreamWaitEvent(s, c->ev_main, 0));
        PrepBufs pb;
        memset(&pb, 0, sizeof(pb));
        const int64_t o = (int64_t)f0 * K;
        pb.kps = kps + o; pb.n = counts + f0; pb.stride = K; pb.depth = d_depth + (int64_t)f0 * W * H; pb.W = W; pb.H = H;
        pb.bf = cam->bf; pb.fx = cam->fx; pb.fy = cam->fy; pb.cx = cam->cx; pb.cy = cam->cy;
        pb.ur = ur + o; pb.dep = dep + o; pb.has = has + o; pb.outl = outl + o; pb.xw = xw + 3 * o;
        pb.nobs = nobsb + o; pb.nobs_value = nobs;
        if (launch_prep(pb, f1 - f0, s, &c->hook)) return hip_err(c, hipGetLastError(), "launch_prep");
        if (chunked) {
            HIP_TRY(c, hipEventRecord(c->ev_prep[k], s));
            if (k > 0) HIP_TRY(c, hipStreamWaitEvent(s, c->ev_prep[k - 1], 0));
        }
        const int p0 = std::max(f0, 1) - 1, np = f1 - std::max(f0, 1);   // pair p: current p+1, last p
        if (np > 0) {
            const int64_t q = (int64_t)p0 * K;
            MatchBufs mb;
            memset(&mb, 0, sizeof(mb));
            mb.cur_kps = kps + q + K; mb.cur_desc = desc + (q + K) * 32; mb.cur_n = counts + p0 + 1; mb.cur_ur = ur + q + K;
            mb.cur_stride = K;
            mb.last_kps = kps + q; mb.last_desc = desc + q * 32; mb.last_n = counts + p0; mb.last_has = has + q;
            mb.last_out = outl + q; mb.last_xw = xw + 3 * q; mb.last_nobs = nobsb + q; mb.last_stride = K;
            mb.Tcw_cur = dT_cur + 16 * p0; mb.Tcw_last = dI + 16 * p0;
            mb.match = match + q + K; mb.nmatch = nm + p0 + 1; mb.scratch = scr + q * kMatchCQ;
            mb.scratch_stride = K * kMatchCQ; mb.err = derr;
            mb.qn = mqn + (int64_t)p0 * qs; mb.qn_stride = qs;
            if (COEB_MATCH_CLOCK && coeb_experiment("COEB_MATCH_TIMING")) {
                long long* tmb;
                if ((rc = ensure(c, "m_timing", (size_t)F * 16, &tmb))) return rc;
                mb.timing = tmb + (int64_t)p0 * 16;
            }
            if (launch_match(mcam, mb, np, th, 0, 1, 20, s, &c->hook)) return hip_err(c, hipGetLastError(), "launch_match");
        }
        if (chunked) HIP_TRY(c, hipEventRecord(c->ev_mdone[k], s));
    }
    c->mdone_valid = chunked;
    if (chunked) c->pending_join = true;
    c->batch_nobs = nobs;
    return COEB_OK;
}

int match_batch_check(coeb_ctx* c, const float* d_depth, int F, int W, int H, const coeb_camera* cam, const float* T)
{
    if (!c || !d_depth || !cam || !T || F <= 0) return set_err(c, COEB_EINVAL, "coeb_match_batch_device: invalid arguments");
    if (!c->has_plan || c->batch_frames != F || c->plan.W != W || c->plan.H != H)
        return set_err(c, COEB_EINVAL, "coeb_match_batch_device: must follow coeb_extract_batch_device on the same batch");
    return COEB_OK;
}

}  // namespace

int coeb_match_batch_device(coeb_ctx* c, const float* d_depth, int F, int W, int H, const coeb_camera* cam,
                            const float* Tcw, float th, int32_t nobs)
{
    int rc;
    if ((rc = match_batch_check(c, d_depth, F, W, H, cam, Tcw))) return rc;
    (void)hipSetDevice(c->device);
    float* dT;
    if ((rc = ensure(c, "b_T", (size_t)F * 16, &dT))) return rc;
    // the previous batch's matchers may still read b_T: join them before overwriting it
    HIP_TRY(c, hipMemcpyAsync(dT, Tcw, (size_t)F * 64, hipMemcpyHostToDevice, main_stream(c)));
    return match_batch_impl(c, d_depth, F, W, H, cam, dT + 16, th, nobs, true);
}

int coeb_match_batch_device_tcw(coeb_ctx* c, const float* d_depth, int F, int W, int H, const coeb_camera* cam,
                                const float* d_Tcw, float th, int32_t nobs)
{
    int rc;
    if ((rc = match_batch_check(c, d_depth, F, W, H, cam, d_Tcw))) return rc;
    (void)hipSetDevice(c->device);
    return match_batch_impl(c, d_depth, F, W, H, cam, d_Tcw + 16, th, nobs, false);
}

int coeb_batch_match_results(coeb_ctx* c, const int32_t** d_match, const int32_t** d_nmatches)
{
    if (!c) return COEB_EINVAL;
    if (d_match) *d_match = static_cast<const int32_t*>(c->bufs["b_match"].p);
    if (d_nmatches) *d_nmatches = static_cast<const int32_t*>(c->bufs["b_nm"].p);
    return COEB_OK;
}

int coeb_pose_batch_device(coeb_ctx* c, const coeb_camera* cam, int F, const float* d_Tcw, int32_t min_matches)
{
    if (!c || !cam || !d_Tcw || F <= 0) return set_err(c, COEB_EINVAL, "coeb_pose_batch_device: invalid arguments");
    if (!c->has_plan || c->batch_frames != F || !c->bufs.count("b_match") || !c->bufs.count("b_xw"))
        return set_err(c, COEB_EINVAL, "coeb_pose_batch_device: must follow coeb_match_batch_device on the same batch");
    (void)hipSetDevice(c->device);
    const int K = c->plan.kcap;
    int rc;
    float *tout, *txw, *isg, *tur;
    coeb_keypoint* tkp;
    uint8_t *thas, *toutl, *tact;
    int32_t *tn, *tres;
    PoseEdgeRec* tedge;
    double* tchi;
    if ((rc = ensure(c, "t_T", (size_t)F * 16, &tout)) || (rc = ensure(c, "t_xw", (size_t)F * K * 3, &txw)) ||
        (rc = ensure(c, "t_isg", COEB_MAXL, &isg)) || (rc = ensure(c, "t_has", (size_t)F * K, &thas)) ||
        (rc = ensure(c, "t_outl", (size_t)F * K, &toutl)) || (rc = ensure(c, "t_act", (size_t)F * K, &tact)) ||
        (rc = ensure(c, "t_n", (size_t)F, &tn)) || (rc = ensure(c, "t_res", (size_t)F, &tres)) ||
        (rc = ensure(c, "t_edge", (size_t)F * K, &tedge)) || (rc = ensure(c, "t_chi", (size_t)F * K, &tchi)) ||
        (rc = ensure(c, "t_kp", (size_t)F * K, &tkp)) || (rc = ensure(c, "t_ur", (size_t)F * K, &tur)))
        return rc;
    hipStream_t s = main_stream(c);                 // joins the matchers' chunk streams
    if (!c->pose_stream) {
        HIP_TRY(c, make_stream(&c->pose_stream, "COEB_POSE_PRIO"));
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_tprep, hipEventDisableTiming));
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_pose, hipEventDisableTiming));
    }
    join_pose(c);                                   // the previous batch's k_pose still reads t_*
    HIP_TRY(c, hipMemsetAsync(thas, 0, (size_t)F * K, s));
    HIP_TRY(c, hipMemsetAsync(toutl, 0, (size_t)F * K, s));
    HIP_TRY(c, hipMemsetAsync(tres, 0, (size_t)F * 4, s));
    TrackPrepBufs t;
    memset(&t, 0, sizeof(t));
    t.match = static_cast<const int32_t*>(c->bufs["b_match"].p);
    t.nmatch = static_cast<const int32_t*>(c->bufs["b_nm"].p);
    t.counts = static_cast<const int32_t*>(c->bufs["counts"].p);
    t.last_xw = static_cast<const float*>(c->bufs["b_xw"].p);
    t.kps_in = c->bufs["kps"].p; t.ur_in = static_cast<const float*>(c->bufs["b_ur"].p);
    t.kps_out = tkp; t.ur_out = tur;
    t.Tin = d_Tcw; t.Tout = tout; t.has = thas; t.xw = txw; t.n = tn; t.isg_out = isg;
    for (int l = 0; l < COEB_MAXL; l++) t.isg[l] = l < c->tab.nlevels ? c->tab.inv_sigma2[l] : 0.f;
    t.stride = K;
    t.min_matches = min_matches;
    if (launch_track_prep(t, F, s, &c->hook)) return hip_err(c, hipGetLastError(), "launch_track_prep");
    if (F < 2) return COEB_OK;
    const int64_t o = K;                            // frame 1 = current frame of pair 0
    PoseBufs b;
    b.n = tn + 1; b.has_mp = thas + o; b.xw = txw + 3 * o;
    b.kps = tkp + o; b.ur = tur + o;
    b.inv_sigma2 = isg; b.Tcw = tout + 16; b.outlier = toutl + o; b.result = tres + 1;
    b.edges = tedge + o; b.active = tact + o; b.chi2 = tchi + o; b.stride = K;
    b.timing = nullptr;
    if (coeb_experiment("COEB_POSE_TIMING")) {               // diagnostic phase clocks, tools/_pose_timing.py
        long long* tmb;
        if ((rc = ensure(c, "p_timing", (size_t)F * 8, &tmb))) return rc;
        HIP_TRY(c, hipMemsetAsync(tmb, 0, (size_t)F * 64, s));
        b.timing = tmb + 8;
    }
    HIP_TRY(c, hipEventRecord(c->ev_tprep, s));
    HIP_TRY(c, hipStreamWaitEvent(c->pose_stream, c->ev_tprep, 0));
    if (launch_pose(b, F - 1, cam->fx, cam->fy, cam->cx, cam->cy, cam->bf, c->pose_stream, &c->hook))
        return hip_err(c, hipGetLastError(), "launch_pose");
    HIP_TRY(c, hipEventRecord(c->ev_pose, c->pose_stream));
    c->pose_pending = true;
    c->pose_frames = F;
    c->pose_min_matches = min_matches;
    c->tlm_frames = 0;
    return COEB_OK;
}

int coeb_batch_pose_results(coeb_ctx* c, const float** d_Tcw, const int32_t** d_ninliers, const uint8_t** d_outlier)
{
    if (!c || !c->bufs.count("t_T")) return set_err(c, COEB_EINVAL, "coeb_batch_pose_results: no batch pose yet");
    join_pose(c);
    if (d_Tcw) *d_Tcw = static_cast<const float*>(c->bufs["t_T"].p);
    if (d_ninliers) *d_ninliers = static_cast<const int32_t*>(c->bufs["t_res"].p);
    if (d_outlier) *d_outlier = static_cast<const uint8_t*>(c->bufs["t_outl"].p);
    return COEB_OK;
}

int coeb_track_local_map_batch_device(coeb_ctx* c, const coeb_camera* cam, int F, int32_t nkf, float th, float nnratio)
{
    if (!c || !cam || F <= 0 || nkf < 1 || nkf > 2 || !(th > 0) || !(nnratio > 0))
        return set_err(c, COEB_EINVAL, "coeb_track_local_map_batch_device: invalid arguments");
    if (!c->has_plan || c->batch_frames != F || c->pose_frames != F || !c->bufs.count("t_T"))
        return set_err(c, COEB_EINVAL, "coeb_track_local_map_batch_device: must follow coeb_pose_batch_device on the same batch");
    if (c->tlm_frames) return set_err(c, COEB_EINVAL, "coeb_track_local_map_batch_device: already run on this batch");
    (void)hipSetDevice(c->device);
    const int K = c->plan.kcap;
    const int64_t FK = (int64_t)F * K, FM = 2 * FK;
    int rc;
    TlmBufs t;
    memset(&t, 0, sizeof(t));
    uint8_t *s_desc, *s_has, *seen, *act, *inv, *has2, *outl2;
    int8_t* s_oct;
    float *s_xw, *px, *py, *pxr, *vc, *lxw, *xw2, *T2;
    int32_t *s_m1, *s_cnt, *s_nm1, *cobs, *nmap, *lvl, *lno, *lmatch, *nloc, *lpath, *n2, *res2, *derr;
    uint32_t* lists;
    if ((rc = ensure(c, "tl_sdesc", (size_t)(FK + K) * 32, &s_desc)) || (rc = ensure(c, "tl_soct", (size_t)FK, &s_oct)) ||
        (rc = ensure(c, "tl_shas", (size_t)FK, &s_has)) || (rc = ensure(c, "tl_sxw", (size_t)FK * 3, &s_xw)) ||
        (rc = ensure(c, "tl_sm1", (size_t)FK, &s_m1)) || (rc = ensure(c, "tl_scnt", (size_t)F, &s_cnt)) ||
        (rc = ensure(c, "tl_snm1", (size_t)F, &s_nm1)) || (rc = ensure(c, "tl_seen", (size_t)FK, &seen)) ||
        (rc = ensure(c, "tl_cobs", (size_t)FK, &cobs)) || (rc = ensure(c, "tl_nmap", (size_t)F, &nmap)) ||
        (rc = ensure(c, "tl_active", (size_t)F, &act)) || (rc = ensure(c, "tl_inview", (size_t)FM, &inv)) ||
        (rc = ensure(c, "tl_px", (size_t)FM, &px)) || (rc = ensure(c, "tl_py", (size_t)FM, &py)) ||
        (rc = ensure(c, "tl_pxr", (size_t)FM, &pxr)) || (rc = ensure(c, "tl_level", (size_t)FM, &lvl)) ||
        (rc = ensure(c, "tl_vcos", (size_t)FM, &vc)) || (rc = ensure(c, "tl_lnobs", (size_t)FM, &lno)) ||
        (rc = ensure(c, "tl_lxw", (size_t)FM * 3, &lxw)) || (rc = ensure(c, "tl_lmatch", (size_t)FK, &lmatch)) ||
        (rc = ensure(c, "tl_nlocal", (size_t)F, &nloc)) || (rc = ensure(c, "tl_path", (size_t)F * 2, &lpath)) ||
        (rc = ensure(c, "tl_lists", (size_t)FM * match_list_cap(), &lists)) ||
        (rc = ensure(c, "tl_has2", (size_t)FK, &has2)) || (rc = ensure(c, "tl_xw2", (size_t)FK * 3, &xw2)) ||
        (rc = ensure(c, "tl_T2", (size_t)F * 16, &T2)) || (rc = ensure(c, "tl_outl2", (size_t)FK, &outl2)) ||
        (rc = ensure(c, "tl_n2", (size_t)F, &n2)) || (rc = ensure(c, "tl_res2", (size_t)F, &res2)) ||
        (rc = ensure(c, "err", 4, &derr)))
        return rc;
    t.K = K; t.nkf = nkf; t.nobs = c->batch_nobs; t.min_matches = c->pose_min_matches; t.min_map = 10;
    t.kps = c->bufs["kps"].p; t.desc = static_cast<const uint8_t*>(c->bufs["desc"].p);
    t.counts = static_cast<const int32_t*>(c->bufs["counts"].p);
    t.match1 = static_cast<const int32_t*>(c->bufs["b_match"].p); t.nmatch1 = static_cast<const int32_t*>(c->bufs["b_nm"].p);
    t.has = static_cast<const uint8_t*>(c->bufs["b_has"].p); t.xw = static_cast<const float*>(c->bufs["b_xw"].p);
    t.s_desc = s_desc; t.s_oct = s_oct; t.s_has = s_has; t.s_xw = s_xw; t.s_m1 = s_m1; t.s_cnt = s_cnt; t.s_nm1 = s_nm1;
    t.T1 = static_cast<const float*>(c->bufs["t_T"].p); t.has1 = static_cast<const uint8_t*>(c->bufs["t_has"].p);
    t.outl1 = static_cast<const uint8_t*>(c->bufs["t_outl"].p); t.xw1 = static_cast<const float*>(c->bufs["t_xw"].p);
    t.seen = seen; t.cur_obs = cobs; t.nmap = nmap; t.active = act;
    t.in_view = inv; t.px = px; t.py = py; t.pxr = pxr; t.level = lvl; t.vcos = vc; t.lm_nobs = lno; t.lm_xw = lxw;
    t.lmatch = lmatch; t.has2 = has2; t.xw2 = xw2; t.T2 = T2; t.outl2 = outl2; t.n2 = n2;
    // the snapshot runs on the context stream, after this batch's matcher and before the next
    // batch's extraction; coeb_pose_batch_device already joined the previous pose-stream work
    hipStream_t s = main_stream(c);
    if (launch_tlm_snapshot(t, F, s, &c->hook)) return hip_err(c, hipGetLastError(), "launch_tlm_snapshot");
    if (F < 2) { c->tlm_frames = F; return COEB_OK; }
    if (!c->ev_tlm) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_tlm, hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(c->ev_tlm, s));
    hipStream_t ps = c->pose_stream;                // after the first k_pose
    HIP_TRY(c, hipStreamWaitEvent(ps, c->ev_tlm, 0));
    const MatchCam mcam = make_cam(c, cam);
    if (launch_tlm_frustum(mcam, t, F, ps, &c->hook)) return hip_err(c, hipGetLastError(), "launch_tlm_frustum");
    LocalBufsHost lb;
    lb.cur_kps = static_cast<const coeb_keypoint*>(c->bufs["t_kp"].p) + K;
    lb.cur_desc = s_desc + (int64_t)2 * K * 32;      // frame 1 = row 2
    lb.cur_ur = static_cast<const float*>(c->bufs["t_ur"].p) + K;
    lb.cur_obs = cobs + K; lb.cur_n = K;
    const int64_t M = 2 * (int64_t)K;
    lb.in_view = inv + M; lb.proj_x = px + M; lb.proj_y = py + M; lb.proj_xr = pxr + M; lb.level = lvl + M;
    lb.view_cos = vc + M; lb.nobs = lno + M; lb.mp_n = (int)M;
    lb.desc = s_desc;                                // frame 1's local map: KF2 = frame -1 (row 0), KF1 = frame 0
    lb.match = lmatch + K; lb.nmatch = nloc + 1; lb.lists = lists; lb.err = derr; lb.path = lpath + 2;
    lb.cur_n_arr = s_cnt + 1; lb.active = act + 1; lb.npairs = F - 1; lb.cur_stride = K; lb.mp_desc_stride = K;
    rc = launch_match_local(mcam, lb, th, nnratio, ps, &c->hook);
    if (rc == -2) return set_err(c, COEB_ERANGE, "coeb_track_local_map_batch_device: frame and local map exceed the LDS budget");
    if (rc) return hip_err(c, hipGetLastError(), "launch_match_local");
    if (launch_tlm_pose_prep(t, F, ps, &c->hook)) return hip_err(c, hipGetLastError(), "launch_tlm_pose_prep");
    PoseBufs b;
    const int64_t o = K;
    b.n = n2 + 1; b.has_mp = has2 + o; b.xw = xw2 + 3 * o;
    b.kps = static_cast<const coeb_keypoint*>(c->bufs["t_kp"].p) + o; b.ur = static_cast<const float*>(c->bufs["t_ur"].p) + o;
    b.inv_sigma2 = static_cast<const float*>(c->bufs["t_isg"].p); b.Tcw = T2 + 16; b.outlier = outl2 + o;
    b.result = res2 + 1;
    b.edges = static_cast<PoseEdgeRec*>(c->bufs["t_edge"].p) + o; b.active = static_cast<uint8_t*>(c->bufs["t_act"].p) + o;
    b.chi2 = static_cast<double*>(c->bufs["t_chi"].p) + o; b.stride = K; b.timing = nullptr;
    if (launch_pose(b, F - 1, cam->fx, cam->fy, cam->cx, cam->cy, cam->bf, ps, &c->hook))
        return hip_err(c, hipGetLastError(), "launch_pose");
    HIP_TRY(c, hipEventRecord(c->ev_pose, ps));
    c->pose_pending = true;
    c->tlm_frames = F;
    return COEB_OK;
}

int coeb_batch_track_results(coeb_ctx* c, const float** d_Tcw, const int32_t** d_ninliers, const int32_t** d_nmatches_map,
                             const int32_t** d_nlocal, const int32_t** d_local_match, const uint8_t** d_outlier)
{
    if (!c || !c->tlm_frames) return set_err(c, COEB_EINVAL, "coeb_batch_track_results: no batch TrackLocalMap yet");
    join_pose(c);
    if (d_Tcw) *d_Tcw = static_cast<const float*>(c->bufs["tl_T2"].p);
    if (d_ninliers) *d_ninliers = static_cast<const int32_t*>(c->bufs["tl_res2"].p);
    if (d_nmatches_map) *d_nmatches_map = static_cast<const int32_t*>(c->bufs["tl_nmap"].p);
    if (d_nlocal) *d_nlocal = static_cast<const int32_t*>(c->bufs["tl_nlocal"].p);
    if (d_local_match) *d_local_match = static_cast<const int32_t*>(c->bufs["tl_lmatch"].p);
    if (d_outlier) *d_outlier = static_cast<const uint8_t*>(c->bufs["tl_outl2"].p);
    return COEB_OK;
}

int coeb_stereo_from_rgbd(coeb_ctx* c, const coeb_keypoint* kps, int n, const float* depth, int W, int H,
                          size_t dstride, float bf, float* ur_out, float* dep_out)
{
    if (!c || (n > 0 && (!kps || !depth || !ur_out || !dep_out)) || n < 0 || dstride < (size_t)W)
        return set_err(c, COEB_EINVAL, "coeb_stereo_from_rgbd: invalid arguments");
    if (n == 0) return COEB_OK;
    (void)hipSetDevice(c->device);
    int rc;
    hipStream_t s = main_stream(c);
    // everything through the context's page-locked buffer, addressed by k_prep in place: the
    // keypoints and their count in, the depth rows (it touches ~n of the W*H values, so copying
    // the whole map to the device -- 1.2 MB at 640x480 -- would cost more than the lookups), and
    // uR / depth written straight back; one launch and one synchronisation, no copy operations
    const size_t o_n = 0, o_k = 256, o_dep = (o_k + (size_t)n * sizeof(coeb_keypoint) + 255) & ~(size_t)255;
    const size_t o_out = (o_dep + (size_t)W * H * 4 + 255) & ~(size_t)255;
    if ((rc = pinned(c, o_out + (size_t)n * 8))) return rc;
    memcpy(c->pin + o_n, &n, 4);
    memcpy(c->pin + o_k, kps, (size_t)n * sizeof(coeb_keypoint));
    float* hdep = reinterpret_cast<float*>(c->pin + o_dep);
    if (dstride == (size_t)W) memcpy(hdep, depth, (size_t)W * H * 4);
    else
        for (int y = 0; y < H; y++) memcpy(hdep + (size_t)y * W, depth + (size_t)y * dstride, (size_t)W * 4);
    PrepBufs pb;
    memset(&pb, 0, sizeof(pb));
    pb.kps = c->pin_dev + o_k;
    pb.n = reinterpret_cast<const int32_t*>(c->pin_dev + o_n);
    pb.stride = n; pb.depth = reinterpret_cast<const float*>(c->pin_dev + o_dep); pb.W = W; pb.H = H;
    pb.bf = bf; pb.fx = 1; pb.fy = 1;
    pb.ur = reinterpret_cast<float*>(c->pin_dev + o_out);
    pb.dep = reinterpret_cast<float*>(c->pin_dev + o_out) + n;
    if (launch_prep(pb, 1, s, &c->hook)) return hip_err(c, hipGetLastError(), "launch_prep");
    HIP_TRY(c, hipStreamSynchronize(s));
    memcpy(ur_out, c->pin + o_out, (size_t)n * 4);
    memcpy(dep_out, c->pin + o_out + (size_t)n * 4, (size_t)n * 4);
    return COEB_OK;
}

int coeb_descriptor_distance(const uint8_t* a, const uint8_t* b)
{
    // ORBmatcher::DescriptorDistance (ORBmatcher.cc:1648-1664): 8 x 32-bit XOR + popcount.
    // Kept on the CPU: it is also called one pair at a time from MapPoint/Frame code.
    int d = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

int coeb_profile_enable(coeb_ctx* c, int enable)
{
    if (!c) return COEB_EINVAL;
    c->prof.enabled = enable != 0;
    return COEB_OK;
}

int coeb_profile_reset(coeb_ctx* c)
{
    if (!c) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    c->prof.drain();
    std::fill(c->prof.ms.begin(), c->prof.ms.end(), 0.0);
    std::fill(c->prof.launches.begin(), c->prof.launches.end(), 0);
    return COEB_OK;
}

int coeb_profile_read(coeb_ctx* c, char* names, int cap, double* total_ms, int64_t* launches, int max_k, int* nk)
{
    if (!c) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    c->prof.drain();
    std::string s;
    const int k = std::min<int>(max_k, (int)c->prof.names.size());
    for (int i = 0; i < k; i++) {
        if (i) s += ",";
        s += c->prof.names[i];
        if (total_ms) total_ms[i] = c->prof.ms[i];
        if (launches) launches[i] = c->prof.launches[i];
    }
    if (names && cap > 0) {
        strncpy(names, s.c_str(), cap - 1);
        names[cap - 1] = 0;
    }
    if (nk) *nk = k;
    return COEB_OK;
}

int coeb_device_alloc(coeb_ctx* c, size_t bytes, void** dptr)
{
    if (!c || !dptr) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    hipError_t e = hipMalloc(dptr, std::max<size_t>(bytes, 1));
    if (e != hipSuccess) return set_err(c, COEB_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return COEB_OK;
}

int coeb_device_free(coeb_ctx* c, void* dptr)
{
    if (!c) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
    if (dptr) HIP_TRY(c, hipFree(dptr));
    return COEB_OK;
}

int coeb_memcpy_h2d(coeb_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c || (bytes && (!dst || !src))) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, main_stream(c)));
    HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
    return COEB_OK;
}

int coeb_memcpy_d2h(coeb_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c || (bytes && (!dst || !src))) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    join_pose(c);
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, main_stream(c)));
    HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
    return COEB_OK;
}

int coeb_host_alloc(size_t bytes, void** ptr)
{
    if (!ptr) return COEB_EINVAL;
    hipError_t e = hipHostMalloc(ptr, std::max<size_t>(bytes, 1), hipHostMallocDefault);
    if (e != hipSuccess) return set_err(nullptr, COEB_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    return COEB_OK;
}

int coeb_host_free(void* ptr)
{
    if (ptr && hipHostFree(ptr) != hipSuccess) return set_err(nullptr, COEB_EDEVICE, "hipHostFree failed");
    return COEB_OK;
}

int coeb_memcpy_h2d_async(coeb_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c || (bytes && (!dst || !src))) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, main_stream(c)));
    return COEB_OK;
}

int coeb_memcpy_d2h_async(coeb_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c || (bytes && (!dst || !src))) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    join_pose(c);
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, main_stream(c)));
    return COEB_OK;
}

// ---- copy queues: a stream of their own beside a context's stream (coeb_front.h) ----
// Each ordering call records a fresh event of a small ring: re-recording one event object while
// another stream still waits on its earlier record measured as a false dependency.
constexpr int kCopyqEvents = 16;
struct coeb_copyq {
    int device = 0;
    hipStream_t s = nullptr;
    hipEvent_t ev[kCopyqEvents] = {};
    int next = 0;
    hipEvent_t take() { hipEvent_t e = ev[next]; next = (next + 1) % kCopyqEvents; return e; }
};

coeb_copyq* coeb_copyq_create(coeb_ctx* c)
{
    if (!c) return nullptr;
    (void)hipSetDevice(c->device);
    coeb_copyq* q = new coeb_copyq;
    q->device = c->device;
    bool ok = hipStreamCreateWithFlags(&q->s, hipStreamNonBlocking) == hipSuccess;
    for (int i = 0; ok && i < kCopyqEvents; i++) ok = hipEventCreateWithFlags(&q->ev[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        set_err(c, COEB_EDEVICE, "coeb_copyq_create: stream / event creation failed");
        for (hipEvent_t e : q->ev)
            if (e) (void)hipEventDestroy(e);
        if (q->s) (void)hipStreamDestroy(q->s);
        delete q;
        return nullptr;
    }
    return q;
}

int coeb_copyq_destroy(coeb_copyq* q)
{
    if (!q) return COEB_OK;
    (void)hipSetDevice(q->device);
    (void)hipStreamSynchronize(q->s);
    for (hipEvent_t e : q->ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(q->s);
    delete q;
    return COEB_OK;
}

int coeb_copyq_h2d(coeb_copyq* q, void* dst, const void* src, size_t bytes)
{
    if (!q || (bytes && (!dst || !src))) return COEB_EINVAL;
    (void)hipSetDevice(q->device);
    if (hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, q->s) != hipSuccess)
        return set_err(nullptr, COEB_EDEVICE, "coeb_copyq_h2d: hipMemcpyAsync failed");
    return COEB_OK;
}

int coeb_copyq_d2h(coeb_copyq* q, void* dst, const void* src, size_t bytes)
{
    if (!q || (bytes && (!dst || !src))) return COEB_EINVAL;
    (void)hipSetDevice(q->device);
    if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, q->s) != hipSuccess)
        return set_err(nullptr, COEB_EDEVICE, "coeb_copyq_d2h: hipMemcpyAsync failed");
    return COEB_OK;
}

int coeb_copyq_after_ctx(coeb_copyq* q, coeb_ctx* c)
{
    if (!q || !c || q->device != c->device) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    hipStream_t s = main_stream(c);
    join_pose(c);
    hipEvent_t e = q->take();
    HIP_TRY(c, hipEventRecord(e, s));
    HIP_TRY(c, hipStreamWaitEvent(q->s, e, 0));
    return COEB_OK;
}

int coeb_ctx_after_copyq(coeb_ctx* c, coeb_copyq* q)
{
    if (!q || !c || q->device != c->device) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    hipEvent_t e = q->take();
    HIP_TRY(c, hipEventRecord(e, q->s));
    HIP_TRY(c, hipStreamWaitEvent(main_stream(c), e, 0));
    return COEB_OK;
}

int coeb_copyq_synchronize(coeb_copyq* q)
{
    if (!q) return COEB_EINVAL;
    (void)hipSetDevice(q->device);
    if (hipStreamSynchronize(q->s) != hipSuccess) return set_err(nullptr, COEB_EDEVICE, "coeb_copyq_synchronize failed");
    return COEB_OK;
}

// ---- markers (coeb_front.h): one HIP event, recorded on a context's or queue's stream ----
struct coeb_marker {
    int device = 0;
    hipEvent_t ev = nullptr;
};

coeb_marker* coeb_marker_create(coeb_ctx* c)
{
    if (!c) return nullptr;
    (void)hipSetDevice(c->device);
    coeb_marker* m = new coeb_marker;
    m->device = c->device;
    if (hipEventCreateWithFlags(&m->ev, hipEventDisableTiming) != hipSuccess) {
        set_err(c, COEB_EDEVICE, "coeb_marker_create: event creation failed");
        delete m;
        return nullptr;
    }
    return m;
}

int coeb_marker_destroy(coeb_marker* m)
{
    if (!m) return COEB_OK;
    (void)hipSetDevice(m->device);
    (void)hipEventSynchronize(m->ev);
    (void)hipEventDestroy(m->ev);
    delete m;
    return COEB_OK;
}

int coeb_marker_record_ctx(coeb_marker* m, coeb_ctx* c)
{
    if (!m || !c || m->device != c->device) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    hipStream_t s = main_stream(c);          // joins pending side-stream work first
    join_pose(c);
    HIP_TRY(c, hipEventRecord(m->ev, s));
    return COEB_OK;
}

int coeb_marker_record_copyq(coeb_marker* m, coeb_copyq* q)
{
    if (!m || !q || m->device != q->device) return COEB_EINVAL;
    (void)hipSetDevice(q->device);
    if (hipEventRecord(m->ev, q->s) != hipSuccess) return set_err(nullptr, COEB_EDEVICE, "coeb_marker_record_copyq failed");
    return COEB_OK;
}

int coeb_ctx_wait_marker(coeb_ctx* c, coeb_marker* m)
{
    if (!m || !c || m->device != c->device) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    HIP_TRY(c, hipStreamWaitEvent(main_stream(c), m->ev, 0));
    return COEB_OK;
}

int coeb_copyq_wait_marker(coeb_copyq* q, coeb_marker* m)
{
    if (!m || !q || m->device != q->device) return COEB_EINVAL;
    (void)hipSetDevice(q->device);
    if (hipStreamWaitEvent(q->s, m->ev, 0) != hipSuccess) return set_err(nullptr, COEB_EDEVICE, "coeb_copyq_wait_marker failed");
    return COEB_OK;
}

int coeb_marker_synchronize(coeb_marker* m)
{
    if (!m) return COEB_EINVAL;
    (void)hipSetDevice(m->device);
    if (hipEventSynchronize(m->ev) != hipSuccess) return set_err(nullptr, COEB_EDEVICE, "coeb_marker_synchronize failed");
    return COEB_OK;
}

int coeb_internal_stream(coeb_ctx* c, hipStream_t* s, int* device)
{
    if (!c) return COEB_EINVAL;
    *s = main_stream(c);
    *device = c->device;
    return COEB_OK;
}

// The side stream for the moving-object batch's LK pyramids, with the context's fork / join events
// (created on first use), when COEB_FLOW_SIDE=1; nonzero otherwise (also with the side stream off
// or per-kernel profiling), and then everything stays on the context stream.  Off by default: config
// D's step measured 13.30-13.37 ms with the fork against 13.10-13.30 without (profiles/r05/s24): the
// step is bound by the kernels' combined demand for CUs, not by the context stream's chain.
int coeb_internal_flow_side(coeb_ctx* c, hipStream_t* side, hipEvent_t* fork, hipEvent_t* join)
{
    if (!c) return COEB_EINVAL;
    const char* e = coeb_experiment("COEB_FLOW_SIDE");
    if (!(e && e[0] == '1')) return 1;
    const SideStream* sd = side_stream(c);
    if (!sd) return 1;
    if (!c->ev_ffork && (hipEventCreateWithFlags(&c->ev_ffork, hipEventDisableTiming) != hipSuccess ||
                         hipEventCreateWithFlags(&c->ev_fjoin, hipEventDisableTiming) != hipSuccess)) {
        if (c->ev_ffork) (void)hipEventDestroy(c->ev_ffork);
        c->ev_ffork = c->ev_fjoin = nullptr;
        return 1;
    }
    *side = sd->s;
    *fork = c->ev_ffork;
    *join = c->ev_fjoin;
    return 0;
}

int coeb_internal_scratch(coeb_ctx* c, const char* name, size_t bytes, void** p)
{
    uint8_t* q;
    int rc = ensure(c, name, bytes, &q);
    *p = q;
    return rc;
}

int coeb_internal_error(coeb_ctx* c, int code, const char* msg) { return set_err(c, code, msg); }

ProfileHook* coeb_internal_prof(coeb_ctx* c) { return c ? &c->hook : nullptr; }

/* Debug readback of intermediate buffers of frame f of the last batch (test support):
 * what = "pyr" | "blur" | "cand_n" | "lvl_n" | "lvl_kp" | "dyn"; copies min(bytes, size). */
int coeb_debug_read(coeb_ctx* c, const char* what, int f, void* host, size_t bytes, size_t* size_out)
{
    if (c) join_pose(c);
    if (c && what && std::string(what) == "fast_timing") {
        // [8] k_fast phase clocks (COEB_FAST_CLOCK builds)
        unsigned long long t[8];
        if (size_out) *size_out = sizeof(t);
        if (!host) return 0;                         // size query: the read below also clears
        if (fast_timing_read(t)) return COEB_EDEVICE;
        memcpy(host, t, std::min(bytes, sizeof(t)));
        return 0;
    }
    if (c && what && std::string(what) == "flow_counts") {     // [pairs][2] {Harris keys, corners}
        static thread_local int t[2 * 8192];
        int np = 0;
        int rc = coeb_internal_flow_counts(c, t, 2 * 8192, &np);
        if (rc) return rc;
        const size_t n = (size_t)std::min(np, 8192) * 8;
        if (size_out) *size_out = n;
        if (host) memcpy(host, t, std::min(bytes, n));
        return COEB_OK;
    }
    if (c && what && std::string(what) == "oct_timing") {       // [4096][6] k_octree clocks (COEB_OCT_CLOCK)
        static long long t[4096 * 6];
        if (size_out) *size_out = sizeof(t);
        if (!host) return 0;
        HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
        if (oct_timing_read(t)) return COEB_EDEVICE;
        memcpy(host, t, std::min(bytes, sizeof(t)));
        return 0;
    }
    if (c && what && std::string(what) == "pose_timing") {      // [F][8] k_pose phase clocks (COEB_POSE_TIMING)
        if (!c->bufs.count("p_timing")) return COEB_EINVAL;
        join_pose(c);
        const size_t nb = c->bufs["p_timing"].n;
        if (size_out) *size_out = nb;
        if (host && bytes) {
            HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
            HIP_TRY(c, hipMemcpy(host, c->bufs["p_timing"].p, std::min(bytes, nb), hipMemcpyDeviceToHost));
        }
        return COEB_OK;
    }
    if (c && what && std::string(what) == "match_timing") {     // [F][16] k_match phase clocks (COEB_MATCH_TIMING)
        if (!c->bufs.count("m_timing")) return COEB_EINVAL;
        const size_t nb = c->bufs["m_timing"].n;
        if (size_out) *size_out = nb;
        if (host && bytes) {
            HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
            HIP_TRY(c, hipMemcpy(host, c->bufs["m_timing"].p, std::min(bytes, nb), hipMemcpyDeviceToHost));
        }
        return COEB_OK;
    }
    if (c && what && (std::string(what) == "search_path" || std::string(what) == "localmap_path")) {
        // {path, iterations} of the last coeb_match_localmap / coeb_match_keyframe
        if (!c->bufs.count("l_path")) return COEB_EINVAL;
        if (size_out) *size_out = 8;
        if (host && bytes) {
            HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
            HIP_TRY(c, hipMemcpy(host, c->bufs["l_path"].p, std::min(bytes, (size_t)8), hipMemcpyDeviceToHost));
        }
        return COEB_OK;
    }
    if (!c || !what || !c->has_plan || f < 0 || f >= c->batch_frames) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    const Plan& P = c->plan;
    const uint8_t* src = nullptr;
    size_t n = 0;
    std::string w(what);
    if (w == "pyr") { src = (const uint8_t*)c->bufs["pyr"].p + (size_t)f * P.pyr_stride; n = P.pyr_stride; }
    else if (w == "blur") {
        // the blurred levels row-major at their pitch, each 256-B aligned (the device copy is tiled,
        // blur_tile_off)
        std::vector<uint8_t> raw(P.blur_stride);
        HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
        HIP_TRY(c, hipMemcpy(raw.data(), (const uint8_t*)c->bufs["blur"].p + (size_t)f * P.blur_stride, raw.size(),
                             hipMemcpyDeviceToHost));
        std::vector<uint8_t> rm;
        size_t off = 0;
        for (int l = 0; l < P.L; l++) {
            const LevelGeom& g = P.lv[l];
            rm.resize(off + (size_t)g.bpitch * g.h);
            for (int y = 0; y < g.h; y++)
                for (int x = 0; x < g.bpitch; x++)
                    rm[off + (size_t)y * g.bpitch + x] = raw[g.blur_off + blur_tile_off(x, y, g.bpitch)];
            off = ((off + (size_t)g.bpitch * g.h) + 255) & ~(size_t)255;
        }
        rm.resize(off);
        if (size_out) *size_out = rm.size();
        if (host && bytes) memcpy(host, rm.data(), std::min(bytes, rm.size()));
        return COEB_OK;
    }
    else if (w == "cand_n") { src = (const uint8_t*)c->bufs["cand_n"].p + (size_t)f * P.ncells * 4; n = (size_t)P.ncells * 4; }
    else if (w == "lvl_n") { src = (const uint8_t*)c->bufs["lvl_n"].p + (size_t)f * P.L * 4; n = (size_t)P.L * 4; }
    else if (w == "lvl_kp") { src = (const uint8_t*)c->bufs["lvl_kp"].p + (size_t)f * P.lvl_stride * 4; n = (size_t)P.lvl_stride * 4; }
    else if (w == "dyn") { src = (const uint8_t*)c->bufs["dyn"].p + (size_t)f * sizeof(DynMask); n = sizeof(DynMask); }
    else if (w == "plan") { if (size_out) *size_out = sizeof(Plan); if (host) memcpy(host, &P, std::min(bytes, sizeof(Plan))); return COEB_OK; }
    else return COEB_EINVAL;
    if (size_out) *size_out = n;
    if (host && bytes) {
        HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
        HIP_TRY(c, hipMemcpy(host, src, std::min(bytes, n), hipMemcpyDeviceToHost));
    }
    return COEB_OK;
}

int coeb_synchronize(coeb_ctx* c)
{
    if (!c) return COEB_EINVAL;
    (void)hipSetDevice(c->device);
    join_pose(c);
    HIP_TRY(c, hipStreamSynchronize(main_stream(c)));
    return check_err_word(c);
}

}  // extern "C"
