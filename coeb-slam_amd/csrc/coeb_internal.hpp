// coeb_internal.hpp -- shared host/device definitions of the MI355X ORB front end.
//
// HBM layout (per frame slot f of a context, all packed, byte offsets 256-aligned):
//   gray      [f][H][W]                 u8   level 0 (caller's device buffer or ctx staging)
//   pyr       [f][pyr_stride]           u8   levels 1..L-1, level l at pyr_off[l], row stride W_l
//   blur      [f][blur_stride]          u8   7x7 Gaussian of levels 0..L-1 (descriptor input), each
//                                            level in 16 x 8 tiles (blur_tile_off; rows padded to 8)
//   cand_n    [f][ncells]               i32  FAST corners kept per cell
//   cand      [f][ncells][cell_cap]     u32  packed (x_rel | y_rel<<12 | score<<24), row-major
//   keys      [f][2][kbuf_stride]       u32  octree key ping-pong buffers (per level kcap_off)
//   nodes     [f][L][2][NCAP] records        octree node scratch (start,cnt,rect,alloc)
//   lvl_n     [f][L]                    i32  keypoints per level after culls
//   lvl_kp    [f][lvl_stride]           u32  packed level keypoints in output order
//   kps       [f][kcap]                 28B  coeb_keypoint (== cv::KeyPoint)
//   desc      [f][kcap][32]             u8
//   dyn       [f]                       DynMask (area flag + zeroed rectangles)
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include <mutex>
#include <set>
#include <utility>

// Runtime switches, the only environment reads of the library (coeb_capi.hip):
//  * coeb_switch(name): a product switch -- one of kSwitches, each run by the GPU test suite
//    against the oracle (side-stream modes, the matcher's sequential / split forms, the
//    pyramid's byte form, the general FAST slab layout, k_fm's threads per pair);
//  * coeb_experiment(name): a measurement-only switch (schedules and kernel forms measured and
//    not kept, diagnostic clocks), read only when COEB_EXPERIMENTS=1, so a stray variable in a
//    caller's environment cannot route the shipped library through an untested path.
// Both return the value or nullptr.
const char* coeb_switch(const char* name);
const char* coeb_experiment(const char* name);

#ifndef COEB_MATCH_CLOCK
#define COEB_MATCH_CLOCK 0     // experiment builds: k_match phase clocks (COEB_MATCH_TIMING, tools/_match_timing.py)
#endif

// Raise a kernel's dynamic-LDS limit once per (kernel, device), to the most any launch may use
// (the CU's 160 KB; the launch's own size still sets the occupancy).  The attribute is
// process-wide: setting it per launch to that launch's size let another host thread's launch of
// the same kernel with a larger size run under a smaller limit set in between.
constexpr int kLdsLimit = 160 * 1024;
inline void lds_limit_max(const void* kern)
{
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    if (!done.insert({kern, dev}).second) return;
    // the device's per-workgroup maximum less the kernel's static LDS
    int lim = kLdsLimit, v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess && v > 0)
        lim = v < lim ? v : lim;
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, kern) == hipSuccess) lim -= (int)fa.sharedSizeBytes;
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, lim) != hipSuccess)
        (void)hipGetLastError();        // not sticky: the launch itself reports a size it cannot take
}

// Byte (x, y) of a blurred level with row pitch bpitch (a 64-byte multiple): the level is stored
// in 128-byte tiles of 16 columns x 8 rows, one tile per cache line, tiles row-major (bpitch / 16
// per tile row).  k_describe reads 37-row x 64-byte patches: row-major, every patch row would be its
// own line (37-74 line lookups per patch, half of each 128-B line unused); tiled, a patch is
// 4 x 5-6 whole lines.
__host__ __device__ inline int64_t blur_tile_off(int x, int y, int bpitch)
{
    return ((int64_t)(y >> 3) * (bpitch >> 4) + (x >> 4)) * 128 + (y & 7) * 16 + (x & 15);
}

#define COEB_MAXL 16
#define COEB_MAXBOX 16
#define COEB_GRID_COLS 64
#define COEB_GRID_ROWS 48
#define COEB_GRID_CELLS (COEB_GRID_COLS * COEB_GRID_ROWS)

// Per-level geometry and offsets, computed on the host once per (W, H) and copied to the
// device as one POD block (kernel argument).
struct LevelGeom {
    int w, h;
    int pitch;             // row pitch of the level image (level 0: W; levels >= 1: 64-byte multiple)
    int bpitch;            // row pitch of the blurred level (64-byte multiple)
    int64_t pyr_off;       // into pyr frame block (-1 for level 0)
    int64_t blur_off;      // into blur frame block
    int rtab_off;          // into resize table (ints): xofs[w], alpha[w], yofs[h], beta[h]
    int xmax;              // resize: columns >= xmax use S[sx]*2048
    int rows_ok;           // k_pyr_rows applies: every even column pair's sources within 6 bytes of
                           // the pair's 4-byte aligned window start (scale <= 2)
    int yrow_off;          // into resize table (ints): per output row {r0 * sp, r1 * sp, beta, dy * pitch}
                           // (the clamped source rows' byte offsets; sp = the source level's pitch)
    int ncols, nrows, wcell, hcell;
    int cell0, ncells;     // range in the cell table (row-major over non-skipped cells)
    int kcap_off, kcap;    // octree key buffers: offset / capacity (u32 entries)
    int nfeat, nfeat_area; // DistributeOctTree N: mnFeaturesPerLevel[l], (int)(N*0.7)
    int nini;              // initial octree nodes
    float hx;              // (maxX-minX)/nIni
    int ini_bound[5];      // initial node i holds x_rel in [ini_bound[i], ini_bound[i+1])
    int ncap;              // node record capacity per set
    int64_t node_off;      // into node scratch (records) per frame
    int out_cap, out_off;  // level keypoint capacity / offset into lvl_kp frame block
    float scale;           // mvScaleFactor[l]
    int size_i;            // (int)(PATCH_SIZE * scale)
    int maxX, maxY;        // octree box: maxBorderX - minBorderX, maxBorderY - minBorderY
};

struct Plan {
    int W, H, L;
    LevelGeom lv[COEB_MAXL];
    int ncells;            // all levels
    int cell_cap;          // u32 entries per cell slot
    int max_roi_w, max_roi_h;
    int64_t pyr_stride, blur_stride;
    int64_t kbuf_stride;   // u32 entries per key buffer (x2 per frame)
    int64_t node_stride;   // node records per frame (all levels, both sets)
    int lvl_stride;        // u32 entries per frame in lvl_kp
    int kcap;              // output keypoints per frame (sum of out_cap)
    int rtab_ints;
    int umax[16];
    int gauss[7];
    int oct_w;             // k_octree: node records per set / work-list entries (max ncap)
    int oct_kl;            // k_octree: keys kept in LDS when a level has <= oct_kl candidates
    int oct_lds;           // k_octree dynamic LDS bytes
};

// FAST cell descriptor (ORBextractor.cc:811-829): ROI in level coordinates
struct CellDesc {
    int16_t level, pad;
    int16_t x0, y0;        // iniX, iniY
    int16_t rw, rh;        // maxX-iniX, maxY-iniY (ROI; detection window = inset 3)
    int16_t i, j;          // cell row / column (for x_rel/y_rel offsets)
};

// Dynamic-object mask of one frame (ORBextractor.cc:1101-1195): the mask is the complement of
// the union of these rectangles (x in [x0,x1), y in [y0,y1)), so the W x H byte mask never
// needs to be materialised.
struct DynMask {
    int area_flag;
    int nrect;
    int rect[COEB_MAXBOX][4];
};

struct NodeSet {           // SoA node records (one set of a level)
    int* start;
    int* cnt;
    int4* rect;            // x0, y0, x1, y1 (relative coordinates)
    int* alloc;
    int* buf;
};

static inline __host__ __device__ uint32_t pack_key(int x, int y, int s)
{
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)s << 24);
}
static inline __host__ __device__ int key_x(uint32_t k) { return (int)(k & 0xFFFu); }
static inline __host__ __device__ int key_y(uint32_t k) { return (int)((k >> 12) & 0xFFFu); }
static inline __host__ __device__ int key_s(uint32_t k) { return (int)(k >> 24); }

// ---- launch wrappers (coeb_extract.hip / coeb_match.hip) ----
int oct_timing_read(long long* out);   // COEB_OCT_CLOCK builds: [4096][6] per-workgroup k_octree clocks
int fast_timing_read(unsigned long long* out);   // COEB_FAST_CLOCK builds: per-cell k_fast phase sums
struct ExtractBufs {
    const uint8_t* gray;   // [F][H][W]
    uint8_t* pyr;
    uint8_t* blur;
    int* cand_n;
    uint32_t* cand;
    uint32_t* keys;
    uint8_t* nodes;        // raw node scratch
    int* lvl_n;
    uint32_t* lvl_kp;
    void* kps;             // coeb_keypoint
    uint8_t* desc;
    int* counts;
    DynMask* dyn;
    const int* rtab;
    const CellDesc* cells;
    const int8_t* pattern; // 512 x (x, y)
    // dynamic-mask inputs
    const float* boxes;    // [nbox_total][4]
    const int* box_off;    // [F+1]
    const float* tm;       // [ntm_total][2]
    const int* tm_off;     // [F+1]
    const int* blurf;      // [nbox_total]
    // T_M computed on the device (coeb_frame_batch_device): frame f's points at
    // tmd + f * tmd_cap * 2, count ntmd[f] (-1: none); used instead of tm / tm_off when set
    const float* tmd;
    const int* ntmd;
    int tmd_cap;
    int* err;              // device error word (capacity overflows)
};

struct ProfileHook {
    void* impl = nullptr;   // owned by the context (coeb_capi.hip)
};
void prof_begin(ProfileHook* p, const char* name, hipStream_t s);
void prof_end(ProfileHook* p, hipStream_t s);

// side (optional): blur + FAST of level 0 run on side.s while the pyramid builds levels 1..;
// those of levels 1..split-1 follow there once the pyramid has built them, and s does levels
// split..L-1 after the pyramid; s joins side.s before the octree.
// With blur_late, the blur of levels split..L-1 also runs on side.s (after the pyramid, beside
// FAST and the octree on s); s then joins it (join2) only before the descriptors.
// With side_octree, the octree of levels < split follows their FAST on side.s.
struct SideStream { hipStream_t s; hipEvent_t fork, mid, join, pyr_done, join2; int split; bool blur_late, side_octree; };
int launch_extract(const Plan& plan, const Plan* d_plan, const ExtractBufs& b, int F, hipStream_t s,
                   ProfileHook* prof, const SideStream* side = nullptr);

struct MatchCam {
    float fx, fy, cx, cy, bf, mb;
    float min_x, max_x, min_y, max_y;
    float grid_inv_w, grid_inv_h;
    float scale[COEB_MAXL];
    int nlevels;       // mnScaleLevels
    float log_sf;      // mfLogScaleFactor = log(mfScaleFactor) (Frame.cc:85), correctly rounded
};
struct MatchBufs {
    // current frames
    const void* cur_kps;       // coeb_keypoint [P][cur_stride]
    const uint8_t* cur_desc;   // [P][cur_stride][32]
    const int* cur_n;          // [P]
    const float* cur_ur;       // [P][cur_stride] (may be computed by prep)
    int cur_stride;
    // last frames
    const void* last_kps;      // coeb_keypoint [P][last_stride]
    const uint8_t* last_desc;  // [P][last_stride][32] MapPoint descriptors
    const int* last_n;         // [P]
    const uint8_t* last_has;   // [P][last_stride]
    const uint8_t* last_out;   // [P][last_stride]
    const float* last_xw;      // [P][last_stride][3]
    const int* last_nobs;      // [P][last_stride]
    int last_stride;
    const float* Tcw_cur;      // [P][16]
    const float* Tcw_last;     // [P][16]
    int* match;                // [P][cur_stride]
    int* nmatch;               // [P]
    int* scratch;              // [P][scratch_stride]
    int scratch_stride;
    int* qn;                   // optional [P][qn_stride >= last_stride + 8]: split-list counts + flags
    int qn_stride;
    long long* timing;         // optional [P][16] phase clocks (COEB_MATCH_TIMING), else nullptr
    int* err;
};
int launch_match(const MatchCam& cam, const MatchBufs& b, int P, float th, int bmono, int check_ori,
                 int retry_below, hipStream_t s, ProfileHook* prof);

// local-map projection search (ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th))
struct LocalBufsHost {
    const void* cur_kps; const uint8_t* cur_desc; const float* cur_ur; const int* cur_obs; int cur_n;
    const uint8_t* in_view; const float* proj_x; const float* proj_y; const float* proj_xr;
    const int* level; const float* view_cos; const uint8_t* desc; const int* nobs; int mp_n;
    int* match; int* nmatch; uint32_t* lists; int* err;
    int* path;   // [0]: 0 parallel claims, 1 forced sequential, 2 list overflow, 3 no convergence; [1]: iterations
    // batch form: npairs workgroups, pair p reads cur_* + p*cur_stride (keypoint count
    // cur_n_arr[p]), the local-map arrays + p*mp_n, desc + p*mp_desc_stride*32, lists + p*mp_n*kCQ,
    // and writes match + p*cur_stride, nmatch[p], path[2p..]; active[p] == 0 skips the pair
    // (no matches).  cur_n_arr == null: the single search above.
    const int* cur_n_arr = nullptr; const uint8_t* active = nullptr;
    int npairs = 1, cur_stride = 0, mp_desc_stride = 0;
};
int launch_match_local(const MatchCam& cam, const LocalBufsHost& b, float th, float nnratio, hipStream_t s,
                       ProfileHook* prof);
int match_list_cap();   // candidate-list entries per query (kCQ)

// Optimizer::PoseOptimization (coeb_pose.hip): per frame f, keypoints [f][stride]
struct PoseEdgeRec { float x, y, z, u, v, ur, w; int stereo, kp; };
struct PoseBufs {
    const int* n;                 // [F] keypoints
    const uint8_t* has_mp;        // [F][stride]
    const float* xw;              // [F][stride][3]
    const void* kps;              // [F][stride] coeb_keypoint
    const float* ur;              // [F][stride]
    const float* inv_sigma2;      // [COEB_MAXL] mvInvLevelSigma2
    float* Tcw;                   // [F][16] in/out
    uint8_t* outlier;             // [F][stride] out (mvbOutlier, where has_mp)
    int* result;                  // [F] nInitialCorrespondences - nBad
    PoseEdgeRec* edges;           // scratch [F][stride]
    uint8_t* active;              // scratch [F][stride]
    double* chi2;                 // scratch [F][stride]
    int stride;
    long long* timing;            // optional [F][8] phase clocks (COEB_POSE_TIMING), else null
};
int launch_pose(const PoseBufs& b, int F, double fx, double fy, double cx, double cy, double bf, hipStream_t s,
                ProfileHook* prof);

// TrackWithMotionModel tail on a device batch (coeb_pose.hip): pair p = (frame p, frame p+1).
// All arrays are indexed from frame 0 ([F][stride]); frame 0 (the halo) is never written.
struct TrackPrepBufs {
    const int32_t* match;         // [F][stride] LastFrame index per current keypoint, or -1
    const int32_t* nmatch;        // [F] SearchByProjection result (after the 2*th retry)
    const int32_t* counts;        // [F] keypoints
    const float* last_xw;         // [F][stride][3] LastFrame MapPoint positions (k_prep)
    const void* kps_in;           // [F][stride] coeb_keypoint (batch output) -> kps_out
    const float* ur_in;           // [F][stride] mvuRight (k_prep) -> ur_out
    void* kps_out;
    float* ur_out;
    const float* Tin;             // [F][16] motion-model prediction
    float* Tout;                  // [F][16] <- Tin, then PoseOptimization's result
    uint8_t* has;                 // [F][stride] CurrentFrame.mvpMapPoints[i] != NULL
    float* xw;                    // [F][stride][3] position of that MapPoint
    int32_t* n;                   // [F] keypoints handed to the optimiser (0: not tracked)
    float* isg_out;               // [COEB_MAXL] device copy of isg
    float isg[COEB_MAXL];         // mvInvLevelSigma2
    int stride, min_matches;
};
int launch_track_prep(const TrackPrepBufs& t, int F, hipStream_t s, ProfileHook* prof);

// Tracking::TrackLocalMap on a device batch (coeb_track.hip), after the TrackWithMotionModel
// tail: current frame f = 1..F-1, KF1 = frame f-1 (the world frame of pair f), KF2 = frame f-2.
// Every [F][K] array is indexed from frame 0; the local map of frame f is [f][2K]: slots [0, K)
// = KF2's keypoint slots, [K, 2K) = KF1's.
struct TlmBufs {
    int K, nkf, nobs, min_matches, min_map;
    // batch outputs of the extraction / matcher (main stream), read by k_tlm_snapshot only
    const void* kps; const uint8_t* desc; const int* counts; const int* match1; const int* nmatch1;
    const uint8_t* has; const float* xw;
    // snapshot (main stream): s_desc holds frame g at row g + 1 (row 0: KF2 of frame 1, never read)
    uint8_t* s_desc; int8_t* s_oct; uint8_t* s_has; float* s_xw; int* s_m1; int* s_cnt; int* s_nm1;
    // TrackWithMotionModel's PoseOptimization (t_* of coeb_pose_batch_device)
    const float* T1; const uint8_t* has1; const uint8_t* outl1; const float* xw1;
    // discard + SearchLocalPoints state
    uint8_t* seen;       // [F][K] KF1 slot matched by the motion model (mnLastFrameSeen)
    int* cur_obs;        // [F][K] Observations() of the MapPoint a keypoint keeps, -1: none
    int* nmap;           // [F] nmatchesMap (Tracking.cc:967-985)
    uint8_t* active;     // [F] TrackWithMotionModel returned true -> TrackLocalMap runs
    uint8_t* in_view; float* px; float* py; float* pxr; int* level; float* vcos; int* lm_nobs; float* lm_xw;
    const int* lmatch;   // [F][K] SearchByProjection(F, vpLocalMapPoints) assignments
    // second PoseOptimization's inputs
    uint8_t* has2; float* xw2; float* T2; uint8_t* outl2; int* n2;
};
int launch_tlm_snapshot(const TlmBufs& t, int F, hipStream_t s, ProfileHook* prof);
int launch_tlm_frustum(const MatchCam& cam, const TlmBufs& t, int F, hipStream_t s, ProfileHook* prof);
int launch_tlm_pose_prep(const TlmBufs& t, int F, hipStream_t s, ProfileHook* prof);

// relocalisation projection search (ORBmatcher::SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist))
struct KfBufsHost {
    const void* cur_kps; const uint8_t* cur_desc; const uint8_t* cur_has; int cur_n;
    const uint8_t* valid; const float* xw; const uint8_t* desc; const float* maxd; const float* mind;
    const float* angle; int kf_n;
    const float* Tcw;   // device, 16 floats row-major
    int* match; int* nmatch; uint32_t* lists; int* err;
    int* path;          // as LocalBufsHost::path
};
int launch_match_kf(const MatchCam& cam, const KfBufsHost& b, float th, int orb_dist, int check_ori, hipStream_t s,
                    ProfileHook* prof);

// frame preparation for batch matching: u_right/depth per keypoint + LastFrame map snapshot
struct PrepBufs {
    const void* kps; const int* n; int stride;
    const float* depth; int W, H;
    float bf, fx, fy, cx, cy;
    float* ur; float* dep;
    uint8_t* has; uint8_t* outl; float* xw; int* nobs; int nobs_value;
    const float* Twc;          // [F][16] inverse poses for UnprojectStereo (may be NULL = I)
};
int launch_prep(const PrepBufs& b, int F, hipStream_t s, ProfileHook* prof);
