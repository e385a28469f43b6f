/*
 * orb_oracle.h -- CPU restatement of COEB-SLAM's per-frame ORB front end.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product (coeb-slam_amd/, libcoeb_front.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned" against the original reference binary.  The reference
 * (src/ORBextractor.cc, src/ORBmatcher.cc, src/Frame.cc) needs OpenCV 3.4, which is absent
 * from this image, and it ships no tests or golden vectors.  This
 * restatement is pinned by the reference's own tables (bit_pattern_31_, umax, level sizes,
 * features per level, DescriptorDistance) and restates the OpenCV 3.4 primitives with the
 * canonical definitions documented in DESIGN.md s3 (resize, FAST, GaussianBlur, fastAtan2,
 * sincosf, Laplacian, cvtColor).
 *
 * Every function cites the reference file:line it follows.
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OC_MAX_LEVELS 16

/* layout-identical to cv::KeyPoint (28 B) */
typedef struct { float x, y, size, angle, response; int32_t octave, class_id; } oc_kp;
typedef struct { float xmin, ymin, xmax, ymax; } oc_box;

/* ORBextractor::ORBextractor tables (src/ORBextractor.cc:418-477) */
typedef struct {
    int nfeatures;
    double scale_factor;           /* `double scaleFactor` member (ORBextractor.h:114) */
    int nlevels;
    int ini_th, min_th;            /* overridden to 20/7 or 30/10 (ORBextractor.cc:775-784) */
    float scale[OC_MAX_LEVELS], inv_scale[OC_MAX_LEVELS];
    float sigma2[OC_MAX_LEVELS], inv_sigma2[OC_MAX_LEVELS];
    int nfeat[OC_MAX_LEVELS];
    int umax[16];
    int pattern[512][2];
} oc_params;

int oc_init(oc_params* p, int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th);
void oc_level_size(const oc_params* p, int w, int h, int level, int* lw, int* lh);

/* cv::resize INTER_LINEAR 8U (canonical) used by ComputePyramid :1356 */
/* first column of VResizeLinear's scalar tail for a row of `width` outputs (OpenCV 3.4 SSE2) */
int oc_resize_simd_end(int width);
void oc_resize_linear(const uint8_t* src, int sw, int sh, int sstride,
                      uint8_t* dst, int dw, int dh, int dstride);
/* ComputePyramid (src/ORBextractor.cc:1344-1367); levels packed, level l stride = lw */
int oc_pyramid(const oc_params* p, const uint8_t* gray, int w, int h, int stride,
               uint8_t* out, int64_t* level_off);

/* cv::FAST(roi, kps, th, nonmax=true) on an ROI (OpenCV FAST_t<16>); xs/ys/score out */
int oc_fast_roi(const uint8_t* img, int stride, int rows, int cols, int threshold,
                int* xs, int* ys, int* score, int cap);
/* FAST stage of ComputeKeyPointsOctTree (src/ORBextractor.cc:786-850) for one level:
 * candidates relative to (16,16), canonical order. */
int oc_level_candidates(const uint8_t* lvl, int lw, int lh, int stride, int ini_th, int min_th,
                        int* xs, int* ys, int* score, int cap);
/* DistributeOctTree (src/ORBextractor.cc:546-769), pointer tie-break = allocation order */
int oc_distribute_octree(const int* xs, const int* ys, const int* score, int n,
                         int minX, int maxX, int minY, int maxY, int N,
                         int* out_idx, int cap);

int oc_ic_angle_moments(const uint8_t* img, int stride, int x, int y, const int* umax,
                        int* m01, int* m10);
float oc_fast_atan2(float y, float x);
void oc_sincos(float a, float* s, float* c);
void oc_gauss_kernel7(int k[7]);
void oc_gaussian_blur7(const uint8_t* src, int w, int h, int sstride, uint8_t* dst, int dstride);
void oc_orb_descriptor(const uint8_t* blurred, int stride, int x, int y, float angle,
                       const int (*pattern)[2], uint8_t desc[32]);

/* mask layers of operator() (src/ORBextractor.cc:1101-1195); mask is w x h */
int oc_dynamic_mask(const oc_box* boxes, int nbox, const float* tm_xy, int ntm,
                    const int32_t* blur_flag, int nblur, int w, int h,
                    uint8_t* mask, float* area_out);

typedef struct {
    uint8_t* pyramid;              /* optional: packed levels (oc_pyramid layout) */
    int64_t level_off[OC_MAX_LEVELS + 1];
    int ncand[OC_MAX_LEVELS];      /* FAST candidates per level (before any cull) */
    int nkept[OC_MAX_LEVELS];      /* keypoints per level in the output */
    int area_flag;
} oc_debug;

/* ORBextractor::operator() (src/ORBextractor.cc:1088-1342), debug imshow block excluded */
int oc_extract(const oc_params* p, const uint8_t* gray, int w, int h, int stride,
               const oc_box* boxes, int nbox, const float* tm_xy, int ntm,
               const int32_t* blur_flag, int nblur,
               oc_kp* kp_out, uint8_t* desc_out, int cap, int* n_out, oc_debug* dbg);

/* Frame blur flag (src/Frame.cc:171-202, 905-913) */
int oc_blur_flags(const uint8_t* gray, int w, int h, int stride,
                  const oc_box* boxes, int nbox, int32_t* out, double* mean_out);
/* Tracking::GrabImageRGBD cvtColor RGB->GRAY 8U (src/Tracking.cc:212-225) */
void oc_rgb2gray(const uint8_t* rgb, int w, int h, int stride, int rgb_order, uint8_t* out);
/* Tracking::GrabImageRGBD image and depth conversions (Tracking.cc:212-228); channels 1/3/4,
   depth_type 0 = 16UC1, 1 = 32FC1 (stride in bytes). */
void oc_image_to_gray(const uint8_t* img, int w, int h, int stride, int channels, int rgb_order, uint8_t* out);
void oc_depth_to_float(const void* depth, int w, int h, size_t stride, int depth_type, float factor, float* out);

/* ---- matcher side ---- */
typedef struct {
    float fx, fy, cx, cy, bf, mb;
    float min_x, max_x, min_y, max_y;
    float grid_inv_w, grid_inv_h;
    float scale[OC_MAX_LEVELS];
    int nlevels;
} oc_camera;
void oc_camera_init(oc_camera* c, float fx, float fy, float cx, float cy, float bf,
                    int w, int h, const oc_params* p);

/* Frame::ComputeStereoFromRGBD (src/Frame.cc:820-842) */
void oc_stereo_from_rgbd(const oc_kp* kps, int n, const float* depth, int w, int dstride,
                         float bf, float* uright, float* dep);

#define OC_GRID_COLS 64
#define OC_GRID_ROWS 48
typedef struct {
    int* cell_start;   /* [GRID_COLS*GRID_ROWS+1], cell index ix*GRID_ROWS+iy */
    int* cell_idx;     /* [n] keypoint indices in insertion order */
} oc_grid;
/* Frame::AssignFeaturesToGrid / PosInGrid (src/Frame.cc:396-411, 558-568) */
void oc_assign_grid(const oc_camera* c, const oc_kp* kps, int n, oc_grid* g);
/* Frame::GetFeaturesInArea (src/Frame.cc:503-556) */
int oc_features_in_area(const oc_camera* c, const oc_kp* kps, const oc_grid* g,
                        float x, float y, float r, int minLevel, int maxLevel,
                        int* out, int cap);

int oc_descriptor_distance(const uint8_t* a, const uint8_t* b);  /* ORBmatcher.cc:1648 */

typedef struct {
    int n;
    const uint8_t* has_mp; const uint8_t* outlier;
    const float* xw; const uint8_t* mp_desc; const int32_t* mp_nobs;
    const oc_kp* keys_un;
} oc_lastframe;
typedef struct {
    int n; const oc_kp* keys_un; const uint8_t* desc; const float* uright;
} oc_curframe;

/* ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) (ORBmatcher.cc:1329-1471)
 * match_out[i2] = index of the LastFrame slot whose MapPoint was assigned, or -1 */
int oc_search_by_projection(const oc_camera* cam, const oc_curframe* cur, const oc_lastframe* last,
                            const float Tcw_cur[16], const float Tcw_last[16],
                            float th, int bMono, int check_ori, int32_t* match_out);

/* Local-map points as Frame::isInFrustum left them (Frame.cc:463-501): the inputs of
 * ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th) */
typedef struct {
    int n;
    const uint8_t* in_view;        /* mbTrackInView && !isBad() */
    const float* proj_x;           /* mTrackProjX */
    const float* proj_y;           /* mTrackProjY */
    const float* proj_xr;          /* mTrackProjXR */
    const int32_t* level;          /* mnTrackScaleLevel */
    const float* view_cos;         /* mTrackViewCos */
    const uint8_t* desc;           /* GetDescriptor(), n x 32 */
    const int32_t* nobs;           /* Observations() */
} oc_localmap;

/* ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th) (ORBmatcher.cc:44-129)
 * with RadiusByViewingCos (:131-137).  cur_obs[i2] = Observations() of the MapPoint already in
 * CurrentFrame.mvpMapPoints[i2] at entry (< 0: none).  match_out[i2] = index of the local-map
 * point assigned to keypoint i2 by this call (the last one), or -1 (entry unchanged). */
int oc_search_local_map(const oc_camera* cam, const oc_curframe* cur, const int32_t* cur_obs,
                        const oc_localmap* mp, float th, float nnratio, int32_t* match_out);

/* Map points of a KeyFrame for the relocalisation search: pKF->GetMapPointMatches() snapshot
 * (ORBmatcher.cc:1487-1530 reads exactly these). */
typedef struct {
    int n;
    const uint8_t* valid;          /* pMP && !pMP->isBad() && !sAlreadyFound.count(pMP) */
    const float* xw;               /* n x 3 GetWorldPos() */
    const uint8_t* desc;           /* n x 32 GetDescriptor() */
    const float* max_dist;         /* mfMaxDistance */
    const float* min_dist;         /* mfMinDistance */
    const float* angle;            /* pKF->mvKeysUn[i].angle */
} oc_kfpoints;

/* ORBmatcher::SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)
 * (ORBmatcher.cc:1473-1560) with MapPoint::PredictScale (MapPoint.cc:402-417).
 * cur_has[i2] = CurrentFrame.mvpMapPoints[i2] != NULL at entry.  match_out[i2] = index of the
 * KeyFrame point assigned to keypoint i2 by this call, or -1. */
int oc_search_keyframe(const oc_camera* cam, const oc_curframe* cur, const uint8_t* cur_has,
                       const oc_kfpoints* kf, const float Tcw[16], float th, int orb_dist, int check_ori,
                       int32_t* match_out);

/* ---- Tracking::TrackLocalMap's local map in the batch chain ----
 * A MapPoint observed by one KeyFrame with camera centre Ow, from a keypoint of that octave
 * (MapPoint::UpdateNormalAndDepth with one observation, MapPoint.cc:330-371). */
void oc_mappoint_normal_depth(const oc_camera* cam, const float P[3], const float Ow[3], int octave,
                              float normal[3], float* max_dist, float* min_dist);
/* Frame::isInFrustum(pMP, viewingCosLimit) (Frame.cc:445-501) with MapPoint::PredictScale
 * (MapPoint.cc:402-417): returns mbTrackInView and, when 1, the mTrack* fields. */
int oc_is_in_frustum(const oc_camera* cam, const float Tcw[16], const float P[3], const float Pn[3],
                     float max_dist, float min_dist, float cos_limit,
                     float* proj_x, float* proj_y, float* proj_xr, int32_t* level, float* view_cos);
/* A KeyFrame's keypoint slots as the local map reads them */
typedef struct {
    int n;
    const oc_kp* keys;             /* octave of each slot */
    const uint8_t* has;            /* depth > 0: the slot holds a MapPoint */
    const float* xw;               /* n x 3, UnprojectStereo in the KeyFrame's own camera frame */
} oc_kfview;
/* Local map of the current frame f: slots [0, stride) = KF2 (frame f-2, may be NULL), whose
 * points are placed in KF1's frame by T_kf1_kf2 (KF1's pose with KF2 as world), slots
 * [stride, 2 stride) = KF1 (frame f-1, the world frame).  seen1[j]: KF1 slot j was matched by
 * the motion-model search (mnLastFrameSeen == current, Tracking.cc:979,1237,1249).  Every point
 * gets Observations() = nobs and goes through isInFrustum(cos_limit) with Tcw_cur; writes the
 * coeb_localmap arrays (2 stride entries) and each point's world position; returns #in view. */
int oc_local_map_build(const oc_camera* cam, const oc_kfview* kf2, const float T_kf1_kf2[16], const oc_kfview* kf1,
                       const uint8_t* seen1, int32_t nobs, int stride, const float Tcw_cur[16], float cos_limit,
                       uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr, int32_t* level,
                       float* view_cos, int32_t* nobs_out, float* xw_out);

/* Optimizer::PoseOptimization(Frame*) (Optimizer.cc:239-451): the frame's matched keypoints
 * and their map points.  fx..bf are the Frame's intrinsics. */
typedef struct {
    int n;
    const uint8_t* has_mp;         /* mvpMapPoints[i] != NULL */
    const float* xw;               /* n x 3 GetWorldPos() */
    const oc_kp* keys_un;          /* mvKeysUn (pt, octave) */
    const float* uright;           /* mvuRight (< 0: monocular edge) */
    const float* inv_sigma2;       /* mvInvLevelSigma2 */
    float fx, fy, cx, cy, bf;
} oc_pose_frame;

/* Returns nInitialCorrespondences - nBad (0 with < 3 correspondences, pose untouched);
 * Tcw (row-major 4x4) is replaced by the optimised pose; outlier[i] = mvbOutlier[i]
 * (written only where has_mp[i]).  Canonical restatement of g2o's Levenberg-Marquardt
 * (OptimizationAlgorithmLevenberg, 2012 release vendored by ORB-SLAM2) with the per-edge
 * sums reduced over 256 lanes in a fixed tree: parity vs g2o UNPINNED. */
int oc_pose_optimization(const oc_pose_frame* fr, float Tcw[16], uint8_t* outlier);
/* LM iterations and trials the last oc_pose_optimization call on this thread ran (test hook). */
void oc_pose_last_stats(int* iterations, int* trials);

/* Frame::UndistortKeyPoints (Frame.cc:579-609): cv::undistortPoints(mat, mat, mK, mDistCoef,
 * Mat(), mK) of OpenCV 3.4 (cvUndistortPointsInternal, 5 fixed iterations) in double,
 * dist = (k1, k2, p1, p2, k3); k1 == 0 copies the keypoints (:581-585). */
void oc_undistort_keypoints(const oc_kp* in, int n, float fx, float fy, float cx, float cy, const float dist[5],
                            oc_kp* out);

/* cv::goodFeaturesToTrack(img, corners, maxCorners, qualityLevel, minDistance, Mat(), 3, true, k)
 * as Frame::ProcessMovingObject calls it (Frame.cc:333): OpenCV 3.4 featureselect.cpp with
 * cornerHarris (corner.cpp, blockSize 3, Sobel 3x3, BORDER_REFLECT_101) in the canonical forms
 * of DESIGN.md s2.1.  Writes up to cap (x, y) pairs; returns the corner count, or -1 when more
 * than max_cand local maxima pass the quality threshold. */
int oc_good_features_harris(const uint8_t* img, int w, int h, int stride, int max_corners, double quality,
                            double min_distance, double k, float* out_xy, int cap, int max_cand);


/* ---- the rest of Frame::ProcessMovingObject (Frame.cc:334-384), DESIGN.md s4.10 ---- */
void oc_rect_subpix_8u32f(const uint8_t* img, int w, int h, int stride, int ww, int wh, float cx, float cy,
                          float* dst);
void oc_subpix_mask(int win, float* mask);
void oc_corner_subpix(const uint8_t* img, int w, int h, int stride, float* xy, int n, int win, int max_iter,
                      double eps);
void oc_pyr_down(const uint8_t* src, int sw, int sh, uint8_t* dst);
int oc_lk_levels(int w, int h, int win, int max_level);
int oc_lk_pyr(const uint8_t* prev, const uint8_t* next, int w, int h, int stride, const float* pxy, int n, int win,
              int max_level, int max_count, double eps, float* nxy, uint8_t* status);
double oc_fd_acos(double x);
double oc_fd_log(double x);
double oc_fd_exp(double x);
double oc_fd_cos(double x);
int oc_solve_cubic(const double c[4], double r[3]);
int oc_run7point(const float* m1, const float* m2, double* F);
int oc_ransac_update_iters(double p, double ep, int max_iters);
int oc_find_fundamental(const float* m1, const float* m2, int n, double thr, double conf, double F[9]);
int oc_moving_tail(const uint8_t* prev, const uint8_t* cur, int w, int h, int stride, const float* pxy,
                   const float* nxy, uint8_t* state, int n, int edge, double limit, float* tm_xy, int tm_cap,
                   double F_out[9], int* nf_out);
int oc_process_moving_object(const uint8_t* prev, const uint8_t* cur, int w, int h, int stride, float* tm_xy,
                             int tm_cap, int* ncorners_out);

#ifdef __cplusplus
}
#endif
#endif
