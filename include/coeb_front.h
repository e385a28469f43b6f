/*
 * coeb_front.h -- C-ABI of the MI355X-native COEB-SLAM per-frame ORB front end.
 *
 * Plain C: pointers, sizes and POD structs only (no OpenCV, no torch types).  Every entry
 * point names the reference interface it replaces (paths are into biscuitzb/COEB-SLAM):
 *
 *   coeb_create / coeb_orb_tables   <- ORBextractor::ORBextractor(nfeatures, scaleFactor,
 *                                      nlevels, iniThFAST, minThFAST)  include/ORBextractor.h:50-51,
 *                                      src/ORBextractor.cc:418-477, accessors ORBextractor.h:77-99
 *   coeb_extract                    <- ORBextractor::operator()(image, mask, img, imD, keypoints,
 *                                      descriptors, box, T_M, mask_result, blur_flag)
 *                                      include/ORBextractor.h:73-75, src/ORBextractor.cc:1088-1342
 *   coeb_extract_batch_device       <- the same, for a device-resident batch of frames
 *   coeb_blur_flags                 <- Frame RGB-D ctor blur-flag loop + Frame::detect_laplacian
 *                                      src/Frame.cc:171-202, 905-913
 *   coeb_rgbd_preprocess            <- Tracking::GrabImageRGBD cvtColor / depth convertTo
 *                                      src/Tracking.cc:207-228
 *   coeb_undistort_keypoints        <- Frame::UndistortKeyPoints  src/Frame.cc:579-609
 *   coeb_boxes_from_int64           <- ImageGrabber::GrabRGBD box copy
 *                                      Examples/ROS/ORB-SLAM2/src/ros_rgbd.cc:106-115
 *   coeb_stereo_from_rgbd           <- Frame::ComputeStereoFromRGBD  src/Frame.cc:820-842
 *   coeb_match_lastframe            <- ORBmatcher::SearchByProjection(Frame&, const Frame&,
 *                                      const float th, const bool bMono)
 *                                      include/ORBmatcher.h:52, src/ORBmatcher.cc:1329-1471
 *                                      (with Frame::GetFeaturesInArea / AssignFeaturesToGrid,
 *                                      src/Frame.cc:396-411, 503-568)
 *   coeb_match_localmap             <- ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&,
 *                                      const float th)  include/ORBmatcher.h:46,
 *                                      src/ORBmatcher.cc:44-129 (RadiusByViewingCos :131-137),
 *                                      the call in Tracking::SearchLocalPoints  src/Tracking.cc:1222-1271
 *   coeb_match_keyframe             <- ORBmatcher::SearchByProjection(Frame&, KeyFrame*,
 *                                      const set<MapPoint*>&, const float th, const int ORBdist)
 *                                      include/ORBmatcher.h:55, src/ORBmatcher.cc:1473-1600
 *                                      (MapPoint::PredictScale  src/MapPoint.cc:402-417), the
 *                                      calls in Tracking::Relocalization  src/Tracking.cc:1531,1545
 *   coeb_pose_optimization          <- Optimizer::PoseOptimization(Frame*)  include/Optimizer.h:47,
 *                                      src/Optimizer.cc:239-451 (g2o LM; g2o itself is not vendored,
 *                                      parity UNPINNED); calls Tracking.cc:841,964,1006
 *   coeb_pose_batch_device          <- Tracking::TrackWithMotionModel after the projection search
 *                                      src/Tracking.cc:947-964 (mvpMapPoints from the matches,
 *                                      nmatches < 20 -> not tracked, PoseOptimization :964)
 *   coeb_good_features, coeb_corner_subpix, coeb_optical_flow_pyr_lk, coeb_moving_tail,
 *   coeb_moving_object_points[_device]  <- Frame::ProcessMovingObject  src/Frame.cc:311-393
 *                                      (OpenCV goodFeaturesToTrack / cornerSubPix / calcOpticalFlowPyrLK /
 *                                      findFundamentalMat as called there)
 *   coeb_descriptor_distance        <- ORBmatcher::DescriptorDistance  src/ORBmatcher.cc:1648-1664
 *   coeb_tum_read_list              <- associate.py read_file_list  associate.py:49-69
 *   coeb_tum_associate              <- associate.py associate  associate.py:71-102 (host only)
 *
 * Conventions: 0 on success, negative COEB_E* code on failure (the reference has no error
 * returns: it asserts or is UB).  The caller owns host buffers; the context
 * owns device buffers and streams.  One context per host thread; calls are not reentrant.
 */
#ifndef COEB_FRONT_H
#define COEB_FRONT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define COEB_OK 0
#define COEB_EINVAL (-22)    /* bad argument / shape outside the context limits */
#define COEB_ENOMEM (-12)    /* device allocation failed */
#define COEB_EDEVICE (-5)    /* HIP runtime error (see coeb_last_error) */
#define COEB_ERANGE (-34)    /* an internal capacity was exceeded (see coeb_last_error) */
#define COEB_ENODEV (-19)    /* no usable gfx950 device */

/* ABI revision of this header.  Bumped whenever an entry point's signature or a struct layout
 * changes (3: coeb_rgbd_preprocess gained channels/depth_type and a byte depth stride); the
 * adapters compare it with coeb_abi_version() of the loaded library and refuse a mismatch. */
#define COEB_ABI_VERSION 3
int coeb_abi_version(void);

#define COEB_MAX_LEVELS 16
#define COEB_MAX_BOXES 16

typedef struct coeb_ctx coeb_ctx;

/* ORBextractor ctor arguments.  iniThFAST/minThFAST are accepted but, as in the reference,
 * overridden per frame to 20/7 (30/10 when the dynamic area exceeds 200000 px)
 * (src/ORBextractor.cc:775-784). */
typedef struct {
    int32_t nfeatures;
    float scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
} coeb_orb_params;

/* layout-identical to cv::KeyPoint {Point2f pt; float size, angle, response; int octave, class_id;} */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} coeb_keypoint;

/* YOLO person box, xyxy, as std::vector<float>{xmin,ymin,xmax,ymax} (ros_rgbd.cc:106-115) */
typedef struct {
    float xmin, ymin, xmax, ymax;
} coeb_box;

/* ORBextractor accessors (include/ORBextractor.h:77-99) and derived per-level constants */
typedef struct {
    int32_t nlevels;
    float scale_factor;
    float scale[COEB_MAX_LEVELS];          /* GetScaleFactors() */
    float inv_scale[COEB_MAX_LEVELS];      /* GetInverseScaleFactors() */
    float sigma2[COEB_MAX_LEVELS];         /* GetScaleSigmaSquares() */
    float inv_sigma2[COEB_MAX_LEVELS];     /* GetInverseScaleSigmaSquares() */
    int32_t features_per_level[COEB_MAX_LEVELS];
    int32_t umax[16];
} coeb_orb_tables;

/* Camera + Frame constants used by the matcher (Frame.cc:231-246, ComputeImageBounds :611-641) */
typedef struct {
    float fx, fy, cx, cy;
    float bf;                   /* mbf */
    float min_x, max_x, min_y, max_y;
} coeb_camera;

/* Snapshot of the previous Frame taken by the caller (MapPoint accessors under their mutexes):
 * ORBmatcher.cc:1352-1396 reads exactly these. */
typedef struct {
    int32_t n;                        /* LastFrame.N */
    const uint8_t* has_mappoint;      /* LastFrame.mvpMapPoints[i] != NULL */
    const uint8_t* outlier;           /* LastFrame.mvbOutlier[i] */
    const float* world_pos;           /* n x 3, MapPoint::GetWorldPos() */
    const uint8_t* mp_descriptor;     /* n x 32, MapPoint::GetDescriptor() */
    const int32_t* mp_observations;   /* MapPoint::Observations() */
    const coeb_keypoint* keys_un;     /* LastFrame.mvKeysUn (octave, angle) */
} coeb_lastframe;

/* The current Frame (after ExtractORB + ComputeStereoFromRGBD) */
typedef struct {
    int32_t n;                        /* CurrentFrame.N */
    const coeb_keypoint* keys_un;     /* CurrentFrame.mvKeysUn */
    const uint8_t* descriptors;       /* n x 32 */
    const float* u_right;             /* CurrentFrame.mvuRight */
} coeb_curframe;

/* ---- context ---- */
coeb_ctx* coeb_create(const coeb_orb_params* params, int device, int max_width, int max_height,
                      int max_batch);
void coeb_destroy(coeb_ctx* ctx);
const char* coeb_last_error(const coeb_ctx* ctx);   /* also valid with ctx == NULL */
int coeb_orb_tables_get(const coeb_ctx* ctx, coeb_orb_tables* out);
/* keypoint capacity per frame needed by coeb_extract for a w x h image */
int coeb_max_keypoints(const coeb_ctx* ctx, int width, int height);

/* ---- ORBextractor::operator() on one host frame ----
 * gray: 8UC1 (stride in bytes).  boxes/T_M/blur_flag as passed by Frame::ExtractORB.
 * Writes up to `cap` keypoints and their 32-byte descriptors; *n_out = keypoint count.
 * An empty image (width or height 0) returns COEB_OK with *n_out = 0 (:1096-1097). */
int coeb_extract(coeb_ctx* ctx, const uint8_t* gray, int width, int height, size_t stride,
                 const coeb_box* boxes, int nbox, const float* tm_xy, int ntm,
                 const int32_t* blur_flag, int nblur,
                 coeb_keypoint* kp_out, uint8_t* desc_out, int cap, int* n_out);

/* ---- device-resident batch (the throughput path) ----
 * d_gray: device pointer, nframes x height x width bytes, packed.  boxes/T_M/blur flags are
 * host arrays: per frame f, boxes[box_off[f] .. box_off[f+1]) etc. (offset arrays of length
 * nframes+1; all may be NULL for "no boxes").  Results stay on the device; fetch them with
 * coeb_batch_results.  Returns without synchronising: the frames are split into contiguous
 * chunks, one per batch stream (coeb_set_batch_streams), so the kernels of different chunks
 * overlap on the device; every other call on the context waits for them. */
int coeb_extract_batch_device(coeb_ctx* ctx, const uint8_t* d_gray, int nframes, int width, int height,
                              const coeb_box* boxes, const int32_t* box_off,
                              const float* tm_xy, const int32_t* tm_off,
                              const int32_t* blur_flag);
/* The RGB-D Frame constructor on a device-resident batch (src/Frame.cc:157-214): for frame f,
 * ProcessMovingObject(frame f-1, frame f) -> T_M (:164-166, coeb_moving_object_points), the
 * detect_laplacian blur flag of every box (:171-202; frame 0 is the sequence's first frame: no
 * T_M, flags 0, :205-208), then ORBextractor::operator() with those boxes, T_M and flags (:214).
 * T_M and the flags never leave the device (coeb_batch_frame_results exposes them).  Boxes are
 * host arrays as in coeb_extract_batch_device (NULL: none).  Runs on the context stream only;
 * results as coeb_extract_batch_device's (coeb_batch_results), and the batch matcher / pose
 * entry points follow it. */
int coeb_frame_batch_device(coeb_ctx* ctx, const uint8_t* d_gray, int nframes, int width, int height,
                            const coeb_box* boxes, const int32_t* box_off);
/* Device pointers of the last coeb_frame_batch_device: T_M of frame f at d_tm + f * tm_cap * 2
 * (x, y floats), |T_M| in d_ntm[f] (-1: the fundamental matrix was empty), blur flags per box
 * (NULL without boxes). */
int coeb_batch_frame_results(coeb_ctx* ctx, const float** d_tm, const int32_t** d_ntm, int* tm_cap,
                             const int32_t** d_blur);
/* Device pointers to the batch outputs: keypoints [nframes][kcap], descriptors
 * [nframes][kcap][32], counts [nframes]. */
int coeb_batch_results(coeb_ctx* ctx, const coeb_keypoint** d_kps, const uint8_t** d_desc,
                       const int32_t** d_counts, int* kcap);
/* Number of HIP streams a batch is spread over (1..16, default 1; chunks of >= 16 frames).
 * 1 = every kernel of the batch on the context stream, one after another. */
int coeb_set_batch_streams(coeb_ctx* ctx, int nstreams);

/* Batch TrackWithMotionModel matching (Tracking.cc:933-958 call pattern): for f = 1..nframes-1
 * frame f is matched to frame f-1 of the last extracted batch.  Frame f-1 is the LastFrame and
 * defines the world frame (its Tcw = I): its map points are its keypoints with depth > 0
 * unprojected with Twc = I (Frame::UnprojectStereo, Frame.cc:844-858), Observations() = nobs.
 * Tcw[f] (row-major 4x4, host, nframes x 16 floats; entry 0 unused) is the pose of frame f
 * relative to frame f-1 (the motion-model prediction mVelocity*mLastFrame.mTcw,
 * Tracking.cc:937).  SearchByProjection(th) and, if < 20 matches, again with 2*th.
 * d_depth: nframes x height x width float (device).  Results: coeb_batch_match_results. */
int coeb_match_batch_device(coeb_ctx* ctx, const float* d_depth, int nframes, int width, int height,
                            const coeb_camera* cam, const float* Tcw, float th, int32_t nobs);
/* The same with the poses already in device memory (d_Tcw: nframes x 16 floats). */
int coeb_match_batch_device_tcw(coeb_ctx* ctx, const float* d_depth, int nframes, int width, int height,
                                const coeb_camera* cam, const float* d_Tcw, float th, int32_t nobs);
int coeb_batch_match_results(coeb_ctx* ctx, const int32_t** d_match, const int32_t** d_nmatches);

/* ---- Tracking::TrackWithMotionModel tail on the batch (Tracking.cc:947-964) ----
 * After coeb_match_batch_device*: for every pair, CurrentFrame.mvpMapPoints = the matcher's
 * assignments (positions from the LastFrame snapshot), then, if nmatches >= min_matches (20 in
 * the reference, :954-958), Optimizer::PoseOptimization (as coeb_pose_optimization) from the
 * prediction d_Tcw (the same nframes x 16 device array the matcher used).  Results (device,
 * frame 0 = halo): coeb_batch_pose_results -> Tcw nframes x 16 (the prediction where the frame
 * was not optimised), ninliers per frame (0: not tracked), outlier flags nframes x capacity. */
int coeb_pose_batch_device(coeb_ctx* ctx, const coeb_camera* cam, int nframes, const float* d_Tcw,
                           int32_t min_matches);
int coeb_batch_pose_results(coeb_ctx* ctx, const float** d_Tcw, const int32_t** d_ninliers,
                            const uint8_t** d_outlier);

/* ---- Tracking::TrackLocalMap on the batch (Tracking.cc:966-993, 996-1047, 1222-1272) ----
 * After coeb_pose_batch_device on the same batch, for every frame f >= 1:
 *   - TrackWithMotionModel's tail: matched keypoints the first PoseOptimization flagged outlier
 *     lose their MapPoint; nmatchesMap = kept MapPoints with Observations() > 0; the frame goes
 *     on only if the motion model ran (>= min_matches) and nmatchesMap >= 10 (:993);
 *   - the local map: the MapPoints of KeyFrames f-1 (KF1, the pair's world frame) and, with
 *     nkf = 2, f-2 (KF2, placed by frame f-1's motion-model pose), one MapPoint per keypoint with
 *     depth > 0; points matched by the motion model are skipped (mnLastFrameSeen),
 *     the rest go through Frame::isInFrustum(pMP, 0.5) with the first pose;
 *   - ORBmatcher(nnratio).SearchByProjection(F, vpLocalMapPoints, th) (3 for RGB-D, :1264-1270);
 *   - Optimizer::PoseOptimization from the first pose over the kept and the new MapPoints.
 * Observations() of every MapPoint = the nobs of coeb_match_batch_device.  Work is enqueued
 * behind the first k_pose on the pose stream.  Results (device, frame 0 = halo):
 * coeb_batch_track_results -> Tcw nframes x 16 (the first pose where TrackLocalMap did not run),
 * ninliers per frame (the second PoseOptimization's return = mnMatchesInliers when nobs > 0;
 * 0: not run), nmatches_map per frame, nlocal = SearchByProjection's return, local_match
 * nframes x capacity (local-map index per keypoint: [0, capacity) KF2 slot, [capacity,
 * 2 capacity) KF1 slot, -1), outlier flags nframes x capacity (mvbOutlier of the second run). */
int coeb_track_local_map_batch_device(coeb_ctx* ctx, const coeb_camera* cam, int nframes, int32_t nkf, float th,
                                      float nnratio);
int coeb_batch_track_results(coeb_ctx* ctx, const float** d_Tcw, const int32_t** d_ninliers,
                             const int32_t** d_nmatches_map, const int32_t** d_nlocal,
                             const int32_t** d_local_match, const uint8_t** d_outlier);

/* ---- ORBmatcher::SearchByProjection(CurrentFrame, LastFrame, th, bMono) ----
 * match_out[i2] (length cur->n) = index of the LastFrame slot whose MapPoint was assigned to
 * current keypoint i2 (CurrentFrame.mvpMapPoints[i2]), or -1; *nmatches = the return value.
 * CurrentFrame.mvpMapPoints is taken as all-NULL on entry (Tracking.cc:943). */
int coeb_match_lastframe(coeb_ctx* ctx, const coeb_camera* cam, const coeb_curframe* cur,
                         const coeb_lastframe* last, const float Tcw_cur[16], const float Tcw_last[16],
                         float th, int bmono, int check_orientation, int32_t* match_out, int* nmatches);

/* Local-map points as Frame::isInFrustum left them (Frame.cc:445-501 writes mbTrackInView,
 * mTrackProjX/Y/XR, mnTrackScaleLevel, mTrackViewCos); ORBmatcher.cc:50-80 reads exactly these. */
typedef struct {
    int32_t n;                        /* vpMapPoints.size() */
    const uint8_t* in_view;           /* mbTrackInView && !isBad() */
    const float* proj_x;              /* mTrackProjX */
    const float* proj_y;              /* mTrackProjY */
    const float* proj_xr;             /* mTrackProjXR */
    const int32_t* level;             /* mnTrackScaleLevel (0 .. nlevels-1 where in_view) */
    const float* view_cos;            /* mTrackViewCos */
    const uint8_t* descriptor;        /* n x 32, GetDescriptor() */
    const int32_t* observations;      /* Observations() */
} coeb_localmap;

/* ---- ORBmatcher::SearchByProjection(CurrentFrame, vpLocalMapPoints, th) ----
 * cur_observations[i] (length cur->n, may be NULL = all NULL): Observations() of the MapPoint
 * already in CurrentFrame.mvpMapPoints[i], or -1 for NULL; keypoints whose holder has
 * Observations() > 0 are skipped (ORBmatcher.cc:86-88), as are keypoints given on the way to a
 * point with Observations() > 0.  match_out[i] (length cur->n) = index of the local-map point
 * assigned to keypoint i by this call (the last one when several were), or -1; *nmatches = the
 * return value (every assignment counts, as in the reference).  nnratio = mfNNratio. */
int coeb_match_localmap(coeb_ctx* ctx, const coeb_camera* cam, const coeb_curframe* cur,
                        const int32_t* cur_observations, const coeb_localmap* mp, float th,
                        float nnratio, int32_t* match_out, int* nmatches);

/* Map points of a KeyFrame as ORBmatcher.cc:1487-1530 reads them (pKF->GetMapPointMatches()). */
typedef struct {
    int32_t n;                        /* vpMPs.size() */
    const uint8_t* valid;             /* pMP && !pMP->isBad() && !sAlreadyFound.count(pMP) */
    const float* world_pos;           /* n x 3, GetWorldPos() */
    const uint8_t* descriptor;        /* n x 32, GetDescriptor() */
    const float* max_distance;        /* mfMaxDistance (GetMaxDistanceInvariance() = 1.2f * it) */
    const float* min_distance;        /* mfMinDistance (GetMinDistanceInvariance() = 0.8f * it) */
    const float* angle;               /* pKF->mvKeysUn[i].angle */
} coeb_keyframe_points;

/* ---- ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) ----
 * cur_has_mappoint[i] (length cur->n, may be NULL = all NULL): CurrentFrame.mvpMapPoints[i] !=
 * NULL on entry; such keypoints are skipped, as are keypoints given earlier in the call.
 * Tcw: CurrentFrame.mTcw (row-major 4x4).  The scale pyramid is the context's (mnScaleLevels,
 * mvScaleFactors, mfLogScaleFactor).  match_out[i] = index of the KeyFrame point assigned to
 * keypoint i, or -1; *nmatches = the return value (after the rotation filter when
 * check_orientation = mbCheckOrientation).  cur->u_right is not read (may be NULL). */
int coeb_match_keyframe(coeb_ctx* ctx, const coeb_camera* cam, const coeb_curframe* cur,
                        const uint8_t* cur_has_mappoint, const coeb_keyframe_points* kf,
                        const float Tcw[16], float th, int orb_dist, int check_orientation,
                        int32_t* match_out, int* nmatches);

/* The Frame fields Optimizer::PoseOptimization reads (Optimizer.cc:276-357). */
typedef struct {
    int32_t n;                        /* pFrame->N */
    const uint8_t* has_mappoint;      /* mvpMapPoints[i] != NULL */
    const float* world_pos;           /* n x 3, GetWorldPos() (read where has_mappoint) */
    const coeb_keypoint* keys_un;     /* mvKeysUn (pt, octave) */
    const float* u_right;             /* mvuRight (< 0: monocular edge) */
} coeb_pose_frame;

/* ---- Optimizer::PoseOptimization(pFrame) ----
 * Tcw: pFrame->mTcw on entry (row-major 4x4), the optimised pose on return (SetPose).
 * outlier_out[i] (length n) = mvbOutlier[i], written where has_mappoint[i].  *ninliers = the
 * return value (nInitialCorrespondences - nBad; 0 and Tcw untouched with < 3 edges).  The
 * information matrices use the context's mvInvLevelSigma2; cam supplies fx, fy, cx, cy, mbf. */
int coeb_pose_optimization(coeb_ctx* ctx, const coeb_camera* cam, const coeb_pose_frame* frame, float Tcw[16],
                           uint8_t* outlier_out, int* ninliers);

/* ---- Frame helpers ---- */
int coeb_blur_flags(coeb_ctx* ctx, const uint8_t* gray, int width, int height, size_t stride,
                    const coeb_box* boxes, int nbox, int32_t* flags_out);
int coeb_stereo_from_rgbd(coeb_ctx* ctx, const coeb_keypoint* kps, int n, const float* depth,
                          int width, int height, size_t depth_stride_floats, float bf,
                          float* u_right_out, float* depth_out);
/* Tracking::GrabImageRGBD's input conversions (src/Tracking.cc:212-228).
 * img: `channels` = 1 (8UC1, copied), 3 (8UC3: RGB2GRAY when rgb_order = 1, as Camera.RGB = 1,
 * else BGR2GRAY) or 4 (8UC4: RGBA2GRAY / BGRA2GRAY, alpha ignored); img_stride in bytes.
 * depth: depth_type COEB_DEPTH_U16 (16UC1) or COEB_DEPTH_F32 (32FC1), depth_stride in bytes;
 * imDepth.convertTo(CV_32F, depth_scale) with depth_scale = mDepthMapFactor (= 1/DepthMapFactor),
 * except that a 32F map with |depth_scale - 1| <= 1e-5 is passed through unchanged (:227).
 * Either input may be NULL. */
#define COEB_DEPTH_U16 0
#define COEB_DEPTH_F32 1
int coeb_rgbd_preprocess(coeb_ctx* ctx, const uint8_t* img, size_t img_stride, int channels, int rgb_order,
                         const void* depth, size_t depth_stride, int depth_type, float depth_scale,
                         int width, int height, uint8_t* gray_out, float* depth_out);

/* The same conversions over a packed device batch: d_img nframes x height x width x channels,
 * d_depth nframes x height x width (16UC1 or 32FC1), outputs packed gray / float depth; width a
 * multiple of 4, image buffers 4-byte and depth buffers 16-byte aligned.  Enqueued on the
 * context stream (the batch pipeline's first step, BASELINE configs[4]). */
int coeb_rgbd_preprocess_batch_device(coeb_ctx* ctx, const uint8_t* d_img, int channels, int rgb_order,
                                      const void* d_depth, int depth_type, float depth_scale, int nframes, int width,
                                      int height, uint8_t* d_gray, float* d_depth_out);
/* mvKeysUn from mvKeys: cv::undistortPoints(.., mK, mDistCoef, Mat(), mK) (OpenCV 3.4, 5
 * iterations) with dist = (k1, k2, p1, p2, k3) (k3 = 0 for a 4-coefficient mDistCoef);
 * dist[0] == 0 copies (Frame.cc:581-585).  out may equal kps. */
int coeb_undistort_keypoints(coeb_ctx* ctx, const coeb_camera* cam, const float dist[5], const coeb_keypoint* kps,
                             int n, coeb_keypoint* out);
/* yolov5_ros_msgs/BoundingBox (int64 xmin, ymin, xmax, ymax) -> coeb_box, as GrabRGBD converts */
int coeb_boxes_from_int64(const int64_t* xyxy, int nbox, coeb_box* out);

/* ---- TUM RGB-D time-stamp lists (associate.py, the ingest step before GrabImageRGBD) ----
 * Host-only (no context, no device).  coeb_tum_read_list parses a list file's text
 * (associate.py:49-69): lines split at '\n'; ',' and TAB separate fields like ' '; a line whose
 * first byte is '#' is a comment; lines with fewer than two fields are ignored; the first field
 * must be a decimal float literal (else COEB_EINVAL, where read_file_list raises).  A stamp that
 * occurs twice keeps its last line at the position of its first (the reference's dict).  Per
 * entry: the stamp, and the byte offset / length in `text` of its data fields (second field to
 * the end of the last).  *n_out = entries; COEB_ERANGE when that exceeds cap (nothing written).
 * coeb_tum_associate (associate.py:71-102): candidates |a - (b + offset)| < max_difference in
 * double, taken greedily by increasing (difference, a, b), each stamp once, returned as index
 * pairs into first / second ordered by (a, b); a stamp given twice is its last index, NaN never
 * matches.  *n_out = matches; COEB_ERANGE when that exceeds cap. */
int coeb_tum_read_list(const char* text, size_t len, double* stamps, int64_t* data_off, int32_t* data_len, int cap,
                       int* n_out);
int coeb_tum_associate(const double* first, int n_first, const double* second, int n_second, double offset,
                       double max_difference, int32_t* first_idx, int32_t* second_idx, int cap, int* n_out);

/* ---- Frame::ProcessMovingObject (src/Frame.cc:311-393): T_M from imGrayPre and imgray ----
 * Each stage replaces the OpenCV 3.4 call Frame.cc makes, in the canonical forms of DESIGN.md
 * s2.1 / s4.10 (parity against the oracle; OpenCV itself is absent, parity vs it UNPINNED):
 *   coeb_good_features        <- cv::goodFeaturesToTrack(img, pts, 1000, 0.01, 8, Mat(), 3, true, 0.04)  :333
 *                                (*n_out = corner count; COEB_ERANGE past 16384 local maxima)
 *   coeb_corner_subpix        <- cv::cornerSubPix(img, pts, Size(10,10), Size(-1,-1), (ITER|EPS, 20, 0.03))  :334
 *                                (in place; win must be 10)
 *   coeb_optical_flow_pyr_lk  <- cv::calcOpticalFlowPyrLK(prev, next, pts, next_pts, status, err,
 *                                Size(22,22), 5, (ITER|EPS, 20, 0.01))  :335  (win <= 22)
 *   coeb_moving_tail          <- the SAD check (:337-365), cv::findFundamentalMat(.., FM_RANSAC, 0.1, 0.99)
 *                                (:373) and the epipolar distance test (:375-384); state in/out
 *   coeb_moving_object_points <- the whole of ProcessMovingObject; *n_tm = |T_M|, or -1 when
 *                                findFundamentalMat returns an empty Mat (the reference then reads
 *                                an empty Mat: undefined behaviour)
 * At most 1024 points per call (the reference asks for 1000 corners). */
typedef struct {
    float* corners_raw;   /* 1000 x 2: goodFeaturesToTrack output (optional) */
    float* corners;       /* 1000 x 2: after cornerSubPix (optional) */
    int* ncorners;
    float* next_pts;      /* 1000 x 2: calcOpticalFlowPyrLK output */
    uint8_t* status;      /* 1000: LK status */
    uint8_t* state;       /* 1000: state after the SAD check */
    double* F;            /* 9: the fundamental matrix */
    int* nf;              /* |F_prepoint| */
} coeb_flow_debug;
int coeb_good_features(coeb_ctx* ctx, const uint8_t* img, int width, int height, size_t stride, int max_corners,
                       double quality, double min_distance, double k, float* xy_out, int cap, int* n_out);
int coeb_corner_subpix(coeb_ctx* ctx, const uint8_t* img, int width, int height, size_t stride, float* xy, int n,
                       int win, int max_iter, double eps);
int coeb_optical_flow_pyr_lk(coeb_ctx* ctx, const uint8_t* prev, const uint8_t* next, int width, int height,
                             size_t stride, const float* prev_xy, int n, int win, int max_level, int max_count,
                             double eps, float* next_xy, uint8_t* status);
int coeb_moving_tail(coeb_ctx* ctx, const uint8_t* prev, const uint8_t* cur, int width, int height, size_t stride,
                     const float* prev_xy, const float* next_xy, uint8_t* state, int n, float* tm_xy, int tm_cap,
                     int* n_tm, double F_out[9], int* nf_out);
int coeb_moving_object_points(coeb_ctx* ctx, const uint8_t* prev, const uint8_t* cur, int width, int height,
                              size_t stride, float* tm_xy, int tm_cap, int* n_tm, coeb_flow_debug* dbg);
/* the same on device-resident frames (pitch stride) */
int coeb_moving_object_points_device(coeb_ctx* ctx, const uint8_t* d_prev, const uint8_t* d_cur, int width,
                                     int height, size_t stride, float* tm_xy, int tm_cap, int* n_tm,
                                     coeb_flow_debug* dbg);

int coeb_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* ---- device memory owned by the caller (for the device-resident batch entry points) ----
 * Plain hipMalloc'ed buffers on the context's device.  Copies are synchronous w.r.t. the
 * context stream (they are enqueued on it and waited for). */
int coeb_device_alloc(coeb_ctx* ctx, size_t bytes, void** dptr);
int coeb_device_free(coeb_ctx* ctx, void* dptr);
int coeb_memcpy_h2d(coeb_ctx* ctx, void* dst, const void* src, size_t bytes);
int coeb_memcpy_d2h(coeb_ctx* ctx, void* dst, const void* src, size_t bytes);
/* Host-resident batches with copy / kernel overlap: page-locked host memory, and copies
 * enqueued on the context stream behind the work already there (returning at once; the data
 * is in place after coeb_synchronize).  From page-locked memory the copies run on the DMA
 * engines beside the kernels of other contexts' streams. */
int coeb_host_alloc(size_t bytes, void** ptr);
int coeb_host_free(void* ptr);
int coeb_memcpy_h2d_async(coeb_ctx* ctx, void* dst, const void* src, size_t bytes);
int coeb_memcpy_d2h_async(coeb_ctx* ctx, void* dst, const void* src, size_t bytes);
/* Copy queues: a HIP stream of their own on a context's device, for pipelines whose uploads
 * must run back to back (one upload queue for all batches: concurrent uploads only split the
 * PCIe bandwidth) while earlier batches compute on the contexts' streams.  Copies are
 * asynchronous (page-locked host memory); ordering against a context is explicit:
 *   coeb_copyq_after_ctx(q, ctx)  work enqueued on q from now on waits for everything enqueued
 *                                 on ctx so far (e.g. the kernels reading the buffer to refill);
 *   coeb_ctx_after_copyq(ctx, q)  work enqueued on ctx from now on waits for everything
 *                                 enqueued on q so far (e.g. the upload of the next batch). */
typedef struct coeb_copyq coeb_copyq;
coeb_copyq* coeb_copyq_create(coeb_ctx* ctx);
int coeb_copyq_destroy(coeb_copyq* q);
int coeb_copyq_h2d(coeb_copyq* q, void* dst, const void* src, size_t bytes);
int coeb_copyq_d2h(coeb_copyq* q, void* dst, const void* src, size_t bytes);
int coeb_copyq_after_ctx(coeb_copyq* q, coeb_ctx* ctx);
int coeb_ctx_after_copyq(coeb_ctx* ctx, coeb_copyq* q);
int coeb_copyq_synchronize(coeb_copyq* q);
/* Markers: a point recorded on a context or copy queue now and waited for later (by another
 * context or queue, or by the host), for pipelines whose waits refer to work enqueued several
 * steps earlier (e.g. "the kernels of batch i - 3 are done with this input buffer"). */
typedef struct coeb_marker coeb_marker;
coeb_marker* coeb_marker_create(coeb_ctx* ctx);
int coeb_marker_destroy(coeb_marker* m);
int coeb_marker_record_ctx(coeb_marker* m, coeb_ctx* ctx);       /* after all work enqueued on ctx */
int coeb_marker_record_copyq(coeb_marker* m, coeb_copyq* q);     /* after all work enqueued on q */
int coeb_ctx_wait_marker(coeb_ctx* ctx, coeb_marker* m);         /* later work on ctx waits for m */
int coeb_copyq_wait_marker(coeb_copyq* q, coeb_marker* m);       /* later work on q waits for m */
int coeb_marker_synchronize(coeb_marker* m);                     /* host waits for m */

/* ---- measurement ---- */
/* Per-kernel device time accumulated with HIP events on the context stream while profiling
 * is enabled.  names: comma-separated list written to `names` (cap bytes). */
int coeb_profile_enable(coeb_ctx* ctx, int enable);
int coeb_profile_read(coeb_ctx* ctx, char* names, int cap, double* total_ms, int64_t* launches,
                      int max_kernels, int* nkernels);
int coeb_profile_reset(coeb_ctx* ctx);
int coeb_synchronize(coeb_ctx* ctx);
int coeb_device_count(void);

/* Test support: copy an intermediate buffer of frame `frame` of the last batch to the host.
 * what: "pyr" (levels 1..L-1, packed), "blur" (levels 0..L-1), "cand_n" (FAST corners per
 * cell), "lvl_n" (keypoints per level), "lvl_kp" (packed level keypoints), "dyn" (mask
 * rectangles), "plan", "search_path" (int32 {path, iterations} of the last
 * coeb_match_localmap / coeb_match_keyframe: 0 parallel claims, 1 forced sequential,
 * 2 candidate-list overflow, 3 no convergence; frame ignored; alias "localmap_path").  Copies min(bytes, size); *size_out = full size. */
int coeb_debug_read(coeb_ctx* ctx, const char* what, int frame, void* host, size_t bytes, size_t* size_out);

#ifdef __cplusplus
}
#endif
#endif
