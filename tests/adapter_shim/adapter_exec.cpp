// Runs the drop-in C++ adapters (coeb-slam_amd/adapter/) against libcoeb_front.so on the GPU,
// with reference-shaped Frame / MapPoint types (include/Frame.h:142-215, include/MapPoint.h:46-75
// member names) and the functional cv stand-in of tests/adapter_shim/opencv2.
//
//   adapter_exec DIR
//
// DIR holds the inputs tests/test_adapter_exec.py writes (raw little-endian arrays) and receives
// the outputs it compares with the oracle:
//   in : size.i32 (W, H), frame0.u8, frame1.u8 (W*H gray), cam.f32 (fx fy cx cy bf minX maxX minY
//        maxY), Tc.f32 / Tl.f32 (4x4 row-major), last_has.u8, last_nobs.i32, last_xw.f32 (N0 x 3),
//        last_desc.u8 (N0 x 32) -- the LastFrame map snapshot of frame 0 -- and cur_ur.f32 (N1)
//   out: kps{0,1}.bin (cv::KeyPoint records), desc{0,1}.u8, match.i32 (per current keypoint the
//        LastFrame keypoint whose MapPoint it got, -1), nmatch.i32, pose_T.f32, pose_outl.u8,
//        pose_nin.i32, checks.txt (reference conventions: empty image, zero keypoints)
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "ORBextractor.h"
#include "ORBmatcher_coeb.h"
#include "Optimizer_coeb.h"

struct MapPoint {
    cv::Mat pos, desc;
    int nobs = 0;
    cv::Mat GetWorldPos() { return pos.clone(); }
    cv::Mat GetDescriptor() { return desc.clone(); }
    int Observations() { return nobs; }
    bool isBad() { return false; }
    static std::mutex mGlobalMutex;
};
std::mutex MapPoint::mGlobalMutex;

struct Frame {
    static float fx, fy, cx, cy, mnMinX, mnMaxX, mnMinY, mnMaxY;
    float mbf = 0;
    int N = 0;
    int mnScaleLevels = 8;
    float mfScaleFactor = 1.2f;
    std::vector<cv::KeyPoint> mvKeysUn;
    std::vector<float> mvuRight;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    cv::Mat mDescriptors, mTcw;
    void SetPose(cv::Mat Tcw) { mTcw = Tcw.clone(); }
};
float Frame::fx, Frame::fy, Frame::cx, Frame::cy, Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY;

template <class T>
static std::vector<T> load(const std::string& path)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) { std::cerr << "missing " << path << "\n"; std::exit(2); }
    std::vector<char> raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::vector<T> v(raw.size() / sizeof(T));
    if (!v.empty()) std::memcpy(v.data(), raw.data(), v.size() * sizeof(T));
    return v;
}

template <class T>
static void save(const std::string& path, const T* p, size_t n)
{
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), (std::streamsize)(n * sizeof(T)));
}

static cv::Mat mat4(const std::vector<float>& t)
{
    cv::Mat m(4, 4, CV_32F);
    for (int r = 0; r < 4; r++)
        for (int k = 0; k < 4; k++) m.at<float>(r, k) = t[4 * r + k];
    return m;
}

int main(int argc, char** argv)
{
    if (argc != 2) { std::cerr << "usage: adapter_exec DIR\n"; return 2; }
    const std::string d = std::string(argv[1]) + "/";
    const std::vector<int32_t> size = load<int32_t>(d + "size.i32");
    const int W = size[0], H = size[1];
    std::vector<uint8_t> f0 = load<uint8_t>(d + "frame0.u8"), f1 = load<uint8_t>(d + "frame1.u8");

    // ---- ORBextractor::operator() (ORBextractor.h:73-75), two extractors with the same
    // parameters (Tracking re-creates them on tracking failure: the context pool serves both)
    std::vector<std::vector<float>> box;
    std::vector<cv::Point2f> tm;
    std::vector<int> blur;
    cv::Mat none, mask_result;
    std::vector<cv::KeyPoint> k0, k1;
    cv::Mat d0, d1;
    {
        ORB_SLAM2::ORBextractor ex(1000, 1.2f, 8, 20, 7);
        cv::Mat im0(H, W, CV_8U, f0.data());
        ex(im0, none, im0, none, k0, d0, box, tm, mask_result, blur);
    }
    ORB_SLAM2::ORBextractor ex2(1000, 1.2f, 8, 20, 7);
    cv::Mat im1(H, W, CV_8U, f1.data());
    ex2(im1, none, im1, none, k1, d1, box, tm, mask_result, blur);
    save(d + "kps0.bin", k0.data(), k0.size());
    save(d + "desc0.u8", d0.data, (size_t)d0.rows * 32);
    save(d + "kps1.bin", k1.data(), k1.size());
    save(d + "desc1.u8", d1.data, (size_t)d1.rows * 32);

    std::ofstream checks(d + "checks.txt");
    {   // empty image: return without touching the outputs (:1096-1097)
        std::vector<cv::KeyPoint> kk(3);
        kk[0].octave = 77;
        cv::Mat dd(2, 32, CV_8U);
        cv::Mat empty;
        ex2(empty, none, empty, none, kk, dd, box, tm, mask_result, blur);
        checks << "empty_untouched " << (kk.size() == 3 && kk[0].octave == 77 && dd.rows == 2) << "\n";
    }
    {   // no keypoints: descriptors.release() (:1296-1297)
        std::vector<uint8_t> flat((size_t)W * H, 128);
        cv::Mat im(H, W, CV_8U, flat.data());
        std::vector<cv::KeyPoint> kk(5);
        cv::Mat dd(2, 32, CV_8U);
        ex2(im, none, im, none, kk, dd, box, tm, mask_result, blur);
        checks << "flat_released " << (kk.empty() && dd.empty()) << "\n";
    }
    {   // an image larger than the pooled context's 1280 x 960: the context grows (no size cap);
        // extracted on a worker thread, whose exit destroys that thread's pooled contexts
        const std::vector<int32_t> bs = load<int32_t>(d + "size_big.i32");
        std::vector<uint8_t> fb = load<uint8_t>(d + "frame_big.u8");
        std::vector<cv::KeyPoint> kb;
        cv::Mat db;
        std::thread th([&] {
            ORB_SLAM2::ORBextractor exb(2000, 1.2f, 8, 20, 7);
            cv::Mat small(H, W, CV_8U, f0.data());
            std::vector<cv::KeyPoint> ks;
            cv::Mat ds;
            exb(small, none, small, none, ks, ds, box, tm, mask_result, blur);   // context at 1280 x 960
            cv::Mat imb(bs[1], bs[0], CV_8U, fb.data());
            exb(imb, none, imb, none, kb, db, box, tm, mask_result, blur);      // grows
        });
        th.join();
        save(d + "kps_big.bin", kb.data(), kb.size());
        save(d + "desc_big.u8", db.data, (size_t)db.rows * 32);
    }
    ORB_SLAM2::ORBextractor ex3(1000, 1.2f, 8, 20, 7);
    checks << "accessors " << (ex3.GetLevels() == 8 && ex3.GetScaleFactors().size() == 8 &&
                               ex3.GetInverseScaleSigmaSquares().size() == 8 && ex3.GetScaleFactor() == 1.2f)
           << "\n";

    // ---- ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) (ORBmatcher.h:52)
    const std::vector<float> cam = load<float>(d + "cam.f32");
    Frame::fx = cam[0]; Frame::fy = cam[1]; Frame::cx = cam[2]; Frame::cy = cam[3];
    Frame::mnMinX = cam[5]; Frame::mnMaxX = cam[6]; Frame::mnMinY = cam[7]; Frame::mnMaxY = cam[8];
    const std::vector<uint8_t> has = load<uint8_t>(d + "last_has.u8");
    const std::vector<int32_t> nobs = load<int32_t>(d + "last_nobs.i32");
    const std::vector<float> xw = load<float>(d + "last_xw.f32");
    const std::vector<uint8_t> mpd = load<uint8_t>(d + "last_desc.u8");
    std::vector<MapPoint> mps(k0.size());
    Frame last, cur;
    last.mbf = cur.mbf = cam[4];
    last.N = (int)k0.size();
    last.mvKeysUn = k0;
    last.mDescriptors = d0;
    last.mvpMapPoints.assign(k0.size(), nullptr);
    last.mvbOutlier.assign(k0.size(), false);
    last.mTcw = mat4(load<float>(d + "Tl.f32"));
    for (size_t i = 0; i < k0.size(); i++) {
        if (!has[i]) continue;
        mps[i].pos = cv::Mat(3, 1, CV_32F);
        for (int k = 0; k < 3; k++) mps[i].pos.at<float>(k) = xw[3 * i + k];
        mps[i].desc = cv::Mat(1, 32, CV_8U);
        std::memcpy(mps[i].desc.data, &mpd[32 * i], 32);
        mps[i].nobs = nobs[i];
        last.mvpMapPoints[i] = &mps[i];
    }
    cur.N = (int)k1.size();
    cur.mvKeysUn = k1;
    cur.mDescriptors = d1;
    cur.mvuRight = load<float>(d + "cur_ur.f32");
    cur.mvpMapPoints.assign(k1.size(), nullptr);
    cur.mvbOutlier.assign(k1.size(), false);
    cur.mTcw = mat4(load<float>(d + "Tc.f32"));
    int nm = coeb::SearchByProjectionLastFrame(cur, last, 15.0f, false, 0.9f, true);
    if (nm < 20) {                                   // Tracking.cc:950-956: clear and retry at 2 th
        std::fill(cur.mvpMapPoints.begin(), cur.mvpMapPoints.end(), nullptr);
        nm = coeb::SearchByProjectionLastFrame(cur, last, 30.0f, false, 0.9f, true);
    }
    std::vector<int32_t> match(k1.size(), -1);
    for (size_t i = 0; i < k1.size(); i++)
        if (cur.mvpMapPoints[i]) match[i] = (int32_t)(cur.mvpMapPoints[i] - mps.data());
    save(d + "match.i32", match.data(), match.size());
    save(d + "nmatch.i32", &nm, 1);

    // ---- Optimizer::PoseOptimization(Frame*) (Optimizer.h:47) on the matched frame
    const int nin = coeb::PoseOptimization(&cur);
    std::vector<float> T(16);
    for (int r = 0; r < 4; r++)
        for (int k = 0; k < 4; k++) T[4 * r + k] = cur.mTcw.at<float>(r, k);
    std::vector<uint8_t> outl(k1.size());
    for (size_t i = 0; i < k1.size(); i++) outl[i] = cur.mvbOutlier[i] ? 1 : 0;
    save(d + "pose_T.f32", T.data(), 16);
    save(d + "pose_outl.u8", outl.data(), outl.size());
    save(d + "pose_nin.i32", &nin, 1);
    std::cout << "adapter_exec: " << k0.size() << "/" << k1.size() << " keypoints, " << nm << " matches, " << nin
              << " pose inliers\n";
    return 0;
}
