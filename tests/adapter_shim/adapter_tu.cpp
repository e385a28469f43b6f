// Compile check of the drop-in adapters against reference-shaped Frame/MapPoint types
// (include/Frame.h:142-215, include/MapPoint.h:46-75 member names and types).
#include "ORBextractor.h"
#include "ORBmatcher_coeb.h"
#include "Optimizer_coeb.h"
#include "Frame_coeb.h"

struct MapPoint {
    cv::Mat GetWorldPos() { return cv::Mat(); }
    cv::Mat GetDescriptor() { return cv::Mat(); }
    int Observations() { return 2; }
    bool isBad() { return false; }
    bool mbTrackInView = false;
    float mTrackProjX = 0, mTrackProjY = 0, mTrackProjXR = 0;
    int mnTrackScaleLevel = 0;
    float mTrackViewCos = 0;
    float GetMaxDistance() { return 0; }   // the two getters INTEGRATION.md s3 adds
    float GetMinDistance() { return 0; }
    static std::mutex mGlobalMutex;
};
std::mutex MapPoint::mGlobalMutex;
struct KeyFrame {
    std::vector<MapPoint*> GetMapPointMatches() { return {}; }
    std::vector<cv::KeyPoint> mvKeysUn;
};
struct Frame {
    static float fx, fy, cx, cy, mnMinX, mnMaxX, mnMinY, mnMaxY;
    float mbf = 0, mb = 0;
    int N = 0;
    int mnScaleLevels = 8;
    float mfScaleFactor = 1.2f;
    std::vector<cv::KeyPoint> mvKeysUn;
    std::vector<float> mvuRight;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    cv::Mat mDescriptors, mTcw;
    void SetPose(cv::Mat Tcw) { mTcw = Tcw; }
};
float Frame::fx, Frame::fy, Frame::cx, Frame::cy, Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY;

int moving_points(const cv::Mat& im)
{
    std::vector<cv::Point2f> T_M;
    coeb::ProcessMovingObject(im, im, T_M);
    return (int)T_M.size();
}

int use_adapters(Frame& cur, const Frame& last, cv::Mat& im)
{
    ORB_SLAM2::ORBextractor ex(1000, 1.2f, 8, 20, 7);
    std::vector<cv::KeyPoint> kps;
    cv::Mat desc, mask_result;
    std::vector<std::vector<float>> box;
    std::vector<cv::Point2f> tm;
    std::vector<int> blur;
    ex(im, cv::Mat(), im, im, kps, desc, box, tm, mask_result, blur);
    std::vector<MapPoint*> local;
    return coeb::SearchByProjectionLastFrame(cur, last, 15.0f, false, 0.9f, true) + ex.GetLevels() +
           coeb::SearchByProjectionLocalMap(cur, local, 3.0f, 0.8f) +
           coeb::SearchByProjectionKeyFrame(cur, (KeyFrame*)nullptr, std::set<MapPoint*>(), 10.0f, 100, true) +
           coeb::PoseOptimization(&cur) + moving_points(im);
}
