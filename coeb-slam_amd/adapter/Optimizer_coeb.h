/*
 * Optimizer_coeb.h -- MI355X body for Optimizer::PoseOptimization(Frame *pFrame)
 * (include/Optimizer.h:47, src/Optimizer.cc:239-451).
 *
 * Included from the reference's src/Optimizer.cc; the function body becomes
 *
 *     return coeb::PoseOptimization(pFrame);
 *
 * What it does, in the reference's terms:
 *   - under MapPoint::mGlobalMutex (as :276) snapshots, per keypoint, mvpMapPoints[i] != NULL
 *     and GetWorldPos(), with mvKeysUn, mvuRight and mTcw;
 *   - calls coeb_pose_optimization (g2o's Levenberg-Marquardt restated on the device: 4 rounds
 *     x 10 iterations, Huber kernels, chi2 5.991 / 7.815 classification);
 *   - writes mvbOutlier for the keypoints with a MapPoint and pFrame->SetPose(Tcw) (:446-448),
 *     and returns nInitialCorrespondences - nBad (0 and no SetPose with < 3 edges, :361-362).
 * g2o is not vendored in the reference: the device code follows g2o's published algorithm,
 * parity with the g2o binary is unpinned.
 */
#ifndef COEB_ADAPTER_OPTIMIZER_H
#define COEB_ADAPTER_OPTIMIZER_H

#include <mutex>
#include <stdexcept>
#include <vector>

#include <opencv2/core/core.hpp>

#include "coeb_front.h"
#include "ORBmatcher_coeb.h"

namespace coeb
{

template <class FrameT>
inline int PoseOptimization(FrameT* pFrame, coeb_ctx* ctx = nullptr)
{
    using MapPointT = typename std::remove_pointer<typename decltype(pFrame->mvpMapPoints)::value_type>::type;
    if (!ctx) ctx = matcher_ctx(pFrame->mnScaleLevels, pFrame->mfScaleFactor);
    const int N = pFrame->N;
    std::vector<uint8_t> has((size_t)N), outl((size_t)N);
    std::vector<float> xw((size_t)N * 3);
    {
        std::unique_lock<std::mutex> lock(MapPointT::mGlobalMutex);
        for (int i = 0; i < N; ++i) {
            MapPointT* pMP = pFrame->mvpMapPoints[i];
            has[i] = pMP != nullptr;
            if (!pMP) continue;
            cv::Mat x3D = pMP->GetWorldPos();
            xw[3 * i + 0] = x3D.at<float>(0);
            xw[3 * i + 1] = x3D.at<float>(1);
            xw[3 * i + 2] = x3D.at<float>(2);
        }
    }
    coeb_pose_frame fr{N, has.data(), xw.data(), reinterpret_cast<const coeb_keypoint*>(pFrame->mvKeysUn.data()),
                       pFrame->mvuRight.data()};
    const coeb_camera cam = frame_camera(*pFrame);
    float T[16];
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 4; ++k) T[4 * r + k] = pFrame->mTcw.template at<float>(r, k);
    int ninl = 0;
    if (coeb_pose_optimization(ctx, &cam, &fr, T, outl.data(), &ninl) != COEB_OK)
        throw std::runtime_error(coeb_last_error(ctx));
    int nInitial = 0;
    for (int i = 0; i < N; ++i)
        if (has[i]) { pFrame->mvbOutlier[i] = outl[i] != 0; nInitial++; }
    if (nInitial < 3) return 0;
    cv::Mat pose(4, 4, CV_32F);
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 4; ++k) pose.at<float>(r, k) = T[4 * r + k];
    pFrame->SetPose(pose);
    return ninl;
}

}  // namespace coeb

#endif
