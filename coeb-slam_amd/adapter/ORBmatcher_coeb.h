/*
 * ORBmatcher_coeb.h -- MI355X bodies for two ORBmatcher::SearchByProjection overloads:
 *   (Frame&, const Frame&, float th, bool bMono)  include/ORBmatcher.h:52, src/ORBmatcher.cc:1329-1471
 *   (Frame&, const vector<MapPoint*>&, float th)  include/ORBmatcher.h:46, src/ORBmatcher.cc:44-129
 *   (Frame&, KeyFrame*, const set<MapPoint*>&, float th, int ORBdist)
 *                                                 include/ORBmatcher.h:55, src/ORBmatcher.cc:1473-1600
 *
 * Included from the reference's src/ORBmatcher.cc (which already includes Frame.h and
 * MapPoint.h); the method body becomes
 *
 *     return coeb::SearchByProjectionLastFrame(CurrentFrame, LastFrame, th, bMono,
 *                                              mfNNratio, mbCheckOrientation);
 *
 * What it does, in the reference's terms:
 *   - snapshots LastFrame under the MapPoint mutexes exactly where :1352-1396 reads them:
 *     mvpMapPoints[i] != NULL, mvbOutlier[i], GetWorldPos(), GetDescriptor(), Observations(),
 *     mvKeysUn[i].octave/.angle;
 *   - hands CurrentFrame.mvKeysUn / mDescriptors / mvuRight / mTcw and the Frame statics
 *     (fx, fy, cx, cy, mbf, mnMinX..mnMaxY) to coeb_match_lastframe;
 *   - writes CurrentFrame.mvpMapPoints[i2] = LastFrame.mvpMapPoints[match[i2]] and returns
 *     nmatches.  Tracking.cc:943 clears CurrentFrame.mvpMapPoints before the first call and
 *     the retry at :950-956 clears it again, which is the precondition the C-ABI documents.
 * mfNNratio is not read by this overload in the reference either (only the distance and
 * orientation tests apply); it is accepted to keep the call site symmetric.
 *
 * The local-map overload body becomes
 *
 *     return coeb::SearchByProjectionLocalMap(F, vpMapPoints, th, mfNNratio);
 *
 * It snapshots, per point, what :50-80 reads (mbTrackInView && !isBad(), mTrackProjX/Y/XR,
 * mnTrackScaleLevel, mTrackViewCos, GetDescriptor(), Observations()) and, per keypoint, the
 * Observations() of F.mvpMapPoints[i] (-1 for NULL), then writes F.mvpMapPoints[i] =
 * vpMapPoints[match[i]] for the keypoints the call assigned.
 *
 * The relocalisation overload body becomes
 *
 *     return coeb::SearchByProjectionKeyFrame(CurrentFrame, pKF, sAlreadyFound, th, ORBdist,
 *                                             mbCheckOrientation);
 *
 * It snapshots pKF->GetMapPointMatches() as :1489-1530 reads it (valid = pMP && !isBad() &&
 * !sAlreadyFound.count(pMP), GetWorldPos(), GetDescriptor(), the distance-invariance range and
 * pKF->mvKeysUn[i].angle) and which keypoints of CurrentFrame already hold a MapPoint.
 * MapPoint::PredictScale reads the protected mfMaxDistance, so the integration adds two locked
 * getters to MapPoint (GetMaxDistance / GetMinDistance).
 *
 * All use a matcher context built with the frame's own pyramid (F.mnScaleLevels,
 * F.mfScaleFactor), so mvScaleFactors on the device are the frame's.
 */
#ifndef COEB_ADAPTER_ORBMATCHER_H
#define COEB_ADAPTER_ORBMATCHER_H

#include <cstring>
#include <set>
#include <stdexcept>
#include <vector>

#include <opencv2/core/core.hpp>

#include "coeb_front.h"

namespace coeb
{

// matcher-only context per (thread, pyramid): only mvScaleFactors is read from its tables
inline coeb_ctx* matcher_ctx(int nlevels, float scale_factor)
{
    struct Entry { int nlevels; float scale; coeb_ctx* ctx; };
    static thread_local std::vector<Entry> pool;
    for (const Entry& e : pool)
        if (e.nlevels == nlevels && e.scale == scale_factor) return e.ctx;
    coeb_orb_params p{1000, scale_factor, nlevels, 20, 7};
    if (coeb_abi_version() != COEB_ABI_VERSION) throw std::runtime_error("libcoeb_front ABI differs from the header");
    coeb_ctx* c = coeb_create(&p, 0, 640, 480, 1);
    if (!c) throw std::runtime_error(coeb_last_error(nullptr));
    pool.push_back(Entry{nlevels, scale_factor, c});
    return c;
}

template <class FrameT>
inline coeb_camera frame_camera(const FrameT& F)
{
    return coeb_camera{FrameT::fx, FrameT::fy, FrameT::cx, FrameT::cy, F.mbf,
                       FrameT::mnMinX, FrameT::mnMaxX, FrameT::mnMinY, FrameT::mnMaxY};
}

template <class FrameT>
inline int SearchByProjectionLastFrame(FrameT& CurrentFrame, const FrameT& LastFrame, float th, bool bMono,
                                       float /*mfNNratio*/, bool mbCheckOrientation, coeb_ctx* ctx = nullptr)
{
    if (!ctx) ctx = matcher_ctx(CurrentFrame.mnScaleLevels, CurrentFrame.mfScaleFactor);
    const int nl = LastFrame.N;
    std::vector<uint8_t> has(nl), outl(nl), mpdesc((size_t)nl * 32);
    std::vector<float> xw((size_t)nl * 3);
    std::vector<int32_t> nobs(nl);
    for (int i = 0; i < nl; ++i) {
        auto* pMP = LastFrame.mvpMapPoints[i];
        has[i] = pMP != nullptr;
        outl[i] = LastFrame.mvbOutlier[i];
        if (!pMP) continue;
        cv::Mat x3D = pMP->GetWorldPos();
        xw[3 * i + 0] = x3D.at<float>(0);
        xw[3 * i + 1] = x3D.at<float>(1);
        xw[3 * i + 2] = x3D.at<float>(2);
        cv::Mat d = pMP->GetDescriptor();
        std::memcpy(&mpdesc[32 * (size_t)i], d.ptr<uint8_t>(0), 32);
        nobs[i] = pMP->Observations();
    }
    coeb_lastframe last{nl, has.data(), outl.data(), xw.data(), mpdesc.data(), nobs.data(),
                        reinterpret_cast<const coeb_keypoint*>(LastFrame.mvKeysUn.data())};
    cv::Mat curDesc = CurrentFrame.mDescriptors.isContinuous() ? CurrentFrame.mDescriptors
                                                               : CurrentFrame.mDescriptors.clone();
    coeb_curframe cur{CurrentFrame.N, reinterpret_cast<const coeb_keypoint*>(CurrentFrame.mvKeysUn.data()),
                      curDesc.empty() ? nullptr : curDesc.ptr<uint8_t>(0), CurrentFrame.mvuRight.data()};
    const coeb_camera cam = frame_camera(CurrentFrame);
    float Tc[16], Tl[16];
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 4; ++k) {
            Tc[4 * r + k] = CurrentFrame.mTcw.template at<float>(r, k);
            Tl[4 * r + k] = LastFrame.mTcw.template at<float>(r, k);
        }
    std::vector<int32_t> match((size_t)CurrentFrame.N);
    int nmatches = 0;
    const int rc = coeb_match_lastframe(ctx, &cam, &cur, &last, Tc, Tl, th, bMono ? 1 : 0,
                                        mbCheckOrientation ? 1 : 0, match.data(), &nmatches);
    if (rc != COEB_OK) throw std::runtime_error(coeb_last_error(ctx));
    for (int i2 = 0; i2 < CurrentFrame.N; ++i2)
        if (match[i2] >= 0) CurrentFrame.mvpMapPoints[i2] = LastFrame.mvpMapPoints[match[i2]];
    return nmatches;
}

template <class FrameT, class MapPointT>
inline int SearchByProjectionLocalMap(FrameT& F, const std::vector<MapPointT*>& vpMapPoints, float th,
                                      float mfNNratio, coeb_ctx* ctx = nullptr)
{
    if (!ctx) ctx = matcher_ctx(F.mnScaleLevels, F.mfScaleFactor);
    const int nq = (int)vpMapPoints.size();
    std::vector<uint8_t> view(nq), desc((size_t)nq * 32);
    std::vector<float> px(nq), py(nq), pxr(nq), vcos(nq);
    std::vector<int32_t> lvl(nq), nobs(nq), cobs((size_t)F.N);
    for (int q = 0; q < nq; ++q) {
        MapPointT* pMP = vpMapPoints[q];
        view[q] = pMP->mbTrackInView && !pMP->isBad();
        px[q] = pMP->mTrackProjX;
        py[q] = pMP->mTrackProjY;
        pxr[q] = pMP->mTrackProjXR;
        lvl[q] = pMP->mnTrackScaleLevel;
        vcos[q] = pMP->mTrackViewCos;
        nobs[q] = pMP->Observations();
        if (view[q]) {
            cv::Mat d = pMP->GetDescriptor();
            std::memcpy(&desc[32 * (size_t)q], d.ptr<uint8_t>(0), 32);
        }
    }
    for (int i = 0; i < F.N; ++i) cobs[i] = F.mvpMapPoints[i] ? F.mvpMapPoints[i]->Observations() : -1;
    coeb_localmap lm{nq, view.data(), px.data(), py.data(), pxr.data(), lvl.data(), vcos.data(), desc.data(),
                     nobs.data()};
    cv::Mat curDesc = F.mDescriptors.isContinuous() ? F.mDescriptors : F.mDescriptors.clone();
    coeb_curframe cur{F.N, reinterpret_cast<const coeb_keypoint*>(F.mvKeysUn.data()),
                      curDesc.empty() ? nullptr : curDesc.ptr<uint8_t>(0), F.mvuRight.data()};
    const coeb_camera cam = frame_camera(F);
    std::vector<int32_t> match((size_t)F.N);
    int nmatches = 0;
    const int rc = coeb_match_localmap(ctx, &cam, &cur, cobs.data(), &lm, th, mfNNratio, match.data(), &nmatches);
    if (rc != COEB_OK) throw std::runtime_error(coeb_last_error(ctx));
    for (int i = 0; i < F.N; ++i)
        if (match[i] >= 0) F.mvpMapPoints[i] = vpMapPoints[match[i]];
    return nmatches;
}

template <class FrameT, class KeyFrameT, class MapPointT>
inline int SearchByProjectionKeyFrame(FrameT& CurrentFrame, KeyFrameT* pKF, const std::set<MapPointT*>& sAlreadyFound,
                                      float th, int ORBdist, bool mbCheckOrientation, coeb_ctx* ctx = nullptr)
{
    if (!ctx) ctx = matcher_ctx(CurrentFrame.mnScaleLevels, CurrentFrame.mfScaleFactor);
    const std::vector<MapPointT*> vpMPs = pKF->GetMapPointMatches();
    const int nq = (int)vpMPs.size();
    std::vector<uint8_t> valid(nq), desc((size_t)nq * 32), has((size_t)CurrentFrame.N);
    std::vector<float> xw((size_t)nq * 3), maxd(nq), mind(nq), ang(nq);
    for (int i = 0; i < nq; ++i) {
        MapPointT* pMP = vpMPs[i];
        valid[i] = pMP && !pMP->isBad() && !sAlreadyFound.count(pMP);
        if (!valid[i]) continue;
        cv::Mat x3D = pMP->GetWorldPos();
        xw[3 * i + 0] = x3D.at<float>(0);
        xw[3 * i + 1] = x3D.at<float>(1);
        xw[3 * i + 2] = x3D.at<float>(2);
        cv::Mat d = pMP->GetDescriptor();
        std::memcpy(&desc[32 * (size_t)i], d.ptr<uint8_t>(0), 32);
        maxd[i] = pMP->GetMaxDistance();
        mind[i] = pMP->GetMinDistance();
        ang[i] = pKF->mvKeysUn[i].angle;
    }
    for (int i = 0; i < CurrentFrame.N; ++i) has[i] = CurrentFrame.mvpMapPoints[i] != nullptr;
    coeb_keyframe_points kf{nq, valid.data(), xw.data(), desc.data(), maxd.data(), mind.data(), ang.data()};
    cv::Mat curDesc = CurrentFrame.mDescriptors.isContinuous() ? CurrentFrame.mDescriptors
                                                               : CurrentFrame.mDescriptors.clone();
    coeb_curframe cur{CurrentFrame.N, reinterpret_cast<const coeb_keypoint*>(CurrentFrame.mvKeysUn.data()),
                      curDesc.empty() ? nullptr : curDesc.ptr<uint8_t>(0), nullptr};
    const coeb_camera cam = frame_camera(CurrentFrame);
    float T[16];
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 4; ++k) T[4 * r + k] = CurrentFrame.mTcw.template at<float>(r, k);
    std::vector<int32_t> match((size_t)CurrentFrame.N);
    int nmatches = 0;
    const int rc = coeb_match_keyframe(ctx, &cam, &cur, has.data(), &kf, T, th, ORBdist, mbCheckOrientation ? 1 : 0,
                                       match.data(), &nmatches);
    if (rc != COEB_OK) throw std::runtime_error(coeb_last_error(ctx));
    for (int i = 0; i < CurrentFrame.N; ++i)
        if (match[i] >= 0) CurrentFrame.mvpMapPoints[i] = vpMPs[match[i]];
    return nmatches;
}

}  // namespace coeb

#endif
