/*
 * ORBmatcher_coeb.h -- MI355X body for ORBmatcher::SearchByProjection(Frame&, const Frame&,
 * float th, bool bMono) (include/ORBmatcher.h:52, src/ORBmatcher.cc:1329-1471).
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
 */
#ifndef COEB_ADAPTER_ORBMATCHER_H
#define COEB_ADAPTER_ORBMATCHER_H

#include <cstring>
#include <stdexcept>
#include <vector>

#include <opencv2/core/core.hpp>

#include "coeb_front.h"

namespace coeb
{

template <class FrameT>
inline int SearchByProjectionLastFrame(FrameT& CurrentFrame, const FrameT& LastFrame, float th, bool bMono,
                                       float /*mfNNratio*/, bool mbCheckOrientation, coeb_ctx* ctx = nullptr)
{
    static thread_local coeb_ctx* tl_ctx = nullptr;
    if (!ctx) {
        if (!tl_ctx) {
            coeb_orb_params p{1000, 1.2f, 8, 20, 7};   // matcher-only context: extractor tables unused
            tl_ctx = coeb_create(&p, 0, 640, 480, 1);
            if (!tl_ctx) throw std::runtime_error(coeb_last_error(nullptr));
        }
        ctx = tl_ctx;
    }
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
    coeb_camera cam{FrameT::fx, FrameT::fy, FrameT::cx, FrameT::cy, CurrentFrame.mbf,
                    FrameT::mnMinX, FrameT::mnMaxX, FrameT::mnMinY, FrameT::mnMaxY};
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

}  // namespace coeb

#endif
