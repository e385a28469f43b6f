/*
 * ORBextractor.h -- drop-in replacement of COEB-SLAM's include/ORBextractor.h backed by the
 * MI355X HIP front end (include/coeb_front.h).
 *
 * Same class name, namespace, constructor, operator() and accessors as the reference
 * (include/ORBextractor.h:44-128), so src/Frame.cc:413-419 (ExtractORB) and
 * src/Tracking.cc:115-120 compile unchanged.  Header-only; link libcoeb_front.so.
 *
 *   ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)    ORBextractor.h:50-51
 *   operator()(image, mask, img, imD, keypoints, descriptors, box, T_M,
 *              mask_result, blur_flag)                                     ORBextractor.h:73-75
 *   GetLevels / GetScaleFactor / GetScaleFactors / GetInverseScaleFactors /
 *   GetScaleSigmaSquares / GetInverseScaleSigmaSquares                     ORBextractor.h:77-99
 *
 * Behaviour kept from the reference: empty image -> return without touching the outputs
 * (:1096-1097); non-8UC1 -> assert (:1099); zero keypoints -> descriptors.release()
 * (:1296-1297); mask / img / imD / mask_result are accepted and unused (SURVEY.md s8a note).
 * Device contexts are pooled per (host thread, device, parameters) so Tracking's leak-and-recreate
 * of extractors on tracking failure (Tracking.cc:434-465) stays cheap; a context grows to the
 * largest image it has seen (no fixed size cap) and is freed when its thread exits.
 */
#ifndef COEB_ADAPTER_ORBEXTRACTOR_H
#define COEB_ADAPTER_ORBEXTRACTOR_H

#include <algorithm>
#include <cassert>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include <opencv2/core/core.hpp>
#include <opencv2/features2d/features2d.hpp>

#include "coeb_front.h"

namespace ORB_SLAM2
{

class ExtractorNode   // kept for source compatibility (unused by the GPU path)
{
public:
    ExtractorNode() : bNoMore(false) {}
    std::vector<cv::KeyPoint> vKeys;
    cv::Point2i UL, UR, BL, BR;
    std::list<ExtractorNode>::iterator lit;
    bool bNoMore;
};

namespace coeb_detail
{
// One context per (host thread, device, ORB parameters): coeb_ctx is not reentrant.  The pool
// is thread_local and destroys its contexts when the thread exits, so thread churn frees device
// memory.  A context is created for at least 1280 x 960 and re-created larger when an image
// exceeds it; extractors therefore look their context up per call instead of caching it.
struct CtxPool {
    struct Entry { coeb_ctx* ctx; int max_w, max_h; };
    std::map<std::tuple<int, int, float, int, int, int>, Entry> m;
    ~CtxPool()
    {
        for (auto& kv : m) coeb_destroy(kv.second.ctx);
    }
};

inline coeb_ctx* pooled_context(const coeb_orb_params& p, int device, int w, int h)
{
    thread_local CtxPool pool;
    const auto key = std::make_tuple(device, p.nfeatures, p.scale_factor, p.nlevels, p.ini_th_fast, p.min_th_fast);
    auto it = pool.m.find(key);
    if (it != pool.m.end() && w <= it->second.max_w && h <= it->second.max_h) return it->second.ctx;
    int mw = std::max(w, 1280), mh = std::max(h, 960);
    if (it != pool.m.end()) {               // grow: keep the larger of the old and new bounds
        mw = std::max(mw, it->second.max_w);
        mh = std::max(mh, it->second.max_h);
        coeb_destroy(it->second.ctx);
        pool.m.erase(it);
    }
    if (coeb_abi_version() != COEB_ABI_VERSION)      // header and loaded library must agree
        throw std::runtime_error("libcoeb_front ABI " + std::to_string(coeb_abi_version()) + ", header " +
                                 std::to_string(COEB_ABI_VERSION));
    coeb_ctx* c = coeb_create(&p, device, mw, mh, 1);
    if (!c) throw std::runtime_error(std::string("coeb_create: ") + coeb_last_error(nullptr));
    pool.m[key] = CtxPool::Entry{c, mw, mh};
    return c;
}
}  // namespace coeb_detail

class ORBextractor
{
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
        : nfeatures(nfeatures), scaleFactor(scaleFactor), nlevels(nlevels), iniThFAST(iniThFAST),
          minThFAST(minThFAST)
    {
        params_.nfeatures = nfeatures;
        params_.scale_factor = scaleFactor;
        params_.nlevels = nlevels;
        params_.ini_th_fast = iniThFAST;
        params_.min_th_fast = minThFAST;
        coeb_ctx* ctx = coeb_detail::pooled_context(params_, device(), 0, 0);
        coeb_orb_tables t;
        if (coeb_orb_tables_get(ctx, &t) != COEB_OK) throw std::runtime_error(coeb_last_error(ctx));
        mvScaleFactor.assign(t.scale, t.scale + nlevels);
        mvInvScaleFactor.assign(t.inv_scale, t.inv_scale + nlevels);
        mvLevelSigma2.assign(t.sigma2, t.sigma2 + nlevels);
        mvInvLevelSigma2.assign(t.inv_sigma2, t.inv_sigma2 + nlevels);
        mnFeaturesPerLevel.assign(t.features_per_level, t.features_per_level + nlevels);
        umax.assign(t.umax, t.umax + 16);
        mvImagePyramid.resize(nlevels);
    }

    ~ORBextractor() {}

    void operator()(cv::InputArray _image, cv::InputArray /*mask*/, const cv::Mat& /*img*/, const cv::Mat& /*imD*/,
                    std::vector<cv::KeyPoint>& _keypoints, cv::OutputArray _descriptors,
                    std::vector<std::vector<float>>& box, std::vector<cv::Point2f> T_M, cv::Mat& /*mask_result*/,
                    std::vector<int> blur_flag)
    {
        if (_image.empty()) return;
        cv::Mat image = _image.getMat();
        assert(image.type() == CV_8UC1);
        std::vector<coeb_box> boxes;
        for (const auto& b : box) boxes.push_back(coeb_box{b[0], b[1], b[2], b[3]});
        std::vector<float> tm;
        for (const auto& p : T_M) { tm.push_back(p.x); tm.push_back(p.y); }
        coeb_ctx* ctx_ = coeb_detail::pooled_context(params_, device(), image.cols, image.rows);
        const int cap = coeb_max_keypoints(ctx_, image.cols, image.rows);
        if (cap < 0) throw std::runtime_error(coeb_last_error(ctx_));
        std::vector<coeb_keypoint> kps((size_t)cap);
        cv::Mat desc((int)cap, 32, CV_8U);
        int n = 0;
        const int rc = coeb_extract(ctx_, image.data, image.cols, image.rows, image.step[0],
                                    boxes.empty() ? nullptr : boxes.data(), (int)boxes.size(),
                                    tm.empty() ? nullptr : tm.data(), (int)T_M.size(),
                                    blur_flag.empty() ? nullptr : blur_flag.data(), (int)blur_flag.size(),
                                    kps.data(), desc.data, cap, &n);
        if (rc != COEB_OK) throw std::runtime_error(coeb_last_error(ctx_));
        _keypoints.resize((size_t)n);
        static_assert(sizeof(coeb_keypoint) == sizeof(cv::KeyPoint), "coeb_keypoint must mirror cv::KeyPoint");
        // cv::KeyPoint is trivially copyable and layout-identical to coeb_keypoint (static_assert above)
        if (n) std::memcpy(static_cast<void*>(&_keypoints[0]), kps.data(), sizeof(coeb_keypoint) * (size_t)n);
        if (n == 0) {
            _descriptors.release();
        } else {
            _descriptors.create(n, 32, CV_8U);
            desc.rowRange(0, n).copyTo(_descriptors.getMat());
        }
    }

    int inline GetLevels() { return nlevels; }
    float inline GetScaleFactor() { return (float)scaleFactor; }
    std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
    std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
    std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
    std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

    std::vector<cv::Mat> mvImagePyramid;   // RGB-D never reads it (Frame.cc:651,741,758 are stereo)

protected:
    static int device()
    {
        const char* e = std::getenv("COEB_DEVICE");
        return e ? std::atoi(e) : 0;
    }
    int nfeatures;
    double scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;
    std::vector<int> mnFeaturesPerLevel;
    std::vector<int> umax;
    std::vector<float> mvScaleFactor;
    std::vector<float> mvInvScaleFactor;
    std::vector<float> mvLevelSigma2;
    std::vector<float> mvInvLevelSigma2;
    coeb_orb_params params_{};
};

}  // namespace ORB_SLAM2

#endif
