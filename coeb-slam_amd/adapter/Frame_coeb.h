/*
 * Frame_coeb.h -- MI355X body for Frame::ProcessMovingObject(const cv::Mat &imgray,
 * std::vector<std::vector<float>> &box) (include/Frame.h, src/Frame.cc:311-393).
 *
 * Included from the reference's src/Frame.cc; the member function body becomes
 *
 *     coeb::ProcessMovingObject(imGrayPre, imgray, T_M);
 *
 * (imGrayPre is the file-scope previous gray frame, Frame.cc:30; box is unused by the
 * reference body too).  What it does, in the reference's terms:
 *   - goodFeaturesToTrack(imGrayPre, 1000, 0.01, 8, Harris k 0.04), cornerSubPix(10x10, 20,
 *     0.03), calcOpticalFlowPyrLK(22x22, 5 levels, 20, 0.01) (:333-335);
 *   - the 3x3 SAD consistency check (edge 5, limit 2120) (:337-365);
 *   - findFundamentalMat(FM_RANSAC, 0.1, 0.99) and the epipolar distance > 1 test (:370-384);
 * all on the device (coeb_moving_object_points), T_M in the reference's order.  When
 * findFundamentalMat would return an empty Mat (the reference then reads F.at<double> of an
 * empty Mat: undefined) T_M is left empty.  The globals prepoint / nextpoint / F_* are only
 * read inside this function in the reference, so they are not maintained.
 * OpenCV is not in the build image: the device code follows OpenCV 3.4's algorithms in the
 * canonical forms of DESIGN.md s2.1 (parity with the OpenCV binary unpinned, s4.9).
 */
#ifndef COEB_ADAPTER_FRAME_H
#define COEB_ADAPTER_FRAME_H

#include <cstring>
#include <stdexcept>
#include <vector>

#include <opencv2/core/core.hpp>

#include "coeb_front.h"
#include "ORBmatcher_coeb.h"

namespace coeb
{

inline void ProcessMovingObject(const cv::Mat& imGrayPre, const cv::Mat& imgray, std::vector<cv::Point2f>& T_M,
                                coeb_ctx* ctx = nullptr)
{
    T_M.clear();
    if (!imGrayPre.data || !imgray.data) return;
    if (imGrayPre.type() != CV_8UC1 || imgray.type() != CV_8UC1 || imGrayPre.rows != imgray.rows ||
        imGrayPre.cols != imgray.cols)
        throw std::invalid_argument("coeb::ProcessMovingObject: two 8UC1 frames of one size expected");
    if (!ctx) ctx = matcher_ctx(8, 1.2f);
    const int w = imgray.cols, h = imgray.rows;
    // one pitch for both frames (the ABI takes a single stride)
    std::vector<uint8_t> a, b;
    const uint8_t* p0 = imGrayPre.data;
    const uint8_t* p1 = imgray.data;
    size_t stride = imgray.step[0];
    if (imGrayPre.step[0] != imgray.step[0]) {
        a.resize((size_t)w * h);
        b.resize((size_t)w * h);
        for (int y = 0; y < h; ++y) {
            std::memcpy(&a[(size_t)y * w], imGrayPre.data + (size_t)y * imGrayPre.step[0], (size_t)w);
            std::memcpy(&b[(size_t)y * w], imgray.data + (size_t)y * imgray.step[0], (size_t)w);
        }
        p0 = a.data();
        p1 = b.data();
        stride = (size_t)w;
    }
    std::vector<cv::Point2f> out(1024);
    int n = 0;
    if (coeb_moving_object_points(ctx, p0, p1, w, h, stride, reinterpret_cast<float*>(out.data()), (int)out.size(), &n,
                                  nullptr) != COEB_OK)
        throw std::runtime_error(coeb_last_error(ctx));
    if (n > 0) {
        out.resize((size_t)n);
        T_M.swap(out);
    }
}

}  // namespace coeb

#endif
