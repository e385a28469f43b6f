// coeb_frame.hip -- per-frame pre-filter kernels around the extractor:
//   Frame blur flag: crop -> Laplacian(CV_16U, ksize 1) -> mean < 4.2   src/Frame.cc:171-202, 905-913
//   Tracking::GrabImageRGBD: cvtColor RGB2GRAY (8U, 14-bit fixed point), depth 16U -> 32F x scale
//                                                                       src/Tracking.cc:207-228
#include <hip/hip_runtime.h>

#include <cstring>

#include <string>
#include <vector>

#include "../../include/coeb_front.h"
#include "coeb_internal.hpp"

namespace {

__device__ __forceinline__ int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - p - 2;
    return p;
}

// one workgroup per box: Laplacian [0 1 0; 1 -4 1; 0 1 0] on the cloned crop (REFLECT_101 at
// the crop edge), negatives saturate to 0 (saturate_cast<ushort>), exact integer sum,
// cv::mean = sum * (1./count).
// box_frame (batch form): frame of box bi in a packed batch of frames fstride bytes apart; boxes
// of frame 0 get flag 0 (the RGB-D Frame constructor's first frame, Frame.cc:205-208).
__global__ __launch_bounds__(256) void k_blur_flags(const uint8_t* __restrict__ img, int W, int H, int stride,
                                                    const float* __restrict__ boxes, int* __restrict__ out,
                                                    double* __restrict__ mean_out, const int* __restrict__ box_frame,
                                                    int64_t fstride)
{
    __shared__ unsigned long long s_part[4];
    const int bi = blockIdx.x;
    if (box_frame) {
        const int f = box_frame[bi];
        if (f == 0) {
            if (threadIdx.x == 0) { out[bi] = 0; if (mean_out) mean_out[bi] = -1.0; }
            return;
        }
        img += (int64_t)f * fstride;
    }
    const float x0f = boxes[4 * bi], y0f = boxes[4 * bi + 1], x1f = boxes[4 * bi + 2], y1f = boxes[4 * bi + 3];
    const int rx = (int)x0f, ry = (int)y0f, rw = (int)(x1f - x0f), rh = (int)(y1f - y0f);
    if (rx < 0 || ry < 0 || rw <= 0 || rh <= 0 || rx + rw > W || ry + rh > H) {
        if (threadIdx.x == 0) { out[bi] = 0; if (mean_out) mean_out[bi] = -1.0; }
        return;
    }
    const uint8_t* c = img + (int64_t)ry * stride + rx;
    unsigned long long acc = 0;
    for (int i = threadIdx.x; i < rw * rh; i += 256) {
        const int y = i / rw, x = i - y * rw;
        const int ym = reflect101(y - 1, rh), yp = reflect101(y + 1, rh);
        const int xm = reflect101(x - 1, rw), xp = reflect101(x + 1, rw);
        const int lap = c[(int64_t)ym * stride + x] + c[(int64_t)yp * stride + x] + c[(int64_t)y * stride + xm] +
                        c[(int64_t)y * stride + xp] - 4 * c[(int64_t)y * stride + x];
        acc += lap > 0 ? (unsigned)lap : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (__lane_id() == 0) s_part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long S = s_part[0] + s_part[1] + s_part[2] + s_part[3];
        const double mean = (double)S * (1. / (double)((long long)rw * rh));
        out[bi] = mean < 4.2 ? 1 : 0;
        if (mean_out) mean_out[bi] = mean;
    }
}

__global__ __launch_bounds__(256) void k_rgbd(const uint8_t* __restrict__ img, int istride, int channels, int rgb_order,
                                              const uint8_t* __restrict__ dsrc, int dstride, int dtype, float dscale,
                                              int dcopy, int W, int H, uint8_t* __restrict__ gray,
                                              float* __restrict__ depth)
{
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= W || y >= H) return;
    if (img) {
        const uint8_t* s = img + (int64_t)y * istride + channels * x;
        uint8_t g = s[0];
        if (channels >= 3) {                 // cvtColor RGB2GRAY / RGBA2GRAY (alpha ignored), 14-bit fixed point
            const int R2Y = 4899, G2Y = 9617, B2Y = 1868;
            const int v = rgb_order ? (s[0] * R2Y + s[1] * G2Y + s[2] * B2Y) : (s[0] * B2Y + s[1] * G2Y + s[2] * R2Y);
            g = (uint8_t)((v + (1 << 13)) >> 14);
        }
        gray[(int64_t)y * W + x] = g;
    }
    if (dsrc) {
        const uint8_t* row = dsrc + (int64_t)y * dstride;
        float v;
        if (dtype == COEB_DEPTH_U16) v = (float)reinterpret_cast<const uint16_t*>(row)[x] * dscale;
        else {
            v = reinterpret_cast<const float*>(row)[x];
            if (!dcopy) v = v * dscale;      // convertTo(CV_32F, scale): float product
        }
        depth[(int64_t)y * W + x] = v;
    }
}

// The same conversions over a packed device batch (frame f of the batch at f * W*H pixels), four
// pixels per thread: one 4/12/16-byte image load, one 8/16-byte depth load, a 4-byte gray and a
// 16-byte depth store (W % 4 == 0; HBM-bound: 3 + 2 bytes in, 1 + 4 out per pixel for RGB + 16U).
__global__ __launch_bounds__(256) void k_rgbd_batch(const uint8_t* __restrict__ img, int channels, int rgb_order,
                                                    const uint8_t* __restrict__ dsrc, int dtype, float dscale, int dcopy,
                                                    int64_t npix, uint8_t* __restrict__ gray, float* __restrict__ depth)
{
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (4 * q >= npix) return;
    const int64_t p0 = (int64_t)blockIdx.y * npix + 4 * q;
    if (img) {
        uint32_t w[4];
        const uint32_t* s = reinterpret_cast<const uint32_t*>(img + p0 * channels);
        for (int k = 0; k < channels; k++) w[k] = s[k];
        uint32_t out = 0;
        for (int k = 0; k < 4; k++) {
            uint32_t g;
            if (channels == 1) {
                g = (w[0] >> (8 * k)) & 0xffu;
            } else {
                const int b0 = k * channels;                       // byte offset of pixel k
                auto byte = [&](int b) { return (int)((w[b >> 2] >> (8 * (b & 3))) & 0xffu); };
                const int c0 = byte(b0), c1 = byte(b0 + 1), c2 = byte(b0 + 2);
                const int R2Y = 4899, G2Y = 9617, B2Y = 1868;
                const int v = rgb_order ? (c0 * R2Y + c1 * G2Y + c2 * B2Y) : (c0 * B2Y + c1 * G2Y + c2 * R2Y);
                g = (uint32_t)((v + (1 << 13)) >> 14);
            }
            out |= g << (8 * k);
        }
        reinterpret_cast<uint32_t*>(gray + p0)[0] = out;
    }
    if (dsrc) {
        float v[4];
        if (dtype == COEB_DEPTH_U16) {
            const uint2 r = *reinterpret_cast<const uint2*>(dsrc + 2 * p0);
            v[0] = (float)(r.x & 0xffffu) * dscale; v[1] = (float)(r.x >> 16) * dscale;
            v[2] = (float)(r.y & 0xffffu) * dscale; v[3] = (float)(r.y >> 16) * dscale;
        } else {
            const float4 r = *reinterpret_cast<const float4*>(dsrc + 4 * p0);
            v[0] = r.x; v[1] = r.y; v[2] = r.z; v[3] = r.w;
            if (!dcopy) for (int k = 0; k < 4; k++) v[k] = v[k] * dscale;
        }
        reinterpret_cast<float4*>(depth + p0)[0] = make_float4(v[0], v[1], v[2], v[3]);
    }
}

// The same conversion for batches whose frame size is a multiple of 16 pixels (channel count a
// template parameter, so every byte select is static): a 256-thread block converts 4096 pixels as
// four passes of 4 pixels per thread, and in every pass the lanes' accesses are contiguous -- 12 B
// (3 channels) / 16 B / 4 B of image, 8 B of 16U depth in, 4 B of gray and 16 B of float depth
// out per lane, so one instruction covers 768 B / 1 KB / 256 B / 512 B / 256 B / 1 KB with no gaps.
// (A 16-pixels-per-lane form issued 16-byte loads 48 B apart: 0.79 ms per 513 frames.)
struct U3 { uint32_t x, y, z; };
template <int CH>
__global__ __launch_bounds__(256) void k_rgbd_batch16(const uint8_t* __restrict__ img, int rgb_order,
                                                      const uint8_t* __restrict__ dsrc, int dtype, float dscale,
                                                      int dcopy, int64_t npix, uint8_t* __restrict__ gray,
                                                      float* __restrict__ depth)
{
    const int64_t b0 = (int64_t)blockIdx.x * 4096;
    if (b0 >= npix) return;
    const int64_t fbase = (int64_t)blockIdx.y * npix;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const int64_t pix = b0 + 4 * (g * 256 + threadIdx.x);          // first of this lane's 4 pixels
        if (pix >= npix) break;
        const int64_t p0 = fbase + pix;
        if (CH > 0 && img) {
            uint32_t w[CH > 0 ? CH : 1];
            if constexpr (CH == 1) {
                w[0] = *reinterpret_cast<const uint32_t*>(img + p0);
            } else if constexpr (CH == 3) {
                const U3 v = *reinterpret_cast<const U3*>(img + p0 * 3);
                w[0] = v.x; w[1] = v.y; w[2] = v.z;
            } else {
                const uint4 v = *reinterpret_cast<const uint4*>(img + p0 * 4);
                w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
            }
            uint32_t out = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t gv;
                if (CH == 1) {
                    gv = (w[0] >> (8 * k)) & 0xffu;
                } else {
                    auto byte = [&](int b) { return (int)((w[b >> 2] >> (8 * (b & 3))) & 0xffu); };
                    const int c0 = byte(k * CH), c1 = byte(k * CH + 1), c2 = byte(k * CH + 2);
                    const int R2Y = 4899, G2Y = 9617, B2Y = 1868;
                    const int v = rgb_order ? (c0 * R2Y + c1 * G2Y + c2 * B2Y) : (c0 * B2Y + c1 * G2Y + c2 * R2Y);
                    gv = (uint32_t)((v + (1 << 13)) >> 14);
                }
                out |= gv << (8 * k);
            }
            *reinterpret_cast<uint32_t*>(gray + p0) = out;
        }
        if (dsrc) {
            float v[4];
            if (dtype == COEB_DEPTH_U16) {
                const uint2 r = *reinterpret_cast<const uint2*>(dsrc + 2 * p0);
                v[0] = (float)(r.x & 0xffffu) * dscale; v[1] = (float)(r.x >> 16) * dscale;
                v[2] = (float)(r.y & 0xffffu) * dscale; v[3] = (float)(r.y >> 16) * dscale;
            } else {
                const float4 r = *reinterpret_cast<const float4*>(dsrc + 4 * p0);
                v[0] = r.x; v[1] = r.y; v[2] = r.z; v[3] = r.w;
                if (!dcopy) for (int k = 0; k < 4; k++) v[k] = v[k] * dscale;
            }
            *reinterpret_cast<float4*>(depth + p0) = make_float4(v[0], v[1], v[2], v[3]);
        }
    }
}

// Frame::UndistortKeyPoints (Frame.cc:579-609): cv::undistortPoints(.., mK, mDistCoef, Mat(), mK)
// of OpenCV 3.4 (cvUndistortPointsInternal, 5 fixed iterations), one thread per keypoint, in
// double with the oracle's operation order.  k = (k1, k2, p1, p2, k3); the remaining rational /
// thin-prism terms of the 14-coefficient model are zero and kept so the sums match.
struct KpRec { float x, y, size, angle, response; int octave, class_id; };
struct DistK { double k[12]; double fx, fy, cx, cy; };

__global__ __launch_bounds__(256) void k_undistort(const KpRec* __restrict__ in, int n, DistK d, KpRec* __restrict__ out)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    KpRec kp = in[i];
    const double* k = d.k;
    const double ifx = 1. / d.fx, ify = 1. / d.fy;
    double x = ((double)kp.x - d.cx) * ifx, y = ((double)kp.y - d.cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = ((((2 * k[2]) * x) * y + k[3] * (r2 + (2 * x) * x)) + k[8] * r2) + (k[9] * r2) * r2;
        const double deltaY = ((k[2] * (r2 + (2 * y) * y) + ((2 * k[3]) * x) * y) + k[10] * r2) + (k[11] * r2) * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    kp.x = (float)(d.fx * x + d.cx);
    kp.y = (float)(d.fy * y + d.cy);
    out[i] = kp;
}

}  // namespace

// host entry points (C-ABI); context internals are reached through small accessors in
// coeb_capi.hip
extern "C" int coeb_internal_stream(coeb_ctx* c, hipStream_t* s, int* device);
extern "C" int coeb_internal_scratch(coeb_ctx* c, const char* name, size_t bytes, void** p);
extern "C" int coeb_internal_error(coeb_ctx* c, int code, const char* msg);
extern "C" ProfileHook* coeb_internal_prof(coeb_ctx* c);

#define FR_TRY(c, expr)                                                                         \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess) return coeb_internal_error((c), COEB_EDEVICE, hipGetErrorString(_e)); \
    } while (0)

// box -> frame map of a batch from its box offsets (frame f owns boxes [box_off[f], box_off[f+1]))
__global__ __launch_bounds__(256) void k_box_frame(const int* __restrict__ box_off, int F, int* __restrict__ box_frame)
{
    const int f = blockIdx.x * 256 + threadIdx.x;
    if (f >= F) return;
    for (int i = box_off[f]; i < box_off[f + 1]; i++) box_frame[i] = f;
}

// The blur flags of every box of a device-resident batch (packed W x H frames): frame f's boxes
// are [d_box_off[f], d_box_off[f+1]) of d_boxes (device arrays); d_box_frame is scratch for nbox
// ints; frame 0's boxes get 0.  Enqueued on stream s, nothing staged from the host.
extern "C" int coeb_internal_blur_flags_batch(coeb_ctx* c, const uint8_t* d_gray, int W, int H, const float* d_boxes,
                                              const int* d_box_off, int F, int* d_box_frame, int nbox, int* d_out,
                                              hipStream_t s)
{
    if (nbox <= 0) return COEB_OK;
    hipLaunchKernelGGL(k_box_frame, dim3((F + 255) / 256), dim3(256), 0, s, d_box_off, F, d_box_frame);
    ProfileHook* prof = coeb_internal_prof(c);
    prof_begin(prof, "k_blur_flags", s);
    hipLaunchKernelGGL(k_blur_flags, dim3(nbox), dim3(256), 0, s, d_gray, W, H, W, d_boxes, d_out, (double*)nullptr,
                       (const int*)d_box_frame, (int64_t)W * H);
    prof_end(prof, s);
    return hipGetLastError() == hipSuccess ? COEB_OK : COEB_EDEVICE;
}

extern "C" int coeb_blur_flags(coeb_ctx* c, const uint8_t* gray, int W, int H, size_t stride, const coeb_box* boxes,
                               int nbox, int32_t* flags_out)
{
    if (!c || nbox < 0 || (nbox > 0 && (!gray || !boxes || !flags_out)) || stride < (size_t)W)
        return coeb_internal_error(c, COEB_EINVAL, "coeb_blur_flags: invalid arguments");
    if (nbox == 0) return COEB_OK;
    hipStream_t s;
    int dev;
    if (coeb_internal_stream(c, &s, &dev)) return COEB_EINVAL;
    (void)hipSetDevice(dev);
    void *dimg, *dbox, *dout;
    int rc;
    if ((rc = coeb_internal_scratch(c, "bf_img", (size_t)W * H, &dimg)) ||
        (rc = coeb_internal_scratch(c, "bf_box", (size_t)nbox * 16, &dbox)) ||
        (rc = coeb_internal_scratch(c, "bf_out", (size_t)nbox * 4, &dout)))
        return rc;
    FR_TRY(c, hipMemcpy2DAsync(dimg, W, gray, stride, W, H, hipMemcpyHostToDevice, s));
    FR_TRY(c, hipMemcpyAsync(dbox, boxes, (size_t)nbox * 16, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_blur_flags, dim3(nbox), dim3(256), 0, s, (const uint8_t*)dimg, W, H, W, (const float*)dbox,
                       (int*)dout, (double*)nullptr, (const int*)nullptr, (int64_t)0);
    FR_TRY(c, hipGetLastError());
    FR_TRY(c, hipMemcpyAsync(flags_out, dout, (size_t)nbox * 4, hipMemcpyDeviceToHost, s));
    FR_TRY(c, hipStreamSynchronize(s));
    return COEB_OK;
}

extern "C" int coeb_rgbd_preprocess(coeb_ctx* c, const uint8_t* img, size_t img_stride, int channels, int rgb_order,
                                    const void* depth, size_t depth_stride, int depth_type, float depth_scale, int W,
                                    int H, uint8_t* gray_out, float* depth_out)
{
    const size_t dbytes = depth_type == COEB_DEPTH_F32 ? 4 : 2;
    if (!c || W <= 0 || H <= 0 ||
        (img && (!gray_out || (channels != 1 && channels != 3 && channels != 4) || img_stride < (size_t)channels * W)) ||
        (depth && (!depth_out || (depth_type != COEB_DEPTH_U16 && depth_type != COEB_DEPTH_F32) ||
                   depth_stride < dbytes * W || depth_stride % dbytes)))
        return coeb_internal_error(c, COEB_EINVAL, "coeb_rgbd_preprocess: invalid arguments");
    hipStream_t s;
    int dev;
    if (coeb_internal_stream(c, &s, &dev)) return COEB_EINVAL;
    (void)hipSetDevice(dev);
    void *dimg = nullptr, *dgray = nullptr, *dd = nullptr, *ddep = nullptr;
    int rc;
    const size_t rowb = (size_t)channels * W;
    if (img) {
        if ((rc = coeb_internal_scratch(c, "pp_img", rowb * H, &dimg)) ||
            (rc = coeb_internal_scratch(c, "pp_gray", (size_t)W * H, &dgray)))
            return rc;
        FR_TRY(c, hipMemcpy2DAsync(dimg, rowb, img, img_stride, rowb, H, hipMemcpyHostToDevice, s));
    }
    // Tracking.cc:227: convertTo unless the map is already 32F and mDepthMapFactor == 1
    const int dcopy = depth_type == COEB_DEPTH_F32 && !(fabsf(depth_scale - 1.0f) > 1e-5f);
    if (depth) {
        if ((rc = coeb_internal_scratch(c, "pp_dsrc", dbytes * W * H, &dd)) ||
            (rc = coeb_internal_scratch(c, "pp_dep", (size_t)W * H * 4, &ddep)))
            return rc;
        FR_TRY(c, hipMemcpy2DAsync(dd, dbytes * W, depth, depth_stride, dbytes * W, H, hipMemcpyHostToDevice, s));
    }
    hipLaunchKernelGGL(k_rgbd, dim3((W + 63) / 64, (H + 3) / 4), dim3(256), 0, s, (const uint8_t*)dimg, (int)rowb, channels,
                       rgb_order, (const uint8_t*)dd, (int)(dbytes * W), depth_type, depth_scale, dcopy, W, H,
                       (uint8_t*)dgray, (float*)ddep);
    FR_TRY(c, hipGetLastError());
    if (img) FR_TRY(c, hipMemcpyAsync(gray_out, dgray, (size_t)W * H, hipMemcpyDeviceToHost, s));
    if (depth) FR_TRY(c, hipMemcpyAsync(depth_out, ddep, (size_t)W * H * 4, hipMemcpyDeviceToHost, s));
    FR_TRY(c, hipStreamSynchronize(s));
    return COEB_OK;
}

extern "C" int coeb_rgbd_preprocess_batch_device(coeb_ctx* c, const uint8_t* d_img, int channels, int rgb_order,
                                                 const void* d_depth, int depth_type, float depth_scale, int F, int W,
                                                 int H, uint8_t* d_gray, float* d_depth_out)
{
    if (!c || F <= 0 || W <= 0 || H <= 0 || (!d_img && !d_depth) ||
        (d_img && (!d_gray || (channels != 1 && channels != 3 && channels != 4))) ||
        (d_depth && (!d_depth_out || (depth_type != COEB_DEPTH_U16 && depth_type != COEB_DEPTH_F32))))
        return coeb_internal_error(c, COEB_EINVAL, "coeb_rgbd_preprocess_batch_device: invalid arguments");
    if (W % 4) return coeb_internal_error(c, COEB_EINVAL, "coeb_rgbd_preprocess_batch_device: width must be a multiple of 4");
    if ((d_img && (reinterpret_cast<uintptr_t>(d_img) | reinterpret_cast<uintptr_t>(d_gray)) % 4) ||
        (d_depth && (reinterpret_cast<uintptr_t>(d_depth) | reinterpret_cast<uintptr_t>(d_depth_out)) % 16))
        return coeb_internal_error(c, COEB_EINVAL, "coeb_rgbd_preprocess_batch_device: misaligned device buffers");
    hipStream_t s;
    int dev;
    if (coeb_internal_stream(c, &s, &dev)) return COEB_EINVAL;
    (void)hipSetDevice(dev);
    const int dcopy = depth_type == COEB_DEPTH_F32 && !(fabsf(depth_scale - 1.0f) > 1e-5f);   // Tracking.cc:227
    const int64_t npix = (int64_t)W * H;
    ProfileHook* prof = coeb_internal_prof(c);
    const bool wide = npix % 16 == 0 &&
                      ((reinterpret_cast<uintptr_t>(d_img) | reinterpret_cast<uintptr_t>(d_gray) |
                        reinterpret_cast<uintptr_t>(d_depth) | reinterpret_cast<uintptr_t>(d_depth_out)) & 15) == 0;
    prof_begin(prof, "k_rgbd_batch", s);
    if (wide) {
        const dim3 grid((unsigned)((npix + 4095) / 4096), F);
        const uint8_t* dd = (const uint8_t*)d_depth;
        if (!d_img) hipLaunchKernelGGL(k_rgbd_batch16<0>, grid, dim3(256), 0, s, d_img, rgb_order, dd, depth_type, depth_scale, dcopy, npix, d_gray, d_depth_out);
        else if (channels == 1) hipLaunchKernelGGL(k_rgbd_batch16<1>, grid, dim3(256), 0, s, d_img, rgb_order, dd, depth_type, depth_scale, dcopy, npix, d_gray, d_depth_out);
        else if (channels == 3) hipLaunchKernelGGL(k_rgbd_batch16<3>, grid, dim3(256), 0, s, d_img, rgb_order, dd, depth_type, depth_scale, dcopy, npix, d_gray, d_depth_out);
        else hipLaunchKernelGGL(k_rgbd_batch16<4>, grid, dim3(256), 0, s, d_img, rgb_order, dd, depth_type, depth_scale, dcopy, npix, d_gray, d_depth_out);
    } else {
        hipLaunchKernelGGL(k_rgbd_batch, dim3((unsigned)((npix / 4 + 255) / 256), F), dim3(256), 0, s, d_img, channels,
                           rgb_order, (const uint8_t*)d_depth, depth_type, depth_scale, dcopy, npix, d_gray, d_depth_out);
    }
    prof_end(prof, s);
    FR_TRY(c, hipGetLastError());
    return COEB_OK;
}

extern "C" int coeb_undistort_keypoints(coeb_ctx* c, const coeb_camera* cam, const float dist[5], const coeb_keypoint* kps,
                                        int n, coeb_keypoint* out)
{
    if (!c || !cam || !dist || n < 0 || (n > 0 && (!kps || !out)))
        return coeb_internal_error(c, COEB_EINVAL, "coeb_undistort_keypoints: invalid arguments");
    if (n == 0) return COEB_OK;
    if (dist[0] == 0.0f) {                                           // Frame.cc:581-585
        if (out != kps) memmove(out, kps, (size_t)n * sizeof(coeb_keypoint));
        return COEB_OK;
    }
    hipStream_t s;
    int dev;
    if (coeb_internal_stream(c, &s, &dev)) return COEB_EINVAL;
    (void)hipSetDevice(dev);
    void *din, *dout;
    int rc;
    if ((rc = coeb_internal_scratch(c, "ud_in", (size_t)n * sizeof(coeb_keypoint), &din)) ||
        (rc = coeb_internal_scratch(c, "ud_out", (size_t)n * sizeof(coeb_keypoint), &dout)))
        return rc;
    DistK d;
    for (int q = 0; q < 12; q++) d.k[q] = q < 5 ? (double)dist[q] : 0.0;
    d.fx = cam->fx; d.fy = cam->fy; d.cx = cam->cx; d.cy = cam->cy;
    FR_TRY(c, hipMemcpyAsync(din, kps, (size_t)n * sizeof(coeb_keypoint), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, s, (const KpRec*)din, n, d, (KpRec*)dout);
    FR_TRY(c, hipGetLastError());
    FR_TRY(c, hipMemcpyAsync(out, dout, (size_t)n * sizeof(coeb_keypoint), hipMemcpyDeviceToHost, s));
    FR_TRY(c, hipStreamSynchronize(s));
    return COEB_OK;
}

// yolov5_ros_msgs/BoundingBox int64 xmin, ymin, xmax, ymax -> the float boxes GrabRGBD builds
// (ros_rgbd.cc:106-115: push_back of int64 into std::vector<float>, i.e. static_cast<float>)
extern "C" int coeb_boxes_from_int64(const int64_t* xyxy, int nbox, coeb_box* out)
{
    if (nbox < 0 || (nbox > 0 && (!xyxy || !out))) return COEB_EINVAL;
    for (int i = 0; i < nbox; i++) {
        out[i].xmin = (float)xyxy[4 * i + 0];
        out[i].ymin = (float)xyxy[4 * i + 1];
        out[i].xmax = (float)xyxy[4 * i + 2];
        out[i].ymax = (float)xyxy[4 * i + 3];
    }
    return COEB_OK;
}
