// The drop-in single-frame path as the reference's C++ Tracking thread drives it, without the
// Python binding in between: per frame coeb_extract (ORBextractor::operator(), called from the
// Frame constructor, Frame.cc:413-419), coeb_stereo_from_rgbd (Frame::ComputeStereoFromRGBD,
// Frame.cc:820-842) and coeb_match_lastframe (TrackWithMotionModel's SearchByProjection th 15,
// retried at 30 below 20 matches, Tracking.cc:947-958), frame i against frame i-1.  The LastFrame
// MapPoint arrays (world positions from frame i-1's depth, its descriptors) are Tracking state
// the adapter packs; they are built outside the timed calls.
//
// usage: single_frame_c <frames.u8> <W> <H> <N> [warm]   (N frames of W*H gray bytes; depth 2 m)
// prints one JSON line: median ms per frame and per call, median / min matches.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "coeb_front.h"

static double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv)
{
    if (argc < 5) {
        fprintf(stderr, "usage: %s frames.u8 W H N [warm]\n", argv[0]);
        return 2;
    }
    const int W = atoi(argv[2]), H = atoi(argv[3]), N = atoi(argv[4]), warm = argc > 5 ? atoi(argv[5]) : 5;
    std::vector<uint8_t> frames((size_t)N * W * H);
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(frames.data(), 1, frames.size(), f) != frames.size()) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    fclose(f);
    const float fx = 535.4f, fy = 539.2f, cx = 320.1f, cy = 247.6f, bf = 40.0f, z = 2.0f;
    std::vector<float> depth((size_t)W * H, z);
    coeb_orb_params p{1000, 1.2f, 8, 20, 7};
    coeb_ctx* ctx = coeb_create(&p, 0, W, H, 1);
    if (!ctx) {
        fprintf(stderr, "coeb_create: %s\n", coeb_last_error(nullptr));
        return 1;
    }
    const int cap = coeb_max_keypoints(ctx, W, H);
    const coeb_camera cam{fx, fy, cx, cy, bf, 0.f, (float)W, 0.f, (float)H};
    float Tc[16] = {1, 0, 0, 2.f * z / fx, 0, 1, 0, 1.f * z / fy, 0, 0, 1, 0, 0, 0, 0, 1};   // synth.motion_pose
    float Tl[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    struct Fr { std::vector<coeb_keypoint> k; std::vector<uint8_t> d; std::vector<float> ur, dep; int n = 0; };
    Fr cur, prev;
    for (Fr* x : {&cur, &prev}) {
        x->k.resize(cap); x->d.resize((size_t)cap * 32); x->ur.resize(cap); x->dep.resize(cap);
    }
    std::vector<uint8_t> has(cap), outl(cap, 0);
    std::vector<float> xw((size_t)cap * 3);
    std::vector<int32_t> nobs(cap, 2), match(cap);
    auto check = [&](int rc, const char* what) {
        if (rc != COEB_OK) {
            fprintf(stderr, "%s: %s\n", what, coeb_last_error(ctx));
            exit(1);
        }
    };
    auto extract = [&](Fr& x, int i) {
        check(coeb_extract(ctx, frames.data() + (size_t)i * W * H, W, H, W, nullptr, 0, nullptr, 0, nullptr, 0, x.k.data(),
                           x.d.data(), cap, &x.n), "coeb_extract");
    };
    auto stereo = [&](Fr& x) {
        check(coeb_stereo_from_rgbd(ctx, x.k.data(), x.n, depth.data(), W, H, W, bf, x.ur.data(), x.dep.data()),
              "coeb_stereo_from_rgbd");
    };
    extract(prev, 0);
    stereo(prev);
    std::vector<double> tot, te, ts, tm, nms;
    for (int i = 1; i < N; i++) {
        // LastFrame MapPoints of frame i-1 (untimed: Tracking state)
        for (int k = 0; k < prev.n; k++) {
            const float d = prev.dep[k];
            has[k] = d > 0;
            xw[3 * k] = (prev.k[k].x - cx) * d / fx;
            xw[3 * k + 1] = (prev.k[k].y - cy) * d / fy;
            xw[3 * k + 2] = d;
        }
        const coeb_lastframe last{prev.n, has.data(), outl.data(), xw.data(), prev.d.data(), nobs.data(), prev.k.data()};
        const double t0 = now_ms();
        extract(cur, i);
        const double t1 = now_ms();
        stereo(cur);
        const double t2 = now_ms();
        const coeb_curframe cf{cur.n, cur.k.data(), cur.d.data(), cur.ur.data()};
        int nm = 0;
        check(coeb_match_lastframe(ctx, &cam, &cf, &last, Tc, Tl, 15.f, 0, 1, match.data(), &nm), "coeb_match_lastframe");
        if (nm < 20) check(coeb_match_lastframe(ctx, &cam, &cf, &last, Tc, Tl, 30.f, 0, 1, match.data(), &nm),
                           "coeb_match_lastframe");
        const double t3 = now_ms();
        if (i > warm) {
            tot.push_back(t3 - t0); te.push_back(t1 - t0); ts.push_back(t2 - t1); tm.push_back(t3 - t2); nms.push_back(nm);
        }
        std::swap(cur, prev);
    }
    coeb_destroy(ctx);
    printf("{\"ms_per_frame\": %.4f, \"ms_extract\": %.4f, \"ms_stereo\": %.4f, \"ms_match\": %.4f, \"frames\": %zu, "
           "\"matches\": %d, \"min_matches\": %d}\n",
           median(tot), median(te), median(ts), median(tm), tot.size(), (int)median(nms),
           nms.empty() ? 0 : (int)*std::min_element(nms.begin(), nms.end()));
    return 0;
}
