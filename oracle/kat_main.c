/* Sanitizer run of the oracle (test infrastructure): `make -C oracle asan` builds this driver and
 * orb_oracle.c with AddressSanitizer + UndefinedBehaviorSanitizer (no recovery) and runs every
 * public entry point once on synthetic TUM-like frames, checking the properties that need no
 * reference run: counts and coordinates in range, determinism, injective matches, a recovered
 * pose, T_M on the moving object.  Exit status 0 = clean. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

#define W 640
#define H 480
#define CHECK(c)                                                             \
    do {                                                                     \
        if (!(c)) {                                                          \
            fprintf(stderr, "kat_main: check failed at %d: %s\n", __LINE__, #c); \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

static uint32_t rng = 12345u;
static uint32_t next(void) { rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5; return rng; }

/* rectangles on a torus canvas, shifted by (dx, dy), plus noise in [-6, 6] */
static void make_frame(uint8_t* img, const int16_t* canvas, int dx, int dy, uint32_t seed)
{
    uint32_t s = seed;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            s ^= s << 13; s ^= s >> 17; s ^= s << 5;
            int v = canvas[((y - dy + H) % H) * W + (x - dx + W) % W] + (int)(s % 13) - 6;
            img[y * W + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
}

int main(void)
{
    static int16_t canvas[W * H];
    for (int i = 0; i < W * H; i++) canvas[i] = 120;
    for (int r = 0; r < 60; r++) {
        const int x0 = next() % W, y0 = next() % H, rw = 16 + next() % 150, rh = 16 + next() % 110, v = next() % 256;
        for (int y = 0; y < rh; y++)
            for (int x = 0; x < rw; x++) canvas[((y0 + y) % H) * W + (x0 + x) % W] = (int16_t)v;
    }
    static uint8_t f0[W * H], f1[W * H];
    make_frame(f0, canvas, 0, 0, 7u);
    make_frame(f1, canvas, 2, 1, 8u);

    oc_params p;
    CHECK(oc_init(&p, 1000, 1.2f, 8, 20, 7) == 0);
    const int cap = 2048;
    oc_kp* k0 = calloc(cap, sizeof(oc_kp));
    oc_kp* k1 = calloc(cap, sizeof(oc_kp));
    oc_kp* k2 = calloc(cap, sizeof(oc_kp));
    uint8_t* d0 = calloc((size_t)cap, 32);
    uint8_t* d1 = calloc((size_t)cap, 32);
    uint8_t* d2 = calloc((size_t)cap, 32);
    int n0 = 0, n1 = 0, n2 = 0;
    oc_debug dbg;
    memset(&dbg, 0, sizeof(dbg));
    CHECK(oc_extract(&p, f0, W, H, W, NULL, 0, NULL, 0, NULL, 0, k0, d0, cap, &n0, &dbg) == 0);
    CHECK(oc_extract(&p, f1, W, H, W, NULL, 0, NULL, 0, NULL, 0, k1, d1, cap, &n1, NULL) == 0);
    CHECK(n0 > 900 && n0 <= 1100 && n1 > 900 && n1 <= 1100);
    for (int i = 0; i < n0; i++)
        CHECK(k0[i].x >= 0 && k0[i].x < W && k0[i].y >= 0 && k0[i].y < H && k0[i].octave >= 0 && k0[i].octave < 8 &&
              k0[i].class_id == -1 && k0[i].angle >= 0 && k0[i].angle < 360);
    CHECK(oc_extract(&p, f1, W, H, W, NULL, 0, NULL, 0, NULL, 0, k2, d2, cap, &n2, NULL) == 0);
    CHECK(n2 == n1 && memcmp(k1, k2, sizeof(oc_kp) * n1) == 0 && memcmp(d1, d2, (size_t)n1 * 32) == 0);

    /* dynamic mask: two boxes, T_M inside one, blur flags from the Laplacian (both layers) */
    oc_box boxes[2] = {{200, 100, 320, 400}, {400, 150, 480, 380}};
    float tm[2 * 40];
    for (int i = 0; i < 40; i++) { tm[2 * i] = 210.f + (float)(i % 10) * 10.f; tm[2 * i + 1] = 110.f + (float)(i / 10) * 60.f; }
    int32_t blur[2];
    double means[2];
    CHECK(oc_blur_flags(f1, W, H, W, boxes, 2, blur, means) == 0);
    CHECK(means[0] >= 0 && means[1] >= 0);
    int32_t bl2[2] = {0, 1};
    CHECK(oc_extract(&p, f1, W, H, W, boxes, 2, tm, 40, bl2, 2, k2, d2, cap, &n2, &dbg) == 0);
    CHECK(n2 > 0 && n2 < n1);
    for (int i = 0; i < n2; i++) CHECK(!(k2[i].x >= 200 && k2[i].x < 320 && k2[i].y >= 100 && k2[i].y < 400));

    /* matcher: LastFrame = frame 0 unprojected at Z = 2 m, motion (+2, +1) px */
    oc_camera cam;
    oc_camera_init(&cam, 535.4f, 539.2f, 320.1f, 247.6f, 40.f, W, H, &p);
    static float depth[W * H];
    for (int i = 0; i < W * H; i++) depth[i] = 2.0f;
    float* ur1 = calloc(cap, 4);
    float* dep1 = calloc(cap, 4);
    oc_stereo_from_rgbd(k1, n1, depth, W, W, 40.f, ur1, dep1);
    float* xw = calloc((size_t)cap * 3, 4);
    uint8_t* has = calloc(cap, 1);
    uint8_t* outl = calloc(cap, 1);
    int32_t* nobs = calloc(cap, 4);
    for (int i = 0; i < n0; i++) {
        xw[3 * i] = (k0[i].x - 320.1f) * 2.f / 535.4f;
        xw[3 * i + 1] = (k0[i].y - 247.6f) * 2.f / 539.2f;
        xw[3 * i + 2] = 2.f;
        has[i] = 1;
        nobs[i] = 2;
    }
    oc_lastframe last = {n0, has, outl, xw, d0, nobs, k0};
    oc_curframe cur = {n1, k1, d1, ur1};
    float Tl[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    float Tc[16];
    memcpy(Tc, Tl, sizeof(Tc));
    Tc[3] = 2.f * 2.f / 535.4f;
    Tc[7] = 1.f * 2.f / 539.2f;
    int32_t* match = calloc(cap, 4);
    const int nm = oc_search_by_projection(&cam, &cur, &last, Tc, Tl, 15.f, 0, 1, match);
    CHECK(nm > n1 / 2);
    {
        uint8_t* used = calloc(cap, 1);
        int cnt = 0;
        for (int i = 0; i < n1; i++)
            if (match[i] >= 0) { CHECK(match[i] < n0 && !used[match[i]]); used[match[i]] = 1; cnt++; }
        CHECK(cnt == nm);
        free(used);
    }

    /* local map and relocalisation searches over the same points */
    uint8_t* inview = calloc(cap, 1);
    float *px = calloc(cap, 4), *py = calloc(cap, 4), *pxr = calloc(cap, 4), *vcos = calloc(cap, 4);
    int32_t* lvl = calloc(cap, 4);
    for (int i = 0; i < n0; i++) {
        inview[i] = 1;
        px[i] = k0[i].x + 2.f;
        py[i] = k0[i].y + 1.f;
        pxr[i] = px[i] - 20.f;
        lvl[i] = k0[i].octave;
        vcos[i] = 1.f;
    }
    oc_localmap lm = {n0, inview, px, py, pxr, lvl, vcos, d0, nobs};
    int32_t* cobs = malloc((size_t)cap * 4);
    for (int i = 0; i < cap; i++) cobs[i] = -1;
    CHECK(oc_search_local_map(&cam, &cur, cobs, &lm, 3.f, 0.8f, match) > n1 / 2);
    float* maxd = calloc(cap, 4);
    float* mind = calloc(cap, 4);
    float* ang = calloc(cap, 4);
    for (int i = 0; i < n0; i++) { maxd[i] = 2.0f * 1.2f * 1.2f; mind[i] = 0.5f; ang[i] = k0[i].angle; }
    oc_kfpoints kf = {n0, has, xw, d0, maxd, mind, ang};
    uint8_t* chas = calloc(cap, 1);
    CHECK(oc_search_keyframe(&cam, &cur, chas, &kf, Tc, 10.f, 100, 1, match) > 0);

    /* PoseOptimization from a perturbed start recovers the motion */
    oc_search_by_projection(&cam, &cur, &last, Tc, Tl, 15.f, 0, 1, match);
    float* pxw = calloc((size_t)cap * 3, 4);
    uint8_t* phas = calloc(cap, 1);
    for (int i = 0; i < n1; i++)
        if (match[i] >= 0) { memcpy(&pxw[3 * i], &xw[3 * match[i]], 12); phas[i] = 1; }
    oc_pose_frame pf = {n1, phas, pxw, k1, ur1, p.inv_sigma2, 535.4f, 539.2f, 320.1f, 247.6f, 40.f};
    float T[16];
    memcpy(T, Tc, sizeof(T));
    T[3] += 0.01f;
    uint8_t* pout = calloc(cap, 1);
    const int nin = oc_pose_optimization(&pf, T, pout);
    int it, tr;
    oc_pose_last_stats(&it, &tr);
    CHECK(nin > nm / 2 && it > 0 && tr >= it);
    /* a fronto-parallel scene at one depth trades x-translation for y-rotation, so check the
       image motion the pose predicts at the principal point: (+2, +1) px */
    {
        const float zc = T[8] * 0 + T[9] * 0 + T[10] * 2.f + T[11];
        const float du = 535.4f * (T[2] * 2.f + T[3]) / zc, dv = 539.2f * (T[6] * 2.f + T[7]) / zc;
        if (!(fabsf(du - 2.f) < 0.25f && fabsf(dv - 1.f) < 0.25f)) fprintf(stderr, "pose motion %g %g\n", du, dv);
        CHECK(fabsf(du - 2.f) < 0.25f && fabsf(dv - 1.f) < 0.25f);
    }

    /* ProcessMovingObject on a pair where one rectangle moves against the background */
    static uint8_t g0[W * H], g1[W * H];
    make_frame(g0, canvas, 0, 0, 21u);
    memcpy(g1, g0, sizeof(g1));
    for (int y = 150; y < 330; y++)
        for (int x = 250; x < 400; x++) g1[(y + 4) * W + (x - 5)] = (uint8_t)(((x * 7) ^ (y * 13)) & 255);
    for (int y = 150; y < 330; y++)
        for (int x = 250; x < 400; x++) g0[y * W + x] = (uint8_t)(((x * 7) ^ (y * 13)) & 255);
    float tmo[2 * 1024];
    int ncorners = 0;
    const int ntm = oc_process_moving_object(g0, g1, W, H, W, tmo, 1024, &ncorners);
    CHECK(ncorners > 100 && ntm >= -1);

    /* conversions, undistortion, primitives */
    static uint8_t rgb[3 * W * H], gray[W * H];
    for (int i = 0; i < 3 * W * H; i++) rgb[i] = (uint8_t)next();
    oc_image_to_gray(rgb, W, H, 3 * W, 3, 1, gray);
    oc_depth_to_float(depth, W, H, 4 * W, 1, 1.0f, depth);
    const float dist[5] = {0.262383f, -0.953104f, -0.005358f, 0.002628f, 1.163314f};
    oc_undistort_keypoints(k1, n1, 535.4f, 539.2f, 320.1f, 247.6f, dist, k2);
    for (int i = 0; i < n1; i++) CHECK(isfinite(k2[i].x) && isfinite(k2[i].y));
    CHECK(oc_descriptor_distance(d0, d0) == 0);
    CHECK(fabsf(oc_fast_atan2(1.f, 1.f) - 45.f) < 0.01f);

    free(k0); free(k1); free(k2); free(d0); free(d1); free(d2); free(ur1); free(dep1); free(xw); free(has);
    free(outl); free(nobs); free(match); free(inview); free(px); free(py); free(pxr); free(vcos); free(lvl);
    free(cobs); free(maxd); free(mind); free(ang); free(chas); free(pxw); free(phas); free(pout);
    printf("kat_main: clean (%d/%d keypoints, %d matches, %d pose inliers, %d corners, %d T_M)\n", n0, n1, nm, nin,
           ncorners, ntm);
    return 0;
}
