/*
 * orb_oracle.c -- literal, single-threaded CPU restatement of COEB-SLAM's ORB front end.
 *
 * TEST INFRASTRUCTURE ONLY (see orb_oracle.h): the checker for the HIP path and the
 * timed CPU baseline ("port").  Parity vs the original binary is UNPINNED (OpenCV 3.4
 * absent, no reference tests); the canonical OpenCV-primitive definitions are DESIGN.md s3.
 *
 * Build: gcc -O3 -march=native -ffp-contract=off -shared -fPIC (oracle/Makefile).
 * -ffp-contract=off matters: every fused multiply-add below is an explicit fma()/fmaf()
 * placed where the reference binary fused (SURVEY.md s7 hard part 3); all else is unfused.
 */
#include "orb_oracle.h"

#include <float.h>
#include <math.h>

#define OC_PI 3.1415926535897932384626433832795   /* CV_PI */
#include <stdlib.h>
#include <string.h>

static const int PATTERN_31[1024] = {
#include "../data/orb_bit_pattern_31.inc"
};

enum { PATCH_SIZE = 31, HALF_PATCH_SIZE = 15, EDGE_THRESHOLD = 19 };

/* ---- OpenCV 3.4 scalar helpers (core/fast_math.hpp) ---- */
static inline int cv_round(float v) { return (int)lrintf(v); }     /* half to even */
static inline int cv_round_d(double v) { return (int)lrint(v); }
static inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
static inline int cv_floor_d(double v) { int i = (int)v; return i - (i > v); }
static inline int cv_ceil_d(double v) { int i = (int)v; return i + (i < v); }
static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline short sat_short(int v) { return (short)(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

/* ================= ORBextractor ctor: src/ORBextractor.cc:418-477 ================= */
int oc_init(oc_params* p, int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th)
{
    if (nlevels < 1 || nlevels > OC_MAX_LEVELS) return -1;
    memset(p, 0, sizeof(*p));
    p->nfeatures = nfeatures;
    p->scale_factor = scale_factor;                 /* float -> double member */
    p->nlevels = nlevels;
    p->ini_th = ini_th;
    p->min_th = min_th;
    p->scale[0] = 1.0f;
    p->sigma2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {               /* :426-430, float * double -> float */
        p->scale[i] = (float)((double)p->scale[i - 1] * p->scale_factor);
        p->sigma2[i] = p->scale[i] * p->scale[i];
    }
    for (int i = 0; i < nlevels; i++) {               /* :434-438 */
        p->inv_scale[i] = 1.0f / p->scale[i];
        p->inv_sigma2[i] = 1.0f / p->sigma2[i];
    }
    float factor = (float)(1.0f / p->scale_factor);  /* :443 */
    float ndesired = nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {           /* :447-453 */
        p->nfeat[l] = cv_round(ndesired);
        sum += p->nfeat[l];
        ndesired *= factor;
    }
    p->nfeat[nlevels - 1] = imax(nfeatures - sum, 0);
    for (int i = 0; i < 512; i++) {                   /* :455-457 */
        p->pattern[i][0] = PATTERN_31[2 * i];
        p->pattern[i][1] = PATTERN_31[2 * i + 1];
    }
    /* umax :461-476 */
    int v, v0;
    int vmax = cv_floor(HALF_PATCH_SIZE * sqrtf(2.f) / 2 + 1);
    int vmin = cv_ceil_d(HALF_PATCH_SIZE * sqrtf(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    for (v = 0; v <= vmax; ++v) p->umax[v] = cv_round_d(sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
        while (p->umax[v0] == p->umax[v0 + 1]) ++v0;
        p->umax[v] = v0;
        ++v0;
    }
    return 0;
}

/* ComputePyramid level size (src/ORBextractor.cc:1348-1349) */
void oc_level_size(const oc_params* p, int w, int h, int level, int* lw, int* lh)
{
    float s = p->inv_scale[level];
    *lw = cv_round((float)w * s);
    *lh = cv_round((float)h * s);
}

/* ============ cv::resize INTER_LINEAR, CV_8U (imgproc resize.cpp, OpenCV 3.4) ============
 * Coefficients: 11-bit fixed point, computed exactly as resize()'s table setup.
 * Horizontal pass: exact int (HResizeLinear).  Vertical pass as VResizeLinear::operator() runs
 * it on x86-64 (SSE2 always present): VResizeLinearVec_32s8u takes 16 columns at a time while
 * x <= width - 16, then 4 at a time while x < width - 4, with the SIMD rounding
 * ((S0>>4)*b0>>16) + ((S1>>4)*b1>>16), +2 >> 2 (_mm_mulhi_epi16 / _mm_adds_epi16); the columns
 * left over use the scalar FixedPtCast<int, uchar, 22>: (S0*b0 + S1*b1 + 2^21) >> 22.  This is
 * the OpenCV 3.4.0/3.4.1 SSE2 loop structure; the reference's minor version is unknown
 * (DESIGN.md s2.1). */
int oc_resize_simd_end(int width)
{
    int x = width >= 16 ? (width / 16) * 16 : 0;      /* for (; x <= width - 16; x += 16) */
    while (x < width - 4) x += 4;                     /* for (; x < width - 4; x += 4) */
    return x;
}

void oc_resize_linear(const uint8_t* src, int sw, int sh, int sstride,
                      uint8_t* dst, int dw, int dh, int dstride)
{
    if (sw == dw && sh == dh) {                       /* resize(): same size -> copy */
        for (int y = 0; y < dh; y++) memcpy(dst + (size_t)y * dstride, src + (size_t)y * sstride, dw);
        return;
    }
    double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    int* xofs = (int*)malloc(sizeof(int) * dw);
    short* ialpha = (short*)malloc(sizeof(short) * 2 * dw);
    int* yofs = (int*)malloc(sizeof(int) * dh);
    short* ibeta = (short*)malloc(sizeof(short) * 2 * dh);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = imin(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        float c0 = 1.f - fx, c1 = fx;
        ialpha[2 * dx] = sat_short(cv_round(c0 * 2048));
        ialpha[2 * dx + 1] = sat_short(cv_round(c1 * 2048));
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        yofs[dy] = sy;
        float c0 = 1.f - fy, c1 = fy;
        ibeta[2 * dy] = sat_short(cv_round(c0 * 2048));
        ibeta[2 * dy + 1] = sat_short(cv_round(c1 * 2048));
    }
    int* h0 = (int*)malloc(sizeof(int) * dw);
    int* h1 = (int*)malloc(sizeof(int) * dw);
    for (int dy = 0; dy < dh; dy++) {
        int sy0 = yofs[dy];
        int r0 = sy0 >= 0 ? (sy0 < sh ? sy0 : sh - 1) : 0;          /* clip(sy, 0, sh) */
        int r1 = sy0 + 1 >= 0 ? (sy0 + 1 < sh ? sy0 + 1 : sh - 1) : 0;
        const uint8_t* S0 = src + (size_t)r0 * sstride;
        const uint8_t* S1 = src + (size_t)r1 * sstride;
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            if (dx < xmax) {
                int a0 = ialpha[2 * dx], a1 = ialpha[2 * dx + 1];
                h0[dx] = S0[sx] * a0 + S0[sx + 1] * a1;
                h1[dx] = S1[sx] * a0 + S1[sx + 1] * a1;
            } else {
                h0[dx] = S0[sx] * 2048;
                h1[dx] = S1[sx] * 2048;
            }
        }
        int b0 = ibeta[2 * dy], b1 = ibeta[2 * dy + 1];
        uint8_t* D = dst + (size_t)dy * dstride;
        const int xs = oc_resize_simd_end(dw);
        for (int dx = 0; dx < xs; dx++) {
            int v0 = sat_short(h0[dx] >> 4), v1 = sat_short(h1[dx] >> 4);
            int m0 = (v0 * b0) >> 16, m1 = (v1 * b1) >> 16;   /* _mm_mulhi_epi16 */
            int s = sat_short(m0 + m1);                         /* _mm_adds_epi16 */
            s = sat_short(s + 2) >> 2;
            D[dx] = sat_u8(s);
        }
        for (int dx = xs; dx < dw; dx++)                        /* scalar tail: FixedPtCast */
            D[dx] = sat_u8((h0[dx] * b0 + h1[dx] * b1 + (1 << 21)) >> 22);
    }
    free(h0); free(h1); free(xofs); free(ialpha); free(yofs); free(ibeta);
}

/* ComputePyramid (src/ORBextractor.cc:1344-1367): cascaded level l from level l-1. The
 * 19-px REFLECT_101 border frame is not materialised: no output-affecting read touches it
 * on the RGB-D path. */
int oc_pyramid(const oc_params* p, const uint8_t* gray, int w, int h, int stride,
               uint8_t* out, int64_t* level_off)
{
    int64_t off = 0;
    for (int l = 0; l < p->nlevels; l++) {
        int lw, lh;
        oc_level_size(p, w, h, l, &lw, &lh);
        level_off[l] = off;
        uint8_t* dst = out + off;
        if (l == 0) {
            for (int y = 0; y < h; y++) memcpy(dst + (size_t)y * lw, gray + (size_t)y * stride, w);
        } else {
            int pw, ph;
            oc_level_size(p, w, h, l - 1, &pw, &ph);
            oc_resize_linear(out + level_off[l - 1], pw, ph, pw, dst, lw, lh, lw);
        }
        off += (int64_t)lw * lh;
    }
    level_off[p->nlevels] = off;
    return 0;
}

/* ======================= FAST-9/16 (OpenCV 3.4 features2d/fast.cpp) ======================= */
static void fast_offsets(int pixel[25], int step)
{
    static const int offsets16[16][2] = {
        {0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
        {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
    int k = 0;
    for (; k < 16; k++) pixel[k] = offsets16[k][0] + offsets16[k][1] * step;
    for (; k < 25; k++) pixel[k] = pixel[k - 16];
}

/* cornerScore<16> (fast_score.cpp), scalar form */
static int corner_score16(const uint8_t* ptr, const int pixel[25], int threshold)
{
    const int K = 8, N = K * 3 + 1;
    int k, v = ptr[0];
    short d[25];
    for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (k = 0; k < 16; k += 2) {
        int a = imin(d[k + 1], d[k + 2]);
        a = imin(a, d[k + 3]);
        if (a <= a0) continue;
        a = imin(a, d[k + 4]);
        a = imin(a, d[k + 5]);
        a = imin(a, d[k + 6]);
        a = imin(a, d[k + 7]);
        a = imin(a, d[k + 8]);
        a0 = imax(a0, imin(a, d[k]));
        a0 = imax(a0, imin(a, d[k + 9]));
    }
    int b0 = -a0;
    for (k = 0; k < 16; k += 2) {
        int b = imax(d[k + 1], d[k + 2]);
        b = imax(b, d[k + 3]);
        b = imax(b, d[k + 4]);
        b = imax(b, d[k + 5]);
        if (b >= b0) continue;
        b = imax(b, d[k + 6]);
        b = imax(b, d[k + 7]);
        b = imax(b, d[k + 8]);
        b0 = imin(b0, imax(b, d[k]));
        b0 = imin(b0, imax(b, d[k + 9]));
    }
    return -b0 - 1;
}

/* FAST_t<16>(img, kps, threshold, nonmax_suppression=true) on an ROI */
int oc_fast_roi(const uint8_t* img, int stride, int rows, int cols, int threshold,
                int* xs, int* ys, int* score, int cap)
{
    const int K = 8, N = 25;
    int pixel[25];
    fast_offsets(pixel, stride);
    threshold = imin(imax(threshold, 0), 255);
    uint8_t tabbuf[512];
    for (int i = -255; i <= 255; i++) tabbuf[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    uint8_t* buf[3];
    int* cpbuf[3];
    uint8_t* sbuf = (uint8_t*)calloc((size_t)cols * 3 + 16, 1);
    int* cbuf = (int*)calloc((size_t)(cols + 1) * 3 + 4, sizeof(int));
    buf[0] = sbuf; buf[1] = sbuf + cols; buf[2] = sbuf + 2 * cols;
    cpbuf[0] = cbuf + 1; cpbuf[1] = cpbuf[0] + cols + 1; cpbuf[2] = cpbuf[1] + cols + 1;
    int nout = 0;
    for (int i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = img + (size_t)i * stride + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (int j = 3; j < cols - 3; j++, ptr++) {
                int v = ptr[0];
                const uint8_t* tab = tabbuf - v + 255;
                int d = tab[ptr[pixel[0]]] | tab[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[2]]] | tab[ptr[pixel[10]]];
                d &= tab[ptr[pixel[4]]] | tab[ptr[pixel[12]]];
                d &= tab[ptr[pixel[6]]] | tab[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= tab[ptr[pixel[1]]] | tab[ptr[pixel[9]]];
                d &= tab[ptr[pixel[3]]] | tab[ptr[pixel[11]]];
                d &= tab[ptr[pixel[5]]] | tab[ptr[pixel[13]]];
                d &= tab[ptr[pixel[7]]] | tab[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; k++) {
            int j = cornerpos[k];
            int s = prev[j];
            if (s > prev[j + 1] && s > prev[j - 1] && s > pprev[j - 1] && s > pprev[j] &&
                s > pprev[j + 1] && s > curr[j - 1] && s > curr[j] && s > curr[j + 1]) {
                if (nout < cap) { xs[nout] = j; ys[nout] = i - 1; score[nout] = s; }
                nout++;
            }
        }
    }
    free(sbuf);
    free(cbuf);
    return nout;
}

/* FAST stage of ComputeKeyPointsOctTree (src/ORBextractor.cc:793-850), one level */
int oc_level_candidates(const uint8_t* lvl, int lw, int lh, int stride, int ini_th, int min_th,
                        int* xs, int* ys, int* score, int cap)
{
    const float W = 30;
    const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
    const int maxBorderX = lw - EDGE_THRESHOLD + 3, maxBorderY = lh - EDGE_THRESHOLD + 3;
    const float width = (float)(maxBorderX - minBorderX);
    const float height = (float)(maxBorderY - minBorderY);
    const int nCols = (int)(width / W), nRows = (int)(height / W);
    if (nCols <= 0 || nRows <= 0) return -1;          /* reference: division by zero (UB) */
    const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
    int n = 0;
    int tmpcap = (wCell + 7) * (hCell + 7);
    int* tx = (int*)malloc(sizeof(int) * tmpcap * 3);
    int *ty = tx + tmpcap, *ts = ty + tmpcap;
    for (int i = 0; i < nRows; i++) {
        const float iniY = (float)(minBorderY + i * hCell);
        float maxY = iniY + hCell + 6;
        if (iniY >= maxBorderY - 3) continue;
        if (maxY > maxBorderY) maxY = (float)maxBorderY;
        for (int j = 0; j < nCols; j++) {
            const float iniX = (float)(minBorderX + j * wCell);
            float maxX = iniX + wCell + 6;
            if (iniX >= maxBorderX - 6) continue;
            if (maxX > maxBorderX) maxX = (float)maxBorderX;
            int r0 = (int)iniY, r1 = (int)maxY, c0 = (int)iniX, c1 = (int)maxX;
            const uint8_t* roi = lvl + (size_t)r0 * stride + c0;
            int k = oc_fast_roi(roi, stride, r1 - r0, c1 - c0, ini_th, tx, ty, ts, tmpcap);
            if (k == 0) k = oc_fast_roi(roi, stride, r1 - r0, c1 - c0, min_th, tx, ty, ts, tmpcap);
            for (int q = 0; q < k; q++) {
                if (n < cap) {
                    xs[n] = tx[q] + j * wCell;   /* :844-845, relative to (16,16) */
                    ys[n] = ty[q] + i * hCell;
                    score[n] = ts[q];
                }
                n++;
            }
        }
    }
    free(tx);
    return n;
}

/* ================= DistributeOctTree (src/ORBextractor.cc:489-769) ================= */
typedef struct OcNode {
    int* keys; int nkeys;
    int ulx, uly, urx, ury, blx, bly, brx, bry;
    int no_more;
    long seq;                         /* allocation order == canonical pointer order */
    struct OcNode *prev, *next;
} OcNode;

typedef struct { OcNode* head; OcNode* tail; int size; long seq; } OcList;

static OcNode* node_new(OcList* L, const OcNode* src)
{
    OcNode* n = (OcNode*)malloc(sizeof(OcNode));
    *n = *src;
    n->seq = L->seq++;
    n->prev = n->next = NULL;
    return n;
}
static void list_push_front(OcList* L, OcNode* n)
{
    n->prev = NULL; n->next = L->head;
    if (L->head) L->head->prev = n; else L->tail = n;
    L->head = n; L->size++;
}
static void list_push_back(OcList* L, OcNode* n)
{
    n->next = NULL; n->prev = L->tail;
    if (L->tail) L->tail->next = n; else L->head = n;
    L->tail = n; L->size++;
}
static OcNode* list_erase(OcList* L, OcNode* n)
{
    OcNode* nx = n->next;
    if (n->prev) n->prev->next = n->next; else L->head = n->next;
    if (n->next) n->next->prev = n->prev; else L->tail = n->prev;
    L->size--;
    free(n->keys);
    free(n);
    return nx;
}

/* ExtractorNode::DivideNode (:489-544); children get fresh key arrays */
static void divide_node(const OcNode* p, const int* xs, const int* ys, OcNode c[4])
{
    const int halfX = (int)ceilf((float)(p->urx - p->ulx) / 2);
    const int halfY = (int)ceilf((float)(p->bry - p->uly) / 2);
    memset(c, 0, sizeof(OcNode) * 4);
    c[0].ulx = p->ulx;          c[0].uly = p->uly;
    c[0].urx = p->ulx + halfX;  c[0].ury = p->uly;
    c[0].blx = p->ulx;          c[0].bly = p->uly + halfY;
    c[0].brx = p->ulx + halfX;  c[0].bry = p->uly + halfY;
    c[1].ulx = c[0].urx;        c[1].uly = c[0].ury;
    c[1].urx = p->urx;          c[1].ury = p->ury;
    c[1].blx = c[0].brx;        c[1].bly = c[0].bry;
    c[1].brx = p->urx;          c[1].bry = p->uly + halfY;
    c[2].ulx = c[0].blx;        c[2].uly = c[0].bly;
    c[2].urx = c[0].brx;        c[2].ury = c[0].bry;
    c[2].blx = p->blx;          c[2].bly = p->bly;
    c[2].brx = c[0].brx;        c[2].bry = p->bly;
    c[3].ulx = c[2].urx;        c[3].uly = c[2].ury;
    c[3].urx = c[1].brx;        c[3].ury = c[1].bry;
    c[3].blx = c[2].brx;        c[3].bly = c[2].bry;
    c[3].brx = p->brx;          c[3].bry = p->bry;
    for (int q = 0; q < 4; q++) c[q].keys = (int*)malloc(sizeof(int) * (p->nkeys > 0 ? p->nkeys : 1));
    for (int i = 0; i < p->nkeys; i++) {
        int k = p->keys[i];
        int q;
        if (xs[k] < c[0].urx) q = (ys[k] < c[0].bry) ? 0 : 2;
        else q = (ys[k] < c[0].bry) ? 1 : 3;
        c[q].keys[c[q].nkeys++] = k;
    }
    for (int q = 0; q < 4; q++) c[q].no_more = (c[q].nkeys == 1);
}

typedef struct { int size; OcNode* node; } SizeNode;
static int cmp_size_node(const void* a, const void* b)
{
    const SizeNode* x = (const SizeNode*)a;
    const SizeNode* y = (const SizeNode*)b;
    if (x->size != y->size) return x->size < y->size ? -1 : 1;
    return x->node->seq < y->node->seq ? -1 : (x->node->seq > y->node->seq ? 1 : 0);
}

int oc_distribute_octree(const int* xs, const int* ys, const int* score, int n,
                         int minX, int maxX, int minY, int maxY, int N,
                         int* out_idx, int cap)
{
    const int nIni = (int)roundf((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    OcList L = {NULL, NULL, 0, 0};
    OcNode** ini = (OcNode**)malloc(sizeof(OcNode*) * (nIni > 0 ? nIni : 1));
    for (int i = 0; i < nIni; i++) {
        OcNode t;
        memset(&t, 0, sizeof(t));
        t.ulx = (int)(hX * (float)i);       t.uly = 0;
        t.urx = (int)(hX * (float)(i + 1)); t.ury = 0;
        t.blx = t.ulx; t.bly = maxY - minY;
        t.brx = t.urx; t.bry = maxY - minY;
        t.keys = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
        OcNode* nn = node_new(&L, &t);
        list_push_back(&L, nn);
        ini[i] = nn;
    }
    for (int i = 0; i < n; i++) {                   /* :573-577 */
        int b = (int)((float)xs[i] / hX);
        ini[b]->keys[ini[b]->nkeys++] = i;
    }
    free(ini);
    for (OcNode* it = L.head; it;) {                /* :579-592 */
        if (it->nkeys == 1) { it->no_more = 1; it = it->next; }
        else if (it->nkeys == 0) it = list_erase(&L, it);
        else it = it->next;
    }
    int bFinish = 0;
    SizeNode* vsz = (SizeNode*)malloc(sizeof(SizeNode) * (4 * (size_t)L.size + 16));
    size_t vsz_cap = 4 * (size_t)L.size + 16;
    int nvsz = 0;
#define VSZ_PUSH(S, ND) do { if ((size_t)nvsz >= vsz_cap) { vsz_cap *= 2; vsz = (SizeNode*)realloc(vsz, sizeof(SizeNode) * vsz_cap); } vsz[nvsz].size = (S); vsz[nvsz].node = (ND); nvsz++; } while (0)
    while (!bFinish) {                                /* :601-745 */
        int prevSize = L.size;
        int nToExpand = 0;
        nvsz = 0;
        OcNode* it = L.head;
        while (it) {
            if (it->no_more) { it = it->next; continue; }
            OcNode c[4];
            divide_node(it, xs, ys, c);
            for (int q = 0; q < 4; q++) {
                if (c[q].nkeys > 0) {
                    OcNode* nn = node_new(&L, &c[q]);
                    list_push_front(&L, nn);
                    if (c[q].nkeys > 1) { nToExpand++; VSZ_PUSH(c[q].nkeys, nn); }
                } else
                    free(c[q].keys);
            }
            it = list_erase(&L, it);
        }
        if (L.size >= N || L.size == prevSize) {
            bFinish = 1;
        } else if (L.size + nToExpand * 3 > N) {
            while (!bFinish) {                        /* :683-743 */
                prevSize = L.size;
                int nprev = nvsz;
                SizeNode* vprev = (SizeNode*)malloc(sizeof(SizeNode) * (nprev > 0 ? nprev : 1));
                memcpy(vprev, vsz, sizeof(SizeNode) * nprev);
                nvsz = 0;
                qsort(vprev, nprev, sizeof(SizeNode), cmp_size_node);
                for (int j = nprev - 1; j >= 0; j--) {
                    OcNode c[4];
                    divide_node(vprev[j].node, xs, ys, c);
                    for (int q = 0; q < 4; q++) {
                        if (c[q].nkeys > 0) {
                            OcNode* nn = node_new(&L, &c[q]);
                            list_push_front(&L, nn);
                            if (c[q].nkeys > 1) VSZ_PUSH(c[q].nkeys, nn);
                        } else
                            free(c[q].keys);
                    }
                    list_erase(&L, vprev[j].node);
                    if (L.size >= N) break;
                }
                free(vprev);
                if (L.size >= N || L.size == prevSize) bFinish = 1;
            }
        }
    }
#undef VSZ_PUSH
    free(vsz);
    int nout = 0;                                     /* :747-766 retain best */
    for (OcNode* it = L.head; it; it = it->next) {
        int best = it->keys[0];
        int maxr = score[best];
        for (int k = 1; k < it->nkeys; k++) {
            if (score[it->keys[k]] > maxr) { best = it->keys[k]; maxr = score[best]; }
        }
        if (nout < cap) out_idx[nout] = best;
        nout++;
    }
    while (L.head) list_erase(&L, L.head);
    return nout;
}

/* ============================ orientation / descriptor ============================ */
/* IC_Angle moments (src/ORBextractor.cc:80-104) */
int oc_ic_angle_moments(const uint8_t* img, int stride, int x, int y, const int* umax,
                        int* m01_out, int* m10_out)
{
    int m_01 = 0, m_10 = 0;
    const uint8_t* center = img + (size_t)y * stride + x;
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0;
        int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = center[u + v * stride], val_minus = center[u - v * stride];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    *m01_out = m_01;
    *m10_out = m_10;
    return 0;
}

/* cv::fastAtan2 (OpenCV 3.4 core mathfuncs_core: atan_f32), degrees, no FMA */
float oc_fast_atan2(float y, float x)
{
    static const float p1 = 0.9997878412794807f * (float)(180 / OC_PI);
    static const float p3 = -0.3258083974640975f * (float)(180 / OC_PI);
    static const float p5 = 0.1555786518463281f * (float)(180 / OC_PI);
    static const float p7 = -0.04432655554792128f * (float)(180 / OC_PI);
    float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.2204460492503131e-16);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)2.2204460492503131e-16);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

/* Canonical sincosf: double evaluation with fdlibm kernels, explicit fma in
 * the Cody-Waite reduction, rounded once to float.  Bit-identical to the HIP device version. */
void oc_sincos(float a, float* s, float* c)
{
    const double two_over_pi = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_1t = 6.07710050650619224932e-11;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double x = (double)a;
    double kd = rint(x * two_over_pi);
    double r = fma(-kd, pio2_1, x);
    r = fma(-kd, pio2_1t, r);
    double z = r * r;
    double v = z * r;
    double sr = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    double sn = r + v * (S1 + z * sr);
    double cr = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    double cs = w + (((1.0 - w) - hz) + z * cr);
    int q = ((int)kd) & 3;
    double so, co;
    switch (q) {
    case 0: so = sn; co = cs; break;
    case 1: so = cs; co = -sn; break;
    case 2: so = -sn; co = -cs; break;
    default: so = -cs; co = sn; break;
    }
    *s = (float)so;
    *c = (float)co;
}

/* Gaussian 7-tap, sigma 2, Q8 (OpenCV 3.4.8+/4.x getGaussianKernelBitExact +
 * getGaussianKernelFixedPoint_ED) */
void oc_gauss_kernel7(int k[7])
{
    const int n = 7, n2 = 3;
    const double sigma = 2.0;
    double scale2X = -0.125 / (sigma * sigma);
    double values[3], sum = 0.0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        double t = exp((double)(x * x) * scale2X);
        values[i] = t;
        sum += t;
    }
    sum *= 2.0;
    sum += 1.0;
    double mul1 = 1.0 / sum;
    double res[7];
    for (int i = 0; i < n2; i++) { res[i] = res[n - 1 - i] = values[i] * mul1; }
    res[n2] = 1.0 * mul1;
    double err = 0.0;
    int64_t s = 0;
    for (int i = 0; i < n2; i++) {
        double adj = res[i] * 256.0 + err;
        int64_t v0 = cv_round_d(adj);
        err = adj - (double)v0;
        k[i] = k[n - 1 - i] = (int)v0;
        s += v0;
    }
    s *= 2;
    k[n2] = (int)(256 - s);
}

static inline int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    }
    return p;
}

/* GaussianBlur(7x7, 2, 2, BORDER_REFLECT_101) on a cloned level (src/ORBextractor.cc:1317-1318):
 * fixedSmoothInvoker<uint8_t, ufixedpoint16>: horizontal u8 x Q8 -> Q8 sums, vertical
 * Q8 x Q8 -> Q16, out = (v + 2^15) >> 16. */
void oc_gaussian_blur7(const uint8_t* src, int w, int h, int sstride, uint8_t* dst, int dstride)
{
    int k[7];
    oc_gauss_kernel7(k);
    uint32_t* hbuf = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)w * h);
    for (int y = 0; y < h; y++) {
        const uint8_t* S = src + (size_t)y * sstride;
        for (int x = 0; x < w; x++) {
            uint32_t acc = 0;
            for (int t = 0; t < 7; t++) acc += (uint32_t)k[t] * S[reflect101(x + t - 3, w)];
            hbuf[(size_t)y * w + x] = acc;
        }
    }
    for (int y = 0; y < h; y++) {
        for (int x = 0; x < w; x++) {
            uint32_t acc = 0;
            for (int t = 0; t < 7; t++) acc += (uint32_t)k[t] * hbuf[(size_t)reflect101(y + t - 3, h) * w + x];
            uint32_t o = (acc + (1u << 15)) >> 16;
            dst[(size_t)y * dstride + x] = (uint8_t)(o > 255 ? 255 : o);
        }
    }
    free(hbuf);
}

/* computeOrbDescriptor (src/ORBextractor.cc:109-156); rotation in the fused forms of the
 * reference binary: row = cvRound(fmaf(x, b, y*a)), col = cvRound(fmaf(x, a, -(y*b))) */
void oc_orb_descriptor(const uint8_t* img, int stride, int x, int y, float angle,
                       const int (*pattern)[2], uint8_t desc[32])
{
    const float factorPI = (float)(OC_PI / 180.f);
    float ang = angle * factorPI;
    float b, a;
    oc_sincos(ang, &b, &a);
    const uint8_t* center = img + (size_t)y * stride + x;
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int t = 0; t < 8; t++) {
            const int* p0 = pattern[16 * i + 2 * t];
            const int* p1 = pattern[16 * i + 2 * t + 1];
            float px0 = (float)p0[0], py0 = (float)p0[1];
            float px1 = (float)p1[0], py1 = (float)p1[1];
            int r0 = cv_round(fmaf(px0, b, py0 * a)), c0 = cv_round(fmaf(px0, a, -(py0 * b)));
            int r1 = cv_round(fmaf(px1, b, py1 * a)), c1 = cv_round(fmaf(px1, a, -(py1 * b)));
            int t0 = center[r0 * stride + c0];
            int t1 = center[r1 * stride + c1];
            val |= (t0 < t1) << t;
        }
        desc[i] = (uint8_t)val;
    }
}

/* ======================== dynamic mask: src/ORBextractor.cc:1101-1195 ======================== */
int oc_dynamic_mask(const oc_box* boxes, int nbox, const float* tm_xy, int ntm,
                    const int32_t* blur_flag, int nblur, int w, int h,
                    uint8_t* mask, float* area_out)
{
    memset(mask, 1, (size_t)w * h);
    float area = 0;
    for (int b = 0; b < nbox; b++) {
        float xmin = boxes[b].xmin, ymin = boxes[b].ymin, xmax = boxes[b].xmax, ymax = boxes[b].ymax;
        /* mask_mark(Rect(int(xmin), int(ymin), int(xmax - xmin), int(ymax - ymin))) = 0 */
        int rx = (int)xmin, ry = (int)ymin, rw = (int)(xmax - xmin), rh = (int)(ymax - ymin);
        float area_box = (xmax - xmin) * (ymax - ymin);
        int mark_box = 0;
        size_t nin = 0;
        for (int t = 0; t < ntm; t++) {
            int px = (int)tm_xy[2 * t], py = (int)tm_xy[2 * t + 1];
            int in = px >= 0 && px < w && py >= 0 && py < h &&
                     px >= rx && px < rx + rw && py >= ry && py < ry + rh;
            if (in) nin++;
            if ((float)(nin * 10000) > area_box) {   /* layer 1, :1145 */
                mark_box = 1;
                area = area + area_box;
                for (int i = imax((int)xmin, 0); i < imin((int)xmax, w); i++)
                    for (int j = imax((int)ymin, 0); j < imin((int)ymax, h); j++) mask[(size_t)j * w + i] = 0;
                break;
            }
        }
        if (mark_box) continue;
        int bf = b < nblur ? blur_flag[b] : 0;
        if (bf == 1 && nin > 0) {                  /* layer 2, :1168 */
            for (int i = imax((int)xmin, 0); i < imin((int)xmax, w); i++)
                for (int j = imax((int)ymin, 0); j < imin((int)ymax, h); j++) mask[(size_t)j * w + i] = 0;
            area = area + area_box;
            continue;
        }
    }
    if (area_out) *area_out = area;
    return area > 200000 ? 1 : 0;                   /* :1192 */
}

/* CheckMovingKeyPoints / _finall lookup (src/ORBextractor.cc:1391-1397, 1426-1440) */
static int masked_out(const uint8_t* mask, int w, int h, float px, float py, float scale)
{
    float sx = px * scale, sy = py * scale;
    if (sx >= (float)(w - 1)) sx = (float)(w - 1);
    if (sy >= (float)(h - 1)) sy = (float)(h - 1);
    int ix = (int)sx, iy = (int)sy;
    return mask[(size_t)iy * w + ix] == 0;
}

/* ============================ operator(): src/ORBextractor.cc:1088-1342 ============================ */
int oc_extract(const oc_params* p, const uint8_t* gray, int w, int h, int stride,
               const oc_box* boxes, int nbox, const float* tm_xy, int ntm,
               const int32_t* blur_flag, int nblur,
               oc_kp* kp_out, uint8_t* desc_out, int cap, int* n_out, oc_debug* dbg)
{
    *n_out = 0;
    if (!gray || w <= 0 || h <= 0) return 0;          /* _image.empty() -> return */
    const int L = p->nlevels;
    if (L < 1 || L > OC_MAX_LEVELS) return -1;
    uint8_t* mask = (uint8_t*)malloc((size_t)w * h);
    float area;
    int area_flag = oc_dynamic_mask(boxes, nbox, tm_xy, ntm, blur_flag, nblur, w, h, mask, &area);
    int64_t off[OC_MAX_LEVELS + 1];
    int64_t total = 0;
    int lw[OC_MAX_LEVELS], lh[OC_MAX_LEVELS];
    for (int l = 0; l < L; l++) { oc_level_size(p, w, h, l, &lw[l], &lh[l]); total += (int64_t)lw[l] * lh[l]; }
    uint8_t* pyr = (uint8_t*)malloc((size_t)total);
    oc_pyramid(p, gray, w, h, stride, pyr, off);
    const int ini_th = area_flag ? 30 : 20, min_th = area_flag ? 10 : 7;   /* :775-784 */

    int* lvl_n = (int*)calloc((size_t)L, sizeof(int));
    int** lvl_x = (int**)calloc((size_t)L, sizeof(int*));
    int** lvl_y = (int**)calloc((size_t)L, sizeof(int*));
    int** lvl_s = (int**)calloc((size_t)L, sizeof(int*));
    int rc = 0;
    for (int l = 0; l < L; l++) {
        const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
        const int maxBorderX = lw[l] - EDGE_THRESHOLD + 3, maxBorderY = lh[l] - EDGE_THRESHOLD + 3;
        int capc = lw[l] * lh[l] / 2 + 16;
        int* cx = (int*)malloc(sizeof(int) * capc * 3);
        int *cy = cx + capc, *cs = cy + capc;
        int nc = oc_level_candidates(pyr + off[l], lw[l], lh[l], lw[l], ini_th, min_th, cx, cy, cs, capc);
        if (nc < 0) { free(cx); rc = -2; break; }
        if (dbg) dbg->ncand[l] = nc;
        if (area_flag) {                                                  /* :854-858 */
            float scale = (l != 0) ? p->scale[l] : 1.0f;
            int m = 0;
            for (int k = 0; k < nc; k++) {
                if (!masked_out(mask, w, h, (float)cx[k], (float)cy[k], scale)) {
                    cx[m] = cx[k]; cy[m] = cy[k]; cs[m] = cs[k]; m++;
                }
            }
            nc = m;
        }
        int N = area_flag ? (int)((double)p->nfeat[l] * 0.7) : p->nfeat[l];   /* :866-875 */
        int ocap = nc + 8;
        int* oidx = (int*)malloc(sizeof(int) * ocap);
        int nk = oc_distribute_octree(cx, cy, cs, nc, minBorderX, maxBorderX, minBorderY, maxBorderY, N, oidx, ocap);
        lvl_x[l] = (int*)malloc(sizeof(int) * (nk + 1));
        lvl_y[l] = (int*)malloc(sizeof(int) * (nk + 1));
        lvl_s[l] = (int*)malloc(sizeof(int) * (nk + 1));
        for (int k = 0; k < nk; k++) {                                    /* :884-890 */
            lvl_x[l][k] = cx[oidx[k]] + minBorderX;
            lvl_y[l][k] = cy[oidx[k]] + minBorderY;
            lvl_s[l][k] = cs[oidx[k]];
        }
        lvl_n[l] = nk;
        free(oidx);
        free(cx);
    }
    if (rc == 0 && !area_flag) {                                          /* :1204-1207 */
        for (int l = 0; l < L && l < 8; l++) {
            float scale = (l != 0) ? p->scale[l] : 1.0f;
            int m = 0;
            for (int k = 0; k < lvl_n[l]; k++) {
                if (!masked_out(mask, w, h, (float)lvl_x[l][k], (float)lvl_y[l][k], scale)) {
                    lvl_x[l][m] = lvl_x[l][k]; lvl_y[l][m] = lvl_y[l][k]; lvl_s[l][m] = lvl_s[l][k]; m++;
                }
            }
            lvl_n[l] = m;
        }
    }
    int n = 0;
    if (rc == 0) {
        uint8_t* blur = (uint8_t*)malloc((size_t)lw[0] * lh[0]);
        for (int l = 0; l < L; l++) {
            if (dbg) dbg->nkept[l] = lvl_n[l];
            if (lvl_n[l] == 0) continue;
            const uint8_t* lvl = pyr + off[l];
            oc_gaussian_blur7(lvl, lw[l], lh[l], lw[l], blur, lw[l]);   /* :1317-1318 */
            const int scaledPatchSize = (int)(PATCH_SIZE * p->scale[l]);   /* :877 */
            for (int k = 0; k < lvl_n[l]; k++) {
                int x = lvl_x[l][k], y = lvl_y[l][k];
                int m01, m10;
                oc_ic_angle_moments(lvl, lw[l], x, y, p->umax, &m01, &m10);
                float angle = oc_fast_atan2((float)m01, (float)m10);
                if (n < cap) {
                    oc_kp* kp = &kp_out[n];
                    kp->x = (float)x; kp->y = (float)y;
                    kp->size = (float)scaledPatchSize;
                    kp->angle = angle;
                    kp->response = (float)lvl_s[l][k];
                    kp->octave = l;
                    kp->class_id = -1;
                    if (desc_out)
                        oc_orb_descriptor(blur, lw[l], x, y, angle, (const int (*)[2])p->pattern, desc_out + (size_t)n * 32);
                    if (l != 0) { kp->x *= p->scale[l]; kp->y *= p->scale[l]; }   /* :1327-1334 */
                }
                n++;
            }
        }
        free(blur);
    }
    if (dbg) {
        dbg->area_flag = area_flag;
        for (int l = 0; l <= L; l++) dbg->level_off[l] = off[l];
        if (dbg->pyramid) memcpy(dbg->pyramid, pyr, (size_t)total);
    }
    for (int l = 0; l < L; l++) { free(lvl_x[l]); free(lvl_y[l]); free(lvl_s[l]); }
    free(lvl_x); free(lvl_y); free(lvl_s); free(lvl_n);
    free(pyr);
    free(mask);
    *n_out = n;
    return rc;
}

/* ===================== Frame blur flag: src/Frame.cc:171-202, 905-913 ===================== */
int oc_blur_flags(const uint8_t* gray, int w, int h, int stride,
                  const oc_box* boxes, int nbox, int32_t* out, double* mean_out)
{
    for (int b = 0; b < nbox; b++) {
        int rx = (int)boxes[b].xmin, ry = (int)boxes[b].ymin;
        int rw = (int)(boxes[b].xmax - boxes[b].xmin), rh = (int)(boxes[b].ymax - boxes[b].ymin);
        if (rx < 0 || ry < 0 || rw <= 0 || rh <= 0 || rx + rw > w || ry + rh > h) {
            out[b] = 0;                   /* reference: cv::Rect assertion; documented as 0 */
            if (mean_out) mean_out[b] = -1.0;
            continue;
        }
        int64_t S = 0;
        for (int y = 0; y < rh; y++) {
            for (int x = 0; x < rw; x++) {
                const uint8_t* c = gray + (size_t)(ry) * stride + rx;
                int ym = reflect101(y - 1, rh), yp = reflect101(y + 1, rh);
                int xm = reflect101(x - 1, rw), xp = reflect101(x + 1, rw);
                int lap = c[(size_t)ym * stride + x] + c[(size_t)yp * stride + x] +
                          c[(size_t)y * stride + xm] + c[(size_t)y * stride + xp] - 4 * c[(size_t)y * stride + x];
                S += lap < 0 ? 0 : lap;   /* saturate_cast<ushort> */
            }
        }
        double mean = (double)S * (1. / (double)((int64_t)rw * rh));   /* cv::mean: s*(1./nz) */
        if (mean_out) mean_out[b] = mean;
        out[b] = mean < 4.2 ? 1 : 0;
    }
    return 0;
}

/* cvtColor RGB2GRAY / BGR2GRAY 8U, 14-bit fixed point (imgproc color.cpp RGB2Gray<uchar>) */
/* Tracking::GrabImageRGBD (Tracking.cc:212-225): cvtColor RGB2GRAY / BGR2GRAY (3 channels),
   RGBA2GRAY / BGRA2GRAY (4 channels, alpha ignored); a 1-channel image is used as is.  OpenCV
   3.4 8U fixed point: R 4899, G 9617, B 1868, 14-bit shift with rounding. */
void oc_image_to_gray(const uint8_t* img, int w, int h, int stride, int channels, int rgb_order, uint8_t* out)
{
    const int R2Y = 4899, G2Y = 9617, B2Y = 1868;
    for (int y = 0; y < h; y++) {
        const uint8_t* s = img + (size_t)y * stride;
        for (int x = 0; x < w; x++) {
            const uint8_t* p = s + (size_t)channels * x;
            if (channels == 1) { out[(size_t)y * w + x] = p[0]; continue; }
            const int c0 = p[0], c1 = p[1], c2 = p[2];
            const int v = rgb_order ? (c0 * R2Y + c1 * G2Y + c2 * B2Y) : (c0 * B2Y + c1 * G2Y + c2 * R2Y);
            out[(size_t)y * w + x] = (uint8_t)((v + (1 << 13)) >> 14);
        }
    }
}

void oc_rgb2gray(const uint8_t* rgb, int w, int h, int stride, int rgb_order, uint8_t* out)
{
    oc_image_to_gray(rgb, w, h, stride, 3, rgb_order, out);
}

/* Tracking.cc:227-228: if (fabs(mDepthMapFactor - 1) > 1e-5 || type != CV_32F)
   imDepth.convertTo(imDepth, CV_32F, mDepthMapFactor) -- float product (cvtScale, WT = float);
   otherwise the 32F map is used unchanged.  depth_type 0 = 16UC1, 1 = 32FC1; stride in bytes. */
void oc_depth_to_float(const void* depth, int w, int h, size_t stride, int depth_type, float factor, float* out)
{
    const int copy = depth_type == 1 && !(fabsf(factor - 1.0f) > 1e-5f);
    for (int y = 0; y < h; y++) {
        const uint8_t* row = (const uint8_t*)depth + (size_t)y * stride;
        for (int x = 0; x < w; x++) {
            float v;
            if (depth_type == 0) v = (float)((const uint16_t*)row)[x] * factor;
            else v = copy ? ((const float*)row)[x] : ((const float*)row)[x] * factor;
            out[(size_t)y * w + x] = v;
        }
    }
}

/* ================================= matcher side ================================= */
void oc_camera_init(oc_camera* c, float fx, float fy, float cx, float cy, float bf,
                    int w, int h, const oc_params* p)
{
    memset(c, 0, sizeof(*c));
    c->fx = fx; c->fy = fy; c->cx = cx; c->cy = cy; c->bf = bf;
    c->mb = bf / fx;                                                  /* Frame.cc:246 */
    c->min_x = 0.0f; c->max_x = (float)w; c->min_y = 0.0f; c->max_y = (float)h;   /* :635-641 */
    c->grid_inv_w = (float)OC_GRID_COLS / (c->max_x - c->min_x);       /* :233-234 */
    c->grid_inv_h = (float)OC_GRID_ROWS / (c->max_y - c->min_y);
    c->nlevels = p->nlevels;
    for (int l = 0; l < p->nlevels; l++) c->scale[l] = p->scale[l];
}

void oc_stereo_from_rgbd(const oc_kp* kps, int n, const float* depth, int w, int dstride,
                         float bf, float* uright, float* dep)
{
    (void)w;
    for (int i = 0; i < n; i++) {
        uright[i] = -1; dep[i] = -1;
        const float v = kps[i].y, u = kps[i].x;
        const float d = depth[(size_t)(int)v * dstride + (int)u];      /* at<float>(v,u) */
        if (d > 0) { dep[i] = d; uright[i] = kps[i].x - bf / d; }
    }
}

void oc_assign_grid(const oc_camera* c, const oc_kp* kps, int n, oc_grid* g)
{
    const int NC = OC_GRID_COLS * OC_GRID_ROWS;
    int* cell = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
    memset(g->cell_start, 0, sizeof(int) * (NC + 1));
    for (int i = 0; i < n; i++) {
        int px = (int)roundf((kps[i].x - c->min_x) * c->grid_inv_w);   /* PosInGrid :560-561 */
        int py = (int)roundf((kps[i].y - c->min_y) * c->grid_inv_h);
        if (px < 0 || px >= OC_GRID_COLS || py < 0 || py >= OC_GRID_ROWS) { cell[i] = -1; continue; }
        cell[i] = px * OC_GRID_ROWS + py;
        g->cell_start[cell[i] + 1]++;
    }
    for (int k = 0; k < NC; k++) g->cell_start[k + 1] += g->cell_start[k];
    int* fill = (int*)malloc(sizeof(int) * NC);
    memcpy(fill, g->cell_start, sizeof(int) * NC);
    for (int i = 0; i < n; i++)
        if (cell[i] >= 0) g->cell_idx[fill[cell[i]]++] = i;
    free(fill);
    free(cell);
}

int oc_features_in_area(const oc_camera* c, const oc_kp* kps, const oc_grid* g,
                        float x, float y, float r, int minLevel, int maxLevel,
                        int* out, int cap)
{
    int n = 0;
    const int nMinCellX = imax(0, (int)floorf((x - c->min_x - r) * c->grid_inv_w));
    if (nMinCellX >= OC_GRID_COLS) return 0;
    const int nMaxCellX = imin(OC_GRID_COLS - 1, (int)ceilf((x - c->min_x + r) * c->grid_inv_w));
    if (nMaxCellX < 0) return 0;
    const int nMinCellY = imax(0, (int)floorf((y - c->min_y - r) * c->grid_inv_h));
    if (nMinCellY >= OC_GRID_ROWS) return 0;
    const int nMaxCellY = imin(OC_GRID_ROWS - 1, (int)ceilf((y - c->min_y + r) * c->grid_inv_h));
    if (nMaxCellY < 0) return 0;
    const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            int cidx = ix * OC_GRID_ROWS + iy;
            for (int j = g->cell_start[cidx]; j < g->cell_start[cidx + 1]; j++) {
                const oc_kp* kp = &kps[g->cell_idx[j]];
                if (bCheckLevels) {
                    if (kp->octave < minLevel) continue;
                    if (maxLevel >= 0 && kp->octave > maxLevel) continue;
                }
                const float distx = kp->x - x, disty = kp->y - y;
                if (fabsf(distx) < r && fabsf(disty) < r) {
                    if (n < cap) out[n] = g->cell_idx[j];
                    n++;
                }
            }
        }
    }
    return n;
}

int oc_descriptor_distance(const uint8_t* a, const uint8_t* b)
{
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t pa, pb;
        memcpy(&pa, a + 4 * i, 4);
        memcpy(&pb, b + 4 * i, 4);
        unsigned int v = pa ^ pb;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

/* ORBmatcher::ComputeThreeMaxima (src/ORBmatcher.cc:1602-1643) */
static void three_maxima(const int* hist, int L, int* i1, int* i2, int* i3)
{
    int max1 = 0, max2 = 0, max3 = 0;
    *i1 = *i2 = *i3 = -1;
    for (int i = 0; i < L; i++) {
        const int s = hist[i];
        if (s > max1) { max3 = max2; max2 = max1; max1 = s; *i3 = *i2; *i2 = *i1; *i1 = i; }
        else if (s > max2) { max3 = max2; max2 = s; *i3 = *i2; *i2 = i; }
        else if (s > max3) { max3 = s; *i3 = i; }
    }
    if (max2 < 0.1f * (float)max1) { *i2 = -1; *i3 = -1; }
    else if (max3 < 0.1f * (float)max1) { *i3 = -1; }
}

int oc_search_by_projection(const oc_camera* cam, const oc_curframe* cur, const oc_lastframe* last,
                            const float Tcw_cur[16], const float Tcw_last[16],
                            float th, int bMono, int check_ori, int32_t* match_out)
{
    enum { HISTO_LENGTH = 30, TH_HIGH = 100 };
    int nmatches = 0;
    const float factor = 1.0f / HISTO_LENGTH;
    const float* T = Tcw_cur;
    const float* Tl = Tcw_last;
    /* twc = -Rcw.t()*tcw (GEMM_1_T: generic path, double accumulation) */
    float twc[3], tlc[3];
    for (int k = 0; k < 3; k++) {
        double s = (double)T[0 * 4 + k] * T[3] + (double)T[1 * 4 + k] * T[7];
        s = s + (double)T[2 * 4 + k] * T[11];
        twc[k] = (float)(s * -1.0);
    }
    /* tlc = Rlw*twc + tlw (small-matrix float path) */
    for (int k = 0; k < 3; k++) {
        float t = Tl[k * 4 + 0] * twc[0] + Tl[k * 4 + 1] * twc[1];
        t = t + Tl[k * 4 + 2] * twc[2];
        tlc[k] = (float)((double)t + (double)Tl[k * 4 + 3]);
    }
    const int bForward = tlc[2] > cam->mb && !bMono;
    const int bBackward = -tlc[2] > cam->mb && !bMono;

    oc_grid g;
    g.cell_start = (int*)malloc(sizeof(int) * (OC_GRID_COLS * OC_GRID_ROWS + 1));
    g.cell_idx = (int*)malloc(sizeof(int) * (cur->n > 0 ? cur->n : 1));
    oc_assign_grid(cam, cur->keys_un, cur->n, &g);

    int* owner = match_out;                       /* CurrentFrame.mvpMapPoints as slot ids */
    for (int i = 0; i < cur->n; i++) owner[i] = -1;
    int* hist_items = (int*)malloc(sizeof(int) * (last->n > 0 ? last->n : 1) * 2);
    int* hist_bin = hist_items + (last->n > 0 ? last->n : 1);
    int nhist = 0;
    int* cand = (int*)malloc(sizeof(int) * (cur->n > 0 ? cur->n : 1));

    for (int i = 0; i < last->n; i++) {
        if (!last->has_mp[i] || last->outlier[i]) continue;
        const float* X = &last->xw[3 * i];
        float p3[3];
        for (int k = 0; k < 3; k++) {             /* x3Dc = Rcw*x3Dw+tcw (small-matrix path) */
            float t = T[k * 4 + 0] * X[0] + T[k * 4 + 1] * X[1];
            t = t + T[k * 4 + 2] * X[2];
            p3[k] = (float)((double)t + (double)T[k * 4 + 3]);
        }
        const float xc = p3[0], yc = p3[1];
        const float invzc = (float)(1.0 / (double)p3[2]);
        if (invzc < 0) continue;
        float u = fmaf(cam->fx * xc, invzc, cam->cx);   /* fused in the reference binary */
        float v = fmaf(cam->fy * yc, invzc, cam->cy);
        if (u < cam->min_x || u > cam->max_x) continue;
        if (v < cam->min_y || v > cam->max_y) continue;
        int nLastOctave = last->keys_un[i].octave;
        float radius = th * cam->scale[nLastOctave];
        int nc;
        if (bForward) nc = oc_features_in_area(cam, cur->keys_un, &g, u, v, radius, nLastOctave, -1, cand, cur->n);
        else if (bBackward) nc = oc_features_in_area(cam, cur->keys_un, &g, u, v, radius, 0, nLastOctave, cand, cur->n);
        else nc = oc_features_in_area(cam, cur->keys_un, &g, u, v, radius, nLastOctave - 1, nLastOctave + 1, cand, cur->n);
        if (nc == 0) continue;
        const uint8_t* dMP = &last->mp_desc[32 * i];
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = cand[c];
            if (owner[i2] >= 0 && last->mp_nobs[owner[i2]] > 0) continue;
            if (cur->uright[i2] > 0) {
                const float ur = fmaf(-cam->bf, invzc, u);   /* u - mbf*invzc, fused */
                const float er = fabsf(ur - cur->uright[i2]);
                if (er > radius) continue;
            }
            const int dist = oc_descriptor_distance(dMP, &cur->desc[32 * i2]);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        }
        if (bestDist <= TH_HIGH) {
            owner[bestIdx2] = i;
            nmatches++;
            if (check_ori) {
                float rot = last->keys_un[i].angle - cur->keys_un[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                hist_items[nhist] = bestIdx2;
                hist_bin[nhist] = bin;
                nhist++;
            }
        }
    }
    if (check_ori) {
        int hist[HISTO_LENGTH] = {0};
        for (int k = 0; k < nhist; k++) hist[hist_bin[k]]++;
        int i1, i2, i3;
        three_maxima(hist, HISTO_LENGTH, &i1, &i2, &i3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == i1 || b == i2 || b == i3) continue;
            for (int k = 0; k < nhist; k++)
                if (hist_bin[k] == b) { owner[hist_items[k]] = -1; nmatches--; }
        }
    }
    free(cand);
    free(hist_items);
    free(g.cell_start);
    free(g.cell_idx);
    return nmatches;
}

/* ORBmatcher::RadiusByViewingCos (src/ORBmatcher.cc:131-137) */
static float radius_by_viewing_cos(float viewCos) { return viewCos > 0.998f ? 2.5f : 4.0f; }

/* ORBmatcher::SearchByProjection(Frame &F, const vector<MapPoint*> &vpMapPoints, const float th)
 * (src/ORBmatcher.cc:44-129).  The MapPoint* written into F.mvpMapPoints is tracked as the
 * local-map index (match_out) plus the Observations() of whoever holds each keypoint. */
int oc_search_local_map(const oc_camera* cam, const oc_curframe* cur, const int32_t* cur_obs,
                        const oc_localmap* mp, float th, float nnratio, int32_t* match_out)
{
    enum { TH_HIGH = 100 };
    int nmatches = 0;
    const int bFactor = th != 1.0f;
    oc_grid g;
    g.cell_start = (int*)malloc(sizeof(int) * (OC_GRID_COLS * OC_GRID_ROWS + 1));
    g.cell_idx = (int*)malloc(sizeof(int) * (cur->n > 0 ? cur->n : 1));
    oc_assign_grid(cam, cur->keys_un, cur->n, &g);
    int* holder_obs = (int*)malloc(sizeof(int) * (cur->n > 0 ? cur->n : 1));   /* Observations() of F.mvpMapPoints[i], -1 = NULL */
    for (int i = 0; i < cur->n; i++) { holder_obs[i] = cur_obs ? cur_obs[i] : -1; match_out[i] = -1; }
    int* cand = (int*)malloc(sizeof(int) * (cur->n > 0 ? cur->n : 1));
    for (int q = 0; q < mp->n; q++) {
        if (!mp->in_view[q]) continue;                            /* :53-57 */
        const int nPredictedLevel = mp->level[q];
        float r = radius_by_viewing_cos(mp->view_cos[q]);         /* :62 */
        if (bFactor) r *= th;
        const float rs = r * cam->scale[nPredictedLevel];
        const int nc = oc_features_in_area(cam, cur->keys_un, &g, mp->proj_x[q], mp->proj_y[q], rs,
                                           nPredictedLevel - 1, nPredictedLevel, cand, cur->n);
        if (nc == 0) continue;
        const uint8_t* dMP = &mp->desc[32 * q];
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int idx = cand[c];
            if (holder_obs[idx] > 0) continue;                   /* :86-88 */
            if (cur->uright[idx] > 0) {                          /* :90-95 */
                const float er = fabsf(mp->proj_xr[q] - cur->uright[idx]);
                if (er > r * cam->scale[nPredictedLevel]) continue;
            }
            const int dist = oc_descriptor_distance(dMP, &cur->desc[32 * idx]);
            if (dist < bestDist) {                               /* :101-113 */
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = cur->keys_un[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = cur->keys_un[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {                               /* :117-125 */
            if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) continue;
            match_out[bestIdx] = q;
            holder_obs[bestIdx] = mp->nobs[q];
            nmatches++;
        }
    }
    free(cand);
    free(holder_obs);
    free(g.cell_start);
    free(g.cell_idx);
    return nmatches;
}

/* MapPoint::PredictScale(currentDist, Frame*) (MapPoint.cc:402-417): ratio = mfMaxDistance /
 * currentDist; nScale = ceil(log(ratio) / mfLogScaleFactor), clamped to the pyramid.  log is
 * std::log(float); canonical: correctly rounded, as (float)log((double)x). */
static float canon_logf(float x) { return (float)log((double)x); }

static int predict_scale(float max_dist, float dist, float log_sf, int nlevels)
{
    const float ratio = max_dist / dist;
    int s = (int)ceilf(canon_logf(ratio) / log_sf);
    if (s < 0) s = 0;
    else if (s >= nlevels) s = nlevels - 1;
    return s;
}

int oc_search_keyframe(const oc_camera* cam, const oc_curframe* cur, const uint8_t* cur_has,
                       const oc_kfpoints* kf, const float Tcw[16], float th, int orb_dist, int check_ori,
                       int32_t* match_out)
{
    enum { HISTO_LENGTH = 30 };
    int nmatches = 0;
    const float factor = 1.0f / HISTO_LENGTH;
    const float* T = Tcw;
    const float log_sf = cam->nlevels > 1 ? canon_logf(cam->scale[1]) : 1.0f;   /* Frame.cc:85 */
    /* Ow = -Rcw.t()*tcw (GEMM_1_T, double accumulation) */
    float Ow[3];
    for (int k = 0; k < 3; k++) {
        double s = (double)T[0 * 4 + k] * T[3] + (double)T[1 * 4 + k] * T[7];
        s = s + (double)T[2 * 4 + k] * T[11];
        Ow[k] = (float)(s * -1.0);
    }
    oc_grid g;
    g.cell_start = (int*)malloc(sizeof(int) * (OC_GRID_COLS * OC_GRID_ROWS + 1));
    g.cell_idx = (int*)malloc(sizeof(int) * (cur->n > 0 ? cur->n : 1));
    oc_assign_grid(cam, cur->keys_un, cur->n, &g);
    /* taken[i2]: CurrentFrame.mvpMapPoints[i2] != NULL (entry holders and this call's) */
    uint8_t* taken = (uint8_t*)malloc(cur->n > 0 ? cur->n : 1);
    for (int i = 0; i < cur->n; i++) { taken[i] = cur_has ? cur_has[i] != 0 : 0; match_out[i] = -1; }
    int* hist_items = (int*)malloc(sizeof(int) * (kf->n > 0 ? kf->n : 1) * 2);
    int* hist_bin = hist_items + (kf->n > 0 ? kf->n : 1);
    int nhist = 0;
    int* cand = (int*)malloc(sizeof(int) * (cur->n > 0 ? cur->n : 1));
    for (int i = 0; i < kf->n; i++) {
        if (!kf->valid[i]) continue;                                    /* :1493-1495 */
        const float* X = &kf->xw[3 * i];
        float p3[3];
        for (int k = 0; k < 3; k++) {                                   /* x3Dc = Rcw*x3Dw+tcw */
            float t = T[k * 4 + 0] * X[0] + T[k * 4 + 1] * X[1];
            t = t + T[k * 4 + 2] * X[2];
            p3[k] = (float)((double)t + (double)T[k * 4 + 3]);
        }
        const float invzc = (float)(1.0 / (double)p3[2]);
        const float u = fmaf(cam->fx * p3[0], invzc, cam->cx);
        const float v = fmaf(cam->fy * p3[1], invzc, cam->cy);
        if (u < cam->min_x || u > cam->max_x) continue;                 /* :1509-1512 */
        if (v < cam->min_y || v > cam->max_y) continue;
        /* dist3D = cv::norm(x3Dw - Ow): float differences, squares summed in double */
        const float d0 = X[0] - Ow[0], d1 = X[1] - Ow[1], d2 = X[2] - Ow[2];
        double ss = 0.0;
        ss += (double)d0 * (double)d0;
        ss += (double)d1 * (double)d1;
        ss += (double)d2 * (double)d2;
        const float dist3D = (float)sqrt(ss);
        const float maxDistance = 1.2f * kf->max_dist[i];                /* MapPoint.cc:373-383 */
        const float minDistance = 0.8f * kf->min_dist[i];
        if (dist3D < minDistance || dist3D > maxDistance) continue;     /* :1522-1523 */
        const int lvl = predict_scale(kf->max_dist[i], dist3D, log_sf, cam->nlevels);
        const float radius = th * cam->scale[lvl];
        const int nc = oc_features_in_area(cam, cur->keys_un, &g, u, v, radius, lvl - 1, lvl + 1, cand, cur->n);
        if (nc == 0) continue;
        const uint8_t* dMP = &kf->desc[32 * i];
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = cand[c];
            if (taken[i2]) continue;                                    /* :1545-1546 */
            const int dist = oc_descriptor_distance(dMP, &cur->desc[32 * i2]);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        }
        if (bestDist <= orb_dist) {                                     /* :1556-1574 */
            taken[bestIdx2] = 1;
            match_out[bestIdx2] = i;
            nmatches++;
            if (check_ori) {
                float rot = kf->angle[i] - cur->keys_un[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                hist_items[nhist] = bestIdx2;
                hist_bin[nhist] = bin;
                nhist++;
            }
        }
    }
    if (check_ori) {                                                    /* :1580-1597 */
        int hist[HISTO_LENGTH] = {0};
        for (int k = 0; k < nhist; k++) hist[hist_bin[k]]++;
        int i1, i2, i3;
        three_maxima(hist, HISTO_LENGTH, &i1, &i2, &i3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == i1 || b == i2 || b == i3) continue;
            for (int k = 0; k < nhist; k++)
                if (hist_bin[k] == b) { match_out[hist_items[k]] = -1; nmatches--; }
        }
    }
    free(cand);
    free(hist_items);
    free(taken);
    free(g.cell_start);
    free(g.cell_idx);
    return nmatches;
}

/* ======================= TrackLocalMap's local map (batch chain) ======================= */
/* x = R*X + t for a row-major 4x4 T, as the cv::Mat expression R*X + t evaluates it (one gemm
 * with the addend: small-matrix float products, the addend added in double), the form
 * oc_search_by_projection uses for Rcw*x3Dw+tcw. */
static void small_gemm_add(const float* T, const float* X, float* out)
{
    for (int k = 0; k < 3; k++) {
        float t = T[k * 4 + 0] * X[0] + T[k * 4 + 1] * X[1];
        t = t + T[k * 4 + 2] * X[2];
        out[k] = (float)((double)t + (double)T[k * 4 + 3]);
    }
}

/* cv::norm of a float 3-vector: float components squared and summed in double */
static double norm3(const float* d)
{
    double ss = 0.0;
    ss += (double)d[0] * (double)d[0];
    ss += (double)d[1] * (double)d[1];
    ss += (double)d[2] * (double)d[2];
    return sqrt(ss);
}

void oc_mappoint_normal_depth(const oc_camera* cam, const float P[3], const float Ow[3], int octave,
                              float normal[3], float* max_dist, float* min_dist)
{
    const float d[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
    const double nd = norm3(d);
    for (int k = 0; k < 3; k++) normal[k] = (float)((double)d[k] / nd);
    const float dist = (float)nd;
    *max_dist = dist * cam->scale[octave];                           /* MapPoint.cc:367 */
    *min_dist = *max_dist / cam->scale[cam->nlevels - 1];            /* :368 */
}

int oc_is_in_frustum(const oc_camera* cam, const float Tcw[16], const float P[3], const float Pn[3],
                     float max_dist, float min_dist, float cos_limit,
                     float* proj_x, float* proj_y, float* proj_xr, int32_t* level, float* view_cos)
{
    const float* T = Tcw;
    float Pc[3];
    small_gemm_add(T, P, Pc);                                        /* Pc = mRcw*P + mtcw (:453) */
    if (Pc[2] < 0.0f) return 0;                                      /* :459-460 */
    const float invz = 1.0f / Pc[2];                                 /* :463 */
    const float u = fmaf(cam->fx * Pc[0], invz, cam->cx);            /* :464-465, fused */
    const float v = fmaf(cam->fy * Pc[1], invz, cam->cy);
    if (u < cam->min_x || u > cam->max_x) return 0;                  /* :467-470 */
    if (v < cam->min_y || v > cam->max_y) return 0;
    /* mOw = -mRcw.t()*mtcw (Frame.cc:442; GEMM_1_T, double accumulation) */
    float Ow[3];
    for (int k = 0; k < 3; k++) {
        double s = (double)T[0 * 4 + k] * T[3] + (double)T[1 * 4 + k] * T[7];
        s = s + (double)T[2 * 4 + k] * T[11];
        Ow[k] = (float)(s * -1.0);
    }
    const float maxDistance = 1.2f * max_dist;                       /* :473-474, MapPoint.cc:373-383 */
    const float minDistance = 0.8f * min_dist;
    const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};  /* :475 */
    const float dist = (float)norm3(PO);                             /* :476 */
    if (dist < minDistance || dist > maxDistance) return 0;          /* :478-479 */
    /* PO.dot(Pn) / dist: Mat::dot of floats accumulates in double (:484) */
    double dot = 0.0;
    dot += (double)PO[0] * (double)Pn[0];
    dot += (double)PO[1] * (double)Pn[1];
    dot += (double)PO[2] * (double)Pn[2];
    const float viewCos = (float)(dot / (double)dist);
    if (viewCos < cos_limit) return 0;                               /* :486-487 */
    const float log_sf = cam->nlevels > 1 ? canon_logf(cam->scale[1]) : 1.0f;
    *level = predict_scale(max_dist, dist, log_sf, cam->nlevels);   /* :490 */
    *proj_x = u;                                                     /* :493-498 */
    *proj_xr = fmaf(-cam->bf, invz, u);                              /* u - mbf*invz, fused */
    *proj_y = v;
    *view_cos = viewCos;
    return 1;
}

int oc_local_map_build(const oc_camera* cam, const oc_kfview* kf2, const float T_kf1_kf2[16], const oc_kfview* kf1,
                       const uint8_t* seen1, int32_t nobs, int stride, const float Tcw_cur[16], float cos_limit,
                       uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr, int32_t* level,
                       float* view_cos, int32_t* nobs_out, float* xw_out)
{
    int nin = 0;
    for (int q = 0; q < 2 * stride; q++) {
        in_view[q] = 0;
        level[q] = 0;
        nobs_out[q] = nobs;
        const int second = q >= stride;
        const int j = second ? q - stride : q;
        const oc_kfview* kf = second ? kf1 : kf2;
        if (!kf || j >= kf->n || !kf->has[j]) continue;
        if (second && seen1 && seen1[j]) continue;                   /* Tracking.cc:1249-1250 */
        float P[3], Ow[3];
        const float* X = &kf->xw[3 * j];
        if (second) {                                                /* KF1 is the world frame */
            P[0] = X[0]; P[1] = X[1]; P[2] = X[2];
            Ow[0] = Ow[1] = Ow[2] = 0.0f;
        } else {                                                     /* UnprojectStereo with KF2's Twc */
            small_gemm_add(T_kf1_kf2, X, P);
            Ow[0] = T_kf1_kf2[3]; Ow[1] = T_kf1_kf2[7]; Ow[2] = T_kf1_kf2[11];
        }
        float Pn[3], maxd, mind;
        oc_mappoint_normal_depth(cam, P, Ow, kf->keys[j].octave, Pn, &maxd, &mind);
        xw_out[3 * q + 0] = P[0]; xw_out[3 * q + 1] = P[1]; xw_out[3 * q + 2] = P[2];
        int32_t lvl;
        float px, py, pxr, vc;
        if (oc_is_in_frustum(cam, Tcw_cur, P, Pn, maxd, mind, cos_limit, &px, &py, &pxr, &lvl, &vc)) {
            in_view[q] = 1;
            proj_x[q] = px; proj_y[q] = py; proj_xr[q] = pxr; level[q] = lvl; view_cos[q] = vc;
            nin++;
        }
    }
    return nin;
}

/* ======================= Optimizer::PoseOptimization (canonical g2o) ======================= */
/* SE3Quat as g2o holds it: unit quaternion (w, x, y, z) and translation, doubles.  Every
 * operation below has a fixed evaluation order; the HIP kernel (csrc/coeb_pose.hip) performs
 * the same operations in the same order. */
typedef struct { double w, x, y, z, t[3]; } oc_se3;

/* Quaterniond(const Matrix3d&) (Eigen quaternionbase_assign_impl) */
static void pq_from_R(const double R[9], oc_se3* s)
{
    double t = (R[0] + R[4]) + R[8];
    double q[4];                     /* x, y, z, w */
    if (t > 0.0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (R[7] - R[5]) * t;
        q[1] = (R[2] - R[6]) * t;
        q[2] = (R[3] - R[1]) * t;
    } else {
        int i = 0;
        if (R[4] > R[0]) i = 1;
        if (R[8] > R[i * 4]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(((R[i * 4] - R[j * 4]) - R[k * 4]) + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (R[k * 3 + j] - R[j * 3 + k]) * t;
        q[j] = (R[j * 3 + i] + R[i * 3 + j]) * t;
        q[k] = (R[k * 3 + i] + R[i * 3 + k]) * t;
    }
    s->x = q[0]; s->y = q[1]; s->z = q[2]; s->w = q[3];
}

/* SE3Quat::normalizeRotation: w >= 0, unit norm */
static void pq_normalize(oc_se3* s)
{
    if (s->w < 0) { s->w = -s->w; s->x = -s->x; s->y = -s->y; s->z = -s->z; }
    const double n = sqrt(((s->x * s->x + s->y * s->y) + s->z * s->z) + s->w * s->w);
    s->x = s->x / n; s->y = s->y / n; s->z = s->z / n; s->w = s->w / n;
}

/* q * v (Eigen _transformVector: uv = 2 q.vec x v; v + w uv + q.vec x uv) */
static void pq_rotate(const oc_se3* s, const double v[3], double o[3])
{
    double uv[3] = {s->y * v[2] - s->z * v[1], s->z * v[0] - s->x * v[2], s->x * v[1] - s->y * v[0]};
    uv[0] = uv[0] + uv[0]; uv[1] = uv[1] + uv[1]; uv[2] = uv[2] + uv[2];
    const double c[3] = {s->y * uv[2] - s->z * uv[1], s->z * uv[0] - s->x * uv[2], s->x * uv[1] - s->y * uv[0]};
    for (int k = 0; k < 3; k++) o[k] = (v[k] + s->w * uv[k]) + c[k];
}

static void pq_map(const oc_se3* s, const double X[3], double o[3])
{
    pq_rotate(s, X, o);
    for (int k = 0; k < 3; k++) o[k] = o[k] + s->t[k];
}

/* a * b (SE3Quat::operator*: t = a.t + a.q b.t, q = a.q b.q, normalise) */
static oc_se3 pq_mul(const oc_se3* a, const oc_se3* b)
{
    oc_se3 r;
    double bt[3];
    pq_rotate(a, b->t, bt);
    for (int k = 0; k < 3; k++) r.t[k] = a->t[k] + bt[k];
    r.w = ((a->w * b->w - a->x * b->x) - a->y * b->y) - a->z * b->z;
    r.x = ((a->w * b->x + a->x * b->w) + a->y * b->z) - a->z * b->y;
    r.y = ((a->w * b->y + a->y * b->w) + a->z * b->x) - a->x * b->z;
    r.z = ((a->w * b->z + a->z * b->w) + a->x * b->y) - a->y * b->x;
    pq_normalize(&r);
    return r;
}

/* canonical sin/cos: Cody-Waite pi/2 reduction, Taylor series to r^27 on
 * |r| <= pi/4 by Horner; coefficients (-1)^n / (2n+1)! and (-1)^n / (2n)! as double
 * products of the integers, rounded once (hex literals shared with the HIP twin). */
static const double kPqSin[14] = {0x1.0000000000000p+0, -0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13, 0x1.71de3a556c734p-19, -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33, -0x1.ae7f3e733b81fp-41, 0x1.952c77030ad4ap-49, -0x1.2f49b46814157p-57, 0x1.71b8ef6dcf572p-66, -0x1.761b413163819p-75, 0x1.3f3ccdd165fa9p-84, -0x1.d1ab1c2dccea3p-94};
static const double kPqCos[14] = {0x1.0000000000000p+0, -0x1.0000000000000p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-16, -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29, -0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-45, -0x1.6827863b97d97p-53, 0x1.e542ba4020225p-62, -0x1.0ce396db7f853p-70, 0x1.f2cf01972f578p-80, -0x1.88e85fc6a4e59p-89};
static void pq_sincos(double x, double* sn, double* cs)
{
    const double k = floor(x * 0.63661977236758134308 + 0.5);
    const double r = (x - k * 1.57079632673412561417e+00) - k * 6.07710050650619224932e-11;
    const double r2 = r * r;
    double ps = kPqSin[13], pc = kPqCos[13];
    for (int n = 12; n >= 0; n--) {
        ps = ps * r2 + kPqSin[n];
        pc = pc * r2 + kPqCos[n];
    }
    const double s0 = r * ps, c0 = pc;
    const int q = ((int)(long)k) & 3;
    if (q == 0) { *sn = s0; *cs = c0; }
    else if (q == 1) { *sn = c0; *cs = -s0; }
    else if (q == 2) { *sn = -s0; *cs = -c0; }
    else { *sn = -c0; *cs = s0; }
}

/* SE3Quat::exp(update), update = (omega, upsilon) */
static oc_se3 pq_exp(const double u[6])
{
    const double o0 = u[0], o1 = u[1], o2 = u[2];
    const double theta = sqrt((o0 * o0 + o1 * o1) + o2 * o2);
    const double Om[9] = {0.0, -o2, o1, o2, 0.0, -o0, -o1, o0, 0.0};
    double Om2[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            Om2[i * 3 + j] = (Om[i * 3] * Om[j] + Om[i * 3 + 1] * Om[3 + j]) + Om[i * 3 + 2] * Om[6 + j];
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = ((i % 4 == 0 ? 1.0 : 0.0) + Om[i]) + Om2[i];
        for (int i = 0; i < 9; i++) V[i] = R[i];
    } else {
        double sn, cs;
        pq_sincos(theta, &sn, &cs);
        const double th2 = theta * theta;
        const double A = sn / theta, B = (1.0 - cs) / th2, Cc = (theta - sn) / (th2 * theta);
        for (int i = 0; i < 9; i++) {
            const double I = i % 4 == 0 ? 1.0 : 0.0;
            R[i] = (I + A * Om[i]) + B * Om2[i];
            V[i] = (I + B * Om[i]) + Cc * Om2[i];
        }
    }
    oc_se3 s;
    pq_from_R(R, &s);
    for (int i = 0; i < 3; i++) s.t[i] = (V[i * 3] * u[3] + V[i * 3 + 1] * u[4]) + V[i * 3 + 2] * u[5];
    pq_normalize(&s);
    return s;
}

/* Converter::toSE3Quat(cv::Mat float) */
static oc_se3 pq_from_Tcw(const float T[16])
{
    double R[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i * 3 + j] = (double)T[i * 4 + j];
    oc_se3 s;
    pq_from_R(R, &s);
    for (int i = 0; i < 3; i++) s.t[i] = (double)T[i * 4 + 3];
    pq_normalize(&s);
    return s;
}

/* Converter::toCvMat(SE3Quat): to_homogeneous_matrix (Eigen toRotationMatrix), cast to float */
static void pq_to_Tcw(const oc_se3* s, float T[16])
{
    const double tx = 2.0 * s->x, ty = 2.0 * s->y, tz = 2.0 * s->z;
    const double twx = tx * s->w, twy = ty * s->w, twz = tz * s->w;
    const double txx = tx * s->x, txy = ty * s->x, txz = tz * s->x;
    const double tyy = ty * s->y, tyz = tz * s->y, tzz = tz * s->z;
    const double R[9] = {1.0 - (tyy + tzz), txy - twz, txz + twy,
                         txy + twz, 1.0 - (txx + tzz), tyz - twx,
                         txz - twy, tyz + twx, 1.0 - (txx + tyy)};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[i * 4 + j] = (float)R[i * 3 + j];
        T[i * 4 + 3] = (float)s->t[i];
    }
    T[12] = 0.f; T[13] = 0.f; T[14] = 0.f; T[15] = 1.f;
}

/* One edge at pose s: error e (2 or 3), raw chi2 = e' Omega e (EdgeSE3ProjectXYZOnlyPose /
 * EdgeStereoSE3ProjectXYZOnlyPose::computeError, ORB-SLAM2 types_six_dof_expmap.cpp); J (the
 * error Jacobian linearizeOplus, rows 6 wide) when J != NULL. */
typedef struct { double X[3], obs[3], w; int stereo; } pq_edge;

static double pq_edge_eval(const oc_pose_frame* fr, const oc_se3* s, const pq_edge* E, double e[3], double* J)
{
    double p[3];
    pq_map(s, E->X, p);
    const double fx = fr->fx, fy = fr->fy, cx = fr->cx, cy = fr->cy, bf = fr->bf;
    if (!E->stereo) {
        const double u = (p[0] / p[2]) * fx + cx, v = (p[1] / p[2]) * fy + cy;   /* project2d, cam_project */
        e[0] = E->obs[0] - u; e[1] = E->obs[1] - v; e[2] = 0.0;
    } else {
        const float invzf = 1.0f / (float)p[2];                  /* const float invz = 1.0f/z */
        const double u = (p[0] * (double)invzf) * fx + cx, v = (p[1] * (double)invzf) * fy + cy;
        const double ur = u - bf * (double)invzf;
        e[0] = E->obs[0] - u; e[1] = E->obs[1] - v; e[2] = E->obs[2] - ur;
    }
    if (J) {
        const double x = p[0], y = p[1], invz = 1.0 / p[2], invz_2 = invz * invz;
        J[0] = ((x * y) * invz_2) * fx;
        J[1] = -(1.0 + ((x * x) * invz_2)) * fx;
        J[2] = (y * invz) * fx;
        J[3] = -invz * fx;
        J[4] = 0.0;
        J[5] = (x * invz_2) * fx;
        J[6] = (1.0 + ((y * y) * invz_2)) * fy;
        J[7] = -((x * y) * invz_2) * fy;
        J[8] = -(x * invz) * fy;
        J[9] = 0.0;
        J[10] = -invz * fy;
        J[11] = (y * invz_2) * fy;
        if (E->stereo) {
            J[12] = J[0] - (bf * y) * invz_2;
            J[13] = J[1] + (bf * x) * invz_2;
            J[14] = J[2];
            J[15] = J[3];
            J[16] = 0.0;
            J[17] = J[5] - bf * invz_2;
        }
    }
    double c = e[0] * (E->w * e[0]) + e[1] * (E->w * e[1]);
    if (E->stereo) c = c + e[2] * (E->w * e[2]);
    return c;
}

/* RobustKernelHuber::robustify */
static void pq_huber(double e2, double delta, double rho[2])
{
    const double dsqr = delta * delta;
    if (e2 <= dsqr) { rho[0] = e2; rho[1] = 1.0; }
    else {
        const double sq = sqrt(e2);
        rho[0] = (2.0 * sq) * delta - dsqr;
        rho[1] = delta / sq;
    }
}

/* The fixed reduction of per-edge terms: edge i -> lane i % 256 (sequential in i, from 0.0);
 * each run of 32 lanes summed in lane order from 0.0; the 8 run sums added in order. */
enum { PQ_LANES = 256, PQ_NV = 28 };
static void pq_reduce(double lanes[PQ_LANES][PQ_NV], int nv, double out[PQ_NV])
{
    for (int k = 0; k < nv; k++) {
        double run[8];
        for (int c = 0; c < 8; c++) {
            double p = 0.0;
            for (int l = 32 * c; l < 32 * c + 32; l++) p = p + lanes[l][k];
            run[c] = p;
        }
        double t = run[0];
        for (int c = 1; c < 8; c++) t = t + run[c];
        out[k] = t;
    }
}

/* LDL' of the 6x6 (no pivoting; fails unless every pivot > 0), then solve */
/* g2o OptimizationAlgorithmLevenberg::solve: alpha = 1 - pow(2*rho - 1, 3).  glibc pow is
   correctly rounded; t^3 is formed exactly as a double-double (t*t = h + l by fma, then
   (h + l)*t = h2 + l2 + l*t) and rounded once, which equals the correctly rounded cube except
   in ties closer than 2^-100 relative. */
static double pq_cube(double t)
{
    const double h = t * t, l = fma(t, t, -h);
    const double h2 = h * t, l2 = fma(h, t, -h2);
    return h2 + fma(l, t, l2);
}

static int pq_solve6(const double H[36], const double b[6], double x[6])
{
    double L[36] = {0}, d[6], y[6];
    for (int j = 0; j < 6; j++) {
        double v = H[j * 6 + j];
        for (int k = 0; k < j; k++) v = v - (L[j * 6 + k] * L[j * 6 + k]) * d[k];
        if (!(v > 0.0)) return 0;
        d[j] = v;
        for (int i = j + 1; i < 6; i++) {
            double w = H[i * 6 + j];
            for (int k = 0; k < j; k++) w = w - (L[i * 6 + k] * L[j * 6 + k]) * d[k];
            L[i * 6 + j] = w / d[j];
        }
    }
    for (int i = 0; i < 6; i++) {
        double v = b[i];
        for (int k = 0; k < i; k++) v = v - L[i * 6 + k] * y[k];
        y[i] = v;
    }
    for (int i = 0; i < 6; i++) y[i] = y[i] / d[i];
    for (int i = 5; i >= 0; i--) {
        double v = y[i];
        for (int k = i + 1; k < 6; k++) v = v - L[k * 6 + i] * x[k];
        x[i] = v;
    }
    return 1;
}

/* robust chi2 of the active edges at s (SparseOptimizer::computeActiveErrors +
 * activeRobustChi2); stores every active edge's raw chi2 in chi2_last */
static double pq_active_chi2(const oc_pose_frame* fr, const oc_se3* s, const pq_edge* E, int ne, const uint8_t* active,
                             int robust, const double* delta, double* chi2_last)
{
    static _Thread_local double lanes[PQ_LANES][PQ_NV];
    memset(lanes, 0, sizeof(lanes));
    for (int i = 0; i < ne; i++) {
        if (!active[i]) continue;
        double e[3];
        const double c = pq_edge_eval(fr, s, &E[i], e, NULL);
        chi2_last[i] = c;
        double r = c;
        if (robust) { double rho[2]; pq_huber(c, delta[E[i].stereo], rho); r = rho[0]; }
        lanes[i % PQ_LANES][0] += r;
    }
    double out[PQ_NV];
    pq_reduce(lanes, 1, out);
    return out[0];
}

/* LM iterations and trials of the last oc_pose_optimization call on this thread (a KAT hook) */
static _Thread_local int pq_stat_iters, pq_stat_trials;

void oc_pose_last_stats(int* iterations, int* trials)
{
    *iterations = pq_stat_iters;
    *trials = pq_stat_trials;
}

/* one SparseOptimizer::optimize(10) with OptimizationAlgorithmLevenberg (g2o 2012) */
static void pq_optimize(const oc_pose_frame* fr, oc_se3* s, const pq_edge* E, int ne, const uint8_t* active, int robust,
                        const double* delta, double* chi2_last, int iterations)
{
    static _Thread_local double lanes[PQ_LANES][PQ_NV];
    double lambda = 0.0, ni = 2.0;
    for (int it = 0; it < iterations; it++) {
        pq_stat_iters++;
        /* computeActiveErrors, activeRobustChi2, buildSystem (H = sum J' w rho1 J, b = -sum J' w rho1 e) */
        double currentChi = pq_active_chi2(fr, s, E, ne, active, robust, delta, chi2_last);
        memset(lanes, 0, sizeof(lanes));
        for (int i = 0; i < ne; i++) {
            if (!active[i]) continue;
            double e[3], J[18];
            const double c = pq_edge_eval(fr, s, &E[i], e, J);
            double rho1 = 1.0;
            if (robust) { double rho[2]; pq_huber(c, delta[E[i].stereo], rho); rho1 = rho[1]; }
            const double wgt = rho1 * E[i].w;
            const int nr = E[i].stereo ? 3 : 2;
            double* L = lanes[i % PQ_LANES];
            int k = 0;
            for (int a = 0; a < 6; a++)
                for (int bb = a; bb < 6; bb++) {
                    double c2 = J[a] * J[bb] + J[6 + a] * J[6 + bb];
                    if (nr == 3) c2 = c2 + J[12 + a] * J[12 + bb];
                    L[k++] += wgt * c2;
                }
            for (int a = 0; a < 6; a++) {
                double c1 = J[a] * e[0] + J[6 + a] * e[1];
                if (nr == 3) c1 = c1 + J[12 + a] * e[2];
                L[21 + a] += -(wgt * c1);
            }
        }
        double red[PQ_NV];
        pq_reduce(lanes, 27, red);
        double H[36], b[6];
        {
            int k = 0;
            for (int a = 0; a < 6; a++)
                for (int bb = a; bb < 6; bb++) { H[a * 6 + bb] = red[k]; H[bb * 6 + a] = red[k]; k++; }
            for (int a = 0; a < 6; a++) b[a] = red[21 + a];
        }
        if (it == 0) {                                   /* computeLambdaInit: tau * max |H_jj| */
            double m = 0.0;
            for (int j = 0; j < 6; j++) m = fmax(fabs(H[j * 6 + j]), m);
            lambda = 1e-5 * m;
            ni = 2.0;
        }
        double rho = 0.0;
        int qmax = 0;
        do {
            const oc_se3 saved = *s;                     /* push */
            double Hl[36], x[6] = {0, 0, 0, 0, 0, 0};
            memcpy(Hl, H, sizeof(Hl));
            for (int j = 0; j < 6; j++) Hl[j * 6 + j] = Hl[j * 6 + j] + lambda;
            const int ok2 = pq_solve6(Hl, b, x);
            if (!ok2) for (int j = 0; j < 6; j++) x[j] = 0.0;
            const oc_se3 up = pq_exp(x);                 /* VertexSE3Expmap::oplusImpl */
            *s = pq_mul(&up, s);
            double tempChi = pq_active_chi2(fr, s, E, ne, active, robust, delta, chi2_last);
            if (!ok2) tempChi = DBL_MAX;
            double scale = 0.0;                          /* computeScale */
            for (int j = 0; j < 6; j++) scale = scale + x[j] * (lambda * x[j] + b[j]);
            scale = scale + 1e-3;                        /* g2o: "make sure it's non-zero" */
            rho = (currentChi - tempChi) / scale;
            if (rho > 0 && isfinite(tempChi)) {
                double alpha = 1.0 - pq_cube(2.0 * rho - 1.0);
                alpha = fmin(alpha, 2.0 / 3.0);
                const double sf = fmax(1.0 / 3.0, alpha);
                lambda = lambda * sf;
                ni = 2.0;
                currentChi = tempChi;
            } else {
                lambda = lambda * ni;
                ni = ni * 2.0;
                *s = saved;                              /* pop */
            }
            qmax++;
            pq_stat_trials++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0) break;               /* Terminate */
    }
}

int oc_pose_optimization(const oc_pose_frame* fr, float Tcw[16], uint8_t* outlier)
{
    const int n = fr->n;
    pq_stat_iters = pq_stat_trials = 0;
    pq_edge* E = (pq_edge*)malloc(sizeof(pq_edge) * (n > 0 ? n : 1));
    int* idx = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
    int ne = 0;
    for (int i = 0; i < n; i++) {
        if (!fr->has_mp[i]) continue;
        pq_edge* e = &E[ne];
        for (int k = 0; k < 3; k++) e->X[k] = (double)fr->xw[3 * i + k];
        e->obs[0] = (double)fr->keys_un[i].x;
        e->obs[1] = (double)fr->keys_un[i].y;
        e->stereo = !(fr->uright[i] < 0);                /* Optimizer.cc:287 */
        e->obs[2] = e->stereo ? (double)fr->uright[i] : 0.0;
        e->w = (double)fr->inv_sigma2[fr->keys_un[i].octave];
        outlier[i] = 0;
        idx[ne++] = i;
    }
    if (ne < 3) { free(E); free(idx); return 0; }
    const float deltaMono = (float)sqrt(5.991), deltaStereo = (float)sqrt(7.815);
    const double delta[2] = {(double)deltaMono, (double)deltaStereo};
    const float chi2Mono = 5.991f, chi2Stereo = 7.815f;
    uint8_t* active = (uint8_t*)malloc(ne);
    double* chi2_last = (double*)malloc(sizeof(double) * ne);
    for (int i = 0; i < ne; i++) { active[i] = 1; chi2_last[i] = 0.0; }
    const oc_se3 s0 = pq_from_Tcw(Tcw);
    oc_se3 s = s0;
    int nBad = 0;
    for (int it = 0; it < 4; it++) {
        s = s0;                                          /* setEstimate(toSE3Quat(pFrame->mTcw)) */
        const int robust = it < 3;                       /* setRobustKernel(0) after round 2 */
        pq_optimize(fr, &s, E, ne, active, robust, delta, chi2_last, 10);
        nBad = 0;
        for (int i = 0; i < ne; i++) {
            double c = chi2_last[i];
            if (!active[i]) { double e[3]; c = pq_edge_eval(fr, &s, &E[i], e, NULL); chi2_last[i] = c; }
            const double th = E[i].stereo ? (double)chi2Stereo : (double)chi2Mono;
            if (c > th) { outlier[idx[i]] = 1; active[i] = 0; nBad++; }
            else { outlier[idx[i]] = 0; active[i] = 1; }
        }
        if (ne < 10) break;                              /* optimizer.edges().size() < 10 */
    }
    pq_to_Tcw(&s, Tcw);
    free(active); free(chi2_last); free(E); free(idx);
    return ne - nBad;
}

/* ======================= Frame::UndistortKeyPoints ======================= */
void oc_undistort_keypoints(const oc_kp* in, int n, float fx_f, float fy_f, float cx_f, float cy_f, const float dist[5],
                            oc_kp* out)
{
    for (int i = 0; i < n; i++) out[i] = in[i];
    if (dist[0] == 0.0f) return;                                   /* mDistCoef.at<float>(0) == 0.0 */
    double k[12] = {0};
    for (int q = 0; q < 5; q++) k[q] = (double)dist[q];
    const double fx = fx_f, fy = fy_f, cx = cx_f, cy = cy_f;
    const double ifx = 1. / fx, ify = 1. / fy;
    for (int i = 0; i < n; i++) {
        double x = (double)in[i].x, y = (double)in[i].y;
        x = (x - cx) * ifx;
        y = (y - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; j++) {                                /* TermCriteria(COUNT, 5, 0.01) */
            const double r2 = x * x + y * y;
            const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            const double deltaX = ((((2 * k[2]) * x) * y + k[3] * (r2 + (2 * x) * x)) + k[8] * r2) + (k[9] * r2) * r2;
            const double deltaY = ((k[2] * (r2 + (2 * y) * y) + ((2 * k[3]) * x) * y) + k[10] * r2) + (k[11] * r2) * r2;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        /* P = mK, R = I: xx = fx x + cx, yy = fy y + cy, ww = 1 */
        out[i].x = (float)(fx * x + cx);
        out[i].y = (float)(fy * y + cy);
    }
}

/* ======================= goodFeaturesToTrack (Harris) ======================= */
static int gf_reflect(int p, int n)                 /* BORDER_REFLECT_101 */
{
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - p - 2;
    return p;
}

/* Harris response at (x, y): Sobel 3x3 scaled by 1/(4 * 3 * 255) (cornerEigenValsVecs),
 * cov = (dx*dx, dx*dy, dy*dy), unnormalised 3x3 box (row sums, then column sum),
 * R = a*c - b*b - k*(a+c)^2 with k double (calcHarris). */
static float gf_response(const uint8_t* img, int w, int h, int stride, int x, int y, double k)
{
    const double scale = 1.0 / (4.0 * 3.0 * 255.0);
    float A[3][3], B[3][3], C[3][3];
    for (int j = 0; j < 3; j++) {
        const int yy = gf_reflect(y + j - 1, h);
        for (int i = 0; i < 3; i++) {
            const int xx = gf_reflect(x + i - 1, w);
            int p[3][3];
            for (int b = 0; b < 3; b++)
                for (int a = 0; a < 3; a++)
                    p[b][a] = img[(size_t)gf_reflect(yy + b - 1, h) * stride + gf_reflect(xx + a - 1, w)];
            const int gx = (p[0][2] - p[0][0]) + 2 * (p[1][2] - p[1][0]) + (p[2][2] - p[2][0]);
            const int gy = (p[2][0] - p[0][0]) + 2 * (p[2][1] - p[0][1]) + (p[2][2] - p[0][2]);
            const float dx = (float)((double)gx * scale), dy = (float)((double)gy * scale);
            A[j][i] = dx * dx; B[j][i] = dx * dy; C[j][i] = dy * dy;
        }
    }
    float sa[3], sb[3], sc[3];
    for (int j = 0; j < 3; j++) {
        sa[j] = (A[j][0] + A[j][1]) + A[j][2];
        sb[j] = (B[j][0] + B[j][1]) + B[j][2];
        sc[j] = (C[j][0] + C[j][1]) + C[j][2];
    }
    const float a = (sa[0] + sa[1]) + sa[2], b = (sb[0] + sb[1]) + sb[2], c = (sc[0] + sc[1]) + sc[2];
    const float ac = a * c - b * b, apc = a + c;
    return (float)((double)ac - (k * (double)apc) * (double)apc);
}

typedef struct { float v; int idx; } gf_cand;

static int gf_cmp(const void* pa, const void* pb)     /* greaterThanPtr: value desc, address desc */
{
    const gf_cand* a = (const gf_cand*)pa;
    const gf_cand* b = (const gf_cand*)pb;
    if (a->v > b->v) return -1;
    if (a->v < b->v) return 1;
    return a->idx > b->idx ? -1 : (a->idx < b->idx ? 1 : 0);
}

int oc_good_features_harris(const uint8_t* img, int w, int h, int stride, int max_corners, double quality,
                            double min_distance, double k, float* out_xy, int cap, int max_cand)
{
    if (w <= 0 || h <= 0) return 0;
    float* eig = (float*)malloc(sizeof(float) * (size_t)w * h);
    float maxv = -FLT_MAX;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const float r = gf_response(img, w, h, stride, x, y, k);
            eig[(size_t)y * w + x] = r;
            if (r > maxv) maxv = r;
        }
    const float thr = (float)((double)maxv * quality);             /* threshold TOZERO */
    for (size_t i = 0; i < (size_t)w * h; i++)
        if (!(eig[i] > thr)) eig[i] = 0.f;
    gf_cand* cand = (gf_cand*)malloc(sizeof(gf_cand) * (size_t)w * h);
    int nc = 0;
    for (int y = 1; y < h - 1; y++)
        for (int x = 1; x < w - 1; x++) {
            const float v = eig[(size_t)y * w + x];
            if (v == 0.f) continue;
            float m = v;                                              /* dilate 3x3 */
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    const float u = eig[(size_t)(y + dy) * w + x + dx];
                    if (u > m) m = u;
                }
            if (v == m) { cand[nc].v = v; cand[nc].idx = y * w + x; nc++; }
        }
    free(eig);
    if (nc > max_cand) { free(cand); return -1; }
    qsort(cand, (size_t)nc, sizeof(gf_cand), gf_cmp);
    const int cell = (int)lrint(min_distance);                       /* cvRound */
    const int gw = (w + cell - 1) / cell, gh = (h + cell - 1) / cell;
    const double md2 = min_distance * min_distance;
    int* gcnt = (int*)calloc((size_t)gw * gh, sizeof(int));
    float* gpt = (float*)malloc(sizeof(float) * 2 * 16 * (size_t)gw * gh);   /* <= 16 per cell */
    int n = 0;
    for (int i = 0; i < nc && (max_corners <= 0 || n < max_corners); i++) {
        const int y = cand[i].idx / w, x = cand[i].idx - y * w;
        const int xc = x / cell, yc = y / cell;
        int good = 1;
        for (int yy = (yc - 1 > 0 ? yc - 1 : 0); good && yy <= (yc + 1 < gh - 1 ? yc + 1 : gh - 1); yy++)
            for (int xx = (xc - 1 > 0 ? xc - 1 : 0); good && xx <= (xc + 1 < gw - 1 ? xc + 1 : gw - 1); xx++) {
                const int g = yy * gw + xx;
                for (int j = 0; j < gcnt[g]; j++) {
                    const float ddx = (float)x - gpt[(g * 16 + j) * 2], ddy = (float)y - gpt[(g * 16 + j) * 2 + 1];
                    if ((double)(ddx * ddx + ddy * ddy) < md2) { good = 0; break; }
                }
            }
        if (good) {
            const int g = yc * gw + xc;
            gpt[(g * 16 + gcnt[g]) * 2] = (float)x;
            gpt[(g * 16 + gcnt[g]) * 2 + 1] = (float)y;
            gcnt[g]++;
            if (n < cap) { out_xy[2 * n] = (float)x; out_xy[2 * n + 1] = (float)y; }
            n++;
        }
    }
    free(gcnt); free(gpt); free(cand);
    return n;
}

/* ======================= cornerSubPix (cornersubpix.cpp, OpenCV 3.4) ======================= */
static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* getRectSubPix(src 8U, Size(ww, wh), center, dst 32F): samplers.cpp getRectSubPix_8u32f when
 * the window (plus one column/row) is inside the image, else getRectSubPix_Cn_ (replicated
 * edges through adjustRect: clamped rows, 2-term edge columns). */
void oc_rect_subpix_8u32f(const uint8_t* img, int w, int h, int stride, int ww, int wh, float cx, float cy,
                          float* dst)
{
    const float ctrx = cx - (float)(ww - 1) * 0.5f, ctry = cy - (float)(wh - 1) * 0.5f;
    const int ipx = cv_floor(ctrx), ipy = cv_floor(ctry);
    if (ipx >= 0 && ipx + ww < w && ipy >= 0 && ipy + wh < h) {
        float a = ctrx - (float)ipx;
        const float b = ctry - (float)ipy;
        a = a < 0.0001f ? 0.0001f : a;
        const float a12 = a * (1.f - b), a22 = a * b, b1 = 1.f - b, b2 = b;
        const double s = (1. - (double)a) / (double)a;
        for (int r = 0; r < wh; r++) {
            const uint8_t* src = img + (size_t)(ipy + r) * stride + ipx;
            float prev = (1.f - a) * (b1 * (float)src[0] + b2 * (float)src[stride]);
            for (int j = 0; j < ww; j++) {
                const float t = a12 * (float)src[j + 1] + a22 * (float)src[j + 1 + stride];
                dst[r * ww + j] = prev + t;
                prev = (float)((double)t * s);
            }
        }
        return;
    }
    const float a = ctrx - (float)ipx, b = ctry - (float)ipy;
    const float a11 = (1.f - a) * (1.f - b), a12 = a * (1.f - b), a21 = (1.f - a) * b, a22 = a * b;
    const float b1 = 1.f - b, b2 = b;
    for (int r = 0; r < wh; r++) {
        const uint8_t* r0 = img + (size_t)clampi(ipy + r, 0, h - 1) * stride;
        const uint8_t* r1 = img + (size_t)clampi(ipy + r + 1, 0, h - 1) * stride;
        for (int j = 0; j < ww; j++) {
            const int c = ipx + j;
            float v;
            if (c < 0) v = (float)r0[0] * b1 + (float)r1[0] * b2;
            else if (c >= w - 1) v = (float)r0[w - 1] * b1 + (float)r1[w - 1] * b2;
            else v = (float)r0[c] * a11 + (float)r0[c + 1] * a12 + (float)r1[c] * a21 + (float)r1[c + 1] * a22;
            dst[r * ww + j] = v;
        }
    }
}

/* The cornerSubPix weight window: mask[i][j] = vy * expf(-x*x), vy = expf(-y*y),
 * y = (float)(i - win)/win (float division), as cornersubpix.cpp builds it. */
void oc_subpix_mask(int win, float* mask)
{
    const int n = 2 * win + 1;
    for (int i = 0; i < n; i++) {
        const float y = (float)(i - win) / (float)win;
        const float vy = expf(-y * y);
        for (int j = 0; j < n; j++) {
            const float x = (float)(j - win) / (float)win;
            mask[i * n + j] = vy * expf(-x * x);
        }
    }
}

/* cv::cornerSubPix(img, corners, Size(win, win), Size(-1,-1), TermCriteria(ITER|EPS, max_iter,
 * eps)) (Frame.cc:334), in place.  Sums in double in the reference's row-major order. */
void oc_corner_subpix(const uint8_t* img, int w, int h, int stride, float* xy, int n, int win, int max_iter,
                      double eps)
{
    const int ww = 2 * win + 1;
    float* mask = (float*)malloc(sizeof(float) * ww * ww);
    float* buf = (float*)malloc(sizeof(float) * (ww + 2) * (ww + 2));
    oc_subpix_mask(win, mask);
    const int iters = max_iter < 1 ? 1 : max_iter > 100 ? 100 : max_iter;
    const double eps2 = (eps > 0 ? eps : 0.) * (eps > 0 ? eps : 0.);
    for (int p = 0; p < n; p++) {
        const float tx = xy[2 * p], ty = xy[2 * p + 1];
        float cx = tx, cy = ty;
        int it = 0;
        double err = 0;
        do {
            double a = 0, b = 0, c = 0, bb1 = 0, bb2 = 0;
            oc_rect_subpix_8u32f(img, w, h, stride, ww + 2, ww + 2, cx, cy, buf);
            for (int i = 0, k = 0; i < ww; i++) {
                const float* sp = buf + (i + 1) * (ww + 2) + 1;
                const double py = i - win;
                for (int j = 0; j < ww; j++, k++) {
                    const double m = mask[k];
                    const double tgx = (double)(sp[j + 1] - sp[j - 1]);
                    const double tgy = (double)(sp[j + ww + 2] - sp[j - ww - 2]);
                    const double gxx = tgx * tgx * m, gxy = tgx * tgy * m, gyy = tgy * tgy * m;
                    const double px = j - win;
                    a += gxx; b += gxy; c += gyy;
                    bb1 += gxx * px + gxy * py;
                    bb2 += gxy * px + gyy * py;
                }
            }
            const double det = a * c - b * b;
            if (fabs(det) <= DBL_EPSILON * DBL_EPSILON) break;
            const double scale = 1.0 / det;
            const float nx = (float)((double)cx + c * scale * bb1 - b * scale * bb2);
            const float ny = (float)((double)cy - b * scale * bb1 + a * scale * bb2);
            err = (double)((nx - cx) * (nx - cx) + (ny - cy) * (ny - cy));
            cx = nx; cy = ny;
            if (cx < 0 || cx >= (float)w || cy < 0 || cy >= (float)h) break;
        } while (++it < iters && err > eps2);
        if (fabsf(cx - tx) > (float)win || fabsf(cy - ty) > (float)win) { cx = tx; cy = ty; }
        xy[2 * p] = cx; xy[2 * p + 1] = cy;
    }
    free(mask); free(buf);
}

/* ======================= calcOpticalFlowPyrLK (lkpyramid.cpp, OpenCV 3.4) ======================= */
/* pyrDown 8U: 5x5 [1 4 6 4 1]^2, (sum + 128) >> 8, REFLECT_101; dst ((sw+1)/2, (sh+1)/2) */
void oc_pyr_down(const uint8_t* src, int sw, int sh, uint8_t* dst)
{
    const int dw = (sw + 1) / 2, dh = (sh + 1) / 2;
    static const int k[5] = {1, 4, 6, 4, 1};
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            int acc = 0;
            for (int i = 0; i < 5; i++) {
                const uint8_t* row = src + (size_t)gf_reflect(2 * y + i - 2, sh) * sw;
                int hs = 0;
                for (int j = 0; j < 5; j++) hs += k[j] * row[gf_reflect(2 * x + j - 2, sw)];
                acc += k[i] * hs;
            }
            dst[(size_t)y * dw + x] = (uint8_t)((acc + 128) >> 8);
        }
}

/* buildOpticalFlowPyramid(img, pyr, winSize, maxLevel, false): number of levels kept */
int oc_lk_levels(int w, int h, int win, int max_level)
{
    for (int level = 0; level <= max_level; level++) {
        w = (w + 1) / 2; h = (h + 1) / 2;
        if (w <= win || h <= win) return level + 1;
    }
    return max_level + 1;
}

/* calcSharrDeriv: interleaved (dx, dy) int16, REFLECT_101 */
static void lk_sharr(const uint8_t* img, int w, int h, int16_t* d)
{
    int* t0 = (int*)malloc(sizeof(int) * (w + 2));
    int* t1 = (int*)malloc(sizeof(int) * (w + 2));
    for (int y = 0; y < h; y++) {
        const uint8_t* s0 = img + (size_t)(y > 0 ? y - 1 : (h > 1 ? 1 : 0)) * w;
        const uint8_t* s1 = img + (size_t)y * w;
        const uint8_t* s2 = img + (size_t)(y < h - 1 ? y + 1 : (h > 1 ? h - 2 : 0)) * w;
        for (int x = 0; x < w; x++) {
            t0[x + 1] = (s0[x] + s2[x]) * 3 + s1[x] * 10;
            t1[x + 1] = s2[x] - s0[x];
        }
        const int x0 = w > 1 ? 1 : 0, x1 = w > 1 ? w - 2 : 0;
        t0[0] = t0[x0 + 1]; t0[w + 1] = t0[x1 + 1];
        t1[0] = t1[x0 + 1]; t1[w + 1] = t1[x1 + 1];
        for (int x = 0; x < w; x++) {
            d[((size_t)y * w + x) * 2] = (int16_t)(t0[x + 2] - t0[x]);
            d[((size_t)y * w + x) * 2 + 1] = (int16_t)((t1[x + 2] + t1[x]) * 3 + t1[x + 1] * 10);
        }
    }
    free(t0); free(t1);
}

#define LK_DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

typedef struct { const uint8_t* img; int w, h; } lk_plane;
static inline int lk_px(const lk_plane* p, int x, int y)   /* copyMakeBorder REFLECT_101 frame */
{
    return p->img[(size_t)gf_reflect(y, p->h) * p->w + gf_reflect(x, p->w)];
}
static inline int lk_dv(const int16_t* d, int w, int h, int x, int y, int c)  /* BORDER_CONSTANT 0 */
{
    return (x < 0 || y < 0 || x >= w || y >= h) ? 0 : d[((size_t)y * w + x) * 2 + c];
}

/* cv::calcOpticalFlowPyrLK(prev, next, prevPts, nextPts, status, err, Size(win, win), max_level,
 * TermCriteria(ITER|EPS, max_count, eps)) (Frame.cc:335), flags 0, minEigThreshold 1e-4.
 * The window sums are exact (int64); OpenCV 3.4 accumulates them in float. */
int oc_lk_pyr(const uint8_t* prev, const uint8_t* next, int w, int h, int stride, const float* pxy, int n, int win,
              int max_level, int max_count, double eps, float* nxy, uint8_t* status)
{
    const int L = oc_lk_levels(w, h, win, max_level);
    uint8_t* P[16]; uint8_t* N[16]; int16_t* D[16]; int lw[16], lh[16];
    lw[0] = w; lh[0] = h;
    P[0] = (uint8_t*)malloc((size_t)w * h); N[0] = (uint8_t*)malloc((size_t)w * h);
    for (int y = 0; y < h; y++) {
        memcpy(P[0] + (size_t)y * w, prev + (size_t)y * stride, w);
        memcpy(N[0] + (size_t)y * w, next + (size_t)y * stride, w);
    }
    for (int l = 1; l < L; l++) {
        lw[l] = (lw[l - 1] + 1) / 2; lh[l] = (lh[l - 1] + 1) / 2;
        P[l] = (uint8_t*)malloc((size_t)lw[l] * lh[l]); N[l] = (uint8_t*)malloc((size_t)lw[l] * lh[l]);
        oc_pyr_down(P[l - 1], lw[l - 1], lh[l - 1], P[l]);
        oc_pyr_down(N[l - 1], lw[l - 1], lh[l - 1], N[l]);
    }
    for (int l = 0; l < L; l++) {
        D[l] = (int16_t*)malloc(sizeof(int16_t) * 2 * (size_t)lw[l] * lh[l]);
        lk_sharr(P[l], lw[l], lh[l], D[l]);
    }
    const double eps2 = eps * eps;
    const float hw = (float)(win - 1) * 0.5f;
    const float FLT_SCALE = 1.f / (1 << 20);
    int16_t* Iw = (int16_t*)malloc(sizeof(int16_t) * 3 * win * win);
    for (int p = 0; p < n; p++) {
        status[p] = 1;
        float nx = 0, ny = 0;
        for (int level = L - 1; level >= 0; level--) {
            const lk_plane I = {P[level], lw[level], lh[level]}, J = {N[level], lw[level], lh[level]};
            const float sc = (float)(1. / (1 << level));
            float px = pxy[2 * p] * sc, py = pxy[2 * p + 1] * sc;
            if (level == L - 1) { nx = px; ny = py; }
            else { nx = nx * 2.f; ny = ny * 2.f; }
            px -= hw; py -= hw;
            const int ipx = cv_floor(px), ipy = cv_floor(py);
            if (ipx < -win || ipx >= lw[level] || ipy < -win || ipy >= lh[level]) {
                if (level == 0) status[p] = 0;
                continue;
            }
            float a = px - (float)ipx, b = py - (float)ipy;
            int iw00 = cv_round((1.f - a) * (1.f - b) * 16384.f);
            int iw01 = cv_round(a * (1.f - b) * 16384.f);
            int iw10 = cv_round((1.f - a) * b * 16384.f);
            int iw11 = 16384 - iw00 - iw01 - iw10;
            int64_t iA11 = 0, iA12 = 0, iA22 = 0;
            for (int y = 0; y < win; y++)
                for (int x = 0; x < win; x++) {
                    const int X = ipx + x, Y = ipy + y;
                    const int ival = LK_DESCALE(lk_px(&I, X, Y) * iw00 + lk_px(&I, X + 1, Y) * iw01 +
                                                lk_px(&I, X, Y + 1) * iw10 + lk_px(&I, X + 1, Y + 1) * iw11, 9);
                    int g[2];
                    for (int c = 0; c < 2; c++)
                        g[c] = LK_DESCALE(lk_dv(D[level], lw[level], lh[level], X, Y, c) * iw00 +
                                          lk_dv(D[level], lw[level], lh[level], X + 1, Y, c) * iw01 +
                                          lk_dv(D[level], lw[level], lh[level], X, Y + 1, c) * iw10 +
                                          lk_dv(D[level], lw[level], lh[level], X + 1, Y + 1, c) * iw11, 14);
                    Iw[3 * (y * win + x)] = (int16_t)ival;
                    Iw[3 * (y * win + x) + 1] = (int16_t)g[0];
                    Iw[3 * (y * win + x) + 2] = (int16_t)g[1];
                    iA11 += (int64_t)g[0] * g[0];
                    iA12 += (int64_t)g[0] * g[1];
                    iA22 += (int64_t)g[1] * g[1];
                }
            const float A11 = (float)iA11 * FLT_SCALE, A12 = (float)iA12 * FLT_SCALE, A22 = (float)iA22 * FLT_SCALE;
            float D2 = A11 * A22 - A12 * A12;
            const float minEig = ((A22 + A11) - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                                 (float)(2 * win * win);
            if (minEig < 1e-4f || D2 < FLT_EPSILON) {
                if (level == 0) status[p] = 0;
                continue;
            }
            D2 = 1.f / D2;
            float lx = nx - hw, ly = ny - hw;         /* nextPt -= halfWin; nx, ny = nextPts[ptidx] */
            float pdx = 0, pdy = 0;
            for (int j = 0; j < max_count; j++) {
                const int inx = cv_floor(lx), iny = cv_floor(ly);
                if (inx < -win || inx >= lw[level] || iny < -win || iny >= lh[level]) {
                    if (level == 0) status[p] = 0;
                    break;
                }
                a = lx - (float)inx; b = ly - (float)iny;
                iw00 = cv_round((1.f - a) * (1.f - b) * 16384.f);
                iw01 = cv_round(a * (1.f - b) * 16384.f);
                iw10 = cv_round((1.f - a) * b * 16384.f);
                iw11 = 16384 - iw00 - iw01 - iw10;
                int64_t ib1 = 0, ib2 = 0;
                for (int y = 0; y < win; y++)
                    for (int x = 0; x < win; x++) {
                        const int X = inx + x, Y = iny + y;
                        const int diff = LK_DESCALE(lk_px(&J, X, Y) * iw00 + lk_px(&J, X + 1, Y) * iw01 +
                                                    lk_px(&J, X, Y + 1) * iw10 + lk_px(&J, X + 1, Y + 1) * iw11, 9) -
                                         Iw[3 * (y * win + x)];
                        ib1 += (int64_t)diff * Iw[3 * (y * win + x) + 1];
                        ib2 += (int64_t)diff * Iw[3 * (y * win + x) + 2];
                    }
                const float b1 = (float)ib1 * FLT_SCALE, b2 = (float)ib2 * FLT_SCALE;
                const float dx = (A12 * b2 - A22 * b1) * D2, dy = (A12 * b1 - A11 * b2) * D2;
                lx += dx; ly += dy;
                nx = lx + hw; ny = ly + hw;           /* nextPts[ptidx] = nextPt + halfWin */
                if ((double)dx * dx + (double)dy * dy <= eps2) break;
                if (j > 0 && fabsf(dx + pdx) < 0.01 && fabsf(dy + pdy) < 0.01) {
                    nx -= dx * 0.5f; ny -= dy * 0.5f;
                    break;
                }
                pdx = dx; pdy = dy;
            }
            if (level == 0 && status[p]) {            /* the err pass's bounds check */
                const float ex = nx - hw, ey = ny - hw;
                const int iex = cv_floor(ex), iey = cv_floor(ey);
                if (iex < -win || iex >= lw[0] || iey < -win || iey >= lh[0]) status[p] = 0;
            }
        }
        nxy[2 * p] = nx; nxy[2 * p + 1] = ny;
    }
    free(Iw);
    for (int l = 0; l < L; l++) { free(P[l]); free(N[l]); free(D[l]); }
    return L;
}

/* ======================= findFundamentalMat (fundam.cpp / ptsetreg.cpp, OpenCV 3.4) ======================= */
/* Canonical double acos / log / exp: the fdlibm algorithms (e_acos.c, e_log.c, e_exp.c), pure
 * IEEE arithmetic so the HIP twin is bit-identical; cos through pq_sincos.  pow(x, y) (solveCubic)
 * = exp(y * log(x)), x > 0; 0 for x == 0. */
static inline uint32_t fd_hi(double x) { uint64_t u; memcpy(&u, &x, 8); return (uint32_t)(u >> 32); }
static inline uint32_t fd_lo(double x) { uint64_t u; memcpy(&u, &x, 8); return (uint32_t)u; }
static inline double fd_make(uint32_t hi, uint32_t lo) { uint64_t u = ((uint64_t)hi << 32) | lo; double d; memcpy(&d, &u, 8); return d; }

double oc_fd_acos(double x)
{
    const double pi = 0x1.921fb54442d18p+1, pio2_hi = 0x1.921fb54442d18p+0, pio2_lo = 0x1.1a62633145c07p-54;
    const double pS0 = 0x1.5555555555555p-3, pS1 = -0x1.4d61203eb6f7dp-2, pS2 = 0x1.9c1550e884455p-3,
                 pS3 = -0x1.48228b5688f3bp-5, pS4 = 0x1.9efe07501b288p-11, pS5 = 0x1.23de10dfdf709p-15;
    const double qS1 = -0x1.33a271c8a2d4bp+1, qS2 = 0x1.02ae59c598ac8p+1, qS3 = -0x1.6066c1b8d0159p-1,
                 qS4 = 0x1.3b8c5b12e9282p-4;
    const int32_t hx = (int32_t)fd_hi(x), ix = hx & 0x7fffffff;
    if (ix >= 0x3ff00000) {
        if (((ix - 0x3ff00000) | fd_lo(x)) == 0) return hx > 0 ? 0.0 : pi + 2.0 * pio2_lo;
        return NAN;
    }
    if (ix < 0x3fe00000) {
        if (ix <= 0x3c600000) return pio2_hi + pio2_lo;
        const double z = x * x;
        const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const double r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    } else if (hx < 0) {
        const double z = (1.0 + x) * 0.5;
        const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const double s = sqrt(z);
        const double r = p / q;
        const double w = r * s - pio2_lo;
        return pi - 2.0 * (s + w);
    } else {
        const double z = (1.0 - x) * 0.5;
        const double s = sqrt(z);
        const double df = fd_make(fd_hi(s), 0);
        const double c = (z - df * df) / (s + df);
        const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const double r = p / q;
        const double w = r * s + c;
        return 2.0 * (df + w);
    }
}

double oc_fd_log(double x)
{
    const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33, two54 = 0x1p54;
    const double Lg1 = 0x1.5555555555593p-1, Lg2 = 0x1.999999997fa04p-2, Lg3 = 0x1.2492494229359p-2,
                 Lg4 = 0x1.c71c51d8e78afp-3, Lg5 = 0x1.7466496cb03dep-3, Lg6 = 0x1.39a09d078c69fp-3,
                 Lg7 = 0x1.2f112df3e5244p-3;
    int32_t hx = (int32_t)fd_hi(x);
    const uint32_t lx = fd_lo(x);
    int32_t k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -INFINITY;
        if (hx < 0) return NAN;
        k -= 54; x *= two54;
        hx = (int32_t)fd_hi(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i0 = (hx + 0x95f64) & 0x100000;
    x = fd_make((uint32_t)(hx | (i0 ^ 0x3ff00000)), fd_lo(x));
    k += (i0 >> 20);
    const double f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            const double dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        const double dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    const double dk = (double)k;
    const double z = s * s;
    int32_t i = hx - 0x6147a;
    const double w = z * z;
    const int32_t j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    const double R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

double oc_fd_exp(double x)
{
    const double ln2HI = 0x1.62e42fee00000p-1, ln2LO = 0x1.a39ef35793c76p-33, invln2 = 0x1.71547652b82fep+0;
    const double P1 = 0x1.555555555553ep-3, P2 = -0x1.6c16c16bebd93p-9, P3 = 0x1.1566aaf25de2cp-14,
                 P4 = -0x1.bbd41c5d26bf1p-20, P5 = 0x1.6376972bea4d0p-25;
    const double o_threshold = 0x1.62e42fefa39efp+9, u_threshold = -0x1.74910d52d3051p+9;
    uint32_t hx = fd_hi(x);
    const int xsb = (hx >> 31) & 1;
    hx &= 0x7fffffff;
    if (hx >= 0x40862E42) {
        if (hx >= 0x7ff00000) {
            if (((hx & 0xfffff) | fd_lo(x)) != 0) return x + x;
            return xsb == 0 ? x : 0.0;
        }
        if (x > o_threshold) return INFINITY;
        if (x < u_threshold) return 0.0;
    }
    double hi = 0, lo = 0;
    int k = 0;
    if (hx > 0x3fd62e42) {
        if (hx < 0x3FF0A2B2) {
            hi = x - (xsb ? -ln2HI : ln2HI); lo = xsb ? -ln2LO : ln2LO; k = 1 - xsb - xsb;
        } else {
            k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
            const double t = k;
            hi = x - t * ln2HI;
            lo = t * ln2LO;
        }
        x = hi - lo;
    } else if (hx < 0x3e300000) {
        return 1.0 + x;
    } else k = 0;
    const double t = x * x;
    const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    if (k >= -1021) return fd_make(fd_hi(y) + ((uint32_t)k << 20), fd_lo(y));
    y = fd_make(fd_hi(y) + ((uint32_t)(k + 1000) << 20), fd_lo(y));
    return y * 0x1p-1000;
}

double oc_fd_cos(double x) { double s, c; pq_sincos(x, &s, &c); return c; }

static double fd_pow_pos(double x, double y) { return x == 0.0 ? 0.0 : oc_fd_exp(y * oc_fd_log(x)); }

/* cv::solveCubic for coeffs c[0..3] (c[0] x^3 + ...): roots and their count */
int oc_solve_cubic(const double c[4], double r[3])
{
    double a0 = c[0], a1 = c[1], a2 = c[2], a3 = c[3], x0 = 0, x1 = 0, x2 = 0;
    int n = 0;
    if (a0 == 0) {
        if (a1 == 0) {
            if (a2 == 0) n = a3 == 0 ? -1 : 0;
            else { x0 = -a3 / a2; n = 1; }
        } else {
            double d = a2 * a2 - 4 * a1 * a3;
            if (d >= 0) {
                d = sqrt(d);
                const double q1 = (-a2 + d) * 0.5, q2 = (a2 + d) * -0.5;
                if (fabs(q1) > fabs(q2)) { x0 = q1 / a1; x1 = a3 / q1; }
                else { x0 = q2 / a1; x1 = a3 / q2; }
                n = d > 0 ? 2 : 1;
            }
        }
    } else {
        a0 = 1. / a0;
        a1 *= a0; a2 *= a0; a3 *= a0;
        const double Q = (a1 * a1 - 3 * a2) * (1. / 9);
        const double R = (2 * a1 * a1 * a1 - 9 * a1 * a2 + 27 * a3) * (1. / 54);
        const double Qcubed = Q * Q * Q;
        double d = Qcubed - R * R;
        if (d > 0) {
            const double theta = oc_fd_acos(R / sqrt(Qcubed));
            const double sqrtQ = sqrt(Q);
            const double t0 = -2 * sqrtQ, t1 = theta * (1. / 3), t2 = a1 * (1. / 3);
            x0 = t0 * oc_fd_cos(t1) - t2;
            x1 = t0 * oc_fd_cos(t1 + (2. * 3.1415926535897932384626433832795 / 3)) - t2;
            x2 = t0 * oc_fd_cos(t1 + (4. * 3.1415926535897932384626433832795 / 3)) - t2;
            n = 3;
        } else if (d == 0) {
            if (R >= 0) { x0 = -2 * fd_pow_pos(R, 1. / 3) - a1 / 3; x1 = fd_pow_pos(R, 1. / 3) - a1 / 3; }
            else { x0 = 2 * fd_pow_pos(-R, 1. / 3) - a1 / 3; x1 = -fd_pow_pos(-R, 1. / 3) - a1 / 3; }
            x2 = 0;
            n = x0 == x1 ? 1 : 2;
            x1 = x0 == x1 ? 0 : x1;
        } else {
            d = sqrt(-d);
            double e = fd_pow_pos(d + fabs(R), 0.333333333333);
            if (R > 0) e = -e;
            x0 = (e + Q / e) - a1 * (1. / 3);
            n = 1;
        }
    }
    r[0] = x0; r[1] = x1; r[2] = x2;
    return n;
}

/* run7Point (fundam.cpp): up to 3 models F[9k..9k+8], returns their count.  The null space of
 * the 7x9 system comes from Gauss-Jordan elimination with complete pivoting (the first largest
 * |a| in row-major order over the remaining block) instead of OpenCV's JacobiSVD: the same
 * two-dimensional space in another basis; every model is scaled to F33 = 1, so the models
 * agree up to rounding. */
int oc_run7point(const float* m1, const float* m2, double* F)
{
    double A[7][9];
    int perm[9];
    for (int i = 0; i < 7; i++) {
        const double x0 = m1[2 * i], y0 = m1[2 * i + 1], x1 = m2[2 * i], y1 = m2[2 * i + 1];
        A[i][0] = x1 * x0; A[i][1] = x1 * y0; A[i][2] = x1;
        A[i][3] = y1 * x0; A[i][4] = y1 * y0; A[i][5] = y1;
        A[i][6] = x0; A[i][7] = y0; A[i][8] = 1;
    }
    for (int j = 0; j < 9; j++) perm[j] = j;
    for (int r = 0; r < 7; r++) {
        int pi = r, pj = r;
        double best = -1.0;
        for (int i = r; i < 7; i++)
            for (int j = r; j < 9; j++)
                if (fabs(A[i][j]) > best) { best = fabs(A[i][j]); pi = i; pj = j; }
        if (!(best > 0.0)) return 0;
        if (pi != r)
            for (int j = 0; j < 9; j++) { const double t = A[r][j]; A[r][j] = A[pi][j]; A[pi][j] = t; }
        if (pj != r) {
            for (int i = 0; i < 7; i++) { const double t = A[i][r]; A[i][r] = A[i][pj]; A[i][pj] = t; }
            const int t = perm[r]; perm[r] = perm[pj]; perm[pj] = t;
        }
        for (int i = 0; i < 7; i++) {
            if (i == r) continue;
            const double f = A[i][r] / A[r][r];
            for (int j = r; j < 9; j++) A[i][j] = A[i][j] - f * A[r][j];
        }
    }
    double f1[9], f2[9];
    for (int q = 0; q < 2; q++) {
        double* v = q == 0 ? f1 : f2;
        const int col = 7 + q;
        v[perm[7]] = q == 0 ? 1.0 : 0.0;
        v[perm[8]] = q == 0 ? 0.0 : 1.0;
        for (int i = 0; i < 7; i++) v[perm[i]] = -A[i][col] / A[i][i];
    }
    for (int i = 0; i < 9; i++) f1[i] -= f2[i];
    double c[4], r[3];
    double t0 = f2[4] * f2[8] - f2[5] * f2[7];
    double t1 = f2[3] * f2[8] - f2[5] * f2[6];
    double t2 = f2[3] * f2[7] - f2[4] * f2[6];
    c[3] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2;
    c[2] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2 - f1[3] * (f2[1] * f2[8] - f2[2] * f2[7]) +
           f1[4] * (f2[0] * f2[8] - f2[2] * f2[6]) - f1[5] * (f2[0] * f2[7] - f2[1] * f2[6]) +
           f1[6] * (f2[1] * f2[5] - f2[2] * f2[4]) - f1[7] * (f2[0] * f2[5] - f2[2] * f2[3]) +
           f1[8] * (f2[0] * f2[4] - f2[1] * f2[3]);
    t0 = f1[4] * f1[8] - f1[5] * f1[7];
    t1 = f1[3] * f1[8] - f1[5] * f1[6];
    t2 = f1[3] * f1[7] - f1[4] * f1[6];
    c[1] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2 - f2[3] * (f1[1] * f1[8] - f1[2] * f1[7]) +
           f2[4] * (f1[0] * f1[8] - f1[2] * f1[6]) - f2[5] * (f1[0] * f1[7] - f1[1] * f1[6]) +
           f2[6] * (f1[1] * f1[5] - f1[2] * f1[4]) - f2[7] * (f1[0] * f1[5] - f1[2] * f1[3]) +
           f2[8] * (f1[0] * f1[4] - f1[1] * f1[3]);
    c[0] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2;
    const int n = oc_solve_cubic(c, r);
    if (n < 1 || n > 3) return n;
    for (int k = 0; k < n; k++) {
        double* fm = F + 9 * k;
        double lambda = r[k], mu = 1.;
        const double s = f1[8] * r[k] + f2[8];
        if (fabs(s) > DBL_EPSILON) { mu = 1. / s; lambda *= mu; fm[8] = 1.; }
        else fm[8] = 0.;
        for (int i = 0; i < 8; i++) fm[i] = f1[i] * lambda + f2[i] * mu;
    }
    return n;
}

/* FMEstimatorCallback::computeError */
static float fm_error(const double* F, float x1, float y1, float x2, float y2)
{
    double a = F[0] * x1 + F[1] * y1 + F[2];
    double b = F[3] * x1 + F[4] * y1 + F[5];
    double c = F[6] * x1 + F[7] * y1 + F[8];
    const double s2 = 1. / (a * a + b * b);
    const double d2 = x2 * a + y2 * b + c;
    a = F[0] * x2 + F[3] * y2 + F[6];
    b = F[1] * x2 + F[4] * y2 + F[7];
    c = F[2] * x2 + F[5] * y2 + F[8];
    const double s1 = 1. / (a * a + b * b);
    const double d1 = x1 * a + y1 * b + c;
    const double e1 = d1 * d1 * s1, e2 = d2 * d2 * s2;
    return (float)(e1 < e2 ? e2 : e1);
}

/* haveCollinearPoints(m, 7): triples that include the last point only (as OpenCV checks) */
static int fm_collinear(const float* m)
{
    const int i = 6;
    for (int j = 0; j < i; j++) {
        const double dx1 = (double)(m[2 * j] - m[2 * i]), dy1 = (double)(m[2 * j + 1] - m[2 * i + 1]);
        for (int k = 0; k < j; k++) {
            const double dx2 = (double)(m[2 * k] - m[2 * i]), dy2 = (double)(m[2 * k + 1] - m[2 * i + 1]);
            if (fabs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return 1;
        }
    }
    return 0;
}

static inline unsigned rng_next(uint64_t* st)
{
    *st = (uint64_t)(unsigned)*st * 4164903690U + (unsigned)(*st >> 32);
    return (unsigned)*st;
}

/* getSubset(m1, m2, ms1, ms2, rng, maxAttempts), checkPartialSubsets = false, checkSubset =
 * !collinear(ms1) && !collinear(ms2): 1 when a subset was drawn */
static int fm_subset(const float* m1, const float* m2, int count, uint64_t* rng, int max_attempts, int idx[7],
                     float s1[14], float s2[14])
{
    int iters = 0, i = 0;
    for (; iters < max_attempts; iters++) {
        for (i = 0; i < 7 && iters < max_attempts;) {
            int id;
            for (;;) {
                id = idx[i] = (int)(rng_next(rng) % (unsigned)count);
                int j;
                for (j = 0; j < i; j++)
                    if (id == idx[j]) break;
                if (j == i) break;
            }
            s1[2 * i] = m1[2 * id]; s1[2 * i + 1] = m1[2 * id + 1];
            s2[2 * i] = m2[2 * id]; s2[2 * i + 1] = m2[2 * id + 1];
            i++;
        }
        if (i == 7 && (fm_collinear(s1) || fm_collinear(s2))) continue;
        break;
    }
    return i == 7 && iters < max_attempts;
}

/* RANSACUpdateNumIters(p, ep, 7, maxIters); std::log -> the canonical fdlibm log, std::pow(x, 7)
 * -> x*x*x*x*x*x*x left to right */
int oc_ransac_update_iters(double p, double ep, int max_iters)
{
    p = p > 0. ? p : 0.; p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.; ep = ep < 1. ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    const double b = 1. - ep;
    double denom = 1. - b * b * b * b * b * b * b;
    if (denom < DBL_MIN) return 0;
    num = oc_fd_log(num);
    denom = oc_fd_log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)lrint(num / denom);
}

/* cv::findFundamentalMat(m1, m2, mask, FM_RANSAC, thr, conf) (Frame.cc:373): returns 1 and F
 * (row-major 3x3 double; the first model when several are stacked) or 0 for an empty result.
 * n < 7: empty; n == 7: run7Point; 8..14: LMeDS; >= 15: RANSAC (maxIters 1000). */
int oc_find_fundamental(const float* m1, const float* m2, int n, double thr, double conf, double F[9])
{
    double models[27];
    if (n < 7) return 0;
    if (n == 7) {
        const int k = oc_run7point(m1, m2, models);
        if (k <= 0) return 0;
        memcpy(F, models, sizeof(double) * 9);
        return 1;
    }
    uint64_t rng = ~(uint64_t)0;
    int idx[7];
    float s1[14], s2[14];
    if (n >= 15) {
        int niters = 1000, max_good = 0, have = 0;
        const float t = (float)(thr * thr);
        for (int iter = 0; iter < niters; iter++) {
            if (!fm_subset(m1, m2, n, &rng, 10000, idx, s1, s2)) {
                if (iter == 0) return 0;
                break;
            }
            const int nm = oc_run7point(s1, s2, models);
            if (nm <= 0) continue;
            for (int m = 0; m < nm; m++) {
                int good = 0;
                for (int i = 0; i < n; i++)
                    good += fm_error(models + 9 * m, m1[2 * i], m1[2 * i + 1], m2[2 * i], m2[2 * i + 1]) <= t;
                if (good > (max_good > 6 ? max_good : 6)) {
                    memcpy(F, models + 9 * m, sizeof(double) * 9);
                    max_good = good; have = 1;
                    niters = oc_ransac_update_iters(conf, (double)(n - good) / n, niters);
                }
            }
        }
        return have && max_good > 0;
    }
    int niters = oc_ransac_update_iters(conf, 0.45, 1000);
    niters = niters > 3 ? niters : 3;
    double min_median = DBL_MAX;
    float err[16];
    for (int iter = 0; iter < niters; iter++) {
        if (!fm_subset(m1, m2, n, &rng, 1000, idx, s1, s2)) {
            if (iter == 0) return 0;
            break;
        }
        const int nm = oc_run7point(s1, s2, models);
        if (nm <= 0) continue;
        for (int m = 0; m < nm; m++) {
            for (int i = 0; i < n; i++) err[i] = fm_error(models + 9 * m, m1[2 * i], m1[2 * i + 1], m2[2 * i], m2[2 * i + 1]);
            for (int a = 1; a < n; a++) {                     /* nth_element: the value is unique */
                const float v = err[a];
                int b = a - 1;
                while (b >= 0 && err[b] > v) { err[b + 1] = err[b]; b--; }
                err[b + 1] = v;
            }
            const double median = err[n / 2];
            if (median < min_median) { min_median = median; memcpy(F, models + 9 * m, sizeof(double) * 9); }
        }
    }
    if (!(min_median < DBL_MAX)) return 0;
    double sigma = 2.5 * 1.4826 * (1 + 5. / (n - 7)) * sqrt(min_median);
    sigma = sigma > 0.001 ? sigma : 0.001;
    const float t = (float)(sigma * sigma);
    int good = 0;
    for (int i = 0; i < n; i++) good += fm_error(F, m1[2 * i], m1[2 * i + 1], m2[2 * i], m2[2 * i + 1]) <= t;
    return good >= 7;
}

/* The SAD consistency check and the epipolar test of Frame::ProcessMovingObject
 * (Frame.cc:337-384) given the tracked pairs: fills the F_ sets in order, F, and T_M.
 * Returns |T_M| (written up to tm_cap), or -1 when findFundamentalMat is empty (the reference
 * then reads an empty Mat: undefined). */
int oc_moving_tail(const uint8_t* prev, const uint8_t* cur, int w, int h, int stride, const float* pxy,
                   const float* nxy, uint8_t* state, int n, int edge, double limit, float* tm_xy, int tm_cap,
                   double F_out[9], int* nf_out)
{
    static const int dx[9] = {-1, 0, 1, -1, 0, 1, -1, 0, 1}, dy[9] = {-1, -1, -1, 0, 0, 0, 1, 1, 1};
    float* m1 = (float*)malloc(sizeof(float) * 2 * (n > 0 ? n : 1));
    float* m2 = (float*)malloc(sizeof(float) * 2 * (n > 0 ? n : 1));
    int nf = 0;
    for (int i = 0; i < n; i++) {
        if (!state[i]) continue;
        const int x1 = (int)pxy[2 * i], y1 = (int)pxy[2 * i + 1], x2 = (int)nxy[2 * i], y2 = (int)nxy[2 * i + 1];
        if (x1 < edge || x1 >= w - edge || x2 < edge || x2 >= w - edge || y1 < edge || y1 >= h - edge ||
            y2 < edge || y2 >= h - edge) {
            state[i] = 0;
            continue;
        }
        double sum = 0;
        for (int j = 0; j < 9; j++)
            sum += abs((int)prev[(size_t)(y1 + dy[j]) * stride + x1 + dx[j]] - (int)cur[(size_t)(y2 + dy[j]) * stride + x2 + dx[j]]);
        if (sum > limit) state[i] = 0;
        if (state[i]) {
            m1[2 * nf] = pxy[2 * i]; m1[2 * nf + 1] = pxy[2 * i + 1];
            m2[2 * nf] = nxy[2 * i]; m2[2 * nf + 1] = nxy[2 * i + 1];
            nf++;
        }
    }
    if (nf_out) *nf_out = nf;
    double F[9];
    const int ok = oc_find_fundamental(m1, m2, nf, 0.1, 0.99, F);
    free(m1); free(m2);
    if (!ok) return -1;
    if (F_out) memcpy(F_out, F, sizeof(F));
    int nt = 0;
    for (int i = 0; i < n; i++) {
        if (!state[i]) continue;
        const double px = pxy[2 * i], py = pxy[2 * i + 1];
        const double A = F[0] * px + F[1] * py + F[2];
        const double B = F[3] * px + F[4] * py + F[5];
        const double Cc = F[6] * px + F[7] * py + F[8];
        const double dd = fabs(A * nxy[2 * i] + B * nxy[2 * i + 1] + Cc) / sqrt(A * A + B * B);
        if (dd <= 1) continue;
        if (nt < tm_cap) { tm_xy[2 * nt] = nxy[2 * i]; tm_xy[2 * nt + 1] = nxy[2 * i + 1]; }
        nt++;
    }
    return nt;
}

/* Frame::ProcessMovingObject (Frame.cc:311-393): T_M from the previous and current gray frames. */
int oc_process_moving_object(const uint8_t* prev, const uint8_t* cur, int w, int h, int stride, float* tm_xy,
                             int tm_cap, int* ncorners_out)
{
    float* pts = (float*)malloc(sizeof(float) * 2 * 1000);
    float* nxt = (float*)malloc(sizeof(float) * 2 * 1000);
    uint8_t* st = (uint8_t*)malloc(1000);
    int n = oc_good_features_harris(prev, w, h, stride, 1000, 0.01, 8, 0.04, pts, 1000, 1 << 30);
    if (n > 1000) n = 1000;
    if (ncorners_out) *ncorners_out = n;
    oc_corner_subpix(prev, w, h, stride, pts, n, 10, 20, 0.03);
    oc_lk_pyr(prev, cur, w, h, stride, pts, n, 22, 5, 20, 0.01, nxt, st);
    const int nt = oc_moving_tail(prev, cur, w, h, stride, pts, nxt, st, n, 5, 2120.0, tm_xy, tm_cap, NULL, NULL);
    free(pts); free(nxt); free(st);
    return nt;
}
