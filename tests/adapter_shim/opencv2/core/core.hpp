// Minimal stand-in for the OpenCV 3.4 types the adapter headers touch: enough of cv::Mat
// (owned or borrowed 2-D buffers, row ranges, copies), InputArray / OutputArray, KeyPoint and
// Point2f for tests/test_adapter_compile.py (compile check) and tests/adapter_shim/adapter_exec.cpp
// (the adapters run against libcoeb_front.so).  Test infrastructure only: the reference build
// uses the real OpenCV.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>
#define CV_8U 0
#define CV_8UC1 0
#define CV_32F 5
namespace cv {
struct Point2f {
    float x = 0, y = 0;
    Point2f() {}
    Point2f(float a, float b) : x(a), y(b) {}
};
struct Point2i { int x = 0, y = 0; };
struct KeyPoint {
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
};
inline size_t elem_size(int type) { return type == CV_32F ? 4 : 1; }
struct Mat {
    unsigned char* data = nullptr;
    int rows = 0, cols = 0;
    size_t step[2] = {0, 0};
    int type_ = CV_8U;
    std::shared_ptr<std::vector<unsigned char>> buf;
    Mat() {}
    Mat(int r, int c, int t) { create(r, c, t); }
    Mat(int r, int c, int t, void* ext, size_t st = 0) : data(static_cast<unsigned char*>(ext)), rows(r), cols(c), type_(t)
    {
        step[1] = elem_size(t);
        step[0] = st ? st : (size_t)c * step[1];
    }
    void create(int r, int c, int t)
    {
        if (data && rows == r && cols == c && type_ == t) return;
        rows = r; cols = c; type_ = t;
        step[1] = elem_size(t);
        step[0] = (size_t)c * step[1];
        buf = std::make_shared<std::vector<unsigned char>>(step[0] * (size_t)r);
        data = buf->data();
    }
    void release() { buf.reset(); data = nullptr; rows = cols = 0; }
    int type() const { return type_; }
    bool empty() const { return !data || rows == 0 || cols == 0; }
    bool isContinuous() const { return rows <= 1 || step[0] == (size_t)cols * step[1]; }
    Mat clone() const
    {
        Mat m(rows, cols, type_);
        for (int r = 0; r < rows; r++) std::memcpy(m.data + r * m.step[0], data + r * step[0], (size_t)cols * step[1]);
        return m;
    }
    Mat rowRange(int a, int b) const
    {
        Mat m = *this;
        m.data = data + (size_t)a * step[0];
        m.rows = b - a;
        return m;
    }
    void copyTo(const Mat& dst) const   // dst already sized (OutputArray::create, then getMat)
    {
        for (int r = 0; r < rows; r++) std::memcpy(dst.data + r * dst.step[0], data + r * step[0], (size_t)cols * step[1]);
    }
    template <class T> T& at(int i) { return reinterpret_cast<T*>(data)[i]; }
    template <class T> const T& at(int i) const { return reinterpret_cast<const T*>(data)[i]; }
    template <class T> T& at(int r, int c) { return reinterpret_cast<T*>(data + (size_t)r * step[0])[c]; }
    template <class T> const T& at(int r, int c) const { return reinterpret_cast<const T*>(data + (size_t)r * step[0])[c]; }
    template <class T> T* ptr(int r) { return reinterpret_cast<T*>(data + (size_t)r * step[0]); }
    template <class T> const T* ptr(int r) const { return reinterpret_cast<const T*>(data + (size_t)r * step[0]); }
};
struct InputArray {
    const Mat* m;
    InputArray(const Mat& x) : m(&x) {}
    bool empty() const { return m->empty(); }
    Mat getMat() const { return *m; }
};
struct OutputArray {
    Mat* m;
    OutputArray(Mat& x) : m(&x) {}
    void release() const { m->release(); }
    void create(int r, int c, int t) const { m->create(r, c, t); }
    Mat getMat() const { return *m; }
};
}  // namespace cv
