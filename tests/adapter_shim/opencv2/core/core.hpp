// Minimal compile-only stand-in for the OpenCV 3.4 types the adapter headers touch
// (tests/test_adapter_compile.py).  Never linked into anything; the reference build uses
// the real OpenCV.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>
#define CV_8U 0
#define CV_8UC1 0
#define CV_32F 5
namespace cv {
struct Point2f { float x, y; };
struct Point2i { int x, y; };
struct KeyPoint { Point2f pt; float size, angle, response; int octave, class_id; };
struct Mat {
    unsigned char* data = nullptr;
    int rows = 0, cols = 0;
    size_t step[2] = {0, 0};
    Mat() {}
    Mat(int r, int c, int) : rows(r), cols(c) {}
    int type() const { return 0; }
    bool empty() const { return !data; }
    bool isContinuous() const { return true; }
    Mat clone() const { return *this; }
    Mat rowRange(int, int) const { return *this; }
    void copyTo(const Mat&) const {}
    template <class T> T& at(int) { return *reinterpret_cast<T*>(data); }
    template <class T> const T& at(int, int) const { return *reinterpret_cast<const T*>(data); }
    template <class T> T& at(int, int) { return *reinterpret_cast<T*>(data); }
    template <class T> T* ptr(int) { return reinterpret_cast<T*>(data); }
    template <class T> const T* ptr(int) const { return reinterpret_cast<const T*>(data); }
};
struct InputArray {
    InputArray(const Mat&) {}
    bool empty() const { return false; }
    Mat getMat() const { return Mat(); }
};
struct OutputArray {
    OutputArray(Mat&) {}
    void release() const {}
    void create(int, int, int) const {}
    Mat getMat() const { return Mat(); }
};
}  // namespace cv
