// Minimal stand-in for the parts of OpenCV's core API that
// include/orbx_orbslam2.hpp uses, so the drop-in adapter can be compiled and
// exercised in this OpenCV-free container.  Test scaffolding for OUR adapter
// only (nothing of the reference is built against it).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#define CV_8U 0
#define CV_8UC1 0
#define CV_8UC3 16
#define CV_8UC4 24
#define CV_32F 5

namespace cv {
enum { BORDER_REFLECT_101 = 4, BORDER_ISOLATED = 16 };

struct Point2f {
    float x = 0, y = 0;
    Point2f() = default;
    Point2f(float a, float b) : x(a), y(b) {}
};
struct Rect {
    int x, y, width, height;
    Rect(int a, int b, int w, int h) : x(a), y(b), width(w), height(h) {}
};
struct KeyPoint {
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
    KeyPoint() = default;
    KeyPoint(Point2f p, float s, float a = -1, float r = 0, int o = 0, int c = -1)
        : pt(p), size(s), angle(a), response(r), octave(o), class_id(c) {}
};

class Mat;
Mat operator*(const Mat &a, const Mat &b);

class Mat {
public:
    int rows = 0, cols = 0;
    size_t step = 0;
    uint8_t *data = nullptr;
    int type_ = CV_8U;
    std::shared_ptr<std::vector<uint8_t>> buf;
    Mat() = default;
    Mat(int r, int c, int t) { create(r, c, t); }
    size_t elemSize() const { return type_ == CV_32F ? 4 : (size_t)channels(); }
    int channels() const { return type_ == CV_32F ? 1 : (type_ >> 3) + 1; }
    void create(int r, int c, int t) {
        if (rows == r && cols == c && type_ == t && data) return;
        type_ = t;
        buf = std::make_shared<std::vector<uint8_t>>((size_t)r * c * elemSize());
        rows = r; cols = c; step = c * elemSize(); data = buf->data();
    }
    void release() { buf.reset(); data = nullptr; rows = cols = 0; step = 0; }
    bool empty() const { return !data || rows == 0 || cols == 0; }
    int type() const { return type_; }
    bool isContinuous() const { return step == (size_t)cols * elemSize(); }
    template <typename T> T *ptr(int r = 0) { return reinterpret_cast<T *>(data + r * step); }
    template <typename T> const T *ptr(int r = 0) const { return reinterpret_cast<const T *>(data + r * step); }
    template <typename T> const T &at(int r, int c) const { return ptr<T>(r)[c]; }
    template <typename T> T &at(int r, int c) { return ptr<T>(r)[c]; }
    // single index: element i of a row or column vector
    template <typename T> T &at(int i) { return rows == 1 ? ptr<T>(0)[i] : ptr<T>(i)[0]; }
    template <typename T> const T &at(int i) const { return rows == 1 ? ptr<T>(0)[i] : ptr<T>(i)[0]; }
    // --- float matrix arithmetic (CV_32F) for the ORB-SLAM2 forwarder tests ---
    Mat(int r, int c, int t, float fill) {
        create(r, c, t);
        for (int i = 0; i < r; ++i)
            for (int j = 0; j < c; ++j) at<float>(i, j) = fill;
    }
    static Mat zeros(int r, int c, int t) { return Mat(r, c, t, 0.f); }
    static Mat eye(int r, int c, int t) {
        Mat m(r, c, t, 0.f);
        for (int i = 0; i < r && i < c; ++i) m.at<float>(i, i) = 1.f;
        return m;
    }
    Mat row(int i) const { return rowRange(i, i + 1); }
    Mat col(int j) const { return colRange(j, j + 1); }
    Mat colRange(int a, int b) const { Mat m = *this; m.data = data + a * elemSize(); m.cols = b - a; return m; }
    Mat t() const {
        Mat m(cols, rows, type_);
        for (int i = 0; i < rows; ++i)
            for (int j = 0; j < cols; ++j) m.at<float>(j, i) = at<float>(i, j);
        return m;
    }
    double dot(const Mat &o) const {
        double s = 0;
        for (int i = 0; i < rows; ++i)
            for (int j = 0; j < cols; ++j) s += (double)at<float>(i, j) * (double)o.at<float>(i, j);
        return s;
    }
    template <typename F> Mat map(F f) const {
        Mat m(rows, cols, type_);
        for (int i = 0; i < rows; ++i)
            for (int j = 0; j < cols; ++j) m.at<float>(i, j) = f(at<float>(i, j), i, j);
        return m;
    }
    Mat operator-() const { return map([](float v, int, int) { return -v; }); }
    Mat operator/(float s) const { return map([s](float v, int, int) { return v / s; }); }
    Mat operator+(const Mat &o) const { return map([&o](float v, int i, int j) { return v + o.at<float>(i, j); }); }
    Mat operator-(const Mat &o) const { return map([&o](float v, int i, int j) { return v - o.at<float>(i, j); }); }
    friend Mat operator*(float s, const Mat &m) { return m.map([s](float v, int, int) { return s * v; }); }
    Mat operator*(float s) const { return map([s](float v, int, int) { return v * s; }); }
    Mat rowRange(int a, int b) const { Mat m = *this; m.data = data + a * step; m.rows = b - a; return m; }
    Mat operator()(Rect r) const {
        Mat m = *this; m.data = data + r.y * step + r.x * elemSize(); m.rows = r.height; m.cols = r.width; return m;
    }
    Mat clone() const {
        Mat m(rows, cols, type_);
        for (int i = 0; i < rows; ++i) std::memcpy(m.data + i * m.step, data + i * step, cols * elemSize());
        return m;
    }
    void copyTo(Mat dst) const {
        for (int i = 0; i < rows; ++i) std::memcpy(dst.data + i * dst.step, data + i * step, cols * elemSize());
    }
};

inline Mat operator*(const Mat &a, const Mat &b) {
    Mat m(a.rows, b.cols, CV_32F);
    for (int i = 0; i < a.rows; ++i)
        for (int j = 0; j < b.cols; ++j) {
            float s = 0.f;
            for (int k = 0; k < a.cols; ++k) s += a.at<float>(i, k) * b.at<float>(k, j);
            m.at<float>(i, j) = s;
        }
    return m;
}
inline double norm(const Mat &m) {
    double s = 0;
    for (int i = 0; i < m.rows; ++i)
        for (int j = 0; j < m.cols; ++j) s += (double)m.at<float>(i, j) * (double)m.at<float>(i, j);
    return std::sqrt(s);
}

class _InputArray {
public:
    _InputArray(const Mat &m) : m_(&m) {}
    Mat getMat() const { return *m_; }
    bool empty() const { return m_->empty(); }
private:
    const Mat *m_;
};
class _OutputArray {
public:
    _OutputArray(Mat &m) : m_(&m) {}
    void create(int r, int c, int t) const { m_->create(r, c, t); }
    Mat getMat() const { return *m_; }
    void release() const { m_->release(); }
private:
    Mat *m_;
};
typedef const _InputArray &InputArray;
typedef const _OutputArray &OutputArray;

// BORDER_REFLECT_101 (+ISOLATED) of the ROI `src` that sits at (left, top) inside `dst`.
inline void copyMakeBorder(const Mat &src, Mat &dst, int top, int bottom, int left, int right, int) {
    auto r101 = [](int p, int n) { while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - p - 2; return p; };
    std::vector<uint8_t> tmp((size_t)src.rows * src.cols);
    for (int y = 0; y < src.rows; ++y) std::memcpy(&tmp[(size_t)y * src.cols], src.data + y * src.step, src.cols);
    // row by row: the interior as one copy, the side borders by reflection
    std::vector<int> lx(left), rx(right);
    for (int x = 0; x < left; ++x) lx[x] = r101(x - left, src.cols);
    for (int x = 0; x < right; ++x) rx[x] = r101(src.cols + x, src.cols);
    for (int y = -top; y < src.rows + bottom; ++y) {
        const uint8_t *s = &tmp[(size_t)r101(y, src.rows) * src.cols];
        uint8_t *d = dst.data + (size_t)(y + top) * dst.step;
        for (int x = 0; x < left; ++x) d[x] = s[lx[x]];
        std::memcpy(d + left, s, src.cols);
        for (int x = 0; x < right; ++x) d[left + src.cols + x] = s[rx[x]];
    }
}
}  // namespace cv
