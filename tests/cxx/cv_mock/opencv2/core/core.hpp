// Minimal stand-in for the parts of OpenCV's core API that
// include/orbx_orbslam2.hpp uses, so the drop-in adapter can be compiled and
// exercised in this OpenCV-free container.  Test scaffolding for OUR adapter
// only (nothing of the reference is built against it).
#pragma once
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
    for (int y = -top; y < src.rows + bottom; ++y)
        for (int x = -left; x < src.cols + right; ++x)
            dst.data[(y + top) * dst.step + (x + left)] = tmp[(size_t)r101(y, src.rows) * src.cols + r101(x, src.cols)];
}
}  // namespace cv
