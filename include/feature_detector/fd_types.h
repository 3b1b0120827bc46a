// fd_types.h -- the value types the detector API exchanges, restated without Eigen.
//
// The reference takes these from its un-vendored Slam_Utility repo (basic_type.h, datatype_image.h;
// SURVEY.md §2 C11). This header provides source-compatible equivalents for exactly the operations
// the detector classes and the reference demos use:
//   GrayImage (row-major u8 view, stride == cols: feature_point_harris_detector.cpp:31),
//   Vec2 / Vec4 / Pixel (x(), y() accessors, Zero/Identity/Constant), MatInt / MatImgF (row-major).
// Build with -DFD_USE_SLAM_UTILITY to compile the detectors against the real Slam_Utility headers
// instead (they must then be on the include path).
#ifndef FEATURE_DETECTOR_FD_TYPES_H_
#define FEATURE_DETECTOR_FD_TYPES_H_

#ifdef FD_USE_SLAM_UTILITY
#include "basic_type.h"
#include "datatype_image.h"
#else

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

// ---- fixed-size vectors ------------------------------------------------------------------------
template <typename T, int N>
class FdVec {
public:
    FdVec() { for (int i = 0; i < N; ++i) v_[i] = T(0); }
    template <typename A, typename B, typename = typename std::enable_if<N == 2 && std::is_arithmetic<A>::value &&
                                                                         std::is_arithmetic<B>::value>::type>
    FdVec(A x, B y) { v_[0] = static_cast<T>(x); v_[1] = static_cast<T>(y); }
    template <typename A, typename = typename std::enable_if<N == 4 && std::is_arithmetic<A>::value>::type>
    FdVec(A x, A y, A z, A w) {
        v_[0] = static_cast<T>(x); v_[1] = static_cast<T>(y); v_[2] = static_cast<T>(z); v_[3] = static_cast<T>(w);
    }
    static FdVec Zero() { return FdVec(); }
    static FdVec Constant(T c) { FdVec r; for (int i = 0; i < N; ++i) r.v_[i] = c; return r; }
    static FdVec Identity() { FdVec r; r.v_[0] = T(1); return r; }  // Eigen: Identity() of a column vector
    T &x() { return v_[0]; }
    T &y() { return v_[1]; }
    T &z() { return v_[2]; }
    T &w() { return v_[3]; }
    const T &x() const { return v_[0]; }
    const T &y() const { return v_[1]; }
    const T &z() const { return v_[2]; }
    const T &w() const { return v_[3]; }
    T &operator()(int i) { return v_[i]; }
    const T &operator()(int i) const { return v_[i]; }
    T &operator[](int i) { return v_[i]; }
    const T &operator[](int i) const { return v_[i]; }
    T *data() { return v_; }
    const T *data() const { return v_; }
    static constexpr int size() { return N; }
    FdVec operator+(const FdVec &o) const { FdVec r; for (int i = 0; i < N; ++i) r.v_[i] = v_[i] + o.v_[i]; return r; }
    FdVec operator-(const FdVec &o) const { FdVec r; for (int i = 0; i < N; ++i) r.v_[i] = v_[i] - o.v_[i]; return r; }
    FdVec operator*(T s) const { FdVec r; for (int i = 0; i < N; ++i) r.v_[i] = v_[i] * s; return r; }
    FdVec operator/(T s) const { FdVec r; for (int i = 0; i < N; ++i) r.v_[i] = v_[i] / s; return r; }
    FdVec &operator+=(const FdVec &o) { for (int i = 0; i < N; ++i) v_[i] += o.v_[i]; return *this; }
    FdVec &operator-=(const FdVec &o) { for (int i = 0; i < N; ++i) v_[i] -= o.v_[i]; return *this; }
    FdVec &operator*=(T s) { for (int i = 0; i < N; ++i) v_[i] *= s; return *this; }
    FdVec &operator/=(T s) { for (int i = 0; i < N; ++i) v_[i] /= s; return *this; }
    bool operator==(const FdVec &o) const { for (int i = 0; i < N; ++i) if (v_[i] != o.v_[i]) return false; return true; }

private:
    T v_[N];
};
template <typename T, int N>
FdVec<T, N> operator*(T s, const FdVec<T, N> &v) { return v * s; }

using Vec2 = FdVec<float, 2>;
using Vec4 = FdVec<float, 4>;
using Pixel = FdVec<int32_t, 2>;  // (col, row)

// ---- dynamic column vector (Vec = Eigen::VectorXf in the reference's basic_type.h) ------------------
template <typename T>
class FdVecX {
public:
    FdVecX() = default;
    explicit FdVecX(int n) : buf_(static_cast<size_t>(n), T(0)) {}
    void resize(int n) { buf_.resize(static_cast<size_t>(n)); }
    void setZero(int n) { buf_.assign(static_cast<size_t>(n), T(0)); }
    void setZero(int rows, int cols) { setZero(rows * cols); }  // descriptor.h:49 setZero(size, 1)
    void setZero() { for (auto &e : buf_) e = T(0); }
    T &operator[](int i) { return buf_[static_cast<size_t>(i)]; }
    const T &operator[](int i) const { return buf_[static_cast<size_t>(i)]; }
    T &operator()(int i) { return buf_[static_cast<size_t>(i)]; }
    const T &operator()(int i) const { return buf_[static_cast<size_t>(i)]; }
    int size() const { return static_cast<int>(buf_.size()); }
    int rows() const { return size(); }
    int cols() const { return 1; }
    T *data() { return buf_.data(); }
    const T *data() const { return buf_.data(); }

private:
    std::vector<T> buf_;
};
using Vec = FdVecX<float>;

// ---- row-major dynamic matrix (MatInt, MatImgF) -------------------------------------------------
template <typename T>
class FdMat {
public:
    FdMat() = default;
    FdMat(int rows, int cols) { resize(rows, cols); }
    void resize(int rows, int cols) {
        rows_ = rows;
        cols_ = cols;
        buf_.resize(static_cast<size_t>(rows) * static_cast<size_t>(cols));
    }
    void setConstant(int rows, int cols, T v) { resize(rows, cols); setConstant(v); }
    void setConstant(T v) { for (auto &e : buf_) e = v; }
    void setZero() { setConstant(T(0)); }
    void setZero(int rows, int cols) { setConstant(rows, cols, T(0)); }
    T &operator()(int r, int c) { return buf_[static_cast<size_t>(r) * cols_ + c]; }
    const T &operator()(int r, int c) const { return buf_[static_cast<size_t>(r) * cols_ + c]; }
    T *data() { return buf_.data(); }
    const T *data() const { return buf_.data(); }
    int rows() const { return rows_; }
    int cols() const { return cols_; }
    size_t size() const { return buf_.size(); }

private:
    int rows_ = 0, cols_ = 0;
    std::vector<T> buf_;
};
using MatInt = FdMat<int32_t>;
using MatImgF = FdMat<float>;

// ---- gray image view ------------------------------------------------------------------------------
// Row-major u8, stride == cols. `owns` = free the buffer (std::free) on destruction, as the
// reference's (ptr, rows, cols, owns) constructor (test_feature_line_detector.cpp:18).
class GrayImage {
public:
    GrayImage() = default;
    GrayImage(uint8_t *data, int32_t rows, int32_t cols, bool owns = false) { SetImage(data, rows, cols, owns); }
    ~GrayImage() { Release(); }
    GrayImage(const GrayImage &) = delete;
    GrayImage &operator=(const GrayImage &) = delete;
    void SetImage(uint8_t *data, int32_t rows, int32_t cols, bool owns = false) {
        Release();
        data_ = data;
        rows_ = rows;
        cols_ = cols;
        owns_ = owns;
    }
    uint8_t *data() const { return data_; }
    int32_t rows() const { return rows_; }
    int32_t cols() const { return cols_; }
    template <typename T = float>
    T GetPixelValueNoCheck(int32_t row, int32_t col) const {
        return static_cast<T>(data_[static_cast<size_t>(row) * cols_ + col]);
    }
    void SetPixelValueNoCheck(int32_t row, int32_t col, uint8_t v) { data_[static_cast<size_t>(row) * cols_ + col] = v; }

private:
    void Release() {
        if (owns_ && data_) std::free(data_);
        data_ = nullptr;
        owns_ = false;
    }
    uint8_t *data_ = nullptr;
    int32_t rows_ = 0, cols_ = 0;
    bool owns_ = false;
};

// slam_basic_math.h constants used by the line detector (feature_line_detector.h:42,
// feature_line_detector.cpp:17,200-202).
constexpr float kPai = 3.14159265358979323846f;
constexpr float k2Pai = 2.0f * kPai;
constexpr float kDegToRad = kPai / 180.0f;

#endif  // FD_USE_SLAM_UTILITY

#endif  // FEATURE_DETECTOR_FD_TYPES_H_
