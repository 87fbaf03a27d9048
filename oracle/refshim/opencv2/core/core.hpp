// ORACLE build aid — NOT OpenCV. A minimal, eager cv::Mat (CV_64F only) that is
// just enough to compile the reference's own
//   /root/reference/include/mantis3/RobustPlanarPose/RPP.cpp
// in place (the source is read from /root/reference at build time and never
// copied). Numerics follow the OpenCV 3.x rules RPP depends on:
//  * Mat copies share data (AbsKernel relies on in-place writes, RPP.cpp:236-256)
//  * A / s multiplies by (1/s); gemm sums k in order from 0
//  * SVD is OpenCV's one-sided JacobiSVD (restated in oracle/o_rpp.cpp)
//  * inv() / determinant() use the 3x3 closed forms.
// Built by oracle/Makefile into oracle/_ref/ only.
#pragma once
#include <cassert>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

namespace orc {
void cv_svd(const double* A, int m, int n, double* w, double* u, double* vt);
}

#ifndef CV_64F
#define CV_64F 6
#endif
#ifndef CV_PI
#define CV_PI 3.1415926535897932384626433832795
#endif

extern "C" void mantis_ref_exit(int code);
#define exit mantis_ref_exit

namespace cv {
typedef unsigned char uchar;

template <typename T, int n>
struct Vec {
  T val[n];
  Vec() { for (int i = 0; i < n; i++) val[i] = 0; }
  Vec(T a, T b, T c) { val[0] = a; val[1] = b; val[2] = c; }
  T& operator[](int i) { return val[i]; }
  const T& operator[](int i) const { return val[i]; }
  T dot(const Vec& o) const { T s = 0; s = val[0] * o.val[0] + val[1] * o.val[1] + val[2] * o.val[2]; return s; }
  Vec cross(const Vec& v) const {
    return Vec(val[1] * v.val[2] - val[2] * v.val[1], val[2] * v.val[0] - val[0] * v.val[2],
               val[0] * v.val[1] - val[1] * v.val[0]);
  }
  Vec operator-() const { return Vec(-val[0], -val[1], -val[2]); }
};
typedef Vec<double, 3> Vec3d;

template <typename T>
struct Point_ { T x, y; Point_() : x(0), y(0) {} Point_(T a, T b) : x(a), y(b) {} };
template <typename T>
struct Point3_ { T x, y, z; Point3_() : x(0), y(0), z(0) {} Point3_(T a, T b, T c) : x(a), y(b), z(c) {} };
typedef Point_<double> Point2d;
typedef Point3_<double> Point3d;

class Mat {
 public:
  int rows = 0, cols = 0;
  uchar* data = nullptr;
  std::shared_ptr<std::vector<double>> buf;
  Mat() {}
  Mat(int r, int c, int type) { create(r, c, type); }
  void create(int r, int c, int /*type*/) {
    if (buf && rows == r && cols == c) return;
    rows = r; cols = c;
    buf = std::make_shared<std::vector<double>>((size_t)(r * c > 0 ? r * c : 1), 0.0);
    data = (r * c > 0) ? (uchar*)buf->data() : (uchar*)buf->data();
  }
  double* p() const { return buf->data(); }
  template <typename T> T& at(int i, int j) { return p()[i * cols + j]; }
  template <typename T> const T& at(int i, int j) const { return p()[i * cols + j]; }
  template <typename T> T& at(int k) { return p()[k]; }
  template <typename T> const T& at(int k) const { return p()[k]; }
  Mat clone() const { Mat m(rows, cols, CV_64F); std::memcpy(m.p(), p(), sizeof(double) * rows * cols); return m; }
  static Mat zeros(int r, int c, int t) { return Mat(r, c, t); }
  static Mat ones(int r, int c, int t) { Mat m(r, c, t); for (int i = 0; i < r * c; i++) m.p()[i] = 1; return m; }
  static Mat eye(int r, int c, int t) { Mat m(r, c, t); for (int i = 0; i < r && i < c; i++) m.at<double>(i, i) = 1; return m; }
  Mat t() const { Mat m(cols, rows, CV_64F); for (int i = 0; i < rows; i++) for (int j = 0; j < cols; j++) m.at<double>(j, i) = at<double>(i, j); return m; }
  Mat inv() const {
    const Mat& M = *this;
    Mat D(3, 3, CV_64F);
    auto m = [&](int i, int j) { return M.at<double>(i, j); };
    double d = m(0, 0) * (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) - m(0, 1) * (m(1, 0) * m(2, 2) - m(1, 2) * m(2, 0)) +
               m(0, 2) * (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0));
    if (d == 0.) return D;
    d = 1. / d;
    D.at<double>(0, 0) = (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) * d;
    D.at<double>(0, 1) = (m(0, 2) * m(2, 1) - m(0, 1) * m(2, 2)) * d;
    D.at<double>(0, 2) = (m(0, 1) * m(1, 2) - m(0, 2) * m(1, 1)) * d;
    D.at<double>(1, 0) = (m(1, 2) * m(2, 0) - m(1, 0) * m(2, 2)) * d;
    D.at<double>(1, 1) = (m(0, 0) * m(2, 2) - m(0, 2) * m(2, 0)) * d;
    D.at<double>(1, 2) = (m(0, 2) * m(1, 0) - m(0, 0) * m(1, 2)) * d;
    D.at<double>(2, 0) = (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0)) * d;
    D.at<double>(2, 1) = (m(0, 1) * m(2, 0) - m(0, 0) * m(2, 1)) * d;
    D.at<double>(2, 2) = (m(0, 0) * m(1, 1) - m(0, 1) * m(1, 0)) * d;
    return D;
  }
  Mat& operator+=(const Mat& o) { for (int i = 0; i < rows * cols; i++) p()[i] = p()[i] + o.p()[i]; return *this; }
};

inline Mat operator*(const Mat& A, const Mat& B) {
  Mat o(A.rows, B.cols, CV_64F);
  for (int i = 0; i < A.rows; i++)
    for (int j = 0; j < B.cols; j++) {
      double s = 0;
      for (int k = 0; k < A.cols; k++) s += A.at<double>(i, k) * B.at<double>(k, j);
      o.at<double>(i, j) = s;
    }
  return o;
}
inline Mat operator*(const Mat& A, double s) { Mat o(A.rows, A.cols, CV_64F); for (int i = 0; i < A.rows * A.cols; i++) o.p()[i] = A.p()[i] * s; return o; }
inline Mat operator*(double s, const Mat& A) { return A * s; }
inline Mat operator/(const Mat& A, double s) { return A * (1. / s); }
inline Mat operator+(const Mat& A, const Mat& B) { Mat o(A.rows, A.cols, CV_64F); for (int i = 0; i < A.rows * A.cols; i++) o.p()[i] = A.p()[i] + B.p()[i]; return o; }
inline Mat operator-(const Mat& A, const Mat& B) { Mat o(A.rows, A.cols, CV_64F); for (int i = 0; i < A.rows * A.cols; i++) o.p()[i] = A.p()[i] - B.p()[i]; return o; }
inline Mat operator-(const Mat& A) { return A * -1.0; }

inline double determinant(const Mat& M) {
  auto m = [&](int i, int j) { return M.at<double>(i, j); };
  return m(0, 0) * (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) - m(0, 1) * (m(1, 0) * m(2, 2) - m(1, 2) * m(2, 0)) +
         m(0, 2) * (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0));
}

class SVD {
 public:
  Mat u, w, vt;
  explicit SVD(const Mat& A) {
    int m = A.rows, n = A.cols;
    u = Mat(m, n, CV_64F);
    w = Mat(n, 1, CV_64F);
    vt = Mat(n, n, CV_64F);
    orc::cv_svd(A.p(), m, n, w.p(), u.p(), vt.p());
  }
};
}  // namespace cv
