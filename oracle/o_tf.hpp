// ORACLE — test infrastructure only. Never linked into the product path.
//
// CPU restatement of the subset of ROS tf/LinearMath (tfScalar = double) that
// the mantis3 hot path uses. The reference includes <tf/tf.h> (not vendored):
//   Hypothesis::setC2W/setW2C       include/mantis3/Mantis3Types.h:68-80
//   Hypothesis::projectPoint        include/mantis3/Mantis3Types.h:88-93
//   rotZ yaw copies                 include/mantis3/HypothesisGeneration.h:91-99
//   generateRandomHypothesis        include/mantis3/PoseAdjustment.h:13-23
//   Pose::getEuler (getRPY)         include/mantis3/PoseClusterer.h:198-205
// Semantics restated from the published LinearMath sources [3P, unpinned]:
// Matrix3x3(q) uses s = 2/|q|^2, getRotation is Shepperd's method,
// getRPY = getEulerYPR solution 1, setRPY(r,p,y) = setEulerYPR(y,p,r),
// Transform::inverse = (R^T, R^T * -t).
#pragma once
#include <cmath>

namespace orc {

struct Vec3 {
  double v[3];
  Vec3() : v{0, 0, 0} {}
  Vec3(double x, double y, double z) : v{x, y, z} {}
  double x() const { return v[0]; }
  double y() const { return v[1]; }
  double z() const { return v[2]; }
  double& operator[](int i) { return v[i]; }
  double operator[](int i) const { return v[i]; }
  double dot(const Vec3& o) const { return v[0] * o.v[0] + v[1] * o.v[1] + v[2] * o.v[2]; }
  Vec3 operator-() const { return Vec3(-v[0], -v[1], -v[2]); }
  Vec3 operator+(const Vec3& o) const { return Vec3(v[0] + o.v[0], v[1] + o.v[1], v[2] + o.v[2]); }
  Vec3 operator-(const Vec3& o) const { return Vec3(v[0] - o.v[0], v[1] - o.v[1], v[2] - o.v[2]); }
  Vec3& operator+=(const Vec3& o) { v[0] += o.v[0]; v[1] += o.v[1]; v[2] += o.v[2]; return *this; }
};

struct Quat {  // (x, y, z, w) as in the tf constructor
  double x, y, z, w;
  Quat() : x(0), y(0), z(0), w(1) {}
  Quat(double x_, double y_, double z_, double w_) : x(x_), y(y_), z(z_), w(w_) {}
  double length2() const { return x * x + y * y + z * z + w * w; }
};

struct Mat3 {
  Vec3 r[3];  // rows
  Mat3() {}
  Mat3(double a, double b, double c, double d, double e, double f, double g, double h, double i) {
    r[0] = Vec3(a, b, c); r[1] = Vec3(d, e, f); r[2] = Vec3(g, h, i);
  }
  static Mat3 identity() { return Mat3(1, 0, 0, 0, 1, 0, 0, 0, 1); }
  explicit Mat3(const Quat& q) { setRotation(q); }
  double operator()(int i, int j) const { return r[i][j]; }

  void setRotation(const Quat& q) {
    double d = q.length2();
    double s = 2.0 / d;
    double xs = q.x * s, ys = q.y * s, zs = q.z * s;
    double wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
    double xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
    double yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
    *this = Mat3(1.0 - (yy + zz), xy - wz, xz + wy,
                 xy + wz, 1.0 - (xx + zz), yz - wx,
                 xz - wy, yz + wx, 1.0 - (xx + yy));
  }

  Quat getRotation() const {
    double trace = r[0][0] + r[1][1] + r[2][2];
    double t[4];
    if (trace > 0.0) {
      double s = std::sqrt(trace + 1.0);
      t[3] = s * 0.5;
      s = 0.5 / s;
      t[0] = (r[2][1] - r[1][2]) * s;
      t[1] = (r[0][2] - r[2][0]) * s;
      t[2] = (r[1][0] - r[0][1]) * s;
    } else {
      int i = r[0][0] < r[1][1] ? (r[1][1] < r[2][2] ? 2 : 1) : (r[0][0] < r[2][2] ? 2 : 0);
      int j = (i + 1) % 3;
      int k = (i + 2) % 3;
      double s = std::sqrt(r[i][i] - r[j][j] - r[k][k] + 1.0);
      t[i] = s * 0.5;
      s = 0.5 / s;
      t[3] = (r[k][j] - r[j][k]) * s;
      t[j] = (r[j][i] + r[i][j]) * s;
      t[k] = (r[k][i] + r[i][k]) * s;
    }
    return Quat(t[0], t[1], t[2], t[3]);
  }

  // tf setEulerYPR(eulerZ, eulerY, eulerX)
  void setEulerYPR(double ez, double ey, double ex) {
    double ci = std::cos(ex), cj = std::cos(ey), ch = std::cos(ez);
    double si = std::sin(ex), sj = std::sin(ey), sh = std::sin(ez);
    double cc = ci * ch, cs = ci * sh, sc = si * ch, ss = si * sh;
    *this = Mat3(cj * ch, sj * sc - cs, sj * cc + ss,
                 cj * sh, sj * ss + cc, sj * cs - sc,
                 -sj, cj * si, cj * ci);
  }
  void setRPY(double roll, double pitch, double yaw) { setEulerYPR(yaw, pitch, roll); }

  // tf getEulerYPR(yaw, pitch, roll, solution_number = 1); getRPY(r, p, y)
  void getRPY(double& roll, double& pitch, double& yaw) const {
    if (std::fabs(r[2][0]) >= 1) {
      yaw = 0;
      double delta = std::atan2(r[2][1], r[2][2]);
      pitch = (r[2][0] < 0) ? M_PI / 2.0 : -M_PI / 2.0;
      roll = delta;
    } else {
      pitch = -std::asin(r[2][0]);
      double cp = std::cos(pitch);
      roll = std::atan2(r[2][1] / cp, r[2][2] / cp);
      yaw = std::atan2(r[1][0] / cp, r[0][0] / cp);
    }
  }

  Mat3 transpose() const {
    return Mat3(r[0][0], r[1][0], r[2][0], r[0][1], r[1][1], r[2][1], r[0][2], r[1][2], r[2][2]);
  }
  // m2.tdotx(v) = m2[0].x*v.x + m2[1].x*v.y + m2[2].x*v.z
  Mat3 operator*(const Mat3& m2) const {
    Mat3 o;
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        o.r[i][j] = m2.r[0][j] * r[i][0] + m2.r[1][j] * r[i][1] + m2.r[2][j] * r[i][2];
    return o;
  }
  Vec3 operator*(const Vec3& v) const { return Vec3(r[0].dot(v), r[1].dot(v), r[2].dot(v)); }
};

struct Transform {
  Mat3 basis;
  Vec3 origin;
  Transform() : basis(Mat3::identity()) {}
  Transform(const Mat3& b, const Vec3& c) : basis(b), origin(c) {}
  explicit Transform(const Quat& q, const Vec3& c = Vec3()) : basis(q), origin(c) {}
  Vec3 operator()(const Vec3& x) const {
    return Vec3(basis.r[0].dot(x) + origin[0], basis.r[1].dot(x) + origin[1], basis.r[2].dot(x) + origin[2]);
  }
  Vec3 operator*(const Vec3& x) const { return (*this)(x); }
  Transform operator*(const Transform& t) const { return Transform(basis * t.basis, (*this)(t.origin)); }
  Transform inverse() const {
    Mat3 inv = basis.transpose();
    return Transform(inv, inv * (-origin));
  }
  Quat getRotation() const { return basis.getRotation(); }
};

// Hypothesis (Mantis3Types.h:26-161): c2w maps WORLD points into the camera
// frame (despite its name); w2c is the camera pose in the world.
struct Hypothesis {
  Transform c2w, w2c;
  Quat q;
  double error = 0;
  void setC2W(const Transform& t) { c2w = t; w2c = c2w.inverse(); q = w2c.getRotation(); }
  void setW2C(const Transform& t) { w2c = t; c2w = w2c.inverse(); q = w2c.getRotation(); }
  Vec3 position() const { return w2c.origin; }
};

}  // namespace orc
