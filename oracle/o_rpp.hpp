// ORACLE — test infrastructure only. Never linked into the product path.
//
// CPU restatement of the planar PnP used by mantis3:
//   CoPlanarPoseEstimator::estimatePose   include/mantis3/CoPlanarPoseEstimator.cpp:16-58
//   RPP::Rpp / ObjPose / AbsKernel / ...   include/mantis3/RobustPlanarPose/RPP.cpp:13-1222
//   rpoly_ak1 (Jenkins–Traub, TOMS 493)   include/mantis3/RobustPlanarPose/Rpoly.cpp:11-754
// plus OpenCV's JacobiSVDImpl_ / 3x3 closed-form inv() / det3 [3P] that
// RPP.cpp calls through cv::SVD, Mat::inv and cv::determinant.
#pragma once
#include <cstdint>
#include <vector>

namespace orc {

// Jenkins–Traub real-polynomial roots. op[0..deg] highest power first.
// zr/zi must hold `slots` entries pre-zeroed by the caller (RPP passes 5 slots
// for a quartic: slot 4 stays (0,0), reproducing SURVEY Q3).
// Returns the (possibly reduced) degree as rpoly_ak1 leaves it in *Degree.
int rpoly(const double* op, int deg, double* zr, double* zi);

// OpenCV JacobiSVD of an m x n row-major matrix A (flags = 0): w[min], u (m x
// n cols used), vt (n x n). Only the shapes RPP uses are exercised (3x3, 3x1).
void cv_svd(const double* A, int m, int n, double* w, double* u, double* vt);

struct RppResult {
  double R[9];
  double t[3];
  double obj_err, img_err;
  int iterations;
  int status;  // 1 = Rpp returned true; 0 = 2nd-pose search failed (R,t from first ObjPose)
  int error;   // 0 ok; 1 = GetRotationbyVector check failed (reference exit(1));
               // 2 = ObjPose iteration cap hit
};

// model: 3 x n (row-major, rows x,y,z); iprts: 3 x n homogeneous image points.
RppResult rpp(const double* model, const double* iprts, int n);

}  // namespace orc
