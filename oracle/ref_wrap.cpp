// ORACLE build aid — C entry points over the reference's own RPP.cpp and
// Rpoly.cpp compiled in place from /root/reference (see Makefile target
// `ref`). Used only by tests/ to pin the oracle restatement (o_rpp.cpp).
#include <csetjmp>
#include <cstring>

#include "RPP.h"

static jmp_buf g_jb;
extern "C" void mantis_ref_exit(int code) { longjmp(g_jb, code ? code : 1); }

extern "C" int ref_rpp(const double* model, const double* iprts, int n, double* R, double* t, double* errs) {
  cv::Mat m(3, n, CV_64F), ip(3, n, CV_64F);
  for (int i = 0; i < 3 * n; i++) {
    m.at<double>(i) = model[i];
    ip.at<double>(i) = iprts[i];
  }
  cv::Mat rot, tvec;
  int it = 0;
  double oe = 0, ie = 0;
  if (setjmp(g_jb)) return -1;  // reference called exit(1) (GetRotationbyVector)
  bool ok = RPP::Rpp(m, ip, rot, tvec, it, oe, ie);
  for (int i = 0; i < 9; i++) R[i] = rot.at<double>(i);
  for (int i = 0; i < 3; i++) t[i] = tvec.at<double>(i);
  errs[0] = oe;
  errs[1] = ie;
  errs[2] = it;
  return ok ? 1 : 0;
}

extern "C" int ref_rpoly(const double* op, int deg, double* zr, double* zi) {
  double o[MDP1], r[MAXDEGREE], im[MAXDEGREE];
  std::memset(o, 0, sizeof(o));
  std::memset(r, 0, sizeof(r));
  std::memset(im, 0, sizeof(im));
  for (int i = 0; i <= deg; i++) o[i] = op[i];
  int d = deg;
  rpoly_ak1(o, &d, r, im);
  for (int i = 0; i < deg + 1; i++) { zr[i] = r[i]; zi[i] = im[i]; }
  return d;
}
