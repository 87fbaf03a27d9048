// ORACLE build aid — a C entry point over the reference's own Rpoly.cpp,
// compiled in place from /root/reference (Makefile target `ref`). Rpoly.cpp
// needs nothing beyond the C++ standard library, so it builds from its own
// sources. RPP.cpp is NOT built: it needs OpenCV core (cv::Mat, cv::SVD),
// which this image lacks, so it is unbuildable here; the RPP
// restatement is pinned by demo.cpp's known answer instead. Used only by
// tests/ to pin the oracle's rpoly (o_rpp.cpp) and by make_golden.py.
#include <cstring>

#include "Rpoly.h"

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
