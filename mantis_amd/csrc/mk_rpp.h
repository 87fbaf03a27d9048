// Robust planar pose (Schweighofer–Pinz RPP) for the 4-point problems of
// CoPlanarPoseEstimator::estimatePose (include/mantis3/CoPlanarPoseEstimator.cpp:16-58),
// as FP64 device/host code: one work-item per (quad, orientation).
//   Rpp / ObjPose / AbsKernel / EstimateT     RPP.cpp:13-332
//   Get2ndPose_Exact / GetRfor2ndPose_V_Exact  RPP.cpp:693-753, 847-945
//   GetRotationY_wrtT (quartic)               RPP.cpp:947-1222
//   DecomposeR / RpyAng(_X) / RpyMat          RPP.cpp:563-808
//   GetRotationbyVector                       RPP.cpp:425-456 (exit(1) -> status -1)
//   rpoly_ak1 Jenkins–Traub                   Rpoly.cpp:11-754 (degree <= 4 here)
// plus OpenCV's one-sided JacobiSVD and 3x3 closed-form inverse/determinant
// (what cv::SVD / Mat::inv / cv::determinant compute for these shapes).
// The cv::Mat evaluation rules that move results by ulps are kept: "A / s"
// multiplies by 1/s, gemm sums k from 0, AbsKernel overwrites its P and Q in
// place, Mean() divides by the column count.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstring>

#include "mk_math.h"

namespace mk {
namespace rpp {

template <class T>
MK_HD void swp(T& a, T& b) { T t = a; a = b; b = t; }

// ------------------------------------------------------------ Jenkins–Traub
MK_HD void jt_quadsd(int nn, double u, double v, const double* p, double* q, double* a, double* b) {
  q[0] = *b = p[0];
  q[1] = *a = -((*b) * u) + p[1];
  for (int i = 2; i < nn; i++) {
    q[i] = -((*a) * u + (*b) * v) + p[i];
    *b = *a;
    *a = q[i];
  }
}
MK_HD int jt_calcsc(int n, double a, double b, double* a1, double* a3, double* a7, double* c, double* d, double* e,
                    double* f, double* g, double* h, const double* K, double u, double v, double* qk) {
  jt_quadsd(n, u, v, K, qk, c, d);
  if (fabs(*c) <= 100.0 * DBL_EPSILON * fabs(K[n - 1]))
    if (fabs(*d) <= 100.0 * DBL_EPSILON * fabs(K[n - 2])) return 3;
  *h = v * b;
  if (fabs(*d) >= fabs(*c)) {
    *e = a / (*d);
    *f = (*c) / (*d);
    *g = u * b;
    *a3 = (*e) * ((*g) + a) + (*h) * (b / (*d));
    *a1 = -a + (*f) * b;
    *a7 = (*h) + ((*f) + u) * a;
    return 2;
  }
  *e = a / (*c);
  *f = (*d) / (*c);
  *g = (*e) * u;
  *a3 = (*e) * a + ((*g) + (*h) / (*c)) * b;
  *a1 = -(a * ((*d) / (*c))) + b;
  *a7 = (*g) * (*d) + (*h) * (*f) + a;
  return 1;
}
MK_HD void jt_nextk(int n, int tflag, double a, double b, double a1, double* a3, double* a7, double* K,
                    const double* qk, const double* qp) {
  if (tflag == 3) {
    K[1] = K[0] = 0.0;
    for (int i = 2; i < n; i++) K[i] = qk[i - 2];
    return;
  }
  double temp = (tflag == 1) ? b : a;
  if (fabs(a1) > 10.0 * DBL_EPSILON * fabs(temp)) {
    (*a7) /= a1;
    (*a3) /= a1;
    K[0] = qp[0];
    K[1] = -((*a7) * qp[0]) + qp[1];
    for (int i = 2; i < n; i++) K[i] = -((*a7) * qp[i - 1]) + (*a3) * qk[i - 2] + qp[i];
  } else {
    K[0] = 0.0;
    K[1] = -(*a7) * qp[0];
    for (int i = 2; i < n; i++) K[i] = -((*a7) * qp[i - 1]) + (*a3) * qk[i - 2];
  }
}
MK_HD void jt_newest(int tflag, double* uu, double* vv, double a, double a1, double a3, double a7, double b, double c,
                     double d, double f, double g, double h, double u, double v, const double* K, int n,
                     const double* p) {
  *vv = *uu = 0.0;
  if (tflag == 3) return;
  double a4, a5;
  if (tflag != 2) {
    a4 = a + u * b + h * f;
    a5 = c + (u + v * f) * d;
  } else {
    a4 = (a + g) * f + h;
    a5 = (f + u) * c + v * d;
  }
  double b1 = -K[n - 1] / p[n];
  double b2 = -(K[n - 2] + b1 * p[n - 1]) / p[n];
  double c1 = v * b2 * a1;
  double c2 = b1 * a7;
  double c3 = b1 * b1 * a3;
  double c4 = -(c2 + c3) + c1;
  double temp = -c4 + a5 + b1 * a4;
  if (temp != 0.0) {
    *uu = -((u * (c3 + c2) + v * (b1 * a1 + b2 * a7)) / temp) + u;
    *vv = v * (1.0 + c4 / temp);
  }
}
MK_HD void jt_quad(double a, double b1, double c, double* sr, double* si, double* lr, double* li) {
  *sr = *si = *lr = *li = 0.0;
  if (a == 0) {
    *sr = (b1 != 0) ? -(c / b1) : *sr;
    return;
  }
  if (c == 0) {
    *lr = -(b1 / a);
    return;
  }
  double b = b1 / 2.0, d, e;
  if (fabs(b) < fabs(c)) {
    e = (c >= 0) ? a : -a;
    e = -e + b * (b / fabs(c));
    d = sqrt(fabs(e)) * sqrt(fabs(c));
  } else {
    e = -((a / b) * (c / b)) + 1.0;
    d = sqrt(fabs(e)) * fabs(b);
  }
  if (e >= 0) {
    d = (b >= 0) ? -d : d;
    *lr = (-b + d) / a;
    *sr = (*lr != 0) ? (c / (*lr)) / a : *sr;
  } else {
    *lr = *sr = -(b / a);
    *si = fabs(d / a);
    *li = -(*si);
  }
}
MK_HD void jt_quadit(int n, int* nz, double uu, double vv, double* szr, double* szi, double* lzr, double* lzi,
                     double* qp, int nn, double* a, double* b, const double* p, double* qk, double* a1, double* a3,
                     double* a7, double* c, double* d, double* e, double* f, double* g, double* h, double* K) {
  int j = 0, tflag, tried = 0;
  double ee, mp, omp = 0, relstp = 0, t, u, ui = 0, v, vi = 0, zm;
  *nz = 0;
  u = uu;
  v = vv;
  do {
    jt_quad(1.0, u, v, szr, szi, lzr, lzi);
    if (fabs(fabs(*szr) - fabs(*lzr)) > 0.01 * fabs(*lzr)) break;
    jt_quadsd(nn, u, v, p, qp, a, b);
    mp = fabs(-((*szr) * (*b)) + (*a)) + fabs((*szi) * (*b));
    zm = sqrt(fabs(v));
    ee = 2.0 * fabs(qp[0]);
    t = -((*szr) * (*b));
    for (int i = 1; i < n; i++) ee = ee * zm + fabs(qp[i]);
    ee = ee * zm + fabs((*a) + t);
    ee = (9.0 * ee + 2.0 * fabs(t) - 7.0 * (fabs((*a) + t) + zm * fabs(*b))) * DBL_EPSILON;
    if (mp <= 20.0 * ee) {
      *nz = 2;
      break;
    }
    j++;
    if (j > 20) break;
    if (j >= 2) {
      if ((relstp <= 0.01) && (mp >= omp) && (!tried)) {
        relstp = (relstp < DBL_EPSILON) ? sqrt(DBL_EPSILON) : sqrt(relstp);
        u -= u * relstp;
        v += v * relstp;
        jt_quadsd(nn, u, v, p, qp, a, b);
        for (int i = 0; i < 5; i++) {
          tflag = jt_calcsc(n, *a, *b, a1, a3, a7, c, d, e, f, g, h, K, u, v, qk);
          jt_nextk(n, tflag, *a, *b, *a1, a3, a7, K, qk, qp);
        }
        tried = 1;
        j = 0;
      }
    }
    omp = mp;
    tflag = jt_calcsc(n, *a, *b, a1, a3, a7, c, d, e, f, g, h, K, u, v, qk);
    jt_nextk(n, tflag, *a, *b, *a1, a3, a7, K, qk, qp);
    tflag = jt_calcsc(n, *a, *b, a1, a3, a7, c, d, e, f, g, h, K, u, v, qk);
    jt_newest(tflag, &ui, &vi, *a, *a1, *a3, *a7, *b, *c, *d, *f, *g, *h, u, v, K, n, p);
    if (vi != 0) {
      relstp = fabs((-v + vi) / vi);
      u = ui;
      v = vi;
    }
  } while (vi != 0);
}
MK_HD void jt_realit(int* iflag, int* nz, double* sss, int n, const double* p, int nn, double* qp, double* szr,
                     double* szi, double* K, double* qk) {
  int j = 0, nm1 = n - 1;
  double ee, kv, mp, ms, omp = 0, pv, s, t = 0;
  *iflag = *nz = 0;
  s = *sss;
  for (;;) {
    pv = p[0];
    qp[0] = pv;
    for (int i = 1; i < nn; i++) qp[i] = pv = pv * s + p[i];
    mp = fabs(pv);
    ms = fabs(s);
    ee = 0.5 * fabs(qp[0]);
    for (int i = 1; i < nn; i++) ee = ee * ms + fabs(qp[i]);
    if (mp <= 20.0 * DBL_EPSILON * (2.0 * ee - mp)) {
      *nz = 1;
      *szr = s;
      *szi = 0.0;
      break;
    }
    j++;
    if (j > 10) break;
    if (j >= 2) {
      if ((fabs(t) <= 0.001 * fabs(-t + s)) && (mp > omp)) {
        *iflag = 1;
        *sss = s;
        break;
      }
    }
    omp = mp;
    qk[0] = kv = K[0];
    for (int i = 1; i < n; i++) qk[i] = kv = kv * s + K[i];
    if (fabs(kv) > fabs(K[nm1]) * 10.0 * DBL_EPSILON) {
      t = -(pv / kv);
      K[0] = qp[0];
      for (int i = 1; i < n; i++) K[i] = t * qk[i - 1] + qp[i];
    } else {
      K[0] = 0.0;
      for (int i = 1; i < n; i++) K[i] = qk[i - 1];
    }
    kv = K[0];
    for (int i = 1; i < n; i++) kv = kv * s + K[i];
    t = (fabs(kv) > fabs(K[nm1]) * 10.0 * DBL_EPSILON) ? -(pv / kv) : 0.0;
    s += t;
  }
}
MK_HD void jt_fxshfr(int l2, int* nz, double sr, double v, double* K, int n, const double* p, int nn, double* qp,
                     double u, double* lzi, double* lzr, double* szi, double* szr) {
  int fflag, iflag = 1, spass, stry, tflag, vpass, vtry;
  double a, a1, a3, a7, b, betas, betav, c, d, e, f, g, h, oss, ots = 0, otv = 0, ovv, s, ss, ts, tss, tv, tvv, ui,
      vi, vv;
  double qk[8], svk[8];
  *nz = 0;
  betav = betas = 0.25;
  oss = sr;
  ovv = v;
  jt_quadsd(nn, u, v, p, qp, &a, &b);
  tflag = jt_calcsc(n, a, b, &a1, &a3, &a7, &c, &d, &e, &f, &g, &h, K, u, v, qk);
  for (int j = 0; j < l2; j++) {
    fflag = 1;
    jt_nextk(n, tflag, a, b, a1, &a3, &a7, K, qk, qp);
    tflag = jt_calcsc(n, a, b, &a1, &a3, &a7, &c, &d, &e, &f, &g, &h, K, u, v, qk);
    jt_newest(tflag, &ui, &vi, a, a1, a3, a7, b, c, d, f, g, h, u, v, K, n, p);
    vv = vi;
    ss = (K[n - 1] != 0.0) ? -(p[n] / K[n - 1]) : 0.0;
    ts = tv = 1.0;
    if ((j != 0) && (tflag != 3)) {
      tv = (vv != 0.0) ? fabs((vv - ovv) / vv) : tv;
      ts = (ss != 0.0) ? fabs((ss - oss) / ss) : ts;
      tvv = (tv < otv) ? tv * otv : 1.0;
      tss = (ts < ots) ? ts * ots : 1.0;
      vpass = (tvv < betav) ? 1 : 0;
      spass = (tss < betas) ? 1 : 0;
      if (spass || vpass) {
        for (int i = 0; i < n; i++) svk[i] = K[i];
        s = ss;
        stry = vtry = 0;
        for (;;) {
          bool skip_quad = false;
          if (fflag) {
            fflag = 0;
            skip_quad = spass && (!vpass || (tss < tvv));
          }
          if (!skip_quad) {
            jt_quadit(n, nz, ui, vi, szr, szi, lzr, lzi, qp, nn, &a, &b, p, qk, &a1, &a3, &a7, &c, &d, &e, &f, &g, &h,
                      K);
            if (*nz > 0) return;
            iflag = vtry = 1;
            betav *= 0.25;
            if (stry || !spass) {
              iflag = 0;
            } else {
              for (int i = 0; i < n; i++) K[i] = svk[i];
            }
          }
          if (iflag != 0) {
            jt_realit(&iflag, nz, &s, n, p, nn, qp, szr, szi, K, qk);
            if (*nz > 0) return;
            stry = 1;
            betas *= 0.25;
            if (iflag != 0) {
              ui = -(s + s);
              vi = s * s;
              continue;
            }
          }
          for (int i = 0; i < n; i++) K[i] = svk[i];
          if (!vpass || vtry) break;
        }
        jt_quadsd(nn, u, v, p, qp, &a, &b);
        tflag = jt_calcsc(n, a, b, &a1, &a3, &a7, &c, &d, &e, &f, &g, &h, K, u, v, qk);
      }
    }
    ovv = vv;
    oss = ss;
    otv = tv;
    ots = ts;
  }
}

// rpoly_ak1 for degree <= 6; zeror/zeroi pre-zeroed by the caller.
MK_HD int rpoly(const double* op, int degree, double* zeror, double* zeroi) {
  double K[8], p[8], pt[8], qp[8], temp[8];
  const double RADFAC = 3.14159265358979323846 / 180;
  const double lb2 = log(2.0);
  const double lo = DBL_MIN / DBL_EPSILON;
  const double cosr = cos(94.0 * RADFAC);
  const double sinr = sin(94.0 * RADFAC);
  if (degree > 6) return -1;
  if (op[0] == 0) return 0;
  int N = degree, NN, NM1, NZ, l, zerok, j, jj;
  double xx = sqrt(0.5), yy = -xx, bnd, df, dx, factor, ff, mx, mn, sc, x, xm, aa, bb, cc, lzi, lzr, sr, szi, szr, t,
         u, xxx;
  j = 0;
  while (op[N] == 0) {
    zeror[j] = zeroi[j] = 0.0;
    N--;
    j++;
  }
  NN = N + 1;
  for (int i = 0; i < NN; i++) p[i] = op[i];
  while (N >= 1) {
    if (N <= 2) {
      if (N < 2) {
        zeror[degree - 1] = -(p[1] / p[0]);
        zeroi[degree - 1] = 0.0;
      } else {
        jt_quad(p[0], p[1], p[2], &zeror[degree - 2], &zeroi[degree - 2], &zeror[degree - 1], &zeroi[degree - 1]);
      }
      break;
    }
    mx = 0.0;
    mn = DBL_MAX;
    for (int i = 0; i < NN; i++) {
      x = fabs(p[i]);
      if (x > mx) mx = x;
      if ((x != 0) && (x < mn)) mn = x;
    }
    sc = lo / mn;
    if (((sc <= 1.0) && (mx >= 10)) || ((sc > 1.0) && (DBL_MAX / sc >= mx))) {
      sc = (sc == 0) ? DBL_MIN : sc;
      l = (int)(log(sc) / lb2 + 0.5);
      factor = pow(2.0, (double)l);
      if (factor != 1.0)
        for (int i = 0; i < NN; i++) p[i] *= factor;
    }
    for (int i = 0; i < NN; i++) pt[i] = fabs(p[i]);
    pt[N] = -(pt[N]);
    NM1 = N - 1;
    x = exp((log(-pt[N]) - log(pt[0])) / (double)N);
    if (pt[NM1] != 0) {
      xm = -pt[N] / pt[NM1];
      x = (xm < x) ? xm : x;
    }
    xm = x;
    do {
      x = xm;
      xm = 0.1 * x;
      ff = pt[0];
      for (int i = 1; i < NN; i++) ff = ff * xm + pt[i];
    } while (ff > 0);
    dx = x;
    do {
      df = ff = pt[0];
      for (int i = 1; i < N; i++) {
        ff = x * ff + pt[i];
        df = x * df + ff;
      }
      ff = x * ff + pt[N];
      dx = ff / df;
      x -= dx;
    } while (fabs(dx / x) > 0.005);
    bnd = x;
    for (int i = 1; i < N; i++) K[i] = (double)(N - i) * p[i] / ((double)N);
    K[0] = p[0];
    aa = p[N];
    bb = p[NM1];
    zerok = (K[NM1] == 0) ? 1 : 0;
    for (jj = 0; jj < 5; jj++) {
      cc = K[NM1];
      if (zerok) {
        for (int i = 0; i < NM1; i++) {
          int k = NM1 - i;
          K[k] = K[k - 1];
        }
        K[0] = 0;
        zerok = (K[NM1] == 0) ? 1 : 0;
      } else {
        t = -aa / cc;
        for (int i = 0; i < NM1; i++) {
          int k = NM1 - i;
          K[k] = t * K[k - 1] + p[k];
        }
        K[0] = p[0];
        zerok = (fabs(K[NM1]) <= fabs(bb) * DBL_EPSILON * 10.0) ? 1 : 0;
      }
    }
    for (int i = 0; i < N; i++) temp[i] = K[i];
    for (jj = 1; jj <= 20; jj++) {
      xxx = -(sinr * yy) + cosr * xx;
      yy = sinr * xx + cosr * yy;
      xx = xxx;
      sr = bnd * xx;
      u = -(2.0 * sr);
      jt_fxshfr(20 * jj, &NZ, sr, bnd, K, N, p, NN, qp, u, &lzi, &lzr, &szi, &szr);
      if (NZ != 0) {
        int k = degree - N;
        zeror[k] = szr;
        zeroi[k] = szi;
        NN = NN - NZ;
        N = NN - 1;
        for (int i = 0; i < NN; i++) p[i] = qp[i];
        if (NZ != 1) {
          zeror[k + 1] = lzr;
          zeroi[k + 1] = lzi;
        }
        break;
      }
      for (int i = 0; i < N; i++) K[i] = temp[i];
    }
    if (jj > 20) {
      degree -= N;
      break;
    }
  }
  return degree;
}

// ---------------------------------------------------------------- JacobiSVD
// One-sided Jacobi as OpenCV's JacobiSVDImpl_ (what cv::SVD computes for
// these shapes). Compile-time sizes throughout so every matrix stays in VGPRs
// (no scratch): At is N rows of length M (A^T), W the N singular values, Vt
// N x N.

// One rotation of rows (i, j) with its skip test; returns whether it rotated.
// The reference's control flow is: skip if |p| <= eps sqrt(a b); else gamma =
// hypot(2p, a - b) and the sign of beta = a - b picks which of c, s comes from
// the square root. Here that is evaluated branch-free in one basic block --
// the skip test's square root beside the rotation's chain, the beta branch as
// selects of the operands -- so the in-order wave never stalls on the skip
// test (the long ObjPose chains rotate in ~all 9 pair visits of their 3
// sweeps; skips are < 0.1 %). Every value is computed by the reference's
// operations on the reference's operands, so the results are identical. When
// |2p| <= 2^-60 |beta|, hypot(2p, beta) == |beta| exactly and both square
// roots are of 1, which the general formula reproduces.
template <int M, int N>
MK_HD bool jacobi_pair(double* At, double* W, double* Vt, int i, int j) {
  const double eps = DBL_EPSILON * 10;
  double a = W[i], p = 0, b = W[j];
#pragma unroll
  for (int k = 0; k < M; k++) p += At[i * M + k] * At[j * M + k];
#ifndef MK_JACOBI_KIND
#define MK_JACOBI_KIND(k)
#endif
  const bool skip = fabs(p) <= eps * sqrt(a * b);
  p *= 2;
  const double beta = a - b;
  const double gamma = hypot(p, beta);
  const bool neg = beta < 0;
  // beta < 0: s = sqrt(((gamma - beta) * 0.5) / gamma), c = p / (gamma * s * 2)
  // else:     c = sqrt((gamma + beta) / (gamma * 2)),   s = p / (gamma * c * 2)
  const double num = neg ? (gamma - beta) * 0.5 : gamma + beta;
  const double den = neg ? gamma : gamma * 2;
  const double r = sqrt(num / den);
  const double o = p / (gamma * r * 2);
  const double c = neg ? o : r, s = neg ? r : o;
  // commit by selects (a branch here would let the compiler sink the rotation
  // behind the skip test again)
  double na = 0, nb = 0;
#pragma unroll
  for (int k = 0; k < M; k++) {
    const double x = At[i * M + k], y = At[j * M + k];
    const double t0 = c * x + s * y;
    const double t1 = -s * x + c * y;
    At[i * M + k] = skip ? x : t0; At[j * M + k] = skip ? y : t1;
    na += t0 * t0; nb += t1 * t1;
  }
  W[i] = skip ? a : na; W[j] = skip ? b : nb;
  if (Vt) {
#pragma unroll
    for (int k = 0; k < N; k++) {
      const double x = Vt[i * N + k], y = Vt[j * N + k];
      const double t0 = c * x + s * y;
      const double t1 = -s * x + c * y;
      Vt[i * N + k] = skip ? x : t0; Vt[j * N + k] = skip ? y : t1;
    }
  }
  MK_JACOBI_KIND(skip ? 0 : 2);
  return !skip;
}

// Noise-phase fast-forward for a 3x3 At whose third components are exactly
// zero (a planar model makes M = sum p q^T have a zero row, so its three
// columns span a plane). Once rows 0 and 1 are converged and row 2 is a small
// residual, every later rotation is (0,2) or (1,2) in the c == 1 branch and
// only shrinks row 2, by ~1e-14 per sweep, until its squares underflow; the
// loop then ends (or hits max_iter) with W[2] == 0, and the regeneration after
// the loop overwrites row 2 from rows 0 and 1 alone. This test certifies, with
// a factor-2 margin on every bound, that none of those rotations can move a
// bit of rows 0/1, of W[0]/W[1] or of Vt, and that row 2 underflows before
// max_iter; then the remaining sweeps are skipped with row 2 set to zero.
// Bounds (n0 = max |row 2 component|, Bn <= |row b|, s = rotation sine):
//   |s| <= 3 n0 / Bn;  c == 1 branch needs n0 <= 2^-64 Bn;
//   row b unchanged:   |s row2[k]| <= 4.5 n0^2 / Bn < 2^-55 min|row b[k]|;
//   Vt unchanged:      |s Vt[k]|   <= 3 n0 / Bn    < 2^-55 min|Vt[k]|;
//   underflow:         n0 (1e-14)^(sweeps left - 1) < 1e-163.
// The only bits it does not reproduce are signs of the zero third
// components of rows 0/1 (+-0 + +-0), which no later result depends on.
// Evaluated without branches or square roots (all conditions are sufficient
// forms; a doubtful case only declines the fast-forward):
//   skip test of (0, 1): p^2 <= eps^2 W0 W1 (1 - 1e-10), W0 W1 in [1e-200, 1e200];
//   underflow: 1.5 n0 < 2^(ilogb(n0) + 2), so (ilogb(n0) + 2) log10(2) <
//   14 (sweeps left - 1) - 163 with log10(2) rounded toward the safe side.
MK_HD bool jacobi_noise_ff(const double* At, const double* W, const double* Vt, int sweeps_left) {
  const double eps = DBL_EPSILON * 10;
  double p = 0;
#pragma unroll
  for (int k = 0; k < 3; k++) p += At[k] * At[3 + k];  // jacobi_pair's skip test of (0, 1)
  const double x = W[0] * W[1];
  const bool skip01 = x >= 1e-200 && x <= 1e200 && p * p <= (eps * eps) * x * (1 - 1e-10);
  const double n0 = fmax(fabs(At[6]), fabs(At[7]));
  const double bmin = fmin(fmin(fabs(At[0]), fabs(At[1])), fmin(fabs(At[3]), fabs(At[4])));
  const double Bn = fmin(fmax(fabs(At[0]), fabs(At[1])), fmax(fabs(At[3]), fabs(At[4])));
  double vmin = fabs(Vt[0]);
#pragma unroll
  for (int k = 1; k < 9; k++) vmin = fmin(vmin, fabs(Vt[k]));
  const double e2 = n0 > 0 ? (double)(ilogb(n0) + 2) : -2000.0;
  const bool under = (e2 < 0 ? e2 * 0.30102 : e2 * 0.30104) < 14.0 * (sweeps_left - 1) - 163.01;
  return At[2] == 0 && At[5] == 0 && At[8] == 0 && skip01 && n0 <= 0x1p-64 * Bn &&
         4.5 * n0 * n0 < 0x1p-55 * bmin * Bn && 3.0 * n0 < 0x1p-55 * vmin * Bn && under;
}

#ifndef MK_JACOBI_FF
#define MK_JACOBI_FF 1
#endif

template <int M, int N>
MK_HD void jacobi_sweeps(double* At, double* W, double* Vt) {
  const int max_iter = M > 30 ? M : 30;
#pragma unroll 1
  for (int iter = 0; iter < max_iter; iter++) {
    if (MK_JACOBI_FF && M == 3 && N == 3 && Vt && iter > 0 && jacobi_noise_ff(At, W, Vt, max_iter - iter)) {
      At[6] = At[7] = At[8] = 0;
      break;
    }
    bool changed = false;
#pragma unroll
    for (int i = 0; i < N - 1; i++)
#pragma unroll
      for (int j = i + 1; j < N; j++) changed |= jacobi_pair<M, N>(At, W, Vt, i, j);
#ifdef MK_JACOBI_COUNT
    MK_JACOBI_COUNT(M, N, iter, changed);
#endif
    if (!changed) break;
  }
}

template <int M, int N>
MK_HD void jacobi_svd(double (&At)[N * M], double (&Wout)[N], double* Vt) {
#ifdef MK_SVD_TRACE
  MK_SVD_TRACE(M, N, At, Vt);
#endif
  const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
  double W[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    double sd = 0;
#pragma unroll
    for (int k = 0; k < M; k++) { double t = At[i * M + k]; sd += t * t; }
    W[i] = sd;
    if (Vt) {
#pragma unroll
      for (int k = 0; k < N; k++) Vt[i * N + k] = (k == i) ? 1.0 : 0.0;
    }
  }
  jacobi_sweeps<M, N>(At, W, Vt);
#pragma unroll
  for (int i = 0; i < N; i++) {
    double sd = 0;
#pragma unroll
    for (int k = 0; k < M; k++) { double t = At[i * M + k]; sd += t * t; }
    W[i] = sqrt(sd);
  }
  // selection sort by descending W; the swap partner is chosen with
  // predicates so every index stays a compile-time constant
#pragma unroll
  for (int i = 0; i < N - 1; i++) {
    int j = i;
    double wj = W[i];
#pragma unroll
    for (int k = i + 1; k < N; k++)
      if (wj < W[k]) { j = k; wj = W[k]; }
#pragma unroll
    for (int k = i + 1; k < N; k++) {
      if (j == k) {
        swp(W[i], W[k]);
        if (Vt) {
#pragma unroll
          for (int q = 0; q < M; q++) swp(At[i * M + q], At[k * M + q]);
#pragma unroll
          for (int q = 0; q < N; q++) swp(Vt[i * N + q], Vt[k * N + q]);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < N; i++) Wout[i] = W[i];
  if (!Vt) return;
  uint64_t rs = 0x12345678ULL;
#pragma unroll
  for (int i = 0; i < N; i++) {
    double sd = W[i];
#pragma unroll 1
    for (int ii = 0; ii < 100 && sd <= minval; ii++) {
      const double val0 = 1. / M;
#pragma unroll
      for (int k = 0; k < M; k++) {
        rs = (uint64_t)(uint32_t)rs * 4164903690ULL + (rs >> 32);
        At[i * M + k] = (((uint32_t)rs) & 256) != 0 ? val0 : -val0;
      }
#pragma unroll 1
      for (int it = 0; it < 2; it++) {
#pragma unroll
        for (int j = 0; j < i; j++) {
          sd = 0;
#pragma unroll
          for (int k = 0; k < M; k++) sd += At[i * M + k] * At[j * M + k];
          double asum = 0;
#pragma unroll
          for (int k = 0; k < M; k++) {
            double t = At[i * M + k] - sd * At[j * M + k];
            At[i * M + k] = t;
            asum += fabs(t);
          }
          asum = asum > eps * 100 ? 1 / asum : 0;
#pragma unroll
          for (int k = 0; k < M; k++) At[i * M + k] *= asum;
        }
      }
      sd = 0;
#pragma unroll
      for (int k = 0; k < M; k++) { double t = At[i * M + k]; sd += t * t; }
      sd = sqrt(sd);
    }
    double s = sd > minval ? 1 / sd : 0.;
#pragma unroll
    for (int k = 0; k < M; k++) At[i * M + k] *= s;
  }
}

// ------------------------------------------------------- fixed-size Mats
template <int R, int C>
struct Mt {
  double a[R * C];
  MK_HD double& operator()(int i, int j) { return a[i * C + j]; }
  MK_HD double operator()(int i, int j) const { return a[i * C + j]; }
};
template <int R, int C>
MK_HD Mt<R, C> zeros() {
  Mt<R, C> m;
#pragma unroll
  for (int i = 0; i < R * C; i++) m.a[i] = 0;
  return m;
}
MK_HD Mt<3, 3> eye3() {
  Mt<3, 3> m = zeros<3, 3>();
  m.a[0] = m.a[4] = m.a[8] = 1;
  return m;
}
// gemm: sum_k A(i,k) B(k,j) from 0, times alpha
template <int R, int K, int C>
MK_HD Mt<R, C> mm(const Mt<R, K>& A, const Mt<K, C>& B, double alpha = 1.0) {
  Mt<R, C> o;
#pragma unroll
  for (int i = 0; i < R; i++)
#pragma unroll
    for (int j = 0; j < C; j++) {
      double s = 0;
#pragma unroll
      for (int k = 0; k < K; k++) s += A(i, k) * B(k, j);
      o(i, j) = s * alpha;
    }
  return o;
}
template <int R, int K, int C>
MK_HD Mt<R, C> mmc(const Mt<R, K>& A, const Mt<K, C>& B, const Mt<R, C>& Cc) {
  Mt<R, C> o = mm(A, B);
#pragma unroll
  for (int i = 0; i < R * C; i++) o.a[i] = o.a[i] + Cc.a[i];
  return o;
}
template <int R, int C>
MK_HD Mt<C, R> tr(const Mt<R, C>& A) {
  Mt<C, R> o;
#pragma unroll
  for (int i = 0; i < R; i++)
#pragma unroll
    for (int j = 0; j < C; j++) o(j, i) = A(i, j);
  return o;
}
template <int R, int C>
MK_HD Mt<R, C> add(const Mt<R, C>& A, const Mt<R, C>& B) {
  Mt<R, C> o;
#pragma unroll
  for (int i = 0; i < R * C; i++) o.a[i] = A.a[i] + B.a[i];
  return o;
}
template <int R, int C>
MK_HD Mt<R, C> sub(const Mt<R, C>& A, const Mt<R, C>& B) {
  Mt<R, C> o;
#pragma unroll
  for (int i = 0; i < R * C; i++) o.a[i] = A.a[i] - B.a[i];
  return o;
}
template <int R, int C>
MK_HD Mt<R, C> scl(const Mt<R, C>& A, double s) {
  Mt<R, C> o;
#pragma unroll
  for (int i = 0; i < R * C; i++) o.a[i] = A.a[i] * s;
  return o;
}
template <int C>
MK_HD Mt<3, 1> col(const Mt<3, C>& A, int j) {
  Mt<3, 1> o;
#pragma unroll
  for (int i = 0; i < 3; i++) o.a[i] = A(i, j);
  return o;
}
MK_HD double det3(const Mt<3, 3>& m) {
  return m(0, 0) * (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) - m(0, 1) * (m(1, 0) * m(2, 2) - m(1, 2) * m(2, 0)) +
         m(0, 2) * (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0));
}
MK_HD Mt<3, 3> inv3(const Mt<3, 3>& M) {
  Mt<3, 3> D = zeros<3, 3>();
  double d = det3(M);
  if (d == 0.) return D;
  d = 1. / d;
  D(0, 0) = (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) * d;
  D(0, 1) = (M(0, 2) * M(2, 1) - M(0, 1) * M(2, 2)) * d;
  D(0, 2) = (M(0, 1) * M(1, 2) - M(0, 2) * M(1, 1)) * d;
  D(1, 0) = (M(1, 2) * M(2, 0) - M(1, 0) * M(2, 2)) * d;
  D(1, 1) = (M(0, 0) * M(2, 2) - M(0, 2) * M(2, 0)) * d;
  D(1, 2) = (M(0, 2) * M(1, 0) - M(0, 0) * M(1, 2)) * d;
  D(2, 0) = (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)) * d;
  D(2, 1) = (M(0, 1) * M(2, 0) - M(0, 0) * M(2, 1)) * d;
  D(2, 2) = (M(0, 0) * M(1, 1) - M(0, 1) * M(1, 0)) * d;
  return D;
}
template <int C>
MK_HD Mt<3, 1> rowsum(const Mt<3, C>& P) {
  Mt<3, 1> o;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    double s = 0;
#pragma unroll
    for (int j = 0; j < C; j++) s += P(i, j);
    o.a[i] = s;
  }
  return o;
}
MK_HD double sqnorm3(const Mt<3, 1>& v) { double x = v.a[0], y = v.a[1], z = v.a[2]; return x * x + y * y + z * z; }
MK_HD int sgn(double x) { return x < 0 ? -1 : (x > 0 ? 1 : 0); }
// RPP Norm(): largest singular value (cv::SVD of the matrix, flags 0)
MK_HD double norm_svd(const Mt<3, 3>& A) {
  double At[9], w[3], vt[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int k = 0; k < 3; k++) At[i * 3 + k] = A(k, i);
  jacobi_svd<3, 3>(At, w, vt);
  return w[0];
}
MK_HD double norm_svd(const Mt<3, 1>& A) {
  double At[3] = {A.a[0], A.a[1], A.a[2]}, w[1];
  jacobi_svd<3, 1>(At, w, (double*)nullptr);
  return w[0];
}
// SVD of a 3x3: u (3x3) and V (3x3 = vt^T)
MK_HD void svd3(const Mt<3, 3>& A, Mt<3, 3>& U, Mt<3, 3>& V) {
  double At[9], w[3], vt[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int k = 0; k < 3; k++) At[i * 3 + k] = A(k, i);
  jacobi_svd<3, 3>(At, w, vt);
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) { U(r, c) = At[c * 3 + r]; V(r, c) = vt[c * 3 + r]; }
}
// SVD API kept for the host checks: m x n with (m,n) in {(3,3),(3,1)}
MK_HD void cv_svd(const double* A, int m, int n, double* w, double* u, double* vt) {
  if (n == 1) {
    double At[3] = {A[0], A[1], A[2]}, ww[1], V1[1];
    jacobi_svd<3, 1>(At, ww, V1);
    w[0] = ww[0];
    if (u) for (int r = 0; r < 3; r++) u[r] = At[r];
    if (vt) vt[0] = V1[0];
    return;
  }
  double At[9], ww[3], V[9];
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) At[i * 3 + k] = A[k * 3 + i];
  jacobi_svd<3, 3>(At, ww, V);
  for (int i = 0; i < 3; i++) w[i] = ww[i];
  if (u)
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) u[r * 3 + c] = At[c * 3 + r];
  if (vt)
    for (int k = 0; k < 9; k++) vt[k] = V[k];
}
MK_HD Mt<3, 3> rpy_mat(double a0, double a1, double a2) {
  double cosA = cos(a2), sinA = sin(a2), cosB = cos(a1), sinB = sin(a1), cosC = cos(a0), sinC = sin(a0);
  double cosAsinB = cosA * sinB, sinAsinB = sinA * sinB;
  Mt<3, 3> R;
  R(0, 0) = cosA * cosB;
  R(0, 1) = cosAsinB * sinC - sinA * cosC;
  R(0, 2) = cosAsinB * cosC + sinA * sinC;
  R(1, 0) = sinA * cosB;
  R(1, 1) = sinAsinB * sinC + cosA * cosC;
  R(1, 2) = sinAsinB * cosC - cosA * sinC;
  R(2, 0) = -sinB;
  R(2, 1) = cosB * sinC;
  R(2, 2) = cosB * cosC;
  return R;
}
MK_HD bool rpy_ang(const Mt<3, 3>& R, double* ang) {
  double R11 = R(0, 0), R12 = R(0, 1), R13 = R(0, 2), R21 = R(1, 0), R22 = R(1, 1), R23 = R(1, 2), R31 = R(2, 0),
         R32 = R(2, 1), R33 = R(2, 2);
  double sinB = -R31, cosB = sqrt(R11 * R11 + R21 * R21), a0, a1, a2;
  if (fabs(cosB) > 1e-15) {
    double sinA = R21 / cosB, cosA = R11 / cosB, sinC = R32 / cosB, cosC = R33 / cosB;
    a0 = atan2(sinC, cosC);
    a1 = atan2(sinB, cosB);
    a2 = atan2(sinA, cosA);
  } else {
    double sinC = (R12 - R23) / 2, cosC = (R22 + R13) / 2;
    a0 = atan2(sinC, cosC);
    a1 = M_PI_2;
    a2 = 0;
    if (sinB < 0) { a0 = -a0; a1 = -a1; a2 = -a2; }
  }
  if (norm_svd(sub(R, rpy_mat(a0, a1, a2))) > 1e-6) return false;
  ang[0] = a0; ang[1] = a1; ang[2] = a2;
  return true;
}
MK_HD bool rpy_ang_x(const Mt<3, 3>& R, double* a) {
  if (!rpy_ang(R, a)) return false;
  if (fabs(a[0]) > M_PI_2) {
    int guard = 0;
    while (fabs(a[0]) > M_PI_2 && guard++ < 64) {
      if (a[0] > 0) {
        a[0] = a[0] + M_PI; a[1] = 3 * M_PI - a[1]; a[2] = a[2] + M_PI;
        a[0] -= 2 * M_PI; a[1] -= 2 * M_PI; a[2] -= 2 * M_PI;
      } else {
        a[0] = a[0] + M_PI; a[1] = 3 * M_PI - a[1]; a[2] = a[2] + M_PI;
      }
    }
  }
  return true;
}
template <int C>
MK_HD Mt<3, C> norm_rv(const Mt<3, C>& R) {
  Mt<3, C> o;
#pragma unroll
  for (int i = 0; i < C; i++) {
    double mag = R(0, i) * R(0, i) + R(1, i) * R(1, i) + R(2, i) * R(2, i);
    double m = 1.0 / sqrt(mag);
#pragma unroll
    for (int r = 0; r < 3; r++) o(r, i) = R(r, i) * m;
  }
  return o;
}

typedef Mt<3, 3> M33;
typedef Mt<3, 1> M31;

__attribute__((always_inline)) MK_HD bool rot_by_vector(const double* v1, const double* v2, M33& R) {
  double d = v2[0] * v1[0] + v2[1] * v1[1] + v2[2] * v1[2];
  double winkel = acos(d);
  M31 axm;
  axm.a[0] = v2[1] * v1[2] - v2[2] * v1[1];
  axm.a[1] = v2[2] * v1[0] - v2[0] * v1[2];
  axm.a[2] = v2[0] * v1[1] - v2[1] * v1[0];
  double nn = norm_svd(axm);
  double ra[3] = {axm.a[0], axm.a[1], axm.a[2]};
#pragma unroll
  for (int i = 0; i < 3; i++) ra[i] /= nn;
#pragma unroll
  for (int i = 0; i < 3; i++) ra[i] *= sin(winkel * 0.5);
  double qs = cos(winkel * 0.5);
  double qn = sqrt(ra[0] * ra[0] + ra[1] * ra[1] + ra[2] * ra[2] + qs * qs);
  double inv = 1 / qn;
  double a = qs * inv, b = ra[0] * inv, c = ra[1] * inv, dd = ra[2] * inv;
  R(0, 0) = a * a + b * b - c * c - dd * dd;
  R(0, 1) = 2 * (b * c - a * dd);
  R(0, 2) = 2 * (b * dd + a * c);
  R(1, 0) = 2 * (b * c + a * dd);
  R(1, 1) = a * a + c * c - b * b - dd * dd;
  R(1, 2) = 2 * (c * dd - a * b);
  R(2, 0) = 2 * (b * dd - a * c);
  R(2, 1) = 2 * (c * dd + a * b);
  R(2, 2) = a * a + dd * dd - b * b - c * c;
  M31 n1, n2;
  double m1 = sqrt(v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2]);
  double m2 = sqrt(v2[0] * v2[0] + v2[1] * v2[1] + v2[2] * v2[2]);
#pragma unroll
  for (int i = 0; i < 3; i++) { n1.a[i] = v1[i] / m1; n2.a[i] = v2[i] / m2; }
  M31 diff = sub(n1, mm(R, n2));
  double s = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) s += diff.a[i] * diff.a[i];
  return !(s * s > 1e-3);
}

__attribute__((always_inline)) MK_HD bool decompose_r(const M33& R, M33& RzN) {
  double cl = atan2(R(2, 1), R(2, 0));
  M33 Rz = rpy_mat(0, 0, cl);
  M33 R_ = mm(R, Rz);
  if (R_(2, 1) > 1e-3) return false;
  double ang[3];
  if (!rpy_ang_x(R_, ang)) return false;
  if (fabs(ang[0]) > 1e-3) return false;
  M33 Rz2 = mm(Rz, rpy_mat(0, 0, M_PI));
  R_ = mm(R, Rz2);
  if (R_(2, 1) > 1e-3) return false;
  if (!rpy_ang_x(R_, ang)) return false;
  RzN = Rz;
  return true;
}

struct Result {
  double R[9], t[3];
  double obj_err, img_err;
  int iterations;
  int status;  // 1 ok; 0 2nd-pose search failed (first ObjPose kept)
  int error;   // 0; 1 GetRotationbyVector failed (reference exit(1)); 2 iteration cap; 3 no best
};

constexpr int NP = 4;  // points per problem (a square's 4 corners)
#include "mk_rpp_np.inc"

// n-point instances (mantis_rpp_solve: RPP::Rpp on any point count the
// reference accepts, e.g. demo.cpp:17-38's 10-point known answer)
#define MK_RPP_INSTANCES(X) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12)
namespace n5 {
constexpr int NP = 5;
#include "mk_rpp_np.inc"
}  // namespace n5
namespace n6 {
constexpr int NP = 6;
#include "mk_rpp_np.inc"
}  // namespace n6
namespace n7 {
constexpr int NP = 7;
#include "mk_rpp_np.inc"
}  // namespace n7
namespace n8 {
constexpr int NP = 8;
#include "mk_rpp_np.inc"
}  // namespace n8
namespace n9 {
constexpr int NP = 9;
#include "mk_rpp_np.inc"
}  // namespace n9
namespace n10 {
constexpr int NP = 10;
#include "mk_rpp_np.inc"
}  // namespace n10
namespace n11 {
constexpr int NP = 11;
#include "mk_rpp_np.inc"
}  // namespace n11
namespace n12 {
constexpr int NP = 12;
#include "mk_rpp_np.inc"
}  // namespace n12

}  // namespace rpp
}  // namespace mk
