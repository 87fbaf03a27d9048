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

constexpr int NP = 4;  // points per problem (a square's 4 corners)
typedef Mt<3, NP> M34;
typedef Mt<3, 3> M33;
typedef Mt<3, 1> M31;

// AbsKernel (RPP.cpp:229-332): overwrites P (re-centred) and Q (F_i q_i) in place
#ifndef MK_OP_STAMP
#define MK_OP_STAMP(k)
#endif
MK_HD void abs_kernel(M34& P, M34& Q, const M33* F, const M33& G, M33& R, M31& t, M34& Qout, double& err2) {
  MK_OP_STAMP(0);
#pragma unroll
  for (int i = 0; i < NP; i++) {
    M31 q = mm(F[i], col(Q, i));
#pragma unroll
    for (int r = 0; r < 3; r++) Q(r, i) = q.a[r];
  }
  M31 pbar = scl(rowsum(P), 1.0 / NP);
#pragma unroll
  for (int i = 0; i < NP; i++)
#pragma unroll
    for (int r = 0; r < 3; r++) P(r, i) -= pbar.a[r];
  M33 M = zeros<3, 3>();
#pragma unroll
  for (int i = 0; i < NP; i++)
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
      for (int b = 0; b < 3; b++) M(a, b) += P(a, i) * Q(b, i);
  M33 U, V;
  MK_OP_STAMP(1);
  svd3(M, U, V);
  MK_OP_STAMP(2);
  M33 Ut = tr(U);
  // ref: RPP.cpp:296-318. det(V U^T) > 0: try R = V U^T, and if t_z < 0
  // flip V's 3rd column and take R = -(V U^T). Otherwise flip first, take
  // R = V U^T and, if t_z < 0, R = -(V U^T). One EstimateT call site.
  const bool pos = sgn(det3(mm(V, Ut))) == 1;
  if (!pos) {
#pragma unroll
    for (int r = 0; r < 3; r++) V(r, 2) = -V(r, 2);
  }
  R = mm(V, Ut);
#pragma unroll 1
  for (int pass = 0; pass < 2; pass++) {
    M31 sum = zeros<3, 1>();
#pragma unroll
    for (int i = 0; i < NP; i++) sum = add(sum, mm(mm(F[i], R), col(P, i)));
    t = mm(G, sum);
    if (pass == 1 || !(t.a[2] < 0)) break;
    if (pos) {
#pragma unroll
      for (int r = 0; r < 3; r++) V(r, 2) = -V(r, 2);
    }
    R = mm(V, Ut, -1.0);
  }
  M33 I = eye3();
  err2 = 0;
#pragma unroll
  for (int i = 0; i < NP; i++) {
    double x = P(0, i), y = P(1, i), z = P(2, i);
    M31 qo;
#pragma unroll
    for (int r = 0; r < 3; r++) {
      qo.a[r] = R(r, 0) * x + R(r, 1) * y + R(r, 2) * z + t.a[r];
      Qout(r, i) = qo.a[r];
    }
    err2 += sqnorm3(mm(sub(I, F[i]), qo));
  }
  MK_OP_STAMP(3);
}

// ObjPose (RPP.cpp:66-208) as a resumable state machine: op_setup (everything
// before the loop), op_step (one trip of the reference's do-while: the stop
// test, then one AbsKernel), op_finish (obj_err, img_err, t re-centring). A GPU
// lane can then hold one job, retire it when op_step reports done and pick up
// the next (k_objpose_q); obj_pose below runs the same three functions in a
// plain loop, so host checks and device kernels share every operation.
constexpr double kObjTol = 1E-5, kObjEps = 1E-8;  // RPP.cpp:7-8
constexpr int kObjCap = 100000;                    // the reference loop is unbounded
struct OpState {
  M34 P;          // model points, re-centred (AbsKernel re-centres them again every call)
  M34 Qi;         // current projections (AbsKernel input and output)
  double F6[NP][6];  // F_i = v v^T / (v^T v), symmetric: xx xy xz yy yz zz
  M33 G;          // tFactor
  M33 R;
  M31 t, pbar;
  double old_err, new_err;
  double qx0, qy0;  // Qp(0,0), Qp(1,0) for img_err (Q2: column 0 only)
  int it;
  int init_pass, first;
};
MK_HD M33 f_full(const double* f) {
  M33 F;
  F.a[0] = f[0]; F.a[1] = f[1]; F.a[2] = f[2];
  F.a[3] = f[1]; F.a[4] = f[3]; F.a[5] = f[4];
  F.a[6] = f[2]; F.a[7] = f[4]; F.a[8] = f[5];
  return F;
}
// Qp is rewritten to F_i q_i when there is no initial rotation (the first
// AbsKernel runs on Qp itself, RPP.cpp:105-110); the caller keeps that copy.
MK_HD void op_setup(const M34& P0, M34& Qp, const M33* initR, OpState& s) {
  s.P = P0;
  s.it = 0;
  s.pbar = scl(rowsum(s.P), 1.0 / NP);
#pragma unroll
  for (int i = 0; i < NP; i++)
#pragma unroll
    for (int r = 0; r < 3; r++) s.P(r, i) -= s.pbar.a[r];
  M33 F[NP];
#pragma unroll
  for (int i = 0; i < NP; i++) {
    M31 V = col(Qp, i);
    double ret = mm(tr(V), V).a[0];
    F[i] = mm(V, tr(V), 1.0 / ret);  // symmetric bit for bit (v_a v_b == v_b v_a)
    s.F6[i][0] = F[i].a[0]; s.F6[i][1] = F[i].a[1]; s.F6[i][2] = F[i].a[2];
    s.F6[i][3] = F[i].a[4]; s.F6[i][4] = F[i].a[5]; s.F6[i][5] = F[i].a[8];
  }
  M33 sumF = zeros<3, 3>();
#pragma unroll
  for (int i = 0; i < NP; i++) sumF = add(sumF, F[i]);
  M33 I = eye3();
  s.G = scl(inv3(sub(I, scl(sumF, 1.0 / NP))), 1.0 / NP);
  s.old_err = 0;
  s.init_pass = initR == nullptr;
  if (initR) {
    s.R = *initR;
    M31 sm = zeros<3, 1>();
#pragma unroll
    for (int i = 0; i < NP; i++) sm = mmc(mm(sub(F[i], I), s.R), col(s.P, i), sm);
    s.t = mm(s.G, sm);
#pragma unroll
    for (int i = 0; i < NP; i++) {
      double x = s.P(0, i), y = s.P(1, i), z = s.P(2, i);
      M31 qo;
#pragma unroll
      for (int r = 0; r < 3; r++) {
        qo.a[r] = s.R(r, 0) * x + s.R(r, 1) * y + s.R(r, 2) * z + s.t.a[r];
        s.Qi(r, i) = qo.a[r];
      }
      s.old_err += sqnorm3(mm(sub(I, F[i]), qo));
    }
  } else {
    s.Qi = Qp;
    // what the first AbsKernel leaves in Qp: F_i q_i, computed as it does
#pragma unroll
    for (int i = 0; i < NP; i++) {
      M31 q = mm(F[i], col(Qp, i));
#pragma unroll
      for (int r = 0; r < 3; r++) Qp(r, i) = q.a[r];
    }
  }
  s.qx0 = Qp(0, 0);
  s.qy0 = Qp(1, 0);
  // the reference computes one AbsKernel before testing the stop rule
  s.new_err = s.old_err;
  s.first = 1;
}
// one loop trip; returns 0 while running, 1 converged, 2 iteration cap
MK_HD int op_step(OpState& s) {
  if (!s.first) {
    if (!(fabs((s.old_err - s.new_err) / s.old_err) > kObjTol && (s.new_err > kObjEps))) return 1;
    if (s.it >= kObjCap) return 2;
    s.old_err = s.new_err;
  }
  M33 F[NP];
#pragma unroll
  for (int i = 0; i < NP; i++) F[i] = f_full(s.F6[i]);
  abs_kernel(s.P, s.Qi, F, s.G, s.R, s.t, s.Qi, s.new_err);
  s.it = s.it + 1;
  if (s.init_pass) {
    s.init_pass = 0;
    s.old_err = s.new_err;
  } else {
    s.first = 0;
  }
  return 0;
}
MK_HD void op_finish(const OpState& s, M33& R, M31& t, double& obj_err, double& img_err) {
  R = s.R;
  obj_err = sqrt(s.new_err / NP);
  img_err = 0;
#pragma unroll
  for (int i = 0; i < NP; i++) {
    M31 Qproj = mmc(s.R, col(s.P, i), s.t);
    double xx = (Qproj.a[0] / Qproj.a[2]) - s.qx0;
    double yy = (Qproj.a[1] / Qproj.a[2]) - s.qy0;
    img_err += (xx * xx + yy * yy);
  }
  img_err = sqrt(img_err / NP);
  t = sub(s.t, mm(s.R, s.pbar));
}

// ObjPose (RPP.cpp:66-208); returns 1 when the (reference-unbounded) loop hit the cap
MK_HD int obj_pose(const M34& P0, M34& Qp, const M33* initR, M33& R, M31& t, int& it, double& obj_err,
                   double& img_err) {
  OpState s;
  op_setup(P0, Qp, initR, s);
  int r;
#pragma unroll 1
  while ((r = op_step(s)) == 0) {
  }
  op_finish(s, R, t, obj_err, img_err);
  it = s.it;
  return r == 2 ? 1 : 0;
}

// Predicted AbsKernel count of an ObjPose from its state (longest-first
// scheduling of the persistent job queues, kernels.hip k_objpose_probe):
// kprobe more steps on a copy, then the stop test |de/e| <= kObjTol
// (RPP.cpp:171) extrapolated with the observed linear convergence rate of
// |de/e| over the last kPredSpan steps. Scheduling only: the results always
// come from the unchanged iteration.
constexpr int kPredSpan = 4;
MK_HD float op_predict(OpState s, int kprobe) {
  double e[2 + kPredSpan];  // the last errors (ring)
  int n = 0;
#pragma unroll 1
  for (int i = 0; i < kprobe; i++) {
    if (op_step(s)) return (float)s.it;  // converged (or capped) inside the probe
#pragma unroll
    for (int j = 0; j < 1 + kPredSpan; j++) e[j] = e[j + 1];
    e[1 + kPredSpan] = s.new_err;
    n++;
  }
  if (n < 2 + kPredSpan) return 1e6f;
  const double r1 = fabs((e[kPredSpan] - e[1 + kPredSpan]) / e[kPredSpan]);
  const double r0 = fabs((e[0] - e[1]) / e[0]);
  if (!(r1 > kObjTol)) return (float)(s.it + 1);
  const double rho = (r0 > 0 && r1 < r0) ? pow(r1 / r0, 1.0 / kPredSpan) : 1.0;
  if (!(rho < 0.99999)) return 1e6f;
  const double rem = log(kObjTol / r1) / log(rho);
  return (float)(s.it + (rem > 0 ? rem : 0) + 1);
}

MK_HD bool rot_by_vector(const double* v1, const double* v2, M33& R) {
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

MK_HD bool decompose_r(const M33& R, M33& RzN) {
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

// GetRotationY_wrtT (RPP.cpp:947-1222): the 5 root slots of the quartic in
// order with a keep flag (the reference's translation candidates are
// overwritten by the following ObjPose and are not formed here).
MK_HD void rot_y_wrt_t(const M34& v, const M34& p, const M33& Rz, double* al, bool* keep) {
  M33 V[NP];
#pragma unroll
  for (int i = 0; i < NP; i++) {
    M31 vv = col(v, i);
    double a = mm(tr(vv), vv).a[0];
    V[i] = mm(vv, tr(vv), 1.0 / a);
  }
  M33 G = zeros<3, 3>();
#pragma unroll
  for (int i = 0; i < NP; i++) G = add(G, V[i]);
  M33 I = eye3();
  G = scl(inv3(sub(I, scl(G, 1.0 / NP))), 1.0 / NP);
  M33 opt = zeros<3, 3>();
  const double r1 = Rz(0, 0), r2 = Rz(0, 1), r3 = Rz(0, 2), r4 = Rz(1, 0), r5 = Rz(1, 1), r6 = Rz(1, 2),
               r7 = Rz(2, 0), r8 = Rz(2, 1), r9 = Rz(2, 2);
#pragma unroll
  for (int i = 0; i < NP; i++) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      double w1 = V[i](k, 0), w2 = V[i](k, 1), w3 = V[i](k, 2);
      if (k == 0) w1 = w1 - 1; else if (k == 1) w2 = w2 - 1; else w3 = w3 - 1;
      double px = p(0, i), py = p(1, i), pz = p(2, i);
      opt(k, 0) += ((w1 * r2 + w2 * r5 + w3 * r8) * py + (-w1 * r1 - w2 * r4 - w3 * r7) * px +
                    (-w1 * r3 - w2 * r6 - w3 * r9) * pz);
      opt(k, 1) += ((2 * w1 * r1 + 2 * w2 * r4 + 2 * w3 * r7) * pz + (-2 * w1 * r3 - 2 * w2 * r6 - 2 * w3 * r9) * px);
      opt(k, 2) += (w1 * r1 + w2 * r4 + w3 * r7) * px + (w1 * r3 + w2 * r6 + w3 * r9) * pz +
                   (w1 * r2 + w2 * r5 + w3 * r8) * py;
    }
  }
  opt = mm(G, opt);
  double E2[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < NP; i++) {
    double px = p(0, i), py = p(1, i), pz = p(2, i);
    M33 Rpi;
    Rpi(0, 0) = -px; Rpi(0, 1) = 2 * pz; Rpi(0, 2) = px;
    Rpi(1, 0) = py;  Rpi(1, 1) = 0;      Rpi(1, 2) = py;
    Rpi(2, 0) = -pz; Rpi(2, 1) = -2 * px; Rpi(2, 2) = pz;
    M33 E = mm(sub(I, V[i]), mmc(Rz, Rpi, opt));
    double s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0;
#pragma unroll
    for (int r = 0; r < 3; r++) s1 += E(r, 0) * E(r, 0);
#pragma unroll
    for (int r = 0; r < 3; r++) s2 += 2 * (E(r, 1) * E(r, 0));
#pragma unroll
    for (int r = 0; r < 3; r++) s3 += (E(r, 2) * E(r, 0)) * 2 + E(r, 1) * E(r, 1) + 0.0;
#pragma unroll
    for (int r = 0; r < 3; r++) s4 += 2 * (E(r, 2) * E(r, 1));
#pragma unroll
    for (int r = 0; r < 3; r++) s5 += E(r, 2) * E(r, 2);
    E2[0] += s1; E2[1] += s2; E2[2] += s3; E2[3] += s4; E2[4] += s5;
  }
  double e4 = E2[0], e3 = E2[1], e2 = E2[2], e1 = E2[3], e0 = E2[4];
  double a4 = -e3, a3 = (4 * e4 - 2 * e2), a2 = (-3 * e1 + 3 * e3), a1 = (-4 * e0 + 2 * e2), a0 = e1;
  double coeffs[5] = {a4, a3, a2, a1, a0};
  double zr[5] = {0, 0, 0, 0, 0}, zi[5] = {0, 0, 0, 0, 0};
  rpoly(coeffs, 4, zr, zi);
#pragma unroll
  for (int i = 0; i < 5; i++) {
    double a = zr[i];
    double p1 = pow(1.0 + a * a, 3.0);
    bool k1 = fabs(p1) > 0.1 && zi[i] == 0;
    double sa = (2.0 * a) / (1.0 + a * a);
    double ca = (1.0 - a * a) / (1.0 + a * a);
    al[i] = atan2(sa, ca) * 180 / M_PI;
    double tMaxMin = (4 * a4 * a * a * a + 3 * a3 * a * a + 2 * a2 * a + a1);
    keep[i] = k1 && tMaxMin > 0;
  }
}

struct Result {
  double R[9], t[3];
  double obj_err, img_err;
  int iterations;
  int status;  // 1 ok; 0 2nd-pose search failed (first ObjPose kept)
  int error;   // 0; 1 GetRotationbyVector failed (reference exit(1)); 2 iteration cap; 3 no best
};

// RPP::Rpp (RPP.cpp:13-64) split in three phases so the GPU runs each with a
// small live state: stage1 = first ObjPose + Get2ndPose_Exact up to the
// candidate rotations; refine = one ObjPose per candidate (independent work
// items); merge = the reference's ordered lowest-obj_err selection.
constexpr int kCand = 5;
struct Stage1 {
  double Q[3 * NP];         // iprts after the first ObjPose (AbsKernel rewrote it)
  double R[9], t[3], obj_err, img_err;
  double sR[kCand][9];      // initial rotations of the 2nd-pose candidates
  int iterations, error;    // error: 0 / 1 (GetRotationbyVector) / 2 (cap)
  int keep_mask;            // bit j: candidate j enters the search
  int pad;
};
struct Refine {
  double R[9], t[3], obj_err, img_err;
  int iterations, capped;
};

// first ObjPose (no initial rotation)
MK_HD void stage1a(const double* model, const double* iprts, Stage1& s) {
  M34 P, Q;
#pragma unroll
  for (int i = 0; i < 3 * NP; i++) { P.a[i] = model[i]; Q.a[i] = iprts[i]; }
  M33 R;
  M31 t;
  int it = 0;
  double oe = 0, ie = 0;
  int capped = obj_pose(P, Q, nullptr, R, t, it, oe, ie);
#pragma unroll
  for (int k = 0; k < 3 * NP; k++) s.Q[k] = Q.a[k];
#pragma unroll
  for (int k = 0; k < 9; k++) s.R[k] = R.a[k];
#pragma unroll
  for (int k = 0; k < 3; k++) s.t[k] = t.a[k];
  s.obj_err = oe;
  s.img_err = ie;
  s.iterations = it;
  s.error = capped ? 2 : 0;
  s.keep_mask = 0;
}

// Get2ndPose_Exact up to the candidate rotations (RPP.cpp:693-753)
MK_HD void stage1b(const double* model, Stage1& s) {
  M34 P, Q;
  M33 R;
#pragma unroll
  for (int i = 0; i < 3 * NP; i++) { P.a[i] = model[i]; Q.a[i] = s.Q[i]; }
#pragma unroll
  for (int k = 0; k < 9; k++) R.a[k] = s.R[k];
  Mt<NP, 3> nv = tr(norm_rv(Q));
  M31 mean;
#pragma unroll
  for (int j = 0; j < 3; j++) {
    double sm = 0;
#pragma unroll
    for (int i = 0; i < NP; i++) sm += nv(i, j);
    mean.a[j] = sm / 3;
  }
  M31 cent = norm_rv(mean);
  double c3[3] = {cent.a[0], cent.a[1], cent.a[2]}, z[3] = {0, 0, 1};
  M33 Rim;
  if (!rot_by_vector(z, c3, Rim)) { s.error = 1; return; }
  M34 v_ = mm(Rim, Q);
  M33 R_ = mm(Rim, R);
  M33 RzN;
  if (!decompose_r(R_, RzN)) return;
  M33 R2 = mm(R_, RzN);
  M34 P_ = mm(tr(RzN), P);
  double ang[3];
  if (!rpy_ang_x(R2, ang)) return;
  M33 Rz = rpy_mat(0, 0, ang[2]);
  double bl[kCand];
  bool keep[kCand];
  rot_y_wrt_t(v_, P_, Rz, bl, keep);
  M33 RimT = tr(Rim);
  M33 RzNt = tr(RzN);
  int mask = 0;
#pragma unroll 1
  for (int j = 0; j < kCand; j++) {
    if (!keep[j]) continue;
    double b = bl[j] / 180 * M_PI;
    M33 sR = mm(RimT, mm(mm(Rz, rpy_mat(0, b, 0)), RzNt));
#pragma unroll
    for (int k = 0; k < 9; k++) s.sR[j][k] = sR.a[k];
    mask |= 1 << j;
  }
  s.keep_mask = mask;
}

MK_HD void stage1(const double* model, const double* iprts, Stage1& s) {
  stage1a(model, iprts, s);
  stage1b(model, s);
}

MK_HD void refine(const double* model, const double* Q, const double* sR, Refine& r) {
  M34 P, Qp;
#pragma unroll
  for (int i = 0; i < 3 * NP; i++) { P.a[i] = model[i]; Qp.a[i] = Q[i]; }
  M33 R0;
#pragma unroll
  for (int k = 0; k < 9; k++) R0.a[k] = sR[k];
  M33 Rl;
  M31 tl;
  int it = 0;
  double oe = 0, ie = 0;
  r.capped = obj_pose(P, Qp, &R0, Rl, tl, it, oe, ie);
#pragma unroll
  for (int k = 0; k < 9; k++) r.R[k] = Rl.a[k];
#pragma unroll
  for (int k = 0; k < 3; k++) r.t[k] = tl.a[k];
  r.obj_err = oe;
  r.img_err = ie;
  r.iterations = it;
}

// ref: RPP.cpp:40-63 — candidates in order, strict "<" on obj_err from 1e6;
// the reported iteration count is the last ObjPose's (the variable is shared)
MK_HD Result merge(const Stage1& s, const Refine* rf) {
  Result res;
  for (int k = 0; k < 9; k++) res.R[k] = s.R[k];
  for (int k = 0; k < 3; k++) res.t[k] = s.t[k];
  res.obj_err = s.obj_err;
  res.img_err = s.img_err;
  res.iterations = s.iterations;
  res.status = 0;
  res.error = s.error;
  if (s.error == 1 || s.keep_mask == 0) return res;
  int best = -1;
  double lowest = 1e6;
  for (int j = 0; j < kCand; j++) {
    if (!(s.keep_mask >> j & 1)) continue;
    if (rf[j].capped) res.error = 2;
    if (rf[j].obj_err < lowest) { lowest = rf[j].obj_err; best = j; }
  }
  if (best < 0) { res.error = 3; return res; }
  const Refine& b = rf[best];
  for (int k = 0; k < 9; k++) res.R[k] = b.R[k];
  for (int k = 0; k < 3; k++) res.t[k] = b.t[k];
  res.obj_err = b.obj_err;
  res.img_err = b.img_err;
  int last = 0;
  for (int j = 0; j < kCand; j++)
    if (s.keep_mask >> j & 1) last = j;
  res.iterations = rf[last].iterations;
  res.status = 1;
  return res;
}

// RPP::Rpp (RPP.cpp:13-64) on model/iprts given as 3 x 4 row-major (host checks)
MK_HD Result solve(const double* model, const double* iprts) {
  Stage1 s;
  stage1(model, iprts, s);
  Refine rf[kCand];
  if (s.error != 1)
    for (int j = 0; j < kCand; j++)
      if (s.keep_mask >> j & 1) refine(model, s.Q, s.sR[j], rf[j]);
  return merge(s, rf);
}

}  // namespace rpp
}  // namespace mk
