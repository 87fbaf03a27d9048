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
// OpenCV JacobiSVDImpl_ on At (n rows of length m), eps = 10 DBL_EPSILON,
// minval = DBL_MIN, null singular vectors from cv::RNG(0x12345678).
MK_HD void jacobi_svd(double* At, int m, int n, double* Wout, double* Vt, int n1) {
  const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
  double W[3];
  int max_iter = m > 30 ? m : 30;
  for (int i = 0; i < n; i++) {
    double sd = 0;
    for (int k = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
    W[i] = sd;
    if (Vt) {
      for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
      Vt[i * n + i] = 1;
    }
  }
  for (int iter = 0; iter < max_iter; iter++) {
    bool changed = false;
    for (int i = 0; i < n - 1; i++)
      for (int j = i + 1; j < n; j++) {
        double *Ai = At + i * m, *Aj = At + j * m;
        double a = W[i], p = 0, b = W[j];
        for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
        if (fabs(p) <= eps * sqrt(a * b)) continue;
        p *= 2;
        double beta = a - b, gamma = hypot(p, beta), c, s;
        if (beta < 0) {
          double delta = (gamma - beta) * 0.5;
          s = sqrt(delta / gamma);
          c = p / (gamma * s * 2);
        } else {
          c = sqrt((gamma + beta) / (gamma * 2));
          s = p / (gamma * c * 2);
        }
        a = b = 0;
        for (int k = 0; k < m; k++) {
          double t0 = c * Ai[k] + s * Aj[k];
          double t1 = -s * Ai[k] + c * Aj[k];
          Ai[k] = t0; Aj[k] = t1;
          a += t0 * t0; b += t1 * t1;
        }
        W[i] = a; W[j] = b;
        changed = true;
        if (Vt) {
          double *Vi = Vt + i * n, *Vj = Vt + j * n;
          for (int k = 0; k < n; k++) {
            double t0 = c * Vi[k] + s * Vj[k];
            double t1 = -s * Vi[k] + c * Vj[k];
            Vi[k] = t0; Vj[k] = t1;
          }
        }
      }
    if (!changed) break;
  }
  for (int i = 0; i < n; i++) {
    double sd = 0;
    for (int k = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
    W[i] = sqrt(sd);
  }
  for (int i = 0; i < n - 1; i++) {
    int j = i;
    for (int k = i + 1; k < n; k++) if (W[j] < W[k]) j = k;
    if (i != j) {
      swp(W[i], W[j]);
      if (Vt) {
        for (int k = 0; k < m; k++) swp(At[i * m + k], At[j * m + k]);
        for (int k = 0; k < n; k++) swp(Vt[i * n + k], Vt[j * n + k]);
      }
    }
  }
  for (int i = 0; i < n; i++) Wout[i] = W[i];
  if (!Vt) return;
  uint64_t rs = 0x12345678ULL;
  for (int i = 0; i < n1; i++) {
    double sd = i < n ? W[i] : 0;
    for (int ii = 0; ii < 100 && sd <= minval; ii++) {
      const double val0 = 1. / m;
      for (int k = 0; k < m; k++) {
        rs = (uint64_t)(uint32_t)rs * 4164903690ULL + (rs >> 32);
        At[i * m + k] = (((uint32_t)rs) & 256) != 0 ? val0 : -val0;
      }
      for (int it = 0; it < 2; it++)
        for (int j = 0; j < i; j++) {
          sd = 0;
          for (int k = 0; k < m; k++) sd += At[i * m + k] * At[j * m + k];
          double asum = 0;
          for (int k = 0; k < m; k++) {
            double t = At[i * m + k] - sd * At[j * m + k];
            At[i * m + k] = t;
            asum += fabs(t);
          }
          asum = asum > eps * 100 ? 1 / asum : 0;
          for (int k = 0; k < m; k++) At[i * m + k] *= asum;
        }
      sd = 0;
      for (int k = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
      sd = sqrt(sd);
    }
    double s = sd > minval ? 1 / sd : 0.;
    for (int k = 0; k < m; k++) At[i * m + k] *= s;
  }
}
// SVD of an m x n (m >= n, m <= 3) row-major A: w, u (m x n), vt (n x n)
MK_HD void cv_svd(const double* A, int m, int n, double* w, double* u, double* vt) {
  double At[9], Vt[9];
  for (int i = 0; i < n; i++)
    for (int k = 0; k < m; k++) At[i * m + k] = A[k * n + i];
  jacobi_svd(At, m, n, w, Vt, n);
  if (u)
    for (int r = 0; r < m; r++)
      for (int c = 0; c < n; c++) u[r * n + c] = At[c * m + r];
  if (vt)
    for (int k = 0; k < n * n; k++) vt[k] = Vt[k];
}

// ------------------------------------------------------------- small Mats
struct Mx {
  int r, c;
  double a[12];
};
MK_HD Mx mx(int r, int c) {
  Mx m;
  m.r = r; m.c = c;
  for (int i = 0; i < 12; i++) m.a[i] = 0;
  return m;
}
MK_HD double& at(Mx& m, int i, int j) { return m.a[i * m.c + j]; }
MK_HD double at(const Mx& m, int i, int j) { return m.a[i * m.c + j]; }
MK_HD Mx eye3() { Mx m = mx(3, 3); m.a[0] = m.a[4] = m.a[8] = 1; return m; }
MK_HD Mx mm(const Mx& A, const Mx& B, double alpha = 1.0) {
  Mx o = mx(A.r, B.c);
  for (int i = 0; i < A.r; i++)
    for (int j = 0; j < B.c; j++) {
      double s = 0;
      for (int k = 0; k < A.c; k++) s += at(A, i, k) * at(B, k, j);
      at(o, i, j) = s * alpha;
    }
  return o;
}
MK_HD Mx mmc(const Mx& A, const Mx& B, const Mx& C) {
  Mx o = mm(A, B);
  for (int i = 0; i < o.r * o.c; i++) o.a[i] = o.a[i] + C.a[i];
  return o;
}
MK_HD Mx tr(const Mx& A) { Mx o = mx(A.c, A.r); for (int i = 0; i < A.r; i++) for (int j = 0; j < A.c; j++) at(o, j, i) = at(A, i, j); return o; }
MK_HD Mx add(const Mx& A, const Mx& B) { Mx o = mx(A.r, A.c); for (int i = 0; i < A.r * A.c; i++) o.a[i] = A.a[i] + B.a[i]; return o; }
MK_HD Mx sub(const Mx& A, const Mx& B) { Mx o = mx(A.r, A.c); for (int i = 0; i < A.r * A.c; i++) o.a[i] = A.a[i] - B.a[i]; return o; }
MK_HD Mx scl(const Mx& A, double s) { Mx o = mx(A.r, A.c); for (int i = 0; i < A.r * A.c; i++) o.a[i] = A.a[i] * s; return o; }
MK_HD Mx col(const Mx& A, int j) { Mx o = mx(3, 1); for (int i = 0; i < 3; i++) o.a[i] = at(A, i, j); return o; }
MK_HD double det3(const Mx& m) {
  return at(m, 0, 0) * (at(m, 1, 1) * at(m, 2, 2) - at(m, 1, 2) * at(m, 2, 1)) -
         at(m, 0, 1) * (at(m, 1, 0) * at(m, 2, 2) - at(m, 1, 2) * at(m, 2, 0)) +
         at(m, 0, 2) * (at(m, 1, 0) * at(m, 2, 1) - at(m, 1, 1) * at(m, 2, 0));
}
MK_HD Mx inv3(const Mx& M) {
  Mx D = mx(3, 3);
  double d = det3(M);
  if (d == 0.) return D;
  d = 1. / d;
  at(D, 0, 0) = (at(M, 1, 1) * at(M, 2, 2) - at(M, 1, 2) * at(M, 2, 1)) * d;
  at(D, 0, 1) = (at(M, 0, 2) * at(M, 2, 1) - at(M, 0, 1) * at(M, 2, 2)) * d;
  at(D, 0, 2) = (at(M, 0, 1) * at(M, 1, 2) - at(M, 0, 2) * at(M, 1, 1)) * d;
  at(D, 1, 0) = (at(M, 1, 2) * at(M, 2, 0) - at(M, 1, 0) * at(M, 2, 2)) * d;
  at(D, 1, 1) = (at(M, 0, 0) * at(M, 2, 2) - at(M, 0, 2) * at(M, 2, 0)) * d;
  at(D, 1, 2) = (at(M, 0, 2) * at(M, 1, 0) - at(M, 0, 0) * at(M, 1, 2)) * d;
  at(D, 2, 0) = (at(M, 1, 0) * at(M, 2, 1) - at(M, 1, 1) * at(M, 2, 0)) * d;
  at(D, 2, 1) = (at(M, 0, 1) * at(M, 2, 0) - at(M, 0, 0) * at(M, 2, 1)) * d;
  at(D, 2, 2) = (at(M, 0, 0) * at(M, 1, 1) - at(M, 0, 1) * at(M, 1, 0)) * d;
  return D;
}
MK_HD Mx rowsum(const Mx& P) {
  Mx o = mx(P.r, 1);
  for (int i = 0; i < P.r; i++) { double s = 0; for (int j = 0; j < P.c; j++) s += at(P, i, j); o.a[i] = s; }
  return o;
}
MK_HD double sqnorm3(const Mx& v) { double x = v.a[0], y = v.a[1], z = v.a[2]; return x * x + y * y + z * z; }
MK_HD int sgn(double x) { return x < 0 ? -1 : (x > 0 ? 1 : 0); }
MK_HD double norm_svd(const Mx& A) {
  double w[3];
  if (A.c == 1) { cv_svd(A.a, A.r, 1, w, nullptr, nullptr); return w[0]; }
  double u[9], vt[9];
  cv_svd(A.a, A.r, A.c, w, u, vt);
  return w[0];
}
MK_HD Mx xform(const Mx& P, const Mx& R, const Mx& t) {
  Mx o = mx(3, P.c);
  for (int i = 0; i < P.c; i++) {
    double x = at(P, 0, i), y = at(P, 1, i), z = at(P, 2, i);
    for (int r = 0; r < 3; r++) at(o, r, i) = at(R, r, 0) * x + at(R, r, 1) * y + at(R, r, 2) * z + t.a[r];
  }
  return o;
}
MK_HD Mx rpy_mat(double a0, double a1, double a2) {
  double cosA = cos(a2), sinA = sin(a2), cosB = cos(a1), sinB = sin(a1), cosC = cos(a0), sinC = sin(a0);
  double cosAsinB = cosA * sinB, sinAsinB = sinA * sinB;
  Mx R = mx(3, 3);
  at(R, 0, 0) = cosA * cosB;
  at(R, 0, 1) = cosAsinB * sinC - sinA * cosC;
  at(R, 0, 2) = cosAsinB * cosC + sinA * sinC;
  at(R, 1, 0) = sinA * cosB;
  at(R, 1, 1) = sinAsinB * sinC + cosA * cosC;
  at(R, 1, 2) = sinAsinB * cosC - cosA * sinC;
  at(R, 2, 0) = -sinB;
  at(R, 2, 1) = cosB * sinC;
  at(R, 2, 2) = cosB * cosC;
  return R;
}
MK_HD bool rpy_ang(const Mx& R, double* ang) {
  double R11 = at(R, 0, 0), R12 = at(R, 0, 1), R13 = at(R, 0, 2), R21 = at(R, 1, 0), R22 = at(R, 1, 1),
         R23 = at(R, 1, 2), R31 = at(R, 2, 0), R32 = at(R, 2, 1), R33 = at(R, 2, 2);
  double sinB = -R31, cosB = sqrt(R11 * R11 + R21 * R21), a[3];
  if (fabs(cosB) > 1e-15) {
    double sinA = R21 / cosB, cosA = R11 / cosB, sinC = R32 / cosB, cosC = R33 / cosB;
    a[0] = atan2(sinC, cosC);
    a[1] = atan2(sinB, cosB);
    a[2] = atan2(sinA, cosA);
  } else {
    double sinC = (R12 - R23) / 2, cosC = (R22 + R13) / 2;
    a[0] = atan2(sinC, cosC);
    a[1] = M_PI_2;
    a[2] = 0;
    if (sinB < 0) { a[0] = -a[0]; a[1] = -a[1]; a[2] = -a[2]; }
  }
  if (norm_svd(sub(R, rpy_mat(a[0], a[1], a[2]))) > 1e-6) return false;
  ang[0] = a[0]; ang[1] = a[1]; ang[2] = a[2];
  return true;
}
MK_HD bool rpy_ang_x(const Mx& R, double* a) {
  if (!rpy_ang(R, a)) return false;
  if (fabs(a[0]) > M_PI_2) {
    while (fabs(a[0]) > M_PI_2) {
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
MK_HD Mx norm_rv(const Mx& R) {
  Mx o = mx(R.r, R.c);
  for (int i = 0; i < R.c; i++) {
    double mag = at(R, 0, i) * at(R, 0, i) + at(R, 1, i) * at(R, 1, i) + at(R, 2, i) * at(R, 2, i);
    double m = 1.0 / sqrt(mag);
    for (int r = 0; r < 3; r++) at(o, r, i) = at(R, r, i) * m;
  }
  return o;
}

constexpr int NP = 4;  // points per problem (a square's 4 corners)

MK_HD void abs_kernel(Mx& P, Mx& Q, const Mx* F, const Mx& G, Mx& R, Mx& t, Mx& Qout, double& err2) {
  const int n = NP;
  for (int i = 0; i < n; i++) {
    Mx q = mm(F[i], col(Q, i));
    for (int r = 0; r < 3; r++) at(Q, r, i) = q.a[r];
  }
  Mx pbar = scl(rowsum(P), 1.0 / n);
  for (int i = 0; i < n; i++)
    for (int r = 0; r < 3; r++) at(P, r, i) -= pbar.a[r];
  Mx M = mx(3, 3);
  for (int i = 0; i < n; i++)
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) at(M, a, b) += at(P, a, i) * at(Q, b, i);
  double w[3], u[9], vt[9];
  cv_svd(M.a, 3, 3, w, u, vt);
  Mx U = mx(3, 3), V = mx(3, 3);
  for (int i = 0; i < 9; i++) U.a[i] = u[i];
  for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) at(V, i, j) = vt[j * 3 + i];
  Mx Ut = tr(U);
  auto estimate_t = [&](const Mx& Rr) {
    Mx sum = mx(3, 1);
    for (int i = 0; i < n; i++) sum = add(sum, mm(mm(F[i], Rr), col(P, i)));
    return mm(G, sum);
  };
  R = mm(V, Ut);
  if (sgn(det3(R)) == 1) {
    t = estimate_t(R);
    if (t.a[2] < 0) {
      for (int r = 0; r < 3; r++) at(V, r, 2) = -at(V, r, 2);
      R = mm(V, Ut, -1.0);
      t = estimate_t(R);
    }
  } else {
    for (int r = 0; r < 3; r++) at(V, r, 2) = -at(V, r, 2);
    R = mm(V, Ut);
    t = estimate_t(R);
    if (t.a[2] < 0) {
      R = mm(V, Ut, -1.0);
      t = estimate_t(R);
    }
  }
  Mx I = eye3();
  err2 = 0;
  Qout = xform(P, R, t);
  for (int i = 0; i < n; i++) err2 += sqnorm3(mm(sub(I, F[i]), col(Qout, i)));
}

// returns 1 when the (reference-unbounded) iteration hit the cap
MK_HD int obj_pose(const Mx& P0, Mx& Qp, const Mx* initR, Mx& R, Mx& t, int& it, double& obj_err, double& img_err) {
  const double TOL = 1E-5, EPS = 1E-8;
  const int n = NP;
  Mx P = P0;
  it = 0;
  Mx pbar = scl(rowsum(P), 1.0 / n);
  for (int i = 0; i < n; i++)
    for (int r = 0; r < 3; r++) at(P, r, i) -= pbar.a[r];
  Mx F[NP];
  for (int i = 0; i < n; i++) {
    Mx V = col(Qp, i);
    double ret = mm(tr(V), V).a[0];
    F[i] = mm(V, tr(V), 1.0 / ret);
  }
  Mx sumF = mx(3, 3);
  for (int i = 0; i < n; i++) sumF = add(sumF, F[i]);
  Mx I = eye3();
  Mx tFactor = scl(inv3(sub(I, scl(sumF, 1.0 / n))), 1.0 / n);
  double old_err, new_err;
  Mx Qi, Ri, ti;
  if (initR) {
    Ri = *initR;
    Mx s = mx(3, 1);
    for (int i = 0; i < n; i++) s = mmc(mm(sub(F[i], I), Ri), col(P, i), s);
    ti = mm(tFactor, s);
    Qi = xform(P, Ri, ti);
    old_err = 0;
    for (int i = 0; i < n; i++) old_err += sqnorm3(mm(sub(I, F[i]), col(Qi, i)));
  } else {
    abs_kernel(P, Qp, F, tFactor, Ri, ti, Qi, old_err);
    it = 1;
  }
  abs_kernel(P, Qi, F, tFactor, Ri, ti, Qi, new_err);
  it = it + 1;
  int capped = 0;
  while (fabs((old_err - new_err) / old_err) > TOL && (new_err > EPS)) {
    if (it >= 100000) { capped = 1; break; }
    old_err = new_err;
    abs_kernel(P, Qi, F, tFactor, Ri, ti, Qi, new_err);
    it = it + 1;
  }
  R = Ri;
  t = ti;
  obj_err = sqrt(new_err / n);
  img_err = 0;
  for (int i = 0; i < n; i++) {
    Mx Qproj = mmc(Ri, col(P, i), ti);
    double xx = (Qproj.a[0] / Qproj.a[2]) - at(Qp, 0, 0);
    double yy = (Qproj.a[1] / Qproj.a[2]) - at(Qp, 1, 0);
    img_err += (xx * xx + yy * yy);
  }
  img_err = sqrt(img_err / n);
  t = sub(t, mm(Ri, pbar));
  return capped;
}

MK_HD bool rot_by_vector(const double* v1, const double* v2, Mx& R) {
  double d = v2[0] * v1[0] + v2[1] * v1[1] + v2[2] * v1[2];
  double winkel = acos(d);
  Mx axm = mx(3, 1);
  axm.a[0] = v2[1] * v1[2] - v2[2] * v1[1];
  axm.a[1] = v2[2] * v1[0] - v2[0] * v1[2];
  axm.a[2] = v2[0] * v1[1] - v2[1] * v1[0];
  double nn = norm_svd(axm);
  double ra[3] = {axm.a[0], axm.a[1], axm.a[2]};
  for (int i = 0; i < 3; i++) ra[i] /= nn;
  for (int i = 0; i < 3; i++) ra[i] *= sin(winkel * 0.5);
  double qs = cos(winkel * 0.5);
  double qn = sqrt(ra[0] * ra[0] + ra[1] * ra[1] + ra[2] * ra[2] + qs * qs);
  double inv = 1 / qn;
  double a = qs * inv, b = ra[0] * inv, c = ra[1] * inv, dd = ra[2] * inv;
  R = mx(3, 3);
  at(R, 0, 0) = a * a + b * b - c * c - dd * dd;
  at(R, 0, 1) = 2 * (b * c - a * dd);
  at(R, 0, 2) = 2 * (b * dd + a * c);
  at(R, 1, 0) = 2 * (b * c + a * dd);
  at(R, 1, 1) = a * a + c * c - b * b - dd * dd;
  at(R, 1, 2) = 2 * (c * dd - a * b);
  at(R, 2, 0) = 2 * (b * dd - a * c);
  at(R, 2, 1) = 2 * (c * dd + a * b);
  at(R, 2, 2) = a * a + dd * dd - b * b - c * c;
  Mx n1 = mx(3, 1), n2 = mx(3, 1);
  double m1 = sqrt(v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2]);
  double m2 = sqrt(v2[0] * v2[0] + v2[1] * v2[1] + v2[2] * v2[2]);
  for (int i = 0; i < 3; i++) { n1.a[i] = v1[i] / m1; n2.a[i] = v2[i] / m2; }
  Mx diff = sub(n1, mm(R, n2));
  double s = 0;
  for (int i = 0; i < 3; i++) s += diff.a[i] * diff.a[i];
  return !(s * s > 1e-3);
}

MK_HD bool decompose_r(const Mx& R, Mx& RzN) {
  double cl = atan2(at(R, 2, 1), at(R, 2, 0));
  Mx Rz = rpy_mat(0, 0, cl);
  Mx R_ = mm(R, Rz);
  if (at(R_, 2, 1) > 1e-3) return false;
  double ang[3];
  if (!rpy_ang_x(R_, ang)) return false;
  if (fabs(ang[0]) > 1e-3) return false;
  Mx Rz2 = mm(Rz, rpy_mat(0, 0, M_PI));
  R_ = mm(R, Rz2);
  if (at(R_, 2, 1) > 1e-3) return false;
  if (!rpy_ang_x(R_, ang)) return false;
  RzN = Rz;
  return true;
}

// GetRotationY_wrtT: returns the number of kept solutions (<= 5)
MK_HD int rot_y_wrt_t(const Mx& v, const Mx& p, const Mx& Rz, double* al, Mx* tnew, double* at_out) {
  const int n = NP;
  Mx V[NP];
  for (int i = 0; i < n; i++) {
    Mx vv = col(v, i);
    double a = mm(tr(vv), vv).a[0];
    V[i] = mm(vv, tr(vv), 1.0 / a);
  }
  Mx G = mx(3, 3);
  for (int i = 0; i < n; i++) G = add(G, V[i]);
  Mx I = eye3();
  G = scl(inv3(sub(I, scl(G, 1.0 / n))), 1.0 / n);
  Mx opt = mx(3, 3);
  const double r1 = at(Rz, 0, 0), r2 = at(Rz, 0, 1), r3 = at(Rz, 0, 2), r4 = at(Rz, 1, 0), r5 = at(Rz, 1, 1),
               r6 = at(Rz, 1, 2), r7 = at(Rz, 2, 0), r8 = at(Rz, 2, 1), r9 = at(Rz, 2, 2);
  for (int i = 0; i < n; i++) {
    for (int k = 0; k < 3; k++) {
      double w1 = at(V[i], k, 0), w2 = at(V[i], k, 1), w3 = at(V[i], k, 2);
      if (k == 0) w1 = w1 - 1; else if (k == 1) w2 = w2 - 1; else w3 = w3 - 1;
      double px = at(p, 0, i), py = at(p, 1, i), pz = at(p, 2, i);
      at(opt, k, 0) += ((w1 * r2 + w2 * r5 + w3 * r8) * py + (-w1 * r1 - w2 * r4 - w3 * r7) * px +
                        (-w1 * r3 - w2 * r6 - w3 * r9) * pz);
      at(opt, k, 1) += ((2 * w1 * r1 + 2 * w2 * r4 + 2 * w3 * r7) * pz + (-2 * w1 * r3 - 2 * w2 * r6 - 2 * w3 * r9) * px);
      at(opt, k, 2) += (w1 * r1 + w2 * r4 + w3 * r7) * px + (w1 * r3 + w2 * r6 + w3 * r9) * pz +
                       (w1 * r2 + w2 * r5 + w3 * r8) * py;
    }
  }
  opt = mm(G, opt);
  double E2[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < n; i++) {
    double px = at(p, 0, i), py = at(p, 1, i), pz = at(p, 2, i);
    Mx Rpi = mx(3, 3);
    at(Rpi, 0, 0) = -px; at(Rpi, 0, 1) = 2 * pz; at(Rpi, 0, 2) = px;
    at(Rpi, 1, 0) = py;  at(Rpi, 1, 1) = 0;      at(Rpi, 1, 2) = py;
    at(Rpi, 2, 0) = -pz; at(Rpi, 2, 1) = -2 * px; at(Rpi, 2, 2) = pz;
    Mx E = mm(sub(I, V[i]), mmc(Rz, Rpi, opt));
    double e0[3], e1[3], e2[3];
    for (int r = 0; r < 3; r++) { e0[r] = at(E, r, 2); e1[r] = at(E, r, 1); e2[r] = at(E, r, 0); }
    double s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0;
    for (int r = 0; r < 3; r++) s1 += e2[r] * e2[r];
    for (int r = 0; r < 3; r++) s2 += 2 * (e1[r] * e2[r]);
    for (int r = 0; r < 3; r++) s3 += (e0[r] * e2[r]) * 2 + e1[r] * e1[r] + 0.0;
    for (int r = 0; r < 3; r++) s4 += 2 * (e0[r] * e1[r]);
    for (int r = 0; r < 3; r++) s5 += e0[r] * e0[r];
    E2[0] += s1; E2[1] += s2; E2[2] += s3; E2[3] += s4; E2[4] += s5;
  }
  double e4 = E2[0], e3 = E2[1], e2 = E2[2], e1 = E2[3], e0 = E2[4];
  double a4 = -e3, a3 = (4 * e4 - 2 * e2), a2 = (-3 * e1 + 3 * e3), a1 = (-4 * e0 + 2 * e2), a0 = e1;
  double coeffs[5] = {a4, a3, a2, a1, a0};
  double zr[5] = {0, 0, 0, 0, 0}, zi[5] = {0, 0, 0, 0, 0};
  rpoly(coeffs, 4, zr, zi);
  double atv[5];
  int nat = 0;
  for (int i = 0; i < 5; i++) {
    double _at = zr[i];
    double p1 = pow(1.0 + _at * _at, 3.0);
    if (fabs(p1) > 0.1 && zi[i] == 0) atv[nat++] = _at;
  }
  int nk = 0;
  for (int q = 0; q < nat; q++) {
    double a = atv[q];
    double sa = (2.0 * a) / (1.0 + a * a);
    double ca = (1.0 - a * a) / (1.0 + a * a);
    double alv = atan2(sa, ca) * 180 / M_PI;
    double tMaxMin = (4 * a4 * a * a * a + 3 * a3 * a * a + 2 * a2 * a + a1);
    if (tMaxMin > 0) { al[nk] = alv; at_out[nk] = a; nk++; }
  }
  for (int k = 0; k < nk; k++) {
    Mx R = mm(Rz, rpy_mat(0, (al[k] * M_PI / 180), 0));
    Mx t_opt = mx(3, 1);
    for (int i = 0; i < n; i++) t_opt = add(t_opt, mm(mm(sub(V[i], I), R), col(p, i)));
    tnew[k] = mm(G, t_opt);
  }
  return nk;
}

struct Result {
  double R[9], t[3];
  double obj_err, img_err;
  int iterations;
  int status;  // 1 ok; 0 2nd-pose search failed (first ObjPose kept)
  int error;   // 0; 1 GetRotationbyVector failed (reference exit(1)); 2 iteration cap; 3 no best
};

// RPP::Rpp (RPP.cpp:13-64) on model/iprts given as 3 x 4 row-major
MK_HD Result solve(const double* model, const double* iprts) {
  Result res;
  res.status = 0;
  res.error = 0;
  Mx P = mx(3, NP), Q = mx(3, NP);
  for (int i = 0; i < 3 * NP; i++) { P.a[i] = model[i]; Q.a[i] = iprts[i]; }
  Mx R, t;
  int it = 0;
  double oe = 0, ie = 0;
  int capped = obj_pose(P, Q, nullptr, R, t, it, oe, ie);
  auto fill = [&](const Mx& Rr, const Mx& tt, double o, double i2) {
    for (int k = 0; k < 9; k++) res.R[k] = Rr.a[k];
    for (int k = 0; k < 3; k++) res.t[k] = tt.a[k];
    res.obj_err = o;
    res.img_err = i2;
    res.iterations = it;
  };
  fill(R, t, oe, ie);
  res.error = capped ? 2 : 0;
  // Get2ndPose_Exact
  const int n = NP;
  Mx nv = tr(norm_rv(Q));
  Mx mean = mx(3, 1);
  for (int j = 0; j < 3; j++) {
    double s = 0;
    for (int i = 0; i < n; i++) s += at(nv, i, j);
    mean.a[j] = s / 3;
  }
  Mx cent = norm_rv(mean);
  double c3[3] = {cent.a[0], cent.a[1], cent.a[2]}, z[3] = {0, 0, 1};
  Mx Rim;
  if (!rot_by_vector(z, c3, Rim)) { res.error = 1; return res; }
  Mx v_ = mm(Rim, Q), R_ = mm(Rim, R), t_ = mm(Rim, t);
  Mx RzN;
  if (!decompose_r(R_, RzN)) return res;
  Mx R2 = mm(R_, RzN);
  Mx P_ = mm(tr(RzN), P);
  double ang[3];
  if (!rpy_ang_x(R2, ang)) return res;
  Mx Rz = rpy_mat(0, 0, ang[2]);
  double bl[5], atv[5];
  Mx tn[5];
  int nb = rot_y_wrt_t(v_, P_, Rz, bl, tn, atv);
  if (nb == 0) return res;
  Mx RimT = tr(Rim);
  int best = -1;
  double lowest = 1e6;
  Mx bestR, bestT;
  double bo = 0, bi = 0;
  for (int j = 0; j < nb; j++) {
    double b = bl[j] / 180 * M_PI;
    Mx sR = mm(RimT, mm(mm(Rz, rpy_mat(0, b, 0)), tr(RzN)));
    Mx st = mm(RimT, tn[j]);
    Mx Rl, tl;
    if (obj_pose(P, Q, &sR, Rl, tl, it, oe, ie)) res.error = 2;
    if (oe < lowest) { lowest = oe; best = j; bestR = Rl; bestT = tl; bo = oe; bi = ie; }
  }
  if (best < 0) { res.error = 3; return res; }
  fill(bestR, bestT, bo, bi);
  res.status = 1;
  return res;
}

}  // namespace rpp
}  // namespace mk
