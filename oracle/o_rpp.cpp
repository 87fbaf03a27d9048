// ORACLE — test infrastructure only. Never linked into the product path.
// Restates RPP.cpp / Rpoly.cpp (file:line in o_rpp.hpp) without cv::Mat.
// cv::Mat semantics reproduced on purpose (they move results by ulps):
//  * MatExpr "A / s" multiplies by (1/s); gemm sums k in order from 0.
//  * AbsKernel receives P and Q as shallow Mat copies and overwrites them in
//    place (RPP.cpp:236-246, 251-256), so the caller's image points are
//    replaced by F_i * q_i on the first ObjPose call (RPP.cpp:155).
//  * Mean() divides by the column count (RPP.cpp:508-523).
#include "o_rpp.hpp"

#include <cfloat>
#include <cmath>
#include <cstring>
#include <utility>

#include "o_cvrng.hpp"

namespace orc {

// ------------------------------------------------------------------- Rpoly
namespace {
struct JT {
  // State of one Jenkins–Traub run (Rpoly.cpp:11-754 restated).
  static void quadsd(int nn, double u, double v, const double* p, double* q, double* a, double* b) {
    q[0] = *b = p[0];
    q[1] = *a = -((*b) * u) + p[1];
    for (int i = 2; i < nn; i++) {
      q[i] = -((*a) * u + (*b) * v) + p[i];
      *b = *a;
      *a = q[i];
    }
  }
  static int calcsc(int n, double a, double b, double* a1, double* a3, double* a7, double* c, double* d,
                    double* e, double* f, double* g, double* h, const double* K, double u, double v, double* qk) {
    quadsd(n, u, v, K, qk, c, d);
    if (std::fabs(*c) <= 100.0 * DBL_EPSILON * std::fabs(K[n - 1]))
      if (std::fabs(*d) <= 100.0 * DBL_EPSILON * std::fabs(K[n - 2])) return 3;
    *h = v * b;
    if (std::fabs(*d) >= std::fabs(*c)) {
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
  static void nextk(int n, int tflag, double a, double b, double a1, double* a3, double* a7, double* K,
                    const double* qk, const double* qp) {
    if (tflag == 3) {
      K[1] = K[0] = 0.0;
      for (int i = 2; i < n; i++) K[i] = qk[i - 2];
      return;
    }
    double temp = (tflag == 1) ? b : a;
    if (std::fabs(a1) > 10.0 * DBL_EPSILON * std::fabs(temp)) {
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
  static void newest(int tflag, double* uu, double* vv, double a, double a1, double a3, double a7, double b,
                     double c, double d, double f, double g, double h, double u, double v, const double* K, int n,
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
  static void quad(double a, double b1, double c, double* sr, double* si, double* lr, double* li) {
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
    if (std::fabs(b) < std::fabs(c)) {
      e = (c >= 0) ? a : -a;
      e = -e + b * (b / std::fabs(c));
      d = std::sqrt(std::fabs(e)) * std::sqrt(std::fabs(c));
    } else {
      e = -((a / b) * (c / b)) + 1.0;
      d = std::sqrt(std::fabs(e)) * std::fabs(b);
    }
    if (e >= 0) {
      d = (b >= 0) ? -d : d;
      *lr = (-b + d) / a;
      *sr = (*lr != 0) ? (c / (*lr)) / a : *sr;
    } else {
      *lr = *sr = -(b / a);
      *si = std::fabs(d / a);
      *li = -(*si);
    }
  }
  static void quadit(int n, int* nz, double uu, double vv, double* szr, double* szi, double* lzr, double* lzi,
                     double* qp, int nn, double* a, double* b, const double* p, double* qk, double* a1, double* a3,
                     double* a7, double* c, double* d, double* e, double* f, double* g, double* h, double* K) {
    int j = 0, tflag, tried = 0;
    double ee, mp, omp = 0, relstp = 0, t, u, ui, v, vi, zm;
    *nz = 0;
    u = uu;
    v = vv;
    do {
      quad(1.0, u, v, szr, szi, lzr, lzi);
      if (std::fabs(std::fabs(*szr) - std::fabs(*lzr)) > 0.01 * std::fabs(*lzr)) break;
      quadsd(nn, u, v, p, qp, a, b);
      mp = std::fabs(-((*szr) * (*b)) + (*a)) + std::fabs((*szi) * (*b));
      zm = std::sqrt(std::fabs(v));
      ee = 2.0 * std::fabs(qp[0]);
      t = -((*szr) * (*b));
      for (int i = 1; i < n; i++) ee = ee * zm + std::fabs(qp[i]);
      ee = ee * zm + std::fabs((*a) + t);
      ee = (9.0 * ee + 2.0 * std::fabs(t) - 7.0 * (std::fabs((*a) + t) + zm * std::fabs(*b))) * DBL_EPSILON;
      if (mp <= 20.0 * ee) {
        *nz = 2;
        break;
      }
      j++;
      if (j > 20) break;
      if (j >= 2) {
        if ((relstp <= 0.01) && (mp >= omp) && (!tried)) {
          relstp = (relstp < DBL_EPSILON) ? std::sqrt(DBL_EPSILON) : std::sqrt(relstp);
          u -= u * relstp;
          v += v * relstp;
          quadsd(nn, u, v, p, qp, a, b);
          for (int i = 0; i < 5; i++) {
            tflag = calcsc(n, *a, *b, a1, a3, a7, c, d, e, f, g, h, K, u, v, qk);
            nextk(n, tflag, *a, *b, *a1, a3, a7, K, qk, qp);
          }
          tried = 1;
          j = 0;
        }
      }
      omp = mp;
      tflag = calcsc(n, *a, *b, a1, a3, a7, c, d, e, f, g, h, K, u, v, qk);
      nextk(n, tflag, *a, *b, *a1, a3, a7, K, qk, qp);
      tflag = calcsc(n, *a, *b, a1, a3, a7, c, d, e, f, g, h, K, u, v, qk);
      newest(tflag, &ui, &vi, *a, *a1, *a3, *a7, *b, *c, *d, *f, *g, *h, u, v, K, n, p);
      if (vi != 0) {
        relstp = std::fabs((-v + vi) / vi);
        u = ui;
        v = vi;
      }
    } while (vi != 0);
  }
  static void realit(int* iflag, int* nz, double* sss, int n, const double* p, int nn, double* qp, double* szr,
                     double* szi, double* K, double* qk) {
    int j = 0, nm1 = n - 1;
    double ee, kv, mp, ms, omp = 0, pv, s, t = 0;
    *iflag = *nz = 0;
    s = *sss;
    for (;;) {
      pv = p[0];
      qp[0] = pv;
      for (int i = 1; i < nn; i++) qp[i] = pv = pv * s + p[i];
      mp = std::fabs(pv);
      ms = std::fabs(s);
      ee = 0.5 * std::fabs(qp[0]);
      for (int i = 1; i < nn; i++) ee = ee * ms + std::fabs(qp[i]);
      if (mp <= 20.0 * DBL_EPSILON * (2.0 * ee - mp)) {
        *nz = 1;
        *szr = s;
        *szi = 0.0;
        break;
      }
      j++;
      if (j > 10) break;
      if (j >= 2) {
        if ((std::fabs(t) <= 0.001 * std::fabs(-t + s)) && (mp > omp)) {
          *iflag = 1;
          *sss = s;
          break;
        }
      }
      omp = mp;
      qk[0] = kv = K[0];
      for (int i = 1; i < n; i++) qk[i] = kv = kv * s + K[i];
      if (std::fabs(kv) > std::fabs(K[nm1]) * 10.0 * DBL_EPSILON) {
        t = -(pv / kv);
        K[0] = qp[0];
        for (int i = 1; i < n; i++) K[i] = t * qk[i - 1] + qp[i];
      } else {
        K[0] = 0.0;
        for (int i = 1; i < n; i++) K[i] = qk[i - 1];
      }
      kv = K[0];
      for (int i = 1; i < n; i++) kv = kv * s + K[i];
      t = (std::fabs(kv) > std::fabs(K[nm1]) * 10.0 * DBL_EPSILON) ? -(pv / kv) : 0.0;
      s += t;
    }
  }
  static void fxshfr(int l2, int* nz, double sr, double v, double* K, int n, const double* p, int nn, double* qp,
                     double u, double* lzi, double* lzr, double* szi, double* szr) {
    int fflag, iflag = 1, spass, stry, tflag, vpass, vtry;
    double a, a1, a3, a7, b, betas, betav, c, d, e, f, g, h, oss, ots = 0, otv = 0, ovv, s, ss, ts, tss, tv, tvv,
        ui, vi, vv;
    double qk[8], svk[8];
    *nz = 0;
    betav = betas = 0.25;
    oss = sr;
    ovv = v;
    quadsd(nn, u, v, p, qp, &a, &b);
    tflag = calcsc(n, a, b, &a1, &a3, &a7, &c, &d, &e, &f, &g, &h, K, u, v, qk);
    for (int j = 0; j < l2; j++) {
      fflag = 1;
      nextk(n, tflag, a, b, a1, &a3, &a7, K, qk, qp);
      tflag = calcsc(n, a, b, &a1, &a3, &a7, &c, &d, &e, &f, &g, &h, K, u, v, qk);
      newest(tflag, &ui, &vi, a, a1, a3, a7, b, c, d, f, g, h, u, v, K, n, p);
      vv = vi;
      ss = (K[n - 1] != 0.0) ? -(p[n] / K[n - 1]) : 0.0;
      ts = tv = 1.0;
      if ((j != 0) && (tflag != 3)) {
        tv = (vv != 0.0) ? std::fabs((vv - ovv) / vv) : tv;
        ts = (ss != 0.0) ? std::fabs((ss - oss) / ss) : ts;
        tvv = (tv < otv) ? tv * otv : 1.0;
        tss = (ts < ots) ? ts * ots : 1.0;
        vpass = (tvv < betav) ? 1 : 0;
        spass = (tss < betas) ? 1 : 0;
        if (spass || vpass) {
          for (int i = 0; i < n; i++) svk[i] = K[i];
          s = ss;
          stry = vtry = 0;
          for (;;) {
            // first pass may skip the quadratic iteration ("short circuit")
            bool skip_quad = false;
            if (fflag) {
              fflag = 0;
              skip_quad = spass && (!vpass || (tss < tvv));
            }
            if (!skip_quad) {
              quadit(n, nz, ui, vi, szr, szi, lzr, lzi, qp, nn, &a, &b, p, qk, &a1, &a3, &a7, &c, &d, &e, &f, &g,
                     &h, K);
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
              realit(&iflag, nz, &s, n, p, nn, qp, szr, szi, K, qk);
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
          quadsd(nn, u, v, p, qp, &a, &b);
          tflag = calcsc(n, a, b, &a1, &a3, &a7, &c, &d, &e, &f, &g, &h, K, u, v, qk);
        }
      }
      ovv = vv;
      oss = ss;
      otv = tv;
      ots = ts;
    }
  }
};
}  // namespace

int rpoly(const double* op, int degree, double* zeror, double* zeroi) {
  double K[8], p[8], pt[8], qp[8], temp[8];
  const double RADFAC = 3.14159265358979323846 / 180;
  const double lb2 = std::log(2.0);
  const double lo = DBL_MIN / DBL_EPSILON;
  const double cosr = std::cos(94.0 * RADFAC);
  const double sinr = std::sin(94.0 * RADFAC);
  if (degree > 6) return -1;
  if (op[0] == 0) return 0;
  int N = degree, NN, NM1, NZ, l, zerok, j, jj;
  double xx = std::sqrt(0.5), yy = -xx, bnd, df, dx, factor, ff, mx, mn, sc, x, xm, aa, bb, cc, lzi, lzr, sr, szi,
         szr, t, u, xxx;
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
        JT::quad(p[0], p[1], p[2], &zeror[degree - 2], &zeroi[degree - 2], &zeror[degree - 1], &zeroi[degree - 1]);
      }
      break;
    }
    mx = 0.0;
    mn = DBL_MAX;
    for (int i = 0; i < NN; i++) {
      x = std::fabs(p[i]);
      if (x > mx) mx = x;
      if ((x != 0) && (x < mn)) mn = x;
    }
    sc = lo / mn;
    if (((sc <= 1.0) && (mx >= 10)) || ((sc > 1.0) && (DBL_MAX / sc >= mx))) {
      sc = (sc == 0) ? DBL_MIN : sc;
      l = (int)(std::log(sc) / lb2 + 0.5);
      factor = std::pow(2.0, l);
      if (factor != 1.0)
        for (int i = 0; i < NN; i++) p[i] *= factor;
    }
    for (int i = 0; i < NN; i++) pt[i] = std::fabs(p[i]);
    pt[N] = -(pt[N]);
    NM1 = N - 1;
    x = std::exp((std::log(-pt[N]) - std::log(pt[0])) / (double)N);
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
    } while (std::fabs(dx / x) > 0.005);
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
        zerok = (std::fabs(K[NM1]) <= std::fabs(bb) * DBL_EPSILON * 10.0) ? 1 : 0;
      }
    }
    for (int i = 0; i < N; i++) temp[i] = K[i];
    for (jj = 1; jj <= 20; jj++) {
      xxx = -(sinr * yy) + cosr * xx;
      yy = sinr * xx + cosr * yy;
      xx = xxx;
      sr = bnd * xx;
      u = -(2.0 * sr);
      JT::fxshfr(20 * jj, &NZ, sr, bnd, K, N, p, NN, qp, u, &lzi, &lzr, &szi, &szr);
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

// ------------------------------------------------------------- JacobiSVD
static void jacobi_svd(double* At, int m, int n, double* Wout, double* Vt, int n1) {
  const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
  double W[8];
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
        if (std::fabs(p) <= eps * std::sqrt(a * b)) continue;
        p *= 2;
        double beta = a - b, gamma = std::hypot(p, beta), c, s;
        if (beta < 0) {
          double delta = (gamma - beta) * 0.5;
          s = std::sqrt(delta / gamma);
          c = p / (gamma * s * 2);
        } else {
          c = std::sqrt((gamma + beta) / (gamma * 2));
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
    W[i] = std::sqrt(sd);
  }
  for (int i = 0; i < n - 1; i++) {
    int j = i;
    for (int k = i + 1; k < n; k++) if (W[j] < W[k]) j = k;
    if (i != j) {
      std::swap(W[i], W[j]);
      if (Vt) {
        for (int k = 0; k < m; k++) std::swap(At[i * m + k], At[j * m + k]);
        for (int k = 0; k < n; k++) std::swap(Vt[i * n + k], Vt[j * n + k]);
      }
    }
  }
  for (int i = 0; i < n; i++) Wout[i] = W[i];
  if (!Vt) return;
  CvRng rng(0x12345678);
  for (int i = 0; i < n1; i++) {
    double sd = i < n ? W[i] : 0;
    for (int ii = 0; ii < 100 && sd <= minval; ii++) {
      const double val0 = 1. / m;
      for (int k = 0; k < m; k++) At[i * m + k] = (rng.next() & 256) != 0 ? val0 : -val0;
      for (int it = 0; it < 2; it++)
        for (int j = 0; j < i; j++) {
          sd = 0;
          for (int k = 0; k < m; k++) sd += At[i * m + k] * At[j * m + k];
          double asum = 0;
          for (int k = 0; k < m; k++) {
            double t = At[i * m + k] - sd * At[j * m + k];
            At[i * m + k] = t;
            asum += std::fabs(t);
          }
          asum = asum > eps * 100 ? 1 / asum : 0;
          for (int k = 0; k < m; k++) At[i * m + k] *= asum;
        }
      sd = 0;
      for (int k = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
      sd = std::sqrt(sd);
    }
    double s = sd > minval ? 1 / sd : 0.;
    for (int k = 0; k < m; k++) At[i * m + k] *= s;
  }
}

void cv_svd(const double* A, int m, int n, double* w, double* u, double* vt) {
  // m >= n only (the shapes RPP uses); At = A^T is n rows of length m.
  double At[64], Vt[64];
  for (int i = 0; i < n; i++)
    for (int k = 0; k < m; k++) At[i * m + k] = A[k * n + i];
  jacobi_svd(At, m, n, w, Vt, n);
  if (u)
    for (int r = 0; r < m; r++)
      for (int c = 0; c < n; c++) u[r * n + c] = At[c * m + r];
  if (vt) std::memcpy(vt, Vt, sizeof(double) * n * n);
}

// --------------------------------------------------------- small matrices
namespace {
struct Mx {
  int r = 0, c = 0;
  double a[3 * 16];
  Mx() {}
  Mx(int r_, int c_, double v = 0) : r(r_), c(c_) { for (int i = 0; i < r * c; i++) a[i] = v; }
  double& operator()(int i, int j) { return a[i * c + j]; }
  double operator()(int i, int j) const { return a[i * c + j]; }
};
Mx eye3() { Mx m(3, 3); m(0, 0) = m(1, 1) = m(2, 2) = 1; return m; }
// gemm: sum_k A(i,k) B(k,j) from 0, times alpha
Mx mm(const Mx& A, const Mx& B, double alpha = 1.0) {
  Mx o(A.r, B.c);
  for (int i = 0; i < A.r; i++)
    for (int j = 0; j < B.c; j++) {
      double s = 0;
      for (int k = 0; k < A.c; k++) s += A(i, k) * B(k, j);
      o(i, j) = s * alpha;
    }
  return o;
}
// gemm with C: (sum)*1 + C*1
Mx mmc(const Mx& A, const Mx& B, const Mx& C) {
  Mx o = mm(A, B);
  for (int i = 0; i < o.r * o.c; i++) o.a[i] = o.a[i] + C.a[i];
  return o;
}
Mx tr(const Mx& A) { Mx o(A.c, A.r); for (int i = 0; i < A.r; i++) for (int j = 0; j < A.c; j++) o(j, i) = A(i, j); return o; }
Mx add(const Mx& A, const Mx& B) { Mx o(A.r, A.c); for (int i = 0; i < A.r * A.c; i++) o.a[i] = A.a[i] + B.a[i]; return o; }
Mx sub(const Mx& A, const Mx& B) { Mx o(A.r, A.c); for (int i = 0; i < A.r * A.c; i++) o.a[i] = A.a[i] - B.a[i]; return o; }
Mx scl(const Mx& A, double s) { Mx o(A.r, A.c); for (int i = 0; i < A.r * A.c; i++) o.a[i] = A.a[i] * s; return o; }
Mx col(const Mx& A, int j) { Mx o(3, 1); for (int i = 0; i < 3; i++) o(i, 0) = A(i, j); return o; }
double det3(const Mx& m) {
  return m(0, 0) * (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) - m(0, 1) * (m(1, 0) * m(2, 2) - m(1, 2) * m(2, 0)) +
         m(0, 2) * (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0));
}
Mx inv3(const Mx& M) {
  Mx D(3, 3);
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
Mx rowsum(const Mx& P) {  // Sum(P, 2)
  Mx o(P.r, 1);
  for (int i = 0; i < P.r; i++) { double s = 0; for (int j = 0; j < P.c; j++) s += P(i, j); o(i, 0) = s; }
  return o;
}
double sqnorm3(const Mx& v) { double x = v(0, 0), y = v(1, 0), z = v(2, 0); return x * x + y * y + z * z; }
int sgn(double x) { return x < 0 ? -1 : (x > 0 ? 1 : 0); }
double norm_svd(const Mx& A) {  // RPP Norm(): largest singular value
  double w[3];
  if (A.c == 1) { cv_svd(A.a, A.r, 1, w, nullptr, nullptr); return w[0]; }
  double u[9], vt[9];
  cv_svd(A.a, A.r, A.c, w, u, vt);
  return w[0];
}
Mx xform(const Mx& P, const Mx& R, const Mx& t) {
  Mx o(3, P.c);
  for (int i = 0; i < P.c; i++) {
    double x = P(0, i), y = P(1, i), z = P(2, i);
    for (int r = 0; r < 3; r++) o(r, i) = R(r, 0) * x + R(r, 1) * y + R(r, 2) * z + t(r, 0);
  }
  return o;
}
Mx rpy_mat(double a0, double a1, double a2) {
  double cosA = std::cos(a2), sinA = std::sin(a2), cosB = std::cos(a1), sinB = std::sin(a1), cosC = std::cos(a0),
         sinC = std::sin(a0);
  double cosAsinB = cosA * sinB, sinAsinB = sinA * sinB;
  Mx R(3, 3);
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
bool rpy_ang(const Mx& R, double ang[3]) {
  double R11 = R(0, 0), R12 = R(0, 1), R13 = R(0, 2), R21 = R(1, 0), R22 = R(1, 1), R23 = R(1, 2), R31 = R(2, 0),
         R32 = R(2, 1), R33 = R(2, 2);
  double sinB = -R31, cosB = std::sqrt(R11 * R11 + R21 * R21), a[3];
  if (std::fabs(cosB) > 1e-15) {
    double sinA = R21 / cosB, cosA = R11 / cosB, sinC = R32 / cosB, cosC = R33 / cosB;
    a[0] = std::atan2(sinC, cosC);
    a[1] = std::atan2(sinB, cosB);
    a[2] = std::atan2(sinA, cosA);
  } else {
    double sinC = (R12 - R23) / 2, cosC = (R22 + R13) / 2;
    a[0] = std::atan2(sinC, cosC);
    a[1] = M_PI_2;
    a[2] = 0;
    if (sinB < 0) { a[0] = -a[0]; a[1] = -a[1]; a[2] = -a[2]; }
  }
  if (norm_svd(sub(R, rpy_mat(a[0], a[1], a[2]))) > 1e-6) return false;
  ang[0] = a[0]; ang[1] = a[1]; ang[2] = a[2];
  return true;
}
bool rpy_ang_x(const Mx& R, double a[3]) {
  if (!rpy_ang(R, a)) return false;
  if (std::fabs(a[0]) > M_PI_2) {
    while (std::fabs(a[0]) > M_PI_2) {
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
Mx norm_rv(const Mx& R) {  // columns scaled by 1/sqrt(|col|^2)
  Mx o(R.r, R.c);
  for (int i = 0; i < R.c; i++) {
    double mag = R(0, i) * R(0, i) + R(1, i) * R(1, i) + R(2, i) * R(2, i);
    double m = 1.0 / std::sqrt(mag);
    for (int r = 0; r < 3; r++) o(r, i) = R(r, i) * m;
  }
  return o;
}

struct Sol { Mx R, t; double at; double obj_err, img_err; };

void abs_kernel(Mx& P, Mx& Q, const Mx* F, const Mx& G, Mx& R, Mx& t, Mx& Qout, double& err2) {
  int n = P.c;
  for (int i = 0; i < n; i++) {
    Mx q = mm(F[i], col(Q, i));
    for (int r = 0; r < 3; r++) Q(r, i) = q(r, 0);
  }
  Mx pbar = scl(rowsum(P), 1.0 / n);
  for (int i = 0; i < n; i++)
    for (int r = 0; r < 3; r++) P(r, i) -= pbar(r, 0);
  Mx M(3, 3);
  for (int i = 0; i < n; i++)
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) M(a, b) += P(a, i) * Q(b, i);
  double w[3], u[9], vt[9];
  cv_svd(M.a, 3, 3, w, u, vt);
  Mx U(3, 3), V(3, 3);
  for (int i = 0; i < 9; i++) U.a[i] = u[i];
  for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) V(i, j) = vt[j * 3 + i];
  Mx Ut = tr(U);
  auto estimate_t = [&](const Mx& Rr) {
    Mx sum(3, 1);
    for (int i = 0; i < n; i++) sum = add(sum, mm(mm(F[i], Rr), col(P, i)));
    return mm(G, sum);
  };
  R = mm(V, Ut);
  if (sgn(det3(R)) == 1) {
    t = estimate_t(R);
    if (t(2, 0) < 0) {
      for (int r = 0; r < 3; r++) V(r, 2) = -V(r, 2);
      R = mm(V, Ut, -1.0);
      t = estimate_t(R);
    }
  } else {
    for (int r = 0; r < 3; r++) V(r, 2) = -V(r, 2);
    R = mm(V, Ut);
    t = estimate_t(R);
    if (t(2, 0) < 0) {
      R = mm(V, Ut, -1.0);
      t = estimate_t(R);
    }
  }
  Mx I = eye3();
  err2 = 0;
  Qout = xform(P, R, t);
  for (int i = 0; i < n; i++) err2 += sqnorm3(mm(sub(I, F[i]), col(Qout, i)));
}

int obj_pose(const Mx& P0, Mx& Qp, const Mx* initR, Mx& R, Mx& t, int& it, double& obj_err, double& img_err) {
  const double TOL = 1E-5, EPS = 1E-8;
  Mx P = P0;
  int n = P.c;
  it = 0;
  Mx pbar = scl(rowsum(P), 1.0 / n);
  for (int i = 0; i < n; i++)
    for (int r = 0; r < 3; r++) P(r, i) -= pbar(r, 0);
  Mx F[16];
  for (int i = 0; i < n; i++) {
    Mx V = col(Qp, i);
    double ret = mm(tr(V), V)(0, 0);
    F[i] = mm(V, tr(V), 1.0 / ret);
  }
  Mx sumF(3, 3);
  for (int i = 0; i < n; i++) sumF = add(sumF, F[i]);
  Mx I = eye3();
  Mx tFactor = scl(inv3(sub(I, scl(sumF, 1.0 / n))), 1.0 / n);
  double old_err, new_err;
  Mx Qi, Ri, ti;
  if (initR) {
    Ri = *initR;
    Mx s(3, 1);
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
  while (std::fabs((old_err - new_err) / old_err) > TOL && (new_err > EPS)) {
    if (it >= 100000) { capped = 1; break; }
    old_err = new_err;
    abs_kernel(P, Qi, F, tFactor, Ri, ti, Qi, new_err);
    it = it + 1;
  }
  R = Ri;
  t = ti;
  obj_err = std::sqrt(new_err / n);
  img_err = 0;
  for (int i = 0; i < n; i++) {
    Mx Qproj = mmc(Ri, col(P, i), ti);
    double xx = (Qproj(0, 0) / Qproj(2, 0)) - Qp(0, 0);
    double yy = (Qproj(1, 0) / Qproj(2, 0)) - Qp(1, 0);
    img_err += (xx * xx + yy * yy);
  }
  img_err = std::sqrt(img_err / n);
  Mx rp = mm(Ri, pbar);
  t = sub(t, rp);
  return capped;
}

bool rot_by_vector(const double v1[3], const double v2[3], Mx& R) {
  double d = v2[0] * v1[0] + v2[1] * v1[1] + v2[2] * v1[2];
  double winkel = std::acos(d);
  double ax[3] = {v2[1] * v1[2] - v2[2] * v1[1], v2[2] * v1[0] - v2[0] * v1[2], v2[0] * v1[1] - v2[1] * v1[0]};
  Mx axm(3, 1);
  for (int i = 0; i < 3; i++) axm(i, 0) = ax[i];
  double nn = norm_svd(axm);
  double ra[3] = {ax[0], ax[1], ax[2]};
  for (int i = 0; i < 3; i++) ra[i] /= nn;
  for (int i = 0; i < 3; i++) ra[i] *= std::sin(winkel * 0.5);
  double qs = std::cos(winkel * 0.5);
  double qn = std::sqrt(ra[0] * ra[0] + ra[1] * ra[1] + ra[2] * ra[2] + qs * qs);
  double inv = 1 / qn;
  double a = qs * inv, b = ra[0] * inv, c = ra[1] * inv, dd = ra[2] * inv;
  R = Mx(3, 3);
  R(0, 0) = a * a + b * b - c * c - dd * dd;
  R(0, 1) = 2 * (b * c - a * dd);
  R(0, 2) = 2 * (b * dd + a * c);
  R(1, 0) = 2 * (b * c + a * dd);
  R(1, 1) = a * a + c * c - b * b - dd * dd;
  R(1, 2) = 2 * (c * dd - a * b);
  R(2, 0) = 2 * (b * dd - a * c);
  R(2, 1) = 2 * (c * dd + a * b);
  R(2, 2) = a * a + dd * dd - b * b - c * c;
  Mx n1(3, 1), n2(3, 1);
  for (int i = 0; i < 3; i++) { n1(i, 0) = v1[i]; n2(i, 0) = v2[i]; }
  auto nrv = [](Mx v) {
    double mag = std::sqrt(v(0, 0) * v(0, 0) + v(1, 0) * v(1, 0) + v(2, 0) * v(2, 0));
    for (int i = 0; i < 3; i++) v(i, 0) = v(i, 0) / mag;
    return v;
  };
  Mx diff = sub(nrv(n1), mm(R, nrv(n2)));
  double s = 0;
  for (int i = 0; i < 3; i++) s += diff(i, 0) * diff(i, 0);
  return !(s * s > 1e-3);
}

bool decompose_r(const Mx& R, Mx& RzN) {
  double cl = std::atan2(R(2, 1), R(2, 0));
  Mx Rz = rpy_mat(0, 0, cl);
  Mx R_ = mm(R, Rz);
  if (R_(2, 1) > 1e-3) return false;
  double ang[3];
  if (!rpy_ang_x(R_, ang)) return false;
  if (std::fabs(ang[0]) > 1e-3) return false;
  Mx Rz2 = mm(Rz, rpy_mat(0, 0, M_PI));
  R_ = mm(R, Rz2);
  if (R_(2, 1) > 1e-3) return false;
  if (!rpy_ang_x(R_, ang)) return false;
  RzN = Rz;
  return true;
}

void rot_y_wrt_t(const Mx& v, const Mx& p, const Mx& Rz, std::vector<double>& al, std::vector<Mx>& tnew,
                 std::vector<double>& at) {
  int n = v.c;
  Mx V[16];
  for (int i = 0; i < n; i++) {
    Mx vv = col(v, i);
    double a = mm(tr(vv), vv)(0, 0);
    V[i] = mm(vv, tr(vv), 1.0 / a);
  }
  Mx G(3, 3);
  for (int i = 0; i < n; i++) G = add(G, V[i]);
  Mx I = eye3();
  G = scl(inv3(sub(I, scl(G, 1.0 / n))), 1.0 / n);
  Mx opt(3, 3);
  const double r1 = Rz(0, 0), r2 = Rz(0, 1), r3 = Rz(0, 2), r4 = Rz(1, 0), r5 = Rz(1, 1), r6 = Rz(1, 2),
               r7 = Rz(2, 0), r8 = Rz(2, 1), r9 = Rz(2, 2);
  for (int i = 0; i < n; i++) {
    // rows k of (V_i - I): (w1, w2, w3); RPP.cpp:1004-1016 expanded per row
    for (int k = 0; k < 3; k++) {
      double w1 = V[i](k, 0), w2 = V[i](k, 1), w3 = V[i](k, 2);
      if (k == 0) w1 = w1 - 1; else if (k == 1) w2 = w2 - 1; else w3 = w3 - 1;
      double px = p(0, i), py = p(1, i), pz = p(2, i);
      // (w1-1 substitution already applied: the reference writes e.g. (v11-1)*r2)
      opt(k, 0) += ((w1 * r2 + w2 * r5 + w3 * r8) * py + (-w1 * r1 - w2 * r4 - w3 * r7) * px +
                    (-w1 * r3 - w2 * r6 - w3 * r9) * pz);
      opt(k, 1) += ((2 * w1 * r1 + 2 * w2 * r4 + 2 * w3 * r7) * pz + (-2 * w1 * r3 - 2 * w2 * r6 - 2 * w3 * r9) * px);
      opt(k, 2) += (w1 * r1 + w2 * r4 + w3 * r7) * px + (w1 * r3 + w2 * r6 + w3 * r9) * pz +
                   (w1 * r2 + w2 * r5 + w3 * r8) * py;
    }
  }
  opt = mm(G, opt);
  double E2[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < n; i++) {
    double px = p(0, i), py = p(1, i), pz = p(2, i);
    Mx Rpi(3, 3);
    Rpi(0, 0) = -px; Rpi(0, 1) = 2 * pz; Rpi(0, 2) = px;
    Rpi(1, 0) = py;  Rpi(1, 1) = 0;      Rpi(1, 2) = py;
    Rpi(2, 0) = -pz; Rpi(2, 1) = -2 * px; Rpi(2, 2) = pz;
    Mx E = mm(sub(I, V[i]), mmc(Rz, Rpi, opt));
    double e0[3], e1[3], e2[3];
    for (int r = 0; r < 3; r++) { e0[r] = E(r, 2); e1[r] = E(r, 1); e2[r] = E(r, 0); }
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
  at.clear();
  for (int i = 0; i < 5; i++) {
    double _at = zr[i];
    double p1 = std::pow(1.0 + _at * _at, 3.0);
    if (std::fabs(p1) > 0.1 && zi[i] == 0) at.push_back(_at);
  }
  std::vector<double> al2, at2;
  for (double a : at) {
    double sa = (2.0 * a) / (1.0 + a * a);
    double ca = (1.0 - a * a) / (1.0 + a * a);
    double alv = std::atan2(sa, ca) * 180 / M_PI;
    double tMaxMin = (4 * a4 * a * a * a + 3 * a3 * a * a + 2 * a2 * a + a1);
    if (tMaxMin > 0) { al2.push_back(alv); at2.push_back(a); }
  }
  al = al2;
  at = at2;
  tnew.clear();
  for (double alv : al) {
    Mx R = mm(Rz, rpy_mat(0, (alv * M_PI / 180), 0));
    Mx t_opt(3, 1);
    for (int i = 0; i < n; i++) t_opt = add(t_opt, mm(mm(sub(V[i], I), R), col(p, i)));
    tnew.push_back(mm(G, t_opt));
  }
}

// returns 0 = fail (Rpp false), 1 = ok, -1 = rotation check failure (exit(1) in the reference)
int second_pose(const Mx& v, const Mx& P, const Mx& R, const Mx& t, std::vector<Sol>& sols) {
  int n = v.c;
  Mx nv = tr(norm_rv(v));  // n x 3
  Mx mean(3, 1);
  for (int j = 0; j < 3; j++) {
    double s = 0;
    for (int i = 0; i < n; i++) s += nv(i, j);
    mean(j, 0) = s / 3;  // Mean() divides by m.cols
  }
  Mx cent = norm_rv(mean);
  double c3[3] = {cent(0, 0), cent(1, 0), cent(2, 0)}, z[3] = {0, 0, 1};
  Mx Rim;
  if (!rot_by_vector(z, c3, Rim)) return -1;
  Mx v_ = mm(Rim, v), R_ = mm(Rim, R), t_ = mm(Rim, t);
  // GetRfor2ndPose_V_Exact
  Mx RzN;
  if (!decompose_r(R_, RzN)) return 0;
  Mx R2 = mm(R_, RzN);
  Mx P_ = mm(tr(RzN), P);
  double ang[3];
  if (!rpy_ang_x(R2, ang)) return 0;
  Mx Rz = rpy_mat(0, 0, ang[2]);
  std::vector<double> bl, at;
  std::vector<Mx> tn;
  rot_y_wrt_t(v_, P_, Rz, bl, tn, at);
  if (bl.empty()) return 0;
  sols.clear();
  Mx RimT = tr(Rim);
  for (size_t j = 0; j < bl.size(); j++) {
    double b = bl[j] / 180 * M_PI;
    Sol s;
    s.at = at[j];
    s.R = mm(mm(Rz, rpy_mat(0, b, 0)), tr(RzN));
    s.t = tn[j];
    s.R = mm(RimT, s.R);
    s.t = mm(RimT, s.t);
    sols.push_back(s);
  }
  return 1;
}
}  // namespace

RppResult rpp(const double* model, const double* iprts, int n) {
  RppResult res{};
  Mx P(3, n), Q(3, n);
  for (int i = 0; i < 3 * n; i++) { P.a[i] = model[i]; Q.a[i] = iprts[i]; }
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
  std::vector<Sol> sols;
  int st = second_pose(Q, P, R, t, sols);
  if (st <= 0) {
    res.status = 0;
    if (st < 0) res.error = 1;
    return res;
  }
  int best = -1;
  double lowest = 1e6;
  for (size_t i = 0; i < sols.size(); i++) {
    Mx Rl, tl;
    if (obj_pose(P, Q, &sols[i].R, Rl, tl, it, oe, ie)) res.error = 2;
    sols[i].R = Rl;
    sols[i].t = tl;
    sols[i].obj_err = oe;
    sols[i].img_err = ie;
    if (oe < lowest) { lowest = oe; best = (int)i; }
  }
  if (best < 0) {  // reference indexes sol[-1] (UB); defined here as "keep first pose"
    res.status = 0;
    res.error = 3;
    return res;
  }
  fill(sols[best].R, sols[best].t, sols[best].obj_err, sols[best].img_err);
  res.status = 1;
  return res;
}

}  // namespace orc
