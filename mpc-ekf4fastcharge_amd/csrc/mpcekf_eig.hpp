// mpcekf_eig.hpp -- eigenvalues and singular values of the closed-loop matrix of
// iterMPC.m:53-60 (CL = Abar - Bbar*Kmpc, 7 x 7), for mpcData.poles / mpcData.sv.
//
// MATLAB's eig(CL) is LAPACK's balanced Hessenberg QR and svd(CL) its bidiagonal QR; the
// order in which eig returns the poles is LAPACK's deflation order.  Here:
//   poles: balancing by powers of 2 (exact), reduction to upper Hessenberg form by
//          stabilised elementary similarity transforms, then the Francis double-shift
//          QR iteration on the Hessenberg matrix; returned sorted by descending real
//          part, then descending imaginary part (conjugate pairs: + first).
//   sv:    one-sided Jacobi (Hestenes) on the columns of CL, the column norms at
//          convergence, descending (as svd returns them).
// Plain double arithmetic, callable from host (the C-ABI's mpcekf_cl_eig, CPU tests)
// and device (k_cl_diag).  Test: tests/test_diag.py against numpy.linalg.eigvals/svd.
#pragma once
#include <math.h>

#if defined(__HIPCC__)
#define MPCEKF_HD __host__ __device__
#else
#define MPCEKF_HD
#endif

namespace mk {
namespace eig {

constexpr int MAXN = 8;

template <class T>
MPCEKF_HD inline void swp(T &a, T &b) {
  T t = a;
  a = b;
  b = t;
}
MPCEKF_HD inline double sgn(double a, double b) { return b >= 0.0 ? fabs(a) : -fabs(a); }

// Balance rows/columns by powers of two so that their off-diagonal 1-norms are similar
// (exact scaling: the eigenvalues are unchanged bit for bit by the similarity).
MPCEKF_HD inline void balance(int n, double a[MAXN][MAXN]) {
  const double radix = 2.0, sq = radix * radix;
  bool done = false;
  for (int guard = 0; !done && guard < 64; ++guard) {
    done = true;
    for (int i = 0; i < n; ++i) {
      double r = 0.0, c = 0.0;
      for (int j = 0; j < n; ++j)
        if (j != i) {
          c += fabs(a[j][i]);
          r += fabs(a[i][j]);
        }
      if (c == 0.0 || r == 0.0 || !isfinite(c) || !isfinite(r)) continue;
      double g = r / radix, f = 1.0;
      const double s = c + r;
      while (c < g) {
        f *= radix;
        c *= sq;
      }
      g = r * radix;
      while (c > g) {
        f /= radix;
        c /= sq;
      }
      if ((c + r) / f < 0.95 * s) {
        done = false;
        const double gi = 1.0 / f;
        for (int j = 0; j < n; ++j) a[i][j] *= gi;
        for (int j = 0; j < n; ++j) a[j][i] *= f;
      }
    }
  }
}

// Reduce to upper Hessenberg form by elimination with partial pivoting (a similarity:
// row and column operations in pairs); the entries below the subdiagonal are zeroed.
MPCEKF_HD inline void hessenberg(int n, double a[MAXN][MAXN]) {
  for (int m = 1; m < n - 1; ++m) {
    double x = 0.0;
    int i = m;
    for (int j = m; j < n; ++j)
      if (fabs(a[j][m - 1]) > fabs(x)) {
        x = a[j][m - 1];
        i = j;
      }
    if (i != m) {
      for (int j = m - 1; j < n; ++j) swp(a[i][j], a[m][j]);
      for (int j = 0; j < n; ++j) swp(a[j][i], a[j][m]);
    }
    if (x != 0.0) {
      for (i = m + 1; i < n; ++i) {
        double y = a[i][m - 1];
        if (y != 0.0) {
          y /= x;
          a[i][m - 1] = y;
          for (int j = m; j < n; ++j) a[i][j] -= y * a[m][j];
          for (int j = 0; j < n; ++j) a[j][m] += y * a[j][i];
        }
      }
    }
  }
  for (int i = 2; i < n; ++i)
    for (int j = 0; j < i - 1; ++j) a[i][j] = 0.0;
}

// Francis double-shift QR on an upper Hessenberg matrix (destroyed): eigenvalues
// (wr + i wi).  Returns false when an eigenvalue needs more than 60 iterations (the
// unconverged ones are NaN).
MPCEKF_HD inline bool hqr(int n, double a[MAXN][MAXN], double wr[MAXN], double wi[MAXN]) {
  double anorm = 0.0;
  for (int i = 0; i < n; ++i)
    for (int j = (i > 0 ? i - 1 : 0); j < n; ++j) anorm += fabs(a[i][j]);
  int nn = n - 1;
  double t = 0.0;
  while (nn >= 0) {
    int its = 0, l;
    do {
      for (l = nn; l >= 1; --l) {  // a small subdiagonal element splits the matrix
        double s = fabs(a[l - 1][l - 1]) + fabs(a[l][l]);
        if (s == 0.0) s = anorm;
        if (fabs(a[l][l - 1]) + s == s) {
          a[l][l - 1] = 0.0;
          break;
        }
      }
      double x = a[nn][nn];
      if (l == nn) {  // one root
        wr[nn] = x + t;
        wi[nn] = 0.0;
        --nn;
      } else {
        double y = a[nn - 1][nn - 1];
        double w = a[nn][nn - 1] * a[nn - 1][nn];
        if (l == nn - 1) {  // two roots
          const double p = 0.5 * (y - x);
          const double q = p * p + w;
          double z = sqrt(fabs(q));
          x += t;
          if (q >= 0.0) {
            z = p + sgn(z, p);
            wr[nn - 1] = wr[nn] = x + z;
            if (z != 0.0) wr[nn] = x - w / z;
            wi[nn - 1] = wi[nn] = 0.0;
          } else {
            wr[nn - 1] = wr[nn] = x + p;
            wi[nn - 1] = -(wi[nn] = z);
          }
          nn -= 2;
        } else {  // a double-shift QR step on rows/columns l..nn
          if (its == 60) {
            for (int i = 0; i <= nn; ++i) wr[i] = wi[i] = NAN;
            return false;
          }
          if (its == 10 || its == 20 || its == 40) {  // exceptional shift
            t += x;
            for (int i = 0; i <= nn; ++i) a[i][i] -= x;
            const double s = fabs(a[nn][nn - 1]) + fabs(a[nn - 1][nn - 2]);
            y = x = 0.75 * s;
            w = -0.4375 * s * s;
          }
          ++its;
          int m;
          double p = 0.0, q = 0.0, r = 0.0, z;
          for (m = nn - 2; m >= l; --m) {
            z = a[m][m];
            r = x - z;
            double s = y - z;
            p = (r * s - w) / a[m + 1][m] + a[m][m + 1];
            q = a[m + 1][m + 1] - z - r - s;
            r = a[m + 2][m + 1];
            s = fabs(p) + fabs(q) + fabs(r);
            p /= s;
            q /= s;
            r /= s;
            if (m == l) break;
            const double u = fabs(a[m][m - 1]) * (fabs(q) + fabs(r));
            const double v = fabs(p) * (fabs(a[m - 1][m - 1]) + fabs(z) + fabs(a[m + 1][m + 1]));
            if (u + v == v) break;
          }
          for (int i = m + 2; i <= nn; ++i) {
            a[i][i - 2] = 0.0;
            if (i != m + 2) a[i][i - 3] = 0.0;
          }
          for (int k = m; k <= nn - 1; ++k) {
            if (k != m) {
              p = a[k][k - 1];
              q = a[k + 1][k - 1];
              r = 0.0;
              if (k != nn - 1) r = a[k + 2][k - 1];
              if ((x = fabs(p) + fabs(q) + fabs(r)) != 0.0) {
                p /= x;
                q /= x;
                r /= x;
              }
            }
            const double s = sgn(sqrt(p * p + q * q + r * r), p);
            if (s != 0.0) {
              if (k == m) {
                if (l != m) a[k][k - 1] = -a[k][k - 1];
              } else {
                a[k][k - 1] = -s * x;
              }
              p += s;
              x = p / s;
              y = q / s;
              z = r / s;
              q /= p;
              r /= p;
              for (int j = k; j <= nn; ++j) {
                p = a[k][j] + q * a[k + 1][j];
                if (k != nn - 1) {
                  p += r * a[k + 2][j];
                  a[k + 2][j] -= p * z;
                }
                a[k + 1][j] -= p * y;
                a[k][j] -= p * x;
              }
              const int mmin = nn < k + 3 ? nn : k + 3;
              for (int i = l; i <= mmin; ++i) {
                p = x * a[i][k] + y * a[i][k + 1];
                if (k != nn - 1) {
                  p += z * a[i][k + 2];
                  a[i][k + 2] -= p * r;
                }
                a[i][k + 1] -= p * q;
                a[i][k] -= p;
              }
            }
          }
        }
      }
    } while (l < nn - 1);
  }
  return true;
}

// eigenvalues of a general n x n (row-major, n <= MAXN), sorted: descending real part,
// then descending imaginary part
MPCEKF_HD inline bool eigvals(int n, const double *A, double *re, double *im) {
  double a[MAXN][MAXN];
  bool fin = true;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      a[i][j] = A[i * n + j];
      fin = fin && isfinite(a[i][j]);
    }
  if (!fin) {
    for (int i = 0; i < n; ++i) re[i] = im[i] = NAN;
    return false;
  }
  balance(n, a);
  hessenberg(n, a);
  double wr[MAXN], wi[MAXN];
  const bool ok = hqr(n, a, wr, wi);
  for (int i = 1; i < n; ++i) {  // insertion sort
    const double r = wr[i], m = wi[i];
    int j = i - 1;
    while (j >= 0 && (wr[j] < r || (wr[j] == r && wi[j] < m))) {
      wr[j + 1] = wr[j];
      wi[j + 1] = wi[j];
      --j;
    }
    wr[j + 1] = r;
    wi[j + 1] = m;
  }
  for (int i = 0; i < n; ++i) {
    re[i] = wr[i];
    im[i] = wi[i];
  }
  return ok;
}

// singular values of a general n x n (row-major), descending: one-sided Jacobi
MPCEKF_HD inline bool singvals(int n, const double *A, double *sv) {
  double u[MAXN][MAXN];  // u[col][row]
  bool fin = true;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      u[j][i] = A[i * n + j];
      fin = fin && isfinite(u[j][i]);
    }
  if (!fin) {
    for (int i = 0; i < n; ++i) sv[i] = NAN;
    return false;
  }
  bool conv = false;
  for (int sweep = 0; sweep < 60 && !conv; ++sweep) {
    conv = true;
    for (int p = 0; p < n - 1; ++p)
      for (int q = p + 1; q < n; ++q) {
        double al = 0.0, be = 0.0, ga = 0.0;
        for (int i = 0; i < n; ++i) {
          al += u[p][i] * u[p][i];
          be += u[q][i] * u[q][i];
          ga += u[p][i] * u[q][i];
        }
        if (ga == 0.0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
        conv = false;
        const double ze = (be - al) / (2.0 * ga);
        const double tt = sgn(1.0, ze) / (fabs(ze) + sqrt(1.0 + ze * ze));
        const double c = 1.0 / sqrt(1.0 + tt * tt), s = c * tt;
        for (int i = 0; i < n; ++i) {
          const double up = u[p][i], uq = u[q][i];
          u[p][i] = c * up - s * uq;
          u[q][i] = s * up + c * uq;
        }
      }
  }
  for (int j = 0; j < n; ++j) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += u[j][i] * u[j][i];
    sv[j] = sqrt(s);
  }
  for (int i = 1; i < n; ++i) {
    const double v = sv[i];
    int j = i - 1;
    while (j >= 0 && sv[j] < v) {
      sv[j + 1] = sv[j];
      --j;
    }
    sv[j + 1] = v;
  }
  return conv;
}

}  // namespace eig
}  // namespace mk
