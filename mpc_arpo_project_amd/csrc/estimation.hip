// estimation.hip -- device-side unscented Kalman filter and nonlinear-plant integration (see
// include/mpcqp_estimation.h).  One thread per chaser: both are small dense fp64 recurrences
// (6-state filter, 4-state ODE) with no cross-instance work, off the QP solve's critical path.
//
// UKF: filterpy 1.4.5 UnscentedKalmanFilter.predict / update with MerweScaledSigmaPoints,
// restated (filterpy is neither vendored in the reference nor installed here):
//   sigma_points(x, P): U = cholesky_upper((lambda + n) P); chi_0 = x; chi_{k+1} = x + U[k];
//                       chi_{n+k+1} = x - U[k]
//   weights:            c = 0.5 / (n + lambda); Wm = Wc = c; Wm0 = lambda / (n + lambda);
//                       Wc0 = Wm0 + (1 - alpha^2 + beta)
//   unscented_transform: mean = Wm . chi; P = Y' diag(Wc) Y + noise  (Y = chi - mean)
//   predict(u):  chi = sigma_points(x, P); F = fx(chi, u); (x, P) = UT(F, Q);
//                sigmas_f = sigma_points(x, P)   (filterpy regenerates them after predicting)
//   update(z):   H = hx(sigmas_f); (zp, S) = UT(H, R); Pxz = sum_i Wc_i (chi_i - x)(H_i - zp)';
//                K = Pxz S^-1; x += K (z - zp); P -= K S K'
#include <hip/hip_runtime.h>

#include <cmath>

#include "../../include/mpcqp_estimation.h"
#include "plant_dev.hpp"

namespace {

using namespace mpcqp;

constexpr int UN = 6, UZ = 2, NSIG = 2 * UN + 1;

struct UkfConsts {
  double Ao[36], Bou[12], Q[36], R[4];
  double lam_n;  // lambda_ + n (sigma_points)
  double wm0, wc0, c;
};

__device__ __forceinline__ double mul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double add(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ double sub(double a, double b) { return __dsub_rn(a, b); }

// upper Cholesky factor of s * P (P's upper triangle; scipy.linalg.cholesky(lower=False))
__device__ __forceinline__ bool chol_upper(const double* P, double s, double U[UN][UN]) {
#pragma unroll
  for (int j = 0; j < UN; ++j) {
    double ajj = mul(s, P[j * UN + j]);
#pragma unroll
    for (int k = 0; k < j; ++k) ajj = sub(ajj, mul(U[k][j], U[k][j]));
    if (!(ajj > 0.0)) return false;
    const double ujj = sqrt(ajj);
    U[j][j] = ujj;
#pragma unroll
    for (int i = j + 1; i < UN; ++i) {
      double a = mul(s, P[j * UN + i]);
#pragma unroll
      for (int k = 0; k < j; ++k) a = sub(a, mul(U[k][j], U[k][i]));
      U[j][i] = __ddiv_rn(a, ujj);
    }
#pragma unroll
    for (int i = 0; i < j; ++i) U[j][i] = 0.0;
  }
  return true;
}

// sigma point i of (x, U): x, x + U[k], x - U[k]
__device__ __forceinline__ void sigma(const double x[UN], const double U[UN][UN], int i,
                                      double s[UN]) {
#pragma unroll
  for (int j = 0; j < UN; ++j) {
    double d = 0.0;
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      if (i == k + 1) d = U[k][j];
      if (i == UN + k + 1) d = -U[k][j];
    }
    s[j] = i == 0 ? x[j] : add(x[j], d);
  }
}

__device__ __forceinline__ void fx(const UkfConsts& c, const double s[UN], double u0, double u1,
                                   double f[UN]) {
#pragma unroll
  for (int r = 0; r < UN; ++r) {
    double a = 0.0;
#pragma unroll
    for (int j = 0; j < UN; ++j) a = add(a, mul(c.Ao[r * UN + j], s[j]));
    const double b = add(mul(c.Bou[r * 2], u0), mul(c.Bou[r * 2 + 1], u1));
    f[r] = add(a, b);
  }
}

__device__ __forceinline__ void hx(const double s[UN], double h[UZ]) {
  h[0] = sqrt(add(mul(s[0], s[0]), mul(s[1], s[1])));
  h[1] = atan2(s[1], s[0]);
}

__device__ __forceinline__ double wm(const UkfConsts& c, int i) { return i == 0 ? c.wm0 : c.c; }
__device__ __forceinline__ double wc(const UkfConsts& c, int i) { return i == 0 ? c.wc0 : c.c; }

__global__ void __launch_bounds__(64) ukf_step_kernel(UkfConsts c, int B, double* xg, double* Pg,
                                                      const double* ug, const double* zg,
                                                      const int32_t* active, int32_t* status) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  if (active && active[b] == 0) return;
  double x[UN], P[UN * UN], U[UN][UN];
#pragma unroll
  for (int j = 0; j < UN; ++j) x[j] = xg[(size_t)b * UN + j];
#pragma unroll
  for (int j = 0; j < UN * UN; ++j) P[j] = Pg[(size_t)b * UN * UN + j];
  const double u0 = ug[(size_t)b * 2], u1 = ug[(size_t)b * 2 + 1];
  const double z0 = zg[(size_t)b * 2], z1 = zg[(size_t)b * 2 + 1];
  bool ok = chol_upper(P, c.lam_n, U);
  // ---- predict: mean of the propagated sigma points, then their covariance (second pass)
  double xm[UN] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < NSIG; ++i) {
    double s[UN], f[UN];
    sigma(x, U, i, s);
    fx(c, s, u0, u1, f);
#pragma unroll
    for (int j = 0; j < UN; ++j) xm[j] = add(xm[j], mul(wm(c, i), f[j]));
  }
  double Pp[UN * UN];
#pragma unroll
  for (int j = 0; j < UN * UN; ++j) Pp[j] = 0.0;
  for (int i = 0; i < NSIG; ++i) {
    double s[UN], f[UN];
    sigma(x, U, i, s);
    fx(c, s, u0, u1, f);
#pragma unroll
    for (int j = 0; j < UN; ++j) f[j] = sub(f[j], xm[j]);
    const double w = wc(c, i);
#pragma unroll
    for (int a = 0; a < UN; ++a)
#pragma unroll
      for (int q = 0; q < UN; ++q) Pp[a * UN + q] = add(Pp[a * UN + q], mul(f[a], mul(w, f[q])));
  }
#pragma unroll
  for (int j = 0; j < UN * UN; ++j) Pp[j] = add(Pp[j], c.Q[j]);
  // ---- sigmas_f regenerated from the prior
  ok = ok && chol_upper(Pp, c.lam_n, U);
  // ---- update
  double zp[UZ] = {0, 0};
  for (int i = 0; i < NSIG; ++i) {
    double s[UN], h[UZ];
    sigma(xm, U, i, s);
    hx(s, h);
    zp[0] = add(zp[0], mul(wm(c, i), h[0]));
    zp[1] = add(zp[1], mul(wm(c, i), h[1]));
  }
  double S[4] = {0, 0, 0, 0}, Pxz[UN * UZ];
#pragma unroll
  for (int j = 0; j < UN * UZ; ++j) Pxz[j] = 0.0;
  for (int i = 0; i < NSIG; ++i) {
    double s[UN], h[UZ];
    sigma(xm, U, i, s);
    hx(s, h);
    const double d0 = sub(h[0], zp[0]), d1 = sub(h[1], zp[1]);
    const double w = wc(c, i);
    S[0] = add(S[0], mul(d0, mul(w, d0)));
    S[1] = add(S[1], mul(d0, mul(w, d1)));
    S[2] = add(S[2], mul(d1, mul(w, d0)));
    S[3] = add(S[3], mul(d1, mul(w, d1)));
#pragma unroll
    for (int a = 0; a < UN; ++a) {
      const double dx = sub(s[a], xm[a]);
      Pxz[a * 2] = add(Pxz[a * 2], mul(w, mul(dx, d0)));
      Pxz[a * 2 + 1] = add(Pxz[a * 2 + 1], mul(w, mul(dx, d1)));
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) S[j] = add(S[j], c.R[j]);
  // S^-1 by LU with partial pivoting (numpy.linalg.inv -> LAPACK gesv on the identity)
  double SI[4];
  {
    const bool sw = fabs(S[2]) > fabs(S[0]);
    const double a = sw ? S[2] : S[0], bq = sw ? S[3] : S[1];
    const double cq = sw ? S[0] : S[2], d = sw ? S[1] : S[3];
    const double l = __ddiv_rn(cq, a);
    const double u11 = sub(d, mul(l, bq));
    // columns of the identity, rows permuted like A
    for (int col = 0; col < 2; ++col) {
      const double e0 = (col == 0) != sw ? 1.0 : 0.0;  // (P e_col)[0]
      const double e1 = (col == 0) != sw ? 0.0 : 1.0;
      const double y1 = sub(e1, mul(l, e0));
      const double x1 = __ddiv_rn(y1, u11);
      const double x0 = __ddiv_rn(sub(e0, mul(bq, x1)), a);
      SI[col] = x0;      // SI[0][col]
      SI[2 + col] = x1;  // SI[1][col]
    }
    ok = ok && u11 != 0.0 && a != 0.0;
  }
  double K[UN * UZ];
#pragma unroll
  for (int a = 0; a < UN; ++a)
#pragma unroll
    for (int q = 0; q < UZ; ++q)
      K[a * 2 + q] = add(mul(Pxz[a * 2], SI[q]), mul(Pxz[a * 2 + 1], SI[2 + q]));
  const double y0 = sub(z0, zp[0]), y1 = sub(z1, zp[1]);
  double T[UZ * UN];  // S K'
#pragma unroll
  for (int r = 0; r < UZ; ++r)
#pragma unroll
    for (int a = 0; a < UN; ++a)
      T[r * UN + a] = add(mul(S[r * 2], K[a * 2]), mul(S[r * 2 + 1], K[a * 2 + 1]));
  const double nan = __builtin_nan("");
#pragma unroll
  for (int a = 0; a < UN; ++a) {
    const double xn = add(xm[a], add(mul(K[a * 2], y0), mul(K[a * 2 + 1], y1)));
    xg[(size_t)b * UN + a] = ok ? xn : nan;
#pragma unroll
    for (int q = 0; q < UN; ++q) {
      const double kk = add(mul(K[a * 2], T[q]), mul(K[a * 2 + 1], T[UN + q]));
      Pg[(size_t)b * UN * UN + a * UN + q] = ok ? sub(Pp[a * UN + q], kk) : nan;
    }
  }
  if (status) status[b] = ok ? 0 : 1;
}

__global__ void __launch_bounds__(64) plant_rk45_kernel(PlantConsts c, int B, double* x,
                                                        const double* u, const double* w,
                                                        double t0, double dt, int nsub,
                                                        double* traj, int32_t* failed) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double y[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = x[(size_t)b * 4 + i];
  const double u0 = u[(size_t)b * 2], u1 = u[(size_t)b * 2 + 1];
  double wv[4] = {0, 0, 0, 0};
  if (w)
#pragma unroll
    for (int i = 0; i < 4; ++i) wv[i] = w[(size_t)b * 4 + i];
  bool ok = true;
  double t = t0;
  for (int k = 0; k < nsub; ++k) {
    const double t1 = __dadd_rn(t, dt);
    ok = rk45_interval(c, t, t1, y, u0, u1) && ok;
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = __dadd_rn(y[i], wv[i]);
    if (traj)
#pragma unroll
      for (int i = 0; i < 4; ++i) traj[((size_t)b * nsub + k) * 4 + i] = y[i];
    t = t1;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) x[(size_t)b * 4 + i] = y[i];
  if (failed && !ok) failed[b] = 1;
}

}  // namespace

struct mpcqp_ukf {
  UkfConsts c;
  int B = 0;
  hipStream_t stream = nullptr;
};

extern "C" {

int mpcqp_ukf_create(const mpcqp_ukf_model* m, int32_t batch, void* stream, mpcqp_ukf** out) {
#pragma clang fp contract(off)
  if (!m || !out || batch <= 0) return -1;
  *out = nullptr;
  mpcqp_ukf* k = new mpcqp_ukf();
  for (int i = 0; i < 36; ++i) k->c.Ao[i] = m->Ao[i], k->c.Q[i] = m->Q[i];
  for (int i = 0; i < 12; ++i) k->c.Bou[i] = m->Bou[i];
  for (int i = 0; i < 4; ++i) k->c.R[i] = m->R[i];
  // MerweScaledSigmaPoints._compute_weights / sigma_points, one rounding per Python operation
  const double n = UN;
  const double a2 = m->alpha * m->alpha;  // alpha**2
  const double nk = n + m->kappa;
  const double an = a2 * nk;
  const double lam = an - n;  // lambda_
  const double lam_n = lam + n;
  const double n_lam = n + lam;
  k->c.lam_n = lam_n;
  k->c.c = 0.5 / n_lam;
  k->c.wm0 = lam / n_lam;
  const double one_a2 = 1.0 - a2;
  const double corr = one_a2 + m->beta;
  k->c.wc0 = k->c.wm0 + corr;
  k->B = batch;
  k->stream = (hipStream_t)stream;
  *out = k;
  return 0;
}

int mpcqp_ukf_destroy(mpcqp_ukf* k) {
  delete k;
  return 0;
}

int mpcqp_ukf_step(mpcqp_ukf* k, double* x, double* P, const double* u, const double* z,
                   const int32_t* active, int32_t* status) {
  if (!k || !x || !P || !u || !z) return -1;
  hipLaunchKernelGGL(ukf_step_kernel, dim3((k->B + 63) / 64), dim3(64), 0, k->stream, k->c, k->B,
                     x, P, u, z, active, status);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int mpcqp_plant_rk45(const mpcqp_plant_model* m, int32_t batch, void* stream, double* x,
                     const double* u, const double* w, double t0, double dt, int32_t nsub,
                     double* traj, int32_t* failed) {
  if (!m || !x || !u || batch <= 0 || nsub < 0 || !(dt >= 0.0)) return -1;
  if (nsub == 0) return 0;
  PlantConsts c{m->two_n, m->m_two_n, m->n2, m->R_T, m->mu, m->g0, m->rtol, m->atol};
  hipLaunchKernelGGL(plant_rk45_kernel, dim3((batch + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     c, batch, x, u, w, t0, dt, nsub, traj, failed);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
