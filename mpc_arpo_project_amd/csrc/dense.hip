// dense.hip -- MI355X (gfx950) dense-inverse engine for small QPs (n <= 128, m <= 256): device
// kernel and its launcher (called from the C ABI in engine.hip).
//
// Same algorithm and results as the KKT engine (OSQP 0.6 semantics: Ruiz scaling, rho classes,
// ADMM with alpha relaxation, unscaled termination, infeasibility tests, adaptive rho, warm
// start), with the ADMM linear system solved in reduced form (dense.hpp):
//     x~ = M^-1 (sigma x - q + A'(rho z - y)),   z~ = A x~,   M = P + sigma I + A' diag(rho) A.
// One instance per 512-thread workgroup (8 waves, 2 per SIMD), one workgroup per CU:
//   * thread t owns x_t (t < n) and constraint row t (t < m): iterates, bounds, rho, scalings
//     live in registers;
//   * -M^-1 lives in registers: wave w = h + 2c holds rows 64h..64h+63 (lane = row), columns
//     32c..32c+31, i.e. 32 doubles per thread; an ADMM mat-vec is 32 FMAs per thread against the
//     right-hand side broadcast from LDS, then the four column-group partials are added;
//   * M^-1 is formed by the symmetric sweep operator (Gauss-Jordan without pivoting on an SPD
//     matrix, result -M^-1) in the same registers: per pivot the owner half publishes the pivot
//     column to LDS, every thread updates its 64 entries; owner threads rotate their window by
//     one slot per pivot (new[s] = old[s + 1] - g col[.]) so the pivot column is always slot 0
//     and no register is indexed dynamically; after 32 pivots per group the order is restored;
//   * scaled A and P values, the A index lists and all vector exchanges live in LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mpcqp.h"
#include "dense.hpp"
#include "dense_dev.hpp"

namespace mpcqp {
namespace {

constexpr double D_INFTY = 1e30;
constexpr double D_RHO_MIN = 1e-06, D_RHO_MAX = 1e06, D_RHO_EQ = 1e03, D_RHO_TOL = 1e-04;
constexpr double D_MIN_SCALING = 1e-04, D_MAX_SCALING = 1e+04, D_DIV_TOL = 1e-30;
enum : uint32_t { DCT_INEQ = 0, DCT_EQ = 1, DCT_FREE = 2 };

struct DDev {
  const uint16_t *Ap, *Ai, *Acol, *Arp, *Ark, *Arj, *Pi, *Pcol, *Psp, *Psk, *Pso;
  const uint16_t *eptr, *ei, *ej, *ep, *ef, *tptr, *ta1, *ta2, *tr;
  const uint16_t *erp, *eri, *ecp, *eci, *lgp, *lgi;  // ELL forms (dense.hpp)
  int n, m, nnzP, nnzA, mp, nlong;
  int long_col[DENSE_NLONG], long_cnt[DENSE_NLONG];
  // LDS layout (byte offsets into the workgroup's dynamic LDS); BUF/COL/COLR (factorization) and
  // TY/R/X/PART/DT/ET/SQX (scaling and iteration vectors) share one region
  int oAv, oPv, oRHO, oERV, oECV, oLGV, oRED, oIAp, oIAi, oIArp, oIArk, oIArj, oERI, oECI, oLGI;
  int oTY, oR, oX, oPART, oDT, oET, oSQX, oBUF, oCOL, oCOLR, lds_bytes;
};

// diagnostic phase timing (-DMPCQP_TIMING builds only): thread 0 accumulates s_memtime deltas
enum { DT_SCALE, DT_FORM, DT_SWEEP, DT_RHS, DT_MATVEC, DT_ZUPD, DT_CHECK, DT_ITERS, DT_NFACT,
       DT_NSLOT };
#ifdef MPCQP_TIMING
#define DT_BEGIN(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define DT_END(slot, v) dtacc[slot] += __builtin_amdgcn_s_memtime() - (v)
#else
#define DT_BEGIN(v)
#define DT_END(slot, v)
#endif

struct DParams {
  DDev d;
  mpcqp_settings s;
  int B;
  const double *Px, *q, *Ax, *l, *u;
  double *xs, *zs, *ys, *rho_state, *Ecls;
  int32_t* has_state;
  double *x_out, *y_out;
  mpcqp_info info;
  unsigned int* counter;
  unsigned long long* timing;
};

__device__ __forceinline__ double dmx(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double dmn(double a, double b) { return a < b ? a : b; }
__device__ __forceinline__ double limit_sc(double d) {
  d = d < D_MIN_SCALING ? 1.0 : d;
  return d > D_MAX_SCALING ? D_MAX_SCALING : d;
}
template <int CTRL>
__device__ __forceinline__ double dppd(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rlane(double x, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                          __builtin_amdgcn_readlane(__double2loint(x), l));
}
__device__ __forceinline__ double wmax(double x) {
  x = dmx(x, dppd<0xB1>(x));
  x = dmx(x, dppd<0x4E>(x));
  x = dmx(x, dppd<0x141>(x));
  x = dmx(x, dppd<0x140>(x));
  return dmx(dmx(rlane(x, 0), rlane(x, 16)), dmx(rlane(x, 32), rlane(x, 48)));
}
__device__ __forceinline__ double wsum(double x) {
  x += dppd<0xB1>(x);
  x += dppd<0x4E>(x);
  x += dppd<0x141>(x);
  x += dppd<0x140>(x);
  return (rlane(x, 0) + rlane(x, 16)) + (rlane(x, 32) + rlane(x, 48));
}

// Workgroup all-reductions of K values at once (one barrier): per wave, then the 4 wave results
// combined in a fixed order, so every thread gets the bitwise-identical result.  `red` alternates
// between two buffers so that no second barrier is needed before the next reduction.
struct Red {
  double* buf;
  int phase;
};
constexpr int NWAVE = DENSE_THREADS / 64;
// after the barrier, lanes 0..NWAVE-1 of every wave pick up one wave partial each and the wave
// reduces again: every thread gets the same (deterministic) result with one register per value
template <int K>
__device__ __forceinline__ void wg_max(double (&x)[K], Red& r, int w, int lane) {
  double* b = r.buf + r.phase * NWAVE * 16;
  r.phase ^= 1;
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = wmax(x[k]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) b[w * 16 + k] = x[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = wmax(lane < NWAVE ? b[16 * lane + k] : -__builtin_inf());
}
template <int K>
__device__ __forceinline__ void wg_sum(double (&x)[K], Red& r, int w, int lane) {
  double* b = r.buf + r.phase * NWAVE * 16;
  r.phase ^= 1;
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = wsum(x[k]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) b[w * 16 + k] = x[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = wsum(lane < NWAVE ? b[16 * lane + k] : 0.0);
}

// Broadcast-operand kernels over a thread's DENSE_W-entry register row.  The operands are read
// from LDS (wave-uniform addresses: broadcast) in chunks of CH, the next chunk issued before the
// current one's FMAs (sched_group_barrier: 0x100 = DS read, 0x002 = VALU), so LDS latency overlaps
// the FMAs.  `op(s, x)` consumes operand s.
constexpr int CH = 8;
constexpr int RW = DENSE_W;
template <typename Op>
__device__ __forceinline__ void row_stream(const double* b, int count, Op op) {
  double c0[CH], c1[CH];
#pragma unroll
  for (int u = 0; u < CH; ++u) c0[u] = (u < count) ? b[u] : 0.0;
#pragma unroll
  for (int ch = 0; ch < RW / CH; ++ch) {
    double* cur = (ch & 1) ? c1 : c0;
    double* nxt = (ch & 1) ? c0 : c1;
    if (ch + 1 < RW / CH) {
#pragma unroll
      for (int u = 0; u < CH; ++u)
        if (CH * (ch + 1) + u < count) nxt[u] = b[CH * (ch + 1) + u];
      __builtin_amdgcn_sched_group_barrier(0x100, CH / 2, 0);
    }
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (CH * ch + u < count) op(CH * ch + u, cur[u]);
    __builtin_amdgcn_sched_group_barrier(0x002, CH, 0);
  }
}
// acc = sum_s M[s] * b[s]
__device__ __forceinline__ double row_dot(const double (&M)[RW], const double* b) {
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  row_stream(b, RW, [&](int s, double x) { a[s & 3] = fma(M[s], x, a[s & 3]); });
  return (a[0] + a[1]) + (a[2] + a[3]);
}
// M[s] = M[s] - g * b[s]   (non-owner sweep update)
__device__ __forceinline__ void row_axpy(double (&M)[RW], double g, const double* b) {
  row_stream(b, RW, [&](int s, double x) { M[s] = fma(-g, x, M[s]); });
}
// M[s] = M[s + 1] - g * b[s] for s < RW - 1, M[RW - 1] = last   (owner update: window rotation)
__device__ __forceinline__ void row_rot(double (&M)[RW], double g, const double* b, double last) {
  row_stream(b, RW - 1, [&](int s, double x) { M[s] = fma(-g, x, M[s + 1]); });
  M[RW - 1] = last;
}

// per-thread instance state (thread t: variable t if t < n, constraint row t if t < m)
struct TS {
  double x, q, D, Dinv;         // variable t
  double z, y, l, u, E, Einv;   // constraint t
  double rv, ri;                // rho_vec / rho_inv_vec of row t
  uint32_t ct;                  // constraint class of row t
  double c, cinv, rho;
  double pri_res, dua_res;
};

__device__ __forceinline__ void set_rho_t(TS& S) {
  const double rv_eq = D_RHO_EQ * S.rho;
  S.rv = S.rho, S.ri = 1. / S.rho;
  if (S.ct == DCT_EQ) S.rv = rv_eq, S.ri = 1. / rv_eq;
  if (S.ct == DCT_FREE) S.rv = D_RHO_MIN, S.ri = 1. / D_RHO_MIN;
}

struct Lds {
  double *Av, *Pv, *RHO, *ERV, *ECV, *LGV, *RED;
  double *TY, *R, *X, *PART, *DT, *ET, *SQX, *BUF, *COL, *COLR;
  uint16_t *Ap, *Ai, *Arp, *Ark, *Arj, *ERI, *ECI, *LGI;
};
__device__ __forceinline__ Lds lds_of(char* base, const DDev& d) {
  Lds L;
  L.Av = (double*)(base + d.oAv);
  L.Pv = (double*)(base + d.oPv);
  L.RHO = (double*)(base + d.oRHO);
  L.ERV = (double*)(base + d.oERV);
  L.ECV = (double*)(base + d.oECV);
  L.LGV = (double*)(base + d.oLGV);
  L.RED = (double*)(base + d.oRED);
  L.TY = (double*)(base + d.oTY);
  L.R = (double*)(base + d.oR);
  L.X = (double*)(base + d.oX);
  L.PART = (double*)(base + d.oPART);
  L.DT = (double*)(base + d.oDT);
  L.ET = (double*)(base + d.oET);
  L.SQX = (double*)(base + d.oSQX);
  L.BUF = (double*)(base + d.oBUF);
  L.COL = (double*)(base + d.oCOL);
  L.COLR = (double*)(base + d.oCOLR);
  L.Ap = (uint16_t*)(base + d.oIAp);
  L.Ai = (uint16_t*)(base + d.oIAi);
  L.Arp = (uint16_t*)(base + d.oIArp);
  L.Ark = (uint16_t*)(base + d.oIArk);
  L.Arj = (uint16_t*)(base + d.oIArj);
  L.ERI = (uint16_t*)(base + d.oERI);
  L.ECI = (uint16_t*)(base + d.oECI);
  L.LGI = (uint16_t*)(base + d.oLGI);
  return L;
}

// ---- ELL mat-vecs (terms in CSR / CSC order, all loads issued before the first product)
// (A x)_t for row t < m (0 beyond m)
__device__ __forceinline__ double ell_row(const DDev& d, const Lds& L, const double* x, int t) {
  if (t >= d.m) return 0.0;
  double a[DENSE_KR];
  uint32_t ix[DENSE_KR];
#pragma unroll
  for (int k = 0; k < DENSE_KR; ++k) a[k] = L.ERV[k * d.mp + t], ix[k] = L.ERI[k * d.mp + t];
  double b[DENSE_KR];
#pragma unroll
  for (int k = 0; k < DENSE_KR; ++k) b[k] = x[ix[k]];
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < DENSE_KR; ++k) s += a[k] * b[k];
  return s;
}
// out[j] = base_j + (A' y)_j for j < n (out[j] = 0 for n <= j < 128): waves 0-1 take the ELL
// columns (thread j), waves 2-3 the long columns (one per wave, summed over the wave); base_j comes
// from `base` (register, thread j) and, for long columns, from bl[j] (LDS).  Caller: barrier after.
__device__ __forceinline__ void ell_cols(const DDev& d, const Lds& L, const double* y, double base,
                                         const double* bl, double* out, int t, int w, int lane) {
  if (t < DENSE_NMAX) {
    double a[DENSE_KC];
    uint32_t ix[DENSE_KC];
#pragma unroll
    for (int k = 0; k < DENSE_KC; ++k)
      a[k] = L.ECV[k * DENSE_NMAX + t], ix[k] = L.ECI[k * DENSE_NMAX + t];
    double b[DENSE_KC];
#pragma unroll
    for (int k = 0; k < DENSE_KC; ++k) b[k] = y[ix[k]];
    double s = t < d.n ? base : 0.0;
#pragma unroll
    for (int k = 0; k < DENSE_KC; ++k) s += a[k] * b[k];
    bool is_long = false;
#pragma unroll
    for (int q = 0; q < DENSE_NLONG; ++q) is_long |= (q < d.nlong && d.long_col[q] == t);
    if (!is_long) out[t] = s;
  } else {
    const int q = w - 2;
    if (q < d.nlong) {
      double s = 0.0;
      for (int k = lane; k < d.long_cnt[q]; k += 64)
        s += L.LGV[q * DENSE_LONGK + k] * y[L.LGI[q * DENSE_LONGK + k]];
      s = wsum(s);
      if (lane == 0) out[d.long_col[q]] = bl[d.long_col[q]] + s;
    }
  }
}

// ---- Ruiz equilibration (scaling.c scale_data), exactly the KKT engine's arithmetic
__device__ void d_scale(const DParams& p, int inst, int hs, TS& S, const Lds& L, int t, int w,
                        int lane, Red& red) {
  const DDev& d = p.d;
  const int n = d.n, m = d.m;
  for (int k = t; k < d.nnzP; k += DENSE_THREADS) L.Pv[k] = p.Px[k];
  for (int k = t; k < d.nnzA; k += DENSE_THREADS) L.Av[k] = p.Ax[(size_t)inst * d.nnzA + k];
  S.q = t < n ? p.q[t] : 0.0;
  S.D = 1.0;
  S.l = t < m ? dmx(p.l[(size_t)inst * m + t], -D_INFTY) : 0.0;
  S.u = t < m ? dmn(p.u[(size_t)inst * m + t], D_INFTY) : 0.0;
  S.E = 1.0;
  S.c = 1.0;
  __syncthreads();
  for (int it = 0; it < p.s.scaling; ++it) {
    double dt = 1.0, et = 1.0;
    {
      double dd = 0.0;
      if (t < n) {
        for (int e = d.Psp[t]; e < d.Psp[t + 1]; ++e) dd = dmx(fabs(L.Pv[d.Psk[e]]), dd);
        double da = 0.0;
        for (int k = L.Ap[t]; k < L.Ap[t + 1]; ++k) da = dmx(fabs(L.Av[k]), da);
        dd = dmx(dd, da);
      }
      dd = sqrt(limit_sc(dd));
      dt = 1. / dd;
      if (t < n) L.DT[t] = dt;
    }
    {
      double e = 0.0;
      if (t < m)
        for (int q = L.Arp[t]; q < L.Arp[t + 1]; ++q) e = dmx(fabs(L.Av[L.Ark[q]]), e);
      e = sqrt(limit_sc(e));
      et = 1. / e;
      if (t < m) L.ET[t] = et;
    }
    __syncthreads();
    for (int k = t; k < d.nnzP; k += DENSE_THREADS)
      L.Pv[k] = (L.Pv[k] * L.DT[d.Pi[k]]) * L.DT[d.Pcol[k]];
    for (int k = t; k < d.nnzA; k += DENSE_THREADS)
      L.Av[k] = (L.Av[k] * L.ET[L.Ai[k]]) * L.DT[d.Acol[k]];
    S.q = dt * S.q;
    S.D = S.D * dt;
    S.E = S.E * et;
    __syncthreads();
    double cs[1] = {0.0}, qm[1] = {0.0};
    if (t < n) {
      double dd = 0.0;
      for (int e = d.Psp[t]; e < d.Psp[t + 1]; ++e) dd = dmx(fabs(L.Pv[d.Psk[e]]), dd);
      cs[0] = dd;
      qm[0] = fabs(S.q);
    }
    wg_sum(cs, red, w, lane);
    wg_max(qm, red, w, lane);
    double c_temp = cs[0] / n;
    const double inq = limit_sc(qm[0]);
    c_temp = limit_sc(dmx(c_temp, inq));
    c_temp = 1. / c_temp;
    for (int k = t; k < d.nnzP; k += DENSE_THREADS) L.Pv[k] = L.Pv[k] * c_temp;
    S.q = S.q * c_temp;
    S.c = S.c * c_temp;
    __syncthreads();
  }
  S.cinv = 1. / S.c;
  // classes on the previous equilibration's E when warm (update_bounds precedes update_A's
  // rescale in the reference call sequence), else on the new one
  const double thr = D_INFTY * D_MIN_SCALING;
  if (t < m) {
    const double ec = hs == 1 ? p.Ecls[(size_t)inst * m + t] : S.E;
    const double lc = S.l * ec, uc = S.u * ec;
    S.ct = (lc < -thr && uc > thr) ? DCT_FREE : ((uc - lc < D_RHO_TOL) ? DCT_EQ : DCT_INEQ);
    S.l = S.E * S.l;
    S.u = S.E * S.u;
  } else {
    S.ct = DCT_INEQ;
  }
  S.Einv = 1. / S.E;
  S.Dinv = 1. / S.D;
  // scaled A values into the ELL forms used by the iteration mat-vecs
  for (int k = t; k < DENSE_KR * d.mp; k += DENSE_THREADS) {
    const uint32_t q = d.erp[k];
    L.ERV[k] = q != 0xffffu ? L.Av[q] : 0.0;
  }
  for (int k = t; k < DENSE_KC * DENSE_NMAX; k += DENSE_THREADS) {
    const uint32_t q = d.ecp[k];
    L.ECV[k] = q != 0xffffu ? L.Av[q] : 0.0;
  }
  for (int k = t; k < DENSE_NLONG * DENSE_LONGK; k += DENSE_THREADS) {
    const uint32_t q = d.lgp[k];
    L.LGV[k] = q != 0xffffu ? L.Av[q] : 0.0;
  }
  __syncthreads();
}

// ---- M = P + sigma I + A' diag(rho) A, then -M^-1 by the symmetric sweep (registers)
__device__ void d_factor(const DParams& p, const TS& S, const Lds& L, double (&MR)[RW], int t,
                         int h, int c, int lane, unsigned long long* dtacc) {
  const DDev& d = p.d;
  const int row = 64 * h + lane;
  (void)dtacc;
  DT_BEGIN(t_form);
  if (t < d.m) L.RHO[t] = S.rv;
  __syncthreads();
#pragma unroll
  for (int b = 0; b < DENSE_NMAX / DENSE_BLK; ++b) {
    for (int k = t; k < DENSE_NMAX * DENSE_BLK; k += DENSE_THREADS) L.BUF[k] = 0.0;
    __syncthreads();
    for (int e = d.eptr[b] + t; e < d.eptr[b + 1]; e += DENSE_THREADS) {
      const int ep = d.ep[e], ef = d.ef[e];
      double val = ep != 0xffff ? L.Pv[ep] : 0.0;
      if (ef & 1) val += p.s.sigma;
      if (ef & 2) val = 1.0;
      for (int q = d.tptr[e]; q < d.tptr[e + 1]; ++q)
        val += (L.Av[d.ta1[q]] * L.RHO[d.tr[q]]) * L.Av[d.ta2[q]];
      L.BUF[d.ei[e] * DENSE_BLK + d.ej[e]] = val;
    }
    __syncthreads();
    if (c == b / (RW / DENSE_BLK)) {
#pragma unroll
      for (int u = 0; u < DENSE_BLK; ++u)
        MR[DENSE_BLK * (b % (RW / DENSE_BLK)) + u] = L.BUF[row * DENSE_BLK + u];
    }
    __syncthreads();
  }
  DT_END(DT_FORM, t_form);
  DT_BEGIN(t_sweep);
  // sweep pivots 0..127 (identity padding beyond n makes every group rotate exactly RW times)
  for (int k = 0; k < DENSE_NMAX; ++k) {
    const int oc = k / RW, tl = k % RW;
    double* Cb = L.COL + (k & 1) * DENSE_NMAX;
    double* CRb = L.COLR + (k & 1) * DENSE_NMAX;
    if (c == oc) {
      Cb[row] = MR[0];
      const int rr = row - RW * oc;  // rotated copy of the group's own rows
      if (rr >= 0 && rr < RW) CRb[rr] = MR[0], CRb[rr + RW] = MR[0];
    }
    __syncthreads();
    const double pk = Cb[k];
    const double piv = 1.0 / pk;
    const double f = Cb[row];
    const double g = (row == k) ? (1.0 - piv) : f * piv;
    if (c == oc)
      row_rot(MR, g, CRb + tl + 1, (row == k) ? -piv : g);
    else
      row_axpy(MR, g, Cb + RW * c);
  }
  __syncthreads();
  DT_END(DT_SWEEP, t_sweep);
  dtacc[DT_NFACT] += 1;
}

// residual vectors for the checks (scaled space): Ax (row t), Px and A'y (variable t)
struct DRes {
  double Ax, Px, Aty;
};
__device__ __forceinline__ void d_residuals(const DParams& p, TS& S, DRes& R, const Lds& L, int t,
                                            int w, int lane, Red& red) {
  const DDev& d = p.d;
  const int n = d.n, m = d.m;
  if (t < n) L.X[t] = S.x;
  if (t < m) L.TY[t] = S.y;
  if (t < DENSE_NMAX) L.SQX[t] = 0.0;
  __syncthreads();
  R.Ax = ell_row(d, L, L.X, t);
  R.Px = 0.0;
  if (t < n)
    for (int e = d.Psp[t]; e < d.Psp[t + 1]; ++e) R.Px += L.Pv[d.Psk[e]] * L.X[d.Pso[e]];
  ell_cols(d, L, L.TY, 0.0, L.SQX, L.R, t, w, lane);
  __syncthreads();
  R.Aty = t < n ? L.R[t] : 0.0;
  double v[2] = {t < m ? fabs(S.Einv * (R.Ax - S.z)) : 0.0,
                 t < n ? fabs(S.Dinv * ((S.q + R.Px) + R.Aty)) : 0.0};
  wg_max(v, red, w, lane);
  S.pri_res = v[0];
  S.dua_res = S.cinv * v[1];
}

__device__ bool d_prim_inf(const DParams& p, TS& S, double& dy, const Lds& L, int t, int w,
                           int lane, Red& red, double eps) {
  const DDev& d = p.d;
  const double thr = D_INFTY * D_MIN_SCALING;
  double a[1] = {0.0};
  if (t < d.m) {
    if (S.u > thr)
      dy = (S.l < -thr) ? 0.0 : dmn(dy, 0.0);
    else if (S.l < -thr)
      dy = dmx(dy, 0.0);
    a[0] = fabs(S.E * dy);
  }
  wg_max(a, red, w, lane);
  const double nrm = a[0];
  if (!(nrm > D_DIV_TOL)) return false;
  double s[1] = {t < d.m ? S.u * dmx(dy, 0.0) + S.l * dmn(dy, 0.0) : 0.0};
  wg_sum(s, red, w, lane);
  if (!(s[0] < eps * nrm)) return false;
  __syncthreads();  // TY / SQX / R are in use until every thread passed the last reduction
  if (t < d.m) L.TY[t] = dy;
  if (t < DENSE_NMAX) L.SQX[t] = 0.0;
  __syncthreads();
  ell_cols(d, L, L.TY, 0.0, L.SQX, L.R, t, w, lane);
  __syncthreads();
  double mx[1] = {0.0};
  if (t < d.n) mx[0] = fabs(L.R[t] * S.Dinv);
  wg_max(mx, red, w, lane);
  return mx[0] < eps * nrm;
}

__device__ bool d_dual_inf(const DParams& p, TS& S, double dx, const Lds& L, int t, int w,
                           int lane, Red& red, double eps) {
  const DDev& d = p.d;
  const double thr = D_INFTY * D_MIN_SCALING;
  double a[1] = {t < d.n ? fabs(S.D * dx) : 0.0};
  wg_max(a, red, w, lane);
  const double nrm = a[0];
  if (!(nrm > D_DIV_TOL)) return false;
  double s[1] = {t < d.n ? S.q * dx : 0.0};
  wg_sum(s, red, w, lane);
  if (!(s[0] < S.c * eps * nrm)) return false;
  __syncthreads();
  if (t < d.n) L.X[t] = dx;
  __syncthreads();
  double mx[1] = {0.0};
  if (t < d.n) {
    double acc = 0.0;
    for (int e = d.Psp[t]; e < d.Psp[t + 1]; ++e) acc += L.Pv[d.Psk[e]] * L.X[d.Pso[e]];
    mx[0] = fabs(acc * S.Dinv);
  }
  wg_max(mx, red, w, lane);
  if (!(mx[0] < S.c * eps * nrm)) return false;
  double bad[1] = {0.0};
  if (t < d.m) {
    double acc = ell_row(d, L, L.X, t);
    acc *= S.Einv;
    if ((S.u < thr && acc > eps * nrm) || (S.l > -thr && acc < -eps * nrm)) bad[0] = 1.0;
  }
  wg_max(bad, red, w, lane);
  return bad[0] == 0.0;
}

__device__ int d_check(const DParams& p, TS& S, const DRes& R, double& dy, double dx, const Lds& L,
                       int t, int w, int lane, Red& red, bool approximate) {
  const DDev& d = p.d;
  double eps_abs = p.s.eps_abs, eps_rel = p.s.eps_rel;
  double eps_pinf = p.s.eps_prim_inf, eps_dinf = p.s.eps_dual_inf;
  if (approximate) eps_abs *= 10, eps_rel *= 10, eps_pinf *= 10, eps_dinf *= 10;
  double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (t < d.m) v[0] = fabs(S.Einv * S.z), v[1] = fabs(S.Einv * R.Ax);
  if (t < d.n)
    v[2] = fabs(S.Dinv * S.q), v[3] = fabs(S.Dinv * R.Aty), v[4] = fabs(S.Dinv * R.Px);
  wg_max(v, red, w, lane);
  const double eps_prim = eps_abs + eps_rel * dmx(v[0], v[1]);
  const double eps_dual = eps_abs + eps_rel * (dmx(dmx(v[2], v[3]), v[4]) * S.cinv);
  bool prim_ok = false, dual_ok = false, prim_inf = false, dual_inf = false;
  if (S.pri_res < eps_prim)
    prim_ok = true;
  else
    prim_inf = d_prim_inf(p, S, dy, L, t, w, lane, red, eps_pinf);
  if (S.dua_res < eps_dual)
    dual_ok = true;
  else
    dual_inf = d_dual_inf(p, S, dx, L, t, w, lane, red, eps_dinf);
  if (prim_ok && dual_ok) return approximate ? MPCQP_SOLVED_INACCURATE : MPCQP_SOLVED;
  if (prim_inf) return approximate ? MPCQP_PRIMAL_INFEASIBLE_INACCURATE : MPCQP_PRIMAL_INFEASIBLE;
  if (dual_inf) return approximate ? MPCQP_DUAL_INFEASIBLE_INACCURATE : MPCQP_DUAL_INFEASIBLE;
  return 0;
}

__device__ double d_rho_estimate(const DParams& p, const TS& S, const DRes& R, int t, int w,
                                 int lane, Red& red) {
  const DDev& d = p.d;
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  if (t < d.m) v[0] = fabs(R.Ax - S.z), v[1] = fabs(S.z), v[2] = fabs(R.Ax);
  if (t < d.n)
    v[3] = fabs((S.q + R.Px) + R.Aty), v[4] = fabs(S.q), v[5] = fabs(R.Aty), v[6] = fabs(R.Px);
  wg_max(v, red, w, lane);
  const double pr = v[0] / (dmx(v[1], v[2]) + D_DIV_TOL);
  const double dr = v[3] / (dmx(dmx(v[4], v[5]), v[6]) + D_DIV_TOL);
  const double est = S.rho * sqrt(pr / (dr + D_DIV_TOL));
  return dmn(dmx(est, D_RHO_MIN), D_RHO_MAX);
}

__device__ __forceinline__ bool d_has_solution(int st) {
  return st != MPCQP_PRIMAL_INFEASIBLE && st != MPCQP_PRIMAL_INFEASIBLE_INACCURATE &&
         st != MPCQP_DUAL_INFEASIBLE && st != MPCQP_DUAL_INFEASIBLE_INACCURATE &&
         st != MPCQP_NON_CVX;
}

__device__ void d_solve_instance(const DParams& p, int inst, const Lds& L, int t, int w, int lane,
                                 Red& red) {
  const DDev& d = p.d;
  const int n = d.n, m = d.m;
  const int h = w & 1, c = w >> 1, row = 64 * h + lane;
  TS S;
  unsigned long long dtacc[DT_NSLOT] = {};
  const int hs = p.has_state[inst];
  DT_BEGIN(t_sc);
  d_scale(p, inst, hs, S, L, t, w, lane, red);
  DT_END(DT_SCALE, t_sc);
  S.rho = (hs != 0) ? p.rho_state[inst] : dmn(dmx(p.s.rho, D_RHO_MIN), D_RHO_MAX);
  set_rho_t(S);
  double MR[RW];
  d_factor(p, S, L, MR, t, h, c, lane, dtacc);

  // ---------------- warm start
  const bool warm = p.s.warm_start && hs != 0;
  S.x = 0.0, S.z = 0.0, S.y = 0.0;
  if (warm && hs == 1) {
    if (t < n) S.x = p.xs[(size_t)inst * n + t];
    if (t < m) S.z = p.zs[(size_t)inst * m + t], S.y = p.ys[(size_t)inst * m + t];
  } else if (warm && hs == 2) {  // osqp_warm_start: scale the user guess, z = A x
    if (t < n) S.x = S.Dinv * p.xs[(size_t)inst * n + t];
    if (t < m) S.y = (S.Einv * p.ys[(size_t)inst * m + t]) * S.c;
    if (t < n) L.X[t] = S.x;
    __syncthreads();
    if (t < m) S.z = ell_row(d, L, L.X, t);
    __syncthreads();
  }
  S.pri_res = S.dua_res = 0.0;

  // ---------------- ADMM (osqp.c osqp_solve)
  const double sigma = p.s.sigma, alpha = p.s.alpha;
  const int chk = p.s.check_termination;
  int ar_int = p.s.adaptive_rho_interval;
  if (p.s.adaptive_rho && ar_int == 0) ar_int = chk ? 4 * chk : 100;
  if (!p.s.adaptive_rho) ar_int = 0;
  int chk_left = chk, ar_left = ar_int;
  int status = MPCQP_UNSOLVED, iter = 0, rho_updates = 0;
  bool can_check = false;
  double dx = 0.0, dy = 0.0;
  DRes R{0.0, 0.0, 0.0};
  for (iter = 1; iter <= p.s.max_iter; ++iter) {
    dtacc[DT_ITERS] += 1;
    DT_BEGIN(t_rhs);
    const double xp = S.x, zp = S.z;
    // right-hand side r = sigma x - q + A'(rho z - y)
    const double sqx = sigma * xp - S.q;
    if (t < m) L.TY[t] = S.rv * zp - S.y;
    if (t < n) L.SQX[t] = sqx;
    __syncthreads();
    ell_cols(d, L, L.TY, sqx, L.SQX, L.R, t, w, lane);
    __syncthreads();
    DT_END(DT_RHS, t_rhs);
    DT_BEGIN(t_mv);
    // x~ = -(-M^-1) r: 64 FMAs per thread per column half, then the halves summed
    const double acc = row_dot(MR, L.R + RW * c);
    if (c != 0) L.PART[(c - 1) * DENSE_NMAX + row] = acc;
    __syncthreads();
    double xt = 0.0;
    if (c == 0) {
      double sum = acc;
#pragma unroll
      for (int q = 1; q < DENSE_CG; ++q) sum += L.PART[(q - 1) * DENSE_NMAX + row];
      xt = -sum;
      L.X[row] = xt;
    }
    __syncthreads();
    DT_END(DT_MATVEC, t_mv);
    DT_BEGIN(t_zu);
    // z~ = A x~; x, z, y updates (auxil.c update_x / update_z / update_y)
    if (t < n) {
      S.x = alpha * xt + (1.0 - alpha) * xp;
      dx = S.x - xp;
    }
    if (t < m) {
      const double zt = ell_row(d, L, L.X, t);
      const double zr = alpha * zt + (1.0 - alpha) * zp;
      S.z = dmn(dmx(zr + S.ri * S.y, S.l), S.u);
      dy = S.rv * (zr - S.z);
      S.y = S.y + dy;
    }
    DT_END(DT_ZUPD, t_zu);
    DT_BEGIN(t_ck);
    can_check = chk && --chk_left == 0;
    if (can_check) chk_left = chk;
    const bool adapt = ar_int && --ar_left == 0;
    if (adapt) ar_left = ar_int;
    if (can_check || adapt) {
      __syncthreads();  // X / TY are restaged by the residuals
      d_residuals(p, S, R, L, t, w, lane, red);
    }
    if (can_check) {
      status = d_check(p, S, R, dy, dx, L, t, w, lane, red, false);
      if (status != 0) break;
      status = MPCQP_UNSOLVED;
    }
    if (adapt) {
      const double rho_new = d_rho_estimate(p, S, R, t, w, lane, red);
      if (rho_new > S.rho * p.s.adaptive_rho_tolerance ||
          rho_new < S.rho / p.s.adaptive_rho_tolerance) {
        S.rho = dmn(dmx(rho_new, D_RHO_MIN), D_RHO_MAX);
        set_rho_t(S);
        rho_updates++;
        __syncthreads();
        d_factor(p, S, L, MR, t, h, c, lane, dtacc);
      }
    }
    __syncthreads();  // LDS vectors are rewritten by the next iteration
    DT_END(DT_CHECK, t_ck);
  }
  if (!can_check) {
    iter = iter - 1;
    __syncthreads();
    d_residuals(p, S, R, L, t, w, lane, red);
    status = d_check(p, S, R, dy, dx, L, t, w, lane, red, false);
    if (status == 0) status = MPCQP_UNSOLVED;
  }
  if (iter > p.s.max_iter) iter = p.s.max_iter;
  if (status == MPCQP_UNSOLVED) {
    const int st = d_check(p, S, R, dy, dx, L, t, w, lane, red, true);
    status = st ? st : MPCQP_MAX_ITER_REACHED;
  }
  // ---------------- objective (compute_obj_val) and store_solution
  const bool sol = d_has_solution(status);
  double obj = 0.0;
  if (sol) {
    __syncthreads();
    if (t < n) L.X[t] = S.x;
    __syncthreads();
    double part[1] = {0.0};
    for (int k = t; k < d.nnzP; k += DENSE_THREADS) {
      const int i = d.Pi[k], j = d.Pcol[k];
      part[0] += (i == j) ? .5 * L.Pv[k] * L.X[i] * L.X[i] : L.Pv[k] * L.X[i] * L.X[j];
    }
    if (t < n) part[0] += S.q * S.x;
    wg_sum(part, red, w, lane);
    obj = part[0] * S.cinv;
  } else if (status == MPCQP_PRIMAL_INFEASIBLE || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE) {
    obj = D_INFTY;
  } else if (status == MPCQP_DUAL_INFEASIBLE || status == MPCQP_DUAL_INFEASIBLE_INACCURATE) {
    obj = -D_INFTY;
  }
  const double qnan = __builtin_nan("");
  if (t < n) {
    if (p.x_out) p.x_out[(size_t)inst * n + t] = sol ? S.D * S.x : qnan;
    p.xs[(size_t)inst * n + t] = sol ? S.x : 0.0;
  }
  if (t < m) {
    if (p.y_out) p.y_out[(size_t)inst * m + t] = sol ? (S.E * S.y) * S.cinv : qnan;
    p.zs[(size_t)inst * m + t] = sol ? S.z : 0.0;
    p.ys[(size_t)inst * m + t] = sol ? S.y : 0.0;
    p.Ecls[(size_t)inst * m + t] = S.E;
  }
#ifdef MPCQP_TIMING
  if (t == 0 && p.timing)
    for (int k = 0; k < DT_NSLOT; ++k) atomicAdd(p.timing + k, dtacc[k]);
#endif
  if (t == 0) {
    p.rho_state[inst] = S.rho;
    p.has_state[inst] = 1;
    if (p.info.status) p.info.status[inst] = status;
    if (p.info.iter) p.info.iter[inst] = iter;
    if (p.info.rho_updates) p.info.rho_updates[inst] = rho_updates;
    if (p.info.obj_val) p.info.obj_val[inst] = obj;
    if (p.info.pri_res) p.info.pri_res[inst] = S.pri_res;
    if (p.info.dua_res) p.info.dua_res[inst] = S.dua_res;
    if (p.info.rho) p.info.rho[inst] = S.rho;
  }
}

// one instance per workgroup, persistent: instances are pulled from an atomic counter
__global__ void __launch_bounds__(DENSE_THREADS) qp_dense_kernel(DParams p) {
  extern __shared__ __attribute__((aligned(16))) char dlds[];
  const int t = (int)threadIdx.x, w = t >> 6, lane = t & 63;
  const Lds L = lds_of(dlds, p.d);
  // problem-constant index lists, once per workgroup
  for (int k = t; k <= p.d.n; k += DENSE_THREADS) L.Ap[k] = p.d.Ap[k];
  for (int k = t; k <= p.d.m; k += DENSE_THREADS) L.Arp[k] = p.d.Arp[k];
  for (int k = t; k < p.d.nnzA; k += DENSE_THREADS)
    L.Ai[k] = p.d.Ai[k], L.Ark[k] = p.d.Ark[k], L.Arj[k] = p.d.Arj[k];
  for (int k = t; k < DENSE_KR * p.d.mp; k += DENSE_THREADS) L.ERI[k] = p.d.eri[k];
  for (int k = t; k < DENSE_KC * DENSE_NMAX; k += DENSE_THREADS) L.ECI[k] = p.d.eci[k];
  for (int k = t; k < DENSE_NLONG * DENSE_LONGK; k += DENSE_THREADS) L.LGI[k] = p.d.lgi[k];
  Red red{L.RED, 0};
  __shared__ unsigned int s_inst;
  for (;;) {
    __syncthreads();
    if (t == 0) s_inst = atomicAdd(p.counter, 1u);
    __syncthreads();
    const unsigned int inst = __builtin_amdgcn_readfirstlane(s_inst);
    if (inst >= (unsigned int)p.B) break;
    d_solve_instance(p, (int)inst, L, t, w, lane, red);
  }
}

template <typename T>
size_t push(std::vector<char>& blob, const std::vector<T>& v) {
  size_t off = (blob.size() + 15) & ~size_t(15);
  blob.resize(off + v.size() * sizeof(T) + 16);
  if (!v.empty()) memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
  return off;
}

}  // namespace

struct DenseEngine {
  DensePlan plan;
  char* d_blob = nullptr;
  DDev dd{};
  int grid = 0, lds_bytes = 0, per_cu = 0;
};

int dense_create(const DenseInputs& in, DenseEngine** out, std::string& err) {
  *out = nullptr;
  DenseEngine* e = new DenseEngine();
  if (!build_dense_plan(in.n, in.m, in.Pp, in.Pi, in.Ap, in.Ai, e->plan)) {
    err = e->plan.error;
    delete e;
    return MPCQP_E_UNSUPPORTED;
  }
  const DensePlan& pl = e->plan;
  std::vector<char> blob;
  const size_t oAp = push(blob, pl.Ap), oAi = push(blob, pl.Ai), oAc = push(blob, pl.Acol),
               oArp = push(blob, pl.Arp), oArk = push(blob, pl.Ark), oArj = push(blob, pl.Arj),
               oPi = push(blob, pl.Pi), oPc = push(blob, pl.Pcol), oPsp = push(blob, pl.Psp),
               oPsk = push(blob, pl.Psk), oPso = push(blob, pl.Pso), oep = push(blob, pl.eptr),
               oei = push(blob, pl.ei), oej = push(blob, pl.ej), oepp = push(blob, pl.ep),
               oef = push(blob, pl.ef), otp = push(blob, pl.tptr), ot1 = push(blob, pl.ta1),
               ot2 = push(blob, pl.ta2), otr = push(blob, pl.tr), oerp = push(blob, pl.erp),
               oeri = push(blob, pl.eri), oecp = push(blob, pl.ecp), oeci = push(blob, pl.eci),
               olgp = push(blob, pl.lgp), olgi = push(blob, pl.lgi);
  if (hipMalloc(&e->d_blob, blob.size()) != hipSuccess ||
      hipMemcpy(e->d_blob, blob.data(), blob.size(), hipMemcpyHostToDevice) != hipSuccess) {
    err = "dense engine: structure upload failed";
    dense_destroy(e);
    return MPCQP_E_HIP;
  }
  const char* b = e->d_blob;
  DDev& d = e->dd;
  d.Ap = (const uint16_t*)(b + oAp), d.Ai = (const uint16_t*)(b + oAi);
  d.Acol = (const uint16_t*)(b + oAc), d.Arp = (const uint16_t*)(b + oArp);
  d.Ark = (const uint16_t*)(b + oArk), d.Arj = (const uint16_t*)(b + oArj);
  d.Pi = (const uint16_t*)(b + oPi), d.Pcol = (const uint16_t*)(b + oPc);
  d.Psp = (const uint16_t*)(b + oPsp), d.Psk = (const uint16_t*)(b + oPsk);
  d.Pso = (const uint16_t*)(b + oPso), d.eptr = (const uint16_t*)(b + oep);
  d.ei = (const uint16_t*)(b + oei), d.ej = (const uint16_t*)(b + oej);
  d.ep = (const uint16_t*)(b + oepp), d.ef = (const uint16_t*)(b + oef);
  d.tptr = (const uint16_t*)(b + otp), d.ta1 = (const uint16_t*)(b + ot1);
  d.ta2 = (const uint16_t*)(b + ot2), d.tr = (const uint16_t*)(b + otr);
  d.erp = (const uint16_t*)(b + oerp), d.eri = (const uint16_t*)(b + oeri);
  d.ecp = (const uint16_t*)(b + oecp), d.eci = (const uint16_t*)(b + oeci);
  d.lgp = (const uint16_t*)(b + olgp), d.lgi = (const uint16_t*)(b + olgi);
  d.n = pl.n, d.m = pl.m, d.nnzP = pl.nnzP, d.nnzA = pl.nnzA, d.mp = pl.mp, d.nlong = pl.nlong;
  for (int q = 0; q < DENSE_NLONG; ++q) d.long_col[q] = pl.long_col[q], d.long_cnt[q] = pl.long_cnt[q];
  // LDS layout
  int off = 0;
  auto take = [&](int bytes) {
    const int o = off;
    off = (off + bytes + 15) & ~15;
    return o;
  };
  d.oAv = take(8 * pl.nnzA);
  d.oPv = take(8 * pl.nnzP);
  d.oRHO = take(8 * DENSE_MMAX);
  d.oERV = take(8 * DENSE_KR * pl.mp);
  d.oECV = take(8 * DENSE_KC * DENSE_NMAX);
  d.oLGV = take(8 * DENSE_NLONG * DENSE_LONGK);
  d.oRED = take(8 * 2 * NWAVE * 16);
  d.oIAp = take(2 * (pl.n + 1));
  d.oIAi = take(2 * pl.nnzA);
  d.oIArp = take(2 * (pl.m + 1));
  d.oIArk = take(2 * pl.nnzA);
  d.oIArj = take(2 * pl.nnzA);
  d.oERI = take(2 * DENSE_KR * pl.mp);
  d.oECI = take(2 * DENSE_KC * DENSE_NMAX);
  d.oLGI = take(2 * DENSE_NLONG * DENSE_LONGK);
  const int ubase = off;  // shared region
  d.oTY = take(8 * DENSE_MMAX);
  d.oR = take(8 * DENSE_NMAX);
  d.oX = take(8 * DENSE_NMAX);
  d.oPART = take(8 * (DENSE_CG - 1) * DENSE_NMAX);
  d.oDT = take(8 * DENSE_NMAX);
  d.oET = take(8 * DENSE_MMAX);
  d.oSQX = take(8 * DENSE_NMAX);
  const int uvec = off;
  off = ubase;
  d.oBUF = take(8 * DENSE_NMAX * DENSE_BLK);
  d.oCOL = take(8 * 2 * DENSE_NMAX);
  d.oCOLR = take(8 * 2 * DENSE_NMAX);
  off = std::max(off, uvec);
  d.lds_bytes = off;
  e->lds_bytes = off;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    err = "dense engine: device query failed";
    dense_destroy(e);
    return MPCQP_E_HIP;
  }
  if (hipFuncSetAttribute((const void*)qp_dense_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          e->lds_bytes) != hipSuccess) {
    err = "dense engine: hipFuncSetAttribute failed";
    dense_destroy(e);
    return MPCQP_E_HIP;
  }
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)qp_dense_kernel,
                                                   DENSE_THREADS, e->lds_bytes) != hipSuccess ||
      nb <= 0) {
    err = "dense engine: kernel does not fit on a CU";
    dense_destroy(e);
    return MPCQP_E_UNSUPPORTED;
  }
  e->per_cu = nb;
  e->grid = std::min(in.batch, nb * ncu);
  *out = e;
  return 0;
}

void dense_destroy(DenseEngine* e) {
  if (!e) return;
  if (e->d_blob) (void)hipFree(e->d_blob);
  delete e;
}

int dense_solve(DenseEngine* e, const DenseSolveArgs& a, hipStream_t stream) {
  DParams p{};
  p.d = e->dd;
  p.s = a.s;
  p.B = a.B;
  p.Px = a.Px, p.q = a.q, p.Ax = a.Ax, p.l = a.l, p.u = a.u;
  p.xs = a.xs, p.zs = a.zs, p.ys = a.ys, p.rho_state = a.rho_state, p.Ecls = a.Ecls;
  p.has_state = a.has_state;
  p.x_out = a.x_out, p.y_out = a.y_out;
  p.info = a.info;
  p.counter = a.counter;
  p.timing = a.timing;
  hipLaunchKernelGGL(qp_dense_kernel, dim3(e->grid), dim3(DENSE_THREADS), e->lds_bytes, stream, p);
  return hipGetLastError() == hipSuccess ? 0 : MPCQP_E_HIP;
}

void dense_info(const DenseEngine* e, int* grid, int* lds_bytes, int* per_cu) {
  if (grid) *grid = e->grid;
  if (lds_bytes) *lds_bytes = e->lds_bytes;
  if (per_cu) *per_cu = e->per_cu;
}

}  // namespace mpcqp
