// emulate.cpp -- host interpretation of the compiled device program (symbolic.hpp) for one
// instance: the KKT assembly, the factorization schedule with its group butterflies, the flat
// pass, the block-inverse tail and one forward / diagonal / backward solve, in the kernel's
// operation order (engine.hip: assemble_and_factor, fac_step, solve_step and the vector passes of
// the ADMM loop).  Diagnostics and tests only: it checks on the CPU that a schedule the host
// compiled (and the layout optimiser rewrote) still solves the KKT system; the product never runs
// it.  Slots nobody initialises hold NaN, so a schedule that reads a stale slot shows up as NaN.
#include <cmath>
#include <cstring>
#include <cstdint>
#include <limits>
#include <vector>

#include "symbolic.hpp"

namespace mpcqp {
namespace {

// partner lane of group-butterfly stage k (engine.hip group_sum: quad_perm xor 1 / xor 2,
// row_half_mirror, row_mirror, then xor shuffles)
int partner(int lane, int k) {
  if (k == 0) return lane ^ 1;
  if (k == 1) return lane ^ 2;
  if (k == 2) return (lane & ~7) | (7 - (lane & 7));
  if (k == 3) return (lane & ~15) | (15 - (lane & 15));
  return lane ^ (1 << k);
}

void run_fac_table(const std::vector<uint32_t>& tbl, int nsteps, std::vector<double>& v) {
  double acc[64];
  for (int s = 0; s < nsteps; ++s) {
    const uint32_t* r = tbl.data() + (size_t)s * FAC_STEP_WORDS;
    const uint32_t m0 = r[0];
    const int C = (int)((m0 >> META_C_SHIFT) & 15u), glog = (int)((m0 >> META_SGLOG_SHIFT) & 7u);
    const int nc = C <= 2 ? 2 : 4;
    for (int l = 0; l < 64; ++l) {
      double a0 = 0.0, a1 = 0.0;
      for (int c = 0; c < nc; ++c) {
        const uint32_t* q = r + 64 + c * 256 + l * 4;
        const double x = v[q[0] / 8u], y = v[q[1] / 8u], d = v[q[2] / 8u];
        if (c & 1)
          a1 = std::fma(x * y, d, a1);
        else
          a0 = std::fma(x * y, d, a0);
      }
      acc[l] = a0 + a1;
    }
    for (int k = 0; k < glog; ++k) {
      double nx[64];
      for (int l = 0; l < 64; ++l) {
        const int gl = (int)((r[l] >> META_GLOG_SHIFT) & 7u);
        nx[l] = gl > k ? acc[l] + acc[partner(l, k)] : acc[l];
      }
      for (int l = 0; l < 64; ++l) acc[l] = nx[l];
    }
    for (int l = 0; l < 64; ++l) {
      const uint32_t mt = r[l];
      if (!(mt & META_HEAD)) continue;
      const double nv = -acc[l];
      v[(mt & META_TGT_MASK) / 8u] = (mt & META_ISD) ? 1.0 / nv : nv;
    }
  }
}

void run_solve_table(const std::vector<uint32_t>& tbl, int nsteps, bool paired, std::vector<double>& v) {
  double nq[4][64];
  for (int s = 0; s < nsteps; ++s) {
    const uint32_t* r = tbl.data() + (size_t)s * SOLVE_STEP_WORDS;
    for (int q = 0; q < 4; ++q)
      for (int l = 0; l < 64; ++l) {
        const uint32_t* w = r + q * 256 + l * 4;
        const double x0 = v[w[0] / 8u], y0 = v[w[1] / 8u], x1 = v[w[2] / 8u], y1 = v[w[3] / 8u];
        nq[q][l] = std::fma(-x1, y1, -(x0 * y0));
      }
    // the ds_add_f64 instructions in issue order: paired steps sum segments 0 + 1 in registers
    // and add them to t0 (three atomics), unpaired steps add every segment to its own target
    for (int q = 0; q < 4; ++q) {
      if (paired && q == 1) continue;
      for (int l = 0; l < 64; ++l)
        v[r[SOLVE_TERM_WORDS + l * 4 + q] / 8u] += (paired && q == 0) ? nq[0][l] + nq[1][l] : nq[q][l];
    }
  }
}

}  // namespace

void emulate_factor(const Plan& pl, const double* Px, const double* Ax, double sigma,
                    const double* rho_vec, std::vector<double>& v) {
  const int n = pl.n, m = pl.m;
  v.assign((size_t)pl.LDS_N + 8, std::numeric_limits<double>::quiet_NaN());
  // assembly (engine.hip assemble_and_factor)
  for (int k = 0; k < pl.nnzL; ++k) v[pl.LX + k] = 0.0;
  for (int k = 0; k < pl.NKP; ++k) v[pl.DINV + k] = 0.0;
  for (int k = 0; k < ZERO_BLOCK; ++k) v[pl.ZERO + k] = 0.0;
  v[pl.ONE] = 1.0;
  v[pl.MONE] = -1.0;
  for (int j = 0; j < n; ++j) v[pl.slotSig[j]] = sigma;
  for (int k = 0; k < pl.nnzP; ++k) v[pl.slotP[k]] = (pl.Pi[k] == pl.Pcol[k]) ? Px[k] + sigma : Px[k];
  for (int k = 0; k < pl.nnzA; ++k) v[pl.slotA[k]] = Ax[k];
  for (int i = 0; i < m; ++i) v[pl.slotRho[i]] = -(1.0 / rho_vec[i]);
  run_fac_table(pl.fac, pl.nfac, v);
  for (int k = 0; k < pl.nnzL; ++k) v[pl.LX + k] *= v[pl.Lcol[k]];
  if (pl.ntail > 0) run_fac_table(pl.tail, pl.ntail, v);
}

bool emulate_solve(const Plan& pl, std::vector<double>& v, const double* rhs, double* sol) {
  const int n = pl.n, m = pl.m;
  // one solve (the ADMM loop's vector passes around run_body(fwd) and run_body(bwd))
  // right-hand side into C; W gets it on the copy rows and 0 elsewhere (every W slot is some
  // lane's register-slot slot)
  const int coff = pl.CACC - pl.W;
  for (int i = 0; i < 64 * pl.RN; ++i) {
    const double b = i < n ? rhs[i] : 0.0;
    v[pl.wsx[i] + coff] = b;
    v[pl.wsx[i]] = (pl.wcopy[i % 64] >> (i / 64)) & 1u ? b : 0.0;
  }
  for (int i = 0; i < 64 * pl.RM; ++i) {
    const double b = i < m ? rhs[n + i] : 0.0;
    v[pl.wsz[i] + coff] = b;
    v[pl.wsz[i]] = (pl.wcopy[i % 64] >> (pl.RN + i / 64)) & 1u ? b : 0.0;
  }
  // the solves' idle segments add -0.0 to sink slots in the 1/D region: every 1/D slot must come
  // out of the solve tables bit-identical (a non-zero "idle" product would corrupt a live 1/D_j)
  const std::vector<double> dinv(v.begin() + pl.DINV, v.begin() + pl.DINV + pl.NKP);
  auto dinv_intact = [&]() {
    return std::memcmp(dinv.data(), v.data() + pl.DINV, sizeof(double) * pl.NKP) == 0;
  };
  run_solve_table(pl.fwd, pl.nfwd, pl.paired, v);
  bool intact = dinv_intact();
  for (int k = 0; k < pl.NKP; ++k) {  // backward copy rows keep (1/D) W in W (Plan::bcopy)
    const double c = v[pl.W + k] * v[pl.DINV + k];
    v[pl.CACC + k] = c;
    v[pl.W + k] = (pl.bcopy[k % 64] >> (k / 64)) & 1u ? c : 0.0;
  }
  run_solve_table(pl.bwd, pl.nbwd, pl.paired, v);
  intact = intact && dinv_intact();
  bool finite = intact;
  for (int j = 0; j < n; ++j) sol[j] = v[pl.wsx[j]], finite = finite && std::isfinite(sol[j]);
  for (int i = 0; i < m; ++i) sol[n + i] = v[pl.wsz[i]], finite = finite && std::isfinite(sol[n + i]);
  // the padding lanes' slots read back 0 (the kernel relies on it)
  for (int i = n; i < 64 * pl.RN; ++i) finite = finite && v[pl.wsx[i]] == 0.0;
  for (int i = m; i < 64 * pl.RM; ++i) finite = finite && v[pl.wsz[i]] == 0.0;
  return finite;
}

bool emulate_kkt_solve(const Plan& pl, const double* Px, const double* Ax, double sigma,
                       const double* rho_vec, const double* rhs, double* sol) {
  std::vector<double> v;
  emulate_factor(pl, Px, Ax, sigma, rho_vec, v);
  return emulate_solve(pl, v, rhs, sol);
}

}  // namespace mpcqp
