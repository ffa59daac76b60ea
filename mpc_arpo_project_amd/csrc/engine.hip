// engine.hip -- MI355X (gfx950) batched OSQP-semantics QP engine: device kernel + C ABI.
//
// Design (DESIGN.md has the long form):
//   * one QP instance per wavefront (64 lanes, one wave per workgroup), persistent grid sized to
//     the resident-wave capacity; waves pull instance ids from an atomic work counter, so the
//     heavy-tailed ADMM iteration counts balance themselves;
//   * the instance's image lives in LDS (39.9 KB at N = 20): the KKT factor L, 1/D, the block
//     inverses of the blocked substitution, the solve vector and the scaled matrix values; the
//     primal/dual iterates, bounds and inverse scalings live in VGPRs (element i on lane i % 64,
//     slot i / 64); a per-wave slab in global memory keeps the scalings D, E;
//   * numeric factorization and both triangular solves are driven by host-compiled step
//     schedules (symbolic.hpp): each step is a 64-lane pass of LDS reads, FMAs and LDS atomics;
//   * wave reductions end with the gfx950 lane swaps (v_permlane16/32_swap), not readlanes;
//   * arithmetic is fp64 throughout and follows OSQP 0.6's algorithm (Ruiz scaling, rho classes,
//     ADMM with alpha relaxation, unscaled termination + infeasibility tests, adaptive rho).
//
// Reference boundary replaced: osqp.OSQP setup/update/solve as called at
// reference src/trajectorySimulate.py:242-348 (see include/mpcqp.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mpcqp.h"
#include "host_abi.hpp"
#include "symbolic.hpp"

using namespace mpcqp;

// OSQP's arithmetic in the data scaling and the checks: no FMA contraction (hipcc contracts
// a * b + c by default; OSQP 0.6 as the reference's wheel and the oracle evaluate every product and
// sum with its own rounding), so the Ruiz passes, the carried data drift, the residual mat-vecs,
// the termination tests, the rho estimate and the certificates round exactly as OSQP's
// (tests/test_gpu_scaling_parity.py: bitwise).  Explicit fma() remains where the engine's rounding
// differs from OSQP's anyway -- the factorization, the triangular solves (their own summation
// orders) and the per-iteration right-hand side and x / z / y updates around them (one rounding
// fewer per update; unfused they cost 1.1 % of the headline, DESIGN.md Parity).
#pragma clang fp contract(off)

#define OSQP_INFTY 1e30
#define RHO_MIN 1e-06
#define RHO_MAX 1e06
#define RHO_EQ_OVER_RHO_INEQ 1e03
#define RHO_TOL 1e-04
#define MIN_SCALING 1e-04
#define MAX_SCALING 1e+04
#define DIVISION_TOL 1e-30

namespace {

// ------------------------------------------------------------------------------------- device
struct EllDev {
  const uint16_t *src, *in, *vpos, *sk;
  const uint32_t* pk;  // lane-major packed (vpos, in) terms of the used slots (symbolic.hpp Ell::pk)
  int K[ELL_MAXR], off[ELL_MAXR];
  int total, nlong;
  int long_out[ELL_MAXLONG], long_off[ELL_MAXLONG], long_cnt[ELL_MAXLONG];
};
struct DevPlan {
  EllDev eA, eAt, eP;  // residual mat-vecs (symbolic.hpp Ell)
  const uint32_t *fac, *tail, *fwd, *bwd;  // fixed-stride step records (symbolic.hpp)
  // KM_MREG kernels: the solve records split into vector-operand + target records (fwdc, bwdc) and
  // the matrix operands' LDS addresses (fwdm, bwdm), built on the host (mpcqp_create)
  const uint32_t *fwdc, *bwdc, *fwdm, *bwdm;
  int nfac, ntail, nfwd, nbwd;
  const uint16_t* Lcol;    // DINV slot of each L entry's column
  int inst_doubles;        // LDS doubles of the instance image (16-byte aligned)
  const uint16_t *slotP, *slotA, *slotRho, *slotSig, *wsx, *wsz;
  const uint16_t *Ap, *Ai, *Acol, *Arp, *Ark, *Arj, *Pi, *Pcol, *Psp, *Psk, *Pso;
  int n, m, nk, nnzP, nnzA, nnzL;
  int LX, DINV, W, CACC, ZERO, ONE, MONE, LDS_N, S_P, S_A, S_DT, S_ET;
  int NKS;  // 64-lane slots of the padded 1/D, W and C regions (symbolic.hpp NKP / 64 = RN + RM)
  const uint32_t* wcopy;  // per lane: register slots whose W starts at the rhs (symbolic.hpp Plan::wcopy)
  const uint32_t* bcopy;  // per lane: diagonal-pass slots whose W starts at (1/D) W (Plan::bcopy)
  int S_ZERO;
  int MV, MVZ;  // resident scaled values [P | A] (CSC orders) and their zero slot
  int mv_slab;  // doubles of the per-wave slab holding them instead (Plan::mv_global), else 0
  const uint16_t *sra, *sca;  // lane-major row / column scaling slots (symbolic.hpp Plan::sra)
  int SJ;
  int XCH, XID;  // two-wave kernel: exchange slots and the handed-over instance id (Plan::XCH)
};

struct KParams {
  DevPlan pl;
  mpcqp_settings s;
  int B;
  const double *Px, *q;      // shared
  const double *Ax, *l, *u;  // [B][nnzA], [B][m]
  // warm-start state carried between solves (OSQP keeps it inside the workspace)
  double *xs, *zs, *ys, *rho_state, *Ecls;  // scaled iterates, rho, E of the previous scaling
  int32_t* has_state;                        // 0 none, 1 scaled iterates, 2 unscaled guess
  double *x_out, *y_out;
  mpcqp_info info;
  // OSQP 0.6's data drift (osqp_update_A: unscale_data, overwrite A, scale_data): per instance the
  // unscaled P values and q that the next solve rescales -- (P_s c^-1) D^-1 D^-1 and (q_s c^-1) D^-1
  // of this solve's scaling, so a warm solve starts its Ruiz passes from the same rounded data as
  // OSQP does (set_data / update_lin_cost write the plain P / q into every instance)
  // Two buffers each ([2][B][nnzP], [2][B][n]), selected per instance by dsel (drift_of): the input
  // of the instance's last scaling is kept beside its unscaled output, because a solve after a
  // bounds-only update (osqp_update_bounds) keeps OSQP's previous scaling -- it re-runs the Ruiz
  // passes on that same input (bitwise the same D, E, c) -- while a solve after an update of A
  // (osqp_update_A) rescales the unscaled output.
  double *Pw, *qw;
  int32_t* dsel;  // [B] -2 never scaled, -1 last scaled from the shared set-up data, 0 / 1 buffer
  int32_t* pend;  // [B] A updated since the instance's last solve (mpcqp_update_A)
  int a_inplace;  // mpcqp_data_buffers handed out the A buffer: every solve follows an update of A
  double* scratch;  // [grid][nnzP + nnzA] scaled P and A values of the wave's current instance
  unsigned int* counter;
  unsigned long long* timing;  // diagnostic builds only (MPCQP_TIMING): cycles per phase
  // initial rho of a cold instance, min(max(settings.rho, RHO_MIN), RHO_MAX), computed on the host:
  // read per instance from the kernel arguments instead of a loop-invariant register (the gfx950
  // backend of ROCm 7.2 was seen to spill such a hoisted double and reload only its low half)
  double rho0;
  const int32_t* skip;  // [B] or null: instances with skip[i] != 0 are not solved (outputs kept)
  const int32_t* order;  // [B] or null: the k-th instance handed out is order[k] (mpcqp_set_order)
};

// Where a solve's Ruiz passes start and where the data they leave for the next solve goes (OSQP
// 0.6's data drift, KParams::Pw).  Wave-uniform.  drift_sel: the buffer indices; drift_of: the
// pointers formed from them at the solve's start (one-wave kernel).  The two-wave kernel forms the
// pointers at their two uses instead: measured per kernel, each form is 1.5-1.9 % faster in its own
// kernel (register allocation).
struct DriftSel {
  int in_b, out_b;  // drift buffer the Ruiz passes scale (-1: the shared set-up data) / unscale into
  bool rebound;     // bounds through E_old, E_old^-1, E_new (osqp_update_A after update_bounds)
  int sel;          // dsel after this solve
};
__device__ __forceinline__ DriftSel drift_sel(const KParams& p, int inst) {
  const int sel = __builtin_amdgcn_readfirstlane(p.dsel[inst]);
  const bool dirty = p.a_inplace != 0 || __builtin_amdgcn_readfirstlane(p.pend[inst]) != 0;
  DriftSel d;
  if (sel == -2) {  // first solve after set_data: scale_data of the set-up data (osqp_setup)
    d.in_b = -1, d.out_b = 0, d.rebound = false, d.sel = -1;
  } else if (dirty) {  // osqp_update_A: unscale_data of the last scaling, then scale_data
    const int ub = sel == 0 ? 1 : 0;
    d.in_b = ub, d.out_b = 1 - ub, d.rebound = true, d.sel = ub;
  } else {  // bounds only: the last scaling again (same input, same D, E, c)
    d.in_b = sel, d.out_b = sel == 0 ? 1 : 0, d.rebound = false, d.sel = sel;
  }
  return d;
}
// the drift buffers' rows of instance inst: P values (cnt = nnzP, base p.Pw) or q (n, p.qw)
__device__ __forceinline__ double* drift_row(double* base, int b, int B, int cnt, int inst) {
  return base + ((size_t)b * B + inst) * cnt;
}
struct Drift {
  const double *P_in, *q_in;  // the unscaled P values / q the Ruiz passes scale
  double *P_out, *q_out;      // unscale_data of this solve's scaled P / q
  bool rebound;               // bounds through E_old, E_old^-1, E_new (osqp_update_A after update_bounds)
  int sel;                    // dsel after this solve
};
__device__ __forceinline__ Drift drift_of(const KParams& p, int inst) {
  const int nP = p.pl.nnzP, n = p.pl.n;
  const int sel = __builtin_amdgcn_readfirstlane(p.dsel[inst]);
  const bool dirty = p.a_inplace != 0 || __builtin_amdgcn_readfirstlane(p.pend[inst]) != 0;
  int in_b, out_b;  // -1: the shared set-up data
  Drift d;
  if (sel == -2) {  // first solve after set_data: scale_data of the set-up data (osqp_setup)
    in_b = -1, out_b = 0, d.rebound = false, d.sel = -1;
  } else if (dirty) {  // osqp_update_A: unscale_data of the last scaling, then scale_data
    const int ub = sel == 0 ? 1 : 0;
    in_b = ub, out_b = 1 - ub, d.rebound = true, d.sel = ub;
  } else {  // bounds only: the last scaling again (same input, same D, E, c)
    in_b = sel, out_b = sel == 0 ? 1 : 0, d.rebound = false, d.sel = sel;
  }
  const size_t BP = (size_t)p.B * nP, Bq = (size_t)p.B * n;
  d.P_in = in_b < 0 ? p.Px : p.Pw + in_b * BP + (size_t)inst * nP;
  d.q_in = in_b < 0 ? p.q : p.qw + in_b * Bq + (size_t)inst * n;
  d.P_out = p.Pw + out_b * BP + (size_t)inst * nP;
  d.q_out = p.qw + out_b * Bq + (size_t)inst * n;
  return d;
}

// Diagnostic phase timing (-DMPCQP_TIMING builds, tools/phase_timing.py; never the product build):
// s_memtime deltas accumulated per wave in SGPRs, added to p.timing at the end of each instance.
enum { T_SCALE, T_FACTOR, T_FWD, T_BWD, T_VEC, T_CHECK, T_TAIL, T_ITERS, T_NFACT, T_RESID, T_TERM, T_NCHK, T_ADAPT, T_SCFIN, T_V0, T_V1, T_V2, T_RS0, T_RS1, T_RS2, T_RS3, T_RS4, T_TM0, T_TM1, T_TM2, T_SC0, T_SC1, T_SC2, T_SC3, T_SCC, T_NSLOT };
#ifdef MPCQP_TIMING
#define T_BEGIN(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define T_END(slot, v) tacc[slot] += __builtin_amdgcn_s_memtime() - (v)
#define T_COUNT(slot) tacc[slot] += 1
// value dependency barrier: the timestamp after it waits for x
#define TSYNC(x) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::"v"(x))
#else
#define T_BEGIN(v)
#define T_END(slot, v)
#define T_COUNT(slot)
#define TSYNC(x)
#endif

// Ordering between dependent wave-synchronous LDS phases.  A wave's LDS instructions are executed
// in issue order, so a ds_read issued after a ds_write observes it; only the compiler has to be
// stopped from reordering the memory operations (no hardware wait is needed).
#define LDS_FENCE() asm volatile("" ::: "memory")

__device__ __forceinline__ double dmaxd(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double dmind(double a, double b) { return a < b ? a : b; }

template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
// gfx950 v_permlane16_swap / v_permlane32_swap with x as both operands: (a, b) = (x of rows 0, 0,
// 2, 2 | x of rows 1, 1, 3, 3), resp. (x of lanes 0-31 twice | x of lanes 32-63 twice)
__device__ __forceinline__ void swap16_d(double x, double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(x), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(x), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap32_d(double x, double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(x), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(x), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ double uniform_d(double x) {
  return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(x)),
                          __builtin_amdgcn_readfirstlane(__double2loint(x)));
}
// Wave all-reductions: DPP butterflies inside each 16-lane row (partners exchange and combine the
// same two operands, so every lane of a row holds the bitwise-identical row result), then the row
// results r0..r3 combined by the two lane swaps as (r0 + r1) + (r2 + r3) in every lane (max:
// order-free) and made wave-uniform.  The swaps replace four readlane pairs per reduction, a
// latency chain through the SGPRs (measured: 918k vs 905k solves/s).
template <bool SUM>
__device__ __forceinline__ double wave_all(double x) {
  auto op = [](double p, double q) { return SUM ? p + q : dmaxd(p, q); };
  x = op(x, dpp_d<0xB1>(x));   // quad_perm [1,0,3,2]
  x = op(x, dpp_d<0x4E>(x));   // quad_perm [2,3,0,1]
  x = op(x, dpp_d<0x141>(x));  // row_half_mirror
  x = op(x, dpp_d<0x140>(x));  // row_mirror
  double a, b;
  swap16_d(x, a, b);
  swap32_d(op(a, b), a, b);
  return uniform_d(op(a, b));
}
__device__ __forceinline__ double wave_max(double x) { return wave_all<false>(x); }
__device__ __forceinline__ double wave_sum(double x) { return wave_all<true>(x); }
// OSQP's sequential sums (lin_alg.c vec_mean / vec_prod, the primal certificate's lhs loop,
// mat_vec's accumulation into one output): s = ((0 + t_0) + t_1) + ... in index order, the
// rounding a tree reduction does not reproduce.  The caller stages t_k at buf[k] in LDS; every lane
// runs the same chain over uniform reads (8 in flight), so the result is wave-uniform.
__device__ __forceinline__ double seq_sum(const double* buf, int cnt) {
  double s = 0.0;
  int k = 0;
  for (; k + 8 <= cnt; k += 8) {  // scalars, not an array (an array here went to scratch)
    const double t0 = buf[k], t1 = buf[k + 1], t2 = buf[k + 2], t3 = buf[k + 3];
    const double t4 = buf[k + 4], t5 = buf[k + 5], t6 = buf[k + 6], t7 = buf[k + 7];
    s = s + t0, s = s + t1, s = s + t2, s = s + t3;
    s = s + t4, s = s + t5, s = s + t6, s = s + t7;
  }
  for (; k < cnt; ++k) s = s + buf[k];
  return s;
}
// two of them at once (independent chains: each add waits for its own chain only), a[0..ca) and
// b[0..cb): bitwise seq_sum(a, ca) and seq_sum(b, cb)
__device__ __forceinline__ void seq_sum2(const double* a, int ca, const double* b, int cb, double& sa,
                                         double& sb) {
  double x = 0.0, y = 0.0;
  const int c = ca < cb ? ca : cb;
  int k = 0;
  for (; k + 4 <= c; k += 4) {
    const double a0 = a[k], a1 = a[k + 1], a2 = a[k + 2], a3 = a[k + 3];
    const double b0 = b[k], b1 = b[k + 1], b2 = b[k + 2], b3 = b[k + 3];
    x = x + a0, y = y + b0, x = x + a1, y = y + b1;
    x = x + a2, y = y + b2, x = x + a3, y = y + b3;
  }
  for (; k < c; ++k) x = x + a[k], y = y + b[k];
  for (int j = k; j < ca; ++j) x = x + a[j];
  for (int j = k; j < cb; ++j) y = y + b[j];
  sa = x, sb = y;
}
// The decision x < thr on OSQP's sequential sum x of cnt staged terms, exactly, without the
// sequential chain in the common case: a tree sum T of the same terms differs from the sequential
// one by at most (gamma_{cnt-1} + gamma_{ceil log2 cnt}) sum |t| (Higham, Accuracy and Stability of
// Numerical Algorithms, 4.2), so when T is farther than a generous bound from thr the sequential
// sum lies on the same side; only a near-tie runs seq_sum.  T, A = the wave's tree sums of t, |t|.
__device__ __forceinline__ double sum_slack(double A, int cnt) {
  return (8.0 * cnt) * (0x1p-53 * A) + 0x1p-1060 * cnt;
}
__device__ __forceinline__ bool seq_sum_lt(const double* buf, int cnt, double T, double A, double thr) {
  const double b = sum_slack(A, cnt);
  if (T + b < thr) return true;
  if (T - b >= thr) return false;
  LDS_FENCE();
  const bool lt = seq_sum(buf, cnt) < thr;
  LDS_FENCE();
  return lt;
}
__device__ __forceinline__ double limit_scaling(double d) {
  d = d < MIN_SCALING ? 1.0 : d;
  return d > MAX_SCALING ? MAX_SCALING : d;
}

// ---- level-scheduled dot-product steps (see symbolic.hpp) ---------------------------------
// The instance image starts at LDS address 0 (one wave per workgroup, no static LDS), so the
// schedule records hold absolute LDS byte addresses and an operand fetch is a bare ds_read.
typedef __attribute__((address_space(3))) double lds_double;
__device__ __forceinline__ double lds_ld(const double*, uint32_t a) {
  return *(const lds_double*)(size_t)a;
}
__device__ __forceinline__ void lds_st(double*, uint32_t a, double x) { *(lds_double*)(size_t)a = x; }

// Group butterflies: DPP inside rows of 16 lanes (quad_perm xor 1, xor 2, row_half_mirror,
// row_mirror pair the partners of an aligned group exactly like an xor butterfly does for an
// all-reduce), the gfx950 lane swaps beyond that (xor 16, xor 32; no LDS round trip).
// all-reduce of acc over this lane's aligned group of 2^gl lanes (glog = widest group of the step,
// wave-uniform); stages beyond the step's widest group are skipped by uniform branches
__device__ __forceinline__ double group_sum(double acc, uint32_t glog, uint32_t gl) {
  if (glog > 0) {
    const bool g0 = gl > 0, g1 = gl > 1, g2 = gl > 2;
    const double o = dpp_d<0xB1>(acc);  // quad_perm [1,0,3,2]
    acc = g0 ? acc + o : acc;
    if (glog > 1) {
      const double o2 = dpp_d<0x4E>(acc);  // quad_perm [2,3,0,1]
      acc = g1 ? acc + o2 : acc;
      if (glog > 2) {
        const double o3 = dpp_d<0x141>(acc);  // row_half_mirror
        acc = g2 ? acc + o3 : acc;
        if (glog > 3) {
          const double o4 = dpp_d<0x140>(acc);  // row_mirror
          if (gl > 3) acc += o4;
          if (glog > 4) {  // xor 16 and xor 32 by the lane swaps (partners: the two operands)
            double a, b;
            swap16_d(acc, a, b);
            if (gl > 4) acc = a + b;
            if (glog > 5) {
              swap32_d(acc, a, b);
              if (gl > 5) acc = a + b;
            }
          }
        }
      }
    }
  }
  return acc;
}

// Schedule records are read through buffer descriptors: table base and size in SGPRs, the step
// offset in an SGPR (soffset), the lane's offset a constant VGPR, so no record address is computed
// per step.  Every table is followed by TABLE_PAD_STEPS zero steps in device memory (push_table), so
// the record pipelines load steps up to n + 2 unclamped and in range (round 5: the clamp's n - 1
// was an SGPR the two-wave kernel spilled, one v_readlane per solve step, +21 % forward-solve time).
constexpr int TABLE_PAD_STEPS = 3;
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc table_rsrc(const uint32_t* tbl, int nsteps, int stride_words) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(tbl), (short)0,
                                           (nsteps + TABLE_PAD_STEPS) * stride_words * 4, 0x00020000);
}

// one lane's records of a solve step: 4 segment quads (a0, b0, a1, b1), targets t0..t3 (paired
// steps: t1 = t0, not read)
struct SolveRec {
  uint32_t a[SOLVE_MAXC], b[SOLVE_MAXC];
  uint32_t t0, t1, t2, t3;
};
__device__ __forceinline__ void load_solve(Rsrc rs, int soff, uint32_t lane, SolveRec& r) {
#pragma unroll
  for (int q = 0; q < SOLVE_MAXC / 2; ++q) {
    const auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lane * 16u) + q * 1024, soff, 0);
    r.a[2 * q] = w[0], r.b[2 * q] = w[1], r.a[2 * q + 1] = w[2], r.b[2 * q + 1] = w[3];
  }
  const auto tg =
      __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lane * 16u) + 4 * SOLVE_TERM_WORDS, soff, 0);
  r.t0 = tg[0], r.t1 = tg[1], r.t2 = tg[2], r.t3 = tg[3];
}
// one lane's records of a factorization step: meta word + FAC_MAXC (a, b, c, -) address quads
struct FacRec {
  uint32_t mt;
  uint32_t a[FAC_MAXC], b[FAC_MAXC], c[FAC_MAXC];
};
__device__ __forceinline__ void load_fac(Rsrc rs, int soff, uint32_t lane, FacRec& r) {
  r.mt = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(lane * 4u), soff, 0);
#pragma unroll
  for (int c = 0; c < FAC_MAXC; ++c) {
    const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lane * 16u) + 256 + c * 1024, soff, 0);
    r.a[c] = q[0], r.b[c] = q[1], r.c[c] = q[2];
  }
}

// straight-line dot product (two accumulators halve the dependent FMA chain).  All LDS reads are
// forced in front of the FMAs (sched_group_barrier: 0x100 = DS read, 0x002 = VALU) so that they
// overlap instead of paying one LDS round trip per term.
template <int C>
__device__ __forceinline__ double dot3(const double* v, const FacRec& r) {
  double x[C], y[C], d[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    x[c] = lds_ld(v, r.a[c]);
    y[c] = lds_ld(v, r.b[c]);
    d[c] = lds_ld(v, r.c[c]);
  }
  __builtin_amdgcn_sched_group_barrier(0x100, 3 * C, 0);
  __builtin_amdgcn_sched_group_barrier(0x002, 3 * C, 0);
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    if (c & 1)
      a1 = fma(x[c] * y[c], d[c], a1);
    else
      a0 = fma(x[c] * y[c], d[c], a0);
  }
  return a0 + a1;
}

// One solve step: segment sums n_q = -(v[a_2q] v[b_2q] + v[a_2q+1] v[b_2q+1]) (the FMA negate
// modifiers are free) are added to targets t_q with LDS atomics (ds_add_f64, no return).  A wave's
// LDS instructions execute in issue order, so the next step's reads see these sums.  Unused
// segments read the ZERO slot and add 0 to the lane's sink slot, so nothing needs a branch.
__device__ __forceinline__ void lds_add(uint32_t a, double x) {
  __hip_atomic_fetch_add((lds_double*)(size_t)a, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <bool PAIRED>
__device__ __forceinline__ void solve_step(const SolveRec& r, double* v) {
  double x[8], y[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = lds_ld(v, r.a[c]), y[c] = lds_ld(v, r.b[c]);
  __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
  __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
  const double n0 = fma(-x[1], y[1], -(x[0] * y[0]));
  const double n1 = fma(-x[3], y[3], -(x[2] * y[2]));
  const double n2 = fma(-x[5], y[5], -(x[4] * y[4]));
  const double n3 = fma(-x[7], y[7], -(x[6] * y[6]));
  if constexpr (PAIRED) {
    // segments 0 and 1 are a pair of one target (or segment 1 is unused: its zero-padding terms
    // give -0, and n0 + -0 == n0 exactly) -- one atomic for both
    lds_add(r.t0, n0 + n1);
  } else {
    lds_add(r.t0, n0);
    lds_add(r.t1, n1);
  }
  lds_add(r.t2, n2);
  lds_add(r.t3, n3);
  LDS_FENCE();
}
// One factorization step: v[t] <- -sum_c v[a_c] v[b_c] v[c_c]; a D_j task (in place on the 1/D slot,
// which holds the KKT diagonal until then) stores 1/D_j instead.  Only group heads store (idle
// lanes have no slot).
__device__ __forceinline__ void fac_step(const FacRec& r, double* v) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(r.mt);
  const uint32_t C = (m0 >> META_C_SHIFT) & 15u, glog = (m0 >> META_SGLOG_SHIFT) & 7u;
  double acc = C <= 2 ? dot3<2>(v, r) : dot3<4>(v, r);
  acc = group_sum(acc, glog, (r.mt >> META_GLOG_SHIFT) & 7u);
  if (r.mt & META_HEAD) {
    const uint32_t t = r.mt & META_TGT_MASK;
    const double nv = -acc;
    // the division only in steps that hold a D_j task (the block-inverse tail has none)
    if (m0 & META_SISD)
      lds_st(v, t, (r.mt & META_ISD) ? 1.0 / nv : nv);
    else
      lds_st(v, t, nv);
  }
  LDS_FENCE();
}

// Step loops.  Records (L2-resident, fixed stride) rotate through three register sets, so the
// records of step s + 2 are in flight while steps s and s + 1 compute.  prefetch() issues the
// first three steps' loads; callers issue it ahead of unrelated work to hide the L2 latency.
// D = record sets in flight: 3 (records of step s + 2 load during step s) or 4 (s + 3; the
// two-wave kernel's first wave, +0.7 % at N = 40 and -4.8 % in the one-wave N = 20 kernel)
template <typename Ops, int D = 3>
struct Pipe {
  typename Ops::Rec a, b, c, d;  // d unused at D = 3
};
template <typename Ops>
__device__ __forceinline__ int step_off(int /*n*/, int s) {  // s <= n + 2: the padded table
  // readfirstlane: a no-op where the step counter is known uniform; inside the two-wave kernel's
  // wave-selected branches LLVM otherwise keeps the offset in a VGPR and waterfalls every load
  return __builtin_amdgcn_readfirstlane(s * (Ops::STRIDE * 4));
}
template <typename Ops, int D>
__device__ __forceinline__ void prefetch(Rsrc rs, int n, uint32_t lane, Pipe<Ops, D>& p) {
  // n >= 1 (checked at plan time); no branch here, so the vmcnt bookkeeping after it is exact
  // the sets are issued in order (sched_barrier) so that the vmcnt wait for one set never
  // includes a later one
  __builtin_amdgcn_sched_barrier(0);
  Ops::load(rs, step_off<Ops>(n, 0), lane, p.a);
  __builtin_amdgcn_sched_barrier(0);
  Ops::load(rs, step_off<Ops>(n, 1), lane, p.b);
  __builtin_amdgcn_sched_barrier(0);
  Ops::load(rs, step_off<Ops>(n, 2), lane, p.c);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (D == 4) {
    Ops::load(rs, step_off<Ops>(n, 3), lane, p.d);
    __builtin_amdgcn_sched_barrier(0);
  }
}
// The rotation is unrolled 12 steps deep: LLVM's waitcnt insertion merges states pessimistically
// at a loop header (the first step after it would wait for all three sets), so the header is
// reached at most once per ~12 steps.
#define MPCQP_STEP(X)                                       \
  ops.step(p.X, s);                                         \
  if (++s >= n) break;                                      \
  __builtin_amdgcn_sched_barrier(0);                        \
  Ops::load(rs, step_off<Ops>(n, s + D - 1), lane, p.X);    \
  __builtin_amdgcn_sched_barrier(0);
template <typename Ops, int D>
__device__ __forceinline__ void run_body(Rsrc rs, int n, uint32_t lane, const Ops& ops,
                                         Pipe<Ops, D>& p) {
  int s = 0;
  if constexpr (D == 4) {
    for (;;) {
      MPCQP_STEP(a) MPCQP_STEP(b) MPCQP_STEP(c) MPCQP_STEP(d)
      MPCQP_STEP(a) MPCQP_STEP(b) MPCQP_STEP(c) MPCQP_STEP(d)
      MPCQP_STEP(a) MPCQP_STEP(b) MPCQP_STEP(c) MPCQP_STEP(d)
    }
  } else {
    for (;;) {
      MPCQP_STEP(a) MPCQP_STEP(b) MPCQP_STEP(c)
      MPCQP_STEP(a) MPCQP_STEP(b) MPCQP_STEP(c)
      MPCQP_STEP(a) MPCQP_STEP(b) MPCQP_STEP(c)
      MPCQP_STEP(a) MPCQP_STEP(b) MPCQP_STEP(c)
    }
  }
}
#undef MPCQP_STEP
// Solve steps with the matrix operands read one step ahead (Plan::mat_first: a = the matrix value
// of every term, constant during a solve): a step issues its 8 vector reads (which follow the
// previous step's atomics in the LDS queue), then the 8 matrix reads of the next step, then its
// products -- which wait only for the vector reads (LDS returns in order: a counted lgkmcnt) --
// and atomics.  The critical path of a step loses 8 of its 16 reads (tools/lds_probe.hip, split
// step: -13 % per step at two waves per CU, -7 % at four).
template <bool PAIRED>
__device__ __forceinline__ void solve_step_pf(const SolveRec& r, const SolveRec& nx, double (&m)[8],
                                              double* v) {
  double y[8], mn[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) y[c] = lds_ld(v, r.b[c]);
#pragma unroll
  for (int c = 0; c < 8; ++c) mn[c] = lds_ld(v, nx.a[c]);
  __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
  __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
  const double n0 = fma(-m[1], y[1], -(m[0] * y[0]));
  const double n1 = fma(-m[3], y[3], -(m[2] * y[2]));
  const double n2 = fma(-m[5], y[5], -(m[4] * y[4]));
  const double n3 = fma(-m[7], y[7], -(m[6] * y[6]));
  if constexpr (PAIRED) {
    lds_add(r.t0, n0 + n1);
  } else {
    lds_add(r.t0, n0);
    lds_add(r.t1, n1);
  }
  lds_add(r.t2, n2);
  lds_add(r.t3, n3);
  LDS_FENCE();
#pragma unroll
  for (int c = 0; c < 8; ++c) m[c] = mn[c];
}
#define MPCQP_PFSTEP(X, Y)                                  \
  solve_step_pf<PAIRED>(p.X, p.Y, m, v);                    \
  if (++s >= n) break;                                      \
  __builtin_amdgcn_sched_barrier(0);                        \
  load_solve(rs, step_off<SolveOps<PAIRED>>(n, s + 2), lane, p.X); \
  __builtin_amdgcn_sched_barrier(0);
template <bool PAIRED>
struct SolveOps;
template <bool PAIRED>
__device__ __forceinline__ void run_body_pf(Rsrc rs, int n, uint32_t lane, double* v,
                                            Pipe<SolveOps<PAIRED>>& p) {
  double m[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) m[c] = lds_ld(v, p.a.a[c]);  // the first step's matrix operands
  int s = 0;
  for (;;) {
    MPCQP_PFSTEP(a, b) MPCQP_PFSTEP(b, c) MPCQP_PFSTEP(c, a)
    MPCQP_PFSTEP(a, b) MPCQP_PFSTEP(b, c) MPCQP_PFSTEP(c, a)
    MPCQP_PFSTEP(a, b) MPCQP_PFSTEP(b, c) MPCQP_PFSTEP(c, a)
    MPCQP_PFSTEP(a, b) MPCQP_PFSTEP(b, c) MPCQP_PFSTEP(c, a)
  }
}
#undef MPCQP_PFSTEP

// ---- matrix operands in registers (kernel mode KM_MREG) -------------------------------------
// Every solve term is (matrix value) x (vector entry); the matrix values (L, the block inverses and
// couplings N | G | G', the ONE / MONE / ZERO constants) are constant between factorizations.  After
// every factorization the matrix operand of every term of the (at most MREG_STEPS) forward and
// backward steps is read once into registers (MatRegs, 96 doubles per lane), and a solve step then
// issues only its 8 vector-entry reads: 16 -> 8 ds_read_b64 per step (tools/lds_probe.hip at four
// waves per CU: 342 -> 258 cycles per wave-step).  The host splits each term into its vector
// address (in W or C) and its matrix address (anything else) -- the product is commutative and
// fma(-x1, y1, -(x0 y0)) does not depend on the operands' order, so the results are bit-identical
// to the LDS-operand kernel on the same plan.
constexpr int MREG_STEPS = 6;
struct MatRegs {
  double m[2][MREG_STEPS][SOLVE_MAXC];  // [forward / backward][step][term]
};
// compact step record: vector addresses of the 8 terms, then the 4 targets (3 rows of 64 lane quads)
constexpr int SOLVEC_STEP_WORDS = 3 * 64 * 4;
constexpr int SOLVEM_STEP_WORDS = 2 * 64 * 4;  // matrix addresses of the 8 terms (2 rows)
struct SolveRecC {
  uint32_t b[SOLVE_MAXC];
  uint32_t t0, t1, t2, t3;
};
__device__ __forceinline__ void load_solve_c(Rsrc rs, int soff, uint32_t lane, SolveRecC& r) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lane * 16u) + q * 1024, soff, 0);
    r.b[4 * q] = w[0], r.b[4 * q + 1] = w[1], r.b[4 * q + 2] = w[2], r.b[4 * q + 3] = w[3];
  }
  const auto tg = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lane * 16u) + 2048, soff, 0);
  r.t0 = tg[0], r.t1 = tg[1], r.t2 = tg[2], r.t3 = tg[3];
}
// the registers of one solve: matrix values of steps 0..MREG_STEPS-1 (steps past n re-read the last
// one: never used)
__device__ __forceinline__ void load_mats(const uint32_t* tbl, int n, uint32_t lane, const double* v,
                                          double (&m)[MREG_STEPS][SOLVE_MAXC]) {
  const Rsrc rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(tbl), (short)0,
                                                    n * SOLVEM_STEP_WORDS * 4, 0x00020000);
#pragma unroll
  for (int st = 0; st < MREG_STEPS; ++st) {
    const int soff = (st < n ? st : n - 1) * (SOLVEM_STEP_WORDS * 4);
    uint32_t a[SOLVE_MAXC];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lane * 16u) + q * 1024, soff, 0);
      a[4 * q] = w[0], a[4 * q + 1] = w[1], a[4 * q + 2] = w[2], a[4 * q + 3] = w[3];
    }
#pragma unroll
    for (int c = 0; c < SOLVE_MAXC; ++c) m[st][c] = lds_ld(v, a[c]);
  }
}
template <bool PAIRED>
__device__ __forceinline__ void solve_step_r(const SolveRecC& r, const double (&x)[SOLVE_MAXC],
                                             double* v) {
  double y[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) y[c] = lds_ld(v, r.b[c]);
  __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
  __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
  const double n0 = fma(-x[1], y[1], -(x[0] * y[0]));
  const double n1 = fma(-x[3], y[3], -(x[2] * y[2]));
  const double n2 = fma(-x[5], y[5], -(x[4] * y[4]));
  const double n3 = fma(-x[7], y[7], -(x[6] * y[6]));
  if constexpr (PAIRED) {
    lds_add(r.t0, n0 + n1);
  } else {
    lds_add(r.t0, n0);
    lds_add(r.t1, n1);
  }
  lds_add(r.t2, n2);
  lds_add(r.t3, n3);
  LDS_FENCE();
}
struct PipeC {
  SolveRecC a, b, c;
};
__device__ __forceinline__ int step_off_c(int /*n*/, int s) {  // s <= n + 1: the padded table
  return __builtin_amdgcn_readfirstlane(s * (SOLVEC_STEP_WORDS * 4));
}
__device__ __forceinline__ void prefetch_c(Rsrc rs, int n, uint32_t lane, PipeC& p) {
  __builtin_amdgcn_sched_barrier(0);
  load_solve_c(rs, step_off_c(n, 0), lane, p.a);
  __builtin_amdgcn_sched_barrier(0);
  load_solve_c(rs, step_off_c(n, 1), lane, p.b);
  __builtin_amdgcn_sched_barrier(0);
  load_solve_c(rs, step_off_c(n, 2), lane, p.c);
  __builtin_amdgcn_sched_barrier(0);
}
// n <= MREG_STEPS (checked at create time): the unrolled positions index the matrix registers
#define MPCQP_RSTEP(X, POS)                                 \
  solve_step_r<PAIRED>(p.X, m[POS], v);                     \
  if (++s >= n) break;                                      \
  __builtin_amdgcn_sched_barrier(0);                        \
  load_solve_c(rs, step_off_c(n, s + 2), lane, p.X);        \
  __builtin_amdgcn_sched_barrier(0);
template <bool PAIRED>
__device__ __forceinline__ void run_body_r(Rsrc rs, int n, uint32_t lane, double* v, PipeC& p,
                                           const double (&m)[MREG_STEPS][SOLVE_MAXC]) {
  int s = 0;
  for (;;) {
    MPCQP_RSTEP(a, 0) MPCQP_RSTEP(b, 1) MPCQP_RSTEP(c, 2)
    MPCQP_RSTEP(a, 3) MPCQP_RSTEP(b, 4) MPCQP_RSTEP(c, 5)
    break;
  }
}
#undef MPCQP_RSTEP

template <bool PAIRED>
struct SolveOps {
  typedef SolveRec Rec;
  static constexpr int STRIDE = SOLVE_STEP_WORDS;
  double* v;
  __device__ __forceinline__ static void load(Rsrc rs, int soff, uint32_t lane, Rec& r) {
    load_solve(rs, soff, lane, r);
  }
  __device__ __forceinline__ void step(const Rec& r, int) const { solve_step<PAIRED>(r, v); }
};
struct FacOps {
  typedef FacRec Rec;
  static constexpr int STRIDE = FAC_STEP_WORDS;
  double* v;
  __device__ __forceinline__ static void load(Rsrc rs, int soff, uint32_t lane, Rec& r) {
    load_fac(rs, soff, lane, r);
  }
  __device__ __forceinline__ void step(const Rec& r, int) const { fac_step(r, v); }
};
template <int D = 3>
__device__ __forceinline__ void run_fac(const uint32_t* tbl, int nsteps, double* v, int lane) {
  Pipe<FacOps, D> pp;
  const Rsrc rs = table_rsrc(tbl, nsteps, FAC_STEP_WORDS);
  prefetch(rs, nsteps, (uint32_t)lane, pp);
  run_body(rs, nsteps, (uint32_t)lane, FacOps{v}, pp);
}

// numeric LDL': U = L D and D by levels, L = U / D (flat pass), then the block-inverse tail
__device__ __forceinline__ void run_factor(const KParams& p, double* v, int lane) {
  const DevPlan& P = p.pl;
  run_fac(P.fac, P.nfac, v, lane);
  LDS_FENCE();
#pragma unroll 4
  for (int k = lane; k < P.nnzL; k += 64) v[P.LX + k] *= v[P.Lcol[k]];
  LDS_FENCE();
  if (P.ntail > 0) run_fac(P.tail, P.ntail, v, lane);
}

// constraint classes packed 2 bits per register slot (auxil.c constr_type)
enum : uint32_t { CT_INEQ = 0, CT_EQ = 1, CT_FREE = 2 };

// Register-resident per-instance state.  Element i of an n- or m-vector lives on lane i % 64,
// slot i / 64.  The scalings D, E live in the wave's scratch slab (read at checks only).
template <int RN, int RM>
struct Inst {
  double x[RN], q[RN];
  double z[RM], y[RM], l[RM], u[RM];
  uint32_t ct;  // 2 bits per slot
  double rinv[RM], rvec[RM];  // rho_inv_vec / rho_vec of the lane's rows
  double c, cinv, rho;
  double rv_eq, ri_eq, ri_in, ri_free;  // rho_vec / rho_inv_vec values per class
  double pri_res, dua_res;
  double Dinv[RN], Einv[RM];  // inverse scalings (termination checks), 1 past the end of x / z
};

// per-wave scratch slab (doubles): the scalings D, E of the wave's current instance (the
// infeasibility certificates and the unscaling of the solution), then -- with Plan::mv_global --
// the scaled matrix values [P | A] (MV-relative indices; otherwise they stay in LDS, Plan::MV).
struct Slab {
  double *D, *E, *MV;
};
__host__ __device__ __forceinline__ size_t slab_doubles(int n, int m, int mv_slab) {
  return (((size_t)n + m + 1) & ~size_t(1)) + mv_slab;
}
__device__ __forceinline__ size_t slab_doubles(const DevPlan& P) { return slab_doubles(P.n, P.m, P.mv_slab); }
__device__ __forceinline__ Slab slab_of(const DevPlan& P, double* scr) {
  Slab s;
  s.D = scr;
  s.E = s.D + P.n;
  s.MV = scr + ((P.n + P.m + 1) & ~1);  // 16-byte aligned (the slab base is)
  return s;
}
// residual mat-vec out[r] = sum_k v[vpos[t]] * in[in_idx[t]], t = off_r + 64 k + lane, for every
// slot r of the instance (terms in order): the scaled values are the LDS-resident copy (MV), the
// two index lists are shared by all instances.  All index loads are issued before the first use.
// This lane's term indices of one mat-vec (shared by all instances: L1/L2 hits), loaded ahead of
// the value reads: packed (value slot, input index) per term, and the first 64 terms of the first
// LPF outputs with more than KMAX terms
constexpr int ELL_LPF = 2;
template <int R, int KMAX>
struct EllTk {
  uint32_t tk[R][KMAX];
  uint32_t lp[ELL_LPF], li[ELL_LPF];
};
template <int R, int KMAX>
__device__ __forceinline__ void ell_load(const EllDev& e, EllTk<R, KMAX>& t, int lane) {
  static_assert(KMAX % 4 == 0, "lane-major term rows are loaded 16 bytes at a time");
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (e.K[r] == 0) continue;  // slot beyond the instance (wave-uniform)
    const uint4* row = reinterpret_cast<const uint4*>(e.pk + (size_t)(r * 64 + lane) * KMAX);
#pragma unroll
    for (int q = 0; q < KMAX / 4; ++q) {
      const uint4 w = row[q];
      t.tk[r][4 * q] = w.x, t.tk[r][4 * q + 1] = w.y, t.tk[r][4 * q + 2] = w.z, t.tk[r][4 * q + 3] = w.w;
    }
  }
#pragma unroll
  for (int L = 0; L < ELL_LPF; ++L) {
    t.lp[L] = 0, t.li[L] = 0;
    if (L < e.nlong && lane < e.long_cnt[L]) {
      const int q = e.long_off[L] + lane;
      t.lp[L] = e.vpos[q], t.li[L] = e.in[q];
    }
  }
}
// mv: the resident scaled values -- the LDS image (Plan::MV slots) or the wave's slab
// (Plan::mv_global, MV-relative); in: the input vector staged in LDS
// Every output accumulates its terms in OSQP's order (symbolic.cpp: mat_vec / mat_tpose_vec /
// the symmetric P x), each product rounded before it is added (no contraction, above).  Long
// outputs: the products of all lanes staged in LDS (stg, wave-private, long_cnt doubles) and summed
// in term order by seq_sum.
template <int R, int KMAX>
__device__ __forceinline__ void ell_apply(const EllDev& e, const EllTk<R, KMAX>& t, const double* mv,
                                          const double* in, double (&out)[R], int lane, double* stg) {
  constexpr int LPF = ELL_LPF;
  const uint32_t(&lp)[LPF] = t.lp;
  const uint32_t(&li)[LPF] = t.li;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    double s = 0.0;
    if (e.K[r] != 0) {
      double a[KMAX], b[KMAX];
#pragma unroll
      for (int k = 0; k < KMAX; ++k) a[k] = mv[t.tk[r][k] & 0xffffu], b[k] = in[t.tk[r][k] >> 16];
#pragma unroll
      for (int k = 0; k < KMAX; ++k) s += a[k] * b[k];
    }
    out[r] = s;
  }
  if (e.nlong == 0) return;
  // every long output's products staged first (each output at its own offset: mpcqp_create checks
  // that they fit), then the sequential sums two at a time
  int base = 0;
  for (int L = 0; L < e.nlong; ++L) {
    int t0 = lane;
#pragma unroll
    for (int k = 0; k < LPF; ++k)
      if (k == L) {
        if (lane < e.long_cnt[L]) stg[base + lane] = mv[lp[k]] * in[li[k]];
        t0 = lane + 64;
      }
    for (int t = t0; t < e.long_cnt[L]; t += 64) {
      const int q = e.long_off[L] + t;
      stg[base + t] = mv[e.vpos[q]] * in[e.in[q]];
    }
    base += e.long_cnt[L];
  }
  LDS_FENCE();
  base = 0;
  for (int L = 0; L < e.nlong; L += 2) {
    const int c0 = e.long_cnt[L], c1 = L + 1 < e.nlong ? e.long_cnt[L + 1] : 0;
    double s0, s1 = 0.0;
    if (c1)
      seq_sum2(stg + base, c0, stg + base + c0, c1, s0, s1);
    else
      s0 = seq_sum(stg + base, c0);
    const int o0 = e.long_out[L], o1 = c1 ? e.long_out[L + 1] : -1;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (o0 == lane + 64 * r) out[r] = s0;
      if (o1 == lane + 64 * r) out[r] = s1;
    }
    base += c0 + c1;
  }
  LDS_FENCE();
}
template <int R, int KMAX>
__device__ __forceinline__ void ell_mv(const EllDev& e, const double* mv, const double* in,
                                       double (&out)[R], int lane, double* stg) {
  EllTk<R, KMAX> t;
  ell_load(e, t, lane);
  ell_apply(e, t, mv, in, out, lane, stg);
}
// The Ruiz passes' index lists, loaded once per solve into registers (lane-major, 8 bytes = four
// u16 slots per load; shared by every instance: L1/L2 hits): the passes then read only values.
template <int R, int KMAX>
struct EllIdx {
  uint32_t w[R][KMAX / 2];  // two u16 overlay slots per register
};
template <int R, int KMAX>
__device__ __forceinline__ void load_idx(const EllDev& e, EllIdx<R, KMAX>& ix, int lane) {
  static_assert(KMAX % 4 == 0, "index rows are loaded 8 bytes at a time");
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (e.K[r] == 0) continue;
    const uint2* row = reinterpret_cast<const uint2*>(e.sk + (size_t)(r * 64 + lane) * KMAX);
#pragma unroll
    for (int q = 0; q < KMAX / 4; ++q) {
      const uint2 w = row[q];
      ix.w[r][2 * q] = w.x, ix.w[r][2 * q + 1] = w.y;
    }
  }
}
// the index words made opaque (asm "+v"): the LDS addresses derived from them are recomputed where
// they are used instead of being hoisted out of an enclosing loop into registers
template <int R, int KMAX>
__device__ __forceinline__ void opaque_idx(EllIdx<R, KMAX>& ix) {
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int k = 0; k < KMAX / 2; ++k) asm volatile("" : "+v"(ix.w[r][k]));
}
template <int N>
__device__ __forceinline__ void opaque_words(uint32_t (&w)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) asm volatile("" : "+v"(w[k]));
}
// out[r] = max_k |v[slot]| over the ELL terms of slot r, indices from registers (max is
// order-free, so any traversal equals OSQP's); long outputs read their slots from global memory
// kf: bit r = slot r used (ell_kflags, read once per solve: the per-pass kernel-argument reads of
// e.K[r] were each an s_load with an lgkmcnt(0) wait)
template <int R>
__device__ __forceinline__ uint32_t ell_kflags(const EllDev& e) {
  uint32_t f = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) f |= (e.K[r] != 0 ? 1u : 0u) << r;
  asm volatile("" : "+v"(f));
  return f;
}
// KF = false ((4, 8) bucket): the flags are not used (there they moved a kernel-argument reload
// into the ADMM loop head, tests/test_isa_hot_loops.py)
template <bool KF, int R, int KMAX>
__device__ __forceinline__ void ell_absmax_r(const EllDev& e, const EllIdx<R, KMAX>& ix, uint32_t kf,
                                             const double* v, double (&out)[R], int lane) {
  const uint32_t kfu = KF ? __builtin_amdgcn_readfirstlane(kf) : 0u;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    double mx = 0.0;
    if (KF ? (kfu & (1u << r)) != 0 : e.K[r] != 0) {
      double b[KMAX];
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        const uint32_t w = ix.w[r][k / 2];
        b[k] = v[(k & 1) ? (w >> 16) : (w & 0xffffu)];  // padding -> S_ZERO
      }
#pragma unroll
      for (int k = 0; k < KMAX; ++k) mx = dmaxd(fabs(b[k]), mx);
    }
    out[r] = mx;
  }
  for (int L = 0; L < e.nlong; ++L) {
    double mx = 0.0;
    for (int t = lane; t < e.long_cnt[L]; t += 64) mx = dmaxd(fabs(v[e.src[e.long_off[L] + t]]), mx);
    mx = wave_max(mx);
    const int o = e.long_out[L];
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (o == lane + 64 * r) out[r] = mx;
  }
}
// Ruiz rescale of the value overlay [P | A] (cnt = nnzP + nnzA values from S_P):
//   v[S_P + k] = ((v[S_P + k] * f) * v[ra[k]]) * v[ca[k]],  f = cp for P's values, 1 for A's
// -- scaling.c's mat_premult_diag / mat_postmult_diag, with the previous pass's cost factor c
// (mat_mult_scalar on P) deferred into this pass: the same multiplications in the same order, and
// x * 1.0 is exact.  The row / column scaling slots come from registers (JW pairs of u16 per
// lane: value k = 64 j + lane, j < 2 JW).
template <int JW>
__device__ __forceinline__ void scale_pa_r(double* v, int S_P, int nnzP, int cnt,
                                           const uint32_t (&ra)[JW], const uint32_t (&ca)[JW],
                                           double cp, int lane) {
  constexpr int U = 8;  // values in flight per lane: all value reads of a batch, then its stores
  static_assert((2 * JW) % U == 0, "batches of U values");
#pragma unroll
  for (int j0 = 0; j0 < 2 * JW; j0 += U) {
    if (64 * j0 >= cnt) break;  // wave-uniform
    double x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u, k = 64 * j + lane, kc = k < cnt ? k : 0;
      const double f = k < nnzP ? cp : 1.0;
      const uint32_t a = (j & 1) ? (ra[j / 2] >> 16) : (ra[j / 2] & 0xffffu);
      const uint32_t b = (j & 1) ? (ca[j / 2] >> 16) : (ca[j / 2] & 0xffffu);
      x[u] = ((v[S_P + kc] * f) * v[a]) * v[b];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = 64 * (j0 + u) + lane;
      if (k < cnt) v[S_P + k] = x[u];
    }
  }
}
// the inverse of the scaled P values for the next solve (unscale_data: mat_mult_scalar(P, c^-1),
// mat_premult_diag / mat_postmult_diag(P, D^-1)): out[k] = ((v[S_P + k] c^-1) v[ra_k]) v[ca_k],
// k < nnzP, the D_temp slots holding D^-1 -- the operand layout of scale_pa_r
template <int JW>
__device__ __forceinline__ void unscale_p_r(const double* v, int S_P, int nnzP, const uint32_t (&ra)[JW],
                                            const uint32_t (&ca)[JW], double cinv, int lane,
                                            double* out) {
#pragma unroll
  for (int j = 0; j < 2 * JW; ++j) {
    if (64 * j >= nnzP) break;  // wave-uniform
    const int k = 64 * j + lane;
    const uint32_t a = (j & 1) ? (ra[j / 2] >> 16) : (ra[j / 2] & 0xffffu);
    const uint32_t b = (j & 1) ? (ca[j / 2] >> 16) : (ca[j / 2] & 0xffffu);
    if (k < nnzP) out[k] = ((v[S_P + k] * cinv) * v[a]) * v[b];
  }
}
// v[base + k] = src[k] for k < cnt, 8 loads per lane in flight
__device__ __forceinline__ void load_vals(double* v, int base, const double* src, int cnt,
                                          int lane) {
  constexpr int U = 8;
  for (int k0 = 0; k0 < cnt; k0 += 64 * U) {
    double x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 64 * u + lane;
      x[u] = src[k < cnt ? k : 0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 64 * u + lane;
      if (k < cnt) v[base + k] = x[u];
    }
  }
}
template <int RN, int RM>
__device__ __forceinline__ uint32_t ctype(const Inst<RN, RM>& S, int r) {
  return (S.ct >> (2 * r)) & 3u;
}
template <int RN, int RM>
__device__ __forceinline__ double rinv_of(const Inst<RN, RM>& S, int r) {
  return S.rinv[r];
}
template <int RN, int RM>
__device__ __forceinline__ double rvec_of(const Inst<RN, RM>& S, int r) {
  return S.rvec[r];
}
// rho_vec / rho_inv_vec values, computed exactly as OSQP computes them
// (auxil.c set_rho_vec, osqp.c osqp_update_rho): rho_inv = 1 / rho_vec elementwise.
template <int RN, int RM>
__device__ __forceinline__ void set_rho(Inst<RN, RM>& S) {
  S.rv_eq = RHO_EQ_OVER_RHO_INEQ * S.rho;
  S.ri_eq = 1. / S.rv_eq;
  S.ri_in = 1. / S.rho;
  S.ri_free = 1. / RHO_MIN;
  // per-row values by explicit predicated moves (a `?:` chain here is turned into a
  // scratch-memory lookup table by the compiler)
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const uint32_t t = ctype(S, r);
    double ri = S.ri_in, rv = S.rho;
    if (t == CT_EQ) ri = S.ri_eq, rv = S.rv_eq;
    if (t == CT_FREE) ri = S.ri_free, rv = RHO_MIN;
    S.rinv[r] = ri;
    S.rvec[r] = rv;
  }
}

template <int RN, int RM>
struct Resid {
  double Ax[RM], Px[RN], Aty[RN];
};

// KKT values [[P + sigma I, A'], [A, -diag(1/rho)]] into the permuted LDS image
// (OSQP kkt.c form_KKT / update_KKT_*), then factorize.
template <int RN, int RM>
__device__ __forceinline__ void assemble_and_factor(const KParams& p, const Slab& sb, double* v,
                                                    const double* mv, int lane, const Inst<RN, RM>& S) {
  const DevPlan& P = p.pl;
  for (int k = lane; k < P.nnzL; k += 64) v[P.LX + k] = 0.0;
  // the whole 1/D region (the D_j tasks' KKT diagonal in, 1/D_j out; 0 in the padding, which the
  // diagonal pass multiplies with the zeroed W padding)
#pragma unroll
  for (int r = 0; r < RN + RM; ++r) v[P.DINV + lane + 64 * r] = 0.0;
  if (lane < ZERO_BLOCK) v[P.ZERO + lane] = 0.0;
  if (lane == 0) {
    v[P.ONE] = 1.0;
    v[P.MONE] = -1.0;
  }
  LDS_FENCE();
  for (int j = lane; j < P.n; j += 64) v[P.slotSig[j]] = p.s.sigma;
  LDS_FENCE();
  for (int k = lane; k < P.nnzP; k += 64) {
    const double val = mv[P.MV + k];
    v[P.slotP[k]] = (P.Pi[k] == P.Pcol[k]) ? val + p.s.sigma : val;
  }
  for (int k = lane; k < P.nnzA; k += 64) v[P.slotA[k]] = mv[P.MV + P.nnzP + k];
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int i = lane + 64 * r;
    if (i < P.m) v[P.slotRho[i]] = -rinv_of(S, r);
  }
  LDS_FENCE();
  run_factor(p, v, lane);
}

// update_info: scaled Ax, Px, A'y and the unscaled residual norms (auxil.c compute_pri_res /
// compute_dua_res).  x and y are staged as plain arrays in the W region.
#ifdef MPCQP_TIMING
#define TACC_PARAM , unsigned long long* tacc
#define TACC_ARG , tacc
#else
#define TACC_PARAM
#define TACC_ARG
#endif
template <int RN, int RM>
__device__ __forceinline__ void compute_residuals(const KParams& p, Inst<RN, RM>& S, Resid<RN, RM>& R,
                                  const Slab& sb, double* v, const double* mv, int lane TACC_PARAM) {
  const DevPlan& P = p.pl;
  const int n = P.n, m = P.m;
  double* xb = v + P.W;
  double* yb = v + P.W + n;
  T_BEGIN(t_r0);
  LDS_FENCE();
  // unconditional stores: x's slots past n land in y's range and are overwritten by the y stores
  // that follow (a wave's LDS stores complete in order); y's slots past m stay inside the padded
  // W region (n + 64 RM <= 64 (RN + RM) = NKP)
#pragma unroll
  for (int r = 0; r < RN; ++r) xb[lane + 64 * r] = S.x[r];
  LDS_FENCE();
#pragma unroll
  for (int r = 0; r < RM; ++r) yb[lane + 64 * r] = S.y[r];
  LDS_FENCE();
  double pr = 0.0, dr = 0.0;
  T_END(T_RS0, t_r0);
  T_BEGIN(t_r1);
  {  // the three mat-vecs' index loads issued together: one L2 round trip instead of three
     // (+0.8 %)
    EllTk<RM, ELL_KA> tA;
    EllTk<RN, ELL_KP> tP;
    EllTk<RN, ELL_KAT> tT;
    ell_load(P.eA, tA, lane);
    ell_load(P.eP, tP, lane);
    ell_load(P.eAt, tT, lane);
    ell_apply(P.eA, tA, mv, xb, R.Ax, lane, v + P.CACC);  // padding terms are 0 * x
    ell_apply(P.eP, tP, mv, xb, R.Px, lane, v + P.CACC);
    ell_apply(P.eAt, tT, mv, yb, R.Aty, lane, v + P.CACC);
  }
  TSYNC(R.Aty[0]);
  T_END(T_RS1, t_r1);  // the three mat-vecs together (slot rs_matvecs)
  T_BEGIN(t_r4);
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int i = lane + 64 * r;
    if (i < m) pr = dmaxd(pr, fabs(S.Einv[r] * (R.Ax[r] - S.z[r])));
    if (i >= m) R.Ax[r] = 0.0;
  }
#pragma unroll
  for (int r = 0; r < RN; ++r) {
    const int j = lane + 64 * r;
    if (j < n) dr = dmaxd(dr, fabs(S.Dinv[r] * ((S.q[r] + R.Px[r]) + R.Aty[r])));
    if (j >= n) R.Px[r] = 0.0, R.Aty[r] = 0.0;
  }
  S.pri_res = wave_max(pr);
  S.dua_res = S.cinv * wave_max(dr);
  TSYNC(S.dua_res);
  T_END(T_RS4, t_r4);
}

template <int RN, int RM>
__device__ __forceinline__ bool is_primal_infeasible(const KParams& p, Inst<RN, RM>& S, double (&dy)[RM],
                                     const Slab& sb, const double (&Ev)[RM], double* v,
                                     const double* mv, int lane, double eps) {
  const DevPlan& P = p.pl;
  const double thr = OSQP_INFTY * MIN_SCALING;
  double nrm = 0.0;
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int i = lane + 64 * r;
    if (i < P.m) {
      if (S.u[r] > thr)
        dy[r] = (S.l[r] < -thr) ? 0.0 : dmind(dy[r], 0.0);
      else if (S.l[r] < -thr)
        dy[r] = dmaxd(dy[r], 0.0);
      nrm = dmaxd(nrm, fabs(Ev[r] * dy[r]));
    }
  }
  nrm = wave_max(nrm);
  if (!(nrm > DIVISION_TOL)) return false;
  // lhs = u' max(dy, 0) + l' min(dy, 0) < eps |dy|, decided on OSQP's sequential sum (the terms
  // staged in C, free during the checks; seq_sum_lt)
  double* stg = v + P.CACC;
  double part = 0.0, apart = 0.0;
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int i = lane + 64 * r;
    if (i < P.m) {
      const double t = S.u[r] * dmaxd(dy[r], 0.0) + S.l[r] * dmind(dy[r], 0.0);
      stg[i] = t;
      part = part + t, apart = apart + fabs(t);
    }
  }
  if (!seq_sum_lt(stg, P.m, wave_sum(part), wave_sum(apart), eps * nrm)) return false;
  double* yb = v + P.W + P.n;
  LDS_FENCE();
#pragma unroll
  for (int r = 0; r < RM; ++r) yb[lane + 64 * r] = dy[r];  // slots past m: W padding
  LDS_FENCE();
  // A' dy by the residual ELL (same term order as the CSC column traversal, loads batched)
  double aty[RN];
  ell_mv<RN, ELL_KAT>(P.eAt, mv, yb, aty, lane, v + P.CACC);
  double mx = 0.0;
#pragma unroll
  for (int r = 0; r < RN; ++r)
    if (lane + 64 * r < P.n) mx = dmaxd(mx, fabs(aty[r] * S.Dinv[r]));
  mx = wave_max(mx);
  return mx < eps * nrm;
}

template <int RN, int RM>
__device__ __forceinline__ bool is_dual_infeasible(const KParams& p, Inst<RN, RM>& S, const double (&dx)[RN],
                                   const Slab& sb, const double (&Dv)[RN], double* v,
                                   const double* mv, int lane, double eps) {
  const DevPlan& P = p.pl;
  const double thr = OSQP_INFTY * MIN_SCALING;
  double nrm = 0.0, part = 0.0, apart = 0.0;
  double* stg = v + P.CACC;  // q' dx (vec_prod) decided on OSQP's order, the products staged in C
#pragma unroll
  for (int r = 0; r < RN; ++r) {
    const int j = lane + 64 * r;
    if (j < P.n) {
      nrm = dmaxd(nrm, fabs(Dv[r] * dx[r]));
      const double t = S.q[r] * dx[r];
      stg[j] = t;
      part = part + t, apart = apart + fabs(t);
    }
  }
  nrm = wave_max(nrm);
  if (!(nrm > DIVISION_TOL)) return false;
  if (!seq_sum_lt(stg, P.n, wave_sum(part), wave_sum(apart), S.c * eps * nrm)) return false;
  double* xb = v + P.W;
  LDS_FENCE();
#pragma unroll
  for (int r = 0; r < RN; ++r) xb[lane + 64 * r] = dx[r];  // slots past n: inside the W region
  LDS_FENCE();
  // P dx and A dx by the residual ELLs (same term orders as the symmetric / CSR traversals)
  double pdx[RN];
  ell_mv<RN, ELL_KP>(P.eP, mv, xb, pdx, lane, v + P.CACC);
  double mx = 0.0;
#pragma unroll
  for (int r = 0; r < RN; ++r)
    if (lane + 64 * r < P.n) mx = dmaxd(mx, fabs(pdx[r] * S.Dinv[r]));
  mx = wave_max(mx);
  if (!(mx < S.c * eps * nrm)) return false;
  double adx[RM];
  ell_mv<RM, ELL_KA>(P.eA, mv, xb, adx, lane, v + P.CACC);
  int bad = 0;
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    if (lane + 64 * r < P.m) {
      const double s = adx[r] * S.Einv[r];
      if ((S.u[r] < thr && s > eps * nrm) || (S.l[r] > -thr && s < -eps * nrm)) bad = 1;
    }
  }
  return !__any(bad);
}

template <int RN, int RM>
__device__ __forceinline__ int check_termination(const KParams& p, Inst<RN, RM>& S, const Resid<RN, RM>& R,
                                 double (&dy)[RM], const double (&dx)[RN], const Slab& sb,
                                 double* v, const double* mv, int lane, bool approximate TACC_PARAM) {
  T_BEGIN(t_m0);
  const DevPlan& P = p.pl;
  // the scalings D, E of the infeasibility certificates: loaded first, in flight under the norms
  double Ev[RM], Dv[RN];
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int i = lane + 64 * r;
    Ev[r] = i < P.m ? sb.E[i] : 0.0;
  }
#pragma unroll
  for (int r = 0; r < RN; ++r) {
    const int j = lane + 64 * r;
    Dv[r] = j < P.n ? sb.D[j] : 0.0;
  }
  double eps_abs = p.s.eps_abs, eps_rel = p.s.eps_rel;
  double eps_pinf = p.s.eps_prim_inf, eps_dinf = p.s.eps_dual_inf;
  if (approximate) eps_abs *= 10, eps_rel *= 10, eps_pinf *= 10, eps_dinf *= 10;
  // compute_pri_tol / compute_dua_tol (unscaled termination)
  double zn = 0.0, axn = 0.0, qn = 0.0, atn = 0.0, pxn = 0.0;
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int i = lane + 64 * r;
    if (i < P.m) {
      const double ei = S.Einv[r];
      zn = dmaxd(zn, fabs(ei * S.z[r]));
      axn = dmaxd(axn, fabs(ei * R.Ax[r]));
    }
  }
#pragma unroll
  for (int r = 0; r < RN; ++r) {
    const int j = lane + 64 * r;
    if (j < P.n) {
      const double di = S.Dinv[r];
      qn = dmaxd(qn, fabs(di * S.q[r]));
      atn = dmaxd(atn, fabs(di * R.Aty[r]));
      pxn = dmaxd(pxn, fabs(di * R.Px[r]));
    }
  }
  zn = wave_max(zn), axn = wave_max(axn), qn = wave_max(qn), atn = wave_max(atn);
  pxn = wave_max(pxn);
  const double eps_prim = eps_abs + eps_rel * dmaxd(zn, axn);
  const double eps_dual = eps_abs + eps_rel * (dmaxd(dmaxd(qn, atn), pxn) * S.cinv);
  bool prim_ok = false, dual_ok = false, prim_inf = false, dual_inf = false;
  TSYNC(eps_dual);
  T_END(T_TM0, t_m0);
  T_BEGIN(t_m1);
  if (S.pri_res < eps_prim)
    prim_ok = true;
  else
    prim_inf = is_primal_infeasible(p, S, dy, sb, Ev, v, mv, lane, eps_pinf);
  T_END(T_TM1, t_m1);
  T_BEGIN(t_m2);
  if (S.dua_res < eps_dual)
    dual_ok = true;
  else
    dual_inf = is_dual_infeasible(p, S, dx, sb, Dv, v, mv, lane, eps_dinf);
  T_END(T_TM2, t_m2);
  if (prim_ok && dual_ok) return approximate ? MPCQP_SOLVED_INACCURATE : MPCQP_SOLVED;
  if (prim_inf) return approximate ? MPCQP_PRIMAL_INFEASIBLE_INACCURATE : MPCQP_PRIMAL_INFEASIBLE;
  if (dual_inf) return approximate ? MPCQP_DUAL_INFEASIBLE_INACCURATE : MPCQP_DUAL_INFEASIBLE;
  return 0;
}

// auxil.c compute_rho_estimate (residual vectors in scaled space)
template <int RN, int RM>
__device__ __forceinline__ double rho_estimate(const KParams& p, const Inst<RN, RM>& S, const Resid<RN, RM>& R,
                               int lane) {
  const DevPlan& P = p.pl;
  double pr = 0.0, zn = 0.0, axn = 0.0, dr = 0.0, qn = 0.0, atn = 0.0, pxn = 0.0;
#pragma unroll
  for (int r = 0; r < RM; ++r)
    if (lane + 64 * r < P.m) {
      pr = dmaxd(pr, fabs(R.Ax[r] - S.z[r]));
      zn = dmaxd(zn, fabs(S.z[r]));
      axn = dmaxd(axn, fabs(R.Ax[r]));
    }
#pragma unroll
  for (int r = 0; r < RN; ++r)
    if (lane + 64 * r < P.n) {
      dr = dmaxd(dr, fabs((S.q[r] + R.Px[r]) + R.Aty[r]));
      qn = dmaxd(qn, fabs(S.q[r]));
      atn = dmaxd(atn, fabs(R.Aty[r]));
      pxn = dmaxd(pxn, fabs(R.Px[r]));
    }
  pr = wave_max(pr), zn = wave_max(zn), axn = wave_max(axn);
  dr = wave_max(dr), qn = wave_max(qn), atn = wave_max(atn), pxn = wave_max(pxn);
  pr /= (dmaxd(zn, axn) + DIVISION_TOL);
  dr /= (dmaxd(dmaxd(qn, atn), pxn) + DIVISION_TOL);
  double est = S.rho * sqrt(pr / (dr + DIVISION_TOL));
  return dmind(dmaxd(est, RHO_MIN), RHO_MAX);
}

__device__ __forceinline__ bool has_solution(int st) {
  return st != MPCQP_PRIMAL_INFEASIBLE && st != MPCQP_PRIMAL_INFEASIBLE_INACCURATE &&
         st != MPCQP_DUAL_INFEASIBLE && st != MPCQP_DUAL_INFEASIBLE_INACCURATE &&
         st != MPCQP_NON_CVX;
}

// Ruiz equilibration (scaling.c scale_data) of the instance's P (shared values) and A, q, l, u:
// the passes.  Matrix values live in the LDS scaling overlay (S_P, S_A, D_temp, E_temp); the index
// lists the passes walk are copied into LDS once (the scaling index overlay, symbolic.hpp), so a
// pass is LDS traffic only.  The column / row norms use the padded ELL lists (max is order-free);
// padding entries read the zero slot S_ZERO, so no LDS read is conditional.  Returns D and E;
// q, l, u (scaled) and c are left in S.
template <int RN, int RM>
__device__ __forceinline__ void scale_problem(const KParams& p, int inst, const Drift& dr, Inst<RN, RM>& S,
                                              double* v, int lane, double (&D)[RN],
                                              double (&E)[RM] TACC_PARAM) {
  const DevPlan& P = p.pl;
  const int n = P.n, m = P.m;
  // P and q: the set-up data, or the unscaled values OSQP holds (drift_of)
  double* const Pw = dr.P_out;
  double* const qw = dr.q_out;
  const double* P_in = dr.P_in;
  const double* q_in = dr.q_in;
  const double* Ax_in = p.Ax + (size_t)inst * P.nnzA;
  const double* l_in = p.l + (size_t)inst * m;
  const double* u_in = p.u + (size_t)inst * m;
  // the passes' index lists in registers (shared structure arrays, loaded once per solve)
  EllIdx<RN, ELL_KP> iP;
  EllIdx<RN, ELL_KAT> iAt;
  EllIdx<RM, ELL_KA> iA;
  load_idx(P.eP, iP, lane);
  load_idx(P.eAt, iAt, lane);
  load_idx(P.eA, iA, lane);
  constexpr bool KF = RN == 2;
  const uint32_t kfP = KF ? ell_kflags<RN>(P.eP) : 0u, kfAt = KF ? ell_kflags<RN>(P.eAt) : 0u,
                 kfA = KF ? ell_kflags<RM>(P.eA) : 0u;
  constexpr int JW = 4 * RN;  // u16 pairs of row / column slots per lane (Plan::SJ <= 2 JW)
  uint32_t ra[JW], ca[JW];
  {
    const uint2* rr = reinterpret_cast<const uint2*>(P.sra + (size_t)lane * P.SJ);
    const uint2* cc = reinterpret_cast<const uint2*>(P.sca + (size_t)lane * P.SJ);
#pragma unroll
    for (int q = 0; q < JW / 2; ++q) {
      ra[2 * q] = ra[2 * q + 1] = ca[2 * q] = ca[2 * q + 1] = 0u;
      if (4 * q < P.SJ) {  // wave-uniform
        const uint2 a = rr[q], c = cc[q];
        ra[2 * q] = a.x, ra[2 * q + 1] = a.y, ca[2 * q] = c.x, ca[2 * q + 1] = c.y;
      }
    }
  }
  if (lane == 0) v[P.S_ZERO] = 0.0;
  load_vals(v, P.S_P, P_in, P.nnzP, lane);
  load_vals(v, P.S_A, Ax_in, P.nnzA, lane);
#pragma unroll
  for (int r = 0; r < RN; ++r) {
    const int j = lane + 64 * r;
    S.q[r] = j < n ? q_in[j] : 0.0;
    D[r] = 1.0;
  }
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int i = lane + 64 * r;
    S.l[r] = i < m ? dmaxd(l_in[i], -OSQP_INFTY) : 0.0;
    S.u[r] = i < m ? dmind(u_in[i], OSQP_INFTY) : 0.0;
    E[r] = 1.0;
  }
  S.c = 1.0;
  double cprev = 1.0;  // cost factor of the last pass, not yet applied to P's values
  double dpc[RN];      // P's column norms before that factor (the cost normalisation's)
  LDS_FENCE();
  for (int it = 0; it < p.s.scaling; ++it) {
    // (4, 8) bucket: the passes' operand addresses recomputed in every pass (hoisted out of the
    // pass loop they held ~190 registers: that kernel's register peak, MPCQP_MAX_KERNEL_REGS)
    if constexpr (RN >= 4) {
      opaque_idx(iP), opaque_idx(iAt), opaque_idx(iA);
      opaque_words(ra), opaque_words(ca);
    }
    // compute_inf_norm_cols_KKT: columns of [P A'; A 0] (P symmetric from its upper triangle).
    // After the first pass P's column norms are the cost normalisation's norms times its factor
    // c (still pending on P's values): max_k |c x_k| = c max_k |x_k| exactly, rounding being
    // monotonic (c > 0)
    double dp[RN], da[RN], er[RM], dt[RN], et[RM];
    T_BEGIN(t_s0);
    if (it == 0) {
      ell_absmax_r<KF>(P.eP, iP, kfP, v, dp, lane);
    } else {
#pragma unroll
      for (int r = 0; r < RN; ++r) dp[r] = cprev * dpc[r];
    }
    ell_absmax_r<KF>(P.eAt, iAt, kfAt, v, da, lane);
    ell_absmax_r<KF>(P.eA, iA, kfA, v, er, lane);
    TSYNC(er[RM - 1]);
    T_END(T_SC0, t_s0);
    T_BEGIN(t_s1);
#pragma unroll
    for (int r = 0; r < RN; ++r) {
      const int j = lane + 64 * r;
      const double d = j < n ? dmaxd(dp[r], da[r]) : 0.0;
      dt[r] = 1. / sqrt(limit_scaling(d));
      if (j < n) v[P.S_DT + j] = dt[r];
    }
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      const int i = lane + 64 * r;
      const double e = i < m ? er[r] : 0.0;
      et[r] = 1. / sqrt(limit_scaling(e));
      if (i < m) v[P.S_ET + i] = et[r];
    }
    LDS_FENCE();
    TSYNC(et[RM - 1]);
    T_END(T_SC1, t_s1);
    T_BEGIN(t_s2);
    scale_pa_r(v, P.S_P, P.nnzP, P.nnzP + P.nnzA, ra, ca, cprev, lane);
#pragma unroll
    for (int r = 0; r < RN; ++r) {
      S.q[r] = dt[r] * S.q[r];
      D[r] = D[r] * dt[r];
    }
#pragma unroll
    for (int r = 0; r < RM; ++r) E[r] = E[r] * et[r];
    LDS_FENCE();
    TSYNC(E[RM - 1]);
    T_END(T_SC2, t_s2);
    T_BEGIN(t_s3);
    // cost normalization: mean of P's column norms, |q|_inf
    ell_absmax_r<KF>(P.eP, iP, kfP, v, dpc, lane);
    // vec_mean of the column norms, summed in index order (staged in the D_temp slots: this
    // pass's factors are consumed) -- unless a tree sum shows it below |q|_inf by more than the
    // summation orders can differ (sum_slack; the norms are >= 0): then max(mean, |q|_inf) does
    // not depend on it
    double qmax = 0.0, csum = 0.0;
#pragma unroll
    for (int r = 0; r < RN; ++r) {
      const int j = lane + 64 * r;
      if (j < n) {
        v[P.S_DT + j] = dpc[r];
        csum = csum + dpc[r];
        qmax = dmaxd(qmax, fabs(S.q[r]));
      }
    }
    const double inq = limit_scaling(wave_max(qmax));
    const double T = wave_sum(csum);
    double c_temp = inq;
    if (!((T + sum_slack(T, n)) / n < inq)) {
      LDS_FENCE();
      c_temp = seq_sum(v + P.S_DT, n) / n;
      LDS_FENCE();
      T_COUNT(T_SCC);
    }
    c_temp = limit_scaling(dmaxd(c_temp, inq));
    c_temp = 1. / c_temp;
    cprev = c_temp;  // P *= c_temp: applied by the next rescale pass (or below, after the last)
#pragma unroll
    for (int r = 0; r < RN; ++r) S.q[r] = S.q[r] * c_temp;
    S.c = S.c * c_temp;
    LDS_FENCE();
    TSYNC(S.c);
    T_END(T_SC3, t_s3);
  }
  for (int k = lane; k < P.nnzP; k += 64) v[P.S_P + k] = v[P.S_P + k] * cprev;
  LDS_FENCE();
  // the next solve's data (scaling.c unscale_data): q <- (q c^-1) D^-1, P <- ((P c^-1) D^-1) D^-1
  // with D^-1 = 1 / D and c^-1 = 1 / c as scale_data leaves them; D^-1 staged in the D_temp slots
  // for the row / column operands of scale_pa_r's layout
  const double cinv = 1. / S.c;
#pragma unroll
  for (int r = 0; r < RN; ++r) {
    const int j = lane + 64 * r;
    const double di = 1. / D[r];
    if (j < n) {
      v[P.S_DT + j] = di;
      qw[j] = (S.q[r] * cinv) * di;
    }
  }
  LDS_FENCE();
  unscale_p_r(v, P.S_P, P.nnzP, ra, ca, cinv, lane, Pw);
}

// end of scale_data: constraint classes, scaled bounds, D / E into the per-wave slab, and the
// scaled values [P | A] copied from the scaling overlay into the resident MV region of the image
// (read from there by the residual mat-vecs, certificates, KKT (re)assembly and the objective)
template <int RN, int RM>
__device__ __forceinline__ void scale_finish(const KParams& p, int inst, bool rebound, Inst<RN, RM>& S,
                                             const Slab& sb, double* v, double* mvw, int lane,
                                             const double (&D)[RN], const double (&E)[RM]) {
  const DevPlan& P = p.pl;
  const int n = P.n, m = P.m;
  S.cinv = 1. / S.c;
  // constraint classes (auxil.c set_rho_vec / update_rho_vec): after an update of A OSQP
  // classifies on bounds scaled by the PREVIOUS equilibration (update_bounds precedes the rescale
  // of update_A); otherwise by the current one (which a bounds-only update keeps).
  const double thr = OSQP_INFTY * MIN_SCALING;
  const double* Eold = p.Ecls + (size_t)inst * m;
  S.ct = 0;
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int i = lane + 64 * r;
    const double ec = (rebound && i < m) ? Eold[i] : E[r];
    const double lc = S.l[r] * ec, uc = S.u[r] * ec;
    const uint32_t t = (lc < -thr && uc > thr) ? CT_FREE : ((uc - lc < RHO_TOL) ? CT_EQ : CT_INEQ);
    S.ct |= t << (2 * r);
    // after an update of A: the bounds as OSQP leaves them, scaled by the previous E
    // (update_bounds), unscaled by its inverse and rescaled by the new E (update_A's unscale_data /
    // scale_data); a bounds-only update scales them by the kept E once
    const double eci = 1. / ec;
    const double lb = rebound ? lc * eci : S.l[r], ub = rebound ? uc * eci : S.u[r];
    S.l[r] = lb * E[r];
    S.u[r] = ub * E[r];
    S.Einv[r] = 1. / E[r];
    if (i < m) sb.E[i] = E[r];
  }
#pragma unroll
  for (int r = 0; r < RN; ++r) {
    const int j = lane + 64 * r;
    S.Dinv[r] = 1. / D[r];
    if (j < n) sb.D[j] = D[r];
  }
  // the scaled values [P | A] stay resident in LDS (MV) for the residuals, certificates,
  // (re)assembly and objective; the scaling overlay they come from is overwritten by the KKT image
  LDS_FENCE();
  {
    const int cnt = P.nnzP + P.nnzA;
    constexpr int U = 8;
    for (int k0 = 0; k0 < cnt; k0 += 64 * U) {
      double x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + 64 * u + lane;
        x[u] = v[P.S_P + (k < cnt ? k : 0)];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + 64 * u + lane;
        if (k < cnt) mvw[P.MV + k] = x[u];
      }
    }
    if (lane == 0) mvw[P.MVZ] = 0.0;
  }
  LDS_FENCE();
  // global slab copy (Plan::mv_global): other lanes read these values back -- the stores must be
  // complete and visible to the wave's later loads (workgroup-scope release/acquire)
  if (P.mv_slab) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

// Register buckets from which the per-lane addresses get an opaque lane id per instance (and per
// check) instead of being hoisted out of the persistent instance loop: all of them (2).  Hoisted,
// the addresses of the RN = 2 kernel held ~100 registers across the loop (256 + 154 allocated vs
// 256 + 50 now, same speed) -- and builds with more register pressure computed wrong results from
// the second instance a wave takes onward, with every first instance bit-exact (DESIGN.md,
// High-register builds; tools/cliff_localize.py).  Diagnostics may raise it (4: round-3/4 builds).
#ifndef MPCQP_OPAQUE_LANE_RN
#define MPCQP_OPAQUE_LANE_RN 2
#endif
// kernel modes of the one-wave kernel: KM_LDS the solve steps read both operands from LDS;
// KM_MATPF matrix operands one step ahead (diagnostic, rejected); KM_MVG the resident scaled values
// in the wave's global slab (Plan::mv_global); KM_MREG matrix operands in registers (MatRegs)
enum { KM_LDS = 0, KM_MATPF = 1, KM_MVG = 2, KM_MREG = 3 };
template <int RN, int RM, bool PAIRED, int KM>
__device__ __forceinline__ void solve_instance(const KParams& p, int inst, double* v, double* scr,
                                               int lane) {
  constexpr bool MATPF = KM == KM_MATPF, MVG = KM == KM_MVG, MREG = KM == KM_MREG;
  const DevPlan& P = p.pl;
  const int n = P.n, m = P.m;
  const Slab sb = slab_of(P, scr);
  double* const mv = MVG ? sb.MV : v;
  Inst<RN, RM> S;
  const int hs = p.has_state[inst];
  const Drift dr = drift_of(p, inst);
#ifdef MPCQP_TIMING
  unsigned long long tacc[T_NSLOT] = {};
#endif
  T_BEGIN(t_sc);
  {
    double D[RN], E[RM];
    scale_problem<RN, RM>(p, inst, dr, S, v, lane, D, E TACC_ARG);
    T_BEGIN(t_sf);
    scale_finish<RN, RM>(p, inst, dr.rebound, S, sb, v, mv, lane, D, E);
    // the drift state after this solve, stored once the scaling has read it (kept to the end of
    // the solve it was an SGPR live across the ADMM loop; the two-wave kernel's other wave has
    // read it before the scaling's barriers)
    if (lane == 0) {
      p.dsel[inst] = dr.sel;
      p.pend[inst] = 0;
    }
    T_END(T_SCFIN, t_sf);
  }
  T_END(T_SCALE, t_sc);
  S.rho = (hs != 0) ? p.rho_state[inst] : p.rho0;
  set_rho(S);
  T_BEGIN(t_f0);
  MatRegs M;  // KM_MREG: the solve steps' matrix operands of the current factorization
  assemble_and_factor<RN, RM>(p, sb, v, mv, lane, S);
  if constexpr (MREG) {
    LDS_FENCE();
    load_mats(P.fwdm, P.nfwd, (uint32_t)lane, v, M.m[0]);
    load_mats(P.bwdm, P.nbwd, (uint32_t)lane, v, M.m[1]);
  }
  T_END(T_FACTOR, t_f0);
  T_COUNT(T_NFACT);

  // ---------------- warm start
  const bool warm = p.s.warm_start && hs != 0;
  if (warm && hs == 1) {
#pragma unroll
    for (int r = 0; r < RN; ++r) {
      const int j = lane + 64 * r;
      S.x[r] = j < n ? p.xs[(size_t)inst * n + j] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      const int i = lane + 64 * r;
      S.z[r] = i < m ? p.zs[(size_t)inst * m + i] : 0.0;
      S.y[r] = i < m ? p.ys[(size_t)inst * m + i] : 0.0;
    }
  } else if (warm && hs == 2) {  // osqp_warm_start: scale the user guess, z = A x
#pragma unroll
    for (int r = 0; r < RN; ++r) {
      const int j = lane + 64 * r;
      S.x[r] = j < n ? S.Dinv[r] * p.xs[(size_t)inst * n + j] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      const int i = lane + 64 * r;
      S.y[r] = i < m ? (S.Einv[r] * p.ys[(size_t)inst * m + i]) * S.c : 0.0;
    }
    double* xb = v + P.W;
    LDS_FENCE();
#pragma unroll
    for (int r = 0; r < RN; ++r)
      if (lane + 64 * r < n) xb[lane + 64 * r] = S.x[r];
    LDS_FENCE();
    double az[RM];
    ell_mv<RM, ELL_KA>(P.eA, mv, xb, az, lane, v + P.CACC);  // CSR row order
#pragma unroll
    for (int r = 0; r < RM; ++r) S.z[r] = lane + 64 * r < m ? az[r] : 0.0;
    LDS_FENCE();
  } else {
#pragma unroll
    for (int r = 0; r < RN; ++r) S.x[r] = 0.0;
#pragma unroll
    for (int r = 0; r < RM; ++r) S.z[r] = 0.0, S.y[r] = 0.0;
  }
  S.pri_res = S.dua_res = 0.0;

  // ---------------- ADMM (osqp.c osqp_solve)
  // LDS slots of this lane's x / z entries in the permuted solve vector (kept in registers); lanes
  // past the end of x or z have their own W padding slot, zeroed every iteration and read back as 0
  int wsx[RN], wsz[RM];
#pragma unroll
  for (int r = 0; r < RN; ++r) wsx[r] = (int)P.wsx[lane + 64 * r];
#pragma unroll
  for (int r = 0; r < RM; ++r) wsz[r] = (int)P.wsz[lane + 64 * r];
  // rhs goes to the accumulator region C, the solution comes back in W; C follows W at a distance
  // of NKP = 64 (RN + RM) doubles (symbolic.cpp relocate), a compile-time constant: the stores'
  // immediate offset, so no second address register per slot
  constexpr int coff = 64 * (RN + RM);
  const uint32_t wcp = P.wcopy[lane], bcp = P.bcopy[lane];
  // the copy-row selections as word masks in VGPRs (W start = value AND mask: the value or +0.0,
  // bitwise the select it replaces).  Held as compare results they were SGPR pairs spilled to VGPR
  // lanes, two readlanes per slot and pass in the loop (927k vs 925k solves/s)
  // The (4, 8) bucket re-derives each mask at its use from the lane's bit word (one v_bfe_i32 on an
  // opaque per-iteration copy, so it is not hoisted back into registers): 24 VGPRs fewer, which
  // keeps that kernel inside the validated register budget (MPCQP_MAX_KERNEL_REGS)
  constexpr bool MASK_REGS = RN < 4;
  constexpr int NMK = MASK_REGS ? RN + RM : 1;
  uint32_t wmk[NMK], bmk[NMK];
#pragma unroll
  for (int r = 0; r < NMK; ++r) {
    wmk[r] = 0u - ((wcp >> r) & 1u);
    bmk[r] = 0u - ((bcp >> r) & 1u);
    asm volatile("" : "+v"(wmk[r]), "+v"(bmk[r]));
  }
  auto slot_mask = [&](const uint32_t (&arr)[NMK], uint32_t bits, int r) -> uint32_t {
    if constexpr (MASK_REGS) return arr[r];
    return (uint32_t)((int32_t)(bits << (31 - r)) >> 31);
  };
  auto and_d = [](double x, uint32_t mk) {
    return __hiloint2double((int)((uint32_t)__double2hiint(x) & mk), (int)((uint32_t)__double2loint(x) & mk));
  };
  // loop constants held in VGPRs (an opaque copy: otherwise they are re-read from the kernel
  // arguments inside the loop, with an lgkmcnt(0) wait that also drains the LDS queue)
  double sigma = p.s.sigma, alpha = p.s.alpha, alpha_c = 1.0 - p.s.alpha;
  asm volatile("" : "+v"(sigma), "+v"(alpha), "+v"(alpha_c));
  const int chk = p.s.check_termination;
  int ar_int = p.s.adaptive_rho_interval;
  if (p.s.adaptive_rho && ar_int == 0) ar_int = chk ? 4 * chk : 100;
  if (!p.s.adaptive_rho) ar_int = 0;
  int chk_left = chk, ar_left = ar_int;  // iterations to the next check / rho adaptation
  int status = MPCQP_UNSOLVED, iter = 0, rho_updates = 0;
  bool can_check = false;
  double dx[RN], dy[RM];
  Resid<RN, RM> R;
  Pipe<SolveOps<PAIRED>> sp;
  PipeC spc;
  const SolveOps<PAIRED> sops{v};
  const Rsrc rs_fwd = MREG ? table_rsrc(P.fwdc, P.nfwd, SOLVEC_STEP_WORDS)
                           : table_rsrc(P.fwd, P.nfwd, SOLVE_STEP_WORDS);
  const Rsrc rs_bwd = MREG ? table_rsrc(P.bwdc, P.nbwd, SOLVEC_STEP_WORDS)
                           : table_rsrc(P.bwd, P.nbwd, SOLVE_STEP_WORDS);
  // the diagonal pass's 1/D in registers between factorizations ((2, 4) bucket: 12 VGPRs; six
  // LDS reads fewer per iteration)
  constexpr bool DREG = RN == 2 && !MREG;
  double dvr[DREG ? RN + RM : 1];
  auto load_dinv = [&](int ln) {
    if constexpr (DREG) {
      LDS_FENCE();
#pragma unroll
      for (int r = 0; r < RN + RM; ++r) dvr[r] = v[P.DINV + ln + 64 * r];
    }
  };
  load_dinv(lane);
  // the loop bounds as opaque SGPR values: not rematerialised from the kernel arguments at the
  // loop head (an s_load whose lgkmcnt(0) wait also drains the LDS queue, every iteration)
  int max_iter = p.s.max_iter;
  int chk_s = chk, ar_s = ar_int;
  asm volatile("" : "+s"(max_iter), "+s"(chk_s), "+s"(ar_s));
  for (iter = 1; iter <= max_iter; ++iter) {
    T_COUNT(T_ITERS);
    T_BEGIN(t_v0);
    if constexpr (MREG)  // lands while the right-hand side is formed
      prefetch_c(rs_fwd, P.nfwd, (uint32_t)lane, spc);
    else
      prefetch(rs_fwd, P.nfwd, (uint32_t)lane, sp);
    double xp[RN], zp[RM], bz[RM];
    uint32_t wbits = wcp, bbits = bcp;  // opaque per iteration (slot_mask)
    if constexpr (!MASK_REGS) asm volatile("" : "+v"(wbits), "+v"(bbits));
    // right-hand side [sigma x - q ; z - rho^-1 y] into the permuted solve vector
    // (lanes past the end of x or z store to the junk slot: no lane masks in the loop)
    // The forward solve accumulates into W, which starts at 0 except on the copy rows
    // (Plan::wcopy: W_r = rhs_r, no solve task); the lanes' slots cover all of W
#pragma unroll
    for (int r = 0; r < RN; ++r) {
      xp[r] = S.x[r];
      const double b = fma(sigma, xp[r], -S.q[r]);
      v[wsx[r] + coff] = b;
      v[wsx[r]] = and_d(b, slot_mask(wmk, wbits, r));
    }
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      zp[r] = S.z[r];
      bz[r] = fma(-rinv_of(S, r), S.y[r], zp[r]);
      v[wsz[r] + coff] = bz[r];
      v[wsz[r]] = and_d(bz[r], slot_mask(wmk, wbits, RN + r));
    }
    LDS_FENCE();
    T_END(T_VEC, t_v0);
    T_END(T_V0, t_v0);
    T_BEGIN(t_fw);
    if constexpr (MREG)
      run_body_r<PAIRED>(rs_fwd, P.nfwd, (uint32_t)lane, v, spc, M.m[0]);
    else if constexpr (MATPF)
      run_body_pf<PAIRED>(rs_fwd, P.nfwd, (uint32_t)lane, v, sp);
    else
      run_body(rs_fwd, P.nfwd, (uint32_t)lane, sops, sp);
    T_END(T_FWD, t_fw);
    T_BEGIN(t_v1);
    if constexpr (MREG)  // lands during the diagonal pass
      prefetch_c(rs_bwd, P.nbwd, (uint32_t)lane, spc);
    else
      prefetch(rs_bwd, P.nbwd, (uint32_t)lane, sp);
    {
      // C = (1/D) W; W restarts at 0, or at C where the row's identity term is folded into it
      // (Plan::bcopy: the backward task has no MONE term)
      double wv[RN + RM], dv[RN + RM];
#pragma unroll
      for (int r = 0; r < RN + RM; ++r) {
        wv[r] = v[P.W + lane + 64 * r];
        if constexpr (DREG)
          dv[r] = dvr[r];
        else
          dv[r] = v[P.DINV + lane + 64 * r];
      }
#pragma unroll
      for (int r = 0; r < RN + RM; ++r) {  // C at the immediate distance coff: one ds_write2st64
        const double c = wv[r] * dv[r];
        v[P.W + lane + 64 * r + coff] = c;
        v[P.W + lane + 64 * r] = and_d(c, slot_mask(bmk, bbits, r));
      }
    }
    LDS_FENCE();
    T_END(T_VEC, t_v1);
    T_END(T_V1, t_v1);
    T_BEGIN(t_bw);
    if constexpr (MREG)
      run_body_r<PAIRED>(rs_bwd, P.nbwd, (uint32_t)lane, v, spc, M.m[1]);
    else if constexpr (MATPF)
      run_body_pf<PAIRED>(rs_bwd, P.nbwd, (uint32_t)lane, v, sp);
    else
      run_body(rs_bwd, P.nbwd, (uint32_t)lane, sops, sp);
    T_END(T_BWD, t_bw);
    T_BEGIN(t_v2);
    // x, z, y updates (auxil.c update_x / update_z / update_y).  The solution reads are issued
    // together before any use (otherwise the compiler reuses one register pair for all of them
    // and waits for each read in turn)
    double wx[RN], wz[RM];
#pragma unroll
    for (int r = 0; r < RN; ++r) wx[r] = v[wsx[r]];  // the junk slot reads back 0
#pragma unroll
    for (int r = 0; r < RM; ++r) wz[r] = v[wsz[r]];
    __builtin_amdgcn_sched_group_barrier(0x100, RN + RM, 0);
#pragma unroll
    for (int r = 0; r < RN; ++r) {
      const double xt = wx[r];
      S.x[r] = fma(alpha, xt, alpha_c * xp[r]);
      dx[r] = S.x[r] - xp[r];
    }
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      const double nu = wz[r];
      const double ri = rinv_of(S, r);
      const double zt = fma(ri, nu, bz[r]);
      const double zr = fma(alpha, zt, alpha_c * zp[r]);
      S.z[r] = dmind(dmaxd(fma(ri, S.y[r], zr), S.l[r]), S.u[r]);
      dy[r] = rvec_of(S, r) * (zr - S.z[r]);
      S.y[r] = S.y[r] + dy[r];
    }
    LDS_FENCE();
    T_END(T_VEC, t_v2);
    T_END(T_V2, t_v2);
    T_BEGIN(t_ck);
    can_check = chk_s && --chk_left == 0;  // iter % chk == 0
    if (can_check) chk_left = chk_s;
    const bool adapt = ar_s && --ar_left == 0;  // iter % ar_int == 0
    if (adapt) ar_left = ar_s;
    // the check-time code gets an opaque copy of the lane id: its per-lane addresses are
    // recomputed at each check instead of being hoisted out of the ADMM loop into registers (at
    // RN = 4 the hoisted addresses spilled to scratch; MPCQP_OPAQUE_LANE_RN above)
    int clane = lane;
    if constexpr (RN >= MPCQP_OPAQUE_LANE_RN) asm volatile("" : "+v"(clane));
    if (can_check || adapt) {
      T_BEGIN(t_rs);
      compute_residuals(p, S, R, sb, v, mv, clane TACC_ARG);
      T_END(T_RESID, t_rs);
      T_COUNT(T_NCHK);
    }
    if (can_check) {
      T_BEGIN(t_tm);
      status = check_termination(p, S, R, dy, dx, sb, v, mv, clane, false TACC_ARG);
      T_END(T_TERM, t_tm);
      if (status != 0) break;
      status = MPCQP_UNSOLVED;
    }
    T_BEGIN(t_ad);
    if (adapt) {
      const double rho_new = rho_estimate(p, S, R, clane);
      if (rho_new > S.rho * p.s.adaptive_rho_tolerance ||
          rho_new < S.rho / p.s.adaptive_rho_tolerance) {
        S.rho = dmind(dmaxd(rho_new, RHO_MIN), RHO_MAX);
        set_rho(S);
        rho_updates++;
        LDS_FENCE();
        T_BEGIN(t_f1);
        assemble_and_factor<RN, RM>(p, sb, v, mv, clane, S);
        if constexpr (MREG) {
          LDS_FENCE();
          load_mats(P.fwdm, P.nfwd, (uint32_t)clane, v, M.m[0]);
          load_mats(P.bwdm, P.nbwd, (uint32_t)clane, v, M.m[1]);
        }
        load_dinv(clane);
#ifdef MPCQP_TIMING
        const unsigned long long dt_f1 = __builtin_amdgcn_s_memtime() - t_f1;
        tacc[T_FACTOR] += dt_f1;
        tacc[T_CHECK] -= dt_f1;  // the check slot excludes the refactorization
        tacc[T_ADAPT] -= dt_f1;
        tacc[T_RS2] -= dt_f1;
#endif
        T_COUNT(T_NFACT);
      }
    }
    T_END(T_ADAPT, t_ad);
    T_END(T_CHECK, t_ck);
#ifdef MPCQP_TIMING
    // the check slot split: iterations that run the residuals (check or rho adaptation) / the rest
    tacc[(can_check || adapt) ? T_RS2 : T_RS3] += __builtin_amdgcn_s_memtime() - t_ck;
#endif
  }
  T_BEGIN(t_tl);
  if (!can_check) {
    iter = iter - 1;
    compute_residuals(p, S, R, sb, v, mv, lane TACC_ARG);
    status = check_termination(p, S, R, dy, dx, sb, v, mv, lane, false TACC_ARG);
    if (status == 0) status = MPCQP_UNSOLVED;
  }
  if (iter > p.s.max_iter) iter = p.s.max_iter;
  if (status == MPCQP_UNSOLVED) {
    const int st = check_termination(p, S, R, dy, dx, sb, v, mv, lane, true TACC_ARG);
    status = st ? st : MPCQP_MAX_ITER_REACHED;
  }

  // ---------------- objective (compute_obj_val) and store_solution
  const bool sol = has_solution(status);
  double obj = 0.0;
  if (sol) {
    double* xb = v + P.W;
    LDS_FENCE();
#pragma unroll
    for (int r = 0; r < RN; ++r)
      if (lane + 64 * r < n) xb[lane + 64 * r] = S.x[r];
    LDS_FENCE();
    double part = 0.0;
    for (int k = lane; k < P.nnzP; k += 64) {
      const int i = P.Pi[k], j = P.Pcol[k];
      const double pk = mv[P.MV + k];
      part += (i == j) ? .5 * pk * xb[i] * xb[i] : pk * xb[i] * xb[j];
    }
#pragma unroll
    for (int r = 0; r < RN; ++r)
      if (lane + 64 * r < n) part += S.q[r] * S.x[r];
    obj = wave_sum(part) * S.cinv;
  } else if (status == MPCQP_PRIMAL_INFEASIBLE || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE) {
    obj = OSQP_INFTY;
  } else if (status == MPCQP_DUAL_INFEASIBLE || status == MPCQP_DUAL_INFEASIBLE_INACCURATE) {
    obj = -OSQP_INFTY;
  }
  const double qnan = __builtin_nan("");
#pragma unroll
  for (int r = 0; r < RN; ++r) {
    const int j = lane + 64 * r;
    if (j < n) {
      if (p.x_out) p.x_out[(size_t)inst * n + j] = sol ? sb.D[j] * S.x[r] : qnan;
      p.xs[(size_t)inst * n + j] = sol ? S.x[r] : 0.0;
    }
  }
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int i = lane + 64 * r;
    if (i < m) {
      const double Ei = sb.E[i];
      if (p.y_out) p.y_out[(size_t)inst * m + i] = sol ? (Ei * S.y[r]) * S.cinv : qnan;
      p.zs[(size_t)inst * m + i] = sol ? S.z[r] : 0.0;
      p.ys[(size_t)inst * m + i] = sol ? S.y[r] : 0.0;
      p.Ecls[(size_t)inst * m + i] = Ei;
    }
  }
  T_END(T_TAIL, t_tl);
#ifdef MPCQP_TIMING
  if (lane == 0 && p.timing)
    for (int k = 0; k < T_NSLOT; ++k) atomicAdd(p.timing + k, tacc[k]);
#endif
  if (lane == 0) {
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

// One wave per workgroup; the instance image is the workgroup's whole (dynamic) LDS, at address 0.
// MPCQP_WAVES_PER_EU: minimum waves per SIMD the register allocation must allow (1: up to 512
// VGPRs + AGPRs per lane; 2: at most 256).  The MVG build (resident values in the global slab, 5
// instances per CU at N = 20) always allows two: one SIMD of the CU then runs two of the waves.
#ifndef MPCQP_WAVES_PER_EU
#define MPCQP_WAVES_PER_EU 1
#endif
template <int RN, int RM, bool PAIRED, int KM>
__global__ void __launch_bounds__(64, KM == KM_MVG ? 2 : MPCQP_WAVES_PER_EU) qp_batch_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = (int)threadIdx.x;
  if ((uint32_t)(uintptr_t)lds != 0u) __builtin_trap();  // schedule byte addresses assume base 0
  double* v = lds;
  double* scr = p.scratch + (size_t)blockIdx.x * slab_doubles(p.pl);
  for (;;) {
    unsigned int inst = 0;
    if (lane == 0) inst = atomicAdd(p.counter, 1u);
    inst = (unsigned int)__shfl((int)inst, 0);
    inst = __builtin_amdgcn_readfirstlane(inst);
    if (inst >= (unsigned int)p.B) break;
    if (p.order) {
      inst = __builtin_amdgcn_readfirstlane((unsigned int)p.order[inst]);
      if (inst >= (unsigned int)p.B) continue;  // not a permutation entry: nothing to solve
    }
    if (p.skip && p.skip[inst]) continue;  // wave-uniform
    // an opaque copy of the lane id per instance, so per-lane address arithmetic is not hoisted
    // out of the instance loop (MPCQP_OPAQUE_LANE_RN above)
    int ilane = lane;
    if constexpr (RN >= MPCQP_OPAQUE_LANE_RN) asm volatile("" : "+v"(ilane));
    solve_instance<RN, RM, PAIRED, KM>(p, (int)inst, v, scr, ilane);
    LDS_FENCE();
  }
}

// record sets in flight of the two-wave kernel's first wave (Pipe; MPCQP_PAIR_PIPE=3 for A/B)
#ifndef MPCQP_PAIR_PIPE
#define MPCQP_PAIR_PIPE 4
#endif
constexpr int PAIR_PIPE = MPCQP_PAIR_PIPE;
#include "engine_pair.inc"

// dst[b][k] = src[k] for every instance b (the drift buffers' start: set_data, update_lin_cost)
__global__ void bcast_rows_kernel(double* dst, const double* src, int B, int cnt) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < (size_t)B * cnt) dst[t] = src[t % (size_t)cnt];
}

// dst[b][k] = the unscaled data the instance's next update of A rescales (drift_of): buffer 1 - dsel
// (dsel 0), buffer 0 (dsel -1 / 1), the shared set-up data (never scaled)
__global__ void drift_gather_kernel(double* dst, const double* W, const double* shared,
                                    const int32_t* dsel, int B, int cnt) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)B * cnt) return;
  const size_t b = t / (size_t)cnt, k = t % (size_t)cnt;
  const int sel = dsel[b];
  dst[t] = sel == -2 ? shared[k] : W[(sel == 0 ? (size_t)B * cnt : 0) + t];
}

// ---------------------------------------------------------------------------------------- host
int fail(int code, const std::string& msg) { return set_error(code, msg); }
#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) return fail(MPCQP_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

typedef void (*kernel_fn)(KParams);

// block caps of the blocked substitution (symbolic.hpp); MPCQP_CAPM / MPCQP_CAPW override them.
// Every MPCQP_* override below is a diagnostic: honoured only with MPCQP_DIAGNOSTICS=1 (diag_env)
int env_int(const char* name, int dflt) { return diag_env_int(name, dflt); }

template <int RN, int RM>
kernel_fn pick(bool paired, int waves, bool matpf, bool mvg, bool mreg) {
  // two waves, the solve steps on the first; MPCQP_W0DIAG=1: the diagonal pass too (mode 3,
  // measured equal to mode 2 at N = 40)
  if (waves == 3)
    return env_int("MPCQP_W0DIAG", 0)
               ? (paired ? qp_pair_kernel<RN / 2, RM / 2, true, 3> : qp_pair_kernel<RN / 2, RM / 2, false, 3>)
               : (paired ? qp_pair_kernel<RN / 2, RM / 2, true, 2> : qp_pair_kernel<RN / 2, RM / 2, false, 2>);
  if (waves == 2) {
    if (matpf)
      return paired ? qp_pair_kernel<RN / 2, RM / 2, true, 1> : qp_pair_kernel<RN / 2, RM / 2, false, 1>;
    return paired ? qp_pair_kernel<RN / 2, RM / 2, true, 0> : qp_pair_kernel<RN / 2, RM / 2, false, 0>;
  }
  if (mvg || mreg) {  // instantiated for the (2, 4) bucket only (the planner offers them there alone)
    if constexpr (RN == 2) {
      if (matpf || (mvg && mreg)) return nullptr;
      if (mreg)
        return paired ? qp_batch_kernel<RN, RM, true, KM_MREG> : qp_batch_kernel<RN, RM, false, KM_MREG>;
      return paired ? qp_batch_kernel<RN, RM, true, KM_MVG> : qp_batch_kernel<RN, RM, false, KM_MVG>;
    }
    return nullptr;
  }
  if (matpf)
    return paired ? qp_batch_kernel<RN, RM, true, KM_MATPF> : qp_batch_kernel<RN, RM, false, KM_MATPF>;
  return paired ? qp_batch_kernel<RN, RM, true, KM_LDS> : qp_batch_kernel<RN, RM, false, KM_LDS>;
}

// RN = ceil(n/64) and RM = ceil(m/64) rounded up to the instantiated buckets; the plan's step kind
// and waves per instance
kernel_fn select_kernel(int n, int m, bool paired, int waves, bool matpf, bool mvg, bool mreg) {
  int rn = 0, rm = 0;
  if (!kernel_bucket(n, m, rn, rm)) return nullptr;
#ifdef MPCQP_DEV20
  // diagnostic A/B builds only (tools/dev20.sh): the N = 20 product kernel alone, a 30 s compile
  // (-DMPCQP_DEV40: the N = 40 two-wave product kernel beside it)
#ifdef MPCQP_DEV40
  if (rn == 4 && waves == 3 && !matpf && !mvg && !mreg)
    return paired ? qp_pair_kernel<2, 4, true, 2> : qp_pair_kernel<2, 4, false, 2>;
#endif
  if (rn != 2 || waves != 1 || matpf || mvg || mreg) return nullptr;
  return paired ? qp_batch_kernel<2, 4, true, KM_LDS> : qp_batch_kernel<2, 4, false, KM_LDS>;
#else
  if (rn == 2) return pick<2, 4>(paired, waves, matpf, mvg, mreg);
#ifndef MPCQP_ONLY_SMALL
  if (rn == 4) return pick<4, 8>(paired, waves, matpf, mvg, mreg);
#endif
  return nullptr;
#endif
}

// Matrix operands of the solve steps in registers (KM_MREG): one-wave plans of the (2, 4) bucket
// whose forward and backward solves take at most MREG_STEPS steps each.  MPCQP_MREG=0/1 forces it
// off / on (diagnostics).
constexpr int MREG_DEFAULT = 0;
bool use_mreg(const Plan& pl) {
  int rn = 0, rm = 0;
  const bool fits = pl.waves == 1 && !pl.mat_first && !pl.mv_global && pl.nfwd <= MREG_STEPS &&
                    pl.nbwd <= MREG_STEPS && kernel_bucket(pl.n, pl.m, rn, rm) && rn == 2;
  return fits && env_int("MPCQP_MREG", MREG_DEFAULT) != 0;
}
// the KM_MREG record tables from the plan's solve records: per step, the terms' vector addresses
// (the operand in the W or C region) + the targets (SolveRecC), and the terms' matrix addresses
// (every other operand: L, N | G | G', ZERO / ONE / MONE); a padding term (both operands zero
// slots) reads its matrix zero from the first and its vector zero from the second
void split_records(const Plan& pl, const std::vector<uint32_t>& rec, int nsteps,
                   std::vector<uint32_t>& vec, std::vector<uint32_t>& mat) {
  auto is_vec = [&](uint32_t byte) {
    const int d = (int)(byte / 8u);
    return (d >= pl.W && d < pl.W + pl.NKP) || (d >= pl.CACC && d < pl.CACC + pl.NKP);
  };
  vec.assign((size_t)nsteps * SOLVEC_STEP_WORDS, 0u);
  mat.assign((size_t)nsteps * SOLVEM_STEP_WORDS, 0u);
  for (int st = 0; st < nsteps; ++st) {
    const uint32_t* r = rec.data() + (size_t)st * SOLVE_STEP_WORDS;
    uint32_t* cv = vec.data() + (size_t)st * SOLVEC_STEP_WORDS;
    uint32_t* cm = mat.data() + (size_t)st * SOLVEM_STEP_WORDS;
    for (int l = 0; l < 64; ++l) {
      for (int c = 0; c < SOLVE_MAXC; ++c) {
        // full record: row q = c / 2 holds lane quads (a_2q, b_2q, a_2q+1, b_2q+1)
        const uint32_t a = r[(c / 2) * 256 + l * 4 + (c % 2) * 2];
        const uint32_t b = r[(c / 2) * 256 + l * 4 + (c % 2) * 2 + 1];
        const bool av = is_vec(a);
        // compact rows: q = c / 4 holds lane quads of terms 4q..4q+3
        cv[(c / 4) * 256 + l * 4 + (c % 4)] = av ? a : b;
        cm[(c / 4) * 256 + l * 4 + (c % 4)] = av ? b : a;
      }
      for (int k = 0; k < 4; ++k) cv[2 * 256 + l * 4 + k] = r[SOLVE_TERM_WORDS + l * 4 + k];
    }
  }
}

template <typename T>
size_t push_blob(std::vector<char>& blob, const std::vector<T>& v, size_t zero_tail = 0) {
  size_t off = (blob.size() + 15) & ~size_t(15);
  blob.resize(off + (v.size() + zero_tail) * sizeof(T) + 16);  // resize zero-fills the tail
  if (!v.empty()) memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
  return off;
}
// a schedule table and the TABLE_PAD_STEPS zero steps behind it (table_rsrc)
size_t push_table(std::vector<char>& blob, const std::vector<uint32_t>& v, int stride_words) {
  return push_blob(blob, v, (size_t)TABLE_PAD_STEPS * stride_words);
}
// Two tables that run one after the other (forward then backward solve; factorization then its
// block-inverse tail), laid out as [A][B][the first TABLE_PAD_STEPS steps of A]: the record
// pipelines' look-ahead loads past the end of A read B's first steps -- the very lines B's own
// prefetch loads next, then L1 hits -- and B's read A's, which the next iteration loads (the
// look-ahead loads are never executed, so their content does not matter).  Measured neutral on the
// N = 20 bench (945k vs 944k solves/s: the shared zero pads were already L1-resident; DESIGN.md,
// Record traffic), kept because it takes the pads' lines out of the L1 working set.
void push_chain(std::vector<char>& blob, const std::vector<uint32_t>& A, const std::vector<uint32_t>& B,
                int stride_words, size_t& oA, size_t& oB) {
  const size_t pad = (size_t)TABLE_PAD_STEPS * stride_words;
  std::vector<uint32_t> all(A);
  all.insert(all.end(), B.begin(), B.end());
  for (size_t k = 0; k < pad; ++k) all.push_back(k < A.size() ? A[k] : 0u);
  oA = push_blob(blob, all, pad);
  oB = oA + A.size() * sizeof(uint32_t);
}

}  // namespace

struct mpcqp_handle {
  Plan plan;
  mpcqp_settings set;
  int B = 0;
  hipStream_t stream = nullptr;
  char* d_blob = nullptr;
  DevPlan dp{};
  double *Px = nullptr, *q = nullptr, *Ax = nullptr, *l = nullptr, *u = nullptr;
  double *xs = nullptr, *zs = nullptr, *ys = nullptr, *rho = nullptr, *Ecls = nullptr;
  double *Pw = nullptr, *qw = nullptr;  // OSQP's data drift (KParams::Pw): two buffers each
  int32_t *dsel = nullptr, *pend = nullptr;
  bool a_inplace = false;  // mpcqp_data_buffers handed out Ax (KParams::a_inplace)
  int32_t* has_state = nullptr;
  double* scratch = nullptr;
  unsigned int* counter = nullptr;
  unsigned long long* timing = nullptr;  // MPCQP_TIMING builds
  bool has_data = false;
  const int32_t* skip = nullptr;   // mpcqp_set_skip
  const int32_t* order = nullptr;  // mpcqp_set_order
  int grid = 0, lds_bytes = 0, waves_per_cu = 0, per_cu = 0;
  int kregs = 0, kscratch = 0;  // the launched kernel's registers per lane and scratch bytes
  int block = 64;  // threads per workgroup: 64 per wave of an instance
  kernel_fn kern = nullptr;
};

extern "C" {

int mpcqp_create(const mpcqp_structure* st, const mpcqp_settings* s, int32_t batch, void* stream,
                 mpcqp_handle** out) {
  if (!st || !s || !out || batch <= 0) return fail(MPCQP_E_INVALID, "invalid argument");
  *out = nullptr;
  if (st->m <= 0) return fail(MPCQP_E_UNSUPPORTED, "problems without constraints (m == 0)");
  if (s->polish) return fail(MPCQP_E_UNSUPPORTED, "polish is not implemented in this build");
  if (s->scaled_termination)
    return fail(MPCQP_E_UNSUPPORTED, "scaled_termination is not implemented in this build");
  if (s->max_iter <= 0 || s->alpha <= 0 || s->alpha >= 2 || s->sigma <= 0 || s->rho <= 0 ||
      s->scaling < 0 || s->check_termination < 0 || s->eps_abs < 0 || s->eps_rel < 0)
    return fail(MPCQP_E_INVALID, "invalid settings");
  mpcqp_handle* h = new mpcqp_handle();
  h->set = *s;
  h->B = batch;
  h->stream = (hipStream_t)stream;
  if (!plan_for(st, h->plan)) {
    std::string e = h->plan.error;
    delete h;
    return fail(MPCQP_E_UNSUPPORTED, e);
  }
  h->block = 64 * h->plan.waves;
  const Plan& pl = h->plan;
  if (pl.CACC - pl.W != pl.NKP) {  // the kernel addresses C as W + NKP (an immediate offset)
    delete h;
    return fail(MPCQP_E_UNSUPPORTED, "internal: accumulator region does not follow the solve vector");
  }
  if (pl.nfac < 1 || pl.nfwd < 1 || pl.nbwd < 1) {
    delete h;
    return fail(MPCQP_E_UNSUPPORTED, "internal: empty schedule");
  }
  auto cleanup_fail = [&](int code, const std::string& msg) {
    mpcqp_destroy(h);
    return fail(code, msg);
  };
  {
    const bool mreg = use_mreg(pl);
    h->kern = select_kernel(pl.n, pl.m, pl.paired,
                            pl.waves == 2 ? (pl.split_steps ? 2 : 3) : 1, pl.mat_first, pl.mv_global,
                            mreg);
    if (!h->kern) {
      delete h;
      return fail(MPCQP_E_UNSUPPORTED, "problem dimensions exceed the instantiated kernels");
    }
    // structure blob
    std::vector<char> blob;
    size_t o_fac = 0, o_tail = 0, o_fwd = 0, o_bwd = 0;
    push_chain(blob, pl.fac, pl.tail, FAC_STEP_WORDS, o_fac, o_tail);
    push_chain(blob, pl.fwd, pl.bwd, SOLVE_STEP_WORDS, o_fwd, o_bwd);
    size_t o_Lc = push_blob(blob, pl.Lcol), o_sP = push_blob(blob, pl.slotP),
           o_sA = push_blob(blob, pl.slotA), o_sR = push_blob(blob, pl.slotRho),
           o_sS = push_blob(blob, pl.slotSig), o_wx = push_blob(blob, pl.wsx),
           o_wz = push_blob(blob, pl.wsz), o_Ap = push_blob(blob, pl.Ap), o_Ai = push_blob(blob, pl.Ai),
           o_Ac = push_blob(blob, pl.Acol), o_Arp = push_blob(blob, pl.Arp),
           o_Ark = push_blob(blob, pl.Ark), o_Arj = push_blob(blob, pl.Arj),
           o_Pi = push_blob(blob, pl.Pi), o_Pc = push_blob(blob, pl.Pcol),
           o_Psp = push_blob(blob, pl.Psp), o_Psk = push_blob(blob, pl.Psk),
           o_Pso = push_blob(blob, pl.Pso), o_eAs = push_blob(blob, pl.ellA.src),
           o_eAi = push_blob(blob, pl.ellA.in), o_eTs = push_blob(blob, pl.ellAt.src),
           o_eTi = push_blob(blob, pl.ellAt.in), o_ePs = push_blob(blob, pl.ellP.src),
           o_ePi = push_blob(blob, pl.ellP.in),
           o_eAv = push_blob(blob, pl.ellA.vpos), o_eTv = push_blob(blob, pl.ellAt.vpos),
           o_ePv = push_blob(blob, pl.ellP.vpos), o_eAk = push_blob(blob, pl.ellA.pk),
           o_eTk = push_blob(blob, pl.ellAt.pk), o_ePk = push_blob(blob, pl.ellP.pk),
           o_eAq = push_blob(blob, pl.ellA.sk), o_eTq = push_blob(blob, pl.ellAt.sk),
           o_ePq = push_blob(blob, pl.ellP.sk), o_sra = push_blob(blob, pl.sra),
           o_sca = push_blob(blob, pl.sca), o_wc = push_blob(blob, pl.wcopy),
           o_bc = push_blob(blob, pl.bcopy);
    std::vector<uint32_t> fwdc, fwdm, bwdc, bwdm;
    if (mreg) {
      split_records(pl, pl.fwd, pl.nfwd, fwdc, fwdm);
      split_records(pl, pl.bwd, pl.nbwd, bwdc, bwdm);
    }
    const size_t o_fwdc = push_table(blob, fwdc, SOLVEC_STEP_WORDS), o_fwdm = push_blob(blob, fwdm),
                 o_bwdc = push_table(blob, bwdc, SOLVEC_STEP_WORDS), o_bwdm = push_blob(blob, bwdm);
    if (hipMalloc(&h->d_blob, blob.size()) != hipSuccess)
      return cleanup_fail(MPCQP_E_HIP, "hipMalloc(structure)");
    if (hipMemcpy(h->d_blob, blob.data(), blob.size(), hipMemcpyHostToDevice) != hipSuccess)
      return cleanup_fail(MPCQP_E_HIP, "hipMemcpy(structure)");
    char* b = h->d_blob;
    DevPlan& dp = h->dp;
    dp.fac = (const uint32_t*)(b + o_fac), dp.tail = (const uint32_t*)(b + o_tail);
    dp.fwd = (const uint32_t*)(b + o_fwd), dp.bwd = (const uint32_t*)(b + o_bwd);
    dp.nfac = pl.nfac, dp.ntail = pl.ntail, dp.nfwd = pl.nfwd, dp.nbwd = pl.nbwd;
    dp.fwdc = (const uint32_t*)(b + o_fwdc), dp.fwdm = (const uint32_t*)(b + o_fwdm);
    dp.bwdc = (const uint32_t*)(b + o_bwdc), dp.bwdm = (const uint32_t*)(b + o_bwdm);
    dp.Lcol = (const uint16_t*)(b + o_Lc);
    dp.slotP = (const uint16_t*)(b + o_sP), dp.slotA = (const uint16_t*)(b + o_sA);
    dp.slotRho = (const uint16_t*)(b + o_sR), dp.slotSig = (const uint16_t*)(b + o_sS);
    dp.wsx = (const uint16_t*)(b + o_wx), dp.wsz = (const uint16_t*)(b + o_wz);
    dp.wcopy = (const uint32_t*)(b + o_wc);
    dp.bcopy = (const uint32_t*)(b + o_bc);
    dp.Ap = (const uint16_t*)(b + o_Ap), dp.Ai = (const uint16_t*)(b + o_Ai);
    dp.Acol = (const uint16_t*)(b + o_Ac), dp.Arp = (const uint16_t*)(b + o_Arp);
    dp.Ark = (const uint16_t*)(b + o_Ark), dp.Arj = (const uint16_t*)(b + o_Arj);
    dp.Pi = (const uint16_t*)(b + o_Pi), dp.Pcol = (const uint16_t*)(b + o_Pc);
    dp.Psp = (const uint16_t*)(b + o_Psp), dp.Psk = (const uint16_t*)(b + o_Psk);
    dp.Pso = (const uint16_t*)(b + o_Pso);
    auto ell = [&](const Ell& e, size_t os, size_t oi, size_t ov, size_t ok, size_t oq,
                   EllDev& d) {
      d.src = (const uint16_t*)(b + os), d.in = (const uint16_t*)(b + oi), d.total = e.total;
      d.vpos = (const uint16_t*)(b + ov), d.pk = (const uint32_t*)(b + ok);
      d.sk = (const uint16_t*)(b + oq);
      for (int r = 0; r < ELL_MAXR; ++r) d.K[r] = e.K[r], d.off[r] = e.off[r];
      d.nlong = e.nlong;
      for (int q = 0; q < ELL_MAXLONG; ++q)
        d.long_out[q] = e.long_out[q], d.long_off[q] = e.long_off[q], d.long_cnt[q] = e.long_cnt[q];
    };
    ell(pl.ellA, o_eAs, o_eAi, o_eAv, o_eAk, o_eAq, dp.eA);
    ell(pl.ellAt, o_eTs, o_eTi, o_eTv, o_eTk, o_eTq, dp.eAt);
    ell(pl.ellP, o_ePs, o_ePi, o_ePv, o_ePk, o_ePq, dp.eP);
    dp.inst_doubles = (pl.LDS_N + 1) & ~1;
    dp.n = pl.n, dp.m = pl.m, dp.nk = pl.nk, dp.nnzP = pl.nnzP, dp.nnzA = pl.nnzA;
    dp.nnzL = pl.nnzL;
    dp.LX = pl.LX, dp.DINV = pl.DINV, dp.W = pl.W, dp.CACC = pl.CACC, dp.ZERO = pl.ZERO;
    dp.ONE = pl.ONE, dp.MONE = pl.MONE, dp.LDS_N = pl.LDS_N, dp.NKS = pl.NKP / 64;
    dp.S_P = pl.S_P, dp.S_A = pl.S_A, dp.S_DT = pl.S_DT, dp.S_ET = pl.S_ET;
    dp.S_ZERO = pl.S_ZERO;
    dp.MV = pl.MV, dp.MVZ = pl.MVZ, dp.mv_slab = pl.mv_slab;
    dp.sra = (const uint16_t*)(b + o_sra), dp.sca = (const uint16_t*)(b + o_sca), dp.SJ = pl.SJ;
    dp.XCH = pl.XCH, dp.XID = pl.XID;
    // the vector passes address C through W's slot plus the compile-time distance 64 (RN + RM)
    if (pl.CACC - pl.W != pl.NKP || pl.NKP != 64 * (pl.RN + pl.RM))
      return cleanup_fail(MPCQP_E_INVALID, "internal: C region not at the kernel's distance from W");
    if (pl.SJ > 8 * pl.RN)  // the kernel holds 8 RN row / column slots per lane (scale_problem)
      return cleanup_fail(MPCQP_E_UNSUPPORTED, "too many matrix values for the scaling registers");
    // the sequential sums stage their terms in the accumulator region C (NKP doubles, free during
    // the checks): a long mat-vec output's products per wave, the certificates' n / m terms
    for (const Ell* e : {&pl.ellA, &pl.ellAt, &pl.ellP}) {
      int tot = 0;  // a mat-vec stages all its long outputs at once (ell_apply)
      for (int L = 0; L < e->nlong; ++L) tot += e->long_cnt[L];
      if (tot > pl.NKP / pl.waves)
        return cleanup_fail(MPCQP_E_UNSUPPORTED, "internal: long mat-vec outputs exceed their staging");
    }

    // occupancy (LDS image and VGPRs) -> persistent grid
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return cleanup_fail(MPCQP_E_HIP, "hipGetDevice");
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return cleanup_fail(MPCQP_E_HIP, "hipDeviceGetAttribute");
    const int inst_bytes = dp.inst_doubles * 8;
    const int lds_cap = 160 * 1024;
    // diagnostic: MPCQP_LDS_PAD extra bytes per workgroup (occupancy scans; never set in product)
    const int lds_alloc = inst_bytes + std::max(0, env_int("MPCQP_LDS_PAD", 0));
    if (lds_alloc > lds_cap)
      return cleanup_fail(MPCQP_E_UNSUPPORTED, "instance image exceeds the LDS of a CU");
    if (hipFuncSetAttribute((const void*)h->kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            lds_cap) != hipSuccess)
      return cleanup_fail(MPCQP_E_HIP, "hipFuncSetAttribute");
    // register / scratch guard: builds above ~440 registers computed wrong
    // iterates from a wave's second instance on (High-register builds); a product kernel
    // beyond the validated budget is refused instead of launched (diagnostic builds may raise it)
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, (const void*)h->kern) != hipSuccess)
      return cleanup_fail(MPCQP_E_HIP, "hipFuncGetAttributes");
    h->kregs = fa.numRegs;
    h->kscratch = (int)fa.localSizeBytes;
    if (h->kregs > env_int("MPCQP_REG_BUDGET", MPCQP_MAX_KERNEL_REGS) ||
        h->kscratch > MPCQP_MAX_KERNEL_SCRATCH)
      return cleanup_fail(MPCQP_E_UNSUPPORTED,
                          "solve kernel allocates " + std::to_string(h->kregs) + " registers / " +
                              std::to_string(h->kscratch) +
                              " scratch bytes per lane: above the validated budget");
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)h->kern, h->block, lds_alloc) !=
            hipSuccess || nb <= 0)
      return cleanup_fail(MPCQP_E_UNSUPPORTED, "kernel does not fit on a CU (LDS/VGPR)");
    h->per_cu = nb;
    h->waves_per_cu = nb * pl.waves;
    h->lds_bytes = lds_alloc;
    h->grid = std::min(batch, nb * ncu);
  }
  const size_t Bz = (size_t)batch;
  bool ok = hipMalloc(&h->Px, sizeof(double) * std::max(1, pl.nnzP)) == hipSuccess &&
            hipMalloc(&h->q, sizeof(double) * pl.n) == hipSuccess &&
            hipMalloc(&h->Ax, sizeof(double) * Bz * std::max(1, pl.nnzA)) == hipSuccess &&
            hipMalloc(&h->l, sizeof(double) * Bz * pl.m) == hipSuccess &&
            hipMalloc(&h->u, sizeof(double) * Bz * pl.m) == hipSuccess &&
            hipMalloc(&h->xs, sizeof(double) * Bz * pl.n) == hipSuccess &&
            hipMalloc(&h->zs, sizeof(double) * Bz * pl.m) == hipSuccess &&
            hipMalloc(&h->ys, sizeof(double) * Bz * pl.m) == hipSuccess &&
            hipMalloc(&h->Ecls, sizeof(double) * Bz * pl.m) == hipSuccess &&
            hipMalloc(&h->Pw, 2 * sizeof(double) * Bz * std::max(1, pl.nnzP)) == hipSuccess &&
            hipMalloc(&h->qw, 2 * sizeof(double) * Bz * pl.n) == hipSuccess &&
            hipMalloc(&h->dsel, sizeof(int32_t) * Bz) == hipSuccess &&
            hipMalloc(&h->pend, sizeof(int32_t) * Bz) == hipSuccess &&
            hipMalloc(&h->rho, sizeof(double) * Bz) == hipSuccess &&
            hipMalloc(&h->has_state, sizeof(int32_t) * Bz) == hipSuccess &&
            hipMalloc(&h->scratch, sizeof(double) * (size_t)h->grid * slab_doubles(pl.n, pl.m, pl.mv_slab)) ==
                hipSuccess &&
            hipMalloc(&h->counter, 64) == hipSuccess;
  if (!ok) return cleanup_fail(MPCQP_E_HIP, "hipMalloc(batch buffers)");
  if (hipMemset(h->has_state, 0, sizeof(int32_t) * Bz) != hipSuccess ||
      hipMemsetD32(h->dsel, -2, Bz) != hipSuccess || hipMemset(h->pend, 0, sizeof(int32_t) * Bz) != hipSuccess)
    return cleanup_fail(MPCQP_E_HIP, "hipMemset");
  *out = h;
  return 0;
}

int mpcqp_destroy(mpcqp_handle* h) {
  if (!h) return 0;
  void* bufs[] = {h->d_blob, h->Px, h->q,    h->Ax,        h->l,       h->u,      h->xs,
                  h->zs,     h->ys, h->Ecls, h->rho, h->has_state, h->scratch, h->counter,
                  h->Pw,     h->qw, h->dsel, h->pend};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  delete h;
  return 0;
}

// every instance's drift buffer row <- src (device), on the handle's stream
static hipError_t bcast_rows(mpcqp_handle* h, double* dst, const double* src, int cnt) {
  const size_t tot = (size_t)h->B * cnt;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(bcast_rows_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, h->stream,
                     dst, src, h->B, cnt);
  return hipGetLastError();
}

int mpcqp_set_data(mpcqp_handle* h, const double* Px, const double* q, const double* Ax,
                   const double* l, const double* u) {
  if (!h || !Px || !q || !Ax || !l || !u) return fail(MPCQP_E_INVALID, "null argument");
  const Plan& pl = h->plan;
  const size_t B = (size_t)h->B;
  HIPCHK(hipMemcpyAsync(h->Px, Px, sizeof(double) * pl.nnzP, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->q, q, sizeof(double) * pl.n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->Ax, Ax, sizeof(double) * B * pl.nnzA, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->l, l, sizeof(double) * B * pl.m, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->u, u, sizeof(double) * B * pl.m, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemsetAsync(h->has_state, 0, sizeof(int32_t) * B, h->stream));
  // a new setup: the next solve scales the given data (drift_of), no update of A pending
  HIPCHK(hipMemsetD32Async(h->dsel, -2, B, h->stream));
  HIPCHK(hipMemsetAsync(h->pend, 0, sizeof(int32_t) * B, h->stream));
  h->has_data = true;
  return 0;
}

int mpcqp_update_bounds(mpcqp_handle* h, const double* l, const double* u) {
  if (!h || !l || !u) return fail(MPCQP_E_INVALID, "null argument");
  if (!h->has_data) return fail(MPCQP_E_NODATA, "update before set_data");
  const size_t B = (size_t)h->B;
  HIPCHK(hipMemcpyAsync(h->l, l, sizeof(double) * B * h->plan.m, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->u, u, sizeof(double) * B * h->plan.m, hipMemcpyDeviceToDevice, h->stream));
  return 0;
}

int mpcqp_update_A(mpcqp_handle* h, const double* Ax) {
  if (!h || !Ax) return fail(MPCQP_E_INVALID, "null argument");
  if (!h->has_data) return fail(MPCQP_E_NODATA, "update before set_data");
  HIPCHK(hipMemcpyAsync(h->Ax, Ax, sizeof(double) * (size_t)h->B * h->plan.nnzA,
                        hipMemcpyDeviceToDevice, h->stream));
  // each instance's next solve follows osqp_update_A (unscale, overwrite, rescale: drift_of)
  HIPCHK(hipMemsetD32Async(h->pend, 1, (size_t)h->B, h->stream));
  return 0;
}

int mpcqp_update_lin_cost(mpcqp_handle* h, const double* q) {
  if (!h || !q) return fail(MPCQP_E_INVALID, "null argument");
  if (!h->has_data) return fail(MPCQP_E_NODATA, "update before set_data");
  HIPCHK(hipMemcpyAsync(h->q, q, sizeof(double) * h->plan.n, hipMemcpyDeviceToDevice, h->stream));
  // the next solve rescales the new q itself (OSQP would carry (q D) c unscaled: an ulp apart; the
  // reference never updates q): both drift buffers, whichever drift_of picks
  HIPCHK(bcast_rows(h, h->qw, h->q, h->plan.n));
  HIPCHK(bcast_rows(h, h->qw + (size_t)h->B * h->plan.n, h->q, h->plan.n));
  return 0;
}

int mpcqp_warm_start(mpcqp_handle* h, const double* x, const double* y) {
  if (!h || !x || !y) return fail(MPCQP_E_INVALID, "null argument");
  if (!h->has_data) return fail(MPCQP_E_NODATA, "warm start before set_data");
  const size_t B = (size_t)h->B;
  HIPCHK(hipMemcpyAsync(h->xs, x, sizeof(double) * B * h->plan.n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->ys, y, sizeof(double) * B * h->plan.m, hipMemcpyDeviceToDevice, h->stream));
  // has_state = 2 for every instance, but keep rho: a warm start does not reset rho in OSQP.
  // (rho_state is only read when has_state != 0; instances never solved start from settings.rho)
  std::vector<int32_t> two(B, 2);
  HIPCHK(hipMemcpyAsync(h->has_state, two.data(), sizeof(int32_t) * B, hipMemcpyHostToDevice,
                        h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int mpcqp_solve(mpcqp_handle* h, double* x, double* y, const mpcqp_info* info) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  if (!h->has_data) return fail(MPCQP_E_NODATA, "solve before set_data");
  KParams p{};
  p.pl = h->dp;
  p.s = h->set;
  p.B = h->B;
  p.Px = h->Px, p.q = h->q, p.Ax = h->Ax, p.l = h->l, p.u = h->u;
  p.xs = h->xs, p.zs = h->zs, p.ys = h->ys, p.rho_state = h->rho, p.Ecls = h->Ecls;
  p.Pw = h->Pw, p.qw = h->qw;
  p.dsel = h->dsel, p.pend = h->pend, p.a_inplace = h->a_inplace ? 1 : 0;
  p.has_state = h->has_state;
  p.x_out = x, p.y_out = y;
  if (info) p.info = *info;
  p.scratch = h->scratch;
  p.counter = h->counter;
  p.timing = h->timing;
  p.rho0 = std::min(std::max(h->set.rho, RHO_MIN), RHO_MAX);
  p.skip = h->skip;
  p.order = h->order;
  HIPCHK(hipMemsetAsync(h->counter, 0, 64, h->stream));
  hipLaunchKernelGGL(h->kern, dim3(h->grid), dim3(h->block), h->lds_bytes, h->stream, p);
  HIPCHK(hipGetLastError());
  return 0;
}

#ifdef MPCQP_TIMING
// diagnostic builds only (not part of include/mpcqp.h): device buffer of T_NSLOT uint64 counters
int mpcqp_debug_timing(mpcqp_handle* h, unsigned long long* dev_buf) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  h->timing = dev_buf;
  return 0;
}
#endif

#ifdef MPCQP_PAIR_CHECKS
// diagnostic builds only (not part of include/mpcqp.h): arm / disarm the injected barrier skip of
// the two-wave kernel (g_pair_inject) for the following launches
int mpcqp_debug_pair_inject(int on) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_pair_inject), &on, sizeof(int)) == hipSuccess ? 0 : MPCQP_E_HIP;
}
#endif

int mpcqp_data_buffers(mpcqp_handle* h, double** Ax, double** l, double** u) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  // the caller may rewrite A in place between solves: every later solve follows an update of A
  if (Ax) h->a_inplace = true;
  if (Ax) *Ax = h->Ax;
  if (l) *l = h->l;
  if (u) *u = h->u;
  return 0;
}

int mpcqp_copy_data(mpcqp_handle* h, double* Ax, double* l, double* u) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  const size_t B = (size_t)h->B;
  if (Ax)
    HIPCHK(hipMemcpyAsync(Ax, h->Ax, sizeof(double) * B * h->plan.nnzA, hipMemcpyDeviceToDevice,
                          h->stream));
  if (l)
    HIPCHK(hipMemcpyAsync(l, h->l, sizeof(double) * B * h->plan.m, hipMemcpyDeviceToDevice,
                          h->stream));
  if (u)
    HIPCHK(hipMemcpyAsync(u, h->u, sizeof(double) * B * h->plan.m, hipMemcpyDeviceToDevice,
                          h->stream));
  return 0;
}

int mpcqp_set_skip(mpcqp_handle* h, const int32_t* skip) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  h->skip = skip;
  return 0;
}

int mpcqp_set_order(mpcqp_handle* h, const int32_t* order) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  h->order = order;
  return 0;
}

int mpcqp_get_state(const mpcqp_handle* h, double* xs, double* zs, double* ys, double* rho,
                    int32_t* has_state) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  const size_t B = (size_t)h->B;
  const Plan& pl = h->plan;
  if (xs) HIPCHK(hipMemcpyAsync(xs, h->xs, sizeof(double) * B * pl.n, hipMemcpyDeviceToDevice, h->stream));
  if (zs) HIPCHK(hipMemcpyAsync(zs, h->zs, sizeof(double) * B * pl.m, hipMemcpyDeviceToDevice, h->stream));
  if (ys) HIPCHK(hipMemcpyAsync(ys, h->ys, sizeof(double) * B * pl.m, hipMemcpyDeviceToDevice, h->stream));
  if (rho) HIPCHK(hipMemcpyAsync(rho, h->rho, sizeof(double) * B, hipMemcpyDeviceToDevice, h->stream));
  if (has_state)
    HIPCHK(hipMemcpyAsync(has_state, h->has_state, sizeof(int32_t) * B, hipMemcpyDeviceToDevice,
                          h->stream));
  return 0;
}

int mpcqp_set_state(mpcqp_handle* h, const double* xs, const double* zs, const double* ys,
                    const double* rho, const int32_t* has_state) {
  if (!h || !xs || !zs || !ys || !rho || !has_state) return fail(MPCQP_E_INVALID, "null argument");
  const size_t B = (size_t)h->B;
  const Plan& pl = h->plan;
  HIPCHK(hipMemcpyAsync(h->xs, xs, sizeof(double) * B * pl.n, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->zs, zs, sizeof(double) * B * pl.m, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->ys, ys, sizeof(double) * B * pl.m, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->rho, rho, sizeof(double) * B, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->has_state, has_state, sizeof(int32_t) * B, hipMemcpyDeviceToDevice,
                        h->stream));
  return 0;
}

int mpcqp_get_scaling(const mpcqp_handle* h, double* E, double* Pu, double* qu) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  const size_t B = (size_t)h->B;
  const Plan& pl = h->plan;
  if (E) HIPCHK(hipMemcpyAsync(E, h->Ecls, sizeof(double) * B * pl.m, hipMemcpyDeviceToDevice, h->stream));
  auto gather = [&](double* dst, const double* W, const double* shared, int cnt) {
    const size_t tot = B * (size_t)cnt;
    if (tot == 0) return hipSuccess;
    hipLaunchKernelGGL(drift_gather_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       h->stream, dst, W, shared, h->dsel, (int)B, cnt);
    return hipGetLastError();
  };
  if (Pu) HIPCHK(gather(Pu, h->Pw, h->Px, pl.nnzP));
  if (qu) HIPCHK(gather(qu, h->qw, h->q, pl.n));
  return 0;
}

int mpcqp_dims(const mpcqp_handle* h, int32_t* n, int32_t* m, int32_t* nnzP, int32_t* nnzA,
               int32_t* nnzL) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  if (n) *n = h->plan.n;
  if (m) *m = h->plan.m;
  if (nnzP) *nnzP = h->plan.nnzP;
  if (nnzA) *nnzA = h->plan.nnzA;
  if (nnzL) *nnzL = h->plan.nnzL;
  return 0;
}

int mpcqp_schedule_info(const mpcqp_handle* h, int32_t* fac, int32_t* fwd, int32_t* bwd,
                        int32_t* lds, int32_t* wpc) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  if (fac) *fac = (int32_t)(h->plan.nfac + h->plan.ntail);
  if (fwd) *fwd = (int32_t)h->plan.nfwd;
  if (bwd) *bwd = (int32_t)h->plan.nbwd;
  if (lds) *lds = h->lds_bytes;
  if (wpc) *wpc = h->waves_per_cu;
  return 0;
}

int mpcqp_schedule_kind(const mpcqp_handle* h, int32_t* atomics_per_step) {
  if (!h || !atomics_per_step) return fail(MPCQP_E_INVALID, "null argument");
  *atomics_per_step = h->plan.paired ? 3 : 4;
  return 0;
}

int mpcqp_kernel_info(const mpcqp_handle* h, int32_t* waves_per_instance, int32_t* instances_per_cu,
                      int32_t* regs, int32_t* scratch_bytes) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  if (waves_per_instance) *waves_per_instance = h->plan.waves;
  if (instances_per_cu) *instances_per_cu = h->per_cu;
  if (regs) *regs = h->kregs;
  if (scratch_bytes) *scratch_bytes = h->kscratch;
  return 0;
}

int mpcqp_engine_kind(const mpcqp_handle* h, int32_t* kind) {
  if (!h || !kind) return fail(MPCQP_E_INVALID, "null argument");
  *kind = MPCQP_ENGINE_KKT;
  return 0;
}

int mpcqp_export_symbolic(const mpcqp_handle* h, int32_t* perm, int32_t* Lp, int32_t* Li) {
  if (!h) return fail(MPCQP_E_INVALID, "null handle");
  const Plan& pl = h->plan;
  if (perm) std::copy(pl.perm.begin(), pl.perm.end(), perm);
  if (Lp) std::copy(pl.Lp.begin(), pl.Lp.end(), Lp);
  if (Li) std::copy(pl.Li.begin(), pl.Li.end(), Li);
  return 0;
}

}  // extern "C"
