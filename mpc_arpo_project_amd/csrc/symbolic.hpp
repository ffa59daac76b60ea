// symbolic.hpp -- host-side symbolic analysis of the batched MPC-QP KKT system and compilation of
// the level schedules that the HIP kernel interprets.
//
// The KKT matrix is OSQP's quasi-definite  [[P + sigma I, A'], [A, -diag(1/rho)]]  (OSQP 0.6
// kkt.c form_KKT), permuted by the same exact minimum-degree ordering the oracle uses, so the
// device factor L D L' has exactly the oracle's (and QDLDL's) sparsity.  Because all instances of
// a batch share the pattern, everything here is computed once per handle; per-instance work on
// the GPU is purely numeric.
//
// Level schedules.  Factorization (left-looking, dot-product form on U = L D), forward solve
// L w = b and backward solve L' x = w are each cut into levels of mutually independent "tasks".
// A factorization task SETS one LDS slot  v[t] <- -sum_k U_ik U_jk (1/D_k)  (a task that updates
// its slot in place gets the extra term (-1) * v[t]); it gets an aligned group of g = 2^glog lanes,
// each lane accumulates <= C terms, the group reduces with an xor butterfly and its first lane
// writes the slot.  A solve task ACCUMULATES  v[t] += -sum_k v[a_k] v[b_k]: its terms are cut into
// two-term segments that may sit in any lanes of any steps of the level, and every segment is
// added to the target with an LDS atomic (targets are zeroed or hold the in-place value before
// the level), so solve steps need no cross-lane reduction.
//
// Step records have a fixed stride (STEP_WORDS 32-bit words) so that the device computes no
// record addresses: rows of 64 lane records of absolute LDS byte addresses -- the factorization's
// meta words then (a, b, c, 0) quads, the solves' (a0, b0, a1, b1) segment quads then the
// (t0, t1, t2, t3) target quads.  Unused terms point at the image's ZERO slot, unused segments
// at the lane's sink slot.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace mpcqp {

// Diagnostic environment switches (plan, layout, kernel-mode and occupancy overrides used by the
// tools/ A/B scripts and a few white-box tests).  They are honoured ONLY when MPCQP_DIAGNOSTICS=1 is
// set as well, so a product handle never picks up an unvalidated plan or kernel from an inherited
// environment.  Returns null when the switch is off or the variable unset.
inline const char* diag_env(const char* name) {
  const char* on = getenv("MPCQP_DIAGNOSTICS");
  if (!on || strcmp(on, "1") != 0) return nullptr;
  const char* e = getenv(name);
  return (e && *e) ? e : nullptr;
}
inline int diag_env_int(const char* name, int dflt) {
  const char* e = diag_env(name);
  return e ? atoi(e) : dflt;
}

constexpr int SOLVE_MAXC = 8;   // terms per lane of a solve step
constexpr int FAC_MAXC = 4;     // terms per lane of a factorization step
// factorization step: meta[64] | FAC_MAXC rows of 64 (a, b, c, 0) quads
constexpr int FAC_STEP_WORDS = 64 + 64 * 4 * FAC_MAXC;
// solve step: SOLVE_MAXC / 2 rows of 64 segment quads (a0, b0, a1, b1) | 64 target quads
// (t0, t1, t2, t3); segments 0 and 1 of a lane are a PAIR: they belong to the same target (or
// segment 1 is unused) and their sum is added to t0 with one LDS atomic; segments 2 and 3 are added
// to t2 and t3 -- three atomics per lane and step (t1 repeats t0 and is not read)
constexpr int SOLVE_TERM_WORDS = 64 * 2 * SOLVE_MAXC;
constexpr int SOLVE_STEP_WORDS = SOLVE_TERM_WORDS + 64 * 4;

// constant slots behind N | G | G': ZERO_BLOCK zeros (one per ds_read_b64 bank class, so the
// padding terms of a solve step can read a zero from a bank no real operand of the instruction
// half uses), ONE, MONE, padding
constexpr int ZERO_BLOCK = 32;
constexpr int CONST_SLOTS = ZERO_BLOCK + 4;
// cross-wave exchange of the two-wave kernel: values per wave and buffer
constexpr int XCH_K = 8;
constexpr int XCH_DOUBLES = 2 * 2 * XCH_K;

// meta word: per-lane fields, then the step-wide C and glog (identical in every lane)
constexpr uint32_t META_TGT_MASK = 0x1ffffu;  // factorization: LDS byte address of the target
constexpr int META_GLOG_SHIFT = 17;           // 3 bits: this lane's group size log2
constexpr uint32_t META_HEAD = 1u << 20;
constexpr uint32_t META_ISD = 1u << 21;       // factorization: target is D_j -> also write 1/D_j
constexpr int META_C_SHIFT = 22;              // 4 bits: terms per lane in this step
constexpr int META_SGLOG_SHIFT = 26;          // 3 bits: widest group log2 in this step
constexpr uint32_t META_SISD = 1u << 29;      // step-wide: some lane of this step stores a 1/D_j

// Sparse mat-vec in padded per-slot ELL form for the residual checks: output element e sits on
// lane e % 64, register slot r = e / 64; every used slot has exactly KMAX terms per lane (compile-
// time width, zero padding), term k of lane l at off[r] + 64 k + l: src = LDS slot of the scaled
// value in the scaling overlay (0xffff = padding), in = index of the input element.  Outputs with
// more than KMAX terms are "long": their terms are listed separately (long_off/long_cnt into the
// tail of src/in) and summed cooperatively by the whole wave.  The per-instance values are gathered
// into the slab in this order once per scaling, so a mat-vec issues all its loads back to back.
constexpr int ELL_MAXR = 16;
constexpr int ELL_MAXLONG = 8;
constexpr int ELL_KA = 8;    // rows of A
constexpr int ELL_KAT = 12;  // columns of A
constexpr int ELL_KP = 4;    // symmetric rows of P
struct Ell {
  int R = 0, total = 0, kmax = 0;
  int K[ELL_MAXR] = {}, off[ELL_MAXR] = {};  // K[r] = kmax for used slots, 0 otherwise
  int nlong = 0;
  int long_out[ELL_MAXLONG] = {}, long_off[ELL_MAXLONG] = {}, long_cnt[ELL_MAXLONG] = {};
  std::vector<uint16_t> src, in;
  // LDS slot (doubles) of each term's scaled value in the resident value region MV (CSC order,
  // Plan::MV); padding terms point at the zero slot MVZ.  The residual mat-vecs read the values
  // from LDS through it (the indices are shared by every instance: L1/L2 hits)
  std::vector<uint16_t> vpos;
  // the same terms lane-major for the kernel's loads: for used slot r, lane l, term k,
  // pk[(r * 64 + l) * kmax + k] = vpos | in << 16 (one 16-byte load covers four terms)
  std::vector<uint32_t> pk;
  // the terms' scaling-overlay slots (src, padding -> S_ZERO) lane-major like pk, u16: the Ruiz
  // passes keep them in registers for the whole scaling
  std::vector<uint16_t> sk;
};

// Register-slot bucket of the engine kernel: RN >= ceil(n / 64) slots for n-vectors, RM >= ceil(m /
// 64) for m-vectors, from the instantiated set (2,4), (4,8), with RN + RM > nk / 64 (a junk slot).
// false if no bucket fits: the reference's horizons (Nx 20-50) all fit (4,8) (up to
// Nx = 51 for the planar model); an (8,16) build spilled 651 VGPRs (profiles/r03/
// resource_usage.txt) and is not shipped, so larger problems are refused at create time.
constexpr int KERNEL_MAX_RN = 4;
inline bool kernel_bucket(int n, int m, int& rn, int& rm) {
  const int need_n = (n + 63) / 64, need_m = (m + 63) / 64, need_k = (n + m) / 64 + 1;
  for (int b = 2; b <= KERNEL_MAX_RN; b *= 2)
    if (need_n <= b && need_m <= 2 * b && 3 * b >= need_k) {
      rn = b, rm = 2 * b;
      return true;
    }
  return false;
}

struct Plan {
  int n = 0, m = 0, nk = 0, nnzP = 0, nnzA = 0, nnzL = 0;
  std::vector<int32_t> perm, pinv, Lp, Li, etree;
  // LDS layout, in doubles, phase by phase over one image (relocate() in symbolic.cpp):
  //   [ L (nnzL): the solve-live entries first, then the entries the solves never read ]
  //       W (solve vector) and C (accumulators) overlay the solve-dead L entries: they are only
  //       used between factorizations, and the factorization rewrites all of L
  //   [ 1/D ]  [ N (negated block inverses) | G | G' ]  [ ZERO x ZERO_BLOCK, ONE, MONE, pad ]
  //       the factorization's D_j tasks run in place on the 1/D slots (KKT diagonal in, 1/D_j out)
  //   unused solve segments add -0.0 (an exact no-op) to a sink slot; the layout optimiser
  //   (lds_layout.cpp) picks any slot of a free bank, the unoptimised layout the W / C padding
  int LX = 0, DINV = 0, W = 0, CACC = 0, NB = 0, GB = 0, GPB = 0, ZERO = 0, ONE = 0, MONE = 0;
  int DS = 0;      // slot base of the D_j tasks' targets (== DINV)
  int RN = 0, RM = 0;  // the kernel's register-slot bucket (kernel_bucket)
  int nLlive = 0;  // L entries the solves read (far-block couplings)
  // the 1/D, W and C regions are NKP = 64 * (RN + RM) doubles long (the kernel's register-slot bucket,
  // kernel_bucket below): whole 64-lane slots, so the per-iteration vector passes store
  // unconditionally, and slot nk of each (the "junk" slot) takes the stores of lanes past the end of x
  // or z (W[nk] is zeroed every iteration and read back as 0)
  int NKP = 0;
  int SINK = 0;   // construction-time base of the 64 sink slots (relocated per lane)
  int LDS_N = 0;
  // blocked substitution: contiguous blocks of the permuted order
  std::vector<int32_t> block_start;  // T + 1 entries
  int nN = 0, nG = 0, nGP = 0;
  // scaling-phase overlay of the same LDS: scaled P, scaled A, D_temp, E_temp
  int S_P = 0, S_A = 0, S_DT = 0, S_ET = 0;
  // S_ZERO: a zero double (in doubles) behind the value overlay, read by the ELL padding of the
  // Ruiz column / row norms
  int S_ZERO = 0;
  // resident scaled matrix values [P (upper CSC) | A (CSC)] behind everything else of the image:
  // written at the end of the Ruiz scaling, read by the residual mat-vecs, the infeasibility
  // certificates, every (re)assembly of the KKT values and the objective; MVZ holds a zero
  int MV = 0, MVZ = 0;
  // round 5: the resident values may instead live in the wave's global scratch slab (mv_global:
  // MV = 0 and MVZ are then indices relative to the slab's value block of mv_slab doubles, and the
  // LDS image ends before them) when that lets more instances share a CU (one-wave plans of the
  // (2, 4) bucket: 5 per CU at N = 20, the kernel built for <= 256 registers; build_plan_tuned)
  bool mv_global = false;
  int mv_slab = 0;
  // the Ruiz rescale's row / column scaling slots of every value k = 64 j + l of [P | A] (CSC
  // orders; S_DT + i for P's rows, S_ET + i for A's, S_DT + j for columns) lane-major at [l][j],
  // j < SJ (a multiple of 4; padding -> 0), held in registers by the Ruiz passes
  int SJ = 0;
  std::vector<uint16_t> sra, sca;
  // KKT assembly: LDS slot of each P entry (diagonal -> D slot), A entry, rho diagonal,
  // sigma diagonal (D slot of x_j)
  std::vector<uint16_t> slotP, slotA, slotRho, slotSig;
  // LDS slot (permuted position in the W region) of x_i and z_i for every lane of the kernel's
  // register slots (64 RN and 64 RM entries; padding lanes get the W padding slots)
  std::vector<uint16_t> wsx, wsz;
  // per lane, bit r: register slot r (x slots 0..RN-1, then z slots) holds a COPY row -- a row of
  // the first block with an empty reach, whose forward-solve output is its right-hand side
  // (W_r = C_r): the right-hand side pass stores it into W directly and no solve task computes it
  std::vector<uint32_t> wcopy;
  // the same for the backward solve, per lane, bit r: W slot lane + 64 r (physical slot order of the
  // diagonal pass) holds a backward copy row, whose W starts at (1/D) W instead of 0; bcopy_row marks
  // them by permuted row (construction order; finish_copy_masks maps them to physical slots)
  std::vector<uint32_t> bcopy;
  std::vector<uint8_t> bcopy_row;
  bool paired = true;  // solve-step kind (build_plan)
  // waves per instance the solve steps are laid out for (build_plan): 1, or 2 -- wave 0 executes
  // segment positions 0 + 1 of every lane, wave 1 positions 2 + 3; within a step every target's
  // segments sit in one of the two halves, so each target is summed by one wave in a fixed order
  int waves = 1;
  // two waves per instance: the solve steps split between them (true: wave 0 executes segment
  // positions 0 + 1, wave 1 positions 2 + 3, the packing constraint above) or all executed by the
  // first wave while the second waits (false)
  bool split_steps = false;
  // every solve term keeps its matrix operand first (segment words a = matrix value, b = vector
  // entry; the layout optimiser does not flip operands): the kernel then reads the matrix operands
  // of the next step during the current one (they are constant during a solve)
  bool mat_first = false;
  // two-wave kernel: LDS slots (doubles) of the cross-wave exchange (XCH_DOUBLES: two buffers x two
  // waves x XCH_K values) and of the instance id the first wave hands the second (XID)
  int XCH = 0, XID = 0;
  // schedules (STEP_WORDS words per step): factorization of U = L D and D by levels, then
  // (after the flat pass L = U * (1/D)_col) the block-inverse tail; forward and backward solves
  std::vector<uint32_t> fac, tail, fwd, bwd;
  int nfac = 0, ntail = 0, nfwd = 0, nbwd = 0;
  std::vector<uint16_t> Lcol;  // column of each L entry (the flat scaling pass)
  // matrix structure for scaling / residual SpMVs
  std::vector<uint16_t> Ap, Ai, Acol;  // CSC of A (Ap has n+1 entries, fits: nnzA < 65536)
  std::vector<uint16_t> Arp, Ark;      // CSR of A: row pointers, CSC position of each entry
  std::vector<uint16_t> Arj;           // CSR of A: column of each entry
  std::vector<uint16_t> Pi, Pcol;      // upper CSC of P: row / column of each entry
  std::vector<uint16_t> Psp, Psk, Pso; // symmetric traversal: per column j the P entries of
                                       // column j and row j, their position and the other index
  Ell ellA, ellAt, ellP;  // A x (rows of A), A' y (columns), P x (symmetric rows of P)
  int levels_fwd = 0, levels_bwd = 0;
  std::vector<int> fwd_level_steps, bwd_level_steps;  // solve steps of each level (diagnostics)
  std::string error;
};

// Physical-slot masks of the diagonal pass (Plan::bcopy) from Plan::bcopy_row and the final slot
// maps wsx / wsz: call after the layout is final (build_plan_tuned does).
void finish_copy_masks(Plan& plan);

// Builds the plan; returns false (with plan.error set) if the structure is unsupported.
// capM / capW: per block, max entries of the block inverse and max solve terms of its w-tasks.
// paired: solve steps with segments 0 + 1 of a lane on one target (three atomics per lane and
// step, SOLVE_TERM_WORDS above) or with four independent segments (four atomics).
bool build_plan(int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                const int32_t* Ai, Plan& plan, int capM = 128, int capW = 384, bool paired = true,
                int waves = 1, bool mv_global = false);

// instances per CU of the one-wave kernel with the resident values in global memory (its build for
// two waves per SIMD: <= 256 registers, __launch_bounds__(64, 2)); the LDS-resident build stays at 4
// (one wave per SIMD: up to 512 registers)
constexpr int MV_GLOBAL_MAX_PER_CU = 5;

// build_plan with the block caps and the step kind chosen per structure: over a grid of (capM <=
// 192, capW) x {paired, unpaired}, the plan with the most instances per CU (LDS image within
// lds_per_cu / k for k <= max_per_cu), then the least solve-step cost per ADMM iteration (a paired
// step costs 0.92 of an unpaired one: one atomic of four saved), then the smallest blocks, then the
// fewest factorization steps.  capM / capW > 0 force a single build (MPCQP_PAIRED=0/1 forces the
// step kind).  Results are memoised per structure within the process.
bool build_plan_tuned(int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                      const int32_t* Ai, Plan& plan, int capM, int capW, int lds_per_cu = 163840,
                      int max_per_cu = 4, int waves = 1, bool mat_first = false);

// ---- lds_layout.cpp: LDS bank-conflict model and optimiser of the solve steps
// Modelled LDS cycles of one ADMM iteration's solve work for one wave (MI355X_MICROARCH.md, LDS):
// every ds_read_b64 serves two 32-lane halves, one cycle per distinct address on the busiest bank
// (double slot mod 32; equal addresses broadcast); every ds_add_f64 / ds_write_b64 serves four
// 16-lane groups, one cycle per lane on the busiest bank (slot mod 16; equal addresses serialise).
struct LdsModel {
  long read = 0, atomic = 0, vec = 0;  // solve-step reads, solve-step atomics, vector passes
  long floor = 0;                      // the same instructions without any conflict
};
LdsModel model_lds(const Plan& pl);
// Rewrites the plan so the solve steps and the per-iteration vector passes conflict less: segments
// move between positions of their step, terms swap operands or segments, unused segments get
// sinks and zero slots in free banks, and the slots of the solve-read matrix values (within the
// L-live and N | G | G' regions) and of the vector entries (W, C and 1/D together) are permuted.
// Every change is a relabelling or a reordering of exact no-op / commutative work except the order
// of the atomic additions into one target (rounding only).  Deterministic.
void optimize_lds(Plan& pl);

// ---- emulate.cpp: host interpretation of the device program (diagnostics and tests only)
// One instance: KKT assembly from Px (upper CSC of P), Ax (CSC of A), sigma and rho_vec (m), the
// factorization schedule, the flat pass, the tail, then one forward / diagonal / backward solve of
// K [x; nu] = rhs (n + m, original order); writes sol (n + m).  Atomic additions are applied in
// lane order (the device's order within one instruction may differ: rounding only).
// the same in two parts: assembly + factorization into the LDS image v, then one solve on it (v's
// W / C regions are rewritten by every solve; the factor is kept)
void emulate_factor(const Plan& pl, const double* Px, const double* Ax, double sigma,
                    const double* rho_vec, std::vector<double>& v);
bool emulate_solve(const Plan& pl, std::vector<double>& v, const double* rhs, double* sol);
bool emulate_kkt_solve(const Plan& pl, const double* Px, const double* Ax, double sigma,
                       const double* rho_vec, const double* rhs, double* sol);

}  // namespace mpcqp
