// symbolic.hpp -- host-side symbolic analysis of the batched MPC-QP KKT system and compilation of
// the level schedules that the HIP kernel interprets.
//
// The KKT matrix is OSQP's quasi-definite  [[P + sigma I, A'], [A, -diag(1/rho)]]  (OSQP 0.6
// kkt.c form_KKT), permuted by the same exact minimum-degree ordering the oracle uses, so the
// device factor L D L' has exactly the oracle's (and QDLDL's) sparsity.  Because all instances of
// a batch share the pattern, everything here is computed once per handle; per-instance work on
// the GPU is purely numeric.
//
// Level schedules.  Factorization (left-looking, dot-product form), forward solve L w = b and
// backward solve L' x = w are each cut into levels of mutually independent "tasks"; a task writes
// one LDS slot  v[t] <- v[t] - sum_k prod(terms_k)  (2-factor terms for the solves, 3-factor terms
// L_ik * L_jk * D_k for the factorization).  A level is packed into one or more 64-lane "steps":
// a task gets an aligned group of g = 2^glog lanes, each lane accumulates <= C terms and the group
// reduces with an xor butterfly; the group's first lane writes the slot.  Scale steps apply
// L_ij *= 1/D_j after each factorization level.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mpcqp {

enum StepKind : uint32_t { KIND_DOT2 = 0, KIND_DOT3 = 1, KIND_SCALE = 2 };

// One 64-lane step.  meta[off_meta + lane], terms[off_terms + c * cnt + lane] for lane < cnt.
struct StepHdr {
  uint32_t off_meta;
  uint32_t off_terms;
  uint32_t cnt;  // lanes with a record (<= 64)
  uint32_t cfg;  // C | glog << 8 | kind << 16
};

// meta bits
constexpr uint32_t META_TGT_MASK = 0xffffu;
constexpr int META_GLOG_SHIFT = 16;  // 3 bits: this lane's group size log2
constexpr uint32_t META_HEAD = 1u << 19;
constexpr uint32_t META_ISD = 1u << 20;  // factorization: target is D_j -> also write 1/D_j
constexpr uint32_t META_ZERO = 1u << 21; // v[t] <- -sum (instead of v[t] - sum)
constexpr uint32_t META_ACTIVE = 1u << 31;

struct Plan {
  int n = 0, m = 0, nk = 0, nnzP = 0, nnzA = 0, nnzL = 0;
  std::vector<int32_t> perm, pinv, Lp, Li, etree;
  // LDS layout, in doubles: L | 1/D | W (solve vector) | C (accumulators) | N (negated block
  // inverses) | G | G' | ZERO ONE MONE pad
  int LX = 0, DINV = 0, W = 0, CACC = 0, NB = 0, GB = 0, GPB = 0, ZERO = 0, ONE = 0, MONE = 0;
  int LDS_N = 0;
  // blocked substitution: contiguous blocks of the permuted order
  std::vector<int32_t> block_start;  // T + 1 entries
  int nN = 0, nG = 0, nGP = 0;
  // scaling-phase overlay of the same LDS: scaled P, scaled A, D_temp, E_temp
  int S_P = 0, S_A = 0, S_DT = 0, S_ET = 0;
  // KKT assembly: LDS slot of each P entry (diagonal -> D slot), A entry, rho diagonal,
  // sigma diagonal (D slot of x_j)
  std::vector<uint16_t> slotP, slotA, slotRho, slotSig;
  // LDS slot (permuted position in the W region) of x_i and z_i
  std::vector<uint16_t> wsx, wsz;
  // schedules
  std::vector<StepHdr> fac, fwd, bwd;
  std::vector<uint32_t> meta, terms2;    // factorization pools (global memory)
  std::vector<uint32_t> smeta, sterms;   // solve pools (copied into LDS, shared per workgroup)
  std::vector<uint64_t> terms3;
  // matrix structure for scaling / residual SpMVs
  std::vector<uint16_t> Ap, Ai, Acol;  // CSC of A (Ap has n+1 entries, fits: nnzA < 65536)
  std::vector<uint16_t> Arp, Ark;      // CSR of A: row pointers, CSC position of each entry
  std::vector<uint16_t> Arj;           // CSR of A: column of each entry
  std::vector<uint16_t> Pi, Pcol;      // upper CSC of P: row / column of each entry
  std::vector<uint16_t> Psp, Psk, Pso; // symmetric traversal: per column j the P entries of
                                       // column j and row j, their position and the other index
  int levels_fwd = 0, levels_bwd = 0;
  std::string error;
};

// Builds the plan; returns false (with plan.error set) if the structure is unsupported.
// max_c / max_c3: max terms per lane per solve / factorization step before a task is widened to
// more lanes.
// capM / capW: per block, max entries of the block inverse and max solve terms of its w-tasks.
bool build_plan(int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                const int32_t* Ai, int max_c, int max_c3, Plan& plan, int capM = 128,
                int capW = 384);

}  // namespace mpcqp
