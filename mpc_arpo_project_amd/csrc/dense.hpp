// dense.hpp -- host-side plan of the dense-inverse engine (dense.hip) for small QPs.
//
// The ADMM linear system of OSQP 0.6 (kkt.c: [[P + sigma I, A'], [A, -diag(1/rho)]]) is solved in
// its reduced form  (P + sigma I + A' diag(rho) A) x~ = sigma x - q + A'(rho z - y),  z~ = A x~,
// which is the same step (the KKT system's Schur complement on the constraint block).  For
// n <= 128 the inverse of the n x n matrix M is formed explicitly once per (re)factorization and
// kept in registers (one 64-entry half row per thread), so an ADMM iteration is a dense mat-vec
// with no sequential dependency chain.  This file compiles the problem structure into the index
// lists the kernel reads: CSC / CSR / symmetric traversals of A and P, and the term lists that
// form M column block by column block.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mpcqp {

constexpr int DENSE_THREADS = 512;  // threads per instance (8 waves: 2 row halves x 4 column groups)
constexpr int DENSE_CG = DENSE_THREADS / 128;  // column groups of M^-1
constexpr int DENSE_W = 128 / DENSE_CG;        // columns of M^-1 per thread
constexpr int DENSE_NMAX = 128;     // n (padded with identity to 128)
constexpr int DENSE_MMAX = 256;     // m (one constraint row per thread)
constexpr int DENSE_BLK = 16;       // columns of M formed per LDS staging pass
constexpr int DENSE_KR = 8;         // ELL width of the rows of A (A x)
constexpr int DENSE_KC = 10;        // ELL width of the columns of A (A' y); longer columns are
constexpr int DENSE_NLONG = 2;      //   summed cooperatively by a whole wave (at most this many,
constexpr int DENSE_LONGK = 64;     //   each with at most this many terms)

struct DensePlan {
  int n = 0, m = 0, nnzP = 0, nnzA = 0;
  // A: CSC (Ap, Ai, Acol), CSR (Arp, Ark = CSC position, Arj = column)
  std::vector<uint16_t> Ap, Ai, Acol, Arp, Ark, Arj;
  // P (upper CSC): row / column of each entry; symmetric traversal per column j: Psp (n + 1),
  // Psk (position), Pso (other index) -- the order OSQP's symmetric mat-vec adds the terms in
  std::vector<uint16_t> Pi, Pcol, Psp, Psk, Pso;
  // M = P + sigma I + A' diag(rho) A, entries grouped by column block of DENSE_BLK columns:
  // entries [eptr[b], eptr[b+1]) of block b; entry e: row ei, local column ej, P position ep
  // (0xffff: none), flags ef (1: + sigma, 2: constant 1 = identity padding), terms
  // [tptr[e], tptr[e+1]): A positions ta1, ta2 and row tr (value A[ta1] * rho[tr] * A[ta2])
  std::vector<uint16_t> eptr, ei, ej, ep, ef, tptr, ta1, ta2, tr;
  int nent = 0, nterm = 0;
  // ELL forms for the iteration mat-vecs: rows of A [DENSE_KR][mp] (mp = m rounded up to 8) and
  // columns [DENSE_KC][DENSE_NMAX]: position of the value in A's CSC order (0xffff: padding) and
  // index of the input element; long columns: output column, term positions / rows
  int mp = 0;
  std::vector<uint16_t> erp, eri, ecp, eci;
  int nlong = 0;
  int long_col[DENSE_NLONG] = {}, long_cnt[DENSE_NLONG] = {};
  std::vector<uint16_t> lgp, lgi;  // [DENSE_NLONG][DENSE_LONGK]
  std::string error;
};

// n <= 128, m <= 256, rows of A with at most DENSE_KR entries, at most DENSE_NLONG columns with
// more than DENSE_KC entries (each at most DENSE_LONGK)
bool dense_supported(int n, int m);
bool build_dense_plan(int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                      const int32_t* Ai, DensePlan& plan);

}  // namespace mpcqp
