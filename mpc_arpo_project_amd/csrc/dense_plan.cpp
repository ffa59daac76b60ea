// dense_plan.cpp -- see dense.hpp.
#include <algorithm>
#include <array>
#include <map>
#include <utility>

#include "dense.hpp"

namespace mpcqp {

bool dense_supported(int n, int m) { return n >= 1 && n <= DENSE_NMAX && m >= 1 && m <= DENSE_MMAX; }

bool build_dense_plan(int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                      const int32_t* Ai, DensePlan& pl) {
  pl = DensePlan();
  if (!dense_supported(n, m)) {
    pl.error = "dense engine: n <= 128 and m <= 256 required";
    return false;
  }
  pl.n = n, pl.m = m, pl.nnzP = Pp[n], pl.nnzA = Ap[n];
  for (int j = 0; j < n; j++) {
    for (int p = Pp[j]; p < Pp[j + 1]; p++)
      if (Pi[p] < 0 || Pi[p] > j || (p > Pp[j] && Pi[p] <= Pi[p - 1])) {
        pl.error = "P must be upper triangular CSC with sorted unique rows";
        return false;
      }
    for (int p = Ap[j]; p < Ap[j + 1]; p++)
      if (Ai[p] < 0 || Ai[p] >= m || (p > Ap[j] && Ai[p] <= Ai[p - 1])) {
        pl.error = "A must be CSC with sorted unique rows in range";
        return false;
      }
  }
  if (pl.nnzA >= 65535 || pl.nnzP >= 65535) {
    pl.error = "dense engine: too many nonzeros for 16-bit indices";
    return false;
  }
  // ---- A: CSC and CSR
  pl.Ap.resize(n + 1);
  for (int j = 0; j <= n; j++) pl.Ap[j] = (uint16_t)Ap[j];
  pl.Ai.resize(pl.nnzA);
  pl.Acol.resize(pl.nnzA);
  for (int j = 0; j < n; j++)
    for (int p = Ap[j]; p < Ap[j + 1]; p++) pl.Ai[p] = (uint16_t)Ai[p], pl.Acol[p] = (uint16_t)j;
  std::vector<int> rc(m + 1, 0);
  for (int p = 0; p < pl.nnzA; p++) rc[Ai[p] + 1]++;
  for (int i = 0; i < m; i++) rc[i + 1] += rc[i];
  pl.Arp.resize(m + 1);
  for (int i = 0; i <= m; i++) pl.Arp[i] = (uint16_t)rc[i];
  pl.Ark.resize(pl.nnzA);
  pl.Arj.resize(pl.nnzA);
  {
    std::vector<int> nx(rc.begin(), rc.end() - 1);
    for (int j = 0; j < n; j++)
      for (int p = Ap[j]; p < Ap[j + 1]; p++) {
        const int q = nx[Ai[p]]++;
        pl.Ark[q] = (uint16_t)p;
        pl.Arj[q] = (uint16_t)j;
      }
  }
  // ---- P: entries and the symmetric traversal (same order as the KKT engine's)
  pl.Pi.resize(pl.nnzP);
  pl.Pcol.resize(pl.nnzP);
  std::vector<std::vector<std::pair<int, int>>> sym(n);
  for (int j = 0; j < n; j++)
    for (int p = Pp[j]; p < Pp[j + 1]; p++) {
      const int i = Pi[p];
      pl.Pi[p] = (uint16_t)i;
      pl.Pcol[p] = (uint16_t)j;
      sym[j].push_back({p, i});
      if (i != j) sym[i].push_back({p, j});
    }
  pl.Psp.assign(n + 1, 0);
  for (int j = 0; j < n; j++) {
    pl.Psp[j + 1] = (uint16_t)(pl.Psp[j] + sym[j].size());
    for (auto& e : sym[j]) pl.Psk.push_back((uint16_t)e.first), pl.Pso.push_back((uint16_t)e.second);
  }
  // ---- entries of M = P + sigma I + A' diag(rho) A (+ identity padding to DENSE_NMAX)
  struct Ent {
    int p = -1, flags = 0;
    std::vector<std::array<int, 3>> terms;
  };
  std::map<std::pair<int, int>, Ent> ent;  // key (column j, row i)
  for (int j = 0; j < n; j++)
    for (int p = Pp[j]; p < Pp[j + 1]; p++) {
      const int i = Pi[p];
      ent[{j, i}].p = p;
      ent[{i, j}].p = p;
    }
  for (int j = 0; j < n; j++) ent[{j, j}].flags |= 1;
  for (int j = n; j < DENSE_NMAX; j++) ent[{j, j}].flags |= 2;
  for (int r = 0; r < m; r++)  // rows in order: each entry's terms are summed by ascending row
    for (int a = rc[r]; a < rc[r + 1]; a++)
      for (int b = rc[r]; b < rc[r + 1]; b++) {
        const int p1 = pl.Ark[a], c1 = pl.Arj[a], p2 = pl.Ark[b], c2 = pl.Arj[b];
        ent[{c2, c1}].terms.push_back({p1, p2, r});  // M[c1][c2] += A[p1] rho[r] A[p2]
      }
  const int nblk = DENSE_NMAX / DENSE_BLK;
  pl.eptr.assign(nblk + 1, 0);
  pl.tptr.push_back(0);
  for (auto& kv : ent) {
    const int j = kv.first.first, i = kv.first.second;
    pl.eptr[j / DENSE_BLK + 1]++;
    pl.ei.push_back((uint16_t)i);
    pl.ej.push_back((uint16_t)(j % DENSE_BLK));
    pl.ep.push_back(kv.second.p >= 0 ? (uint16_t)kv.second.p : (uint16_t)0xffff);
    pl.ef.push_back((uint16_t)kv.second.flags);
    for (auto& t : kv.second.terms) {
      pl.ta1.push_back((uint16_t)t[0]);
      pl.ta2.push_back((uint16_t)t[1]);
      pl.tr.push_back((uint16_t)t[2]);
    }
    pl.tptr.push_back((uint16_t)pl.ta1.size());
    if (pl.ta1.size() >= 65535) {
      pl.error = "dense engine: too many terms in A' diag(rho) A";
      return false;
    }
  }
  for (int b = 0; b < nblk; b++) pl.eptr[b + 1] += pl.eptr[b];  // map order is column-major
  pl.nent = (int)pl.ei.size();
  pl.nterm = (int)pl.ta1.size();
  // ---- ELL forms (terms in CSR / CSC order, as the mat-vecs sum them)
  pl.mp = (m + 7) & ~7;
  pl.erp.assign((size_t)DENSE_KR * pl.mp, 0xffff);
  pl.eri.assign((size_t)DENSE_KR * pl.mp, 0);
  for (int i = 0; i < m; i++) {
    if (rc[i + 1] - rc[i] > DENSE_KR) {
      pl.error = "dense engine: a row of A has more than 8 entries";
      return false;
    }
    for (int q = rc[i]; q < rc[i + 1]; q++) {
      const int k = q - rc[i];
      pl.erp[(size_t)k * pl.mp + i] = pl.Ark[q];
      pl.eri[(size_t)k * pl.mp + i] = pl.Arj[q];
    }
  }
  pl.ecp.assign((size_t)DENSE_KC * DENSE_NMAX, 0xffff);
  pl.eci.assign((size_t)DENSE_KC * DENSE_NMAX, 0);
  pl.lgp.assign((size_t)DENSE_NLONG * DENSE_LONGK, 0xffff);
  pl.lgi.assign((size_t)DENSE_NLONG * DENSE_LONGK, 0);
  for (int j = 0; j < n; j++) {
    const int cnt = Ap[j + 1] - Ap[j];
    if (cnt > DENSE_KC) {
      if (pl.nlong >= DENSE_NLONG || cnt > DENSE_LONGK) {
        pl.error = "dense engine: too many long columns in A";
        return false;
      }
      pl.long_col[pl.nlong] = j;
      pl.long_cnt[pl.nlong] = cnt;
      for (int k = 0; k < cnt; k++) {
        pl.lgp[(size_t)pl.nlong * DENSE_LONGK + k] = (uint16_t)(Ap[j] + k);
        pl.lgi[(size_t)pl.nlong * DENSE_LONGK + k] = (uint16_t)Ai[Ap[j] + k];
      }
      pl.nlong++;
      continue;
    }
    for (int k = 0; k < cnt; k++) {
      pl.ecp[(size_t)k * DENSE_NMAX + j] = (uint16_t)(Ap[j] + k);
      pl.eci[(size_t)k * DENSE_NMAX + j] = (uint16_t)Ai[Ap[j] + k];
    }
  }
  return true;
}

}  // namespace mpcqp
