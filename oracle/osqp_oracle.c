/*
 * osqp_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of OSQP 0.6.x (see osqp_oracle.h
 * for provenance, scope and the two documented deviations).  Used as the parity checker for the
 * HIP engine and as the timed CPU baseline ("port").  Never linked by the product.
 *
 * Section map (OSQP 0.6 source file the restated function follows):
 *   csc helpers ............................ lin_alg.c (mat_vec, mat_tpose_vec, norms)
 *   scale_data / unscale_data .............. scaling.c
 *   set_rho_vec / update_rho_vec ........... auxil.c
 *   form_kkt + min-degree ordering ......... kkt.c form_KKT (+ AMD replaced by min degree)
 *   etree / factor / solve ................. qdldl.c QDLDL_etree / QDLDL_factor / QDLDL_solve
 *   admm step, residuals, termination ...... auxil.c, osqp.c osqp_solve
 *   polish ................................. polish.c
 */
#include "osqp_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define RHO_MIN 1e-06
#define RHO_MAX 1e06
#define RHO_EQ_OVER_RHO_INEQ 1e03
#define RHO_TOL 1e-04
#define MIN_SCALING 1e-04
#define MAX_SCALING 1e+04
#define DIVISION_TOL 1e-30 /* OSQP_DIVISION_TOL = 1.0 / OSQP_INFTY */
#define ADAPTIVE_RHO_MULTIPLE_TERMINATION 4
#define ADAPTIVE_RHO_FIXED 100

static double dmax(double a, double b) { return a > b ? a : b; }
static double dmin(double a, double b) { return a < b ? a : b; }

/* ---------------------------------------------------------------- CSC helpers (lin_alg.c) */
typedef struct {
  int m, n;
  int *p, *i;
  double *x;
} csc;

static csc *csc_alloc(int m, int n, int nnz) {
  csc *M = (csc *)calloc(1, sizeof(csc));
  M->m = m;
  M->n = n;
  M->p = (int *)calloc((size_t)n + 1, sizeof(int));
  M->i = (int *)calloc((size_t)(nnz > 0 ? nnz : 1), sizeof(int));
  M->x = (double *)calloc((size_t)(nnz > 0 ? nnz : 1), sizeof(double));
  return M;
}
static void csc_free(csc *M) {
  if (!M) return;
  free(M->p);
  free(M->i);
  free(M->x);
  free(M);
}
static csc *csc_copy(int m, int n, const int *p, const int *i, const double *x) {
  int nnz = p[n];
  csc *M = csc_alloc(m, n, nnz);
  memcpy(M->p, p, sizeof(int) * ((size_t)n + 1));
  memcpy(M->i, i, sizeof(int) * (size_t)nnz);
  memcpy(M->x, x, sizeof(double) * (size_t)nnz);
  return M;
}
static int csc_nnz(const csc *M) { return M->p[M->n]; }

/* y = A*x (plus_eq: 0 overwrite, 1 add, -1 subtract) -- lin_alg.c mat_vec */
static void mat_vec(const csc *A, const double *x, double *y, int plus_eq) {
  int i, j;
  if (!plus_eq)
    for (i = 0; i < A->m; i++) y[i] = 0.0;
  if (A->p[A->n] == 0) return;
  if (plus_eq == -1) {
    for (j = 0; j < A->n; j++)
      for (i = A->p[j]; i < A->p[j + 1]; i++) y[A->i[i]] -= A->x[i] * x[j];
  } else {
    for (j = 0; j < A->n; j++)
      for (i = A->p[j]; i < A->p[j + 1]; i++) y[A->i[i]] += A->x[i] * x[j];
  }
}
/* y = A'*x (skip_diag for the symmetric-upper trick) -- lin_alg.c mat_tpose_vec */
static void mat_tpose_vec(const csc *A, const double *x, double *y, int plus_eq, int skip_diag) {
  int i, j, k;
  if (!plus_eq)
    for (i = 0; i < A->n; i++) y[i] = 0.0;
  if (A->p[A->n] == 0) return;
  if (plus_eq == -1) {
    if (skip_diag) {
      for (j = 0; j < A->n; j++)
        for (k = A->p[j]; k < A->p[j + 1]; k++) {
          i = A->i[k];
          y[j] -= i == j ? 0.0 : A->x[k] * x[i];
        }
    } else {
      for (j = 0; j < A->n; j++)
        for (k = A->p[j]; k < A->p[j + 1]; k++) y[j] -= A->x[k] * x[A->i[k]];
    }
  } else {
    if (skip_diag) {
      for (j = 0; j < A->n; j++)
        for (k = A->p[j]; k < A->p[j + 1]; k++) {
          i = A->i[k];
          y[j] += i == j ? 0.0 : A->x[k] * x[i];
        }
    } else {
      for (j = 0; j < A->n; j++)
        for (k = A->p[j]; k < A->p[j + 1]; k++) y[j] += A->x[k] * x[A->i[k]];
    }
  }
}
/* full symmetric P*x from its upper triangle: mat_vec + mat_tpose_vec(skip_diag) */
static void sym_mat_vec(const csc *P, const double *x, double *y) {
  mat_vec(P, x, y, 0);
  mat_tpose_vec(P, x, y, 1, 1);
}
static double vec_norm_inf(const double *v, int n) {
  double r = 0.0;
  for (int i = 0; i < n; i++) r = dmax(r, fabs(v[i]));
  return r;
}
static double vec_scaled_norm_inf(const double *S, const double *v, int n) {
  double r = 0.0;
  for (int i = 0; i < n; i++) r = dmax(r, fabs(S[i] * v[i]));
  return r;
}
static double vec_prod(const double *a, const double *b, int n) {
  double r = 0.0;
  for (int i = 0; i < n; i++) r += a[i] * b[i];
  return r;
}
static double vec_mean(const double *a, int n) {
  double s = 0.0;
  for (int i = 0; i < n; i++) s += a[i];
  return s / n;
}
static void mat_premult_diag(csc *A, const double *d) {
  for (int j = 0; j < A->n; j++)
    for (int i = A->p[j]; i < A->p[j + 1]; i++) A->x[i] *= d[A->i[i]];
}
static void mat_postmult_diag(csc *A, const double *d) {
  for (int j = 0; j < A->n; j++)
    for (int i = A->p[j]; i < A->p[j + 1]; i++) A->x[i] *= d[j];
}
static void mat_mult_scalar(csc *A, double sc) {
  for (int i = 0; i < A->p[A->n]; i++) A->x[i] *= sc;
}
static void mat_inf_norm_cols(const csc *M, double *E) {
  for (int j = 0; j < M->n; j++) {
    E[j] = 0.;
    for (int p = M->p[j]; p < M->p[j + 1]; p++) E[j] = dmax(fabs(M->x[p]), E[j]);
  }
}
static void mat_inf_norm_rows(const csc *M, double *E) {
  for (int i = 0; i < M->m; i++) E[i] = 0.;
  for (int j = 0; j < M->n; j++)
    for (int p = M->p[j]; p < M->p[j + 1]; p++) {
      int i = M->i[p];
      E[i] = dmax(fabs(M->x[p]), E[i]);
    }
}
static void mat_inf_norm_cols_sym_triu(const csc *M, double *E) {
  for (int j = 0; j < M->n; j++) E[j] = 0.;
  for (int j = 0; j < M->n; j++)
    for (int p = M->p[j]; p < M->p[j + 1]; p++) {
      int i = M->i[p];
      double a = fabs(M->x[p]);
      E[j] = dmax(a, E[j]);
      if (i != j) E[i] = dmax(a, E[i]);
    }
}
static double quad_form(const csc *P, const double *x) {
  double r = 0.;
  for (int j = 0; j < P->n; j++)
    for (int p = P->p[j]; p < P->p[j + 1]; p++) {
      int i = P->i[p];
      if (i == j)
        r += .5 * P->x[p] * x[i] * x[i];
      else if (i < j)
        r += P->x[p] * x[i] * x[j];
    }
  return r;
}

/* ---------------------------------------------------------------- KKT linear system (QDLDL) */
typedef struct {
  int nk;      /* n + m */
  int *perm;   /* perm[k] = original index placed at position k */
  int *pinv;   /* pinv[orig] = position */
  int *Kp, *Ki; /* permuted upper-triangular KKT pattern (CSC) */
  double *Kx;
  int *PtoK, *AtoK, *rhotoK, *sigtoK; /* value maps into Kx */
  int *etree, *Lnz, *Lp, *Li;
  double *Lx, *D, *Dinv;
  int *iwork;
  unsigned char *bwork;
  double *fwork, *bp;
  int solve_order; /* parity-floor diagnostics (oqp_set_solve_order), 0 = QDLDL's */
} kkt_sys;

/* Exact minimum-degree ordering on the symmetric pattern given by an adjacency bitmatrix.
 * Ties are broken by the lowest index.  Replaces SuiteSparse AMD (see header). */
static void min_degree_order(int nk, unsigned char *adj /* nk*nk, symmetric, no diag */,
                             int *perm) {
  unsigned char *alive = (unsigned char *)malloc((size_t)nk);
  int *deg = (int *)malloc(sizeof(int) * (size_t)nk);
  int *nbr = (int *)malloc(sizeof(int) * (size_t)nk);
  memset(alive, 1, (size_t)nk);
  for (int i = 0; i < nk; i++) {
    int d = 0;
    for (int j = 0; j < nk; j++) d += adj[(size_t)i * nk + j];
    deg[i] = d;
  }
  for (int k = 0; k < nk; k++) {
    int best = -1;
    for (int i = 0; i < nk; i++)
      if (alive[i] && (best < 0 || deg[i] < deg[best])) best = i;
    perm[k] = best;
    alive[best] = 0;
    int cnt = 0;
    for (int j = 0; j < nk; j++)
      if (alive[j] && adj[(size_t)best * nk + j]) nbr[cnt++] = j;
    /* eliminate: neighbours become a clique */
    for (int a = 0; a < cnt; a++) {
      int ia = nbr[a];
      adj[(size_t)ia * nk + best] = 0;
      for (int b = 0; b < cnt; b++) {
        int ib = nbr[b];
        if (ia != ib && !adj[(size_t)ia * nk + ib]) {
          adj[(size_t)ia * nk + ib] = 1;
          deg[ia]++;
        }
      }
      deg[ia]--; /* lost `best` */
    }
  }
  free(alive);
  free(deg);
  free(nbr);
}

/* qdldl.c QDLDL_etree */
static int qdldl_etree(int n, const int *Ap, const int *Ai, int *work, int *Lnz, int *etree) {
  int i, j, p, sum = 0;
  for (i = 0; i < n; i++) {
    work[i] = 0;
    Lnz[i] = 0;
    etree[i] = -1;
    if (Ap[i] == Ap[i + 1]) return -1;
  }
  for (j = 0; j < n; j++) {
    work[j] = j;
    for (p = Ap[j]; p < Ap[j + 1]; p++) {
      i = Ai[p];
      if (i > j) return -1;
      while (work[i] != j) {
        if (etree[i] == -1) etree[i] = j;
        Lnz[i]++;
        work[i] = j;
        i = etree[i];
      }
    }
  }
  for (i = 0; i < n; i++) sum += Lnz[i];
  return sum;
}

/* qdldl.c QDLDL_factor (up-looking LDL^T) */
static int qdldl_factor(int n, const int *Ap, const int *Ai, const double *Ax, int *Lp, int *Li,
                        double *Lx, double *D, double *Dinv, const int *Lnz, const int *etree,
                        unsigned char *bwork, int *iwork, double *fwork) {
  int i, j, k, nnzY, bidx, cidx, nextIdx, nnzE, tmpIdx, positive = 0;
  unsigned char *yMarkers = bwork;
  int *yIdx = iwork, *elimBuffer = iwork + n, *LNext = iwork + 2 * n;
  double *yVals = fwork;
  Lp[0] = 0;
  for (i = 0; i < n; i++) {
    Lp[i + 1] = Lp[i] + Lnz[i];
    yMarkers[i] = 0;
    yVals[i] = 0.0;
    D[i] = 0.0;
    LNext[i] = Lp[i];
  }
  D[0] = Ax[0];
  if (D[0] == 0.0) return -1;
  if (D[0] > 0.0) positive++;
  Dinv[0] = 1 / D[0];
  for (k = 1; k < n; k++) {
    nnzY = 0;
    tmpIdx = Ap[k + 1];
    for (i = Ap[k]; i < tmpIdx; i++) {
      bidx = Ai[i];
      if (bidx == k) {
        D[k] = Ax[i];
        continue;
      }
      yVals[bidx] = Ax[i];
      nextIdx = bidx;
      if (yMarkers[nextIdx] == 0) {
        yMarkers[nextIdx] = 1;
        elimBuffer[0] = nextIdx;
        nnzE = 1;
        nextIdx = etree[bidx];
        while (nextIdx != -1 && nextIdx < k) {
          if (yMarkers[nextIdx] == 1) break;
          yMarkers[nextIdx] = 1;
          elimBuffer[nnzE] = nextIdx;
          nnzE++;
          nextIdx = etree[nextIdx];
        }
        while (nnzE) yIdx[nnzY++] = elimBuffer[--nnzE];
      }
    }
    for (i = nnzY - 1; i >= 0; i--) {
      cidx = yIdx[i];
      tmpIdx = LNext[cidx];
      double yc = yVals[cidx];
      for (j = Lp[cidx]; j < tmpIdx; j++) yVals[Li[j]] -= Lx[j] * yc;
      Li[tmpIdx] = k;
      Lx[tmpIdx] = yc * Dinv[cidx];
      D[k] -= yc * Lx[tmpIdx];
      LNext[cidx]++;
      yVals[cidx] = 0.0;
      yMarkers[cidx] = 0;
    }
    if (D[k] == 0.0) return -1;
    if (D[k] > 0.0) positive++;
    Dinv[k] = 1 / D[k];
  }
  return positive;
}

static void qdldl_solve(int n, const int *Lp, const int *Li, const double *Lx, const double *Dinv,
                        double *x) {
  for (int i = 0; i < n; i++) {
    double v = x[i];
    for (int j = Lp[i]; j < Lp[i + 1]; j++) x[Li[j]] -= Lx[j] * v;
  }
  for (int i = 0; i < n; i++) x[i] *= Dinv[i];
  for (int i = n - 1; i >= 0; i--) {
    double v = x[i];
    for (int j = Lp[i]; j < Lp[i + 1]; j++) v -= Lx[j] * x[Li[j]];
    x[i] = v;
  }
}

/* Build the KKT system [[P + sigma I, A'], [A, -diag(param2)]] (kkt.c form_KKT), its min-degree
 * permutation and QDLDL symbolic factorization.  Values are filled by kkt_fill(). */
static kkt_sys *kkt_init(const csc *P, const csc *A) {
  int n = P->n, m = A->m, nk = n + m;
  kkt_sys *s = (kkt_sys *)calloc(1, sizeof(kkt_sys));
  s->nk = nk;
  /* symmetric adjacency for ordering */
  unsigned char *adj = (unsigned char *)calloc((size_t)nk * nk, 1);
  for (int j = 0; j < n; j++)
    for (int p = P->p[j]; p < P->p[j + 1]; p++) {
      int i = P->i[p];
      if (i != j) adj[(size_t)i * nk + j] = adj[(size_t)j * nk + i] = 1;
    }
  for (int j = 0; j < n; j++)
    for (int p = A->p[j]; p < A->p[j + 1]; p++) {
      int r = n + A->i[p];
      adj[(size_t)r * nk + j] = adj[(size_t)j * nk + r] = 1;
    }
  s->perm = (int *)malloc(sizeof(int) * (size_t)nk);
  s->pinv = (int *)malloc(sizeof(int) * (size_t)nk);
  min_degree_order(nk, adj, s->perm);
  free(adj);
  for (int k = 0; k < nk; k++) s->pinv[s->perm[k]] = k;

  /* entries of the upper KKT in original coordinates: P upper (incl. forced diagonal), A' block,
   * -1/rho diagonal.  Collect (row, col) in permuted coordinates, upper triangle. */
  int nnzP = csc_nnz(P), nnzA = csc_nnz(A);
  int maxe = nnzP + n + nnzA + m;
  int *er = (int *)malloc(sizeof(int) * (size_t)maxe), *ec = (int *)malloc(sizeof(int) * (size_t)maxe);
  int *etag = (int *)malloc(sizeof(int) * (size_t)maxe); /* encodes the source */
  int ne = 0;
  for (int j = 0; j < n; j++) {
    int has_diag = 0;
    for (int p = P->p[j]; p < P->p[j + 1]; p++) {
      int i = P->i[p];
      if (i == j) has_diag = 1;
      er[ne] = i, ec[ne] = j, etag[ne] = p; /* P entry p */
      ne++;
    }
    if (!has_diag) {
      er[ne] = j, ec[ne] = j, etag[ne] = -1 - j; /* sigma-only diagonal */
      ne++;
    }
  }
  for (int j = 0; j < n; j++)
    for (int p = A->p[j]; p < A->p[j + 1]; p++) {
      er[ne] = j, ec[ne] = n + A->i[p], etag[ne] = nnzP + p; /* A entry p */
      ne++;
    }
  for (int i = 0; i < m; i++) {
    er[ne] = n + i, ec[ne] = n + i, etag[ne] = nnzP + nnzA + i; /* rho diagonal */
    ne++;
  }
  /* permute to upper triangle and build CSC with a slot map */
  int *cnt = (int *)calloc((size_t)nk + 1, sizeof(int));
  for (int e = 0; e < ne; e++) {
    int a = s->pinv[er[e]], b = s->pinv[ec[e]];
    int col = a > b ? a : b;
    cnt[col + 1]++;
  }
  s->Kp = (int *)malloc(sizeof(int) * ((size_t)nk + 1));
  s->Kp[0] = 0;
  for (int k = 0; k < nk; k++) s->Kp[k + 1] = s->Kp[k] + cnt[k + 1];
  s->Ki = (int *)malloc(sizeof(int) * (size_t)ne);
  s->Kx = (double *)calloc((size_t)ne, sizeof(double));
  int *next = (int *)malloc(sizeof(int) * (size_t)nk);
  for (int k = 0; k < nk; k++) next[k] = s->Kp[k];
  int *slot = (int *)malloc(sizeof(int) * (size_t)ne);
  for (int e = 0; e < ne; e++) {
    int a = s->pinv[er[e]], b = s->pinv[ec[e]];
    int row = a < b ? a : b, col = a > b ? a : b;
    slot[e] = next[col];
    s->Ki[next[col]++] = row;
  }
  /* sort row indices within each column (QDLDL requires the diagonal anywhere, but keep sorted
   * for determinism); carry the slot map along */
  int *where = (int *)malloc(sizeof(int) * (size_t)ne); /* position -> entry */
  for (int e = 0; e < ne; e++) where[slot[e]] = e;
  for (int k = 0; k < nk; k++) {
    for (int a = s->Kp[k] + 1; a < s->Kp[k + 1]; a++) {
      int ri = s->Ki[a], we = where[a], b = a - 1;
      while (b >= s->Kp[k] && s->Ki[b] > ri) {
        s->Ki[b + 1] = s->Ki[b];
        where[b + 1] = where[b];
        b--;
      }
      s->Ki[b + 1] = ri;
      where[b + 1] = we;
    }
  }
  for (int pos = 0; pos < ne; pos++) slot[where[pos]] = pos;
  s->PtoK = (int *)malloc(sizeof(int) * (size_t)(nnzP > 0 ? nnzP : 1));
  s->AtoK = (int *)malloc(sizeof(int) * (size_t)(nnzA > 0 ? nnzA : 1));
  s->rhotoK = (int *)malloc(sizeof(int) * (size_t)m);
  s->sigtoK = (int *)malloc(sizeof(int) * (size_t)n);
  for (int j = 0; j < n; j++) s->sigtoK[j] = -1;
  for (int e = 0; e < ne; e++) {
    int t = etag[e];
    if (t < 0)
      s->sigtoK[-1 - t] = slot[e];
    else if (t < nnzP) {
      s->PtoK[t] = slot[e];
      if (er[e] == ec[e]) s->sigtoK[er[e]] = slot[e];
    } else if (t < nnzP + nnzA)
      s->AtoK[t - nnzP] = slot[e];
    else
      s->rhotoK[t - nnzP - nnzA] = slot[e];
  }
  free(er), free(ec), free(etag), free(cnt), free(next), free(slot), free(where);

  s->etree = (int *)malloc(sizeof(int) * (size_t)nk);
  s->Lnz = (int *)malloc(sizeof(int) * (size_t)nk);
  s->iwork = (int *)malloc(sizeof(int) * 3 * (size_t)nk);
  s->bwork = (unsigned char *)malloc((size_t)nk);
  s->fwork = (double *)malloc(sizeof(double) * (size_t)nk);
  s->bp = (double *)malloc(sizeof(double) * (size_t)nk);
  int sumL = qdldl_etree(nk, s->Kp, s->Ki, s->iwork, s->Lnz, s->etree);
  if (sumL < 0) sumL = 0;
  s->Lp = (int *)malloc(sizeof(int) * ((size_t)nk + 1));
  s->Li = (int *)malloc(sizeof(int) * (size_t)(sumL > 0 ? sumL : 1));
  s->Lx = (double *)malloc(sizeof(double) * (size_t)(sumL > 0 ? sumL : 1));
  s->D = (double *)malloc(sizeof(double) * (size_t)nk);
  s->Dinv = (double *)malloc(sizeof(double) * (size_t)nk);
  return s;
}

static void kkt_free(kkt_sys *s) {
  if (!s) return;
  free(s->perm), free(s->pinv), free(s->Kp), free(s->Ki), free(s->Kx);
  free(s->PtoK), free(s->AtoK), free(s->rhotoK), free(s->sigtoK);
  free(s->etree), free(s->Lnz), free(s->Lp), free(s->Li), free(s->Lx), free(s->D), free(s->Dinv);
  free(s->iwork), free(s->bwork), free(s->fwork), free(s->bp);
  free(s);
}

/* fill values: P + sigma I, A', -param2 diagonal; then numeric factorization */
static int kkt_fill_factor(kkt_sys *s, const csc *P, const csc *A, double sigma,
                           const double *param2) {
  int n = P->n, m = A->m;
  memset(s->Kx, 0, sizeof(double) * (size_t)s->Kp[s->nk]);
  for (int p = 0; p < csc_nnz(P); p++) s->Kx[s->PtoK[p]] += P->x[p];
  for (int j = 0; j < n; j++) s->Kx[s->sigtoK[j]] += sigma;
  for (int p = 0; p < csc_nnz(A); p++) s->Kx[s->AtoK[p]] = A->x[p];
  for (int i = 0; i < m; i++) s->Kx[s->rhotoK[i]] = -param2[i];
  int pos = qdldl_factor(s->nk, s->Kp, s->Ki, s->Kx, s->Lp, s->Li, s->Lx, s->D, s->Dinv, s->Lnz,
                         s->etree, s->bwork, s->iwork, s->fwork);
  return pos < 0 ? -1 : 0;
}

/* Parity-floor diagnostics only (oqp_set_solve_order): QDLDL's three solve phases with every
 * entry's products summed apart and subtracted once -- forward y_t = b_t - (sum_i L_ti y_i) with the
 * sum in QDLDL's column order, backward x_i = y_i - (sum_t L_ti x_t) in descending (order 1) or
 * ascending (order 2) row order.  The same solution in exact arithmetic with another valid rounding:
 * the class of difference a blocked or atomic-accumulation solve makes (the GPU engine's remaining
 * arithmetic difference from OSQP, DESIGN.md Parity). */
static void qdldl_solve_sum(int n, const int *Lp, const int *Li, const double *Lx, const double *Dinv,
                            double *x, double *acc, int order) {
  for (int i = 0; i < n; i++) acc[i] = 0.0;
  for (int i = 0; i < n; i++) {
    double v = x[i] - acc[i];
    x[i] = v;
    for (int j = Lp[i]; j < Lp[i + 1]; j++) acc[Li[j]] += Lx[j] * v;
  }
  for (int i = 0; i < n; i++) x[i] *= Dinv[i];
  for (int i = n - 1; i >= 0; i--) {
    double sum = 0.0;
    if (order == 1)
      for (int j = Lp[i + 1] - 1; j >= Lp[i]; j--) sum += Lx[j] * x[Li[j]];
    else
      for (int j = Lp[i]; j < Lp[i + 1]; j++) sum += Lx[j] * x[Li[j]];
    x[i] = x[i] - sum;
  }
}

/* solve K [x; nu] = b in place (original ordering) -- qdldl_interface solve (polish flavour) */
static void kkt_solve(kkt_sys *s, double *b) {
  for (int k = 0; k < s->nk; k++) s->bp[k] = b[s->perm[k]];
  qdldl_solve(s->nk, s->Lp, s->Li, s->Lx, s->Dinv, s->bp);
  for (int k = 0; k < s->nk; k++) b[s->perm[k]] = s->bp[k];
}

/* ---------------------------------------------------------------- workspace */
struct oqp_work {
  int n, m;
  csc *P, *A; /* scaled data */
  double *q, *l, *u;
  oqp_settings set;
  /* scaling */
  double *D, *Dinv, *E, *Einv, c, cinv;
  double *D_temp, *D_temp_A, *E_temp;
  /* iterates */
  double *x, *y, *z, *xz_tilde, *x_prev, *z_prev;
  double *Ax, *Px, *Aty, *delta_y, *Atdelta_y, *delta_x, *Pdelta_x, *Adelta_x;
  double *rho_vec, *rho_inv_vec;
  int *constr_type;
  kkt_sys *kkt;
  /* solution + info */
  double *sol_x, *sol_y;
  int status, iter, status_polish, rho_updates;
  double obj_val, pri_res, dua_res;
  /* parity-floor diagnostics only (oqp_set_jitter): xorshift state, 0 = off */
  unsigned long long jitter;
  /* hybrid parity runs only (oqp_set_kkt_hook): an external KKT factorization + solve in place of
   * QDLDL's, and the engine's fused updates (oqp_set_fused_updates) */
  oqp_kkt_factor_fn hook_factor;
  oqp_kkt_solve_fn hook_solve;
  void *hook_ctx;
  double *hook_sol;
  int fused;
};

/* scaling.c scale_data */
static void scale_data(oqp_work *w) {
  int n = w->n, m = w->m;
  w->c = 1.0;
  for (int i = 0; i < n; i++) w->D[i] = w->Dinv[i] = 1.;
  for (int i = 0; i < m; i++) w->E[i] = w->Einv[i] = 1.;
  for (int it = 0; it < w->set.scaling; it++) {
    mat_inf_norm_cols_sym_triu(w->P, w->D_temp);
    mat_inf_norm_cols(w->A, w->D_temp_A);
    for (int i = 0; i < n; i++) w->D_temp[i] = dmax(w->D_temp[i], w->D_temp_A[i]);
    mat_inf_norm_rows(w->A, w->E_temp);
    for (int i = 0; i < n; i++) {
      double d = w->D_temp[i];
      d = d < MIN_SCALING ? 1.0 : d;
      d = d > MAX_SCALING ? MAX_SCALING : d;
      w->D_temp[i] = 1. / sqrt(d);
    }
    for (int i = 0; i < m; i++) {
      double e = w->E_temp[i];
      e = e < MIN_SCALING ? 1.0 : e;
      e = e > MAX_SCALING ? MAX_SCALING : e;
      w->E_temp[i] = 1. / sqrt(e);
    }
    mat_premult_diag(w->P, w->D_temp);
    mat_postmult_diag(w->P, w->D_temp);
    mat_premult_diag(w->A, w->E_temp);
    mat_postmult_diag(w->A, w->D_temp);
    for (int i = 0; i < n; i++) w->q[i] *= w->D_temp[i];
    for (int i = 0; i < n; i++) w->D[i] *= w->D_temp[i];
    for (int i = 0; i < m; i++) w->E[i] *= w->E_temp[i];
    /* cost normalization */
    mat_inf_norm_cols_sym_triu(w->P, w->D_temp);
    double c_temp = vec_mean(w->D_temp, n);
    double inf_norm_q = vec_norm_inf(w->q, n);
    inf_norm_q = inf_norm_q < MIN_SCALING ? 1.0 : inf_norm_q;
    inf_norm_q = inf_norm_q > MAX_SCALING ? MAX_SCALING : inf_norm_q;
    c_temp = dmax(c_temp, inf_norm_q);
    c_temp = c_temp < MIN_SCALING ? 1.0 : c_temp;
    c_temp = c_temp > MAX_SCALING ? MAX_SCALING : c_temp;
    c_temp = 1. / c_temp;
    mat_mult_scalar(w->P, c_temp);
    for (int i = 0; i < n; i++) w->q[i] *= c_temp;
    w->c *= c_temp;
  }
  w->cinv = 1. / w->c;
  for (int i = 0; i < n; i++) w->Dinv[i] = 1. / w->D[i];
  for (int i = 0; i < m; i++) w->Einv[i] = 1. / w->E[i];
  for (int i = 0; i < m; i++) {
    w->l[i] *= w->E[i];
    w->u[i] *= w->E[i];
  }
}

/* scaling.c unscale_data */
static void unscale_data(oqp_work *w) {
  mat_mult_scalar(w->P, w->cinv);
  mat_premult_diag(w->P, w->Dinv);
  mat_postmult_diag(w->P, w->Dinv);
  for (int i = 0; i < w->n; i++) {
    w->q[i] *= w->cinv;
    w->q[i] *= w->Dinv[i];
  }
  mat_premult_diag(w->A, w->Einv);
  mat_postmult_diag(w->A, w->Dinv);
  for (int i = 0; i < w->m; i++) {
    w->l[i] *= w->Einv[i];
    w->u[i] *= w->Einv[i];
  }
}

/* auxil.c set_rho_vec */
static void set_rho_vec(oqp_work *w) {
  w->set.rho = dmin(dmax(w->set.rho, RHO_MIN), RHO_MAX);
  for (int i = 0; i < w->m; i++) {
    if (w->l[i] < -OQP_INFTY * MIN_SCALING && w->u[i] > OQP_INFTY * MIN_SCALING) {
      w->constr_type[i] = -1;
      w->rho_vec[i] = RHO_MIN;
    } else if (w->u[i] - w->l[i] < RHO_TOL) {
      w->constr_type[i] = 1;
      w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->set.rho;
    } else {
      w->constr_type[i] = 0;
      w->rho_vec[i] = w->set.rho;
    }
    w->rho_inv_vec[i] = 1. / w->rho_vec[i];
  }
}

static int refactor(oqp_work *w) {
  if (w->hook_factor) return w->hook_factor(w->hook_ctx, w->P->x, w->A->x, w->set.sigma, w->rho_vec);
  return kkt_fill_factor(w->kkt, w->P, w->A, w->set.sigma, w->rho_inv_vec);
}

/* auxil.c update_rho_vec */
static int update_rho_vec(oqp_work *w) {
  int changed = 0;
  for (int i = 0; i < w->m; i++) {
    if (w->l[i] < -OQP_INFTY * MIN_SCALING && w->u[i] > OQP_INFTY * MIN_SCALING) {
      if (w->constr_type[i] != -1) {
        w->constr_type[i] = -1;
        w->rho_vec[i] = RHO_MIN;
        w->rho_inv_vec[i] = 1. / RHO_MIN;
        changed = 1;
      }
    } else if (w->u[i] - w->l[i] < RHO_TOL) {
      if (w->constr_type[i] != 1) {
        w->constr_type[i] = 1;
        w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->set.rho;
        w->rho_inv_vec[i] = 1. / w->rho_vec[i];
        changed = 1;
      }
    } else {
      if (w->constr_type[i] != 0) {
        w->constr_type[i] = 0;
        w->rho_vec[i] = w->set.rho;
        w->rho_inv_vec[i] = 1. / w->set.rho;
        changed = 1;
      }
    }
  }
  return changed ? refactor(w) : 0;
}

static void reset_info(oqp_work *w) {
  w->status = OQP_UNSOLVED;
  w->rho_updates = 0;
}

void oqp_default_settings(oqp_settings *s) {
  s->rho = 0.1;
  s->sigma = 1e-06;
  s->scaling = 10;
  s->adaptive_rho = 1;
  s->adaptive_rho_interval = 0;
  s->adaptive_rho_tolerance = 5;
  s->max_iter = 4000;
  s->eps_abs = 1e-3;
  s->eps_rel = 1e-3;
  s->eps_prim_inf = 1e-4;
  s->eps_dual_inf = 1e-4;
  s->alpha = 1.6;
  s->delta = 1e-6;
  s->polish = 0;
  s->polish_refine_iter = 3;
  s->scaled_termination = 0;
  s->check_termination = 25;
  s->warm_start = 1;
}

#define ALLOCD(k) (double *)calloc((size_t)((k) > 0 ? (k) : 1), sizeof(double))

oqp_work *oqp_setup(int n, int m, const int *Pp, const int *Pi, const double *Px, const double *q,
                    const int *Ap, const int *Ai, const double *Ax, const double *l,
                    const double *u, const oqp_settings *s, int *err) {
  *err = 0;
  for (int i = 0; i < m; i++)
    if (dmax(l[i], -OQP_INFTY) > dmin(u[i], OQP_INFTY)) {
      *err = 1;
      return NULL;
    }
  oqp_work *w = (oqp_work *)calloc(1, sizeof(oqp_work));
  w->n = n;
  w->m = m;
  w->set = *s;
  w->P = csc_copy(n, n, Pp, Pi, Px);
  w->A = csc_copy(m, n, Ap, Ai, Ax);
  w->q = ALLOCD(n);
  w->l = ALLOCD(m);
  w->u = ALLOCD(m);
  memcpy(w->q, q, sizeof(double) * (size_t)n);
  for (int i = 0; i < m; i++) {
    w->l[i] = dmax(l[i], -OQP_INFTY);
    w->u[i] = dmin(u[i], OQP_INFTY);
  }
  w->D = ALLOCD(n), w->Dinv = ALLOCD(n), w->E = ALLOCD(m), w->Einv = ALLOCD(m);
  w->D_temp = ALLOCD(n), w->D_temp_A = ALLOCD(n), w->E_temp = ALLOCD(m);
  w->x = ALLOCD(n), w->y = ALLOCD(m), w->z = ALLOCD(m), w->xz_tilde = ALLOCD(n + m);
  w->x_prev = ALLOCD(n), w->z_prev = ALLOCD(m);
  w->Ax = ALLOCD(m), w->Px = ALLOCD(n), w->Aty = ALLOCD(n);
  w->delta_y = ALLOCD(m), w->Atdelta_y = ALLOCD(n), w->delta_x = ALLOCD(n);
  w->Pdelta_x = ALLOCD(n), w->Adelta_x = ALLOCD(m);
  w->rho_vec = ALLOCD(m), w->rho_inv_vec = ALLOCD(m);
  w->constr_type = (int *)calloc((size_t)(m > 0 ? m : 1), sizeof(int));
  w->sol_x = ALLOCD(n), w->sol_y = ALLOCD(m);
  if (w->set.scaling) {
    scale_data(w);
  } else {
    w->c = w->cinv = 1.;
    for (int i = 0; i < n; i++) w->D[i] = w->Dinv[i] = 1.;
    for (int i = 0; i < m; i++) w->E[i] = w->Einv[i] = 1.;
  }
  set_rho_vec(w);
  w->kkt = kkt_init(w->P, w->A);
  if (refactor(w)) {
    *err = 2;
    oqp_cleanup(w);
    return NULL;
  }
  if (w->set.adaptive_rho && !w->set.adaptive_rho_interval)
    w->set.adaptive_rho_interval = w->set.check_termination
                                       ? ADAPTIVE_RHO_MULTIPLE_TERMINATION * w->set.check_termination
                                       : ADAPTIVE_RHO_FIXED;
  reset_info(w);
  w->iter = 0;
  return w;
}

void oqp_cleanup(oqp_work *w) {
  if (!w) return;
  csc_free(w->P), csc_free(w->A);
  free(w->q), free(w->l), free(w->u);
  free(w->D), free(w->Dinv), free(w->E), free(w->Einv), free(w->D_temp), free(w->D_temp_A);
  free(w->E_temp), free(w->x), free(w->y), free(w->z), free(w->xz_tilde), free(w->x_prev);
  free(w->z_prev), free(w->Ax), free(w->Px), free(w->Aty), free(w->delta_y), free(w->Atdelta_y);
  free(w->delta_x), free(w->Pdelta_x), free(w->Adelta_x), free(w->rho_vec), free(w->rho_inv_vec);
  free(w->constr_type), free(w->sol_x), free(w->sol_y), free(w->hook_sol);
  kkt_free(w->kkt);
  free(w);
}

int oqp_update_lin_cost(oqp_work *w, const double *q) {
  for (int i = 0; i < w->n; i++) {
    w->q[i] = q[i];
    if (w->set.scaling) w->q[i] = (w->q[i] * w->D[i]) * w->c;
  }
  reset_info(w);
  return 0;
}

/* osqp.c osqp_update_bounds */
int oqp_update_bounds(oqp_work *w, const double *l, const double *u) {
  for (int i = 0; i < w->m; i++)
    if (dmax(l[i], -OQP_INFTY) > dmin(u[i], OQP_INFTY)) return 1;
  for (int i = 0; i < w->m; i++) {
    w->l[i] = dmax(l[i], -OQP_INFTY);
    w->u[i] = dmin(u[i], OQP_INFTY);
    if (w->set.scaling) {
      w->l[i] *= w->E[i];
      w->u[i] *= w->E[i];
    }
  }
  reset_info(w);
  return update_rho_vec(w);
}

/* osqp.c osqp_update_A: unscale, overwrite, rescale, refactor (warm-start iterates are kept in
 * their old scaled coordinates, as OSQP 0.6 does) */
int oqp_update_A(oqp_work *w, const double *Ax) {
  if (w->set.scaling) unscale_data(w);
  memcpy(w->A->x, Ax, sizeof(double) * (size_t)csc_nnz(w->A));
  if (w->set.scaling) scale_data(w);
  int e = refactor(w);
  reset_info(w);
  return e;
}

/* osqp.c osqp_update_rho */
int oqp_update_rho(oqp_work *w, double rho_new) {
  if (rho_new <= 0) return 1;
  w->set.rho = dmin(dmax(rho_new, RHO_MIN), RHO_MAX);
  for (int i = 0; i < w->m; i++) {
    if (w->constr_type[i] == 0) {
      w->rho_vec[i] = w->set.rho;
      w->rho_inv_vec[i] = 1. / w->set.rho;
    } else if (w->constr_type[i] == 1) {
      w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->set.rho;
      w->rho_inv_vec[i] = 1. / w->rho_vec[i];
    }
  }
  return refactor(w);
}

/* osqp.c osqp_warm_start: scale the user vectors into the solver's coordinates */
int oqp_warm_start(oqp_work *w, const double *x, const double *y) {
  w->set.warm_start = 1;
  for (int i = 0; i < w->n; i++) w->x[i] = w->set.scaling ? w->Dinv[i] * x[i] : x[i];
  for (int i = 0; i < w->m; i++) w->y[i] = w->set.scaling ? (w->Einv[i] * y[i]) * w->c : y[i];
  mat_vec(w->A, w->x, w->z, 0);
  return 0;
}

/* ---------------------------------------------------------------- ADMM pieces (auxil.c) */
static void update_xz_tilde(oqp_work *w) {
  int n = w->n, m = w->m;
  kkt_sys *s = w->kkt;
  if (w->fused) { /* the engine's right-hand side: one rounding per entry (engine.hip) */
    for (int i = 0; i < n; i++) w->xz_tilde[i] = fma(w->set.sigma, w->x_prev[i], -w->q[i]);
    for (int i = 0; i < m; i++) w->xz_tilde[n + i] = fma(-w->rho_inv_vec[i], w->y[i], w->z_prev[i]);
  } else {
    for (int i = 0; i < n; i++) w->xz_tilde[i] = w->set.sigma * w->x_prev[i] - w->q[i];
    for (int i = 0; i < m; i++) w->xz_tilde[n + i] = w->z_prev[i] - w->rho_inv_vec[i] * w->y[i];
  }
  if (w->hook_solve) { /* the external solver works in the original order: [x~; nu] */
    w->hook_solve(w->hook_ctx, w->xz_tilde, w->hook_sol);
    for (int i = 0; i < n; i++) w->xz_tilde[i] = w->hook_sol[i];
    for (int i = 0; i < m; i++)
      w->xz_tilde[n + i] = w->fused ? fma(w->rho_inv_vec[i], w->hook_sol[n + i], w->xz_tilde[n + i])
                                    : w->xz_tilde[n + i] + w->rho_inv_vec[i] * w->hook_sol[n + i];
    return;
  }
  /* qdldl_interface solve (non-polish): permute, solve, copy x~, z~ = b_z + rho^-1 nu */
  for (int k = 0; k < s->nk; k++) s->bp[k] = w->xz_tilde[s->perm[k]];
  if (w->jitter) {
    /* parity-floor diagnostics (oqp_set_jitter): every right-hand side entry moved by one ulp up
     * or down -- a backward error of one ulp per KKT solve, the size of the difference between
     * two valid summation orders of the triangular solves */
    for (int k = 0; k < s->nk; k++) {
      unsigned long long x = w->jitter;
      x ^= x << 13, x ^= x >> 7, x ^= x << 17;
      w->jitter = x;
      s->bp[k] = nextafter(s->bp[k], (x >> 63) ? INFINITY : -INFINITY);
    }
  }
  if (s->solve_order)
    qdldl_solve_sum(s->nk, s->Lp, s->Li, s->Lx, s->Dinv, s->bp, s->fwork, s->solve_order);
  else
    qdldl_solve(s->nk, s->Lp, s->Li, s->Lx, s->Dinv, s->bp);
  for (int i = 0; i < n; i++) w->xz_tilde[i] = s->bp[s->pinv[i]];
  for (int i = 0; i < m; i++) w->xz_tilde[n + i] += w->rho_inv_vec[i] * s->bp[s->pinv[n + i]];
}

static void update_x(oqp_work *w) {
  double a = w->set.alpha;
  for (int i = 0; i < w->n; i++) {
    w->x[i] = w->fused ? fma(a, w->xz_tilde[i], (1.0 - a) * w->x_prev[i])
                       : a * w->xz_tilde[i] + (1.0 - a) * w->x_prev[i];
    w->delta_x[i] = w->x[i] - w->x_prev[i];
  }
}

static void update_z(oqp_work *w) {
  double a = w->set.alpha;
  int n = w->n;
  for (int i = 0; i < w->m; i++) {
    double v = w->fused ? fma(w->rho_inv_vec[i], w->y[i], fma(a, w->xz_tilde[n + i], (1.0 - a) * w->z_prev[i]))
                        : a * w->xz_tilde[n + i] + (1.0 - a) * w->z_prev[i] + w->rho_inv_vec[i] * w->y[i];
    w->z[i] = dmin(dmax(v, w->l[i]), w->u[i]);
  }
}

static void update_y(oqp_work *w) {
  double a = w->set.alpha;
  int n = w->n;
  for (int i = 0; i < w->m; i++) {
    const double zr = w->fused ? fma(a, w->xz_tilde[n + i], (1.0 - a) * w->z_prev[i])
                               : a * w->xz_tilde[n + i] + (1.0 - a) * w->z_prev[i];
    w->delta_y[i] = w->rho_vec[i] * (zr - w->z[i]);
    w->y[i] += w->delta_y[i];
  }
}

static double compute_obj_val(oqp_work *w, const double *x) {
  double o = quad_form(w->P, x) + vec_prod(w->q, x, w->n);
  return w->set.scaling ? o * w->cinv : o;
}

/* z_prev <- Ax - z (used as temporary, as OSQP does) */
static double compute_pri_res(oqp_work *w, const double *x, const double *z) {
  mat_vec(w->A, x, w->Ax, 0);
  for (int i = 0; i < w->m; i++) w->z_prev[i] = w->Ax[i] - z[i];
  if (w->set.scaling && !w->set.scaled_termination)
    return vec_scaled_norm_inf(w->Einv, w->z_prev, w->m);
  return vec_norm_inf(w->z_prev, w->m);
}

/* x_prev <- Px + q + A'y (temporary, as OSQP does) */
static double compute_dua_res(oqp_work *w, const double *x, const double *y) {
  int n = w->n;
  memcpy(w->x_prev, w->q, sizeof(double) * (size_t)n);
  sym_mat_vec(w->P, x, w->Px);
  for (int i = 0; i < n; i++) w->x_prev[i] += w->Px[i];
  if (w->m > 0) {
    mat_tpose_vec(w->A, y, w->Aty, 0, 0);
    for (int i = 0; i < n; i++) w->x_prev[i] += w->Aty[i];
  }
  if (w->set.scaling && !w->set.scaled_termination)
    return w->cinv * vec_scaled_norm_inf(w->Dinv, w->x_prev, n);
  return vec_norm_inf(w->x_prev, n);
}

static double compute_pri_tol(oqp_work *w, double eps_abs, double eps_rel) {
  double r;
  if (w->set.scaling && !w->set.scaled_termination) {
    r = vec_scaled_norm_inf(w->Einv, w->z, w->m);
    r = dmax(r, vec_scaled_norm_inf(w->Einv, w->Ax, w->m));
  } else {
    r = dmax(vec_norm_inf(w->z, w->m), vec_norm_inf(w->Ax, w->m));
  }
  return eps_abs + eps_rel * r;
}

static double compute_dua_tol(oqp_work *w, double eps_abs, double eps_rel) {
  double r;
  if (w->set.scaling && !w->set.scaled_termination) {
    r = vec_scaled_norm_inf(w->Dinv, w->q, w->n);
    r = dmax(r, vec_scaled_norm_inf(w->Dinv, w->Aty, w->n));
    r = dmax(r, vec_scaled_norm_inf(w->Dinv, w->Px, w->n));
    r *= w->cinv;
  } else {
    r = dmax(vec_norm_inf(w->q, w->n), vec_norm_inf(w->Aty, w->n));
    r = dmax(r, vec_norm_inf(w->Px, w->n));
  }
  return eps_abs + eps_rel * r;
}

static int is_primal_infeasible(oqp_work *w, double eps) {
  int m = w->m;
  double norm_dy, lhs = 0.0;
  for (int i = 0; i < m; i++) {
    if (w->u[i] > OQP_INFTY * MIN_SCALING) {
      if (w->l[i] < -OQP_INFTY * MIN_SCALING)
        w->delta_y[i] = 0.0;
      else
        w->delta_y[i] = dmin(w->delta_y[i], 0.0);
    } else if (w->l[i] < -OQP_INFTY * MIN_SCALING) {
      w->delta_y[i] = dmax(w->delta_y[i], 0.0);
    }
  }
  if (w->set.scaling && !w->set.scaled_termination) {
    for (int i = 0; i < m; i++) w->Adelta_x[i] = w->E[i] * w->delta_y[i];
    norm_dy = vec_norm_inf(w->Adelta_x, m);
  } else {
    norm_dy = vec_norm_inf(w->delta_y, m);
  }
  if (norm_dy > DIVISION_TOL) {
    for (int i = 0; i < m; i++)
      lhs += w->u[i] * dmax(w->delta_y[i], 0) + w->l[i] * dmin(w->delta_y[i], 0);
    if (lhs < eps * norm_dy) {
      mat_tpose_vec(w->A, w->delta_y, w->Atdelta_y, 0, 0);
      if (w->set.scaling && !w->set.scaled_termination)
        for (int i = 0; i < w->n; i++) w->Atdelta_y[i] *= w->Dinv[i];
      return vec_norm_inf(w->Atdelta_y, w->n) < eps * norm_dy;
    }
  }
  return 0;
}

static int is_dual_infeasible(oqp_work *w, double eps) {
  int n = w->n, m = w->m;
  double norm_dx, cost_scaling;
  if (w->set.scaling && !w->set.scaled_termination) {
    norm_dx = vec_scaled_norm_inf(w->D, w->delta_x, n);
    cost_scaling = w->c;
  } else {
    norm_dx = vec_norm_inf(w->delta_x, n);
    cost_scaling = 1.0;
  }
  if (norm_dx > DIVISION_TOL) {
    if (vec_prod(w->q, w->delta_x, n) < cost_scaling * eps * norm_dx) {
      sym_mat_vec(w->P, w->delta_x, w->Pdelta_x);
      if (w->set.scaling && !w->set.scaled_termination)
        for (int i = 0; i < n; i++) w->Pdelta_x[i] *= w->Dinv[i];
      if (vec_norm_inf(w->Pdelta_x, n) < cost_scaling * eps * norm_dx) {
        mat_vec(w->A, w->delta_x, w->Adelta_x, 0);
        if (w->set.scaling && !w->set.scaled_termination)
          for (int i = 0; i < m; i++) w->Adelta_x[i] *= w->Einv[i];
        for (int i = 0; i < m; i++)
          if ((w->u[i] < OQP_INFTY * MIN_SCALING && w->Adelta_x[i] > eps * norm_dx) ||
              (w->l[i] > -OQP_INFTY * MIN_SCALING && w->Adelta_x[i] < -eps * norm_dx))
            return 0;
        return 1;
      }
    }
  }
  return 0;
}

static int check_termination(oqp_work *w, int approximate) {
  double eps_abs = w->set.eps_abs, eps_rel = w->set.eps_rel;
  double eps_pinf = w->set.eps_prim_inf, eps_dinf = w->set.eps_dual_inf;
  int prim_ok = 0, dual_ok = 0, prim_inf = 0, dual_inf = 0;
  if (approximate) {
    eps_abs *= 10, eps_rel *= 10, eps_pinf *= 10, eps_dinf *= 10;
  }
  if (w->m == 0) {
    prim_ok = 1;
  } else {
    if (w->pri_res < compute_pri_tol(w, eps_abs, eps_rel))
      prim_ok = 1;
    else
      prim_inf = is_primal_infeasible(w, eps_pinf);
  }
  if (w->dua_res < compute_dua_tol(w, eps_abs, eps_rel))
    dual_ok = 1;
  else
    dual_inf = is_dual_infeasible(w, eps_dinf);
  if (prim_ok && dual_ok) {
    w->status = approximate ? OQP_SOLVED_INACCURATE : OQP_SOLVED;
    return 1;
  } else if (prim_inf) {
    w->status = approximate ? OQP_PRIMAL_INFEASIBLE_INACCURATE : OQP_PRIMAL_INFEASIBLE;
    if (w->set.scaling && !w->set.scaled_termination)
      for (int i = 0; i < w->m; i++) w->delta_y[i] *= w->E[i];
    w->obj_val = OQP_INFTY;
    return 1;
  } else if (dual_inf) {
    w->status = approximate ? OQP_DUAL_INFEASIBLE_INACCURATE : OQP_DUAL_INFEASIBLE;
    if (w->set.scaling && !w->set.scaled_termination)
      for (int i = 0; i < w->n; i++) w->delta_x[i] *= w->D[i];
    w->obj_val = -OQP_INFTY;
    return 1;
  }
  return 0;
}

static void update_info(oqp_work *w, int iter) {
  w->iter = iter;
  w->pri_res = w->m == 0 ? 0.0 : compute_pri_res(w, w->x, w->z);
  w->dua_res = compute_dua_res(w, w->x, w->y);
}

/* auxil.c compute_rho_estimate (z_prev / x_prev hold the residual vectors) */
static double compute_rho_estimate(oqp_work *w) {
  int n = w->n, m = w->m;
  double pri = vec_norm_inf(w->z_prev, m), dua = vec_norm_inf(w->x_prev, n);
  double pn = dmax(vec_norm_inf(w->z, m), vec_norm_inf(w->Ax, m));
  pri /= (pn + DIVISION_TOL);
  double dn = dmax(vec_norm_inf(w->q, n), vec_norm_inf(w->Aty, n));
  dn = dmax(dn, vec_norm_inf(w->Px, n));
  dua /= (dn + DIVISION_TOL);
  double est = w->set.rho * sqrt(pri / (dua + DIVISION_TOL));
  return dmin(dmax(est, RHO_MIN), RHO_MAX);
}

static int adapt_rho(oqp_work *w) {
  double rho_new = compute_rho_estimate(w);
  if (rho_new > w->set.rho * w->set.adaptive_rho_tolerance ||
      rho_new < w->set.rho / w->set.adaptive_rho_tolerance) {
    w->rho_updates++;
    return oqp_update_rho(w, rho_new);
  }
  return 0;
}

static int has_solution(int st) {
  return st != OQP_PRIMAL_INFEASIBLE && st != OQP_PRIMAL_INFEASIBLE_INACCURATE &&
         st != OQP_DUAL_INFEASIBLE && st != OQP_DUAL_INFEASIBLE_INACCURATE && st != OQP_NON_CVX;
}

/* ---------------------------------------------------------------- polish (polish.c) */
static void polish(oqp_work *w) {
  int n = w->n, m = w->m;
  int *A_to_Alow = (int *)malloc(sizeof(int) * (size_t)m), *A_to_Aupp = (int *)malloc(sizeof(int) * (size_t)m);
  int *Alow_to_A = (int *)malloc(sizeof(int) * (size_t)m), *Aupp_to_A = (int *)malloc(sizeof(int) * (size_t)m);
  int n_low = 0, n_upp = 0;
  for (int j = 0; j < m; j++) {
    if (w->z[j] - w->l[j] < -w->y[j]) {
      Alow_to_A[n_low] = j;
      A_to_Alow[j] = n_low++;
    } else
      A_to_Alow[j] = -1;
  }
  for (int j = 0; j < m; j++) {
    if (w->u[j] - w->z[j] < w->y[j]) {
      Aupp_to_A[n_upp] = j;
      A_to_Aupp[j] = n_upp++;
    } else
      A_to_Aupp[j] = -1;
  }
  int mred = n_low + n_upp;
  int nnzA = csc_nnz(w->A), rn = 0;
  for (int p = 0; p < nnzA; p++)
    if (A_to_Alow[w->A->i[p]] != -1 || A_to_Aupp[w->A->i[p]] != -1) rn++;
  csc *Ared = csc_alloc(mred, n, rn);
  rn = 0;
  for (int j = 0; j < n; j++) {
    Ared->p[j] = rn;
    for (int p = w->A->p[j]; p < w->A->p[j + 1]; p++) {
      int r = w->A->i[p];
      if (A_to_Alow[r] != -1) {
        Ared->i[rn] = A_to_Alow[r];
        Ared->x[rn++] = w->A->x[p];
      } else if (A_to_Aupp[r] != -1) {
        Ared->i[rn] = A_to_Aupp[r] + n_low;
        Ared->x[rn++] = w->A->x[p];
      }
    }
  }
  Ared->p[n] = rn;
  kkt_sys *ks = kkt_init(w->P, Ared);
  double *param2 = ALLOCD(mred);
  for (int i = 0; i < mred; i++) param2[i] = w->set.delta;
  int fail = kkt_fill_factor(ks, w->P, Ared, w->set.delta, param2);
  free(param2);
  if (fail) {
    w->status_polish = -1;
  } else {
    int nr = n + mred;
    double *rhs = ALLOCD(nr), *sol = ALLOCD(nr), *tmp = ALLOCD(nr);
    for (int j = 0; j < n; j++) rhs[j] = -w->q[j];
    for (int j = 0; j < n_low; j++) rhs[n + j] = w->l[Alow_to_A[j]];
    for (int j = 0; j < n_upp; j++) rhs[n + n_low + j] = w->u[Aupp_to_A[j]];
    memcpy(sol, rhs, sizeof(double) * (size_t)nr);
    kkt_solve(ks, sol);
    for (int it = 0; it < w->set.polish_refine_iter; it++) {
      memcpy(tmp, rhs, sizeof(double) * (size_t)nr);
      mat_vec(w->P, sol, tmp, -1);
      mat_tpose_vec(w->P, sol, tmp, -1, 1);
      mat_tpose_vec(Ared, sol + n, tmp, -1, 0);
      mat_vec(Ared, sol, tmp + n, -1);
      kkt_solve(ks, tmp);
      for (int j = 0; j < nr; j++) sol[j] += tmp[j];
    }
    double *px = ALLOCD(n), *pz = ALLOCD(m), *py = ALLOCD(m);
    memcpy(px, sol, sizeof(double) * (size_t)n);
    mat_vec(w->A, px, pz, 0);
    for (int j = 0; j < m; j++) {
      if (A_to_Alow[j] != -1)
        py[j] = sol[n + A_to_Alow[j]];
      else if (A_to_Aupp[j] != -1)
        py[j] = sol[n + n_low + A_to_Aupp[j]];
      else
        py[j] = 0.0;
    }
    /* project_normalcone */
    for (int j = 0; j < m; j++) {
      double t = pz[j] + py[j];
      pz[j] = dmin(dmax(t, w->l[j]), w->u[j]);
      py[j] = t - pz[j];
    }
    double pol_obj = compute_obj_val(w, px);
    double pol_pri = compute_pri_res(w, px, pz);
    double pol_dua = compute_dua_res(w, px, py);
    int ok = (pol_pri < w->pri_res && pol_dua < w->dua_res) ||
             (pol_pri < w->pri_res && w->dua_res < 1e-10) ||
             (pol_dua < w->dua_res && w->pri_res < 1e-10);
    if (ok) {
      w->obj_val = pol_obj;
      w->pri_res = pol_pri;
      w->dua_res = pol_dua;
      w->status_polish = 1;
      memcpy(w->x, px, sizeof(double) * (size_t)n);
      memcpy(w->z, pz, sizeof(double) * (size_t)m);
      memcpy(w->y, py, sizeof(double) * (size_t)m);
    } else {
      w->status_polish = -1;
    }
    free(px), free(pz), free(py), free(rhs), free(sol), free(tmp);
  }
  kkt_free(ks);
  csc_free(Ared);
  free(A_to_Alow), free(A_to_Aupp), free(Alow_to_A), free(Aupp_to_A);
}

/* ---------------------------------------------------------------- solve (osqp.c osqp_solve) */
int oqp_solve(oqp_work *w) {
  int n = w->n, m = w->m, iter, can_check = 0;
  w->status_polish = 0;
  if (!w->set.warm_start) {
    memset(w->x, 0, sizeof(double) * (size_t)n);
    memset(w->z, 0, sizeof(double) * (size_t)m);
    memset(w->y, 0, sizeof(double) * (size_t)m);
  }
  for (iter = 1; iter <= w->set.max_iter; iter++) {
    double *t = w->x;
    w->x = w->x_prev;
    w->x_prev = t;
    t = w->z;
    w->z = w->z_prev;
    w->z_prev = t;
    update_xz_tilde(w);
    update_x(w);
    update_z(w);
    update_y(w);
    can_check = w->set.check_termination && (iter % w->set.check_termination == 0);
    if (can_check) {
      update_info(w, iter);
      if (check_termination(w, 0)) break;
    }
    if (w->set.adaptive_rho && w->set.adaptive_rho_interval &&
        iter % w->set.adaptive_rho_interval == 0) {
      if (!can_check) update_info(w, iter);
      if (adapt_rho(w)) {
        w->status = OQP_NON_CVX;
        break;
      }
    }
  }
  if (!can_check) {
    update_info(w, iter - 1);
    check_termination(w, 0);
  }
  if (has_solution(w->status) && w->status != OQP_UNSOLVED) w->obj_val = compute_obj_val(w, w->x);
  if (w->status == OQP_UNSOLVED) {
    if (!check_termination(w, 1)) w->status = OQP_MAX_ITER_REACHED;
    if (has_solution(w->status)) w->obj_val = compute_obj_val(w, w->x);
  }
  if (w->set.polish && w->status == OQP_SOLVED) polish(w);
  /* store_solution */
  if (has_solution(w->status)) {
    for (int i = 0; i < n; i++) w->sol_x[i] = w->set.scaling ? w->D[i] * w->x[i] : w->x[i];
    for (int i = 0; i < m; i++)
      w->sol_y[i] = w->set.scaling ? w->E[i] * w->y[i] * w->cinv : w->y[i];
  } else {
    for (int i = 0; i < n; i++) w->sol_x[i] = NAN;
    for (int i = 0; i < m; i++) w->sol_y[i] = NAN;
    memset(w->x, 0, sizeof(double) * (size_t)n);
    memset(w->z, 0, sizeof(double) * (size_t)m);
    memset(w->y, 0, sizeof(double) * (size_t)m);
  }
  return 0;
}

void oqp_get_x(const oqp_work *w, double *x) { memcpy(x, w->sol_x, sizeof(double) * (size_t)w->n); }
void oqp_get_y(const oqp_work *w, double *y) { memcpy(y, w->sol_y, sizeof(double) * (size_t)w->m); }
/* parity-floor diagnostics: order 1 / 2 = the ADMM's KKT solves with every entry's products summed
 * apart (qdldl_solve_sum), 0 = QDLDL's order */
void oqp_set_solve_order(oqp_work *w, int order) { w->kkt->solve_order = order; }

int oqp_set_kkt_hook(oqp_work *w, oqp_kkt_factor_fn factor, oqp_kkt_solve_fn solve, void *ctx) {
  free(w->hook_sol);
  w->hook_sol = NULL;
  w->hook_factor = factor, w->hook_solve = solve, w->hook_ctx = ctx;
  if (!factor) return 0;
  w->hook_sol = (double *)calloc((size_t)(w->n + w->m), sizeof(double));
  return refactor(w); /* the current scaled data and rho */
}

void oqp_set_fused_updates(oqp_work *w, int on) { w->fused = on ? 1 : 0; }

/* parity-floor diagnostics: seed != 0 turns on the one-ulp right-hand-side jitter of every KKT
 * solve (update_xz_tilde), with a deterministic per-solver stream; 0 turns it off */
void oqp_set_jitter(oqp_work *w, unsigned long long seed) {
  w->jitter = seed ? seed * 0x9E3779B97F4A7C15ull | 1ull : 0ull;
}
int oqp_status(const oqp_work *w) { return w->status; }
int oqp_iter(const oqp_work *w) { return w->iter; }
int oqp_status_polish(const oqp_work *w) { return w->status_polish; }
int oqp_rho_updates(const oqp_work *w) { return w->rho_updates; }
double oqp_obj_val(const oqp_work *w) { return w->obj_val; }
double oqp_pri_res(const oqp_work *w) { return w->pri_res; }
double oqp_dua_res(const oqp_work *w) { return w->dua_res; }
double oqp_rho(const oqp_work *w) { return w->set.rho; }
int oqp_nnz_L(const oqp_work *w) { return w->kkt->Lp[w->kkt->nk]; }
void oqp_get_state(const oqp_work *w, double *x_s, double *z_s, double *y_s, double *D, double *E,
                   double *c) {
  if (x_s) memcpy(x_s, w->x, sizeof(double) * (size_t)w->n);
  if (z_s) memcpy(z_s, w->z, sizeof(double) * (size_t)w->m);
  if (y_s) memcpy(y_s, w->y, sizeof(double) * (size_t)w->m);
  if (D) memcpy(D, w->D, sizeof(double) * (size_t)w->n);
  if (E) memcpy(E, w->E, sizeof(double) * (size_t)w->m);
  if (c) *c = w->c;
}

/* the solver's current (scaled) data: P values (upper CSC, nnzP), q [n], l, u [m] -- white-box tests
 * of the engine's carried scaling (mpcqp_get_scaling) */
void oqp_get_data(const oqp_work *w, double *Px, double *q, double *l, double *u) {
  if (Px) memcpy(Px, w->P->x, sizeof(double) * (size_t)csc_nnz(w->P));
  if (q) memcpy(q, w->q, sizeof(double) * (size_t)w->n);
  if (l) memcpy(l, w->l, sizeof(double) * (size_t)w->m);
  if (u) memcpy(u, w->u, sizeof(double) * (size_t)w->m);
}

/* White-box hook (parity characterisation only): overwrite the scaled warm-start iterates and
 * rho with another solver's (e.g. the GPU engine's mpcqp_get_state), so that the next
 * update + solve of both starts from bitwise-identical state.  A changed rho re-factors exactly as
 * osqp_update_rho does. */
int oqp_set_state(oqp_work *w, const double *x_s, const double *z_s, const double *y_s, double rho) {
  if (x_s) memcpy(w->x, x_s, sizeof(double) * (size_t)w->n);
  if (z_s) memcpy(w->z, z_s, sizeof(double) * (size_t)w->m);
  if (y_s) memcpy(w->y, y_s, sizeof(double) * (size_t)w->m);
  if (rho > 0 && rho != w->set.rho) return oqp_update_rho(w, rho);
  return 0;
}

int oqp_batch_set_state(int B, oqp_work **works, const double *x_s, const double *z_s,
                        const double *y_s, const double *rho) {
  int rc = 0;
  for (int b = 0; b < B; b++) {
    oqp_work *w = works[b];
    if (oqp_set_state(w, x_s + (size_t)b * w->n, z_s + (size_t)b * w->m, y_s + (size_t)b * w->m,
                      rho[b]))
      rc = 1;
  }
  return rc;
}

/* ---------------------------------------------------------------- batch driver */
typedef struct {
  int b0, b1, n, m;
  const int *Pp, *Pi, *Ap, *Ai;
  const double *Px, *q, *Ax, *l, *u;
  const oqp_settings *s;
  double *x, *y;
  int *status, *iter;
  int rc;
} batch_job;

static void *batch_worker(void *arg) {
  batch_job *j = (batch_job *)arg;
  int nnzA = j->Ap[j->n];
  for (int b = j->b0; b < j->b1; b++) {
    int err = 0;
    oqp_work *w = oqp_setup(j->n, j->m, j->Pp, j->Pi, j->Px, j->q, j->Ap, j->Ai,
                            j->Ax + (size_t)b * nnzA, j->l + (size_t)b * j->m,
                            j->u + (size_t)b * j->m, j->s, &err);
    if (!w) {
      j->rc = err;
      if (j->status) j->status[b] = OQP_NON_CVX;
      continue;
    }
    oqp_solve(w);
    if (j->x) oqp_get_x(w, j->x + (size_t)b * j->n);
    if (j->y) oqp_get_y(w, j->y + (size_t)b * j->m);
    if (j->status) j->status[b] = w->status;
    if (j->iter) j->iter[b] = w->iter;
    oqp_cleanup(w);
  }
  return NULL;
}

int oqp_batch_solve(int B, int n, int m, const int *Pp, const int *Pi, const double *Px,
                    const double *q, const int *Ap, const int *Ai, const double *Ax_batch,
                    const double *l_batch, const double *u_batch, const oqp_settings *s,
                    int nthreads, double *x_out, double *y_out, int *status_out, int *iter_out) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > B) nthreads = B > 0 ? B : 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
  batch_job *jobs = (batch_job *)calloc((size_t)nthreads, sizeof(batch_job));
  for (int t = 0; t < nthreads; t++) {
    batch_job *j = &jobs[t];
    j->b0 = (int)((long long)B * t / nthreads);
    j->b1 = (int)((long long)B * (t + 1) / nthreads);
    j->n = n, j->m = m, j->Pp = Pp, j->Pi = Pi, j->Px = Px, j->q = q, j->Ap = Ap, j->Ai = Ai;
    j->Ax = Ax_batch, j->l = l_batch, j->u = u_batch, j->s = s;
    j->x = x_out, j->y = y_out, j->status = status_out, j->iter = iter_out;
    pthread_create(&th[t], NULL, batch_worker, j);
  }
  int rc = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc) rc = jobs[t].rc;
  }
  free(th);
  free(jobs);
  return rc;
}

/* ---------------------------------------------------------------- warm batch driver */
typedef struct {
  int b0, b1;
  oqp_work **works;
  const double *Ax, *l, *u;
  double *x;
  int *status, *iter;
} warm_job;

static void *warm_worker(void *arg) {
  warm_job *j = (warm_job *)arg;
  for (int b = j->b0; b < j->b1; b++) {
    oqp_work *w = j->works[b];
    int nnzA = csc_nnz(w->A);
    if (j->l && j->u) oqp_update_bounds(w, j->l + (size_t)b * w->m, j->u + (size_t)b * w->m);
    if (j->Ax) oqp_update_A(w, j->Ax + (size_t)b * nnzA);
    oqp_solve(w);
    if (j->x) oqp_get_x(w, j->x + (size_t)b * w->n);
    if (j->status) j->status[b] = w->status;
    if (j->iter) j->iter[b] = w->iter;
  }
  return NULL;
}

int oqp_batch_update_solve(int B, oqp_work **works, const double *Ax_batch, const double *l_batch,
                           const double *u_batch, int nthreads, double *x_out, int *status_out,
                           int *iter_out) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > B) nthreads = B > 0 ? B : 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
  warm_job *jobs = (warm_job *)calloc((size_t)nthreads, sizeof(warm_job));
  for (int t = 0; t < nthreads; t++) {
    warm_job *j = &jobs[t];
    j->b0 = (int)((long long)B * t / nthreads);
    j->b1 = (int)((long long)B * (t + 1) / nthreads);
    j->works = works, j->Ax = Ax_batch, j->l = l_batch, j->u = u_batch;
    j->x = x_out, j->status = status_out, j->iter = iter_out;
    pthread_create(&th[t], NULL, warm_worker, j);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}
