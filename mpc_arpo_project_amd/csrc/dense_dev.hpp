// dense_dev.hpp -- interface between the C ABI (engine.hip) and the dense-inverse engine
// (dense.hip).  The batch buffers (data, warm-start state, counter) are owned by the ABI handle.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/mpcqp.h"

namespace mpcqp {

struct DenseEngine;

struct DenseInputs {
  int n, m, batch;
  const int32_t *Pp, *Pi, *Ap, *Ai;
};

struct DenseSolveArgs {
  mpcqp_settings s;
  int B;
  const double *Px, *q, *Ax, *l, *u;
  double *xs, *zs, *ys, *rho_state, *Ecls;
  int32_t* has_state;
  double *x_out, *y_out;
  mpcqp_info info;
  unsigned int* counter;
  unsigned long long* timing;  // diagnostic builds only (MPCQP_TIMING)
};

// returns 0 or an MPCQP_E_* code (err set)
int dense_create(const DenseInputs& in, DenseEngine** out, std::string& err);
void dense_destroy(DenseEngine* e);
int dense_solve(DenseEngine* e, const DenseSolveArgs& a, hipStream_t stream);
void dense_info(const DenseEngine* e, int* grid, int* lds_bytes, int* per_cu);

}  // namespace mpcqp
