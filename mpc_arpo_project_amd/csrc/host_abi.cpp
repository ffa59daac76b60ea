// host_abi.cpp -- the host-only part of the C ABI (no HIP call): the calling thread's error
// message, default settings and status strings, and the planner entry points -- symbolic analysis
// (mpcqp_analyze) and the CPU interpretation of the compiled device program
// (mpcqp_schedule_check).  Linked into libmpcqp.so with the HIP sources; built on its own with
// g++ -fsanitize=address,undefined together with symbolic.cpp, lds_layout.cpp and emulate.cpp for
// the sanitizer check of the host code (tests/test_sanitize.py).
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>

#include "host_abi.hpp"

namespace mpcqp {

namespace {
thread_local std::string g_err;
// block caps of the blocked substitution forced by MPCQP_CAPM / MPCQP_CAPW (diagnostics; 0: chosen
// per structure by build_plan_tuned)
int cap_m() { return diag_env_int("MPCQP_CAPM", 0); }
int cap_w() { return diag_env_int("MPCQP_CAPW", 0); }
// matrix operands of the solve steps read one step ahead (MPCQP_MATPF: 0 or 1; Plan::mat_first)
bool matrix_prefetch() { return diag_env_int("MPCQP_MATPF", 0) == 1; }
}  // namespace

int set_error(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// waves per instance of the solve kernel (MPCQP_WAVES: 1; 2 = two waves, solve steps split
// between them; 3 = two waves, solve steps on the first; unset or 0: chosen per structure by
// auto_waves; DESIGN.md, Two waves per instance)
int waves_per_instance() {
  const int w = diag_env_int("MPCQP_WAVES", 0);
  return (w == 1 || w == 2 || w == 3) ? w : 0;
}

// The automatic choice: two waves per instance with the solve steps on the first (3) when the
// one-wave image leaves at most two instances per CU -- then two of the CU's four SIMDs would idle,
// and the second wave takes half of the vector passes, checks and Ruiz passes onto them (N = 40:
// +8 % solves/s, profiles/r04/pair2); one wave otherwise (N = 20: four instances per CU, where the
// second wave's barriers cost more than its share saves: -4 %)
int auto_waves(const mpcqp_structure* st) {
  Plan p1;
  if (!build_plan_tuned(st->n, st->m, st->Pp, st->Pi, st->Ap, st->Ai, p1, cap_m(), cap_w(), 163840,
                        4, 1, false))
    return 1;
  const int bytes = ((p1.LDS_N + 1) & ~1) * 8;
  return 163840 / std::max(bytes, 1) <= 2 ? 3 : 1;
}

bool plan_for(const mpcqp_structure* st, Plan& pl) {
  const int w = waves_per_instance();
  return build_plan_tuned(st->n, st->m, st->Pp, st->Pi, st->Ap, st->Ai, pl, cap_m(), cap_w(), 163840,
                          4, w ? w : auto_waves(st), matrix_prefetch());
}

}  // namespace mpcqp

using namespace mpcqp;

extern "C" {

int mpcqp_version(void) { return 100; }
const char* mpcqp_last_error(void) { return g_err.c_str(); }

const char* mpcqp_status_string(int32_t st) {
  switch (st) {
    case MPCQP_SOLVED: return "solved";
    case MPCQP_SOLVED_INACCURATE: return "solved inaccurate";
    case MPCQP_PRIMAL_INFEASIBLE_INACCURATE: return "primal infeasible inaccurate";
    case MPCQP_DUAL_INFEASIBLE_INACCURATE: return "dual infeasible inaccurate";
    case MPCQP_MAX_ITER_REACHED: return "maximum iterations reached";
    case MPCQP_PRIMAL_INFEASIBLE: return "primal infeasible";
    case MPCQP_DUAL_INFEASIBLE: return "dual infeasible";
    case -5: return "interrupted";
    case -6: return "run time limit reached";
    case MPCQP_NON_CVX: return "problem non convex";
    case MPCQP_UNSOLVED: return "unsolved";
    default: return "unknown";
  }
}

int mpcqp_default_settings(mpcqp_settings* s) {
  if (!s) return set_error(MPCQP_E_INVALID, "null settings");
  s->rho = 0.1;
  s->sigma = 1e-06;
  s->alpha = 1.6;
  s->eps_abs = 1e-3;
  s->eps_rel = 1e-3;
  s->eps_prim_inf = 1e-4;
  s->eps_dual_inf = 1e-4;
  s->delta = 1e-6;
  s->adaptive_rho_tolerance = 5;
  s->max_iter = 4000;
  s->scaling = 10;
  s->adaptive_rho = 1;
  s->adaptive_rho_interval = 0;
  s->polish = 0;
  s->polish_refine_iter = 3;
  s->check_termination = 25;
  s->warm_start = 1;
  s->scaled_termination = 0;
  return 0;
}

int mpcqp_analyze(const mpcqp_structure* st, int32_t* perm, int32_t* Lp, int32_t* Li,
                  int32_t* nnzL, int32_t* stats) {
  if (!st || !nnzL) return set_error(MPCQP_E_INVALID, "null argument");
  Plan pl;
  if (!plan_for(st, pl)) return set_error(MPCQP_E_UNSUPPORTED, pl.error);
  const int cap = *nnzL;
  *nnzL = pl.nnzL;
  if (perm) std::copy(pl.perm.begin(), pl.perm.end(), perm);
  if (Lp) std::copy(pl.Lp.begin(), pl.Lp.end(), Lp);
  if (Li && cap >= pl.nnzL) std::copy(pl.Li.begin(), pl.Li.end(), Li);
  if (stats) {
    stats[0] = (int32_t)(pl.nfac + pl.ntail);
    stats[1] = (int32_t)pl.nfwd;
    stats[2] = (int32_t)pl.nbwd;
    stats[3] = pl.levels_fwd;
    stats[4] = pl.levels_bwd;
    stats[5] = pl.LDS_N * (int)sizeof(double);
  }
  return 0;
}

int mpcqp_schedule_check(const mpcqp_structure* st, const double* Px, const double* Ax,
                         double sigma, const double* rho_vec, const double* rhs, double* sol,
                         int64_t* model) {
  if (!st || !Px || !Ax || !rho_vec || !rhs || !sol) return set_error(MPCQP_E_INVALID, "null argument");
  Plan pl;  // the plan mpcqp_create would build (MPCQP_WAVES included)
  if (!plan_for(st, pl)) return set_error(MPCQP_E_UNSUPPORTED, pl.error);
  if (model) {
    const LdsModel md = model_lds(pl);
    model[0] = md.read, model[1] = md.atomic, model[2] = md.vec, model[3] = md.floor;
  }
  if (!emulate_kkt_solve(pl, Px, Ax, sigma, rho_vec, rhs, sol))
    return set_error(MPCQP_E_INVALID, "schedule emulation produced a non-finite or unzeroed slot, or changed a 1/D slot");
  return 0;
}

// The compiled device program's factorization and solves on the CPU, factor and solve apart (a
// KKT solver for the oracle's hybrid parity runs: tests/sweep_parity.py, DESIGN.md Parity)
struct mpcqp_emu {
  std::shared_ptr<const Plan> pl;  // shared by clones (read-only)
  std::vector<double> v;
  bool factored = false;
};

int mpcqp_emu_create(const mpcqp_structure* st, mpcqp_emu** out) {
  if (!st || !out) return set_error(MPCQP_E_INVALID, "null argument");
  *out = nullptr;
  auto pl = std::make_shared<Plan>();
  if (!plan_for(st, *pl)) return set_error(MPCQP_E_UNSUPPORTED, pl->error);
  mpcqp_emu* e = new mpcqp_emu();
  e->pl = pl;
  *out = e;
  return 0;
}

int mpcqp_emu_clone(const mpcqp_emu* src, mpcqp_emu** out) {
  if (!src || !out) return set_error(MPCQP_E_INVALID, "null argument");
  mpcqp_emu* e = new mpcqp_emu();
  e->pl = src->pl;
  *out = e;
  return 0;
}

int mpcqp_emu_destroy(mpcqp_emu* e) {
  delete e;
  return 0;
}

int mpcqp_emu_factor(mpcqp_emu* e, const double* Px, const double* Ax, double sigma,
                     const double* rho_vec) {
  if (!e || !Px || !Ax || !rho_vec) return set_error(MPCQP_E_INVALID, "null argument");
  emulate_factor(*e->pl, Px, Ax, sigma, rho_vec, e->v);
  e->factored = true;
  return 0;
}

int mpcqp_emu_solve(mpcqp_emu* e, const double* rhs, double* sol) {
  if (!e || !rhs || !sol) return set_error(MPCQP_E_INVALID, "null argument");
  if (!e->factored) return set_error(MPCQP_E_NODATA, "solve before factor");
  // a non-finite solution is returned as computed (ADMM on an infeasible problem may diverge)
  (void)emulate_solve(*e->pl, e->v, rhs, sol);
  return 0;
}

}  // extern "C"

#ifdef MPCQP_HOST_ONLY_BUILD
// marker of the host-only (sanitizer) build: mpc_arpo_project_amd/_lib.py then binds only the
// host entry points above; never defined in libmpcqp.so
extern "C" int mpcqp_host_only_build(void) { return 1; }
#endif
