// closed_loop.hip -- device-side closed-loop step around the batched QP solve (see
// include/mpcqp_closed_loop.h).  One thread per chaser; this is scalar per-instance logic, a few
// hundred bytes of traffic per instance and step, far off the solve's critical path.
//
// Arithmetic that feeds comparisons with the reference (slopes, intercepts, norms, the plant) is
// evaluated in the reference's order with FP contraction off (see mul / add below), so the
// controller, plant and QP reconfiguration reproduce the reference's floating-point results.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "../../include/mpcqp_closed_loop.h"
#include "../../include/mpcqp_estimation.h"
#include "plant_dev.hpp"

namespace {

using mpcqp::PlantConsts;
using mpcqp::rk45_interval;

constexpr int NX = 4, NU = 2, NY = 5, NDI = 2;

// per-chaser run summary (mpcqp_cl_set_tracking), updated by cl_step_kernel
struct Track {
  int32_t *iterm, *success, *n_fallback;
  double* final_err;
  double dist_tol, ang_tol, rad2deg;
  int32_t step;  // loop index i of the step being launched: x_true holds x(i)
};
struct ClDev {
  mpcqp_cl_scenario sc;  // host pointers inside are not used on the device
  const int32_t *pos_c1, *pos_c2, *pos_slope;
  int B;
  Track tr;
};

// No FMA contraction in this file's own arithmetic (hipcc contracts a * b + c by default, and
// __dmul_rn / __dadd_rn are plain operators in ROCm's headers, so they fuse too): the scalar logic
// below restates numpy / scipy operation by operation, and a fused multiply-add rounds once where
// the reference rounds twice.  Fused operations appear only where numpy's own kernels fuse
// (norm2 / norm4, __fma_rn).
#pragma clang fp contract(off)
__device__ __forceinline__ double mul(double a, double b) { return a * b; }
__device__ __forceinline__ double add(double a, double b) { return a + b; }
__device__ __forceinline__ double sub(double a, double b) { return a - b; }

// numpy's evaluation orders on the reference's host (numpy 2.2 + OpenBLAS, measured bit for bit in
// tests/test_closed_loop_host.py): np.linalg.norm of a short vector is sqrt of the OpenBLAS ddot
// FMA chain; a 2x4 @ 4 product (dgemv) sums the four products as (a0 + a2) + (a1 + a3)
__device__ __forceinline__ double norm2(double x0, double x1) {
  return sqrt(__fma_rn(x1, x1, mul(x0, x0)));
}
__device__ __forceinline__ double norm4(const double* v) {
  return sqrt(__fma_rn(v[3], v[3], __fma_rn(v[2], v[2], __fma_rn(v[1], v[1], mul(v[0], v[0])))));
}
__device__ __forceinline__ double dot4(const double* k, const double* x) {
  return add(add(mul(k[0], x[0]), mul(k[2], x[2])), add(mul(k[1], x[1]), mul(k[3], x[3])));
}

// configureDynamicConstraints (reference src/simhelpers.py:66-138) for one chaser
__global__ void __launch_bounds__(256) cl_configure_kernel(ClDev d, double* xest, double* Ax,
                                                           double* l, double* u) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  const mpcqp_cl_scenario& s = d.sc;
  double* xe = xest + (size_t)b * 6;
  const double xc0 = xe[0], xc1 = xe[1];
  const double C1 = xe[2] >= 0 ? 1.0 : -1.0;
  const double C2 = xe[3] >= 0 ? 1.0 : -1.0;
  double cx = s.center[0], cy = s.center[1];
  double xs0 = xc0, xs1 = xc1;
  if (s.inTrack) {
    xs0 = xc1, xs1 = xc0;
    const double t = cx;
    cx = cy, cy = t;
  }
  (void)cy;
  const double h = s.side / 2;
  const bool inside = sub(xs0, add(cx, h)) < 0 && sub(xs0, sub(cx, h)) > 0;
  const bool nearb = sub(xs0, add(cx, h)) < s.detect && sub(xs0, add(cx, h)) > 0;
  const bool up = xs1 >= 0;
  double slope = 0.0, inter = 0.0;
  if (s.has_debris) {
    const int vi = up ? (inside ? 1 : 0) : (inside ? 2 : 3);
    const double vx = s.verts[2 * vi], vy = s.verts[2 * vi + 1];
    slope = sub(xc1, vy) / sub(xc0, vx);
    inter = add(mul(-slope, xc0), xc1);
  }
  const double l1 = add(fabs(sub(xc0, s.xr[0])), fabs(sub(xc1, s.xr[1])));
  const double inf = __builtin_inf();
  const bool act = inside || nearb;
  const double lo5 = (up && act) ? inter : -inf;
  const double hi5 = (!up && act) ? inter : inf;
  double* axb = Ax + (size_t)b * s.nnzA;
  for (int k = 0; k <= s.Nx; ++k) {
    axb[d.pos_c1[k]] = C1;
    axb[d.pos_c2[k]] = C2;
    if (d.pos_slope) axb[d.pos_slope[k]] = -slope;
  }
  double* lb = l + (size_t)b * s.m;
  double* ub = u + (size_t)b * s.m;
  for (int i = 0; i < NX; ++i) lb[i] = ub[i] = -xe[i];
  const int r0 = (s.Nx + 1) * NX;
  const double xmin[NY] = {1., 1., s.rp, 0., lo5};
  const double xmax[NY] = {inf, inf, inf, l1, hi5};
  for (int k = 0; k <= s.Nb; ++k)
    for (int j = 0; j < NY; ++j) {
      lb[r0 + k * NY + j] = xmin[j];
      ub[r0 + k * NY + j] = xmax[j];
    }
  const int r3 = r0 + (s.Nx + 1) * NY + s.Nc * (NU + NY);
  for (int j = 0; j < NDI; ++j) {
    const double dj = s.isReject ? xe[4 + j] : 0.0;
    lb[r3 + j] = ub[r3 + j] = dj;
  }
  if (s.inTrack) {  // quirk Q4: the caller's estimate is swapped in place
    xe[0] = xc1;
    xe[1] = xc0;
  }
}

// controller select + input-norm clip (reference src/trajectorySimulate.py:296-319,
// src/trajectorySimulateC.py:338-361): MPC if the solve succeeded, else deadbeat debris avoidance
// inside the debris box, else the LQR failsafe; returns the controller id (1 / 3 / 2)
__device__ __forceinline__ int select_control(const mpcqp_cl_scenario& s, int32_t st,
                                              const double* xsol, const double* xe, double& xi,
                                              double& c0, double& c1) {
  int seq;
  if (st != 1) {
    const double h = s.side / 2;
    const bool in_box = s.has_debris && sub(xe[0], add(s.center[0], h)) < 0 &&
                        sub(xe[0], sub(s.center[0], h)) > 0 && xe[1] < add(s.center[1], h) &&
                        xe[1] > sub(s.center[1], h);
    if (in_box) {  // deadbeat debris avoidance
      xi = sub(add(xi, dot4(s.Crefy, xe)), add(s.center[1], h));
      c0 = sub(-dot4(s.Ktot, xe), mul(s.Ki[0], xi));
      c1 = sub(-dot4(s.Ktot + 4, xe), mul(s.Ki[1], xi));
      seq = 3;
    } else {  // LQR failsafe (homing)
      xi = sub(add(xi, dot4(s.Crefx, xe)), s.xr[0]);
      c0 = sub(-dot4(s.Kpf, xe), mul(s.Kif[0], xi));
      c1 = sub(-dot4(s.Kpf + 4, xe), mul(s.Kif[1], xi));
      seq = 2;
    }
  } else {
    xi = 0.0;
    c0 = xsol[0];
    c1 = xsol[1];
    seq = 1;
  }
  // input-norm clip with the reference's sequential rescale (quirk Q2)
  const double um = s.umax[0];
  double nr = norm2(c0, c1);
  if (nr > um) {
    c0 = mul(c0, um / nr);
    nr = norm2(c0, c1);
    c1 = mul(c1, um / nr);
  }
  return seq;
}

// termination test at the top of a loop iteration (src/trajectorySimulate.py:288-293,
// src/trajectorySimulateC.py:328-333)
__device__ __forceinline__ bool terminated(const mpcqp_cl_scenario& s, const double* x) {
  const double rn = norm2(x[0], x[1]);
  const double pos = s.inTrack ? x[1] : x[0];
  return rn < s.rp || pos < sub(s.rp, s.rtol);
}

// range / bearing measurement hx (src/trajectorySimulate.py:330-332)
__device__ __forceinline__ void measure(const double* x, double* z) {
  z[0] = norm2(x[0], x[1]);
  z[1] = atan2(x[1], x[0]);
}

// reference src/trajectorySimulate.py:288-337 for one chaser: controller, plant
// x+ = Ad x + Bd u_prev + w (one-sample actuation delay, quirk Q1), perfect-state estimate,
// optional measurement z of x+ and the applied control (the UKF's predict input)
__global__ void __launch_bounds__(256) cl_step_kernel(ClDev d, const int32_t* status,
                                                      const double* x_sol, int n, int u0,
                                                      double* x_true, double* ctrl_prev,
                                                      double* xintf, double* xest, int32_t* done,
                                                      int32_t* ctrl_seq, double* ctrl_out,
                                                      const double* noise, double* z_out,
                                                      double* u_applied) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  const mpcqp_cl_scenario& s = d.sc;
  if (done[b]) {
    ctrl_seq[b] = 0;
    return;
  }
  const double* xe = xest + (size_t)b * 6;
  double c0, c1, xi = xintf[b];
  const int seq = select_control(s, status[b], x_sol + (size_t)b * n + u0, xe, xi, c0, c1);
  xintf[b] = xi;
  ctrl_seq[b] = seq;
  const Track& tr = d.tr;
  if (tr.iterm) {
    // the reference's run reduction (src/trajectorySimulate.py:369-376 success test over the
    // states 1 .. iterm-1 of the run; test/disturbRejComp.py:88 final error |x(iterm-1) - xr|)
    const double* x = x_true + (size_t)b * NX;
    const double dist = norm2(sub(x[0], s.xr[0]), sub(x[1], s.xr[1]));
    const double ang = mul(fabs(atan(x[3] / x[2])), tr.rad2deg);
    if (tr.step >= 1 && dist <= tr.dist_tol && ang <= tr.ang_tol) tr.success[b] = 1;
    double e[NX];
    for (int k = 0; k < NX; ++k) e[k] = sub(x[k], s.xr[k]);
    tr.final_err[b] = norm4(e);
    if (seq != 1) tr.n_fallback[b] += 1;
  }
  ctrl_out[(size_t)b * 2] = c0;
  ctrl_out[(size_t)b * 2 + 1] = c1;
  // plant in CSC column order (scipy sparse mat-vec), then + noise
  double* xt = x_true + (size_t)b * NX;
  double* up = ctrl_prev + (size_t)b * NU;
  double ax[NX] = {0, 0, 0, 0}, bu[NX] = {0, 0, 0, 0};
  for (int j = 0; j < NX; ++j)
    for (int i = 0; i < NX; ++i)
      if (s.Ad[i * NX + j] != 0.0) ax[i] = add(ax[i], mul(s.Ad[i * NX + j], xt[j]));
  for (int j = 0; j < NU; ++j)
    for (int i = 0; i < NX; ++i)
      if (s.Bd[i * NU + j] != 0.0) bu[i] = add(bu[i], mul(s.Bd[i * NU + j], up[j]));
  double xn[NX];
  for (int i = 0; i < NX; ++i)
    xn[i] = add(add(ax[i], bu[i]), noise ? noise[(size_t)b * NX + i] : 0.0);
  for (int i = 0; i < NX; ++i) xt[i] = xn[i];
  if (u_applied) {
    u_applied[(size_t)b * 2] = up[0];
    u_applied[(size_t)b * 2 + 1] = up[1];
  }
  up[0] = c0;
  up[1] = c1;
  double* xw = xest + (size_t)b * 6;
  for (int i = 0; i < NX; ++i) xw[i] = xn[i];
  xw[4] = 0.0;
  xw[5] = 0.0;
  if (z_out) measure(xn, z_out + (size_t)b * 2);
  if (terminated(s, xn)) {
    done[b] = 1;
    if (tr.iterm) tr.iterm[b] = tr.step + 1;
  }
}

// Philox-4x32-10 (Salmon et al., SC'11): counter (draw, id) under key (seed)
__device__ __forceinline__ void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// noiseVec = sigMat @ normal(0, 1, 4), sigMat = diag(sig_x, sig_y, 0, 0)
// (src/trajectorySimulate.py:268,352-353), from a counter-based stream keyed by the global chaser
// id, so that a chaser's noise does not depend on how the batch is sharded
__global__ void __launch_bounds__(256) cl_noise_kernel(int B, uint64_t seed, int64_t id0,
                                                       uint64_t draw, double sx, double sy,
                                                       double* noise) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t id = (uint64_t)(id0 + b);
  uint32_t c[4] = {(uint32_t)draw, (uint32_t)(draw >> 32), (uint32_t)id, (uint32_t)(id >> 32)};
  philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  double g[4];
  for (int k = 0; k < 2; ++k) {  // Box-Muller on (0, 1] uniforms
    const double u1 = ((double)c[2 * k] + 1.0) * 2.3283064365386963e-10;
    const double u2 = (double)c[2 * k + 1] * 2.3283064365386963e-10;
    const double r = sqrt(-2.0 * log(u1));
    g[2 * k] = r * cos(6.283185307179586 * u2);
    g[2 * k + 1] = r * sin(6.283185307179586 * u2);
  }
  double* o = noise + (size_t)b * NX;
  o[0] = sx * g[0];
  o[1] = sy * g[1];
  o[2] = 0.0;
  o[3] = 0.0;
}

// One sample period of the continuous-time closed loop (reference
// src/trajectorySimulateC.py:325-409) for one chaser: the loop iterations i_s .. i_s + nsub - 1
// that start at a sample instant i_s.  At i_s: controller select from the estimate of the previous
// sample; the plant sub-step i_s still runs with the previous control ctrls[:, i_s] (one-sub-step
// delay); the measurement is taken of x(i_s + 1).  Sub-steps i_s + 1 .. use the new control.
// Each sub-step: termination test of x(i) (-> done, iterm = i), then
// x(i+1) = solve_ivp(stateEqnN, (t, t + T_cont), x(i), args=(u,)).y[:, -1] (+ [0, 0, u_prev] at
// the sample for the delta-v model) + w;  t <- t + T_cont.
__global__ void __launch_bounds__(64) clc_period_kernel(
    ClDev d, PlantConsts pc, int isDeltaV, const int32_t* status, const double* x_sol, int n,
    int u0, double* x_true, double* ctrl_prev, double* xintf, double* xest, int32_t* done,
    int32_t* iterm, int32_t* ctrl_seq, double* ctrl_out, const double* noise, double* z_out,
    double* u_applied, double t_start, double dt, int i_start, int nsub, double* traj) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  const mpcqp_cl_scenario& s = d.sc;
  if (done[b]) {
    ctrl_seq[b] = 0;
    return;
  }
  const double* xe = xest + (size_t)b * 6;
  double c0, c1, xi = xintf[b];
  const int seq = select_control(s, status[b], x_sol + (size_t)b * n + u0, xe, xi, c0, c1);
  xintf[b] = xi;
  ctrl_seq[b] = seq;
  ctrl_out[(size_t)b * 2] = c0;
  ctrl_out[(size_t)b * 2 + 1] = c1;
  double* up = ctrl_prev + (size_t)b * NU;
  const double p0 = up[0], p1 = up[1];
  if (u_applied) {
    u_applied[(size_t)b * 2] = p0;
    u_applied[(size_t)b * 2 + 1] = p1;
  }
  double w[NX] = {0, 0, 0, 0};
  if (noise)
    for (int i = 0; i < NX; ++i) w[i] = noise[(size_t)b * NX + i];
  double x[NX];
  for (int i = 0; i < NX; ++i) x[i] = x_true[(size_t)b * NX + i];
  double t = t_start;
  int stop = -1;
  for (int k = 0; k < nsub; ++k) {
    if (k > 0 && terminated(s, x)) {
      stop = i_start + k;
      break;
    }
    const double t1 = add(t, dt);
    const double ua = isDeltaV ? 0.0 : (k == 0 ? p0 : c0);
    const double ub = isDeltaV ? 0.0 : (k == 0 ? p1 : c1);
    rk45_interval(pc, t, t1, x, ua, ub);
    if (isDeltaV && k == 0) {
      x[2] = add(x[2], p0);
      x[3] = add(x[3], p1);
    }
    for (int i = 0; i < NX; ++i) x[i] = add(x[i], w[i]);
    if (traj)
      for (int i = 0; i < NX; ++i) traj[((size_t)b * nsub + k) * NX + i] = x[i];
    if (k == 0) {
      double* xw = xest + (size_t)b * 6;
      for (int i = 0; i < NX; ++i) xw[i] = x[i];
      xw[4] = 0.0;
      xw[5] = 0.0;
      if (z_out) measure(x, z_out + (size_t)b * 2);
    }
    t = t1;
  }
  if (stop < 0 && terminated(s, x)) stop = i_start + nsub;
  if (stop >= 0) {
    done[b] = 1;
    iterm[b] = stop;
  }
  for (int i = 0; i < NX; ++i) x_true[(size_t)b * NX + i] = x[i];
  up[0] = c0;
  up[1] = c1;
}

thread_local std::string g_cl_err;

}  // namespace

struct mpcqp_cl {
  ClDev d;
  int32_t* dpos = nullptr;
  hipStream_t stream = nullptr;
  int64_t id0 = 0;          // global id of instance 0 (noise streams)
  bool has_plant = false;   // continuous-time plant set (mpcqp_cl_set_plant)
  PlantConsts pc{};
  int isDeltaV = 0;
  int32_t steps = 0;  // mpcqp_cl_step calls so far (the loop index of the next step)
};

extern "C" {

int mpcqp_cl_create(const mpcqp_cl_scenario* sc, int32_t batch, void* stream, mpcqp_cl** out) {
  if (!sc || !out || batch <= 0 || sc->Nx < sc->Nc || sc->Nx < sc->Nb) return -1;
  *out = nullptr;
  mpcqp_cl* cl = new mpcqp_cl();
  cl->d.sc = *sc;
  cl->d.B = batch;
  cl->stream = (hipStream_t)stream;
  const int np = sc->Nx + 1;
  if (hipMalloc(&cl->dpos, sizeof(int32_t) * 3 * np) != hipSuccess) {
    delete cl;
    return -2;
  }
  if (hipMemcpy(cl->dpos, sc->pos_c1, sizeof(int32_t) * np, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(cl->dpos + np, sc->pos_c2, sizeof(int32_t) * np, hipMemcpyHostToDevice) !=
          hipSuccess ||
      (sc->pos_slope && hipMemcpy(cl->dpos + 2 * np, sc->pos_slope, sizeof(int32_t) * np,
                                  hipMemcpyHostToDevice) != hipSuccess)) {
    (void)hipFree(cl->dpos);
    delete cl;
    return -2;
  }
  cl->d.pos_c1 = cl->dpos;
  cl->d.pos_c2 = cl->dpos + np;
  cl->d.pos_slope = sc->pos_slope ? cl->dpos + 2 * np : nullptr;
  cl->d.sc.pos_c1 = cl->d.sc.pos_c2 = cl->d.sc.pos_slope = nullptr;
  *out = cl;
  return 0;
}

int mpcqp_cl_destroy(mpcqp_cl* cl) {
  if (!cl) return 0;
  if (cl->dpos) (void)hipFree(cl->dpos);
  delete cl;
  return 0;
}

int mpcqp_cl_configure(mpcqp_cl* cl, double* xest, double* Ax, double* l, double* u) {
  if (!cl || !xest || !Ax || !l || !u) return -1;
  const int B = cl->d.B;
  hipLaunchKernelGGL(cl_configure_kernel, dim3((B + 255) / 256), dim3(256), 0, cl->stream, cl->d,
                     xest, Ax, l, u);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int mpcqp_cl_step(mpcqp_cl* cl, const int32_t* status, const double* x_sol, int32_t n,
                  int32_t u0_offset, double* x_true, double* ctrl_prev, double* xintf,
                  double* xest, int32_t* done, int32_t* ctrl_seq, double* ctrl_out,
                  const double* noise, double* z, double* u_applied) {
  if (!cl || !status || !x_sol || !x_true || !ctrl_prev || !xintf || !xest || !done ||
      !ctrl_seq || !ctrl_out)
    return -1;
  const int B = cl->d.B;
  cl->d.tr.step = cl->steps++;
  hipLaunchKernelGGL(cl_step_kernel, dim3((B + 255) / 256), dim3(256), 0, cl->stream, cl->d,
                     status, x_sol, n, u0_offset, x_true, ctrl_prev, xintf, xest, done, ctrl_seq,
                     ctrl_out, noise, z, u_applied);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int mpcqp_cl_set_tracking(mpcqp_cl* cl, int32_t* iterm, int32_t* success, double* final_err,
                          int32_t* n_fallback, double dist_tol, double ang_tol) {
  if (!cl) return -1;
  const bool any = iterm || success || final_err || n_fallback;
  if (any && !(iterm && success && final_err && n_fallback)) return -1;
  Track& t = cl->d.tr;
  t.iterm = iterm, t.success = success, t.final_err = final_err, t.n_fallback = n_fallback;
  t.dist_tol = dist_tol, t.ang_tol = ang_tol;
  t.rad2deg = 180.0 / 3.141592653589793;  // the reference's (180/np.pi)
  return 0;
}

int mpcqp_cl_set_ids(mpcqp_cl* cl, int64_t id0) {
  if (!cl || id0 < 0) return -1;
  cl->id0 = id0;
  return 0;
}

int mpcqp_cl_noise(mpcqp_cl* cl, uint64_t seed, uint64_t draw, double sig_x, double sig_y,
                   double* noise) {
  if (!cl || !noise) return -1;
  const int B = cl->d.B;
  hipLaunchKernelGGL(cl_noise_kernel, dim3((B + 255) / 256), dim3(256), 0, cl->stream, B, seed,
                     cl->id0, draw, sig_x, sig_y, noise);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int mpcqp_cl_set_plant(mpcqp_cl* cl, const mpcqp_plant_model* m, int32_t isDeltaV) {
  if (!cl || !m) return -1;
  cl->pc = PlantConsts{m->two_n, m->m_two_n, m->n2, m->R_T, m->mu, m->g0, m->rtol, m->atol};
  cl->isDeltaV = isDeltaV ? 1 : 0;
  cl->has_plant = true;
  return 0;
}

int mpcqp_clc_period(mpcqp_cl* cl, const int32_t* status, const double* x_sol, int32_t n,
                     int32_t u0_offset, double* x_true, double* ctrl_prev, double* xintf,
                     double* xest, int32_t* done, int32_t* iterm, int32_t* ctrl_seq,
                     double* ctrl_out, const double* noise, double* z, double* u_applied,
                     double t_start, double dt, int32_t i_start, int32_t nsub, double* traj) {
  if (!cl || !cl->has_plant || !status || !x_sol || !x_true || !ctrl_prev || !xintf || !xest ||
      !done || !iterm || !ctrl_seq || !ctrl_out || nsub < 1 || !(dt > 0.0))
    return -1;
  const int B = cl->d.B;
  hipLaunchKernelGGL(clc_period_kernel, dim3((B + 63) / 64), dim3(64), 0, cl->stream, cl->d,
                     cl->pc, cl->isDeltaV, status, x_sol, n, u0_offset, x_true, ctrl_prev, xintf,
                     xest, done, iterm, ctrl_seq, ctrl_out, noise, z, u_applied, t_start, dt,
                     i_start, nsub, traj);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
