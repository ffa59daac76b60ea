// closed_loop.hip -- device-side closed-loop step around the batched QP solve (see
// include/mpcqp_closed_loop.h).  One thread per chaser; this is scalar per-instance logic, a few
// hundred bytes of traffic per instance and step, far off the solve's critical path.
//
// Arithmetic that feeds comparisons with the reference (slopes, intercepts, norms, the plant) uses
// explicitly rounded operations (__dmul_rn / __dadd_rn) in the reference's evaluation order, so
// that no FMA contraction changes a branch the reference would take.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "../../include/mpcqp_closed_loop.h"

namespace {

constexpr int NX = 4, NU = 2, NY = 5, NDI = 2;

struct ClDev {
  mpcqp_cl_scenario sc;  // host pointers inside are not used on the device
  const int32_t *pos_c1, *pos_c2, *pos_slope;
  int B;
};

__device__ __forceinline__ double mul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double add(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ double sub(double a, double b) { return __dsub_rn(a, b); }

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

// reference src/trajectorySimulate.py:288-337 for one chaser (noise = None)
__global__ void __launch_bounds__(256) cl_step_kernel(ClDev d, const int32_t* status,
                                                      const double* x_sol, int n, int u0,
                                                      double* x_true, double* ctrl_prev,
                                                      double* xintf, double* xest, int32_t* done,
                                                      int32_t* ctrl_seq, double* ctrl_out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  const mpcqp_cl_scenario& s = d.sc;
  if (done[b]) {
    ctrl_seq[b] = 0;
    return;
  }
  const double* xe = xest + (size_t)b * 6;
  double c0, c1;
  int seq;
  if (status[b] != 1) {
    const double h = s.side / 2;
    const bool in_box = s.has_debris && sub(xe[0], add(s.center[0], h)) < 0 &&
                        sub(xe[0], sub(s.center[0], h)) > 0 && xe[1] < add(s.center[1], h) &&
                        xe[1] > sub(s.center[1], h);
    double xi = xintf[b];
    if (in_box) {  // deadbeat debris avoidance
      double cy = 0.0;
      for (int k = 0; k < NX; ++k) cy = add(cy, mul(s.Crefy[k], xe[k]));
      xi = sub(add(xi, cy), add(s.center[1], h));
      c0 = sub(-(add(add(add(mul(s.Ktot[0], xe[0]), mul(s.Ktot[1], xe[1])), mul(s.Ktot[2], xe[2])),
                     mul(s.Ktot[3], xe[3]))),
               mul(s.Ki[0], xi));
      c1 = sub(-(add(add(add(mul(s.Ktot[4], xe[0]), mul(s.Ktot[5], xe[1])), mul(s.Ktot[6], xe[2])),
                     mul(s.Ktot[7], xe[3]))),
               mul(s.Ki[1], xi));
      seq = 3;
    } else {  // LQR failsafe (homing)
      double cxr = 0.0;
      for (int k = 0; k < NX; ++k) cxr = add(cxr, mul(s.Crefx[k], xe[k]));
      xi = sub(add(xi, cxr), s.xr[0]);
      c0 = sub(-(add(add(add(mul(s.Kpf[0], xe[0]), mul(s.Kpf[1], xe[1])), mul(s.Kpf[2], xe[2])),
                     mul(s.Kpf[3], xe[3]))),
               mul(s.Kif[0], xi));
      c1 = sub(-(add(add(add(mul(s.Kpf[4], xe[0]), mul(s.Kpf[5], xe[1])), mul(s.Kpf[6], xe[2])),
                     mul(s.Kpf[7], xe[3]))),
               mul(s.Kif[1], xi));
      seq = 2;
    }
    xintf[b] = xi;
  } else {
    xintf[b] = 0.0;
    c0 = x_sol[(size_t)b * n + u0];
    c1 = x_sol[(size_t)b * n + u0 + 1];
    seq = 1;
  }
  // input-norm clip with the reference's sequential rescale (quirk Q2)
  const double um = s.umax[0];
  double nr = sqrt(add(mul(c0, c0), mul(c1, c1)));
  if (nr > um) {
    c0 = mul(c0, um / nr);
    nr = sqrt(add(mul(c0, c0), mul(c1, c1)));
    c1 = mul(c1, um / nr);
  }
  ctrl_seq[b] = seq;
  ctrl_out[(size_t)b * 2] = c0;
  ctrl_out[(size_t)b * 2 + 1] = c1;
  // plant: x+ = Ad x + Bd u_prev (one-sample actuation delay, quirk Q1); CSC column order
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
  for (int i = 0; i < NX; ++i) xn[i] = add(add(ax[i], bu[i]), 0.0);
  for (int i = 0; i < NX; ++i) xt[i] = xn[i];
  up[0] = c0;
  up[1] = c1;
  double* xw = xest + (size_t)b * 6;
  for (int i = 0; i < NX; ++i) xw[i] = xn[i];
  xw[4] = 0.0;
  xw[5] = 0.0;
  // termination test of the next loop iteration (src/trajectorySimulate.py:288-293)
  const double rn = sqrt(add(mul(xn[0], xn[0]), mul(xn[1], xn[1])));
  const double pos = s.inTrack ? xn[1] : xn[0];
  if (rn < s.rp || pos < sub(s.rp, s.rtol)) done[b] = 1;
}

thread_local std::string g_cl_err;

}  // namespace

struct mpcqp_cl {
  ClDev d;
  int32_t* dpos = nullptr;
  hipStream_t stream = nullptr;
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
                  double* xest, int32_t* done, int32_t* ctrl_seq, double* ctrl_out) {
  if (!cl || !status || !x_sol || !x_true || !ctrl_prev || !xintf || !xest || !done ||
      !ctrl_seq || !ctrl_out)
    return -1;
  const int B = cl->d.B;
  hipLaunchKernelGGL(cl_step_kernel, dim3((B + 255) / 256), dim3(256), 0, cl->stream, cl->d,
                     status, x_sol, n, u0_offset, x_true, ctrl_prev, xintf, xest, done, ctrl_seq,
                     ctrl_out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
