// lane_swap_check.hip -- GPU check that the lane-swap cross-row stage of the wave sums (engine.hip wave_all)
// gives bitwise the readlane combination (r0 + r1) + (r2 + r3).  hipcc --offload-arch=gfx950 -O3 tools/lane_swap_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
template <int CTRL> __device__ double dpp_d(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ double rl(double x, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l), __builtin_amdgcn_readlane(__double2loint(x), l));
}
__device__ void sw16(double x, double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(x), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(x), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]); b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ void sw32(double x, double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(x), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(x), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]); b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__global__ void k(const double* in, double* out) {
  double x = in[blockIdx.x * 64 + threadIdx.x];
  x += dpp_d<0xB1>(x); x += dpp_d<0x4E>(x); x += dpp_d<0x141>(x); x += dpp_d<0x140>(x);
  const double r = (rl(x, 0) + rl(x, 16)) + (rl(x, 32) + rl(x, 48));
  double a, b;
  sw16(x, a, b); double y = a + b;
  sw32(y, a, b); y = a + b;
  out[(blockIdx.x * 64 + threadIdx.x) * 2] = r;
  out[(blockIdx.x * 64 + threadIdx.x) * 2 + 1] = y;
}
int main() {
  const int NB = 4096, N = NB * 64;
  double *h = (double*)malloc(N * 8), *o = (double*)malloc(N * 16), *di, *dout;
  srand(1);
  for (int i = 0; i < N; i++) h[i] = ((double)rand() / RAND_MAX - 0.5) * pow(10.0, rand() % 12 - 6);
  hipMalloc(&di, N * 8); hipMalloc(&dout, N * 16);
  hipMemcpy(di, h, N * 8, hipMemcpyHostToDevice);
  k<<<NB, 64>>>(di, dout);
  hipMemcpy(o, dout, N * 16, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int i = 0; i < N; i++) if (memcmp(&o[2 * i], &o[2 * i + 1], 8)) bad++;
  printf("redtest: %ld of %d lanes differ\n", bad, N);
  return bad != 0;
}
