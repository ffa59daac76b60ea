// pmc_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access width the QP
// kernel uses (8 bytes per lane, coalesced: the per-instance Ax / l / u / iterate vectors).
// MI355X_MICROARCH.md: FETCH_SIZE is exact only up to a width-dependent factor on gfx950, so each
// counter is measured here against a known byte count.  Buffers are 1 GiB (> 256 MiB Infinity Cache).
//
//   hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
//   rocprofv3 --pmc FETCH_SIZE -d ... -- tools/pmc_calib      (and a second pass with WRITE_SIZE)
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void calib_read8(const double* __restrict__ a, double* __restrict__ out, size_t n) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    s += a[i];
  for (int k = 1; k < 64; k <<= 1) s += __shfl_xor(s, k);
  if (threadIdx.x == 0 && s == 12345.678) out[blockIdx.x] = s;  // never true: keeps the loads
}

__global__ void calib_write8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    a[i] = (double)i;
}

int main() {
  const size_t n = (size_t)1 << 27;  // 1 GiB of doubles
  double *a = nullptr, *o = nullptr;
  if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&o, 1 << 20) != hipSuccess) return 1;
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(calib_write8, dim3(8192), dim3(256), 0, 0, a, n);
    hipLaunchKernelGGL(calib_read8, dim3(8192), dim3(256), 0, 0, a, o, n);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"bytes_per_launch\": %zu}\n", n * 8);
  hipFree(a);
  hipFree(o);
  return 0;
}
