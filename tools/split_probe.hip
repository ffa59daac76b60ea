// split_probe.hip -- prices a solve step shared by the two waves of one QP instance (VERDICT r03
// item 1) against today's one-wave step, with the dependent chain of the engine: per step the
// lanes read operands, form products and add them into targets with LDS atomics; the next step's
// reads must see the sums.  One wave: LDS executes a wave's operations in order, no wait.  Two
// waves: each wave does half of the step, then s_waitcnt lgkmcnt(0) + s_barrier (the other wave's
// sums must have landed before either reads).  Reported: CU cycles per INSTANCE-step at 1, 2, 4
// instances per CU (LDS allocation per workgroup sets the residency).
//   hipcc --offload-arch=gfx950 -O3 tools/split_probe.hip -o tools/split_probe && tools/split_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((address_space(3))) double lds_double;

__device__ __forceinline__ void add_at(uint32_t a, double v) {
  __hip_atomic_fetch_add((lds_double*)(size_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// MODE 0: one wave per instance, full step (16 reads, 3 atomics), no barrier (today's engine)
// MODE 1: two waves, each a half step (8 reads, 2 atomics) + lgkmcnt(0) + barrier
// MODE 2: two waves, each a half step (8 reads, 1 atomic)  + lgkmcnt(0) + barrier
// MODE 3: two waves, each a full step (16 reads, 3 atomics) + lgkmcnt(0) + barrier (per instance-
//         step: two steps' work per barrier interval, counted as 2 instance-steps)
// MODE 4: one wave, full step + lgkmcnt(0) + barrier (the price of the wait alone)
// MODE 5: two waves, half step (8 reads, 2 atomics), no wait and no barrier (upper bound)
template <int MODE>
__global__ void __launch_bounds__(128) probe(double* out, int iters) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nt = blockDim.x;
  for (int k = 0; k < 40; ++k) lds[tid + nt * k] = 1e-3 * (tid + k);
  __syncthreads();
  const uint32_t base = (uint32_t)(uintptr_t)lds + (uint32_t)(wave * 64 + lane) * 8u;
  uint32_t ad[24];
#pragma unroll
  for (int k = 0; k < 24; ++k) {
    ad[k] = base + (uint32_t)nt * 8u * k;
    asm volatile("" : "+v"(ad[k]));
  }
  double acc = 0.0;
  constexpr bool HALF = (MODE == 1 || MODE == 2 || MODE == 5);
  constexpr bool SYNC = (MODE >= 1 && MODE <= 4);
#pragma unroll 1
  for (int i = 0; i < iters; ++i) {
    if constexpr (HALF) {
      double x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = *(lds_double*)(size_t)ad[k];
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
      const double n0 = fma(-x[1], x[5], -(x[0] * x[4]));
      const double n1 = fma(-x[3], x[7], -(x[2] * x[6]));
      if constexpr (MODE == 2) {
        add_at(ad[16], n0 + n1);
      } else {
        add_at(ad[16], n0);
        add_at(ad[17], n1);
      }
    } else {
      double x[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) x[k] = *(lds_double*)(size_t)ad[k];
      __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
      const double n0 = fma(-x[1], x[9], -(x[0] * x[8])) + fma(-x[3], x[11], -(x[2] * x[10]));
      const double n2 = fma(-x[5], x[13], -(x[4] * x[12]));
      const double n3 = fma(-x[7], x[15], -(x[6] * x[14]));
      add_at(ad[16], n0);
      add_at(ad[17], n2);
      add_at(ad[18], n3);
    }
    asm volatile("" ::: "memory");
    if constexpr (SYNC) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  out[blockIdx.x * nt + tid] = acc + lds[tid];
}

int main() {
  double* out;
  (void)hipMalloc(&out, sizeof(double) * 128 * 256 * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  const char* names[6] = {"1 wave full 16r+3a", "2 waves half 8r+2a+bar", "2 waves half 8r+1a+bar",
                          "2 waves full 16r+3a+bar", "1 wave full +wait+bar", "2 waves half, no bar"};
  const int wpi[6] = {1, 2, 2, 2, 1, 2};
  // instance-steps per trip: half steps complete one instance-step per trip, full steps on two
  // waves complete two
  const int isteps[6] = {1, 1, 1, 2, 1, 1};
  typedef void (*kfn)(double*, int);
  const kfn ks[6] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>};
  for (int mode = 0; mode < 6; ++mode) {
    for (int ipc : {1, 2, 4}) {
      const int lds = (160 * 1024) / ipc / 16 * 16;
      const int blocks = 256 * ipc;
      const kfn k = ks[mode];
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, blocks, 64 * wpi[mode], lds, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
      }
      const double cyc = best * 1e-3 * 2.4e9;
      const double steps = (double)iters * isteps[mode];
      printf("%-26s inst/CU %d (waves/CU %d): %8.3f ms  %7.2f CU cycles per instance-step  (%7.2f per step per instance)\n",
             names[mode], ipc, ipc * wpi[mode], best, cyc / (steps * ipc), cyc / steps);
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) printf("error %s\n", hipGetErrorString(e));
  return 0;
}
