// lds_probe.hip -- microbenchmark of the LDS operations the solve steps issue (Where the
// time goes): throughput per wave-instruction of ds_read_b64, ds_add_f64 (no return) and
// ds_write_b64 with 64 distinct conflict-free addresses, and the latency of a dependent solve-step
// chain (16 reads -> 8 fp64 products -> 3 atomics, the next step's reads behind them), at 1..8
// resident waves per CU (one wave per workgroup; the LDS allocation sets the waves per CU).
//   hipcc --offload-arch=gfx950 -O3 tools/lds_probe.hip -o tools/lds_probe && tools/lds_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((address_space(3))) double lds_double;

template <int MODE>
__global__ void __launch_bounds__(64) probe(double* out, int iters) {
  extern __shared__ double lds[];
  const int lane = threadIdx.x;
  for (int k = 0; k < 32; ++k) lds[lane + 64 * k] = 1e-3 * (lane + k);
  __syncthreads();
  const uint32_t base = (uint32_t)(uintptr_t)lds + lane * 8;
  double acc = 0.0;
  // opaque per-slot addresses (as the engine's records): stops the compiler from merging two
  // reads into one ds_read2st64_b64
  uint32_t ad[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    ad[k] = base + 512u * k;
    asm volatile("" : "+v"(ad[k]));
  }
  double mat[8], mat2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) mat[k] = lds[lane + 64 * k], mat2[k] = 0.0;
#pragma unroll 1
  for (int i = 0; i < iters; ++i) {
    if constexpr (MODE == 0) {  // 16 independent reads
      double x[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) x[k] = *(lds_double*)(size_t)(base + 512u * k);
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += x[k];
    } else if constexpr (MODE == 1) {  // 16 atomics
#pragma unroll
      for (int k = 0; k < 16; ++k)
        __hip_atomic_fetch_add((lds_double*)(size_t)(base + 512u * k), 1e-9, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (MODE == 2) {  // 16 writes
#pragma unroll
      for (int k = 0; k < 16; ++k) *(lds_double*)(size_t)(base + 512u * k) = acc + k;
      acc += 1.0;
    } else if constexpr (MODE >= 4 && MODE <= 9) {  // solve-step variants (see names[])
      // 4: 16 reads + 3 writes; 5: 16 reads + 2 atomics; 6: 4 b128 + 8 b64 reads + 3 atomics;
      // 7: 16 reads + 4 atomics; 8: 16 reads + 1 atomic; 9: 8 reads + 3 atomics, the other 8
      // operands (matrix values) from registers
      double x[16];
      if constexpr (MODE == 6) {
        typedef double d2 __attribute__((ext_vector_type(2)));
        typedef __attribute__((address_space(3))) d2 lds_d2;
        const uint32_t b2 = (uint32_t)(uintptr_t)lds + lane * 16;  // b128 pairs: conflict-free
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const d2 v = *(lds_d2*)(size_t)(b2 + 1024u * k);
          x[2 * k] = v.x, x[2 * k + 1] = v.y;
        }
#pragma unroll
        for (int k = 8; k < 16; ++k) x[k] = *(lds_double*)(size_t)ad[k];
        __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
      } else if constexpr (MODE == 9) {
#pragma unroll
        for (int k = 8; k < 16; ++k) x[k] = *(lds_double*)(size_t)ad[k];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = mat[k];  // matrix operands held in registers
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = *(lds_double*)(size_t)ad[k];
        __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
      const double n0 = fma(-x[1], x[9], -(x[0] * x[8]));
      const double n1 = fma(-x[3], x[11], -(x[2] * x[10]));
      const double n2 = fma(-x[5], x[13], -(x[4] * x[12]));
      const double n3 = fma(-x[7], x[15], -(x[6] * x[14]));
      auto add = [&](int slot, double v) {
        __hip_atomic_fetch_add((lds_double*)(size_t)ad[slot], v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      };
      if constexpr (MODE == 4) {
        *(lds_double*)(size_t)ad[16] = n0 + n1;
        *(lds_double*)(size_t)ad[17] = n2;
        *(lds_double*)(size_t)ad[18] = n3;
      } else if constexpr (MODE == 5) {
        add(16, n0 + n1), add(17, n2 + n3);
      } else if constexpr (MODE == 7) {
        add(16, n0), add(17, n1), add(18, n2), add(19, n3);
      } else if constexpr (MODE == 8) {
        add(16, (n0 + n1) + (n2 + n3));
      } else {
        add(16, n0 + n1), add(17, n2), add(18, n3);
      }
      asm volatile("" ::: "memory");
    } else if constexpr (MODE == 10) {
      // split step: the 8 operands the previous step's atomics cannot have written (the matrix
      // values) are read one step ahead, issued between this step's 8 dependent reads and its
      // products; the dependent reads follow the previous step's atomics.  Two steps per trip
      // (register sets mat / mat2 alternate), so no moves.
      auto step = [&](const double(&cur)[8], double(&nxt)[8]) {
        double y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) y[k] = *(lds_double*)(size_t)ad[8 + k];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 8; ++k) nxt[k] = *(lds_double*)(size_t)ad[k];
        __builtin_amdgcn_sched_barrier(0);
        const double n0 = fma(-cur[1], y[1], -(cur[0] * y[0])) + fma(-cur[3], y[3], -(cur[2] * y[2]));
        const double n2 = fma(-cur[5], y[5], -(cur[4] * y[4]));
        const double n3 = fma(-cur[7], y[7], -(cur[6] * y[6]));
        __hip_atomic_fetch_add((lds_double*)(size_t)ad[16], n0, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add((lds_double*)(size_t)ad[17], n2, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add((lds_double*)(size_t)ad[18], n3, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      };
      step(mat, mat2);
      step(mat2, mat);
      ++i;
    } else {  // one solve step: 16 reads, 8 products, 3 atomics; the next step reads behind them
      double x[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) x[k] = *(lds_double*)(size_t)ad[k];
      __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
      const double n0 = fma(-x[1], x[9], -(x[0] * x[8])) + fma(-x[3], x[11], -(x[2] * x[10]));
      const double n2 = fma(-x[5], x[13], -(x[4] * x[12]));
      const double n3 = fma(-x[7], x[15], -(x[6] * x[14]));
      __hip_atomic_fetch_add((lds_double*)(size_t)ad[16], n0, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add((lds_double*)(size_t)ad[17], n2, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add((lds_double*)(size_t)ad[18], n3, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      asm volatile("" ::: "memory");
    }
  }
  out[blockIdx.x * 64 + lane] = acc + lds[lane] + mat[lane & 7] + mat2[lane & 7];
}

int main() {
  double* out;
  (void)hipMalloc(&out, sizeof(double) * 64 * 256 * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  const char* names[11] = {"ds_read_b64 x16", "ds_add_f64 x16", "ds_write_b64 x16", "solve step",
                           "step 16r+3w", "step 16r+2a", "step 4q+8r+3a", "step 16r+4a",
                           "step 16r+1a", "step 8r+8reg+3a", "step split 8+8r+3a"};
  typedef void (*kfn)(double*, int);
  const kfn ks[11] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>,
                      probe<6>, probe<7>, probe<8>, probe<9>, probe<10>};
  for (int mode = 0; mode < 11; ++mode) {
    for (int wpc : {1, 2, 4, 8}) {
      const int lds = (160 * 1024) / wpc / 16 * 16;
      const int blocks = 256 * wpc;
      const kfn k = ks[mode];
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, blocks, 64, lds, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
      }
      const double cyc = best * 1e-3 * 2.4e9;
      const double ops = (double)iters * (mode >= 3 ? 1 : 16);
      printf("%-18s waves/CU %d: %8.3f ms  %7.2f CU cycles per wave-%s  (%7.2f per %s per wave)\n",
             names[mode], wpc, best, cyc / (ops * wpc), mode >= 3 ? "step" : "instr",
             cyc / ops, mode >= 3 ? "step" : "instr");
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) printf("error %s\n", hipGetErrorString(e));
  return 0;
}
