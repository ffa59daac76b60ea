#include <hip/hip_runtime.h>
#include <cstdio>
typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
__device__ v4f raw_load_fmt(Rsrc rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.ptr.buffer.load.format.v4f32");
__global__ void check(const uint32_t* tbl, uint32_t* out) {
  Rsrc rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(tbl), (short)0, 4096, 0x64FAC);
  v4f x = raw_load_fmt(rs, threadIdx.x * 8, 0, 0);
  *(v4u*)(out + threadIdx.x * 4) = __builtin_bit_cast(v4u, x);
}
template <int MODE>
__global__ void bench(const uint32_t* tbl, uint32_t* out, int iters) {
  Rsrc rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(tbl), (short)0, 1 << 16, MODE == 2 ? 0x64FAC : 0x00020000);
  unsigned acc = 0;
  int off = (threadIdx.x & 63) * 16;
  #pragma unroll 1
  for (int i = 0; i < iters; ++i) {
    #pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int o = off + ((i * 5 + k) & 31) * 1024;
      if constexpr (MODE == 0) {
        v4u v = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
        acc += v.x ^ v.y ^ v.z ^ v.w;
      } else if constexpr (MODE == 1) {
        v2u v = __builtin_bit_cast(v2u, __builtin_amdgcn_raw_buffer_load_b64(rs, o / 2, 0, 0));
        acc += (v.x & 0xffff) ^ (v.x >> 16) ^ (v.y & 0xffff) ^ (v.y >> 16);
      } else {
        v4u v = __builtin_bit_cast(v4u, raw_load_fmt(rs, o / 2, 0, 0));
        acc += v.x ^ v.y ^ v.z ^ v.w;
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
int main() {
  uint32_t* h = new uint32_t[16384];
  for (int i = 0; i < 16384; ++i) h[i] = (uint32_t)(((2*i+1) & 0xffff) << 16 | ((2*i) & 0xffff));
  uint32_t *d, *o; (void)hipMalloc(&d, 65536); (void)hipMalloc(&o, 1 << 24); (void)hipMemcpy(d, h, 65536, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(check, 1, 64, 0, 0, d, o); uint32_t r[256]; (void)hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
  bool ok = true;
  for (int l = 0; l < 64; ++l) for (int c = 0; c < 4; ++c) ok = ok && r[4*l+c] == (uint32_t)(4*l+c);
  printf("format check %s: lane1 %u %u %u %u\n", ok ? "OK" : "FAIL", r[4], r[5], r[6], r[7]);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000;
  for (int mode = 0; mode < 3; ++mode) for (int wpc : {4, 8, 16}) {
    int blocks = 256 * wpc / 4;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(bench<0>, blocks, 256, 0, 0, d, o, iters);
      if (mode == 1) hipLaunchKernelGGL(bench<1>, blocks, 256, 0, 0, d, o, iters);
      if (mode == 2) hipLaunchKernelGGL(bench<2>, blocks, 256, 0, 0, d, o, iters);
      hipEventRecord(e1); hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("mode %d waves/CU %2d: %.3f ms, %.2f cycles per wave-load per CU (2.4GHz)\n", mode, wpc, ms,
                      ms * 1e-3 * 2.4e9 / ((double)iters * 5 * wpc));
    }
  }
  return 0;
}
