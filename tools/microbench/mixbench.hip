// mixbench.hip — does interleaving a wave's v_mad_u64_u32 with independent full-rate VALU instructions
// (as opposed to a block of mads followed by a block of other instructions) shorten the SIMD's time?
// The SOP engine's product loop (lcv_sop.hpp sop_products) runs ~70-140 conversion / add instructions
// and then 147 back-to-back mads per product.  Three kernels, same instructions per iteration:
//   block : 49 mads (7 x 7 column MAC), then 49 simple ops (xor/add chains on other registers)
//   inter : the same, forced into mad / simple alternation with __builtin_amdgcn_sched_barrier(0)
//   mad   : the 49 mads alone
// Grid = 1024 W one-wave blocks (W waves per SIMD); wall time per iteration per SIMD at 2.4 GHz.
//   hipcc -O3 --offload-arch=gfx950 mixbench.hip -o mixbench && ./mixbench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048
#define SB() __builtin_amdgcn_sched_barrier(0)

template <int MODE>
__global__ __launch_bounds__(64) void k_bench(uint64_t* out, uint32_t s) {
  uint32_t x[7], y[7], d[7], e[7];
  uint64_t c[13];
  for (int i = 0; i < 7; ++i) {
    x[i] = (threadIdx.x + s) * 2654435761u + i; y[i] = x[i] ^ 0x9e3779b9u;
    d[i] = x[i] * 3u; e[i] = y[i] + 7u;
  }
  for (int i = 0; i < 13; ++i) c[i] = i;
  for (int it = 0; it < ITERS; ++it) {
    if (MODE == 1) {  // interleaved: mad, simple, mad, simple ...
#pragma unroll
      for (int i = 0; i < 7; ++i)
#pragma unroll
        for (int j = 0; j < 7; ++j) {
          c[i + j] += (uint64_t)x[i] * y[j];
          d[j] = (d[j] ^ e[i]) + i;  // v_xad_u32 (1 instruction), independent of the mads
          SB();
        }
    } else {
#pragma unroll
      for (int i = 0; i < 7; ++i)
#pragma unroll
        for (int j = 0; j < 7; ++j) c[i + j] += (uint64_t)x[i] * y[j];
      SB();
      if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < 7; ++i)
#pragma unroll
          for (int j = 0; j < 7; ++j) d[j] = (d[j] ^ e[i]) + i;
        SB();
      }
    }
#pragma unroll
    for (int i = 0; i < 7; ++i) { x[i] ^= (uint32_t)c[i]; e[i] ^= d[i]; }
    SB();
  }
  uint64_t r = 0;
  for (int i = 0; i < 13; ++i) r ^= c[i];
  for (int i = 0; i < 7; ++i) r ^= d[i] ^ e[i];
  out[blockIdx.x * 64 + threadIdx.x] = r;
}

int main() {
  struct { const char* name; void (*f)(uint64_t*, uint32_t); } ks[] = {
      {"block (49 mad, then 49 xad)", k_bench<0>}, {"inter (49 x (mad, xad))", k_bench<1>},
      {"mad   (49 mad)", k_bench<2>}};
  uint64_t* out;
  hipMalloc(&out, (size_t)8 * 1024 * 64 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (auto& k : ks)
    for (int W : {1, 2, 3, 4, 8}) {
      hipLaunchKernelGGL(k.f, dim3(1024 * W), dim3(64), 0, 0, out, 1);
      hipDeviceSynchronize();
      hipEventRecord(a);
      hipLaunchKernelGGL(k.f, dim3(1024 * W), dim3(64), 0, 0, out, 2);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("%-30s W=%d : %8.1f SIMD-cyc/iter (wall %.3f ms)\n", k.name, W, ms * 1e-3 * 2.4e9 / ITERS / W, ms);
    }
  return 0;
}
