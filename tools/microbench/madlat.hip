#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define ITERS 4096
// NCH independent accumulator chains of v_mad_u64_u32 + v_addc (the SOP column MAC pattern)
template <int NCH>
__global__ void k_chain(uint64_t* out, uint32_t s) {
  uint64_t acc[NCH];
  uint32_t hi[NCH];
  uint32_t x = threadIdx.x * 7 + s, y = threadIdx.x * 13 + 1;
  for (int c = 0; c < NCH; ++c) { acc[c] = c + s; hi[c] = 0; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1"
                   : "+v"(acc[c]), "=&s"(cc), "+v"(hi[c]) : "v"(x), "v"(y));
    }
    x += 0x9e3779b9u;
  }
  uint64_t r = 0;
  for (int c = 0; c < NCH; ++c) r += acc[c] + hi[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int NCH> void run(uint64_t* out, int blocks, int waves_per_block) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(k_chain<NCH>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, 1);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_chain<NCH>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, 2 + r);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double cyc = ms * 1e-3 * 2.4e9 / (3.0 * ITERS * NCH);
  printf("chains %d blocks %d waves/block %d : %.2f cycles per (mad+addc) per wave\n", NCH, blocks, waves_per_block, cyc);
}
int main() {
  uint64_t* out; hipMalloc(&out, (size_t)4096 * 1024 * 8);
  run<1>(out, 1, 1); run<2>(out, 1, 1); run<4>(out, 1, 1); run<8>(out, 1, 1);
  run<1>(out, 1, 2); run<1>(out, 1, 4); run<2>(out, 1, 2); run<2>(out, 1, 4);
  // one CU's SIMDs: 4 waves per block = one per SIMD? measure chip-level too
  run<1>(out, 1024, 2); run<2>(out, 1024, 2); run<1>(out, 2048, 4);
  return 0;
}
