// fpbench.hip — measured cost of one 12x32-bit Montgomery Fp multiplication (lcv_field.hpp) on
// gfx950: "lone" = one wave (latency of a dependent chain), "full" = the whole chip (throughput).
// Variants: 1 chain per lane (inline product scanning), 2 independent chains interleaved, and the
// out-of-line call the engine uses (fp_mul -> fp_mul_call).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../light-client-consensus-specs_amd/csrc/lcv_field.hpp"

#define ITERS 256
using namespace lcv;

__global__ __launch_bounds__(64) void k_inline1(uint32_t* out, uint32_t s) {
  uint32_t x[12], y[12];
  for (int j = 0; j < 12; ++j) { x[j] = (threadIdx.x + s) * 2654435761u + j; y[j] = x[j] ^ 0x5bd1e995u; }
  x[11] &= 0xfffffff; y[11] &= 0xfffffff;
  for (int i = 0; i < ITERS; ++i) LCV_MUL_IMPL(x, x, y);
  uint32_t r = 0;
  for (int j = 0; j < 12; ++j) r ^= x[j];
  out[blockIdx.x * 64 + threadIdx.x] = r;
}
__global__ __launch_bounds__(64) void k_inline2(uint32_t* out, uint32_t s) {
  uint32_t x[12], z[12], y[12];
  for (int j = 0; j < 12; ++j) { x[j] = (threadIdx.x + s) * 2654435761u + j; y[j] = x[j] ^ 0x5bd1e995u; z[j] = x[j] + 7; }
  x[11] &= 0xfffffff; y[11] &= 0xfffffff; z[11] &= 0xfffffff;
  for (int i = 0; i < ITERS / 2; ++i) { LCV_MUL_IMPL(x, x, y); LCV_MUL_IMPL(z, z, y); }
  uint32_t r = 0;
  for (int j = 0; j < 12; ++j) r ^= x[j] ^ z[j];
  out[blockIdx.x * 64 + threadIdx.x] = r;
}
__global__ __launch_bounds__(64) void k_call1(uint32_t* out, uint32_t s) {
  fp x, y;
  for (int j = 0; j < 12; ++j) { x.v[j] = (threadIdx.x + s) * 2654435761u + j; y.v[j] = x.v[j] ^ 0x5bd1e995u; }
  x.v[11] &= 0xfffffff; y.v[11] &= 0xfffffff;
  for (int i = 0; i < ITERS; ++i) fp_mul(x, x, y);
  uint32_t r = 0;
  for (int j = 0; j < 12; ++j) r ^= x.v[j];
  out[blockIdx.x * 64 + threadIdx.x] = r;
}

typedef void (*kfn)(uint32_t*, uint32_t);
int main() {
  struct { const char* name; kfn f; } ks[] = {{"inline, 1 chain", k_inline1}, {"inline, 2 chains", k_inline2}, {"fp_mul call", k_call1}};
  uint32_t* out;
  hipMalloc(&out, (size_t)16384 * 64 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (auto& k : ks) {
    for (int blocks : {1, 1024, 2048, 4096, 16384}) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, out, 1);
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, out, 2 + r);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double muls = (double)blocks * 64 * ITERS * 3.0;
      printf("%-18s blocks %6d: %8.1f cycles per mul per wave @2.4GHz, %7.2f G Fp mul/s\n", k.name, blocks,
             ms * 1e-3 / 3.0 * 2.4e9 / ITERS, muls / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
