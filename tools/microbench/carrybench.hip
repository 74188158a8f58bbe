// carrybench.hip — issue cost of the product-scan multiply-accumulate forms on gfx950:
//   sgpr : v_mad_u64_u32 (carry-out to an SGPR pair) + VOP3 v_addc_co_u32 reading it (the SOP engine's form)
//   vcc  : the same with the carry in VCC and the VOP2 (e32) v_addc_co_u32
//   mad  : v_mad_u64_u32 alone (no carry add: the reduced-radix form, 64-bit column accumulators)
// NCH independent chains per lane; "lone" = one wave, "full" = 2048 blocks x 4 waves (8 waves per SIMD).
//   hipcc -O3 --offload-arch=gfx950 carrybench.hip -o carrybench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048

template <int MODE, int NCH>
__global__ void k_chain(uint64_t* out, uint32_t s) {
  uint64_t acc[NCH];
  uint32_t hi[NCH];
  uint32_t x = threadIdx.x * 7 + s, y = threadIdx.x * 13 + 1;
  for (int c = 0; c < NCH; ++c) { acc[c] = c + s; hi[c] = 0; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      uint64_t cc;
      if constexpr (MODE == 0) {
        asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1"
                     : "+v"(acc[c]), "=&s"(cc), "+v"(hi[c]) : "v"(x), "v"(y));
      } else if constexpr (MODE == 1) {
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                     : "+v"(acc[c]), "+v"(hi[c]) : "v"(x), "v"(y) : "vcc");
      } else {
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=&s"(cc) : "v"(x), "v"(y));
      }
    }
    x += 0x9e3779b9u;
  }
  uint64_t r = 0;
  for (int c = 0; c < NCH; ++c) r += acc[c] + hi[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int MODE, int NCH> void run(const char* name, uint64_t* out, int blocks, int waves_per_block) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((k_chain<MODE, NCH>), dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, 1);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_chain<MODE, NCH>), dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, 2 + r);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  const double waves_per_simd = blocks * waves_per_block / 1024.0;
  const double cyc = ms * 1e-3 * 2.4e9 / (3.0 * ITERS * NCH);
  printf("%-5s chains %d %s: %6.2f cycles per MAC per wave, %6.2f SIMD cycles per MAC\n", name, NCH,
         blocks == 1 ? "lone wave     " : "8 waves / SIMD", cyc, blocks == 1 ? cyc : cyc / waves_per_simd);
}

int main() {
  uint64_t* out; hipMalloc(&out, (size_t)2048 * 256 * 8);
  run<0, 1>("sgpr", out, 1, 1); run<0, 4>("sgpr", out, 1, 1); run<0, 4>("sgpr", out, 2048, 4);
  run<1, 1>("vcc", out, 1, 1); run<1, 4>("vcc", out, 1, 1); run<1, 4>("vcc", out, 2048, 4);
  run<2, 1>("mad", out, 1, 1); run<2, 4>("mad", out, 1, 1); run<2, 4>("mad", out, 2048, 4);
  return 0;
}
