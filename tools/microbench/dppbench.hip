// dppbench.hip — what a lone wave pays per instruction on gfx950 (the fan engine's row tail runs one wave per SIMD):
// shader cycles per instruction of short inline-asm streams, one wave per block, one block per CU, timed with
// s_memtime around ITER repetitions (printed per kind: the median over the 256 waves).
//   mov     : 32 independent v_mov_b32
//   bcast   : 32 v_mov_b32_dpp row_newbcast (independent destinations)
//   shr     : 32 v_mov_b32_dpp row_shr
//   mad_ind : 32 v_mad_u64_u32 into 8 accumulators round robin
//   mad_dep : 32 v_mad_u64_u32 into one accumulator (a dependent chain)
//   mad_4   : 32 v_mad_u64_u32 into 4 accumulators round robin
//   rowprod : 8 x (bcast, shr, shl, mad, mad) into 4 accumulators — the row product's pattern (40 instructions)
//   dpp_mad : 16 x (bcast, mad reading it at once) into 8 accumulators
//   hipcc -O3 --offload-arch=gfx950 dppbench.hip -o dppbench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define ITER 256

#define R8(X) X X X X X X X X
#define R4(X) X X X X

template <int KIND>
__global__ __launch_bounds__(64) void k_bench(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 7 + seed, b = threadIdx.x * 13 + 1, c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  uint64_t m0 = 0, m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0, m6 = 0, m7 = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
    if constexpr (KIND == 0) {
      asm volatile(R8("v_mov_b32 %0, %4\n v_mov_b32 %1, %4\n v_mov_b32 %2, %4\n v_mov_b32 %3, %4\n")
                   : "=v"(c0), "=v"(c1), "=v"(c2), "=v"(c3) : "v"(a));
    } else if constexpr (KIND == 1) {
      asm volatile(R8("v_mov_b32_dpp %0, %4 row_newbcast:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mov_b32_dpp %1, %4 row_newbcast:5 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mov_b32_dpp %2, %4 row_newbcast:9 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mov_b32_dpp %3, %4 row_newbcast:13 row_mask:0xf bank_mask:0xf bound_ctrl:1\n")
                   : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3) : "v"(a));
    } else if constexpr (KIND == 2) {
      asm volatile(R8("v_mov_b32_dpp %0, %4 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mov_b32_dpp %1, %4 row_shr:5 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mov_b32_dpp %2, %4 row_shr:9 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mov_b32_dpp %3, %4 row_shr:13 row_mask:0xf bank_mask:0xf bound_ctrl:1\n")
                   : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3) : "v"(a));
    } else if constexpr (KIND == 3) {
      asm volatile(R4("v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_mad_u64_u32 %1, vcc, %8, %9, %1\n"
                      "v_mad_u64_u32 %2, vcc, %8, %9, %2\n v_mad_u64_u32 %3, vcc, %8, %9, %3\n"
                      "v_mad_u64_u32 %4, vcc, %8, %9, %4\n v_mad_u64_u32 %5, vcc, %8, %9, %5\n"
                      "v_mad_u64_u32 %6, vcc, %8, %9, %6\n v_mad_u64_u32 %7, vcc, %8, %9, %7\n")
                   : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3), "+v"(m4), "+v"(m5), "+v"(m6), "+v"(m7)
                   : "v"(a), "v"(b) : "vcc");
    } else if constexpr (KIND == 4) {
      asm volatile(R8("v_mad_u64_u32 %0, vcc, %1, %2, %0\n v_mad_u64_u32 %0, vcc, %1, %2, %0\n"
                      "v_mad_u64_u32 %0, vcc, %1, %2, %0\n v_mad_u64_u32 %0, vcc, %1, %2, %0\n")
                   : "+v"(m0) : "v"(a), "v"(b) : "vcc");
    } else if constexpr (KIND == 5) {
      asm volatile(R8("v_mad_u64_u32 %0, vcc, %4, %5, %0\n v_mad_u64_u32 %1, vcc, %4, %5, %1\n"
                      "v_mad_u64_u32 %2, vcc, %4, %5, %2\n v_mad_u64_u32 %3, vcc, %4, %5, %3\n")
                   : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(a), "v"(b) : "vcc");
    } else if constexpr (KIND == 6) {
      asm volatile(R8("v_mov_b32_dpp %4, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mov_b32_dpp %5, %9 row_shr:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mov_b32_dpp %6, %9 row_shl:11 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mad_u64_u32 %0, vcc, %4, %5, %0\n"
                      "v_mad_u64_u32 %2, vcc, %4, %6, %2\n"
                      "v_mov_b32_dpp %7, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mov_b32_dpp %5, %9 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mov_b32_dpp %6, %9 row_shl:10 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mad_u64_u32 %1, vcc, %7, %5, %1\n"
                      "v_mad_u64_u32 %3, vcc, %7, %6, %3\n")
                   : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3), "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3)
                   : "v"(a), "v"(b) : "vcc");
    } else if constexpr (KIND == 7) {
      asm volatile(R8("v_mov_b32_dpp %8, %10 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mad_u64_u32 %0, vcc, %8, %11, %0\n"
                      "v_mov_b32_dpp %9, %10 row_newbcast:7 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                      "v_mad_u64_u32 %1, vcc, %9, %11, %1\n")
                   : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3), "+v"(m4), "+v"(m5), "+v"(m6), "+v"(m7),
                     "=&v"(c0), "=&v"(c1)
                   : "v"(a), "v"(b) : "vcc");
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t sink = m0 + m1 + m2 + m3 + m4 + m5 + m6 + m7 + c0 + c1 + c2 + c3;
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (sink == 0x123456789ull) out[blockIdx.x + 4096] = sink;
}

template <int KIND>
static double run(const char* name, int insts, uint64_t* d, int blocks, double mhz_ratio) {
  k_bench<KIND><<<blocks, 64>>>(d, 1);
  (void)hipDeviceSynchronize();
  k_bench<KIND><<<blocks, 64>>>(d, 2);
  (void)hipDeviceSynchronize();
  std::vector<uint64_t> h(blocks);
  (void)hipMemcpy(h.data(), d, blocks * sizeof(uint64_t), hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double ticks = (double)h[blocks / 2];
  const double cyc = ticks * mhz_ratio / ((double)ITER * insts);
  printf("%-8s %3d insts: %8.2f shader cycles per instruction (median of %d waves)\n", name, insts, cyc, blocks);
  return cyc;
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  // s_memtime counts at the shader clock on gfx9 (checked against the v_mov baseline: ~4 cycles a wave64 op)
  const int blocks = prop.multiProcessorCount;
  uint64_t* d;
  (void)hipMalloc(&d, 8192 * sizeof(uint64_t));
  printf("# dppbench: %d CUs, one wave per CU (ITER %d)\n", blocks, ITER);
  run<0>("mov", 32, d, blocks, 1.0);
  run<1>("bcast", 32, d, blocks, 1.0);
  run<2>("shr", 32, d, blocks, 1.0);
  run<3>("mad_ind", 32, d, blocks, 1.0);
  run<4>("mad_dep", 32, d, blocks, 1.0);
  run<5>("mad_4", 32, d, blocks, 1.0);
  run<6>("rowprod", 80, d, blocks, 1.0);
  run<7>("dpp_mad", 32, d, blocks, 1.0);
  return 0;
}
