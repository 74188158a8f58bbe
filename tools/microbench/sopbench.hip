// sopbench.hip — cost of one SOP op (lcv_sop.hpp sop_exec: 32-bit words in LDS, 28-bit limb column
// products) by round shape: K products, 2-term operands, the X * m multiplier, subtraction steps, shadow.  Each lane runs ITER ops on its own LDS slots (one
// team of 64 lanes per block); "full" = 2048 one-wave blocks (2 waves per SIMD).
//   hipcc -O3 --offload-arch=gfx950 -I../../light-client-consensus-specs_amd/csrc sopbench.hip -o sopbench
#define LCV_HD __device__
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "lcv_sop.hpp"

#define ITER 64
#define NS 16

__global__ __launch_bounds__(64) void k_op(const uint32_t* rec, uint32_t h0, uint32_t words, uint32_t* out) {
  // NS input slots shared by the block's lanes (read-only), one output slot per lane, the constant table
  // (per-lane records: lane L runs record L & 7, so operands differ across lanes as in the programs)
  __shared__ uint32_t lds[NS * 12 + 64 * 24 + 2 * 12];
  uint32_t* in = lds;
  uint32_t* wr = lds + NS * 12 + threadIdx.x * 24;
  uint32_t* cl = lds + NS * 12 + 64 * 24;  // constant 0 = zero
  if (threadIdx.x < NS)
    for (int j = 0; j < 12; ++j) in[12 * threadIdx.x + j] = (j < 11) ? (0x9e3779b9u * (threadIdx.x + 3 * j + 1)) : 0x0a000000u + threadIdx.x;
  if (threadIdx.x == 0)
    for (int j = 0; j < 24; ++j) cl[j] = 0;
  __syncthreads();
  for (int it = 0; it < ITER; ++it) lcv::sop_exec(h0, ((h0 >> 7) & 1u ? 0xFFFFu : 0u) | ((h0 >> 8) & 1u ? 0xFFFF0000u : 0u), rec + (threadIdx.x & 7) * words, lcv::sop_pre(h0, rec + (threadIdx.x & 7) * words), in, wr, cl, NS, nullptr, nullptr);
  out[blockIdx.x * 64 + threadIdx.x] = wr[0];
}

struct Shape { const char* name; int K, x2, y2, neg, mflag, x15, red, sh, kara; };

int main() {
  Shape shapes[] = {{"K0 red0", 0, 0, 0, 0, 0, 0, 0, 0, 0}, {"K1 red0", 1, 0, 0, 0, 0, 0, 0, 0, 0},
                    {"K1 red0 kara", 1, 0, 0, 0, 0, 0, 0, 0, 1}, {"K1 red3", 1, 0, 0, 0, 0, 0, 3, 0, 0},
                    {"K4 red0", 4, 0, 0, 0, 0, 0, 0, 0, 0}, {"K4 red0 kara", 4, 0, 0, 0, 0, 0, 0, 0, 1},
                    {"K7 red0", 7, 0, 0, 0, 0, 0, 0, 0, 0}, {"K7 red0 kara", 7, 0, 0, 0, 0, 0, 0, 0, 1},
                    {"K4 +x2y2 red0", 4, 1, 1, 0, 0, 0, 0, 0, 0}, {"K4 +m red0", 4, 0, 0, 0, 1, 0, 0, 0, 0},
                    {"K4 +m x15 red0", 4, 0, 0, 0, 1, 1, 0, 0, 0}, {"K3 fexp-like", 3, 1, 0, 0, 1, 0, 3, 1, 0},
                    {"K3 fexp-like kara", 3, 1, 0, 0, 1, 0, 3, 1, 1}, {"K7 acc-like", 7, 1, 0, 0, 1, 0, 2, 0, 0},
                    {"K7 acc-like kara", 7, 1, 0, 0, 1, 0, 2, 0, 1}};
  uint32_t *drec, *dout;
  hipMalloc(&drec, 8 * 64 * 4);
  hipMalloc(&dout, 4096 * 64 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (auto& sh : shapes) {
    const uint32_t words = 4 + 3 * sh.K;
    uint32_t rec[8 * 64] = {0};
    for (int L = 0; L < 8; ++L) {
      uint32_t* r = rec + L * words;
      r[0] = 0;                                            // dst: the lane's output slot
      r[1] = (sh.sh ? 1u : 0x3FFu) << 12 | 0x3FFu << 22;   // shadow slot: the lane's second slot
      r[2] = r[3] = NS;                                    // add-ins: the zero constant, coefficient 0
      for (int k = 0; k < sh.K; ++k) {
        const uint32_t x0 = (k + L) % NS, x1 = sh.x2 ? ((k + 1 + 2 * L) % NS) : NS;
        const uint32_t y0 = (k + 3 + 3 * L) % NS, y1 = sh.y2 ? ((k + 5 + L) % NS) : NS;
        r[4 + 3 * k] = x0 | x1 << 16;
        r[5 + 3 * k] = y0 | y1 << 16;
        r[6 + 3 * k] = sh.mflag ? 6 : 1;
      }
    }
    const uint32_t h0 = sh.K | (sh.K ? 0u : 1u) << 4 | sh.mflag << 6 | sh.x2 << 7 | sh.y2 << 8 | sh.neg << 9 |
                        sh.sh << 13 | (uint32_t)sh.red << 16 | sh.x15 << 21 | sh.kara << 22 | 1u << 24;
    hipMemcpy(drec, rec, sizeof(rec), hipMemcpyHostToDevice);
    for (int mode = 0; mode < 2; ++mode) {
      const int blocks = mode ? 2048 : 1;
      hipLaunchKernelGGL(k_op, dim3(blocks), dim3(64), 0, 0, drec, h0, words, dout);
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_op, dim3(blocks), dim3(64), 0, 0, drec, h0, words, dout);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double waves_per_simd = mode ? 2048.0 / 1024.0 : 1.0;
      const double cyc = ms * 1e-3 * 2.4e9 / (3.0 * ITER) / waves_per_simd;  // SIMD cycles per op per wave
      printf("%-18s %s: %8.0f SIMD cycles per op (%6.0f per product)\n", sh.name, mode ? "full(2/SIMD)" : "lone wave  ",
             cyc, cyc / (sh.K ? sh.K : 1));
    }
  }
  return 0;
}
