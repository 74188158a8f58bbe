// valubench.hip — cycles per wave64 VALU instruction on gfx950 for the instruction classes of the SOP
// engine (lcv_col28.hpp / lcv_sop.hpp), measured with the shader clock (s_memtime) inside each wave,
// at W = 1, 2, 3, 4, 8 waves per SIMD (grid = 1024 W one-wave blocks: 256 CUs x 4 SIMDs).  This is the
// calibration of the VALU-pipe model in tools/valu_model.py (bench.py's roofline "valu_pipe" block):
//   pipe cycles of a launch = N_mad64 * C_mad + (N_valu - N_mad64) * C_valu
// and answers whether a quarter-rate v_mad_u64_u32 blocks the SIMD's VALU for its whole duration (the
// "mix" kernel: mads and full-rate adds interleaved 1:1; additive = blocking, max = overlap).
//   hipcc -O3 --offload-arch=gfx950 valubench.hip -o valubench && ./valubench
// Each kernel's loop body is 49 instructions of the class under test on 13 (or 49) independent
// accumulators plus 7 feedback XORs (so nothing is hoisted); per-iteration instruction counts are
// printed from the kernel's own loop shape, and tools/valu_model.py --isa checks them against the ISA.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048

__global__ __launch_bounds__(64) void k_mad(unsigned long long* cyc, uint64_t* out, uint32_t s) {
  uint32_t x[7], y[7];
  uint64_t c[13];
  for (int i = 0; i < 7; ++i) { x[i] = (threadIdx.x + s) * 2654435761u + i; y[i] = x[i] ^ 0x9e3779b9u; }
  for (int i = 0; i < 13; ++i) c[i] = i;
  const unsigned long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = 0; j < 7; ++j) c[i + j] += (uint64_t)x[i] * y[j];  // 49 v_mad_u64_u32
#pragma unroll
    for (int i = 0; i < 7; ++i) x[i] ^= (uint32_t)c[i];  // 7 v_xor_b32
  }
  const unsigned long long t1 = clock64();
  uint64_t r = 0;
  for (int i = 0; i < 13; ++i) r ^= c[i];
  out[blockIdx.x * 64 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_add(unsigned long long* cyc, uint64_t* out, uint32_t s) {
  uint32_t x[7], y[7], c[13];
  for (int i = 0; i < 7; ++i) { x[i] = (threadIdx.x + s) * 2654435761u + i; y[i] = x[i] ^ 0x9e3779b9u; }
  for (int i = 0; i < 13; ++i) c[i] = i;
  const unsigned long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = 0; j < 7; ++j) c[i + j] = (c[i + j] + x[i]) ^ y[j];  // 49 v_add3 / v_xad... (2 ops)
#pragma unroll
    for (int i = 0; i < 7; ++i) x[i] ^= c[i];
  }
  const unsigned long long t1 = clock64();
  uint64_t r = 0;
  for (int i = 0; i < 13; ++i) r ^= c[i];
  out[blockIdx.x * 64 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_mix(unsigned long long* cyc, uint64_t* out, uint32_t s) {
  uint32_t x[7], y[7], d[13];
  uint64_t c[13];
  for (int i = 0; i < 7; ++i) { x[i] = (threadIdx.x + s) * 2654435761u + i; y[i] = x[i] ^ 0x9e3779b9u; }
  for (int i = 0; i < 13; ++i) { c[i] = i; d[i] = 3 * i; }
  const unsigned long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        c[i + j] += (uint64_t)x[i] * y[j];  // v_mad_u64_u32
        d[i + j] += x[j] ^ y[i];            // simple ops on independent registers
      }
#pragma unroll
    for (int i = 0; i < 7; ++i) x[i] ^= (uint32_t)c[i] ^ d[i];
  }
  const unsigned long long t1 = clock64();
  uint64_t r = 0;
  for (int i = 0; i < 13; ++i) r ^= c[i] ^ d[i];
  out[blockIdx.x * 64 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_fma64(unsigned long long* cyc, uint64_t* out, uint32_t s) {
  double a[7], b[7], c[13];
  for (int i = 0; i < 7; ++i) { a[i] = 1.0 + (threadIdx.x + s + i) * 1e-9; b[i] = 0.999 - i * 1e-7; }
  for (int i = 0; i < 13; ++i) c[i] = i;
  const unsigned long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = 0; j < 7; ++j) c[i + j] = fma(a[i], b[j], c[i + j]);  // 49 v_fma_f64
#pragma unroll
    for (int i = 0; i < 7; ++i) a[i] = c[i] * 1e-30 + 1.0;  // 7 v_fma_f64
  }
  const unsigned long long t1 = clock64();
  double r = 0;
  for (int i = 0; i < 13; ++i) r += c[i];
  out[blockIdx.x * 64 + threadIdx.x] = (uint64_t)r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_add64(unsigned long long* cyc, uint64_t* out, uint32_t s) {
  uint64_t x[7], c[13];
  for (int i = 0; i < 7; ++i) x[i] = ((uint64_t)(threadIdx.x + s) << 33) * 2654435761u + i;
  for (int i = 0; i < 13; ++i) c[i] = i;
  const unsigned long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = 0; j < 7; ++j) c[i + j] += (x[i] << 2) + x[j];  // v_lshl_add_u64 (x2: shift-add, add)
#pragma unroll
    for (int i = 0; i < 7; ++i) x[i] ^= c[i];
  }
  const unsigned long long t1 = clock64();
  uint64_t r = 0;
  for (int i = 0; i < 13; ++i) r ^= c[i];
  out[blockIdx.x * 64 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// half the waves run the mad loop, half the add loop (by block parity): does a SIMD overlap one wave's
// back-to-back v_mad_u64_u32 with ANOTHER wave's full-rate instructions (compare with mad and add alone)?
__global__ __launch_bounds__(64) void k_split(unsigned long long* cyc, uint64_t* out, uint32_t s) {
  if (blockIdx.x & 1) {
    uint32_t x[7], y[7];
    uint64_t c[13];
    for (int i = 0; i < 7; ++i) { x[i] = (threadIdx.x + s) * 2654435761u + i; y[i] = x[i] ^ 0x9e3779b9u; }
    for (int i = 0; i < 13; ++i) c[i] = i;
    const unsigned long long t0 = clock64();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int i = 0; i < 7; ++i)
#pragma unroll
        for (int j = 0; j < 7; ++j) c[i + j] += (uint64_t)x[i] * y[j];
#pragma unroll
      for (int i = 0; i < 7; ++i) x[i] ^= (uint32_t)c[i];
    }
    const unsigned long long t1 = clock64();
    uint64_t r = 0;
    for (int i = 0; i < 13; ++i) r ^= c[i];
    out[blockIdx.x * 64 + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  } else {
    uint32_t x[7], y[7], d[13];
    for (int i = 0; i < 7; ++i) { x[i] = (threadIdx.x + s) * 2654435761u + i; y[i] = x[i] ^ 0x9e3779b9u; }
    for (int i = 0; i < 13; ++i) d[i] = 3 * i;
    const unsigned long long t0 = clock64();
    // 2 x 49 + 14 simple ops per iteration, about the mad loop's duration alone
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int i = 0; i < 7; ++i)
#pragma unroll
        for (int j = 0; j < 7; ++j) d[i + j] += x[j] ^ y[i];
#pragma unroll
      for (int i = 0; i < 7; ++i) x[i] ^= d[i];
    }
    const unsigned long long t1 = clock64();
    uint64_t r = 0;
    for (int i = 0; i < 13; ++i) r ^= d[i];
    out[blockIdx.x * 64 + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  }
}

typedef void (*kfn)(unsigned long long*, uint64_t*, uint32_t);
struct K { const char* name; kfn f; };

int main() {
  K ks[] = {{"mad  (49 v_mad_u64_u32 + 7 xor)", k_mad}, {"add  (49 x (add, xor) + 7 xor)", k_add},
            {"mix  (49 mad + 49 x (xor, add) + 14)", k_mix}, {"fma64 (56 v_fma_f64)", k_fma64},
            {"add64 (49 x 2 u64 shift-add + 7 u64 xor)", k_add64},
            {"split (odd waves: mad loop; even: xad loop)", k_split}};
  const int Ws[] = {1, 2, 3, 4, 8};
  unsigned long long* dcyc;
  uint64_t* out;
  hipMalloc(&dcyc, 8 * 1024 * sizeof(unsigned long long));
  hipMalloc(&out, (size_t)8 * 1024 * 64 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  unsigned long long* hc = (unsigned long long*)malloc(8 * 1024 * sizeof(unsigned long long));
  printf("kernel | waves/SIMD | shader cycles per loop iteration per wave (mean over waves) | SIMD cycles per "
         "iteration (wall, @2.4 GHz, = wall / (iters * W) per SIMD)\n");
  for (auto& k : ks) {
    for (int W : Ws) {
      const int blocks = 1024 * W;
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, dcyc, out, 1);
      hipDeviceSynchronize();
      hipEventRecord(a);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, dcyc, out, 2);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      hipMemcpy(hc, dcyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
      double sum = 0;
      for (int i = 0; i < blocks; ++i) sum += (double)hc[i];
      const double per_wave = sum / blocks / ITERS;
      const double simd_wall = ms * 1e-3 * 2.4e9 / ITERS / W;
      printf("%-44s W=%d : %9.1f cyc/iter/wave  | %8.1f SIMD-cyc/iter (wall %.3f ms)\n", k.name, W, per_wave, simd_wall, ms);
    }
  }
  return 0;
}
