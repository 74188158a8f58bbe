// peakbench.hip — the roofline denominator: the chip's issue rate of exactly the
// instructions the SOP engine's products are made of, measured in wall time, with no compiler freedom.
// Every loop body is inline asm: 128 instructions per iteration on 16 independent accumulators (no
// dependent chain shorter than 8 instructions, no shifts, no loads), plus a 3-instruction scalar loop.
// Grid: 1024 * W one-wave blocks = W waves per SIMD on the 1,024 SIMDs of the MI355X (256 CUs x 4).
//   mad   : v_mad_u64_u32 (a 28 x 28-bit column MAC of lcv_col28.hpp: col[i + j] += x_i * y_j)
//   madi  : v_mad_i64_i32 (the signed Karatsuba middle term)
//   add   : v_add_u32 (a full-rate 32-bit instruction)
//   mix   : 64 mad interleaved with 64 add
//   add64 : v_lshl_add_u64 (64-bit column joins / carries)
//   mullo : v_mul_lo_u32 (Montgomery quotient digits)
//   fma64 : v_fma_f64
// Output, per kernel and W: wall ms, instructions per second (whole chip), SIMD cycles per instruction at
// the measured shader clock (s_memtime over the kernel, per wave, mean) and at 2.4 GHz.  The MAC peak
// in the op model's units (bench.py roofline) is 2 ops per v_mad_u64_u32 issued: 2 * mad_per_s.
//   hipcc -O3 --offload-arch=gfx950 peakbench.hip -o peakbench && ./peakbench > peakbench.txt
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096
#define PER_ITER 128

// one asm statement per 16 instructions: inside it the compiler inserts nothing (between separate inline
// asm statements its hazard recognizer would put an s_nop); 16 accumulators c (VGPR pairs), 16 words x
#define OPS16 "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]), \
    "+v"(c[8]), "+v"(c[9]), "+v"(c[10]), "+v"(c[11]), "+v"(c[12]), "+v"(c[13]), "+v"(c[14]), "+v"(c[15]), \
    "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), \
    "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]), \
    "=s"(sc)
#define OPS16F "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7]), \
    "+v"(f[8]), "+v"(f[9]), "+v"(f[10]), "+v"(f[11]), "+v"(f[12]), "+v"(f[13]), "+v"(f[14]), "+v"(f[15]), \
    "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), \
    "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15])
#define MAD16 "v_mad_u64_u32 %0, %32, %16, %33, %0\n" \
"v_mad_u64_u32 %1, %32, %17, %33, %1\n" \
"v_mad_u64_u32 %2, %32, %18, %33, %2\n" \
"v_mad_u64_u32 %3, %32, %19, %33, %3\n" \
"v_mad_u64_u32 %4, %32, %20, %33, %4\n" \
"v_mad_u64_u32 %5, %32, %21, %33, %5\n" \
"v_mad_u64_u32 %6, %32, %22, %33, %6\n" \
"v_mad_u64_u32 %7, %32, %23, %33, %7\n" \
"v_mad_u64_u32 %8, %32, %24, %33, %8\n" \
"v_mad_u64_u32 %9, %32, %25, %33, %9\n" \
"v_mad_u64_u32 %10, %32, %26, %33, %10\n" \
"v_mad_u64_u32 %11, %32, %27, %33, %11\n" \
"v_mad_u64_u32 %12, %32, %28, %33, %12\n" \
"v_mad_u64_u32 %13, %32, %29, %33, %13\n" \
"v_mad_u64_u32 %14, %32, %30, %33, %14\n" \
"v_mad_u64_u32 %15, %32, %31, %33, %15\n"
#define MADI16 "v_mad_i64_i32 %0, %32, %16, %33, %0\n" \
"v_mad_i64_i32 %1, %32, %17, %33, %1\n" \
"v_mad_i64_i32 %2, %32, %18, %33, %2\n" \
"v_mad_i64_i32 %3, %32, %19, %33, %3\n" \
"v_mad_i64_i32 %4, %32, %20, %33, %4\n" \
"v_mad_i64_i32 %5, %32, %21, %33, %5\n" \
"v_mad_i64_i32 %6, %32, %22, %33, %6\n" \
"v_mad_i64_i32 %7, %32, %23, %33, %7\n" \
"v_mad_i64_i32 %8, %32, %24, %33, %8\n" \
"v_mad_i64_i32 %9, %32, %25, %33, %9\n" \
"v_mad_i64_i32 %10, %32, %26, %33, %10\n" \
"v_mad_i64_i32 %11, %32, %27, %33, %11\n" \
"v_mad_i64_i32 %12, %32, %28, %33, %12\n" \
"v_mad_i64_i32 %13, %32, %29, %33, %13\n" \
"v_mad_i64_i32 %14, %32, %30, %33, %14\n" \
"v_mad_i64_i32 %15, %32, %31, %33, %15\n"
#define ADD16 "v_add_u32 %16, %16, %33\n" \
"v_add_u32 %17, %17, %33\n" \
"v_add_u32 %18, %18, %33\n" \
"v_add_u32 %19, %19, %33\n" \
"v_add_u32 %20, %20, %33\n" \
"v_add_u32 %21, %21, %33\n" \
"v_add_u32 %22, %22, %33\n" \
"v_add_u32 %23, %23, %33\n" \
"v_add_u32 %24, %24, %33\n" \
"v_add_u32 %25, %25, %33\n" \
"v_add_u32 %26, %26, %33\n" \
"v_add_u32 %27, %27, %33\n" \
"v_add_u32 %28, %28, %33\n" \
"v_add_u32 %29, %29, %33\n" \
"v_add_u32 %30, %30, %33\n" \
"v_add_u32 %31, %31, %33\n"
#define MIX16 "v_mad_u64_u32 %0, %32, %16, %33, %0\n" \
"v_add_u32 %17, %17, %33\n" \
"v_mad_u64_u32 %2, %32, %18, %33, %2\n" \
"v_add_u32 %19, %19, %33\n" \
"v_mad_u64_u32 %4, %32, %20, %33, %4\n" \
"v_add_u32 %21, %21, %33\n" \
"v_mad_u64_u32 %6, %32, %22, %33, %6\n" \
"v_add_u32 %23, %23, %33\n" \
"v_mad_u64_u32 %8, %32, %24, %33, %8\n" \
"v_add_u32 %25, %25, %33\n" \
"v_mad_u64_u32 %10, %32, %26, %33, %10\n" \
"v_add_u32 %27, %27, %33\n" \
"v_mad_u64_u32 %12, %32, %28, %33, %12\n" \
"v_add_u32 %29, %29, %33\n" \
"v_mad_u64_u32 %14, %32, %30, %33, %14\n" \
"v_add_u32 %31, %31, %33\n"
#define ADD64_16 "v_lshl_add_u64 %0, %0, 0, %1\n" \
"v_lshl_add_u64 %1, %1, 0, %2\n" \
"v_lshl_add_u64 %2, %2, 0, %3\n" \
"v_lshl_add_u64 %3, %3, 0, %4\n" \
"v_lshl_add_u64 %4, %4, 0, %5\n" \
"v_lshl_add_u64 %5, %5, 0, %6\n" \
"v_lshl_add_u64 %6, %6, 0, %7\n" \
"v_lshl_add_u64 %7, %7, 0, %8\n" \
"v_lshl_add_u64 %8, %8, 0, %9\n" \
"v_lshl_add_u64 %9, %9, 0, %10\n" \
"v_lshl_add_u64 %10, %10, 0, %11\n" \
"v_lshl_add_u64 %11, %11, 0, %12\n" \
"v_lshl_add_u64 %12, %12, 0, %13\n" \
"v_lshl_add_u64 %13, %13, 0, %14\n" \
"v_lshl_add_u64 %14, %14, 0, %15\n" \
"v_lshl_add_u64 %15, %15, 0, %0\n"
#define MULLO16 "v_mul_lo_u32 %16, %16, %33\n" \
"v_mul_lo_u32 %17, %17, %33\n" \
"v_mul_lo_u32 %18, %18, %33\n" \
"v_mul_lo_u32 %19, %19, %33\n" \
"v_mul_lo_u32 %20, %20, %33\n" \
"v_mul_lo_u32 %21, %21, %33\n" \
"v_mul_lo_u32 %22, %22, %33\n" \
"v_mul_lo_u32 %23, %23, %33\n" \
"v_mul_lo_u32 %24, %24, %33\n" \
"v_mul_lo_u32 %25, %25, %33\n" \
"v_mul_lo_u32 %26, %26, %33\n" \
"v_mul_lo_u32 %27, %27, %33\n" \
"v_mul_lo_u32 %28, %28, %33\n" \
"v_mul_lo_u32 %29, %29, %33\n" \
"v_mul_lo_u32 %30, %30, %33\n" \
"v_mul_lo_u32 %31, %31, %33\n"
#define FMA16 "v_fma_f64 %0, %0, %33, %33\n" \
"v_fma_f64 %1, %1, %33, %33\n" \
"v_fma_f64 %2, %2, %33, %33\n" \
"v_fma_f64 %3, %3, %33, %33\n" \
"v_fma_f64 %4, %4, %33, %33\n" \
"v_fma_f64 %5, %5, %33, %33\n" \
"v_fma_f64 %6, %6, %33, %33\n" \
"v_fma_f64 %7, %7, %33, %33\n" \
"v_fma_f64 %8, %8, %33, %33\n" \
"v_fma_f64 %9, %9, %33, %33\n" \
"v_fma_f64 %10, %10, %33, %33\n" \
"v_fma_f64 %11, %11, %33, %33\n" \
"v_fma_f64 %12, %12, %33, %33\n" \
"v_fma_f64 %13, %13, %33, %33\n" \
"v_fma_f64 %14, %14, %33, %33\n" \
"v_fma_f64 %15, %15, %33, %33\n"

template <int K>
__global__ __launch_bounds__(64) void k_peak(uint64_t* out, uint64_t* cyc, uint32_t s) {
  uint64_t c[16];
  uint32_t x[16];
  double f[16];
  uint64_t sc;  // the mads' carry-out (unused)
  for (int i = 0; i < 16; ++i) {
    x[i] = (threadIdx.x + s) * 2654435761u + i * 0x9e3779b9u;
    c[i] = x[i] * 3ull;
    f[i] = (double)x[i];
  }
  const uint32_t y = s * 0x85ebca6bu + 1u;
  const double g = 1.0000001;
  const uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int rep = 0; rep < PER_ITER / 16; ++rep) {
      if constexpr (K == 0) asm volatile(MAD16 : OPS16 : "v"(y));
      else if constexpr (K == 1) asm volatile(MADI16 : OPS16 : "v"(y));
      else if constexpr (K == 2) asm volatile(ADD16 : OPS16 : "v"(y));
      else if constexpr (K == 3) asm volatile(MIX16 : OPS16 : "v"(y));
      else if constexpr (K == 4) asm volatile(ADD64_16 : OPS16 : "v"(y));
      else if constexpr (K == 5) asm volatile(MULLO16 : OPS16 : "v"(y));
      else asm volatile(FMA16 : OPS16F : "v"(g));
    }
  }
  const uint64_t t1 = clock64();
  uint64_t r = 0;
  for (int i = 0; i < 16; ++i) r ^= c[i] ^ x[i] ^ (uint64_t)f[i];
  out[blockIdx.x * 64 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  struct K { const char* name; void (*f)(uint64_t*, uint64_t*, uint32_t); int mads; };
  const K ks[] = {{"mad   v_mad_u64_u32", k_peak<0>, PER_ITER}, {"madi  v_mad_i64_i32", k_peak<1>, PER_ITER},
                  {"add   v_add_u32", k_peak<2>, 0},           {"mix   mad/add 64+64", k_peak<3>, PER_ITER / 2},
                  {"add64 v_lshl_add_u64", k_peak<4>, 0},      {"mullo v_mul_lo_u32", k_peak<5>, 0},
                  {"fma64 v_fma_f64", k_peak<6>, 0}};
  int dev = 0, cus = 0, khz = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, dev);
  const int simds = 4 * cus;
  printf("# peakbench: %d CUs, %d SIMDs, max shader clock %.0f MHz; %d instructions per wave per launch\n", cus, simds,
         khz / 1e3, ITERS * PER_ITER);
  printf("# kernel               W | wall ms | G wave-instr/s | SIMD cyc/instr @clock64 | @2.4GHz | mad T/s | op-model T ops/s (2/mad)\n");
  uint64_t *out, *cyc;
  hipMalloc(&out, (size_t)8 * simds * 64 * 8);
  hipMalloc(&cyc, (size_t)8 * simds * 8);
  uint64_t* hc = (uint64_t*)malloc((size_t)8 * simds * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (const K& k : ks)
    for (int W : {1, 2, 3, 4, 8}) {
      const int blocks = simds * W;
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, out, cyc, 1);  // warm-up
      hipDeviceSynchronize();
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, out, cyc, 2 + rep);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      hipMemcpy(hc, cyc, (size_t)blocks * 8, hipMemcpyDeviceToHost);
      double mean_cyc = 0;
      for (int i = 0; i < blocks; ++i) mean_cyc += (double)hc[i];
      mean_cyc /= blocks;
      const double instr = (double)ITERS * PER_ITER;                // per wave
      const double wave_instr_per_s = instr * blocks / (best * 1e-3);
      const double cyc_clock = mean_cyc / instr / W;                // a wave's cycles shared by W waves per SIMD
      const double cyc_24 = best * 1e-3 * 2.4e9 / (instr * W);
      const double mad_per_s = wave_instr_per_s * 64.0 * k.mads / PER_ITER;
      printf("%-22s %d | %7.3f | %14.1f | %23.2f | %7.2f | %7.2f | %7.2f\n", k.name, W, best, wave_instr_per_s / 1e9,
             cyc_clock, cyc_24, mad_per_s / 1e12, 2 * mad_per_s / 1e12);
      fflush(stdout);
    }
  return 0;
}
