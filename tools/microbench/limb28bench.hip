// limb28bench.hip — cost of a SOP-shaped op (K products + one Montgomery reduction) with 14 x 28-bit
// limbs and 64-bit column accumulators (no carry adds: every column stays below 2^64 for K <= 7), for
// comparison with sopbench (the 12 x 32-bit product scan with a carry add per product).
//   hipcc -O3 -w --offload-arch=gfx950 limb28bench.hip -o limb28bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITER 64
#define NS 16
#define NL 14
#define M28 0x0FFFFFFFu

// p of BLS12-381 in 14 x 28-bit limbs (little-endian), n' = -p^-1 mod 2^28 (filled on the host)
__constant__ uint32_t c_p28[NL];
__constant__ uint32_t c_np28;

template <int K>
__device__ __forceinline__ void op28(uint32_t* dst, const uint32_t* lds, int lane) {
  uint64_t col[2 * NL];
#pragma unroll
  for (int c = 0; c < 2 * NL; ++c) col[c] = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t* xs = lds + NL * ((k + lane) % 8);
    const uint32_t* ys = lds + NL * ((k + 3 + lane) % 8);
    uint32_t x[NL], y[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) { x[i] = xs[i]; y[i] = ys[i]; }
#pragma unroll
    for (int i = 0; i < NL; ++i)
#pragma unroll
      for (int j = 0; j < NL; ++j) col[i + j] += (uint64_t)x[i] * y[j];
  }
  uint32_t p[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) p[j] = c_p28[j];
  const uint32_t np = c_np28;
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint64_t v = col[i] + carry;
    const uint32_t q = ((uint32_t)v * np) & M28;
    carry = (v + (uint64_t)q * p[0]) >> 28;
#pragma unroll
    for (int j = 1; j < NL; ++j) col[i + j] += (uint64_t)q * p[j];
  }
  uint32_t r[NL];
#pragma unroll
  for (int i = NL; i < 2 * NL; ++i) {
    const uint64_t v = col[i] + carry;
    r[i - NL] = (uint32_t)v & M28;
    carry = v >> 28;
  }
#pragma unroll
  for (int j = 0; j < NL; ++j) dst[j] = r[j];
}

template <int K>
__global__ __launch_bounds__(64) void k_op(uint32_t* out) {
  __shared__ uint32_t lds[NS * NL + 64 * NL];
  uint32_t* in = lds;
  uint32_t* wr = lds + NS * NL + threadIdx.x * NL;
  if (threadIdx.x < NS)
    for (int j = 0; j < NL; ++j) in[NL * threadIdx.x + j] = (0x9e3779b9u * (threadIdx.x + 3 * j + 1)) & (j < 13 ? M28 : 0xFFFFFu);
  __syncthreads();
  for (int it = 0; it < ITER; ++it) {
    op28<K>(wr, in, (threadIdx.x + it) & 7);
    __syncthreads();
  }
  out[blockIdx.x * 64 + threadIdx.x] = wr[0];
}

template <int K> void run(uint32_t* dout) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int mode = 0; mode < 2; ++mode) {
    const int blocks = mode ? 2048 : 1;
    hipLaunchKernelGGL(k_op<K>, dim3(blocks), dim3(64), 0, 0, dout);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_op<K>, dim3(blocks), dim3(64), 0, 0, dout);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double waves_per_simd = mode ? 2048.0 / 1024.0 : 1.0;
    const double cyc = ms * 1e-3 * 2.4e9 / (3.0 * ITER) / waves_per_simd;
    printf("28-bit K%d %s: %8.0f SIMD cycles per op (%6.0f per product)\n", K, mode ? "full(2/SIMD)" : "lone wave  ", cyc,
           cyc / K);
  }
}

int main() {
  // p = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
  const char* hex = "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab";
  uint32_t w[12] = {0};
  for (int i = 0; i < 96; ++i) {
    const char ch = hex[95 - i];
    const uint32_t d = ch <= '9' ? ch - '0' : ch - 'a' + 10;
    w[i / 8] |= d << (4 * (i % 8));
  }
  uint32_t p28[NL];
  for (int l = 0; l < NL; ++l) {
    uint32_t v = 0;
    for (int bit = 0; bit < 28; ++bit) {
      const int g = 28 * l + bit;
      if (g < 384 && (w[g / 32] >> (g % 32)) & 1u) v |= 1u << bit;
    }
    p28[l] = v;
  }
  uint32_t inv = 1;  // p^-1 mod 2^32 by Newton
  for (int i = 0; i < 5; ++i) inv *= 2 - p28[0] * inv;
  const uint32_t np = (0u - inv) & M28;
  hipMemcpyToSymbol(HIP_SYMBOL(c_p28), p28, sizeof(p28));
  hipMemcpyToSymbol(HIP_SYMBOL(c_np28), &np, sizeof(np));
  uint32_t* dout;
  hipMalloc(&dout, 2048 * 64 * 4);
  run<1>(dout);
  run<4>(dout);
  run<7>(dout);
  return 0;
}
