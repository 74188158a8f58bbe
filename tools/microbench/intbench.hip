// intbench.hip — measured gfx950 rates of the integer instructions the Fp arithmetic is built from
// (roofline denominators for BASELINE.md / DESIGN.md).  Each kernel runs ITERS iterations of 8
// independent dependency chains per lane; "lone" launches one wave (per-wave issue/latency), "full"
// launches 2048 workgroups x 256 threads (chip throughput).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096
#define CH 8

__global__ void k_mad64(uint64_t* out, uint32_t s) {  // v_mad_u64_u32
  uint64_t acc[CH];
  uint32_t x = threadIdx.x * 2654435761u + s;
  for (int k = 0; k < CH; ++k) acc[k] = x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = (uint64_t)(uint32_t)acc[k] * (x + k) + (acc[k] >> 32);
  }
  uint64_t r = 0;
  for (int k = 0; k < CH; ++k) r ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mullo(uint64_t* out, uint32_t s) {  // v_mul_lo_u32 + v_add
  uint32_t acc[CH];
  uint32_t x = threadIdx.x * 2654435761u + s;
  for (int k = 0; k < CH; ++k) acc[k] = x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = acc[k] * (x | 1u) + k;
  }
  uint32_t r = 0;
  for (int k = 0; k < CH; ++k) r ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mulhi(uint64_t* out, uint32_t s) {  // v_mul_hi_u32
  uint32_t acc[CH];
  uint32_t x = threadIdx.x * 2654435761u + s;
  for (int k = 0; k < CH; ++k) acc[k] = x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = __umulhi(acc[k], x | 0x80000001u) ^ k;
  }
  uint32_t r = 0;
  for (int k = 0; k < CH; ++k) r ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_add(uint64_t* out, uint32_t s) {  // v_add_u32 (+ xor)
  uint32_t acc[CH];
  uint32_t x = threadIdx.x * 2654435761u + s;
  for (int k = 0; k < CH; ++k) acc[k] = x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = (acc[k] + x) ^ (k * 0x9e3779b9u);
  }
  uint32_t r = 0;
  for (int k = 0; k < CH; ++k) r ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_u24(uint64_t* out, uint32_t s) {  // v_mad_u32_u24
  uint32_t acc[CH];
  uint32_t x = (threadIdx.x * 2654435761u + s) & 0xffffff;
  for (int k = 0; k < CH; ++k) acc[k] = x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = __umul24(acc[k] & 0xffffff, x) + k;
  }
  uint32_t r = 0;
  for (int k = 0; k < CH; ++k) r ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_fma64(uint64_t* out, uint32_t s) {  // v_fma_f64
  double acc[CH];
  double x = 1.0 + (threadIdx.x + s) * 1e-9;
  for (int k = 0; k < CH; ++k) acc[k] = x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = fma(acc[k], 0.999999, x);
  }
  double r = 0;
  for (int k = 0; k < CH; ++k) r += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)r;
}
__global__ void k_addc(uint64_t* out, uint32_t s) {  // 64-bit add = v_add_co_u32 + v_addc_co_u32
  uint64_t acc[CH];
  uint64_t x = (uint64_t)(threadIdx.x * 2654435761u + s) << 20 | 0xfffff;
  for (int k = 0; k < CH; ++k) acc[k] = x + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = (acc[k] + x) ^ k;
  }
  uint64_t r = 0;
  for (int k = 0; k < CH; ++k) r ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef void (*kfn)(uint64_t*, uint32_t);
struct K { const char* name; kfn f; int ops; };  // ops per chain-iteration (instructions counted)

int main() {
  K ks[] = {{"v_mad_u64_u32 (+v_lshr)", k_mad64, 1}, {"v_mul_lo_u32(+add)", k_mullo, 1}, {"v_mul_hi_u32(+xor)", k_mulhi, 1},
            {"v_add_u32(+xor)", k_add, 2}, {"v_mul_u32_u24(+and/add)", k_u24, 1}, {"v_fma_f64", k_fma64, 1},
            {"u64 add(+xor)", k_addc, 1}};
  uint64_t* out;
  hipMalloc(&out, (size_t)2048 * 256 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (auto& k : ks) {
    for (int mode = 0; mode < 2; ++mode) {
      const int blocks = mode ? 2048 : 1, threads = mode ? 256 : 64;
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1);
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 2 + r);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double lanes = (double)blocks * threads, chains = lanes * CH * ITERS * 3.0;
      const double per_s = chains * k.ops / (ms * 1e-3);
      if (mode == 0)
        printf("%-26s lone wave : %8.2f cycles/chain-iter/wave @2.4GHz (8 chains interleaved)\n", k.name,
               ms * 1e-3 * 2.4e9 / (ITERS * 3.0 * CH));
      else
        printf("%-26s full chip : %8.2f T lane-ops/s (%d counted op/iter)\n", k.name, per_s / 1e12, k.ops);
    }
  }
  return 0;
}
