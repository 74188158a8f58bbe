// fp64bench.hip — VERDICT r05 item 2(d): is a 381 x 381-bit product cheaper on the FP64 FMA pipe than on the
// 28-bit-limb integer column engine the SOP programs use (lcv_col28.hpp)?
//   int28  : 14 x 28-bit limbs, one subtractive Karatsuba level (three 7 x 7 products = 147 v_mad_u64_u32 /
//            v_mad_i64_i32 into 64-bit columns) and the join — exactly sop_kara_mac + sop_kara_join.
//   fp49   : 8 x 49-bit limbs held in doubles (392 bits), schoolbook 8 x 8; each limb product a b < 2^98 is
//            split exactly by two FMAs: h = fma(a, b, C) with C = 3 * 2^100 (so C + ab lies in [2^101, 2^102)
//            and its ulp is 2^49), s = h - C (exact, a multiple of 2^49), l = fma(a, b, -s) (exact, |l| <=
//            2^48); the column sums H_k += s (multiples of 2^49 below 2^101: exact) and L_k += l (|L_k| <=
//            2^51: exact) — 2 FMA + 3 ADD per limb product, every intermediate exact, no integer instruction.
//   fp49k  : the same with one Karatsuba level over 4-limb halves (three 4 x 4 products: 48 limb products;
//            the middle term's limbs are signed differences in (-2^49, 2^49), inside C's window), joined in
//            int64 after an exact one-op conversion of each partial column.
// Both engines produce the same 762-bit integer: the check kernel normalises the three column vectors to
// 32-bit words on the device and the host compares them for 4,096 random operand pairs (bit-exact or not).
// Timing: W one-wave blocks per SIMD, every lane multiplying ITER times, each product's low column fed
// back into the next operands (the same xor in all kernels), wall time with HIP events; reported as SIMD
// cycles per product at 2.4 GHz (a wave's 64 products).
//   hipcc -O3 --offload-arch=gfx950 -I../../light-client-consensus-specs_amd/csrc fp64bench.hip -o fp64bench
#define LCV_HD __device__
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "lcv_col28.hpp"

#define ITER 256

static constexpr double CSPLIT = 3.0 * 1267650600228229401496703205376.0;  // 3 * 2^100
static constexpr double TWO49 = 562949953421312.0;                        // 2^49 (the limb base)

__device__ __forceinline__ void fp_split(double a, double b, double& H, double& L) {
  const double h = __fma_rn(a, b, CSPLIT);
  const double s = h - CSPLIT;
  const double l = __fma_rn(a, b, -s);
  H += s;
  L += l;
}

// 12 x 32-bit words (< 2^384) -> 8 x 49-bit limbs as doubles
__device__ __forceinline__ void to49(double d[8], const uint32_t w[12]) {
#pragma unroll
  for (int l = 0; l < 8; ++l) {
    const int b = 49 * l, k = b / 32, s = b % 32;
    uint64_t x = k < 12 ? (uint64_t)w[k] >> s : 0;
    if (k + 1 < 12) x |= (uint64_t)w[k + 1] << (32 - s);
    if (s > 15 && k + 2 < 12) x |= (uint64_t)w[k + 2] << (64 - s);
    d[l] = (double)(x & ((1ull << 49) - 1));
  }
}

__device__ __forceinline__ void mul_int28(uint64_t col[28], const uint32_t a[12], const uint32_t b[12]) {
  uint32_t X[15], Y[14];
  lcv::sop_to28<12, 14>(X, a);
  lcv::sop_to28<12, 14>(Y, b);
  X[14] = 0;
  uint64_t p0[13], p2[13];
  int64_t pd[13];
  lcv::sop_kara_mac<true>(p0, p2, pd, X, Y);
  lcv::sop_kara_join(col, p0, p2, pd);
}

__device__ __forceinline__ void mul_fp49(double H[16], double L[16], const double A[8], const double B[8]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) H[k] = L[k] = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) fp_split(A[i], B[j], H[i + j], L[i + j]);
}

// one Karatsuba level: A B = P0 + (P0 + P2 + D) 2^196 + P2 2^392, D = (A0 - A1)(B1 - B0) (limb differences in
// (-2^49, 2^49): the products stay inside C's window).  The three partial column sums (H multiples of 2^49,
// |H| < 4 * 2^98; |L| <= 2^50) are converted to int64 exactly by one FP op each (fma(H, 2^-49, M) and L + M
// with M = 1.5 * 2^52: |integer| < 2^51 sits in the low mantissa bits) and joined with 64-bit integer adds:
// col[k] = value of column k in units of 2^(49 k) (H of column k counts in column k + 1).
__device__ __forceinline__ int64_t magic_i64(double x) {
  return (int64_t)(__double_as_longlong(x) - __double_as_longlong(6755399441055744.0));
}
__device__ __forceinline__ void mul_fp49k(int64_t col[17], const double A[8], const double B[8]) {
  double h0[7], l0[7], h2[7], l2[7], hd[7], ld[7], da[4], db[4];
#pragma unroll
  for (int k = 0; k < 7; ++k) h0[k] = l0[k] = h2[k] = l2[k] = hd[k] = ld[k] = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) { da[i] = A[i] - A[i + 4]; db[i] = B[i + 4] - B[i]; }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      fp_split(A[i], B[j], h0[i + j], l0[i + j]);
      fp_split(A[i + 4], B[j + 4], h2[i + j], l2[i + j]);
      fp_split(da[i], db[j], hd[i + j], ld[i + j]);
    }
  const double M = 6755399441055744.0, S = 1.0 / TWO49;
  int64_t q0[8], q2[8], qd[8];  // per part: column k (units 2^(49 k)), k = 0..7
#pragma unroll
  for (int k = 0; k < 8; ++k) q0[k] = q2[k] = qd[k] = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    q0[k] += magic_i64(l0[k] + M); q0[k + 1] += magic_i64(__fma_rn(h0[k], S, M));
    q2[k] += magic_i64(l2[k] + M); q2[k + 1] += magic_i64(__fma_rn(h2[k], S, M));
    qd[k] += magic_i64(ld[k] + M); qd[k + 1] += magic_i64(__fma_rn(hd[k], S, M));
  }
#pragma unroll
  for (int k = 0; k < 17; ++k) col[k] = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    col[k] += q0[k];
    col[k + 4] += q0[k] + q2[k] + qd[k];
    col[k + 8] += q2[k];
  }
}

template <int E>
__global__ __launch_bounds__(64) void k_bench(const uint32_t* in, uint64_t* out) {
  uint32_t a[12], b[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    a[j] = in[(blockIdx.x * 64 + threadIdx.x) % 4096 * 24 + j];
    b[j] = in[(blockIdx.x * 64 + threadIdx.x) % 4096 * 24 + 12 + j];
  }
  uint64_t acc = 0;
  if constexpr (E == 0) {
    for (int it = 0; it < ITER; ++it) {
      uint64_t col[28];
      mul_int28(col, a, b);
      // feed back: every column (all 64 bits of it) reaches the next operands
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        a[j] = (a[j] ^ (uint32_t)(col[j] >> 24)) & 0x3FFFFFFFu;
        b[j] = (b[j] ^ (uint32_t)(col[j + 14] >> 24)) & 0x3FFFFFFFu;
      }
      acc ^= col[12] ^ col[13] ^ col[26] ^ col[27];
    }
  } else {
    double A[8], B[8];
    to49(A, a);
    to49(B, b);
    for (int it = 0; it < ITER; ++it) {
      if constexpr (E == 1) {
        double H[16], L[16];
        mul_fp49(H, L, A, B);
        // feed back: every column (H and L) reaches the next operands (limbs kept below 2^49)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          A[i] = fabs(__fma_rn(H[i], 0x1p-102, L[i] * 0x1p-3));
          B[i] = fabs(__fma_rn(H[i + 8], 0x1p-102, L[i + 8] * 0x1p-3));
        }
      } else {
        int64_t col[17];
        mul_fp49k(col, A, B);
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // feed back: every column reaches the next operands
          A[i] = (double)((uint64_t)col[i] >> 16);
          B[i] = (double)((uint64_t)col[i + 8] >> 16);
        }
        acc ^= (uint64_t)col[16];
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= (uint64_t)__double_as_longlong(A[i]) ^ (uint64_t)__double_as_longlong(B[i]);
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}

// the 768-bit product as 24 words from each representation (check kernel, one product per lane)
__global__ __launch_bounds__(64) void k_check(const uint32_t* in, uint32_t* out, int n) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= n) return;
  uint32_t a[12], b[12];
  for (int j = 0; j < 12; ++j) { a[j] = in[t * 24 + j]; b[j] = in[t * 24 + 12 + j]; }
  // int28 columns -> words
  uint64_t col[28];
  mul_int28(col, a, b);
  {
    uint32_t w[25] = {0};
    unsigned __int128 c = 0;
    int bit = 0, wi = 0;
    unsigned __int128 buf = 0;
    for (int k = 0; k < 28; ++k) {
      c += col[k];
      buf |= (unsigned __int128)(uint32_t)(c & ((1u << 28) - 1)) << bit;
      c >>= 28;
      bit += 28;
      while (bit >= 32 && wi < 25) { w[wi++] = (uint32_t)buf; buf >>= 32; bit -= 32; }
    }
    buf |= c << bit;
    while (wi < 24) { w[wi++] = (uint32_t)buf; buf >>= 32; }
    for (int j = 0; j < 24; ++j) out[t * 72 + j] = w[j];
  }
  for (int e = 1; e <= 2; ++e) {
    double A[8], B[8], H[16], L[16];
    int64_t col[17];
    to49(A, a);
    to49(B, b);
    if (e == 1) mul_fp49(H, L, A, B);
    else mul_fp49k(col, A, B);
    // value = sum_k (H_k + L_k) 2^(49 k), H_k a multiple of 2^49: column k = H_k / 2^49 (as 2^49 units of
    // column k + 1) + L_k (signed); fp49k: the int64 columns
    __int128 c = 0;
    unsigned __int128 buf = 0;
    int bit = 0, wi = 0;
    uint32_t w[25] = {0};
    for (int k = 0; k < 17; ++k) {
      if (e == 2) c += (__int128)col[k];
      if (e == 1 && k < 16) c += (__int128)(long long)L[k];
      if (e == 1 && k > 0) c += (__int128)(long long)(H[k - 1] / TWO49);
      const uint64_t limb = (uint64_t)(c & (((__int128)1 << 49) - 1));
      c >>= 49;  // arithmetic: c is non-negative once the column is complete (the value is)
      buf |= (unsigned __int128)limb << bit;
      bit += 49;
      while (bit >= 32 && wi < 25) { w[wi++] = (uint32_t)buf; buf >>= 32; bit -= 32; }
    }
    while (wi < 24) { w[wi++] = (uint32_t)buf; buf >>= 32; }
    for (int j = 0; j < 24; ++j) out[t * 72 + 24 * e + j] = w[j];
  }
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int simds = 4 * cus, N = 4096;
  uint32_t* h_in = (uint32_t*)malloc((size_t)N * 24 * 4);
  uint64_t s = 0x243F6A8885A308D3ull;
  for (int i = 0; i < N * 24; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h_in[i] = (uint32_t)(s >> 32);
  }
  for (int i = 0; i < N; ++i)  // operands < 2p < 2^382 (edge rows: all ones below 2^382)
    for (int h = 0; h < 2; ++h) {
      uint32_t* w = h_in + i * 24 + 12 * h;
      if (i < 8) for (int j = 0; j < 12; ++j) w[j] = 0xFFFFFFFFu;
      w[11] &= 0x3FFFFFFFu;
    }
  uint32_t *d_in, *d_chk;
  uint64_t* d_out;
  hipMalloc(&d_in, (size_t)N * 24 * 4);
  hipMalloc(&d_chk, (size_t)N * 72 * 4);
  hipMalloc(&d_out, (size_t)8 * simds * 64 * 8);
  hipMemcpy(d_in, h_in, (size_t)N * 24 * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_check, dim3(N / 64), dim3(64), 0, 0, d_in, d_chk, N);
  uint32_t* h_chk = (uint32_t*)malloc((size_t)N * 72 * 4);
  hipMemcpy(h_chk, d_chk, (size_t)N * 72 * 4, hipMemcpyDeviceToHost);
  int bad1 = 0, bad2 = 0;
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < 24; ++j) {
      bad1 += h_chk[i * 72 + j] != h_chk[i * 72 + 24 + j];
      bad2 += h_chk[i * 72 + j] != h_chk[i * 72 + 48 + j];
    }
  printf("# fp64bench: %d CUs; check over %d operand pairs (< 2^382): fp49 %s (%d word mismatches), fp49k %s (%d)\n", cus, N,
         bad1 ? "NOT bit-exact" : "bit-exact", bad1, bad2 ? "NOT bit-exact" : "bit-exact", bad2);
  printf("# engine  W | wall ms | SIMD cycles per 381x381 product @2.4GHz (a wave = 64 products)\n");
  struct K { const char* name; void (*f)(const uint32_t*, uint64_t*); };
  const K ks[] = {{"int28 ", k_bench<0>}, {"fp49  ", k_bench<1>}, {"fp49k ", k_bench<2>}};
  hipEvent_t ea, eb;
  hipEventCreate(&ea);
  hipEventCreate(&eb);
  for (const K& k : ks)
    for (int W : {1, 2, 3, 4, 8}) {
      const int blocks = simds * W;
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, d_in, d_out);
      hipDeviceSynchronize();
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(ea);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, d_in, d_out);
        hipEventRecord(eb);
        hipEventSynchronize(eb);
        float ms;
        hipEventElapsedTime(&ms, ea, eb);
        if (ms < best) best = ms;
      }
      printf("%s %d | %7.3f | %8.1f\n", k.name, W, best, best * 1e-3 * 2.4e9 / ((double)ITER * W));
      fflush(stdout);
    }
  return (bad1 || bad2) ? 1 : 0;
}
