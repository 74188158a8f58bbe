// rowtest.hip — unit check of the fan engine's row tail (lcv_sop_row.hpp) against the one-lane tail it replaces:
// for random ops (the column sums of up to four products of values < p, up to two add-in terms of random sign and
// magnitude, the header's reduction bound, a shadow), each 16-lane row runs rw_redc_limbs / rw_value / rw_store and
// the row's lane 0 runs sop_redc28 / sop_addin_apply / sop_reduce / sop_store_neg on the same op; the host compares
// r (after the reduction), v (after add-ins and reduction) and the stored value and shadow word for word and prints
// the mismatch count of each stage (all zero = the row tail is sop_tail_value + sop_tail_store bit for bit).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../light-client-consensus-specs_amd/csrc \
//         -I../../light-client-consensus-specs_amd/build rowtest.hip -o rowtest
#define LCV_HD __device__
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "lcv_sop_row.hpp"

struct Op {
  uint32_t x[8][12], y[8][12], m[8], u[2][12];
  uint32_t nk, nadd, a0, a1, red, shadow;
};
// per op: r (13), v (12), stored (12), shadow (12) from the row; the same from the lane reference
enum { OUTW = 13 + 12 + 12 + 12 };

__device__ void cols_of(uint64_t col[28], const Op& op) {
  for (int c = 0; c < 28; ++c) col[c] = 0;
  for (uint32_t k = 0; k < op.nk; ++k) {
    uint32_t X[15], Y[14], xw[13];
    uint32_t carry = 0;
    for (int q = 0; q < 12; ++q) {  // m X (< 2^392): 13 words
      const uint64_t t = (uint64_t)op.x[k][q] * op.m[k] + carry;
      xw[q] = (uint32_t)t;
      carry = (uint32_t)(t >> 32);
    }
    xw[12] = carry;
    lcv::sop_to28<13, 14>(X, xw);
    lcv::sop_to28<12, 14>(Y, op.y[k]);
    X[14] = 0;
    uint64_t p0[13], p2[13], c1[28];
    int64_t pd[13];
    lcv::sop_kara_mac<true>(p0, p2, pd, X, Y);
    lcv::sop_kara_join(c1, p0, p2, pd);
    for (int c = 0; c < 28; ++c) col[c] += c1[c];
  }
}

__global__ __launch_bounds__(64) void k_rowtest(const Op* ops, uint32_t nops, uint32_t* out_row, uint32_t* out_ref) {
  __shared__ uint64_t acc[4][28];
  __shared__ uint32_t val[4][2][12];
  __shared__ uint32_t wr[4][2][12];
  const uint32_t L = threadIdx.x, row = L >> 4, j = L & 15u;
  const uint32_t id = blockIdx.x * 4 + row;
  const bool live = id < nops;
  const Op* op = ops + (live ? id : 0);
  if (j == 0) {
    uint64_t col[28];
    cols_of(col, *op);
    for (int c = 0; c < 28; ++c) acc[row][c] = col[c];
    for (int q = 0; q < 12; ++q) { val[row][0][q] = op->u[0][q]; val[row][1][q] = op->u[1][q]; }
    for (int q = 0; q < 12; ++q) wr[row][0][q] = wr[row][1][q] = 0xDEADBEEFu;
  }
  __syncthreads();
  lcv::RowTabs T;
  lcv::rw_tabs(T);
  // the row's tail
  const uint32_t nadd = op->nadd, red = op->red;
  const uint32_t tl0 = nadd > 0 ? lcv::rw_limb(val[row][0]) : 0u, tl1 = nadd > 1 ? lcv::rw_limb(val[row][1]) : 0u;
  uint32_t rl = 0;
  if (op->nk) {
    const uint64_t lo = j < 14u ? acc[row][j] : 0ull, hi = j < 14u ? acc[row][j + 14] : 0ull;
    rl = lcv::rw_redc_limbs(lo, hi, T);
  }
  const uint32_t vl = lcv::rw_value(rl, nadd, op->a0, op->a1, tl0, tl1, red, T);
  const uint32_t h0 = op->shadow ? (1u << 13) : 0u;
  // dst slot 0, shadow slot 1 (of wr[row]); every 8th op has no dst (a padding op: nothing stored, its shadow
  // word 0 must not be taken for a slot)
  const bool none = id % 8 == 6;
  const uint32_t r0 = none ? (uint32_t)lcv::SOP_SLOT_NONE : 0u, r1 = none ? 0u : 1u << 12;
  uint32_t rw[13], vw[13];
  lcv::rw_gather(rw, lcv::rw_word(lcv::rw_norm_exact(rl)));  // (rl: partly normalised limbs)
  lcv::rw_gather(vw, lcv::rw_word(vl));
  lcv::rw_store(vl, h0, r0, r1, &wr[row][0][0], T);
  __syncthreads();
  if (j == 0 && live) {
    uint32_t* o = out_row + (size_t)id * OUTW;
    for (int q = 0; q < 13; ++q) o[q] = rw[q];
    for (int q = 0; q < 12; ++q) o[13 + q] = vw[q];
    for (int q = 0; q < 12; ++q) o[25 + q] = wr[row][0][q];
    for (int q = 0; q < 12; ++q) o[37 + q] = wr[row][1][q];
    // the lane reference
    uint64_t col[28];
    cols_of(col, *op);
    uint32_t r[13];
    if (op->nk) lcv::sop_redc28(r, col);
    else for (int q = 0; q < 13; ++q) r[q] = 0;
    uint32_t* e = out_ref + (size_t)id * OUTW;
    for (int q = 0; q < 13; ++q) e[q] = r[q];
    for (uint32_t a = 0; a < nadd; ++a) {
      uint32_t t[12];
      for (int q = 0; q < 12; ++q) t[q] = op->u[a][q];
      lcv::sop_addin_apply(r, a ? op->a1 : op->a0, t);
    }
    lcv::sop_reduce(r, red, nullptr);
    for (int q = 0; q < 12; ++q) e[13 + q] = r[q];
    const bool none = id % 8 == 6;
    for (int q = 0; q < 12; ++q) e[25 + q] = none ? 0xDEADBEEFu : r[q];
    uint32_t neg[12];
    for (int q = 0; q < 12; ++q) neg[q] = 0xDEADBEEFu;
    if (op->shadow && !none) lcv::sop_store_neg(neg, r);
    for (int q = 0; q < 12; ++q) e[37 + q] = neg[q];
  }
}

static const uint32_t PW[12] = {0xffffaaab, 0xb9feffff, 0xb153ffff, 0x1eabfffe, 0xf6b0f624, 0x6730d2a0,
                                0xf38512bf, 0x64774b84, 0x434bacd7, 0x4b1ba7b6, 0x397fe69a, 0x1a0111ea};
static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
  return (uint32_t)(rng >> 11);
}
static bool lt_p(const uint32_t* v) {
  for (int q = 11; q >= 0; --q) if (v[q] != PW[q]) return v[q] < PW[q];
  return false;
}
static void rnd_fp(uint32_t* v, int kind) {
  do {
    for (int q = 0; q < 12; ++q) v[q] = rnd();
    v[11] &= 0x1FFFFFFFu;
    if (kind == 1) for (int q = 0; q < 12; ++q) v[q] = q < 11 ? PW[q] : PW[q];  // p itself -> fixed below
    if (kind == 1) v[0] -= 1 + (rnd() & 7);  // p - small
    if (kind == 2) { for (int q = 1; q < 12; ++q) v[q] = 0; v[0] &= 7; }  // small
  } while (!lt_p(v));
}

int main() {
  const uint32_t N = 1 << 14;
  Op* h = (Op*)calloc(N, sizeof(Op));
  for (uint32_t i = 0; i < N; ++i) {
    Op& op = h[i];
    const int kind = (i % 16 == 3) ? 1 : (i % 16 == 7) ? 2 : 0;
    const bool big = i % 2 == 1;  // m-scaled products, up to 8 of them: r' up to ~2^10 p
    op.nk = i % 8 == 5 ? 0 : 1 + rnd() % (big ? 8 : 4);
    uint32_t mmax = 0;
    for (int k = 0; k < 8; ++k) {
      rnd_fp(op.x[k], kind);
      rnd_fp(op.y[k], (i % 16 == 11) ? 1 : kind);
      op.m[k] = big ? 1 + rnd() % 1024 : 1;
      if ((uint32_t)k < op.nk && op.m[k] > mmax) mmax = op.m[k];
    }
    op.nadd = rnd() % 3;
    uint32_t mags = 0;
    uint32_t a[2];
    for (int t = 0; t < 2; ++t) {
      rnd_fp(op.u[t], (i % 5 == 1) ? 1 : (i % 5 == 2) ? 2 : 0);
      int c = 1 + rnd() % (i % 3 == 0 ? 3 : 40);
      if (rnd() & 1) c = -c;
      a[t] = (uint32_t)t | ((uint32_t)(uint16_t)(int16_t)c << 16);
      if ((uint32_t)t < op.nadd) mags += (uint32_t)(c < 0 ? -c : c);
    }
    op.a0 = a[0];
    op.a1 = a[1];
    // r' < T / 2^384 + p < (nk m p / 2^384 + 1) p < (nk m / 8 + 1) p; the add-ins add below mags p
    uint32_t red = 0;
    while ((1u << red) < 2 + op.nk * mmax / 8 + mags) ++red;
    op.red = (i % 4 == 0) ? red + (rnd() % 3) : red;
    op.shadow = rnd() & 1;
  }
  Op* d;
  uint32_t *orow, *oref;
  (void)hipMalloc(&d, N * sizeof(Op));
  (void)hipMalloc(&orow, N * OUTW * 4);
  (void)hipMalloc(&oref, N * OUTW * 4);
  (void)hipMemcpy(d, h, N * sizeof(Op), hipMemcpyHostToDevice);
  k_rowtest<<<N / 4, 64>>>(d, N, orow, oref);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
  uint32_t* a = (uint32_t*)malloc(N * OUTW * 4);
  uint32_t* b = (uint32_t*)malloc(N * OUTW * 4);
  (void)hipMemcpy(a, orow, N * OUTW * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b, oref, N * OUTW * 4, hipMemcpyDeviceToHost);
  const char* stage[4] = {"redc r", "value v", "store", "shadow"};
  const int lo[4] = {0, 13, 25, 37}, hi[4] = {13, 25, 37, 49};
  int bad_total = 0;
  for (int s = 0; s < 4; ++s) {
    int bad = 0, first = -1;
    for (uint32_t i = 0; i < N; ++i)
      for (int q = lo[s]; q < hi[s]; ++q)
        if (a[i * OUTW + q] != b[i * OUTW + q]) { if (first < 0) first = (int)i; ++bad; break; }
    printf("%-8s: %d of %u ops differ", stage[s], bad, N);
    if (first >= 0) {
      const Op& op = h[first];
      printf("  (first: op %d nk %u nadd %u a0 %08x a1 %08x red %u shadow %u)\n   row:", first, op.nk, op.nadd, op.a0,
             op.a1, op.red, op.shadow);
      for (int q = lo[s]; q < hi[s]; ++q) printf(" %08x", a[first * OUTW + q]);
      printf("\n   ref:");
      for (int q = lo[s]; q < hi[s]; ++q) printf(" %08x", b[first * OUTW + q]);
    }
    printf("\n");
    bad_total += bad;
  }
  printf("rowtest: %s\n", bad_total ? "MISMATCH" : "bit-exact");
  return bad_total ? 1 : 0;
}
