// lcv_sha.hpp — SHA-256 (FIPS 180-4) on 32-bit VALU words + SSZ merkleization helpers.
//
// A 32-byte SSZ chunk / root is carried as 8 big-endian words (`h256`), so hashing a node pair
// is one 16-word block plus the constant padding block of a 64-byte message (whose message
// schedule the compiler folds at compile time).  Used by `hash_tree_root`, `is_valid_merkle_branch`,
// `compute_domain`/`compute_signing_root` (reference sync-protocol.md:191,212,234,354-362,427-449,
// 460-463) and by expand_message_xmd inside hash_to_G2.
#pragma once
#include "lcv_common.hpp"
#include "lcv_consts.inc"

namespace lcv {

struct h256 { uint32_t w[8]; };

LCV_FN uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

LCV_FN void sha256_compress(uint32_t st[8], const uint32_t blk[16]) {
  LCV_COUNT(2);
  constexpr uint32_t K[64] = LCV_SHA_K_INIT;
  uint32_t w[16];
  LCV_UNROLL for (int t = 0; t < 16; ++t) w[t] = blk[t];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  LCV_UNROLL for (int t = 0; t < 64; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
      w[t & 15] = wt;
    }
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + K[t] + wt;
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + maj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

LCV_FN void sha256_iv(uint32_t st[8]) {
  constexpr uint32_t IV[8] = LCV_SHA_IV_INIT;
  LCV_UNROLL for (int i = 0; i < 8; ++i) st[i] = IV[i];
}

// H(x || y) — SSZ node hash
#ifndef LCV_SHA_CALL
#define LCV_SHA_CALL 0
#endif
#if LCV_SHA_CALL && defined(__HIP_DEVICE_COMPILE__)
// LCV_SHA_CALL=1: one out-of-line node hash per kernel (16 scalar words in, 8 out in registers), so a
// kernel with many hash sites keeps one copy of the two unrolled compressions (register pressure).
__device__ __noinline__ h256 hash_pair_call(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, uint32_t x4,
                                            uint32_t x5, uint32_t x6, uint32_t x7, uint32_t y0, uint32_t y1,
                                            uint32_t y2, uint32_t y3, uint32_t y4, uint32_t y5, uint32_t y6,
                                            uint32_t y7) {
  uint32_t st[8];
  sha256_iv(st);
  const uint32_t blk[16] = {x0, x1, x2, x3, x4, x5, x6, x7, y0, y1, y2, y3, y4, y5, y6, y7};
  sha256_compress(st, blk);
  uint32_t pad[16];
  pad[0] = 0x80000000u;
  LCV_UNROLL for (int i = 1; i < 15; ++i) pad[i] = 0;
  pad[15] = 512;
  sha256_compress(st, pad);
  h256 out;
  LCV_UNROLL for (int i = 0; i < 8; ++i) out.w[i] = st[i];
  return out;
}
LCV_FN void hash_pair(h256& out, const h256& x, const h256& y) {
  out = hash_pair_call(x.w[0], x.w[1], x.w[2], x.w[3], x.w[4], x.w[5], x.w[6], x.w[7], y.w[0], y.w[1], y.w[2],
                       y.w[3], y.w[4], y.w[5], y.w[6], y.w[7]);
}
#else
LCV_FN void hash_pair(h256& out, const h256& x, const h256& y) {
  uint32_t st[8];
  sha256_iv(st);
  uint32_t blk[16];
  LCV_UNROLL for (int i = 0; i < 8; ++i) { blk[i] = x.w[i]; blk[8 + i] = y.w[i]; }
  sha256_compress(st, blk);
  uint32_t pad[16];
  pad[0] = 0x80000000u;
  LCV_UNROLL for (int i = 1; i < 15; ++i) pad[i] = 0;
  pad[15] = 512;
  sha256_compress(st, pad);
  LCV_UNROLL for (int i = 0; i < 8; ++i) out.w[i] = st[i];
}
#endif

LCV_FN void h256_zero(h256& r) { LCV_UNROLL for (int i = 0; i < 8; ++i) r.w[i] = 0; }
LCV_FN bool h256_is_zero(const h256& a) {
  uint32_t x = 0;
  LCV_UNROLL for (int i = 0; i < 8; ++i) x |= a.w[i];
  return x == 0;
}
LCV_FN bool h256_eq(const h256& a, const h256& b) {
  uint32_t x = 0;
  LCV_UNROLL for (int i = 0; i < 8; ++i) x |= a.w[i] ^ b.w[i];
  return x == 0;
}
// zero_hash(d) = root of a depth-d all-zero subtree
LCV_FN void zero_hash(h256& r, int d) {
  constexpr uint32_t ZH[16][8] = LCV_ZERO_HASHES_INIT;
  LCV_UNROLL for (int i = 0; i < 8; ++i) r.w[i] = ZH[d][i];
}

// ---- loads: raw little-endian byte records in global memory -> chunk words
LCV_FN void ld_chunk(h256& r, const uint8_t* p) {  // 32 bytes, 4-byte aligned
  LCV_UNROLL for (int i = 0; i < 8; ++i) r.w[i] = bswap32(*(const uint32_t*)(p + 4 * i));
}
LCV_FN void st_chunk(uint8_t* p, const h256& r) {
  LCV_UNROLL for (int i = 0; i < 8; ++i) *(uint32_t*)(p + 4 * i) = bswap32(r.w[i]);
}
// uint64 SSZ chunk: 8 little-endian bytes then zeros
LCV_FN void u64_chunk(h256& r, uint64_t v) {
  h256_zero(r);
  r.w[0] = bswap32((uint32_t)v);
  r.w[1] = bswap32((uint32_t)(v >> 32));
}

// is_valid_merkle_branch (phase0): fold `depth` hashes, side chosen by the bits of `index`
LCV_FN bool merkle_branch_ok(const h256& leaf, const uint8_t* branch, int depth, uint64_t index, const h256& root) {
  h256 v = leaf;
  for (int i = 0; i < depth; ++i) {
    h256 b;
    ld_chunk(b, branch + 32 * i);
    if ((index >> i) & 1u) hash_pair(v, b, v);
    else hash_pair(v, v, b);
  }
  return h256_eq(v, root);
}

LCV_FN bool bytes_all_zero(const uint8_t* p, int n4) {  // n4 = number of 32-bit words
  uint32_t x = 0;
  for (int i = 0; i < n4; ++i) x |= ((const uint32_t*)p)[i];
  return x == 0;
}

}  // namespace lcv
