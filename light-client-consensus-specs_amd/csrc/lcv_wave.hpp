// lcv_wave.hpp — wave-cooperative limb-form Montgomery products (R = 2^392) for the square-root chains of the
// latency-mode twins (lcv_k_lat.hip: one SSWU map / one signature per 64-lane wave, LCV_POW_LF 3).
//
// A lone lane runs a chain product as ~300 dependent instructions (84 multiply-adds, the 196 of the
// reduction and its 14-step quotient chain).  Here the wave holds a value with limb l (< 2^29) in lane l
// (lanes 14..63: 0) and one product is
//   columns   lane k accumulates column k = sum_j a_j b_(k-j): a_j broadcast from lane j (v_readlane), b
//             moved up one lane per step (DPP wave_shr:1) — 14 multiply-adds per lane;
//   quotient  the column vector's low 14 lanes, partly normalised (two carry rounds: limbs < 2^28 + 2^9,
//             value kept), times -p^-1 mod 2^392 (a per-lane table of its limbs shifted by j), truncated to
//             lanes 0..13 and partly normalised again: q = T (-p^-1) mod 2^392, 14 multiply-adds;
//   reduction T + q p (a per-lane table of p's limbs shifted by j: 14 multiply-adds), two carry rounds; the
//             low 392 bits are then zero, and the carry they still hold into lane 14 is (v_13 + [any of
//             v_0..v_12 nonzero]) >> 28 (a ballot: the low lanes sum to a multiple of 2^392 with every lane
//             below 2^28 + 2^9); lanes 14..27 move down to 0..13 (ds_bpermute).
// The result (T + q p) / 2^392 < 4p^2 / 2^392 + p (1 + 2^-19) < 1.01 p for operands < 2p, so the chain never
// leaves the limb form; its limbs stay below 2^28 + 2^9, its columns below 2^62.  Every lane of the wave
// must call these functions together with the same operands (the twins run one item per wave: all lanes
// compute the same item), so the exponent's branches are wave-uniform.  Device-only.
#pragma once
#include "lcv_col28.hpp"

#if defined(__HIP_DEVICE_COMPILE__)
namespace lcv {

struct WaveTabs {
  uint32_t pn[14];  // lane l: p_(l-j), 0 outside 0 <= l - j < 14
  uint32_t pq[14];  // lane l < 14: (-p^-1 mod 2^392)_(l-j), 0 for l < j and for l >= 14
};

LCV_FN uint32_t wv_lane() { return __lane_id(); }
// lane l <- lane l - 1, lane 0 <- 0 (DPP wave_shr:1, row and bank masks full)
LCV_FN uint32_t wv_shr1(uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, false); }
LCV_FN uint32_t wv_rd(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }

LCV_FN void wv_tabs(WaveTabs& T) {
  constexpr uint32_t NQ[14] = LCV_NP392_L28_INIT;
  const uint32_t l = wv_lane();
  uint32_t p = 0, q = 0;
  LCV_UNROLL for (int i = 0; i < 14; ++i) {
    p = l == (uint32_t)i ? kP28.v[i] : p;
    q = l == (uint32_t)i ? NQ[i] : q;
  }
  T.pn[0] = p;
  T.pq[0] = q;
  const uint32_t lo = l < 14u ? 0xFFFFFFFFu : 0u;
  LCV_UNROLL for (int j = 1; j < 14; ++j) {
    T.pn[j] = wv_shr1(T.pn[j - 1]);
    T.pq[j] = wv_shr1(T.pq[j - 1]) & lo;
  }
}

// two carry rounds over the whole wave (value kept): columns < 2^63 -> limbs < 2^28 + 2^9
LCV_FN uint32_t wv_norm(uint64_t c) {
  const uint64_t cy = c >> 28;
  const uint64_t up = ((uint64_t)wv_shr1((uint32_t)(cy >> 32)) << 32) | wv_shr1((uint32_t)cy);
  const uint64_t v = (c & SOP_M28) + up;
  return ((uint32_t)v & SOP_M28) + wv_shr1((uint32_t)(v >> 28));
}

// a b / 2^392 mod p (< 1.01 p for a, b < 2p; see above), one value per wave.  The column passes issue back to
// back (the compiler folds the two accumulators into one chain; kept apart they measured 1-5 % slower: the wave
// is bound by instruction issue, not by the multiply-add latency)
LCV_FN uint32_t wv_mul(uint32_t a, uint32_t b, const WaveTabs& T) {
  const uint32_t l = wv_lane();
  uint32_t s[14];
  LCV_UNROLL for (int j = 0; j < 14; ++j) s[j] = wv_rd(a, j);
  uint64_t c0 = 0, c1 = 0;
  uint32_t bs = b;
  LCV_UNROLL for (int j = 0; j < 14; ++j) {
    if (j & 1) c1 += (uint64_t)s[j] * bs;
    else c0 += (uint64_t)s[j] * bs;
    if (j < 13) bs = wv_shr1(bs);
  }
  const uint32_t t = wv_norm(c0 + c1);
  LCV_UNROLL for (int j = 0; j < 14; ++j) s[j] = wv_rd(t, j);
  c0 = 0;
  c1 = 0;
  LCV_UNROLL for (int j = 0; j < 14; ++j) {
    if (j & 1) c1 += (uint64_t)s[j] * T.pq[j];
    else c0 += (uint64_t)s[j] * T.pq[j];
  }
  const uint32_t q = wv_norm(c0 + c1) & (l < 14u ? 0xFFFFFFFFu : 0u);  // mod 2^392
  LCV_UNROLL for (int j = 0; j < 14; ++j) s[j] = wv_rd(q, j);
  c0 = t;
  c1 = 0;
  LCV_UNROLL for (int j = 0; j < 14; ++j) {
    if (j & 1) c1 += (uint64_t)s[j] * T.pn[j];
    else c0 += (uint64_t)s[j] * T.pn[j];
  }
  uint32_t v = wv_norm(c0 + c1);
  const uint64_t nz = __builtin_amdgcn_ballot_w64(l < 13u && v != 0u);
  const uint32_t m = (wv_rd(v, 13) + (nz != 0 ? 1u : 0u)) >> 28;
  v += l == 14u ? m : 0u;
  const uint32_t r = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((l + 14u) << 2), (int)v);
  return l < 14u ? r : 0u;
}

// uniform 14-limb value (every lane the same) <-> the wave layout
LCV_FN uint32_t wv_scatter(const uint32_t L[14]) {
  const uint32_t l = wv_lane();
  uint32_t x = 0;
  LCV_UNROLL for (int i = 0; i < 14; ++i) x = l == (uint32_t)i ? L[i] : x;
  return x;
}
LCV_FN void wv_gather(uint32_t L[14], uint32_t x) {  // normalised 28-bit limbs (the value is < 2^392)
  uint32_t c = 0;
  LCV_UNROLL for (int i = 0; i < 14; ++i) {
    const uint32_t v = wv_rd(x, i) + c;
    L[i] = v & SOP_M28;
    c = v >> 28;
  }
}

}  // namespace lcv
#endif
