// lcv_sop_row.hpp — the fan engine's Montgomery reduction spread over a row of 16 lanes (latency mode,
// lcv_functors_sop.hpp k_sop_fan with LCV_FAN_ROW): one op's 28 column sums, lane j holding columns j and
// j + 14, instead of one lane running sop_redc28's 196 multiply-adds back to back.
//
// A lone wave is bound by instruction issue in sop_redc28 (4.2-4.8 shader cycles per wave64 instruction at one wave
// per SIMD, DPP moves and 64-bit multiply-adds alike, chained or not: tools/microbench/dppbench.hip; 1,850 of a
// final-exponentiation round's ~7,000 cycles, profiles/r06_ab/tail_timing_A.txt), so the row form cuts the
// instructions on the tail's wave: per lane
//   t  = T mod 2^392, partly normalised (two carry rounds: limbs < 2^28 + 2^9, value kept);
//   M  = t (-p^-1) mod 2^384 as a column pass (14 row broadcasts + multiply-adds), normalised exactly and cut
//        to 384 bits: the canonical Montgomery quotient (M < 2^384, T + M p = 0 mod 2^384), the one
//        sop_redc28's digits spell;
//   T + M p as a second column pass (lane j: column j and column j + 14);
//   r' from the columns: the low half's carry across bit 384 is (u13 + [u0..u12 not all zero]) >> 20 (its low
//        384 bits are zero and every partly normalised limb is below 2^28 + 2^9), the high half after one carry
//        round moved up 8 bits (2^392 = 2^8 2^384) and carried once more.
// So r' = (T + M p) / 2^384 is sop_redc28's r as a value (limbs partly normalised); the rest of the op's tail runs on
// the row too (rw_value: the add-in terms, the quotient estimate from the top limbs, one exact normalisation — a
// carry round, then a carry-lookahead over two row ballots: generate = limb >= 2^28, propagate = limb 2^28 - 1;
// rw_store: the value's words and its shadow's, p - v by a borrow lookahead, one word per lane).  Bit for bit
// sop_tail_value + sop_tail_store:
// tools/microbench/rowtest.hip.  Row lanes 14 and 15 hold zeros (lane 14: a signed top limb in the tail's steps).
// Device-only (DPP row_newbcast / row_shr / row_shl within 16-lane rows, gfx90a+).
#pragma once
#include <utility>

#include "lcv_sop.hpp"  // (+ lcv_col28.hpp)

#if !defined(LCV_HOSTSIM)
namespace lcv {

template <int CTRL>
LCV_FN uint32_t rw_dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
template <int K> LCV_FN uint32_t rw_bcast(uint32_t x) { return rw_dpp<0x150 + K>(x); }  // lane j <- lane K
LCV_FN uint32_t rw_shr1(uint32_t x) { return rw_dpp<0x111>(x); }                       // lane j <- lane j - 1
template <int K> LCV_FN uint32_t rw_shl(uint32_t x) { return rw_dpp<0x100 + K>(x); }     // lane j <- lane j + K
LCV_FN uint64_t rw_shr1_64(uint64_t x) {
  return ((uint64_t)rw_shr1((uint32_t)(x >> 32)) << 32) | rw_shr1((uint32_t)x);
}
template <int... I, class Fn>
LCV_FN void rw_for(std::integer_sequence<int, I...>, Fn&& fn) {
  (fn(std::integral_constant<int, I>{}), ...);
}
#define LCV_RW_FOR(N, body) rw_for(std::make_integer_sequence<int, N>{}, [&](auto I_) { constexpr int I = decltype(I_)::value; body; })

LCV_FN uint32_t rw_j() { return __lane_id() & 15u; }

// per-lane tables (lane j of a row): nq[i] = n_(j-i) for i <= j < 14 (n = -p^-1 mod 2^392, 28-bit limbs);
// pl[i] = p_(j-i) for i <= j < 14; ph[i] = p_(j+14-i) for j < i (the column pass's low / high column terms)
struct RowTabs { uint32_t nq[14], pl[14], ph[14], pj, pw; };  // pj: p's limb j (0 on lanes 14, 15); pw: p's word j
LCV_FN void rw_tabs(RowTabs& T) {
  constexpr uint32_t NQ[14] = LCV_NP392_L28_INIT;
  constexpr uint32_t PW[12] = LCV_P_INIT;
  const uint32_t j = rw_j();
  uint32_t n = 0, p = 0, w = 0;
  LCV_UNROLL for (int i = 0; i < 14; ++i) {
    n = j == (uint32_t)i ? NQ[i] : n;
    p = j == (uint32_t)i ? kP28.v[i] : p;
    if (i < 12) w = j == (uint32_t)i ? PW[i] : w;
  }
  T.pw = w;
  const uint32_t lo = j < 14u ? 0xFFFFFFFFu : 0u;
  T.pj = p;
  T.nq[0] = n;
  T.pl[0] = p;
  LCV_UNROLL for (int i = 1; i < 14; ++i) {
    T.nq[i] = rw_shr1(T.nq[i - 1]) & lo;
    T.pl[i] = rw_shr1(T.pl[i - 1]) & lo;
  }
  // ph[i] on lane j < i: p_(j + 14 - i), i.e. p shifted down by 14 - i lanes
  T.ph[0] = 0;
  LCV_RW_FOR(13, { T.ph[I + 1] = rw_shl<13 - I>(p) & (j < (uint32_t)(I + 1) ? 0xFFFFFFFFu : 0u); });
}

// two carry rounds over the row (unsigned; the value over the 16 lanes is kept while lane 15 carries nothing
// out): limbs < 2^64 -> < 2^28 + 2^9
LCV_FN uint64_t rw_norm2(uint64_t x) {
  LCV_UNROLL for (int k = 0; k < 2; ++k) x = (x & SOP_M28) + rw_shr1_64(x >> 28);
  return x;
}
// the row's 16 bits of a wave ballot
LCV_FN uint32_t rw_bits(uint64_t ballot) { return (uint32_t)(ballot >> (__lane_id() & 48u)) & 0xFFFFu; }
// exact normalisation of limbs below 2^29 - 1 (lanes 0..13; lanes 14, 15 zero): limb + carry-in stays below 2^29,
// so every carry is 0 or 1 and a lookahead resolves them at once: carry into lane j+1 = g_j | (p_j & carry_j) with
// g = (limb >= 2^28), p = (limb == 2^28 - 1) — the carries of the addition (G | P) + G
LCV_FN uint32_t rw_norm_exact(uint32_t x) {
  const uint32_t g = rw_bits(__builtin_amdgcn_ballot_w64(x > SOP_M28));
  const uint32_t pr = rw_bits(__builtin_amdgcn_ballot_w64(x == SOP_M28));
  const uint32_t a = g | pr, cin = ((a + g) ^ a ^ g) >> rw_j();
  return (x + (cin & 1u)) & SOP_M28;
}

// signed rows (the tail's add-in and reduction steps): lanes 0..13 hold non-negative limbs, lane 14 a signed top limb
// (it receives the bias terms' compensation, below) that is never masked and carries nothing on
// exact: lanes 0..13 in [0, 2^29 - 1) (non-negative limbs after a carry round, or a biased difference) become
// canonical, lane 14 (signed) receives their carry: the carry-lookahead of rw_norm_exact
LCV_FN int64_t rw_norm_exact_s(int64_t x) {
  const uint32_t j = rw_j();
  const bool low = j < 14u;
  const uint32_t g = rw_bits(__builtin_amdgcn_ballot_w64(low && x > (int64_t)SOP_M28));
  const uint32_t pr = rw_bits(__builtin_amdgcn_ballot_w64(low && x == (int64_t)SOP_M28));
  const uint32_t a = g | pr, cin = (((a + g) ^ a ^ g) >> j) & 1u;
  return low ? ((x + cin) & SOP_M28) : x + cin;
}
// u - v as limbs with a bias that keeps lanes 0..13 non-negative (limbs u_j, v_j in [0, 2^28), j < 14): lane j gets
// u_j - v_j + 2^28 [j < 14] - [1 <= j <= 14]; the biases cancel (sum of 2^(28 (j+1)) over j < 14 minus sum of 2^(28 j)
// over 1 <= j <= 14), so lane 14 ends at 0 when u >= v and at -1 when u < v, after rw_norm_exact_s
LCV_FN int64_t rw_biased_sub(uint32_t u, uint32_t v) {
  const uint32_t j = rw_j();
  return (int64_t)u - (int64_t)v + (j < 14u ? (int64_t)(1u << 28) : 0) - ((j >= 1u && j <= 14u) ? 1 : 0);
}
// 12-word value in LDS -> its limb j on lane j (lanes 14, 15: 0), in two steps so that the loads can be issued
// early and the limb cut out where it is used: rw_limb_words reads the two words that hold limb j
LCV_FN void rw_limb_words(const uint32_t* val, uint32_t& w0, uint32_t& w1) {
  const uint32_t j = rw_j();
  const uint32_t k = (28u * j) >> 5;
  w0 = j < 14u ? val[k] : 0u;
  w1 = j < 14u && k + 1u < 12u ? val[k + 1u] : 0u;
}
LCV_FN uint32_t rw_limb_of(uint32_t w0, uint32_t w1) {
  return (uint32_t)((((uint64_t)w1 << 32) | w0) >> ((28u * rw_j()) & 31u)) & SOP_M28;
}
LCV_FN uint32_t rw_limb(const uint32_t* val) {
  uint32_t w0, w1;
  rw_limb_words(val, w0, w1);
  return rw_limb_of(w0, w1);
}
// canonical limbs (lanes 0..13) -> word w on lane w < 13: limbs k, k + 1 with k = w + w / 7, shift 32 w mod 28
LCV_FN uint32_t rw_word(uint32_t L) {
  const uint32_t j = rw_j();
  const uint32_t a1 = rw_shl<1>(L), a2 = rw_shl<2>(L);
  const bool hiw = j >= 7u;
  const uint32_t x0 = hiw ? a1 : L, x1 = hiw ? a2 : a1;
  const uint32_t sh = hiw ? 4u * j - 28u : 4u * j;
  return (x0 >> sh) | (x1 << (28u - sh));  // 28 - sh in [4, 28]: two limbs cover the word
}
// the row's 13 words onto its lane 0
LCV_FN void rw_gather(uint32_t r[13], uint32_t word) {
  r[0] = word;
  LCV_RW_FOR(12, { r[I + 1] = rw_shl<I + 1>(word); });
}

// r = sop_redc28(T) as canonical limbs (limb j on lane j < 14) for the op whose column sums this row holds: lane
// j < 14 passes lo = column j and hi = column j + 14 (lanes 14, 15: 0); see the header for the value
LCV_FN uint32_t rw_redc_limbs(uint64_t lo, uint64_t hi, const RowTabs& T) {
  const uint32_t j = rw_j();
  // t = T mod 2^392 (lanes 0..13), the carries past lane 13 into columns 14 / 15 = hi's lanes 0 / 1
  uint64_t t = rw_norm2(lo);
  hi += rw_shl<14>((uint32_t)t);
  const uint32_t t32 = j < 14u ? (uint32_t)t : 0u;
  // M' = t n mod 2^392 (column k on lane k), two accumulators for the multiply-add chain
  uint64_t c0 = 0, c1 = 0;
  LCV_RW_FOR(14, {
    const uint32_t s = rw_bcast<I>(t32);
    if (I & 1) c1 += (uint64_t)s * T.nq[I];
    else c0 += (uint64_t)s * T.nq[I];
  });
  // exact M = T n mod 2^384 (canonical limbs, the top one 20 bits), so r' is sop_redc28's r itself
  uint32_t m = j < 14u ? (uint32_t)rw_norm2(c0 + c1) : 0u;
  m = rw_norm_exact(m);
  if (j == 13u) m &= 0xFFFFFu;
  // S = T + M' p: lane j accumulates column j (terms i <= j) and column j + 14 (terms i > j)
  uint64_t l0 = t32, l1 = 0, h0 = hi, h1 = 0;
  LCV_RW_FOR(14, {
    const uint32_t s = rw_bcast<I>(m);
    if (I & 1) { l1 += (uint64_t)s * T.pl[I]; h1 += (uint64_t)s * T.ph[I]; }
    else { l0 += (uint64_t)s * T.pl[I]; h0 += (uint64_t)s * T.ph[I]; }
  });
  // low half: its bits below 384 are zero; what crosses bit 384 is (u13 + e) >> 20 + u14 2^8 + u15 2^36
  const uint32_t u = (uint32_t)rw_norm2(l0 + l1);
  const uint32_t e = (rw_bits(__builtin_amdgcn_ballot_w64(j < 13u && u != 0u)) & 0x1FFFu) != 0u ? 1u : 0u;
  const uint32_t u13 = rw_bcast<13>(u), u14 = rw_bcast<14>(u), u15 = rw_bcast<15>(u);
  // high half (relative to 2^392): one carry round (limbs below 2^28 + 2^36), moved up 8 bits; r' < 2^391 and the
  // limbs are non-negative, so its lanes 14, 15 are zero
  const uint64_t hs = h0 + h1, hn = (hs & SOP_M28) + rw_shr1_64(hs >> 28);
  uint64_t R = hn << 8;
  if (j == 0) R += ((uint64_t)(u13 + e) >> 20) + ((uint64_t)u14 << 8);
  if (j == 1) R += (uint64_t)u15 << 8;
  // partly normalised by one carry round (R's limbs are below 2^45: lanes 0..13 end below 2^28 + 2^17; lanes 14, 15
  // zero: the limbs are non-negative and r' < 2^391); rw_value normalises exactly once, after the add-ins and the
  // reduction
  return (uint32_t)((R & SOP_M28) + rw_shr1_64(R >> 28));
}

// The rest of the op's tail on its row: from r's limbs (lanes 0..13 in [0, 2^28 + 2^17), rw_redc_limbs) to
// v = (r + sum |c| u) mod p canonical, the value sop_tail_value stores (u = the add-in slot's value, or p - it for
// c < 0; the terms' limbs tl0 / tl1 were read from LDS at the top of the round).  The terms are multiply-adds per
// lane (a negative one as |c| times the biased p - u).  For red > 0 (x < 2^red p, the header's bound) the quotient
// comes from x's limbs 11..14 as they stand — one carry round, no exact normalisation: the lanes below 11 add
// less than 2^309 to x, so top 2^308 / p is x / p to within 2^-71 — in FP64 with sop_reduce's margin (q or q - 1)
// and its exactness test (a fractional part of e at most 1 - 2^-29 proves q exact); x - q p (biased, lanes
// non-negative) is then normalised exactly once.  Only an inexact estimate (~2^-29 of the ops; row-uniform)
// takes the conditional subtraction of p, decided by the biased difference's lane 14.  v's limb on lane j.
LCV_FN int64_t rw_carry1s(int64_t x) {  // one carry round over lanes 0..13 into lane 14 (signed rows)
  const bool low = rw_j() < 14u;
  return (low ? (x & SOP_M28) : x) + (int64_t)rw_shr1_64(low ? (uint64_t)(x >> 28) : 0ull);
}
LCV_FN uint32_t rw_value(uint32_t rl, uint32_t nadd, uint32_t a0, uint32_t a1, uint32_t tl0, uint32_t tl1,
                         uint32_t red, const RowTabs& T) {
  const uint32_t j = rw_j();
  const uint32_t pj = T.pj;
  int64_t x = rl;
  if (nadd) {
    LCV_UNROLL for (int k = 0; k < 2; ++k) {
      if ((uint32_t)k < nadd) {
        const uint32_t a = k ? a1 : a0, t = k ? tl1 : tl0;
        const int c = (int)(int16_t)(a >> 16);
        const int64_t mag = c < 0 ? -c : c;
        x += mag * (c < 0 ? rw_biased_sub(pj, t) : (int64_t)t);
      }
    }
  }
  if (red) {
    if (nadd) x = rw_carry1s(x);  // lanes 0..13 below 2^28 + 2 (1 + sum |c|): 32-bit broadcasts
    const double top = (((double)(int32_t)rw_bcast<14>((uint32_t)x) * 268435456.0 +
                         (double)rw_bcast<13>((uint32_t)x)) * 268435456.0 + (double)rw_bcast<12>((uint32_t)x)) *
                           268435456.0 + (double)rw_bcast<11>((uint32_t)x);
    const double e = top * 0x1.3b06ba5e7993dp-73 - 0x1p-30;  // x / p from x's bits >= 308 (2^308 / p)
    const int qi = (int)e;
    int64_t q = qi > 0 ? qi : 0;
    bool exact = e - (double)qi <= 1.0 - 0x1p-29;  // e < 0: q = 0 and x < p, exact too
#ifdef LCV_RW_TEST_INEXACT  // rowtest only: every op takes the conditional subtraction, about half of them with
    // q - 1 (an exact q lowered by one: x - q p in [p, 2p))
    if (exact && q > 0 && (rw_bcast<0>((uint32_t)x) & 1u)) q -= 1;
    exact = false;
#endif
    int64_t y = x - q * (int64_t)pj + (j < 14u ? q << 28 : 0) - ((j >= 1u && j <= 14u) ? q : 0);
    y = rw_norm_exact_s(rw_carry1s(y));  // x - q p: in [0, p) when exact, else in [0, 2p) (limbs < 2^44: one round)
    if (__builtin_expect(!exact, 0)) {
      const int64_t z = rw_norm_exact_s(rw_biased_sub((uint32_t)y, pj));  // (biased limbs < 2^29)
      const bool ge = (int32_t)rw_bcast<14>((uint32_t)z) == 0;  // y >= p
      y = ge ? z : y;
    }
    x = y;
  } else if (nadd) {
    x = rw_norm_exact_s(rw_carry1s(x));  // (limbs below 2^28 + 2^17 + 2^29 sum |c| < 2^45: one round)
  } else {
    x = rw_norm_exact(rl);
  }
  return (uint32_t)x & (j < 14u ? 0xFFFFFFFFu : 0u);
}
// p - v as words (v < p, word w on lane w < 12; p's word from the table): per-word differences and a borrow
// lookahead over two row ballots — generate p_w < v_w, propagate p_w == v_w: the borrows are the carries of
// (G | P) + G, as in rw_norm_exact
LCV_FN uint32_t rw_neg_word(uint32_t vw, uint32_t pw) {
  const uint32_t j = rw_j();
  const bool act = j < 12u;
  const uint32_t g = rw_bits(__builtin_amdgcn_ballot_w64(act && pw < vw));
  const uint32_t pr = rw_bits(__builtin_amdgcn_ballot_w64(act && pw == vw));
  const uint32_t a = g | pr, bin = (((a + g) ^ a ^ g) >> j) & 1u;
  return pw - vw - bin;
}
// v's store on its row (sop_tail_store without side-loads / emits, which take the gathered path): lane w < 12
// writes word w of v to the destination slot and of p - v to its shadow; r0 / r1 are the op's record words 0 / 1
LCV_FN void rw_store(uint32_t vl, uint32_t h0, uint32_t r0, uint32_t r1, uint32_t* wr, const RowTabs& T) {
  const uint32_t j = rw_j();
  const uint32_t dst = r0 & 0xFFFu, dsh = (r1 >> 12) & 0x3FFu;
  if (dst == SOP_SLOT_NONE) return;  // (no op: its record's shadow word is not meaningful either)
  const uint32_t word = rw_word(vl);
  if (j < 12u) wr[12u * dst + j] = word;
  if (((h0 >> 13) & 1u) && dsh != 0x3FFu) {  // shadow: p - v in (0, p]
    const uint32_t sw = rw_neg_word(word, T.pw);
    if (j < 12u) wr[12u * dsh + j] = sw;
  }
}

}  // namespace lcv
#endif
