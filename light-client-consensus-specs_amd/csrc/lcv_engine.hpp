// lcv_engine.hpp — team interpreter for the generated pairing programs (tools/gen_programs.py ->
// lcv_programs.inc): the Miller loop of e(PK, H(m)) * e(-G1, sig) and the final exponentiation,
// i.e. the pairing check inside bls.FastAggregateVerify (reference call site sync-protocol.md:464).
//
// A program is a list of ROUNDS; in round r, lane t of an update's team (TEAM lanes, 64 / TEAM
// updates per wave) executes one op:  dst <- A * B (MUL), dst <- A^-1 (INV) or dst <- A (LIN), where
// A and B are signed small-coefficient combinations of Fp values held in the update's LDS slots (or
// in the constant table).  Every round reads only values written by earlier rounds (the generator's
// allocator guarantees it), so a barrier between rounds is the only synchronisation.  The Fp
// arithmetic is the same 12 x 32-bit Montgomery code as everywhere else (lcv_field.hpp).
//
// Encoding (uint16): round header [nA, nB, stride, used], then `used` entries of `stride` words:
//   dst | 0x1000 (MUL) | 0x2000 (INV),  nA terms,  nB terms;   term = slot | coef << 12 (4-bit signed)
// (header words 0/1: n | max|coef| << 8 | reduction bits << 11 | full << 14; slots >= nslots are constants)
#pragma once
#include "lcv_items.hpp"

namespace lcv {

enum { ENG_SLOT_NONE = 0xFFF, ENG_MUL = 0x1000, ENG_INV = 0x2000 };

struct ProgView {
  const uint16_t* words;
  const uint32_t* offs;
  const uint32_t* consts;  // 12 limbs per constant (Montgomery), copied into LDS slots nslots..
  uint32_t rounds;
  uint32_t nslots, nconst;
};

// prologue helper: the program's constants go to the block's shared LDS region `cl` (slot nslots + k
// is constant k); every team writes the same values, the round barrier publishes them
LCV_FN void eng_load_consts(const ProgView& P, uint32_t lane, uint32_t team, uint32_t* cl) {
  for (uint32_t k = lane; k < 12 * P.nconst; k += team) cl[k] = P.consts[k];
}

LCV_FN void eng_load(fp& v, const uint32_t* lds, uint32_t slot) {
  const uint32_t* src = lds + 12 * slot;
  LCV_UNROLL for (int k = 0; k < 12; ++k) v.v[k] = src[k];
}
LCV_FN void eng_store(uint32_t* lds, uint32_t slot, const fp& v) {
  uint32_t* dst = lds + 12 * slot;
  LCV_UNROLL for (int k = 0; k < 12; ++k) dst[k] = v.v[k];
}

// out = sum_k c_k * value(slot_k) (mod p).  Branch-free and uniform across the wave: the round
// header h gives n (terms), maxc (largest |c| in the round), k (2^k > sum |c|) and whether the
// result must be fully reduced (< p, LIN results are stored) or only <= 2p (a Montgomery operand:
// a, b <= 2p gives ab < R p and a result < 2p).  Each term adds |c| * v (c > 0) or |c| * (p - v)
// (c < 0, p - v in [1, p]) into an UNREDUCED 13-limb accumulator (< 2^k p <= 2^6 p), then
// conditional subtraction of 2^s p for s = k-1 .. (full ? 0 : 1).  |c| * v: masked repeated
// addition when maxc <= 2, else a v_mad_u64_u32 chain (cost independent of |c|).
LCV_FN void eng_eval(fp& out, const uint16_t* t, uint32_t h, const uint32_t* lds, const uint32_t* cl, uint32_t ns) {
  constexpr uint32_t PL[12] = LCV_P_INIT;
  const uint32_t n = h & 0xFFu, maxc = (h >> 8) & 7u, kb = (h >> 11) & 7u, lo = (h >> 14) & 1u ? 0u : 1u;
  uint32_t acc[13];
  LCV_UNROLL for (int j = 0; j < 13; ++j) acc[j] = 0;
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t w = t[k];
    uint32_t slot = w & 0xFFFu;
    int c = (int)(w >> 12);
    if (c >= 8) c -= 16;
    if (slot == ENG_SLOT_NONE) { slot = 0; c = 0; }
    const uint32_t* src = slot >= ns ? cl + 12 * (slot - ns) : lds + 12 * slot;
    uint32_t v[12], d[12];
    LCV_UNROLL for (int j = 0; j < 12; ++j) v[j] = src[j];
    uint32_t br = 0;
    LCV_UNROLL for (int j = 0; j < 12; ++j) d[j] = subc32(PL[j], v[j], br, br);  // d = p - v in [1, p]
    const uint32_t a = (uint32_t)(c < 0 ? -c : c);
    const bool neg = c < 0;
    LCV_UNROLL for (int j = 0; j < 12; ++j) v[j] = neg ? d[j] : v[j];  // v_cndmask
    if (maxc <= 2) {
      for (uint32_t rep = 0; rep < maxc; ++rep) {
        const uint32_t keep = rep < a ? 0xFFFFFFFFu : 0u;
        uint32_t cy = 0;
        LCV_UNROLL for (int j = 0; j < 12; ++j) acc[j] = addc32(acc[j], v[j] & keep, cy, cy);
        acc[12] += cy;
      }
    } else {
      uint32_t hi = 0, cy = 0;
      LCV_UNROLL for (int j = 0; j < 12; ++j) {
        const uint64_t pr = (uint64_t)v[j] * a + hi;  // < 2^35: one v_mad_u64_u32
        hi = (uint32_t)(pr >> 32);
        acc[j] = addc32(acc[j], (uint32_t)pr, cy, cy);
      }
      acc[12] += hi + cy;
    }
  }
  for (uint32_t s = kb; s-- > lo;) {  // acc < 2^kb p  ->  acc < 2^lo p
    uint32_t sp[13], d[13];
    uint32_t cy = 0;
    LCV_UNROLL for (int j = 0; j < 12; ++j) {  // sp = p << s
      sp[j] = (PL[j] << s) | cy;
      cy = s ? (PL[j] >> (32 - s)) : 0u;
    }
    sp[12] = cy;
    uint32_t br = 0;
    LCV_UNROLL for (int j = 0; j < 13; ++j) d[j] = subc32(acc[j], sp[j], br, br);
    LCV_UNROLL for (int j = 0; j < 13; ++j) acc[j] = br ? acc[j] : d[j];
  }
  LCV_UNROLL for (int j = 0; j < 12; ++j) out.v[j] = acc[j];
}

// one round of a program for lane `lane` of the team whose LDS slots start at `lds`
LCV_FN void eng_round(const ProgView& P, uint32_t r, uint32_t lane, uint32_t* lds, const uint32_t* cl) {
  const uint16_t* rp = P.words + P.offs[r];
  const uint32_t hA = rp[0], hB = rp[1], stride = rp[2], used = rp[3];
  const uint32_t nA = hA & 0xFFu;
  if (lane >= used) return;
  const uint16_t* e = rp + 4 + lane * stride;
  const uint32_t dst = e[0];
  fp a;
  eng_eval(a, e + 1, hA, lds, cl, P.nslots);
  if (dst & ENG_MUL) {
    fp b;
    eng_eval(b, e + 1 + nA, hB, lds, cl, P.nslots);
    fp_mul(a, a, b);
  } else if (dst & ENG_INV) {
    fp_inv_bingcd(a, a);
  }
  eng_store(lds, dst & 0xFFFu, a);
}

}  // namespace lcv

// ============================================================================ pairing stages
#include "lcv_programs.inc"

namespace lcv {

// fp2 coefficient g_i (of w^i) -> its fp2 slot in the SoA Fp12 layout of soa_st_fp12 (c0.c0, c0.c1,
// c0.c2, c1.c0, c1.c1, c1.c2 = g0, g2, g4, g1, g3, g5)
LCV_FN uint32_t fp12_soa_slot(uint32_t g) { return (g & 1u) ? 3u + (g >> 1) : (g >> 1); }

// Miller loop of both pairings.  Prologue (lane k < 12 loads input k): Q1 = H(m), Q2 = signature,
// P1 = aggregate pubkey, P2 = -G1; an identity Q_k becomes (Q_k = G2 generator, P_k = (0, 0)), whose
// lines are Fp2 constants killed by the final exponentiation (e(P, O) = 1).  Epilogue: f -> W.f.
// out of line: keeps the prologue's constants (G2 generator, -G1) from being hoisted into registers
// that would stay live across the whole round loop
LCV_OUTLINE void miller_prologue(uint32_t i, uint32_t lane, uint32_t* lds, const Work& W) {
  if (lane >= 12) return;
  const bool q1_id = W.qh_inf[i] != 0, q2_id = W.sig_status[i] != PT_OK;
  fp v;
  if (lane < 8) {
    const bool id = lane < 4 ? q1_id : q2_id;
    const uint32_t k = lane & 3u;
    if (id) {
      fp2 g;
      if (k < 2) LCV_FP2_SET(g, LCV_G2X);
      else LCV_FP2_SET(g, LCV_G2Y);
      v = (k & 1u) ? g.c1 : g.c0;
    } else {
      soa_ld_fp(v, lane < 4 ? W.qh : W.qs, W.cap, i, k);
    }
  } else if (lane < 10) {  // P1 = (-x, y) of the aggregate pubkey
    soa_ld_fp(v, W.pk, W.cap, i, lane - 8);
    if (lane == 8) fp_neg(v, v);
    if (q1_id) fp_zero(v);
  } else {                 // P2 = -G1: (-x, y) = (-G1x, -G1y)
    if (lane == 10) { LCV_FP_SET(v, LCV_G1X_INIT); fp_neg(v, v); }
    else LCV_FP_SET(v, LCV_G1NEGY_INIT);
    if (q2_id) fp_zero(v);
  }
  eng_store(lds, lane, v);  // input slots 0..11 in the order of LCV_PROG_MILLER_SLOT_*
}

LCV_FN void item_miller_team(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl, const ProgView& P, const Work& W) {
  if (r == 0) {
    eng_load_consts(P, lane, LCV_PROG_MILLER_TEAM, cl);
    miller_prologue(i, lane, lds, W);
  } else if (r <= P.rounds) {
    eng_round(P, r - 1, lane, lds, cl);
  } else if (lane < 12) {
    fp v;
    eng_load(v, lds, LCV_PROG_MILLER_SLOT_F0_0 + lane);
    soa_st_fp(W.f, W.cap, i, 2 * fp12_soa_slot(lane >> 1) + (lane & 1u), v);
  }
}

// Final exponentiation; epilogue stores the pairing value (e^3) and the "== 1" verdict.
LCV_FN void item_fexp_team(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl, const ProgView& P, const Work& W) {
  if (r == 0) {
    eng_load_consts(P, lane, LCV_PROG_FEXP_TEAM, cl);
    if (lane >= 12) return;
    fp v;
    soa_ld_fp(v, W.f, W.cap, i, 2 * fp12_soa_slot(lane >> 1) + (lane & 1u));
    eng_store(lds, LCV_PROG_FEXP_SLOT_F0_0 + lane, v);
  } else if (r <= P.rounds) {
    eng_round(P, r - 1, lane, lds, cl);
  } else if (lane < 12) {
    fp v;
    eng_load(v, lds, LCV_PROG_FEXP_SLOT_R0_0 + lane);
    soa_st_fp(W.f, W.cap, i, 2 * fp12_soa_slot(lane >> 1) + (lane & 1u), v);
    if (lane == 0) {
      fp one;
      fp_one(one);
      bool ok = fp_eq(v, one);
      for (uint32_t k = 1; k < 12; ++k) {
        fp w;
        eng_load(w, lds, LCV_PROG_FEXP_SLOT_R0_0 + k);
        ok = ok && fp_is_zero(w);
      }
      W.pair_ok[i] = ok ? 1 : 0;
    }
  }
}

// hash_to_G2 tail: isogeny of both SSWU points, addition, cofactor clearing, affine H(m) -> W.qh
LCV_FN void item_h2c_team(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl, const ProgView& P, const Work& W) {
  if (r == 0) {
    eng_load_consts(P, lane, LCV_PROG_H2C_TEAM, cl);
    for (uint32_t k = lane; k < 8; k += LCV_PROG_H2C_TEAM) {
      fp v;
      soa_ld_fp(v, W.qmap, W.cap, i, k);
      eng_store(lds, LCV_PROG_H2C_SLOT_M0X0 + k, v);
    }
  } else if (r <= P.rounds) {
    eng_round(P, r - 1, lane, lds, cl);
  } else if (lane < 4) {
    fp v;
    eng_load(v, lds, LCV_PROG_H2C_SLOT_HX0 + lane);
    soa_st_fp(W.qh, W.cap, i, lane, v);
    if (lane == 0) {
      fp z0, z1;
      eng_load(z0, lds, LCV_PROG_H2C_SLOT_HZ0);
      eng_load(z1, lds, LCV_PROG_H2C_SLOT_HZ0 + 1);
      W.qh_inf[i] = (fp_is_zero(z0) && fp_is_zero(z1)) ? 1 : 0;
    }
  }
}

// G2 subgroup check of the decoded signature (psi(P) == [x]P); a failure turns PT_OK into PT_BAD
LCV_FN void item_g2sub_team(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl, const ProgView& P, const Work& W) {
  if (r == 0) {
    eng_load_consts(P, lane, LCV_PROG_G2SUB_TEAM, cl);
    for (uint32_t k = lane; k < 4; k += LCV_PROG_G2SUB_TEAM) {
      fp v;
      soa_ld_fp(v, W.qs, W.cap, i, k);
      eng_store(lds, LCV_PROG_G2SUB_SLOT_SX0 + k, v);
    }
  } else if (r <= P.rounds) {
    eng_round(P, r - 1, lane, lds, cl);
  } else if (lane == 0 && W.sig_status[i] == PT_OK) {
    bool e_zero = true;
    for (uint32_t k = 0; k < 4; ++k) {
      fp v;
      eng_load(v, lds, LCV_PROG_G2SUB_SLOT_E10 + k);
      e_zero = e_zero && fp_is_zero(v);
    }
    fp z0, z1;
    eng_load(z0, lds, LCV_PROG_G2SUB_SLOT_Z0);
    eng_load(z1, lds, LCV_PROG_G2SUB_SLOT_Z0 + 1);
    const bool z_zero = fp_is_zero(z0) && fp_is_zero(z1);
    if (!e_zero || z_zero) W.sig_status[i] = PT_BAD;
  }
}

}  // namespace lcv
