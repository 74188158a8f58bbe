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
// Encoding (tools/gen_programs.py Program.encode): per round two wave-uniform header words and, per
// lane, a fixed 32-byte record (16 x uint16: dst | MUL << 12 | INV << 13, A terms from halfword 1,
// B terms from halfword LCV_PROG_B_AT; term = slot | coef << 12, signed 4-bit, padding = slot 0 coef 0).
// Fixed-size records let the kernel prefetch round r+1 (two 16-byte loads + the header) while it
// executes round r, so no global-memory latency sits on the round's critical path.
#pragma once
#include "lcv_items.hpp"
#include "lcv_programs.inc"

namespace lcv {

enum { ENG_SLOT_NONE = 0xFFF, ENG_MUL = 0x1000, ENG_INV = 0x2000 };

struct ProgView {
  const uint32_t* hdr;     // 2 words per round
  const uint32_t* rec;     // LCV_PROG_REC_HW / 2 words per lane per round, TEAM lanes per round
  const uint32_t* consts;  // 12 limbs per constant (Montgomery), copied into LDS slots nslots..
  uint32_t rounds;
  uint32_t nslots, nconst;
  uint32_t zero;           // slot of the zero constant (record padding terms read it)
};
enum { ENG_REC_WORDS = LCV_PROG_REC_HW / 2 };

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

// halfword j of a lane record (j is a compile-time constant after unrolling)
LCV_FN uint32_t eng_hw(const uint32_t* w, int j) { return (w[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu; }

LCV_FN const uint32_t* eng_src(uint32_t term, const uint32_t* lds, const uint32_t* cl, uint32_t ns) {
  const uint32_t slot = term & 0xFFFu;
  return slot >= ns ? cl + 12 * (slot - ns) : lds + 12 * slot;
}

// out = sum_k c_k * value(slot_k) (mod p) over the NMAX-unrolled terms at halfwords BASE.. of the
// record; n, maxc, kb, lo are wave-uniform (round header), so every branch below is scalar.  The
// 13-limb accumulator starts at the bias 2^kb p (the signed sum lies in (-2^kb p, 2^kb p), 2^kb >
// sum |c|) and each term adds t = |c| * v (< 7p < 2^384, 12 limbs) or its two's complement
// (t ^ m) + 1 (m = all-ones when c < 0), so it stays in [0, 2^(kb+1) p) without any p - v.  Then
// conditional subtraction of 2^s p for s = kb .. lo: lo = 0 fully reduces (LIN results are
// stored), lo = 1 leaves < 2p (a Montgomery operand: a, b < 2p gives ab < R p, a result < 2p).
// |c| * v: v itself when maxc = 1 (records pad with a zero constant at coefficient +1, so no
// masking), a per-lane select of v / 2v when maxc = 2, else a v_mad_u64_u32 chain.  The LDS read of
// term k+1 is issued before term k is accumulated.
template <int BASE, int NMAX>
LCV_FN void eng_eval(fp& out, const uint32_t* w, uint32_t n, uint32_t maxc, uint32_t kb, uint32_t lo,
                     const uint32_t* lds, const uint32_t* cl, uint32_t ns) {
  constexpr uint32_t PL[12] = LCV_P_INIT;
  uint32_t acc[13];
  acc[0] = PL[0] << kb;  // 1 <= kb <= 6 (wave-uniform: scalar shifts)
  LCV_UNROLL for (int j = 1; j < 12; ++j) acc[j] = (PL[j] << kb) | (PL[j - 1] >> (32 - kb));
  acc[12] = PL[11] >> (32 - kb);
  uint32_t v[12];
  {
    const uint32_t* src = eng_src(eng_hw(w, BASE), lds, cl, ns);
    LCV_UNROLL for (int j = 0; j < 12; ++j) v[j] = src[j];
  }
  LCV_UNROLL for (int k = 0; k < NMAX; ++k) {
    if ((uint32_t)k >= n) break;
    const uint32_t term = eng_hw(w, BASE + k);
    uint32_t nx[12];
    if (k + 1 < NMAX && (uint32_t)(k + 1) < n) {
      const uint32_t* src = eng_src(eng_hw(w, BASE + (k + 1 < NMAX ? k + 1 : k)), lds, cl, ns);
      LCV_UNROLL for (int j = 0; j < 12; ++j) nx[j] = src[j];
    }
    int c = (int)(term >> 12);
    if (c >= 8) c -= 16;
    const uint32_t a = (uint32_t)(c < 0 ? -c : c);
    const uint32_t m = c < 0 ? 0xFFFFFFFFu : 0u;
    uint32_t t[12];
    if (maxc <= 1) {
      LCV_UNROLL for (int j = 0; j < 12; ++j) t[j] = v[j];
    } else if (maxc <= 2) {  // v < 2^381: 2v needs no 13th limb
      const bool dbl = a == 2u;
      t[0] = dbl ? v[0] << 1 : v[0];
      LCV_UNROLL for (int j = 1; j < 12; ++j) t[j] = dbl ? ((v[j] << 1) | (v[j - 1] >> 31)) : v[j];
    } else {  // |c| <= 7: |c| v < 2^384, the chain's last high word is 0
      uint32_t hi = 0;
      LCV_UNROLL for (int j = 0; j < 12; ++j) {
        const uint64_t pr = (uint64_t)v[j] * a + hi;  // one v_mad_u64_u32
        t[j] = (uint32_t)pr;
        hi = (uint32_t)(pr >> 32);
      }
    }
    uint32_t cy = m & 1u;  // two's complement of t when c < 0: (t ^ m) + 1 over 13 limbs
    LCV_UNROLL for (int j = 0; j < 12; ++j) acc[j] = addc32(acc[j], t[j] ^ m, cy, cy);
    acc[12] = acc[12] + m + cy;
    if (k + 1 < NMAX && (uint32_t)(k + 1) < n) {
      LCV_UNROLL for (int j = 0; j < 12; ++j) v[j] = nx[j];
    }
  }
  // acc < 2^(kb+1) p  ->  acc < 2^lo p; s is a constant after unrolling, so p << s folds into literals
  LCV_UNROLL for (int s = 6; s >= 0; --s) {
    if ((uint32_t)s <= kb && (uint32_t)s >= lo) {
      uint32_t sp[13], dd[13];
      LCV_UNROLL for (int j = 0; j < 12; ++j) sp[j] = (PL[j] << s) | (s && j ? (PL[j - 1] >> (32 - s)) : 0u);
      sp[12] = s ? (PL[11] >> (32 - s)) : 0u;
      uint32_t br = 0;
      LCV_UNROLL for (int j = 0; j < 13; ++j) dd[j] = subc32(acc[j], sp[j], br, br);
      LCV_UNROLL for (int j = 0; j < 13; ++j) acc[j] = br ? acc[j] : dd[j];
    }
  }
  LCV_UNROLL for (int j = 0; j < 12; ++j) out.v[j] = acc[j];
}

// one round for one lane: record w (ENG_REC_WORDS words), header h0/h1 (wave-uniform)
LCV_FN void eng_exec(const uint32_t* w, uint32_t h0, uint32_t h1, uint32_t* lds, const uint32_t* cl, uint32_t ns,
                     uint32_t zero) {
  (void)zero;
  const uint32_t nA = h0 & 0xFu, mA = (h0 >> 4) & 0xFu, kA = (h0 >> 8) & 7u, loA = (h0 >> 11) & 1u ? 0u : 1u;
  const uint32_t nB = (h0 >> 12) & 0xFu, mB = (h0 >> 16) & 0xFu, kB = (h0 >> 20) & 7u;
  const uint32_t dst = eng_hw(w, 0);
  fp a;
  eng_eval<1, LCV_PROG_KLIN>(a, w, nA, mA, kA, loA, lds, cl, ns);
#if defined(LCV_HOSTSIM)
  // host simulation: only the lanes that own a MUL multiply (the device runs the product in every
  // lane of a MUL round and discards it), so the op counter sees the program's algorithmic work:
  // one Fp multiplication per MUL op, (terms - 1) Fp additions per combination
  if ((dst & 0xFFFu) != ENG_SLOT_NONE) {
    auto terms = [&](int base, uint32_t n) {  // the lane's own terms (padding reads the zero constant)
      uint32_t t = 0;
      for (uint32_t k = 0; k < n; ++k) t += (eng_hw(w, base + (int)k) & 0xFFFu) != zero;
      return t;
    };
    for (uint32_t k = 1; k < terms(1, nA); ++k) LCV_COUNT(1);
    if ((h1 & 0x100u) && (dst & ENG_MUL)) {
      for (uint32_t k = 1; k < terms(LCV_PROG_B_AT, nB); ++k) LCV_COUNT(1);
      fp b;
      eng_eval<LCV_PROG_B_AT, LCV_PROG_REC_HW - LCV_PROG_B_AT>(b, w, nB, mB, kB, 1u, lds, cl, ns);
      fp_mul(a, a, b);
    }
  }
#else
  if (h1 & 0x100u) {  // a MUL round (B operands have <= 4 terms); LIN lanes keep A
    fp b, m;
    eng_eval<LCV_PROG_B_AT, LCV_PROG_REC_HW - LCV_PROG_B_AT>(b, w, nB, mB, kB, 1u, lds, cl, ns);
    fp_mul(m, a, b);
    if (dst & ENG_MUL) a = m;
  }
#endif
  if (h1 & 0x200u) {
    if (dst & ENG_INV) fp_inv_bingcd(a, a);
  }
  if ((dst & 0xFFFu) != ENG_SLOT_NONE) eng_store(lds, dst & 0xFFFu, a);
}

// one round of a program for lane `lane` (host simulation and the generic round loop)
LCV_FN void eng_round(const ProgView& P, uint32_t r, uint32_t lane, uint32_t team, uint32_t* lds, const uint32_t* cl) {
  const uint32_t* w = P.rec + ((size_t)r * team + lane) * ENG_REC_WORDS;
  eng_exec(w, P.hdr[2 * r], P.hdr[2 * r + 1], lds, cl, P.nslots, P.zero);
}

}  // namespace lcv

// ============================================================================ pairing stages

namespace lcv {

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
    eng_round(P, r - 1, lane, LCV_PROG_MILLER_TEAM, lds, cl);
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
    eng_round(P, r - 1, lane, LCV_PROG_FEXP_TEAM, lds, cl);
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
    eng_round(P, r - 1, lane, LCV_PROG_H2C_TEAM, lds, cl);
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
    eng_round(P, r - 1, lane, LCV_PROG_G2SUB_TEAM, lds, cl);
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
