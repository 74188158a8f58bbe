// lcv_wide_sop.hpp — the latency engine's SOP round (device only): the same generated programs
// (lcv_sop_programs.inc) as the batch engine, for ONE item per workgroup of TEAM waves — wave t plays
// team lane t, so every op of a round runs on a whole wave at once.  An op
//     dst = REDC( sum_{k<K} m_k X_k Y_k + R (c_0 v_a + c_1 v_b) )
// keeps X_k replicated in every lane and stages Y_k in the wave's LDS window (lcv_field.hpp wide engine),
// so lane c accumulates column c of every product (13 multiply-accumulates per product instead of
// 144); the add-ins enter columns 12..24; the 25 column sums are normalised and reduced with the
// separated Montgomery reduction (wide_redc: the unique M, so the result is the batch engine's bit for
// bit), then the same conditional subtractions (sop_reduce), inversion, loads, emits and stores.
// Reference: the pairing of bls.FastAggregateVerify, call site sync-protocol.md:464, one update per call
// (sync-protocol.md:512).
#pragma once
#include "lcv_sop.hpp"

namespace lcv {

// a wave's LDS accesses execute in program order; this only keeps the compiler from moving them
LCV_FN void wide_fence() { __builtin_amdgcn_wave_barrier(); }

// the replicated 12-word value v at words [16, 28) of the wave's window (lane 0 stores it)
LCV_FN void wide_stage(uint32_t* win, const uint32_t v[12]) {
  wide_fence();
  if (wide_lane() == 0) {
    LCV_UNROLL for (int j = 0; j < 12; ++j) win[WIDE_OFF + j] = v[j];
  }
  wide_fence();
}

// (hi:acc) += (hi1:acc1)
LCV_FN void wide_acc_merge(uint64_t& acc, uint32_t& hi, uint64_t acc1, uint32_t hi1) {
  uint32_t lo = (uint32_t)acc, mid = (uint32_t)(acc >> 32), c;
  lo = addc32(lo, (uint32_t)acc1, 0u, c);
  mid = addc32(mid, (uint32_t)(acc1 >> 32), c, c);
  hi = hi + hi1 + c;
  acc = ((uint64_t)mid << 32) | lo;
}

// One op of a round on the calling wave (header h0 as sop_exec; w: the op's record, 4 + 3 MAXK words
// already in registers — the kernel prefetches it a round ahead; lds: the item's slots, cl: the program's
// constants).  Contains the round's read/write barrier: every wave of the workgroup (every op of the
// round) calls it once per round.  The product and add-in loops are unrolled to MAXK / 3 (guarded by
// the wave-uniform K and add-in count) so the record stays in registers.
template <uint32_t MAXK>
LCV_FN void sop_exec_wide(uint32_t h0, const uint32_t (&w)[4 + 3 * MAXK], uint32_t* lds, const uint32_t* cl,
                          uint32_t ns, const uint32_t* io_in, uint32_t* io_out) {
  const uint32_t K = h0 & 15u, nadd = (h0 >> 4) & 3u, red = (h0 >> 16) & 31u;
  const bool mflag = (h0 >> 6) & 1u, x2 = (h0 >> 7) & 1u, y2 = (h0 >> 8) & 1u;
  const uint32_t lane = wide_lane();
  uint32_t* win = wide_scratch();
  const uint32_t* wl = win + WIDE_OFF + lane;
  const uint32_t r0 = w[0];
  const uint32_t dst = r0 & 0xFFFu;
  uint64_t acc = 0, acc1 = 0;
  uint32_t hi = 0, hi1 = 0;
  LCV_UNROLL for (uint32_t k = 0; k < MAXK; ++k) {
    if (k >= K) break;
    const uint32_t xw = w[4 + 3 * k], yw = w[5 + 3 * k], mk = w[6 + 3 * k];
    uint32_t X[13], Y[12];
    sop_operand(X, xw, x2, lds, cl, ns);
    sop_operand(Y, yw, y2, lds, cl, ns);
    X[12] = 0;
    if (mflag) {  // X *= m (m < 2^16): 13 words
      uint32_t carry = 0;
      LCV_UNROLL for (int j = 0; j < 12; ++j) {
        const uint64_t t = (uint64_t)X[j] * mk + carry;
        X[j] = (uint32_t)t;
        carry = (uint32_t)(t >> 32);
      }
      X[12] = carry;
    }
    wide_stage(win, Y);
    // lane c: sum_i X_i Y_{c - i} (the window is zero outside [16, 28)); two accumulators halve the
    // dependent multiply-accumulate chain
    LCV_UNROLL for (int i = 0; i < 12; i += 2) {
      mac_vv(acc, hi, X[i], wl[-i]);
      mac_vv(acc1, hi1, X[i + 1], wl[-i - 1]);
    }
    mac_vv(acc, hi, X[12], wl[-12]);
  }
  // add-ins: columns 12..24 += |c| (v or p - v)
  LCV_UNROLL for (uint32_t j = 0; j < 2; ++j) {
    if (j >= nadd) break;
    const uint32_t a = w[2 + j];
    const int c = (int)(int16_t)(a >> 16);
    uint32_t t[12];
    sop_term(t, (a & 0xFFFu) | (c < 0 ? SOP_NEG : 0u), true, lds, cl, ns);
    const uint32_t mag = (uint32_t)(c < 0 ? -c : c);
    wide_stage(win, t);
    mac_vs(acc, hi, wl[-12], mag);
  }
  wide_acc_merge(acc, hi, acc1, hi1);
  const uint32_t Tw = wide_norm<25>(acc, hi);
  uint32_t r[13];
  if (K == 0) {  // an add-in-only op: the sum is R x, REDC(R x) = x exactly (as sop_exec)
    LCV_UNROLL for (int j = 0; j < 13; ++j) r[j] = __builtin_amdgcn_readlane(Tw, 12 + j);
  } else {
    wide_redc(r, Tw);
  }
  sop_reduce(r, red);
  fp v;
  LCV_UNROLL for (int j = 0; j < 12; ++j) v.v[j] = r[j];
  const uint32_t fl = (r0 >> 12) & 7u;
  if ((h0 >> 10) & 1u) {  // an inversion round: the op's flag selects (wave-uniform)
    if (fl & SOP_F_INV) fp_inv(v, v);
  }
  __syncthreads();  // every op of the round has read its operands: the stores may overwrite them
  const uint32_t r1 = w[1];
  const uint32_t io = r1 & 0xFFFu, dsh = (r1 >> 12) & 0x3FFu, lsh = (r1 >> 22) & 0x3FFu;
  const bool shadow = (h0 >> 13) & 1u;
  if (lane == 0) {
    if ((h0 >> 11) & 1u) {  // side-load round: Fp value io_in[index] -> LDS slot r0 >> 16
      if (fl & SOP_F_LOAD) {
        const uint32_t* src = io_in + 12 * (size_t)io;
        uint32_t* d = lds + 12 * ((r0 >> 16) & 0xFFFu);
        uint32_t t[12];
        LCV_UNROLL for (int j = 0; j < 12; ++j) t[j] = src[j];
        LCV_UNROLL for (int j = 0; j < 12; ++j) d[j] = t[j];
        if (shadow && lsh != 0x3FFu) sop_store_neg(lds + 12 * lsh, t);
      }
    }
    if ((h0 >> 12) & 1u) {  // emit round: the result also goes to io_out[index]
      if (fl & SOP_F_EMIT) {
        uint32_t* o = io_out + 12 * (size_t)io;
        LCV_UNROLL for (int j = 0; j < 12; ++j) o[j] = v.v[j];
      }
    }
    if (dst != SOP_SLOT_NONE) {
      uint32_t* d = lds + 12 * dst;
      LCV_UNROLL for (int j = 0; j < 12; ++j) d[j] = v.v[j];
      if (shadow && dsh != 0x3FFu) sop_store_neg(lds + 12 * dsh, v.v);
    }
  }
}

}  // namespace lcv
