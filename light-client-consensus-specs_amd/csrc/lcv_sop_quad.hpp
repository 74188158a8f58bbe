// lcv_sop_quad.hpp — the quad engine: the SOP programs (lcv_sop.hpp, tools/gen_sop.py) with every op of
// a round spread over FOUR lanes, for the latency path (lcv_set_latency_mode: batches of a few updates,
// the reference's one-update-per-call usage, sync-protocol.md:512 -> :464).  One item per wave; op o of
// the team runs on lanes 4o .. 4o + 3 (quarter q = lane & 3).  A lone wave pays every instruction of a
// round (1,100-1,600 per op in the batch engine), so the latency of a round is its per-lane instruction
// count: here each lane multiplies a quarter of the limb products and carries a quarter of the
// Montgomery reduction's column updates.
//
//   products   lane q takes the limbs x_q, x_(q+4), x_(q+8), x_(q+12) of X against all 14 limbs of Y
//              (56 multiply-adds per product instead of 147 Karatsuba ones), into 26 partial columns
//              pc[t] of column t + q;
//   transpose  through the op's LDS scratch (4 rows of 29 columns; row q holds pc at t + q, the rest of
//              the row stays zero): lane q then owns the full columns c = 4k + q, k = 0..6;
//   reduction  digit i (0..13) of the Montgomery quotient is computed from column i + carry, broadcast
//              from its owner lane by a DPP quad_perm (every lane then computes the same digit and
//              carry), and each lane adds digit * p's limb into the columns it owns (4-5 multiply-adds);
//   tail       columns 14..27 broadcast to all four lanes, normalised and packed into 13 words, then
//              lcv::sop_tail (add-ins, conditional subtractions, store, shadow) on all four lanes alike.
// The result is the unique (T + M p) / R with M < R, T + M p = 0 mod R: the batch engine's value bit
// for bit (tests/test_latency_gpu.py).  Device-only; the host simulation runs the batch engine.
#pragma once
#include "lcv_sop.hpp"

namespace lcv {

enum : uint32_t { QUAD_ROW = 29, QUAD_SCRATCH_U64 = 4 * QUAD_ROW };  // per op: 4 rows x 29 64-bit columns

// value of lane SRC of each quad, in every lane of the quad
template <int SRC> LCV_FN uint32_t qb32(uint32_t v) {
  // every lane of an active quad is active (ops are per quad), so no lane reads an invalid source:
  // bound_ctrl, no old value to preserve (a plain v_mov_b32_dpp quad_perm:[SRC x 4])
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, SRC | (SRC << 2) | (SRC << 4) | (SRC << 6), 0xF, 0xF, true);
}
template <int SRC> LCV_FN uint64_t qb64(uint64_t v) {
  return (uint64_t)qb32<SRC>((uint32_t)v) | ((uint64_t)qb32<SRC>((uint32_t)(v >> 32)) << 32);
}

// pz[e] = p's 28-bit limb e - 2 + q when that index is 1..13, else 0 (the limb a column of this lane
// meets in a reduction step, lane-independent register index)
LCV_FN void quad_ptable(uint32_t pz[16], uint32_t q) {
  LCV_UNROLL for (int e = 0; e < 16; ++e) {
    uint32_t v[4];
    LCV_UNROLL for (int s = 0; s < 4; ++s) {
      const int idx = e - 2 + s;
      v[s] = (idx >= 1 && idx <= 13) ? kP28.v[idx] : 0u;
    }
    pz[e] = q == 0 ? v[0] : q == 1 ? v[1] : q == 2 ? v[2] : v[3];
    // opaque 32-bit values from here on: otherwise clang carries the table as 64-bit selects of
    // constants and emits a 64 x 32-bit multiply (two v_mad_u64_u32 and moves) per column update
    asm volatile("" : "+v"(pz[e]));
  }
}

// the K products of an op, this lane's quarter: pc[t] (t = 4m + j) += x_(q + 4m) y_j
template <bool FIRST>
LCV_FN void quad_mac(uint64_t pc[26], const uint32_t xs[4], const uint32_t Y[14]) {
  LCV_UNROLL for (int m = 0; m < 4; ++m)
    LCV_UNROLL for (int j = 0; j < 14; ++j) {
      const int t = 4 * m + j;
      const int mfirst = t > 13 ? (t - 13 + 3) / 4 : 0;  // the first m whose products reach column t
      if (FIRST && m == mfirst) pc[t] = (uint64_t)xs[m] * Y[j];
      else pc[t] += (uint64_t)xs[m] * Y[j];
    }
}
LCV_FN void quad_products(uint64_t pc[26], const uint32_t* pw0, uint32_t K, uint32_t masks, bool mflag,
                          const SopBase& base, uint32_t q, uint32_t nxw, uint32_t nyw, uint32_t nmk) {
  LCV_NOUNROLL for (uint32_t k = 0; k < K; ++k) {
    const uint32_t xw = nxw, yw = nyw, mk = nmk;
    {
      const uint32_t kn = k + 1 < K ? k + 1 : k;
      nxw = pw0[3 * kn]; nyw = pw0[3 * kn + 1]; nmk = pw0[3 * kn + 2];
    }
    uint32_t Xw[13], Yw[12], X[16], Y[14];
    sop_operand(Xw, xw, (masks >> k) & 1u, base);
    sop_operand(Yw, yw, (masks >> (16 + k)) & 1u, base);
    Xw[12] = 0;
    if (mflag) {
      uint32_t carry = 0;
      LCV_UNROLL for (int j = 0; j < 12; ++j) {
        const uint64_t t = (uint64_t)Xw[j] * mk + carry;
        Xw[j] = (uint32_t)t;
        carry = (uint32_t)(t >> 32);
      }
      Xw[12] = carry;
    }
    sop_to28<12, 14>(Y, Yw);
    sop_to28<13, 14>(X, Xw);  // m X < 2^392 in every product round (LCV_SOP_SCHOOLBOOK 0)
    X[14] = X[15] = 0;
    uint32_t xs[4];
    LCV_UNROLL for (int m = 0; m < 4; ++m)
      xs[m] = q == 0 ? X[4 * m] : q == 1 ? X[4 * m + 1] : q == 2 ? X[4 * m + 2] : X[4 * m + 3];
    if (k == 0) quad_mac<true>(pc, xs, Y);
    else quad_mac<false>(pc, xs, Y);
  }
}

// partial columns -> this lane's full columns A[k] = column 4k + q, through the op's scratch S
LCV_FN void quad_transpose(uint64_t A[7], const uint64_t pc[26], uint64_t* S, uint32_t q) {
  uint64_t* row = S + q * QUAD_ROW + q;
  LCV_UNROLL for (int t = 0; t < 26; ++t) row[t] = pc[t];
  __builtin_amdgcn_wave_barrier();
  const uint64_t* col = S + q;
  LCV_UNROLL for (int k = 0; k < 7; ++k)
    A[k] = col[4 * k] + col[QUAD_ROW + 4 * k] + col[2 * QUAD_ROW + 4 * k] + col[3 * QUAD_ROW + 4 * k];
  __builtin_amdgcn_wave_barrier();
}

// one reduction digit: column i (owner lane i & 3) + carry -> digit; this lane's columns += digit * p
template <int I>
LCV_FN void quad_digit(uint64_t A[7], uint64_t& carry, uint64_t& vout, const uint32_t pz[16]) {
  const uint64_t v = qb64<I & 3>(A[I >> 2] + carry);
  const uint32_t qd = ((uint32_t)v * kNP28) & (I < 13 ? SOP_M28 : 0xFFFFFu);
  const uint64_t t = v + (uint64_t)qd * kP28.v[0];
  carry = t >> 28;
  vout = t;
  LCV_UNROLL for (int k = 0; k < 7; ++k) {
    const int e = 4 * k - I + 2;
    if (e >= 0 && e < 16) A[k] += (uint64_t)qd * pz[e];
  }
}
template <int I> LCV_FN void quad_digits(uint64_t A[7], uint64_t& carry, uint64_t& v, const uint32_t pz[16]) {
  if constexpr (I < 14) {
    quad_digit<I>(A, carry, v, pz);
    quad_digits<I + 1>(A, carry, v, pz);
  }
}
template <int C> LCV_FN void quad_norm(uint32_t L[16], const uint64_t A[7], uint64_t& carry) {
  if constexpr (C < 28) {
    const uint64_t t = qb64<C & 3>(A[C >> 2]) + carry;
    L[C - 13] = (uint32_t)t & SOP_M28;
    carry = t >> 28;
    quad_norm<C + 1>(L, A, carry);
  }
}
// r (13 words, replicated in the quad) = (T + M p) / 2^384 (lcv_col28.hpp sop_redc28's digits)
LCV_FN void quad_redc(uint32_t r[13], uint64_t A[7], const uint32_t pz[16]) {
  uint64_t carry = 0, v = 0;
  quad_digits<0>(A, carry, v, pz);
  // after the 20-bit digit 13, v = column 13 + carry + q p_0 has its low 20 bits zero
  uint32_t L[16];
  L[0] = (uint32_t)v & SOP_M28;
  carry = v >> 28;
  quad_norm<14>(L, A, carry);
  L[15] = (uint32_t)carry;
  LCV_UNROLL for (int k = 0; k < 13; ++k) {
    const int b = 20 + 32 * k, j = b / 28, s = b % 28;
    uint32_t x = L[j] >> s;
    x |= L[j + 1] << (28 - s);
    if (s > 24) x |= L[j + 2] << (56 - s);
    r[k] = x;
  }
}

// one round of op o for the lane of quarter q (every lane of the quad runs it)
LCV_FN void sop_exec_quad(uint32_t h0, uint32_t h3, const uint32_t* w, const SopPre& pre, const uint32_t* lds,
                          uint32_t* wr, const uint32_t* cl, uint32_t ns, const uint32_t* io_in, uint32_t* io_out,
                          uint32_t q, uint64_t* S, const uint32_t pz[16]) {
  const uint32_t K = h0 & 15u;
  const bool mflag = (h0 >> 6) & 1u;
  uint32_t r[13];
  if (K == 0) {
    LCV_UNROLL for (int j = 0; j < 13; ++j) r[j] = 0;
  } else {
    const SopBase base{lds, cl, (int32_t)((const char*)cl - (const char*)lds)};
    uint64_t pc[26], A[7];
    quad_products(pc, w + 4, K, h3, mflag, base, q, pre.x, pre.y, pre.m);
    quad_transpose(A, pc, S, q);
    quad_redc(r, A, pz);
  }
  sop_tail(h0, w, pre, lds, wr, cl, ns, io_in, io_out, r);
}

}  // namespace lcv
