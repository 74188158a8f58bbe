// lcv_h2c.hpp — hash_to_G2 for the POP ciphersuite: RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ with
// DST "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_" (43 bytes), as called by FastAggregateVerify on
// the signing root (reference sync-protocol.md:463-464).
//
//   expand_message_xmd (SHA-256, 256 output bytes): the first block of b0 is the all-zero Z_pad,
//   so its midstate is a compile-time constant; every later block tail is constant too (DST').
//   hash_to_field -> u0, u1 in Fp2; simplified SWU onto E2'; 3-isogeny to E2 (emitted directly
//   in Jacobian coordinates: Z = xd*yd, so the two inversions of the affine map disappear);
//   Q0 + Q1; clear_cofactor via psi (RFC 9380 App. G.3).
#pragma once
#include "lcv_curve.hpp"
#include "lcv_sha.hpp"

namespace lcv {

// b_i = H((b0 ^ b_{i-1}) || i || DST')   (b_0 ^ 0 = b_0 gives b_1)
LCV_FN void xmd_next(h256& out, const h256& b0, const h256& prev, uint32_t i) {
  constexpr uint32_t C1T[8] = LCV_XMD_C1_TAIL_INIT;
  constexpr uint32_t C2[16] = LCV_XMD_C2_INIT;
  uint32_t st[8], blk[16];
  sha256_iv(st);
  LCV_UNROLL for (int k = 0; k < 8; ++k) { blk[k] = b0.w[k] ^ prev.w[k]; blk[8 + k] = C1T[k]; }
  blk[8] |= i << 24;
  sha256_compress(st, blk);
  LCV_UNROLL for (int k = 0; k < 16; ++k) blk[k] = C2[k];
  sha256_compress(st, blk);
  LCV_UNROLL for (int k = 0; k < 8; ++k) out.w[k] = st[k];
}

LCV_FN void xmd_b0(h256& b0, const h256& msg) {
  constexpr uint32_t H1[8] = LCV_XMD_H1_INIT;
  constexpr uint32_t B2T[8] = LCV_XMD_B2_TAIL_INIT;
  constexpr uint32_t B3[16] = LCV_XMD_B3_INIT;
  uint32_t st[8], blk[16];
  LCV_UNROLL for (int k = 0; k < 8; ++k) { st[k] = H1[k]; blk[k] = msg.w[k]; blk[8 + k] = B2T[k]; }
  sha256_compress(st, blk);
  LCV_UNROLL for (int k = 0; k < 16; ++k) blk[k] = B3[k];
  sha256_compress(st, blk);
  LCV_UNROLL for (int k = 0; k < 8; ++k) b0.w[k] = st[k];
}

// 64-byte big-endian integer (hi || lo) mod p, Montgomery form
LCV_FN void fp_from_xmd64(fp& r, const h256& hi, const h256& lo) {
  fp h, l, c, t;
  LCV_UNROLL for (int k = 0; k < 8; ++k) { h.v[k] = hi.w[7 - k]; l.v[k] = lo.w[7 - k]; }
  LCV_UNROLL for (int k = 8; k < 12; ++k) { h.v[k] = 0; l.v[k] = 0; }
  LCV_FP_SET(c, LCV_C256_INIT);
  fp_mul(t, h, c);
  LCV_FP_SET(c, LCV_R2_INIT);
  fp_mul(r, l, c);
  fp_add(r, r, t);
}

// 3-isogeny E2' -> E2, result in Jacobian coordinates (Z = 0 <=> exceptional case -> identity)
LCV_FN void iso_map_g2(g2j& r, const fp2& x, const fp2& y) {
  fp2 x2, x3, xn, xd, yn, yd, t, c;
  fp2_sqr(x2, x);
  fp2_mul(x3, x2, x);
  LCV_FP2_SET(c, LCV_ISO_XNUM3); fp2_mul(xn, c, x3);
  LCV_FP2_SET(c, LCV_ISO_XNUM2); fp2_mul(t, c, x2); fp2_add(xn, xn, t);
  LCV_FP2_SET(c, LCV_ISO_XNUM1); fp2_mul(t, c, x); fp2_add(xn, xn, t);
  LCV_FP2_SET(c, LCV_ISO_XNUM0); fp2_add(xn, xn, c);
  LCV_FP2_SET(c, LCV_ISO_XDEN1); fp2_mul(t, c, x); fp2_add(xd, x2, t);
  LCV_FP2_SET(c, LCV_ISO_XDEN0); fp2_add(xd, xd, c);
  LCV_FP2_SET(c, LCV_ISO_YNUM3); fp2_mul(yn, c, x3);
  LCV_FP2_SET(c, LCV_ISO_YNUM2); fp2_mul(t, c, x2); fp2_add(yn, yn, t);
  LCV_FP2_SET(c, LCV_ISO_YNUM1); fp2_mul(t, c, x); fp2_add(yn, yn, t);
  LCV_FP2_SET(c, LCV_ISO_YNUM0); fp2_add(yn, yn, c);
  LCV_FP2_SET(c, LCV_ISO_YDEN2); fp2_mul(t, c, x2); fp2_add(yd, x3, t);
  LCV_FP2_SET(c, LCV_ISO_YDEN1); fp2_mul(t, c, x); fp2_add(yd, yd, t);
  LCV_FP2_SET(c, LCV_ISO_YDEN0); fp2_add(yd, yd, c);
  // x = xn/xd, y = y*yn/yd  ->  Z = xd yd, X = xn xd yd^2, Y = y yn xd^3 yd^2
  fp2 yd2, xd3;
  fp2_sqr(yd2, yd);
  fp2_mul(r.z, xd, yd);
  fp2_mul(r.x, xn, xd);
  fp2_mul(r.x, r.x, yd2);
  fp2_sqr(xd3, xd);
  fp2_mul(xd3, xd3, xd);
  fp2_mul(t, xd3, yd2);
  fp2_mul(t, t, yn);
  fp2_mul(r.y, t, y);
}

// simplified SWU onto E2' (RFC 9380 §6.6.2, straight-line form): affine (x, y) on E2'
LCV_FN void sswu_e2prime(fp2& xo, fp2& yo, const fp2& u) {
  fp2 A, B, Z, t, u2, zu2, den, x1, gx1, x2, gx2, x, gx, y, one, c;
  LCV_FP2_SET(A, LCV_ISO_A);
  LCV_FP2_SET(B, LCV_ISO_B);
  LCV_FP2_SET(Z, LCV_SSWU_Z);
  fp2_one(one);
  fp2_sqr(u2, u);
  fp2_mul(zu2, Z, u2);
  fp2_sqr(den, zu2);
  fp2_add(den, den, zu2);
  const bool den0 = fp2_is_zero(den);
  fp2_inv(t, den);  // inv0
  fp2_add(t, t, one);
  LCV_FP2_SET(c, LCV_SSWU_NEGB_OVER_A);
  fp2_mul(x1, c, t);
  LCV_FP2_SET(c, LCV_SSWU_B_OVER_ZA);
  fp2_sel(x1, den0, c, x1);
  fp2_sqr(t, x1);
  fp2_mul(gx1, t, x1);
  fp2_mul(t, A, x1);
  fp2_add(gx1, gx1, t);
  fp2_add(gx1, gx1, B);
  fp2_mul(x2, zu2, x1);
  fp2_sqr(t, x2);
  fp2_mul(gx2, t, x2);
  fp2_mul(t, A, x2);
  fp2_add(gx2, gx2, t);
  fp2_add(gx2, gx2, B);
  fp alpha;
  const bool sq1 = fp2_is_square_alpha(gx1, alpha);
  fp2_sel(x, sq1, x1, x2);
  fp2_sel(gx, sq1, gx1, gx2);
  // gx1 not a square: gx2 = (Z u^2)^3 gx1, hence norm(gx2)^((p+1)/4) = +-norm(Z)^(3(p+1)/4) norm(u)^3 alpha
  // (fp2_sqrt_alpha accepts either sign).  Four multiplications replace a second 381-bit exponentiation
  // that a wave would otherwise run whenever any of its lanes takes this branch.  (The exceptional
  // den0 case has gx1 square by the choice of Z, RFC 9380 §6.6.2, so it never reads alpha2.)
  fp nu, alpha2, c2;
  fp2_norm(nu, u);
  fp_sqr(alpha2, nu);
  fp_mul(alpha2, alpha2, nu);
  LCV_FP_SET(c2, LCV_SSWU_ALPHA2_C_INIT);
  fp_mul(alpha2, alpha2, c2);
  fp_mul(alpha2, alpha2, alpha);
  fp alpha_sel;
  fp_sel(alpha_sel, sq1, alpha, alpha2);
  fp2_sqrt_alpha(y, gx, alpha_sel);
  if (fp2_sgn0(u) != fp2_sgn0(y)) fp2_neg(y, y);
  xo = x;
  yo = y;
}


// map_to_curve = SSWU then the 3-isogeny (used by the signer; verification runs the isogeny and the
// cofactor clearing as the SOP program `h2c`, F_sop_h2c)
LCV_FN void map_to_curve_g2(g2j& r, const fp2& u) {
  fp2 x, y;
  sswu_e2prime(x, y, u);
  iso_map_g2(r, x, y);
}

// hash_to_field(msg, 2)[m] (RFC 9380 §5.2; u_1 needs the xmd chain through u_0's blocks)
// b0 of expand_message_xmd for a message of any length: SHA-256(Z_pad || msg || I2OSP(256, 2) ||
// I2OSP(0, 1) || DST || I2OSP(43, 1)), streamed byte by byte after the constant Z_pad midstate
// (FastAggregateVerify drop-in with a message that is not a 32-byte signing root; one lane per message)
LCV_FN void xmd_b0_bytes(h256& b0, const uint8_t* msg, uint64_t len) {
  constexpr uint32_t H1[8] = LCV_XMD_H1_INIT;
  const char* dst = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
  uint32_t st[8], blk[16];
  LCV_UNROLL for (int k = 0; k < 8; ++k) st[k] = H1[k];
  const uint64_t body = len + 47;                 // msg || 01 00 || 00 || DST (43) || 2b
  const uint64_t total = (body + 9 + 63) / 64 * 64;  // + 0x80 + 64-bit bit length, whole blocks
  const uint64_t bits = (64 + body) * 8;          // Z_pad included in the message length
  LCV_NOUNROLL for (uint64_t base = 0; base < total; base += 64) {
    LCV_NOUNROLL for (int w = 0; w < 16; ++w) {
      uint32_t word = 0;
      for (int b = 0; b < 4; ++b) {
        const uint64_t k = base + 4 * w + b;
        uint32_t byte;
        if (k < len) byte = msg[k];
        else if (k == len) byte = 0x01;
        else if (k < len + 3) byte = 0x00;
        else if (k < len + 46) byte = (uint8_t)dst[k - len - 3];
        else if (k == len + 46) byte = 43;
        else if (k == body) byte = 0x80;
        else if (k >= total - 8) byte = (uint32_t)(bits >> (8 * (total - 1 - k))) & 0xFFu;
        else byte = 0;
        word = (word << 8) | byte;
      }
      blk[w] = word;
    }
    sha256_compress(st, blk);
  }
  LCV_UNROLL for (int k = 0; k < 8; ++k) b0.w[k] = st[k];
}

// u_m from a given b0 (the rest of expand_message_xmd + hash_to_field)
LCV_FN void hash_to_field_u_b0(fp2& u, const h256& b0, uint32_t m) {
  h256 prev, hi, lo;
  h256_zero(prev);
  LCV_NOUNROLL for (uint32_t k = 0; k <= m; ++k) {
    xmd_next(hi, b0, prev, 4 * k + 1);
    xmd_next(lo, b0, hi, 4 * k + 2);
    fp_from_xmd64(u.c0, hi, lo);
    xmd_next(hi, b0, lo, 4 * k + 3);
    xmd_next(lo, b0, hi, 4 * k + 4);
    fp_from_xmd64(u.c1, hi, lo);
    prev = lo;
  }
}

LCV_FN void hash_to_field_u(fp2& u, const h256& msg, uint32_t m) {
  h256 b0, prev, hi, lo;
  xmd_b0(b0, msg);
  h256_zero(prev);
  LCV_NOUNROLL for (uint32_t k = 0; k <= m; ++k) {
    xmd_next(hi, b0, prev, 4 * k + 1);
    xmd_next(lo, b0, hi, 4 * k + 2);
    fp_from_xmd64(u.c0, hi, lo);
    xmd_next(hi, b0, lo, 4 * k + 3);
    xmd_next(lo, b0, hi, 4 * k + 4);
    fp_from_xmd64(u.c1, hi, lo);
    prev = lo;
  }
}

// H(m) in G2 (Jacobian) for a 32-byte message given as 8 big-endian words
LCV_FN void hash_to_g2(g2j& r, const h256& msg) {
  h256 b0, prev, hi, lo;
  xmd_b0(b0, msg);
  h256_zero(prev);
  g2j acc;
  jac_set_inf(acc);
  LCV_NOUNROLL for (uint32_t m = 0; m < 2; ++m) {
    fp2 u;
    xmd_next(hi, b0, prev, 4 * m + 1);
    xmd_next(lo, b0, hi, 4 * m + 2);
    fp_from_xmd64(u.c0, hi, lo);
    xmd_next(hi, b0, lo, 4 * m + 3);
    xmd_next(lo, b0, hi, 4 * m + 4);
    fp_from_xmd64(u.c1, hi, lo);
    prev = lo;
    g2j q;
    map_to_curve_g2(q, u);
    jac_add(acc, acc, q);
  }
  g2_clear_cofactor(r, acc);
}

}  // namespace lcv
