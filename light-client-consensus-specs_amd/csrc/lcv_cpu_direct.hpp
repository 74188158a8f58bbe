// lcv_cpu_direct.hpp — CPU-BASELINE build only (liblcv_cpu.so, -DLCV_CPU_FAST; bench.py's
// cpu_baseline leg).  On a CPU core the team programs' lane interpreter is pure overhead, so this
// build runs the BLS half of validate_light_client_update (sync-protocol.md:464) as direct per-update
// code over the same field / tower / curve functions as the device: signature decode + psi subgroup
// check, hash_to_G2, both Miller loops with a shared accumulator and the final exponentiation (the
// same hard-part chain as tools/gen_programs.py::fexp_program, result e^3).  The product (liblcv.so)
// never includes this file.
#pragma once
#include "lcv_h2c.hpp"
#include "lcv_items.hpp"
#include "lcv_pairing.hpp"
#include "lcv_tower.hpp"

namespace lcv {

LCV_FN void item_sig_direct(uint32_t i, const BatchDev& B, const Work& W) {
  g2a s;
  fp2_zero(s.x);
  fp2_zero(s.y);
  int st = g2_decompress(s, B.sig + 96 * (size_t)i);
  if (st == PT_OK && !g2_in_subgroup(s)) st = PT_BAD;
  st_g2a(W.qs, W.cap, i, s);
  W.sig_status[i] = (uint8_t)st;
}

LCV_FN void item_h2c_direct(uint32_t i, const Work& W) {
  h256 msg;
  soa_ld_h256(msg, W.msg, W.cap, i);
  g2j h;
  hash_to_g2(h, msg);
  const bool inf = jac_is_inf(h);
  g2a a;
  jac_to_aff(a, h);
  st_g2a(W.qh, W.cap, i, a);
  W.qh_inf[i] = inf ? 1 : 0;
}

LCV_FN void item_pairing_direct(uint32_t i, const Work& W) {
  // e(P1, Q1) e(P2, Q2): Q1 = H(m), P1 = aggregate pubkey; Q2 = signature, P2 = -G1.  An identity Q_k
  // becomes (G2 generator, P_k = (0, 0)): constant lines, killed by the final exponentiation.
  const bool id[2] = {W.qh_inf[i] != 0, W.sig_status[i] != PT_OK};
  g2a Q[2];
  fp nx[2], y[2];
  if (id[0]) g2_generator(Q[0]); else ld_g2a(Q[0], W.qh, W.cap, i);
  if (id[1]) g2_generator(Q[1]); else ld_g2a(Q[1], W.qs, W.cap, i);
  soa_ld_fp(nx[0], W.pk, W.cap, i, 0);
  fp_neg(nx[0], nx[0]);
  soa_ld_fp(y[0], W.pk, W.cap, i, 1);
  LCV_FP_SET(nx[1], LCV_G1X_INIT);
  fp_neg(nx[1], nx[1]);
  LCV_FP_SET(y[1], LCV_G1NEGY_INIT);
  for (int k = 0; k < 2; ++k)
    if (id[k]) { fp_zero(nx[k]); fp_zero(y[k]); }
  g2j T[2];
  for (int k = 0; k < 2; ++k) { T[k].x = Q[k].x; T[k].y = Q[k].y; fp2_one(T[k].z); }
  fp12 f;
  fp12_one(f);
  for (int bit = 62; bit >= 0; --bit) {
    fp12_sqr(f, f);
    for (int k = 0; k < 2; ++k) {
      line3 L;
      line_dbl(T[k], L);
      fp12_apply_line(f, L, nx[k], y[k]);
    }
    if ((LCV_X_ABS >> bit) & 1ull) {
      for (int k = 0; k < 2; ++k) {
        line3 L;
        line_add(T[k], L, Q[k]);
        fp12_apply_line(f, L, nx[k], y[k]);
      }
    }
  }
  fp12_conj(f, f);  // x < 0
  // final exponentiation: easy part, then the hard part (x-1)^2 (x+p)(x^2+p^2-1) + 3 -> e^3
  fp12 m, a, a2, bv, t, c, u;
  final_exp_easy(m, f);
  fp12_exp_xabs(t, m);
  fp12_mul(a, t, m);
  fp12_conj(a, a);
  fp12_exp_xabs(t, a);
  fp12_mul(a2, t, a);
  fp12_conj(a2, a2);
  fp12_exp_xabs(t, a2);
  fp12_conj(t, t);
  fp12_frob1(u, a2);
  fp12_mul(bv, t, u);
  fp12_exp_xabs(t, bv);
  fp12_exp_xabs(t, t);
  fp12_frob2(u, bv);
  fp12_mul(c, t, u);
  fp12_conj(u, bv);
  fp12_mul(c, c, u);
  fp12_cyclotomic_sqr(u, m);
  fp12_mul(u, u, m);
  fp12_mul(c, c, u);
  W.pair_ok[i] = fp12_is_one(c) ? 1 : 0;
}

}  // namespace lcv
