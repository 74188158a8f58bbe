// lcv_tower.hpp — Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v), xi = 1 + u.
// Coefficient view used by Frobenius: f = sum_i g_i w^i with c0 = (g0, g2, g4), c1 = (g1, g3, g5).
#pragma once
#include "lcv_field.hpp"

namespace lcv {

struct fp6 { fp2 c0, c1, c2; };
struct fp12 { fp6 c0, c1; };

LCV_FN void fp6_zero(fp6& r) { fp2_zero(r.c0); fp2_zero(r.c1); fp2_zero(r.c2); }
LCV_FN void fp6_add(fp6& r, const fp6& a, const fp6& b) { fp2_add(r.c0, a.c0, b.c0); fp2_add(r.c1, a.c1, b.c1); fp2_add(r.c2, a.c2, b.c2); }
LCV_FN void fp6_sub(fp6& r, const fp6& a, const fp6& b) { fp2_sub(r.c0, a.c0, b.c0); fp2_sub(r.c1, a.c1, b.c1); fp2_sub(r.c2, a.c2, b.c2); }
LCV_FN void fp6_neg(fp6& r, const fp6& a) { fp2_neg(r.c0, a.c0); fp2_neg(r.c1, a.c1); fp2_neg(r.c2, a.c2); }
LCV_FN bool fp6_eq(const fp6& a, const fp6& b) { return fp2_eq(a.c0, b.c0) && fp2_eq(a.c1, b.c1) && fp2_eq(a.c2, b.c2); }

// r = a * v  (v^3 = xi)
LCV_FN void fp6_mul_by_v(fp6& r, const fp6& a) {
  fp2 t;
  fp2_mul_xi(t, a.c2);
  r.c2 = a.c1;
  r.c1 = a.c0;
  r.c0 = t;
}

// Karatsuba, 6 Fp2 multiplications.  r may alias a or b.
LCV_FN void fp6_mul(fp6& r, const fp6& a, const fp6& b) {
  fp2 t0, t1, t2, s0, s1, x0, x1, x2;
  fp2_mul(t0, a.c0, b.c0);
  fp2_mul(t1, a.c1, b.c1);
  fp2_mul(t2, a.c2, b.c2);
  // c0 = ((a1 + a2)(b1 + b2) - t1 - t2) xi + t0
  fp2_add(s0, a.c1, a.c2);
  fp2_add(s1, b.c1, b.c2);
  fp2_mul(x0, s0, s1);
  fp2_sub(x0, x0, t1);
  fp2_sub(x0, x0, t2);
  fp2_mul_xi(x0, x0);
  fp2_add(x0, x0, t0);
  // c1 = (a0 + a1)(b0 + b1) - t0 - t1 + xi t2
  fp2_add(s0, a.c0, a.c1);
  fp2_add(s1, b.c0, b.c1);
  fp2_mul(x1, s0, s1);
  fp2_sub(x1, x1, t0);
  fp2_sub(x1, x1, t1);
  fp2_mul_xi(s0, t2);
  fp2_add(x1, x1, s0);
  // c2 = (a0 + a2)(b0 + b2) - t0 - t2 + t1
  fp2_add(s0, a.c0, a.c2);
  fp2_add(s1, b.c0, b.c2);
  fp2_mul(x2, s0, s1);
  fp2_sub(x2, x2, t0);
  fp2_sub(x2, x2, t2);
  fp2_add(x2, x2, t1);
  r.c0 = x0;
  r.c1 = x1;
  r.c2 = x2;
}

LCV_FN void fp6_sqr(fp6& r, const fp6& a) { fp6_mul(r, a, a); }

LCV_FN void fp6_inv(fp6& r, const fp6& a) {
  fp2 t0, t1, t2, x, d;
  // t0 = a0^2 - xi a1 a2
  fp2_sqr(t0, a.c0);
  fp2_mul(x, a.c1, a.c2);
  fp2_mul_xi(x, x);
  fp2_sub(t0, t0, x);
  // t1 = xi a2^2 - a0 a1
  fp2_sqr(t1, a.c2);
  fp2_mul_xi(t1, t1);
  fp2_mul(x, a.c0, a.c1);
  fp2_sub(t1, t1, x);
  // t2 = a1^2 - a0 a2
  fp2_sqr(t2, a.c1);
  fp2_mul(x, a.c0, a.c2);
  fp2_sub(t2, t2, x);
  // d = a0 t0 + xi (a2 t1 + a1 t2)
  fp2_mul(d, a.c2, t1);
  fp2_mul(x, a.c1, t2);
  fp2_add(d, d, x);
  fp2_mul_xi(d, d);
  fp2_mul(x, a.c0, t0);
  fp2_add(d, d, x);
  fp2_inv(d, d);
  fp2_mul(r.c0, t0, d);
  fp2_mul(r.c1, t1, d);
  fp2_mul(r.c2, t2, d);
}

// ============================================================================ Fp12
LCV_FN void fp12_one(fp12& r) { fp6_zero(r.c0); fp6_zero(r.c1); fp2_one(r.c0.c0); }
LCV_FN bool fp12_eq(const fp12& a, const fp12& b) { return fp6_eq(a.c0, b.c0) && fp6_eq(a.c1, b.c1); }
LCV_FN bool fp12_is_one(const fp12& a) {
  fp12 one;
  fp12_one(one);
  return fp12_eq(a, one);
}
LCV_FN void fp12_conj(fp12& r, const fp12& a) { r.c0 = a.c0; fp6_neg(r.c1, a.c1); }

// Karatsuba over Fp6: 3 Fp6 multiplications (18 Fp2).  r may alias a or b.
LCV_FN void fp12_mul_inl(fp12& r, const fp12& a, const fp12& b) {
  fp6 t0, t1, s0, s1;
  fp6_mul(t0, a.c0, b.c0);
  fp6_mul(t1, a.c1, b.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_add(s1, b.c0, b.c1);
  fp6_mul(s0, s0, s1);
  fp6_sub(s0, s0, t0);
  fp6_sub(r.c1, s0, t1);
  fp6_mul_by_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}

// complex squaring: c0 = (a0 + a1)(a0 + v a1) - t - v t, c1 = 2t, t = a0 a1
LCV_FN void fp12_sqr(fp12& r, const fp12& a) {
  fp6 t, s0, s1;
  fp6_mul(t, a.c0, a.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_mul_by_v(s1, a.c1);
  fp6_add(s1, s1, a.c0);
  fp6_mul(s0, s0, s1);
  fp6_sub(s0, s0, t);
  fp6_mul_by_v(s1, t);
  fp6_sub(r.c0, s0, s1);
  fp6_add(r.c1, t, t);
}

LCV_FN void fp12_inv_inl(fp12& r, const fp12& a) {
  fp6 t0, t1;
  fp6_sqr(t0, a.c0);
  fp6_sqr(t1, a.c1);
  fp6_mul_by_v(t1, t1);
  fp6_sub(t0, t0, t1);
  fp6_inv(t0, t0);
  fp6_mul(r.c0, a.c0, t0);
  fp6_mul(t1, a.c1, t0);
  fp6_neg(r.c1, t1);
}

// Out-of-line on the device: a full Fp12 product is ~54 Fp multiplications of straight-line code;
// one shared copy per kernel keeps the final-exponentiation kernels small (and quick to compile).
LCV_OUTLINE void fp12_mul(fp12& r, const fp12& a, const fp12& b) { fp12_mul_inl(r, a, b); }
LCV_OUTLINE void fp12_inv(fp12& r, const fp12& a) { fp12_inv_inl(r, a); }

// Frobenius^k: g_i -> conj^k(g_i) * xi^(i (p^k - 1)/6)
#define LCV_FROB_APPLY(K, g, i, CONJ)            \
  do {                                           \
    fp2 _c;                                      \
    LCV_FP2_SET(_c, LCV_FROB##K##_##i);          \
    if (CONJ) fp2_conj(g, g);                    \
    fp2_mul(g, g, _c);                           \
  } while (0)

LCV_FN void fp12_frob1(fp12& r, const fp12& a) {
  r = a;
  fp2_conj(r.c0.c0, r.c0.c0);
  LCV_FROB_APPLY(1, r.c1.c0, 1, true);
  LCV_FROB_APPLY(1, r.c0.c1, 2, true);
  LCV_FROB_APPLY(1, r.c1.c1, 3, true);
  LCV_FROB_APPLY(1, r.c0.c2, 4, true);
  LCV_FROB_APPLY(1, r.c1.c2, 5, true);
}
LCV_FN void fp12_frob2(fp12& r, const fp12& a) {
  r = a;
  LCV_FROB_APPLY(2, r.c1.c0, 1, false);
  LCV_FROB_APPLY(2, r.c0.c1, 2, false);
  LCV_FROB_APPLY(2, r.c1.c1, 3, false);
  LCV_FROB_APPLY(2, r.c0.c2, 4, false);
  LCV_FROB_APPLY(2, r.c1.c2, 5, false);
}

// Granger-Scott squaring for elements of the cyclotomic subgroup.  With Fp4 = Fp2[s]/(s^2 - xi),
// s = w^3, f = A + B w + C w^2 (A = g0 + g3 s, B = g1 + g4 s, C = g2 + g5 s):
//   f^2 = (3A^2 - 2 conj(A)) + (3 s C^2 + 2 conj(B)) w + (3 B^2 - 2 conj(C)) w^2.
LCV_FN void fp4_sqr(fp2& r0, fp2& r1, const fp2& x0, const fp2& x1) {
  // (x0 + x1 s)^2 = (x0^2 + xi x1^2) + 2 x0 x1 s
  fp2 t0, t1, t2;
  fp2_sqr(t0, x0);
  fp2_sqr(t1, x1);
  fp2_add(t2, x0, x1);
  fp2_sqr(t2, t2);
  fp2_sub(t2, t2, t0);
  fp2_sub(r1, t2, t1);
  fp2_mul_xi(t1, t1);
  fp2_add(r0, t0, t1);
}
LCV_FN void fp12_cyclotomic_sqr(fp12& r, const fp12& a) {
  const fp2& g0 = a.c0.c0; const fp2& g2 = a.c0.c1; const fp2& g4 = a.c0.c2;
  const fp2& g1 = a.c1.c0; const fp2& g3 = a.c1.c1; const fp2& g5 = a.c1.c2;
  fp2 A0, A1, B0, B1, C0, C1, t;
  fp4_sqr(A0, A1, g0, g3);  // A^2
  fp4_sqr(B0, B1, g1, g4);  // B^2
  fp4_sqr(C0, C1, g2, g5);  // C^2
  fp12 z;
  // g0' = 3 A0 - 2 g0 ; g3' = 3 A1 + 2 g3
  fp2_sub(t, A0, g0); fp2_dbl(t, t); fp2_add(z.c0.c0, t, A0);
  fp2_add(t, A1, g3); fp2_dbl(t, t); fp2_add(z.c1.c1, t, A1);
  // s C^2 = xi C1 + C0 s:  g1' = 3 xi C1 + 2 g1 ; g4' = 3 C0 - 2 g4
  fp2 xc1;
  fp2_mul_xi(xc1, C1);
  fp2_add(t, xc1, g1); fp2_dbl(t, t); fp2_add(z.c1.c0, t, xc1);
  fp2_sub(t, C0, g4); fp2_dbl(t, t); fp2_add(z.c0.c2, t, C0);
  // g2' = 3 B0 - 2 g2 ; g5' = 3 B1 + 2 g5
  fp2_sub(t, B0, g2); fp2_dbl(t, t); fp2_add(z.c0.c1, t, B0);
  fp2_add(t, B1, g5); fp2_dbl(t, t); fp2_add(z.c1.c2, t, B1);
  r = z;
}

// f * L for the sparse line L = a + b v + c v w  (coefficients of w^0, w^2, w^3):
// L0 = a + b v, L1 = c v.  15 Fp2 multiplications.
LCV_FN void fp12_mul_line(fp12& f, const fp2& a, const fp2& b, const fp2& c) {
  const fp6& F0 = f.c0;
  const fp6& F1 = f.c1;
  fp6 x, y, z;
  fp2 t0, t1, t2, s;
  // x = F0 * (a + b v) = (f0 a + xi f2 b) + (f0 b + f1 a) v + (f1 b + f2 a) v^2   [Karatsuba-ish, 5 mul]
  fp2_mul(t0, F0.c0, a);
  fp2_mul(t1, F0.c1, b);
  fp2_mul(t2, F0.c2, b);
  fp2_mul_xi(t2, t2);
  fp2_add(x.c0, t0, t2);
  fp2_add(s, a, b);
  fp2_add(t2, F0.c0, F0.c1);
  fp2_mul(t2, t2, s);
  fp2_sub(t2, t2, t0);
  fp2_sub(x.c1, t2, t1);
  fp2_mul(t2, F0.c2, a);
  fp2_add(x.c2, t1, t2);
  // y = F1 * (c v) = xi g2 c + g0 c v + g1 c v^2   [3 mul]
  fp2_mul(t0, F1.c2, c);
  fp2_mul_xi(y.c0, t0);
  fp2_mul(y.c1, F1.c0, c);
  fp2_mul(y.c2, F1.c1, c);
  // z = (F0 + F1) * (a + (b + c) v)   [6 mul, schoolbook over the 2-term operand]
  fp6 h;
  fp6_add(h, F0, F1);
  fp2 bc;
  fp2_add(bc, b, c);
  fp2_mul(t0, h.c0, a);
  fp2_mul(t1, h.c2, bc);
  fp2_mul_xi(t1, t1);
  fp2_add(z.c0, t0, t1);
  fp2_mul(t0, h.c0, bc);
  fp2_mul(t1, h.c1, a);
  fp2_add(z.c1, t0, t1);
  fp2_mul(t0, h.c1, bc);
  fp2_mul(t1, h.c2, a);
  fp2_add(z.c2, t0, t1);
  // c1 = z - x - y ; c0 = x + v y
  fp6_sub(z, z, x);
  fp6_sub(f.c1, z, y);
  fp6_mul_by_v(y, y);
  fp6_add(f.c0, x, y);
}

}  // namespace lcv
