"""Canonical-algorithm operation counter — TEST / MEASUREMENT INFRASTRUCTURE ONLY (oracle/).

The roofline numerator of SURVEY.md §8(d): W = 600 N_fpmul + 24 N_fpadd + 2100 N_sha INT32 ops per
update, with "N_* from the oracle's op counter on the canonical algorithm".  This module runs the
verification of one light-client update (reference `sync-protocol.md:386-465`, FastAggregateVerify at
`:464`) with textbook algorithms over a COUNTING Fp type, checks every result against the definitional
oracle (`oracle/bls12_381.py`: affine formulas, definitional final exponentiation, r * P membership), and
reports the counts per device stage.  Only tests/ and tools/ import it; the product path never does.

Counted: Fp multiplications M and squarings S (both are "fp_mul" in the op model), Fp additions,
subtractions, negations and multiplications by small integers A ("fp_add"; k * a counts as its
double-and-add chain), SHA-256 compressions (oracle/ssz.py and the expand_message_xmd of
oracle/bls12_381.py count ceil((len + 9) / 64) per call).  Known-zero operands (sparse line values) are
skipped, as a sparse multiplication does.

The canonical algorithms (the standard efficient textbook ones; none is the device's SOP program):
  * Fp: Montgomery multiplication (one M / S each); inversion by Fermat a^(p-2), square roots a^((p+1)/4)
    and Legendre symbols a^((p-1)/2) by left-to-right binary exponentiation.
  * Tower Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3 - (1+u)), Fp12 = Fp6[w]/(w^2 - v), two models:
      - "karatsuba" (the conservative, lower count; the default): Fp2 mul 3M, Fp2 sqr 2M (complex),
        Fp6 mul 6 Fp2 mul, Fp6 sqr Chung-Hasan SQR2 (2 mul + 3 sqr), Fp12 mul 3 Fp6 mul, Fp12 sqr 2 Fp6
        mul (complex);
      - "schoolbook" (Karatsuba-free): Fp2 mul 4M, Fp2 sqr 2S + 1M, Fp6 mul 9 Fp2 mul,
        Fp6 sqr 3 Fp2 sqr + 3 Fp2 mul, Fp12 mul 4 Fp6 mul, Fp12 sqr 2 Fp6 sqr + 1 Fp6 mul;
    cyclotomic squaring: Granger-Scott (three Fp4 squarings) in both; Frobenius maps by constant Fp2
    multiplications.
  * G1 aggregation: Jacobian mixed additions (madd-2007-bl, 7M + 4S) over the participants,
    or — above 256 participants — the committee's precomputed sum (per committee, like KeyValidate)
    minus the non-participants (SURVEY §8(a) a13's complement form), then one conversion to affine.
  * Signature decode: y^2 = x^3 + 4(1 + u), Fp2 square root by the norm method (two Fp square roots and
    one Fermat inversion), as py_ecc's rules require; G2 membership: Scott's psi(Q) == [x]Q with [|x|]Q in
    homogeneous projective coordinates (63 doublings, 5 additions).
  * hash_to_G2 (RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_): expand_message_xmd (SHA-256), four 512-bit
    reductions mod p (2 M each), simplified SWU per RFC 9380 §6.6.2 (one Fp2 inversion, an is_square by
    the norm's Legendre symbol, one Fp2 square root), the 3-isogeny by Horner's rule in projective form
    (no inversion), projective Q0 + Q1, clear_cofactor by RFC 9380 G.3 (Budroni-Pintore: two [x]
    multiplications, psi, psi^2), one Fp2 inversion to affine.
  * Pairing check e(PK, H(m)) e(-G1, sig) == 1: optimal ate Miller loop over |x| with one shared Fp12
    accumulator (f <- f^2, then one sparse line multiplication per pairing and step), T in homogeneous
    projective coordinates with Costello-Lange-Naehrig lines (doubling: l = (Y^2 - 3b'Z^2) - 3X^2 x_P w^2
    + 2YZ y_P w^3), final exponentiation: easy part (p^6 - 1)(p^2 + 1) with one Fp12 inversion, hard part
    by Hayashida-Hayasaka-Teruya: 3 (p^4 - p^2 + 1)/r = (x - 1)^2 (x + p)(x^2 + p^2 - 1) + 3 (five
    exponentiations by |x|: 63 cyclotomic squarings + 5 multiplications each).
  * SSZ / SHA-256: the oracle's own merkleization (oracle/ssz.py), the reference's calls.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

from . import bls12_381 as B
from . import ssz as Z

P = B.P
X_ABS = B.X_ABS


# ----------------------------------------------------------------------------- counting Fp
class Ops:
    __slots__ = ("M", "S", "A")

    def __init__(self):
        self.M = self.S = self.A = 0

    def snap(self):
        return (self.M, self.S, self.A)


OPS = Ops()
MODE = {"tower": "karatsuba"}


class Fp:
    __slots__ = ("v",)

    def __init__(self, v: int):
        self.v = v % P

    def __add__(self, o):
        OPS.A += 1
        return Fp(self.v + o.v)

    def __sub__(self, o):
        OPS.A += 1
        return Fp(self.v - o.v)

    def __neg__(self):
        OPS.A += 1
        return Fp(-self.v)

    def __mul__(self, o):
        OPS.M += 1
        return Fp(self.v * o.v)

    def sq(self):
        OPS.S += 1
        return Fp(self.v * self.v)

    def small(self, k: int):
        """k * a for a small integer k >= 1: its double-and-add chain of additions."""
        OPS.A += (k.bit_length() - 1) + (bin(k).count("1") - 1)
        return Fp(self.v * k)

    def pow(self, e: int):
        r = self
        for bit in bin(e)[3:]:
            r = r.sq()
            if bit == "1":
                r = r * self
        return r

    def inv(self):
        return self.pow(P - 2)

    def is_zero(self):
        return self.v == 0

    def __eq__(self, o):
        return self.v == o.v


FP0 = 0  # sentinel for known-zero Fp2 coefficients (sparse values): operations with it are free


class Fp2:
    __slots__ = ("a", "b")

    def __init__(self, a: Fp, b: Fp):
        self.a, self.b = a, b

    @staticmethod
    def of(t) -> "Fp2":
        return Fp2(Fp(t[0]), Fp(t[1]))

    def t(self) -> Tuple[int, int]:
        return (self.a.v, self.b.v)

    def __add__(self, o):
        if o is FP0:
            return self
        return Fp2(self.a + o.a, self.b + o.b)

    def __sub__(self, o):
        if o is FP0:
            return self
        return Fp2(self.a - o.a, self.b - o.b)

    def __neg__(self):
        return Fp2(-self.a, -self.b)

    def __mul__(self, o):
        if o is FP0:
            return FP0
        a0, a1, b0, b1 = self.a, self.b, o.a, o.b
        if MODE["tower"] == "karatsuba":
            v0, v1 = a0 * b0, a1 * b1
            return Fp2(v0 - v1, (a0 + a1) * (b0 + b1) - v0 - v1)
        return Fp2(a0 * b0 - a1 * b1, a0 * b1 + a1 * b0)

    def sq(self):
        a0, a1 = self.a, self.b
        if MODE["tower"] == "karatsuba":
            return Fp2((a0 + a1) * (a0 - a1), (a0 * a1).small(2))
        return Fp2(a0.sq() - a1.sq(), (a0 * a1).small(2))

    def mul_fp(self, k: Fp):
        return Fp2(self.a * k, self.b * k)

    def small(self, k: int):
        return Fp2(self.a.small(k), self.b.small(k))

    def mul_xi(self):  # * (1 + u)
        return Fp2(self.a - self.b, self.a + self.b)

    def conj(self):
        return Fp2(self.a, -self.b)

    def norm(self) -> Fp:
        return self.a.sq() + self.b.sq()

    def inv(self):
        ni = self.norm().inv()
        return Fp2(self.a * ni, -(self.b * ni))

    def pow(self, e: int):
        r = self
        for bit in bin(e)[3:]:
            r = r.sq()
            if bit == "1":
                r = r * self
        return r

    def is_zero(self):
        return self.a.v == 0 and self.b.v == 0

    def __eq__(self, o):
        return self.t() == o.t()


def _z(x):
    return x is FP0


def f2c(t) -> Fp2:
    """An Fp2 constant (not counted)."""
    return Fp2.of(t)


def _sum(*xs):
    acc = FP0
    for x in xs:
        acc = x if acc is FP0 else (acc if x is FP0 else acc + x)
    return acc


def _mxi(x):
    return FP0 if x is FP0 else x.mul_xi()


def _mul(x, y):
    return FP0 if (x is FP0 or y is FP0) else x * y


def _sq(x):
    return FP0 if x is FP0 else x.sq()


def _neg(x):
    return FP0 if x is FP0 else -x


def _sub(x, y):
    if y is FP0:
        return x
    if x is FP0:
        return -y
    return x - y


def _dbl(x):
    return FP0 if x is FP0 else x + x


# Fp6 = (c0, c1, c2) over Fp2, v^3 = xi
def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    if MODE["tower"] == "karatsuba":
        v0, v1, v2 = _mul(a0, b0), _mul(a1, b1), _mul(a2, b2)
        c0 = _sum(_mxi(_sub(_sub(_mul(_sum(a1, a2), _sum(b1, b2)), v1), v2)), v0)
        c1 = _sum(_sub(_sub(_mul(_sum(a0, a1), _sum(b0, b1)), v0), v1), _mxi(v2))
        c2 = _sum(_sub(_sub(_mul(_sum(a0, a2), _sum(b0, b2)), v0), v2), v1)
        return (c0, c1, c2)
    c0 = _sum(_mul(a0, b0), _mxi(_sum(_mul(a1, b2), _mul(a2, b1))))
    c1 = _sum(_mul(a0, b1), _mul(a1, b0), _mxi(_mul(a2, b2)))
    c2 = _sum(_mul(a0, b2), _mul(a1, b1), _mul(a2, b0))
    return (c0, c1, c2)


def f6_sqr(a):
    a0, a1, a2 = a
    if MODE["tower"] == "karatsuba":  # Chung-Hasan SQR2
        s0 = _sq(a0)
        s1 = _dbl(_mul(a0, a1))
        s2 = _sq(_sum(_sub(a0, a1), a2))
        s3 = _dbl(_mul(a1, a2))
        s4 = _sq(a2)
        c0 = _sum(_mxi(s3), s0)
        c1 = _sum(_mxi(s4), s1)
        c2 = _sub(_sub(_sum(s1, s2, s3), s0), s4)
        return (c0, c1, c2)
    s0, s1, s2 = _sq(a0), _sq(a1), _sq(a2)
    m01, m02, m12 = _dbl(_mul(a0, a1)), _dbl(_mul(a0, a2)), _dbl(_mul(a1, a2))
    return (_sum(s0, _mxi(m12)), _sum(m01, _mxi(s2)), _sum(m02, s1))


def f6_add(a, b):
    return tuple(_sum(x, y) for x, y in zip(a, b))


def f6_sub(a, b):
    return tuple(_sub(x, y) for x, y in zip(a, b))


def f6_neg(a):
    return tuple(_neg(x) for x in a)


def f6_mul_v(a):
    return (_mxi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    t0 = _sub(_sq(a0), _mxi(_mul(a1, a2)))
    t1 = _sub(_mxi(_sq(a2)), _mul(a0, a1))
    t2 = _sub(_sq(a1), _mul(a0, a2))
    d = _sum(_mul(a0, t0), _mxi(_sum(_mul(a2, t1), _mul(a1, t2))))
    di = d.inv()
    return (_mul(t0, di), _mul(t1, di), _mul(t2, di))


# Fp12 = (c0, c1) over Fp6, w^2 = v
def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    if MODE["tower"] == "karatsuba":
        t0, t1 = f6_mul(a0, b0), f6_mul(a1, b1)
        c1 = f6_sub(f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), t0), t1)
        return (f6_add(t0, f6_mul_v(t1)), c1)
    return (f6_add(f6_mul(a0, b0), f6_mul_v(f6_mul(a1, b1))), f6_add(f6_mul(a0, b1), f6_mul(a1, b0)))


def f12_sqr(a):
    a0, a1 = a
    if MODE["tower"] == "karatsuba":  # complex squaring
        t = f6_mul(a0, a1)
        c0 = f6_sub(f6_sub(f6_mul(f6_add(a0, a1), f6_add(a0, f6_mul_v(a1))), t), f6_mul_v(t))
        return (c0, f6_add(t, t))
    t = f6_mul(a0, a1)
    return (f6_add(f6_sqr(a0), f6_mul_v(f6_sqr(a1))), f6_add(t, t))


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    d = f6_sub(f6_sqr(a0), f6_mul_v(f6_sqr(a1)))
    di = f6_inv(d)
    return (f6_mul(a0, di), f6_neg(f6_mul(a1, di)))


def _fp4_sqr(a, b):
    """(a + b s)^2 in Fp4 = Fp2[s]/(s^2 - xi): (a^2 + xi b^2, 2ab)."""
    t0, t1 = a.sq(), b.sq()
    if MODE["tower"] == "karatsuba":
        return t0 + t1.mul_xi(), (a + b).sq() - t0 - t1
    return t0 + t1.mul_xi(), (a * b).small(2)


def f12_cyc_sqr(f):
    """Granger-Scott squaring of an element of the cyclotomic subgroup (after the easy part)."""
    (a00, a01, a02), (a10, a11, a12) = f
    t00, t01 = _fp4_sqr(a00, a11)
    t10, t11 = _fp4_sqr(a10, a02)
    t20, t21 = _fp4_sqr(a01, a12)
    t21x = t21.mul_xi()
    r00 = (t00 - a00).small(2) + t00
    r11 = (t01 + a11).small(2) + t01
    r10 = (t21x + a10).small(2) + t21x
    r02 = (t20 - a02).small(2) + t20
    r01 = (t10 - a01).small(2) + t10
    r12 = (t11 + a12).small(2) + t11
    return ((r00, r01, r02), (r10, r11, r12))


# Frobenius: coefficient g_i of w^i -> conj(g_i) * gamma_i^(k) (constants not counted)
_W = lambda f: [f[0][0], f[1][0], f[0][1], f[1][1], f[0][2], f[1][2]]  # noqa: E731
_UNW = lambda g: ((g[0], g[2], g[4]), (g[1], g[3], g[5]))  # noqa: E731
GAMMA = {k: [f2c(B.f2_pow(B.XI, i * (P ** k - 1) // 6)) for i in range(6)] for k in (1, 2)}


def f12_frob(f, k: int = 1):
    g = _W(f)
    out = []
    for i, c in enumerate(g):
        c = c.conj() if k % 2 else c
        gam = GAMMA[k][i]
        if i == 0:
            out.append(c)
        elif gam.b.v == 0:
            out.append(c.mul_fp(gam.a))
        else:
            out.append(c * gam)
    return _UNW(out)


def f12_from_oracle(t) -> tuple:
    return tuple(tuple(f2c(c) for c in c6) for c6 in t)


def f12_to_oracle(f):
    return tuple(tuple(c.t() for c in c6) for c6 in f)


def _cyc_exp_abs_x(f):
    """f^|x| in the cyclotomic subgroup: 63 Granger-Scott squarings + 5 multiplications."""
    r = f
    for bit in bin(X_ABS)[3:]:
        r = f12_cyc_sqr(r)
        if bit == "1":
            r = f12_mul(r, f)
    return r


def _exp_x(f):  # f^x, x < 0: conj(f^|x|) (inverse in the cyclotomic subgroup)
    return f12_conj(_cyc_exp_abs_x(f))


def final_exponentiation(f):
    """f^(3 (p^12 - 1) / r): easy part, then HHT's (x-1)^2 (x+p)(x^2+p^2-1) + 3."""
    f1 = f12_mul(f12_conj(f), f12_inv(f))          # f^(p^6 - 1)
    m = f12_mul(f12_frob(f1, 2), f1)                # ^(p^2 + 1): cyclotomic from here
    u = f12_mul(_exp_x(m), f12_conj(m))             # m^(x - 1)
    a = f12_mul(_exp_x(u), f12_conj(u))             # m^((x - 1)^2)
    b = f12_mul(_exp_x(a), f12_frob(a, 1))          # a^(x + p)
    c = f12_mul(f12_mul(_exp_x(_exp_x(b)), f12_frob(b, 2)), f12_conj(b))  # b^(x^2 + p^2 - 1)
    return f12_mul(c, f12_mul(f12_cyc_sqr(m), m))   # * m^3


# ----------------------------------------------------------------------------- G2 in homogeneous projective
B2 = f2c(B.B2)


def g2_dbl(T):
    """2T (homogeneous projective, a = 0): X3 = XY/2 (Y^2 - 9b'Z^2), Y3 = ((Y^2 + 9b'Z^2)/2)^2 - 27 b'^2 Z^4,
    Z3 = 2 Y^3 Z, computed with the halvings folded into a common factor 2: (2X3, 2Y3 * 2, 2Z3 * ...)."""
    X, Y, Z = T
    y2, z2 = Y.sq(), Z.sq()
    bz = (z2 * B2).small(3)           # 3 b' Z^2
    b9 = bz.small(3)                  # 9 b' Z^2
    xy = X * Y
    X3 = (xy * (y2 - b9)).small(2)    # 2 X Y (Y^2 - 9b'Z^2)          (= 4 * X3_true)
    s = y2 + b9
    Y3 = s.sq() - bz.sq().small(12)   # (Y^2 + 9b'Z^2)^2 - 108 b'^2 Z^4 (= 4 * Y3_true)
    Z3 = (y2 * (Y * Z)).small(8)      # 8 Y^3 Z                        (= 4 * Z3_true)
    return (X3, Y3, Z3), (y2, z2, bz, X, Y, Z)


def g2_add_mixed(T, Q):
    """T + Q, Q affine (add-1998-cmo-2 with Z2 = 1): u = yQ Z - Y, v = xQ Z - X."""
    X, Y, Z = T
    xq, yq = Q
    u = yq * Z - Y
    v = xq * Z - X
    uu, vv = u.sq(), v.sq()
    vvv = v * vv
    R = vv * X
    A = uu * Z - vvv - R.small(2)
    return (v * A, u * (R - A) - vvv * Y, vvv * Z), (u, v)


def g2_add(T, U):
    """T + U, both homogeneous projective (add-1998-cmo-2)."""
    X1, Y1, Z1 = T
    X2, Y2, Z2 = U
    y1z2, x1z2, z1z2 = Y1 * Z2, X1 * Z2, Z1 * Z2
    u = Y2 * Z1 - y1z2
    v = X2 * Z1 - x1z2
    uu, vv = u.sq(), v.sq()
    vvv = v * vv
    R = vv * x1z2
    A = uu * z1z2 - vvv - R.small(2)
    return (v * A, u * (R - A) - vvv * y1z2, vvv * z1z2)


def g2_neg(T):
    return (T[0], -T[1], T[2])


def g2_mul_abs_x(T):
    """[|x|]T: 63 doublings, 5 additions (x's Hamming weight is 6)."""
    R = T
    for bit in bin(X_ABS)[3:]:
        R, _ = g2_dbl(R)
        if bit == "1":
            R = g2_add(R, T)
    return R


def g2_to_affine(T):
    zi = T[2].inv()
    return (T[0] * zi, T[1] * zi)


PSI_CX, PSI_CY = f2c(B.PSI_CX), f2c(B.PSI_CY)
PSI2_CX = f2c(B.f2_mul(B.f2_conj(B.PSI_CX), B.PSI_CX))
PSI2_CY = f2c(B.f2_mul(B.f2_conj(B.PSI_CY), B.PSI_CY))


def g2_psi(T):
    return (T[0].conj() * PSI_CX, T[1].conj() * PSI_CY, T[2].conj())


def g2_psi2(T):  # psi(psi(T)): the constants are in Fp
    return (T[0].mul_fp(PSI2_CX.a), T[1].mul_fp(PSI2_CY.a), T[2])


# ----------------------------------------------------------------------------- stages
def _fp_sqrt(a: Fp) -> Optional[Fp]:
    y = a.pow((P + 1) // 4)
    return y if y.sq() == a else None


def fp2_sqrt(a: Fp2) -> Optional[Fp2]:
    """Norm method (as oracle f2_sqrt): alpha = sqrt(norm a), x0 = sqrt((a0 + alpha) / 2) (or with
    -alpha), x1 = a1 / (2 x0); the candidate is checked by one squaring."""
    if a.b.v == 0:
        r = _fp_sqrt(a.a)
        if r is not None:
            return Fp2(r, Fp(0))
        r = _fp_sqrt(-a.a)
        return Fp2(Fp(0), r) if r is not None else None
    alpha = _fp_sqrt(a.norm())
    if alpha is None:
        return None
    half = Fp((P + 1) // 2)
    x0 = _fp_sqrt((a.a + alpha) * half)
    if x0 is None:
        x0 = _fp_sqrt((a.a - alpha) * half)
        if x0 is None:
            return None
    y = Fp2(x0, a.b * x0.small(2).inv())
    return y if y.sq() == a else None


def sig_decode(sig: bytes):
    """96-byte compressed G2 -> affine point (py_ecc rules; flags / range checks cost nothing)."""
    q = B.g2_decompress(sig)  # the reference decoding's branch structure and validity (not counted)
    if q is None:
        return None
    x = f2c(q[0])
    y = fp2_sqrt(x.sq() * x + B2)
    assert y is not None
    if y.t() != q[1]:
        y = -y
    assert y.t() == q[1]
    return (x, y)


def g2_subgroup_psi(Q) -> bool:
    """Scott: psi(Q) == [x]Q, [x]Q = -[|x|]Q in projective form, compared without inversion."""
    X, Y, Z = g2_neg(g2_mul_abs_x((Q[0], Q[1], Fp2(Fp(1), Fp(0)))))
    px, py = Q[0].conj() * PSI_CX, Q[1].conj() * PSI_CY
    return X == px * Z and Y == py * Z


SSWU_Z, ISO_A, ISO_B = f2c(B.SSWU_Z), f2c(B.ISO_A), f2c(B.ISO_B)
MINUS_B_OVER_A = f2c(B.f2_mul(B.f2_neg(B.ISO_B), B.f2_inv(B.ISO_A)))
B_OVER_ZA = f2c(B.f2_mul(B.ISO_B, B.f2_inv(B.f2_mul(B.SSWU_Z, B.ISO_A))))


def _is_square_fp2(a: Fp2) -> bool:
    n = a.norm()
    return n.v == 0 or n.pow((P - 1) // 2).v == 1


def sswu(u: Fp2):
    """RFC 9380 §6.6.2 simplified SWU onto E2' (straight-line, exceptional case included)."""
    u2 = u.sq()
    zu2 = u2 * SSWU_Z
    den = zu2.sq() + zu2
    if den.is_zero():
        x1 = B_OVER_ZA
    else:
        x1 = (den.inv() + Fp2(Fp(1), Fp(0))) * MINUS_B_OVER_A
    gx1 = (x1.sq() + ISO_A) * x1 + ISO_B
    x2 = zu2 * x1
    gx2 = (x2.sq() + ISO_A) * x2 + ISO_B
    if _is_square_fp2(gx1):
        x, y = x1, fp2_sqrt(gx1)
    else:
        x, y = x2, fp2_sqrt(gx2)
    if B.sgn0_fp2(u.t()) != B.sgn0_fp2(y.t()):
        y = -y
    return x, y


ISO = {k: [f2c(c) for c in v] for k, v in (("xn", B.ISO_XNUM), ("xd", B.ISO_XDEN), ("yn", B.ISO_YNUM),
                                           ("yd", B.ISO_YDEN))}


def _horner(cs, x: Fp2) -> Fp2:
    acc = cs[-1]
    for c in reversed(cs[:-1]):
        acc = acc * x + c
    return acc


def iso_map_projective(pt):
    """3-isogeny E2' -> E2 in homogeneous projective form: (xn yd : y' yn xd : xd yd)."""
    x, y = pt
    xn, xd, yn, yd = (_horner(ISO[k], x) for k in ("xn", "xd", "yn", "yd"))
    return (xn * yd, y * (yn * xd), xd * yd)


def clear_cofactor(Pt):
    """RFC 9380 G.3: h_eff P = [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P), with c1 = x < 0."""
    t1 = g2_neg(g2_mul_abs_x(Pt))                 # [x]P
    t2 = g2_psi(Pt)
    t3 = g2_psi2(g2_dbl(Pt)[0])
    t3 = g2_add(t3, g2_neg(t2))
    t2 = g2_neg(g2_mul_abs_x(g2_add(t1, t2)))     # [x](t1 + t2)
    t3 = g2_add(t3, t2)
    t3 = g2_add(t3, g2_neg(t1))
    return g2_add(t3, g2_neg(Pt))


def hash_to_field(msg: bytes):
    """expand_message_xmd (SHA-256, counted by oracle/bls12_381.py) + four 512-bit reductions (2 M each)."""
    ub = B.expand_message_xmd(msg, B.DST_POP, 256)
    out = []
    for i in range(2):
        e = []
        for j in range(2):
            OPS.M += 2
            e.append(Fp(int.from_bytes(ub[64 * (2 * i + j):64 * (2 * i + j) + 64], "big")))
        out.append(Fp2(e[0], e[1]))
    return out


# G1 (Jacobian, a = 0)
def g1_madd(T, Q):
    """madd-2007-bl: T (Jacobian) + Q (affine), 7M + 4S."""
    X1, Y1, Z1 = T
    x2, y2 = Q
    z1z1 = Z1.sq()
    u2 = x2 * z1z1
    s2 = y2 * Z1 * z1z1
    h = u2 - X1
    hh = h.sq()
    i = hh.small(4)
    j = h * i
    r = (s2 - Y1).small(2)
    v = X1 * i
    X3 = r.sq() - j - v.small(2)
    Y3 = r * (v - X3) - (Y1 * j).small(2)
    Z3 = (Z1 + h).sq() - z1z1 - hh
    return (X3, Y3, Z3)


def g1_add_jac(T, U):
    """add-2007-bl: Jacobian + Jacobian (11M + 5S)."""
    X1, Y1, Z1 = T
    X2, Y2, Z2 = U
    z1z1, z2z2 = Z1.sq(), Z2.sq()
    u1, u2 = X1 * z2z2, X2 * z1z1
    s1, s2 = Y1 * Z2 * z2z2, Y2 * Z1 * z1z1
    h = u2 - u1
    i = h.small(2).sq()
    j = h * i
    r = (s2 - s1).small(2)
    v = u1 * i
    X3 = r.sq() - j - v.small(2)
    Y3 = r * (v - X3) - (s1 * j).small(2)
    Z3 = ((Z1 + Z2).sq() - z1z1 - z2z2) * h
    return (X3, Y3, Z3)


def g1_to_affine(T):
    zi = T[2].inv()
    zi2 = zi.sq()
    return (T[0] * zi2, T[1] * zi2 * zi)


def g1_aggregate(points, bits, committee_sum):
    """participants summed by mixed additions; above 256 participants the committee's
    precomputed sum (per committee) minus the non-participants."""
    sel = [p for p, b in zip(points, bits) if b]
    if len(sel) > 256:
        rest = [(p[0], -p[1]) for p, b in zip(points, bits) if not b]
        acc = committee_sum
        if rest:
            acc2 = (rest[0][0], rest[0][1], Fp(1))
            for q in rest[1:]:
                acc2 = g1_madd(acc2, q)
            acc = g1_add_jac(acc, acc2)
    else:
        acc = (sel[0][0], sel[0][1], Fp(1))
        for q in sel[1:]:
            acc = g1_madd(acc, q)
    return g1_to_affine(acc) if acc[2].v != 1 else (acc[0], acc[1])


# ----------------------------------------------------------------------------- Miller loop
def line_dbl(T, P1):
    """Doubling step: the line at T evaluated at P (CLN, scaled by an Fp2 factor) and 2T."""
    T2, (y2, z2, bz, X, Y, Z) = g2_dbl(T)
    xp, yp = P1
    c0 = y2 - bz                                   # Y^2 - 3 b' Z^2
    c2 = -((X.sq()).small(3).mul_fp(xp))           # -3 X^2 x_P   (w^2 = v)
    c3 = (Y * Z).small(2).mul_fp(yp)               # 2 Y Z y_P    (w^3 = v w)
    return T2, ((c0, c2, FP0), (FP0, c3, FP0))


def line_add(T, Q, P1):
    """Addition step: the line through T and Q evaluated at P, and T + Q."""
    T2, (u, v) = g2_add_mixed(T, Q)
    xp, yp = P1
    xq, yq = Q
    c0 = u * xq - v * yq                           # (slope x_Q - y_Q) * v
    c2 = -(u.mul_fp(xp))
    c3 = v.mul_fp(yp)
    return T2, ((c0, c2, FP0), (FP0, c3, FP0))


def miller_lines(P1, Q):
    """The T-walk of one pairing: the 68 sparse line values (stage `miller_lines` of the device)."""
    T = (Q[0], Q[1], Fp2(Fp(1), Fp(0)))
    lines = []
    for bit in bin(X_ABS)[3:]:
        T, l = line_dbl(T, P1)
        lines.append(l)
        if bit == "1":
            T, l = line_add(T, Q, P1)
            lines.append(l)
    return lines


def miller_acc(lines1, lines2):
    """f <- f^2 * l1 * l2 per doubling, f <- f * l1 * l2 after additions (shared accumulator)."""
    f = ((Fp2(Fp(1), Fp(0)), FP0, FP0), (FP0, FP0, FP0))
    k = 0
    first = True
    for bit in bin(X_ABS)[3:]:
        if not first:
            f = f12_sqr(f)
        f = f12_mul(f12_mul(f, lines1[k]), lines2[k]) if not first else f12_mul(lines1[k], lines2[k])
        first = False
        k += 1
        if bit == "1":
            f = f12_mul(f12_mul(f, lines1[k]), lines2[k])
            k += 1
    return f12_conj(f)


def _densify(f):
    return tuple(tuple(Fp2(Fp(0), Fp(0)) if c is FP0 else c for c in c6) for c6 in f)


# ----------------------------------------------------------------------------- one update, per stage
STAGES = ("pre_checks", "signing_root", "h2c_sswu", "hash_to_g2", "sig_decode", "g1_aggregate", "miller_lines",
          "miller_lines_sig", "miller_loop", "final_exp")


def _sha_total() -> int:
    return Z.SHA_COMPRESSIONS[0] + B.SHA_COMPRESSIONS[0]


class Stage:
    def __init__(self, out: Dict[str, dict], name: str):
        self.out, self.name = out, name

    def __enter__(self):
        self.m0, self.s0, self.a0 = OPS.snap()
        self.h0 = _sha_total()
        return self

    def __exit__(self, *exc):
        m, s, a = OPS.snap()
        d = self.out.setdefault(self.name, {"M": 0, "S": 0, "A": 0, "sha": 0})
        d["M"] += m - self.m0
        d["S"] += s - self.s0
        d["A"] += a - self.a0
        d["sha"] += _sha_total() - self.h0
        return False


def count_update(update, store, genesis_validators_root: bytes, committee_points=None, tower: str = "karatsuba"
                 ) -> Tuple[Dict[str, dict], Dict[str, dict], bool]:
    """Canonical counts of validating one update (oracle containers, oracle/sync_protocol.py), per device
    stage: (per_update, per_committee, verdict).  The update must pass every check before the signature
    (configs[1]-shaped: valid, all branches).  Every value is checked against the definitional oracle."""
    from . import spec as S
    from . import sync_protocol as O
    MODE["tower"] = tower
    per: Dict[str, dict] = {}
    per_comm: Dict[str, dict] = {}
    u = update
    with Stage(per_comm, "nsc_htr"):
        nsc_root = Z.hash_tree_root(u.next_sync_committee)
    with Stage(per, "pre_checks"):
        assert O.is_valid_light_client_header(u.attested_header)
        assert O.is_valid_light_client_header(u.finalized_header)
        fin_root = Z.hash_tree_root(u.finalized_header.beacon)
        assert S.is_valid_merkle_branch(fin_root, u.finality_branch, S.floorlog2(S.FINALIZED_ROOT_GINDEX),
                                        O.get_subtree_index(S.FINALIZED_ROOT_GINDEX), u.attested_header.beacon.state_root)
        assert S.is_valid_merkle_branch(nsc_root, u.next_sync_committee_branch, S.floorlog2(S.NEXT_SYNC_COMMITTEE_GINDEX),
                                        O.get_subtree_index(S.NEXT_SYNC_COMMITTEE_GINDEX),
                                        u.attested_header.beacon.state_root)
    with Stage(per, "signing_root"):
        msg = O.signing_root_of(u, genesis_validators_root)
    sig = bytes(u.sync_aggregate.sync_committee_signature)
    bits = list(u.sync_aggregate.sync_committee_bits)
    sig_period = O.compute_sync_committee_period_at_slot(u.signature_slot)
    store_period = O.compute_sync_committee_period_at_slot(store.finalized_header.beacon.slot)
    committee = store.current_sync_committee if sig_period == store_period else store.next_sync_committee
    pks = [bytes(pk) for pk in committee.pubkeys]
    if committee_points is None:
        committee_points = [B.g1_decompress(pk) for pk in pks]
    pts = [(Fp(p[0]), Fp(p[1])) for p in committee_points]
    # the committee's sum is per-committee work (precomputed once, like KeyValidate): not counted here
    saved = OPS.snap()
    csum = (pts[0][0], pts[0][1], Fp(1))
    for q in pts[1:]:
        csum = g1_madd(csum, q)
    OPS.M, OPS.S, OPS.A = saved
    with Stage(per, "h2c_sswu"):
        us = hash_to_field(msg)
        maps = [sswu(x) for x in us]
    with Stage(per, "hash_to_g2"):
        q0, q1 = (iso_map_projective(m) for m in maps)
        H = g2_to_affine(clear_cofactor(g2_add(q0, q1)))
    assert (H[0].t(), H[1].t()) == B.hash_to_g2(msg)
    with Stage(per, "sig_decode"):
        S2 = sig_decode(sig)
    with Stage(per, "g1_aggregate"):
        pk = g1_aggregate(pts, bits, csum)
    assert (pk[0].v, pk[1].v) == B.aggregate_pubkeys([p for p, b in zip(pks, bits) if b])
    with Stage(per, "miller_lines"):
        l1 = miller_lines(pk, H)
    with Stage(per, "miller_lines_sig"):
        in_g2 = g2_subgroup_psi(S2)
        ng = B.g1_neg(B.G1_GEN)
        l2 = miller_lines((Fp(ng[0]), Fp(ng[1])), S2)
    assert in_g2 == B.g2_in_subgroup((S2[0].t(), S2[1].t()))
    with Stage(per, "miller_loop"):
        f = miller_acc(l1, l2)
    with Stage(per, "final_exp"):
        e = final_exponentiation(_densify(f))
    one = f12_from_oracle(B.F12_ONE)
    verdict = in_g2 and f12_to_oracle(e) == f12_to_oracle(one)
    MODE["tower"] = "karatsuba"
    return per, per_comm, verdict


def as_opmodel(d: dict) -> dict:
    """{M, S, A, sha} -> the §8(d) op model's fp_mul / fp_add / sha / int32_ops."""
    fm = d["M"] + d["S"]
    return {"fp_mul": fm, "fp_add": d["A"], "sha": d["sha"], "fp_mul_detail": {"M": d["M"], "S": d["S"]},
            "int32_ops": 600 * fm + 24 * d["A"] + 2100 * d["sha"]}
