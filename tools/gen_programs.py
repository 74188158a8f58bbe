#!/usr/bin/env python3
"""Generate the team programs of liblcv.so (csrc/lcv_programs.inc): the Miller loop and the final
exponentiation of the two-pairing check inside FastAggregateVerify (reference call site
sync-protocol.md:464), compiled into ROUNDS of independent Fp operations for a team of T lanes.

Why: one lane per update leaves a 10^4-update batch with ~160 waves on a 1,024-SIMD chip, so the
pairing time is the latency of one lane's serial chain of ~17k Fp multiplications.  Here the Fp12 /
G2 formulas are TRACED symbolically (the same Karatsuba tower as lcv_tower.hpp): every Fp
multiplication becomes a MUL op whose operands are small linear combinations (+-coefficients) of
earlier values; additions are folded into those combinations or into LIN ops.  A list scheduler packs
the ops into rounds of at most T ops (critical path first); values live in per-update LDS slots
(linear-scan allocation, a slot is reused only in a later round than its last read, so every round
reads only what previous rounds wrote).  The device kernel (lcv_engine.hpp) is a small interpreter:
per round, lane t of a team evaluates its two combinations from LDS, multiplies (Montgomery, 12x32
limbs), stores the result.  Programs are straight-line (|x| is a constant), so they are data.

The generator also EMULATES every program on random inputs with Python integers and checks the
outputs against independent formulas (oracle/bls12_381.py), so a scheduling or allocation bug fails
here, not on the GPU.

    python tools/gen_programs.py [--team 32] [--check]
"""
from __future__ import annotations

import argparse
import heapq
import os
import random
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
X_ABS = 0xD201000000010000
RM = 1 << 384
KOP = 4            # max terms of a MUL operand combination (longer ones are materialised by LIN ops)
KLIN = 11          # max terms of one LIN op (record halfwords 1..11)
REC_HW = 16        # uint16 per lane record: dst, A terms from 1, B terms from B_AT
B_AT = 12          # MUL operand B at rec[12..15] (KOP <= 4)
COEF_MAX = 7       # term coefficients are signed 4-bit
SLOT_NONE = 0xFFF
CONST_BASE = 3072  # slots >= CONST_BASE index the constant table


# ============================================================================ symbolic values
class Val:
    __slots__ = ("id", "kind", "a", "b", "name", "const", "round", "slot", "last_use", "readers")

    def __init__(self, vid, kind, a=None, b=None, name=None, const=None):
        self.id, self.kind, self.a, self.b, self.name, self.const = vid, kind, a, b, name, const
        self.round, self.slot, self.last_use, self.readers = None, None, -1, []

    def __lt__(self, o):
        return self.id < o.id

    def __repr__(self):
        return f"V{self.id}:{self.kind}"


class Tracer:
    def __init__(self):
        self.vals = []
        self.consts = {}   # value -> Val
        self.inputs = {}   # name -> Val
        self.lin_cache = {}

    def _new(self, kind, **kw):
        v = Val(len(self.vals), kind, **kw)
        self.vals.append(v)
        return v

    def input(self, name):
        v = self._new("in", name=name)
        self.inputs[name] = v
        return F(self, {v: 1})

    def const(self, value):
        value %= P
        if value == 0:
            return F(self, {})
        if value not in self.consts:
            self.consts[value] = self._new("const", const=value)
        return F(self, {self.consts[value]: 1})

    def one(self):
        return self.const(1)

    def _operand(self, f):
        if len(f.t) > KOP or any(abs(c) > COEF_MAX for c in f.t.values()):
            return {self.lin(f): 1}
        return dict(f.t)

    def lin(self, f, name=None):
        """Materialise a combination (split into chained LIN ops of <= KLIN terms)."""
        key = tuple(sorted((v.id, c) for v, c in f.t.items()))
        if name is None and key in self.lin_cache:
            return self.lin_cache[key]
        items = list(f.t.items())
        big = [(v, c) for v, c in items if abs(c) > COEF_MAX]
        terms = [(v, c) for v, c in items if abs(c) <= COEF_MAX]
        for v, c in big:  # large coefficients: split c = q*7 + r through doubling chains
            s = -1 if c < 0 else 1
            c = abs(c)
            while c > COEF_MAX:
                terms.append((v, s * COEF_MAX))
                c -= COEF_MAX
            if c:
                terms.append((v, s * c))
        def too_big(ts):  # the device accumulator holds < 2^6 p: sum |coef| <= 63 per op
            return len(ts) > KLIN or sum(abs(c) for _, c in ts) > 60
        while too_big(terms):
            cut = 1
            while cut < len(terms) and not too_big(terms[:cut + 1]):
                cut += 1
            hv = self._new("lin", a=list(terms[:cut]))
            terms = [(hv, 1)] + terms[cut:]
        out = self._new("lin", a=list(terms), name=name)
        if name is None:
            self.lin_cache[key] = out
        return out

    def mul(self, x, y):
        # constant folding: 0, +-small constants, products of constants
        if not x.t or not y.t:
            return F(self, {})
        cx, cy = x.const_value(), y.const_value()
        if cx is not None and cy is not None:
            return self.const(cx * cy)
        for u, w in ((x, y), (y, x)):
            c = u.const_value()
            if c is not None:
                for small in range(-COEF_MAX, COEF_MAX + 1):
                    if small and c == small % P:
                        return w * small
        a, b = self._operand(x), self._operand(y)
        return F(self, {self._new("mul", a=a, b=b): 1})

    def inv(self, x):
        return F(self, {self._new("inv", a=self._operand(x)): 1})


def _merge(terms):
    d = defaultdict(int)
    for v, c in terms:
        d[v] += c
    return {v: c for v, c in d.items() if c}


class F:
    """An Fp value as a linear combination of materialised Vals."""
    __slots__ = ("tr", "t")

    def __init__(self, tr, t):
        self.tr, self.t = tr, {v: c for v, c in t.items() if c}

    def const_value(self):
        if all(v.kind == "const" for v in self.t):
            return sum(v.const * c for v, c in self.t.items()) % P
        return None

    def __add__(self, o):
        d = defaultdict(int, self.t)
        for v, c in o.t.items():
            d[v] += c
        return F(self.tr, d)

    def __sub__(self, o):
        return self + o * -1

    def __neg__(self):
        return self * -1

    def __mul__(self, o):
        if isinstance(o, int):
            return F(self.tr, {v: c * o for v, c in self.t.items()})
        return self.tr.mul(self, o)

    def dbl(self):
        return self * 2

    def mat(self):
        """Force materialisation (a LIN op) — used for values read by many later products."""
        if len(self.t) == 1 and next(iter(self.t.values())) == 1:
            return self
        return F(self.tr, {self.tr.lin(self): 1})


# ============================================================================ tower (as lcv_tower.hpp)
class Fp2:
    def __init__(self, c0, c1):
        self.c0, self.c1 = c0, c1

    def __add__(s, o): return Fp2(s.c0 + o.c0, s.c1 + o.c1)
    def __sub__(s, o): return Fp2(s.c0 - o.c0, s.c1 - o.c1)
    def __neg__(s): return Fp2(-s.c0, -s.c1)
    def scale(s, k): return Fp2(s.c0 * k, s.c1 * k)
    def conj(s): return Fp2(s.c0, -s.c1)
    def mul_xi(s): return Fp2(s.c0 - s.c1, s.c0 + s.c1)
    def mul_fp(s, x): return Fp2(s.c0 * x, s.c1 * x)
    def mat(s): return Fp2(s.c0.mat(), s.c1.mat())

    def __mul__(a, b):
        t0 = a.c0 * b.c0
        t1 = a.c1 * b.c1
        t2 = (a.c0 + a.c1) * (b.c0 + b.c1)
        return Fp2(t0 - t1, t2 - t0 - t1)

    def sqr(a):
        return Fp2((a.c0 + a.c1) * (a.c0 - a.c1), (a.c0 * a.c1).dbl())

    def inv(a):
        t = (a.c0 * a.c0 + a.c1 * a.c1)
        ti = a.c0.tr.inv(t)
        return Fp2(a.c0 * ti, -(a.c1 * ti))


class Fp6:
    def __init__(self, c0, c1, c2):
        self.c0, self.c1, self.c2 = c0, c1, c2

    def __add__(s, o): return Fp6(s.c0 + o.c0, s.c1 + o.c1, s.c2 + o.c2)
    def __sub__(s, o): return Fp6(s.c0 - o.c0, s.c1 - o.c1, s.c2 - o.c2)
    def __neg__(s): return Fp6(-s.c0, -s.c1, -s.c2)
    def mul_v(s): return Fp6(s.c2.mul_xi(), s.c0, s.c1)
    def mat(s): return Fp6(s.c0.mat(), s.c1.mat(), s.c2.mat())

    def __mul__(a, b):
        t0, t1, t2 = a.c0 * b.c0, a.c1 * b.c1, a.c2 * b.c2
        x0 = ((a.c1 + a.c2) * (b.c1 + b.c2) - t1 - t2).mul_xi() + t0
        x1 = (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1 + t2.mul_xi()
        x2 = (a.c0 + a.c2) * (b.c0 + b.c2) - t0 - t2 + t1
        return Fp6(x0, x1, x2)

    def sqr(a):  # Chung-Hasan SQR2: 2 mul + 3 sqr in Fp2
        s0 = a.c0.sqr()
        ab = a.c0 * a.c1
        s1 = ab + ab
        s2 = (a.c0 - a.c1 + a.c2).sqr()
        bc = a.c1 * a.c2
        s3 = bc + bc
        s4 = a.c2.sqr()
        return Fp6(s3.mul_xi() + s0, s4.mul_xi() + s1, s1 + s2 + s3 - s0 - s4)

    def inv(a):
        t0 = a.c0.sqr() - (a.c1 * a.c2).mul_xi()
        t1 = a.c2.sqr().mul_xi() - a.c0 * a.c1
        t2 = a.c1.sqr() - a.c0 * a.c2
        t0, t1, t2 = t0.mat(), t1.mat(), t2.mat()
        d = ((a.c2 * t1 + a.c1 * t2).mul_xi() + a.c0 * t0).inv()
        d = d.mat()
        return Fp6(t0 * d, t1 * d, t2 * d)


class Fp12:
    def __init__(self, c0, c1):
        self.c0, self.c1 = c0, c1

    def conj(s): return Fp12(s.c0, -s.c1)
    def mat(s): return Fp12(s.c0.mat(), s.c1.mat())

    def __mul__(a, b):
        t0, t1 = a.c0 * b.c0, a.c1 * b.c1
        s = (a.c0 + a.c1) * (b.c0 + b.c1)
        return Fp12(t0 + t1.mul_v(), s - t0 - t1)

    def sqr(a):
        t = a.c0 * a.c1
        s = (a.c0 + a.c1) * (a.c0 + a.c1.mul_v())
        return Fp12(s - t - t.mul_v(), t + t)

    def inv(a):
        t = (a.c0 * a.c0 - (a.c1 * a.c1).mul_v()).mat().inv()
        return Fp12(a.c0 * t, -(a.c1 * t))

    def coeffs(s):  # g0..g5 of w^i
        return [s.c0.c0, s.c1.c0, s.c0.c1, s.c1.c1, s.c0.c2, s.c1.c2]

    @staticmethod
    def from_coeffs(g):
        return Fp12(Fp6(g[0], g[2], g[4]), Fp6(g[1], g[3], g[5]))

    def cyclo_sqr(a):
        g0, g1, g2, g3, g4, g5 = a.coeffs()

        def fp4_sqr(x0, x1):
            t0, t1 = x0.sqr(), x1.sqr()
            t2 = (x0 + x1).sqr() - t0 - t1
            return t0 + t1.mul_xi(), t2

        A0, A1 = fp4_sqr(g0, g3)
        B0, B1 = fp4_sqr(g1, g4)
        C0, C1 = fp4_sqr(g2, g5)
        xc1 = C1.mul_xi()
        z = [(A0 - g0).scale(2) + A0, (xc1 + g1).scale(2) + xc1, (B0 - g2).scale(2) + B0,
             (A1 + g3).scale(2) + A1, (C0 - g4).scale(2) + C0, (B1 + g5).scale(2) + B1]
        return Fp12.from_coeffs(z)

    def frob(a, k, tr):
        g = a.coeffs()
        out = []
        for i in range(6):
            gi = g[i].conj() if k % 2 else g[i]
            out.append(gi * const_fp2(tr, FROB[k][i]) if i else gi)
        return Fp12.from_coeffs(out)

    def mul_line(f, a, b, c):
        """f * (a + b v + c v w) (sparse line: coefficients of w^0, w^2, w^3)."""
        F0, F1 = f.c0, f.c1
        t0, t1 = F0.c0 * a, F0.c1 * b
        t2 = F0.c2 * b
        x = Fp6(t0 + t2.mul_xi(), (F0.c0 + F0.c1) * (a + b) - t0 - t1, t1 + F0.c2 * a)
        y = Fp6((F1.c2 * c).mul_xi(), F1.c0 * c, F1.c1 * c)
        h = F0 + F1
        bc = b + c
        z = Fp6(h.c0 * a + (h.c2 * bc).mul_xi(), h.c0 * bc + h.c1 * a, h.c1 * bc + h.c2 * a)
        return Fp12(x + y.mul_v(), z - x - y)


def fp2_pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = ((r[0] * a[0] - r[1] * a[1]) % P, (r[0] * a[1] + r[1] * a[0]) % P)
        a = ((a[0] * a[0] - a[1] * a[1]) % P, (2 * a[0] * a[1]) % P)
        e >>= 1
    return r


XI = (1, 1)
FROB = {k: [fp2_pow(XI, i * (P ** k - 1) // 6) for i in range(6)] for k in (1, 2, 3)}


def const_fp2(tr, c):
    return Fp2(tr.const(c[0]), tr.const(c[1]))


def in_fp2(tr, name):
    return Fp2(tr.input(name + "0"), tr.input(name + "1"))


def in_fp12(tr, name):
    return Fp12.from_coeffs([in_fp2(tr, f"{name}{i}_") for i in range(6)])


# ============================================================================ G2 lines (as lcv_pairing.hpp)
B2X3 = (12, 12)  # 3 * 4(1 + u)


def line_dbl(T):
    """Doubling step of lcv_pairing.hpp::line_dbl with the projective representative scaled by 4
    (no halvings): T and the line change by Fp2 factors only, which the final exponentiation kills."""
    X, Y, Z = T
    XY = X * Y
    B = Y.sqr()
    C = Z.sqr()
    E = C * const_fp2(X.c0.tr, B2X3)
    Fv = E.scale(3)
    H = (Y + Z).sqr() - B - C
    J = X.sqr()
    L = (B - E, J.scale(3), H)
    nX = (XY * (B - Fv)).scale(2)
    nY = (B + Fv).sqr() - E.sqr().scale(12)
    nZ = (B * H).scale(4)
    return L, (nX, nY, nZ)


def line_add(T, Q):
    X, Y, Z = T
    qx, qy = Q
    theta = Y - qy * Z
    lam = X - qx * Z
    C = theta.sqr()
    D = lam.sqr()
    E = lam * D
    Fv = Z * C
    G = X * D
    H = E + Fv - G - G
    L = (theta * qx - lam * qy, theta, lam)
    nX = lam * H
    nY = theta * (G - H) - Y * E
    nZ = Z * E
    return L, (nX, nY, nZ)


def miller_program(tr):
    """Both Miller loops of e(P1, Q1) * e(P2, Q2) with a shared accumulator.  Inputs are affine
    Q_k and (-x_P, y_P) of P_k; the prologue maps an identity Q_k to (Q_k = G2 generator, P_k = (0, 0)):
    its lines are then Fp2 constants, killed by the final exponentiation, i.e. e(P_k, O) = 1."""
    Q = [(in_fp2(tr, "q1x"), in_fp2(tr, "q1y")), (in_fp2(tr, "q2x"), in_fp2(tr, "q2y"))]
    nxP = [tr.input("p1nx"), tr.input("p2nx")]
    yP = [tr.input("p1y"), tr.input("p2y")]
    one = tr.one()
    T = [(q[0], q[1], Fp2(one, tr.const(0))) for q in Q]
    f = None
    for bit in bin(X_ABS)[3:]:
        for step in ("dbl", "add") if bit == "1" else ("dbl",):
            lines = []
            for k in range(2):
                L, T[k] = line_dbl(T[k]) if step == "dbl" else line_add(T[k], Q[k])
                T[k] = tuple(t.mat() for t in T[k])
                c00, c01, c11 = L
                lines.append((c00.mat(), c01.mul_fp(nxP[k]).mat(), c11.mul_fp(yP[k]).mat()))
            f = sparse_step(f, lines, square=(step == "dbl" and f is not None))
    return f.conj()


def sparse_step(f, lines, square):
    (a1, b1, c1), (a2, b2, c2) = lines
    if f is None:  # f = 1: f * l1 * l2 = l1 * l2 as a dense element
        tr = a1.c0.tr
        z = Fp2(tr.const(0), tr.const(0))
        one12 = Fp12(Fp6(a1, b1, z), Fp6(z, c1, z))
        return one12.mul_line(a2, b2, c2).mat()
    if square:
        f = f.sqr().mat()
    f = f.mul_line(a1, b1, c1).mat()
    f = f.mul_line(a2, b2, c2).mat()
    return f


def fexp_program(tr):
    """Final exponentiation f^((p^12-1)/r) * 3 (hard part (x-1)^2 (x+p)(x^2+p^2-1) + 3), as lcv_items."""
    f = in_fp12(tr, "f")
    t0 = f.inv()
    t1 = f.conj() * t0
    m = (t1.frob(2, tr) * t1).mat()

    def exp_x(a):  # a^|x| (cyclotomic)
        acc = a
        for bit in bin(X_ABS)[3:]:
            acc = acc.cyclo_sqr().mat()
            if bit == "1":
                acc = (acc * a).mat()
        return acc

    A = (exp_x(m) * m).conj().mat()
    A2 = (exp_x(A) * A).conj().mat()
    Bv = (exp_x(A2).conj() * A2.frob(1, tr)).mat()
    t = exp_x(exp_x(Bv))
    C = (t * Bv.frob(2, tr) * Bv.conj()).mat()
    r = C * (m.cyclo_sqr() * m)
    return r


# ============================================================================ G2 points (complete formulas)
# Twist E2: y^2 = x^3 + 4(1 + u).  Homogeneous projective (X : Y : Z) with the complete addition and
# doubling of Renes-Costello-Batina 2016 (Alg. 7 / 9, a = 0, b3 = 3b = 12(1 + u)): exact for every
# input, including the identity (0 : 1 : 0), P + (-P) and P + P, so the straight-line programs need
# no branches.  #E2(Fp2) = h2 * r is odd (no 2-torsion), the formulas' completeness condition.
ISO_XNUM = [
    (0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
     0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
    (0, 0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
    (0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1, 0),
]
ISO_XDEN = [(0, P - 72), (12, P - 12), (1, 0)]
ISO_YNUM = [
    (0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
     0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
    (0, 0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
    (0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10, 0),
]
ISO_YDEN = [(P - 432, P - 432), (0, P - 216), (18, P - 18), (1, 0)]


def fp2_inv_int(a):
    n = pow((a[0] * a[0] + a[1] * a[1]) % P, P - 2, P)
    return (a[0] * n % P, (-a[1]) * n % P)


PSI_CX = fp2_inv_int(fp2_pow(XI, (P - 1) // 3))
PSI_CY = fp2_inv_int(fp2_pow(XI, (P - 1) // 2))


def b3_mul(t):
    return t.mul_xi().scale(12)


def g2_dbl_c(Pt):
    X, Y, Z = Pt
    t0 = Y.sqr().mat()
    Z3 = t0.scale(8)
    t1 = Y * Z
    t2 = b3_mul(Z.sqr()).mat()
    X3 = t2 * Z3
    Y3 = t0 + t2
    Z3 = t1 * Z3
    t0 = (t0 - t2.scale(3)).mat()
    Y3 = t0 * Y3 + X3
    X3 = (t0 * (X * Y)).scale(2)
    return (X3.mat(), Y3.mat(), Z3.mat())


def g2_add_c(P1, P2):
    X1, Y1, Z1 = P1
    X2, Y2, Z2 = P2
    t0, t1, t2 = X1 * X2, Y1 * Y2, Z1 * Z2
    t3 = ((X1 + Y1) * (X2 + Y2) - t0 - t1).mat()
    t4 = ((Y1 + Z1) * (Y2 + Z2) - t1 - t2).mat()
    y3 = (X1 + Z1) * (X2 + Z2) - t0 - t2
    x3t = t0.scale(3).mat()
    t2b = b3_mul(t2)
    Z3 = (t1 + t2b).mat()
    t1m = (t1 - t2b).mat()
    y3b = b3_mul(y3).mat()
    X3 = t3 * t1m - t4 * y3b
    Y3 = y3b * x3t + t1m * Z3
    Z3 = Z3 * t4 + x3t * t3
    return (X3.mat(), Y3.mat(), Z3.mat())


def g2_neg(Pt):
    return (Pt[0], -Pt[1], Pt[2])


def g2_mul_xabs(Pt):
    acc = Pt
    for bit in bin(X_ABS)[3:]:
        acc = g2_dbl_c(acc)
        if bit == "1":
            acc = g2_add_c(acc, Pt)
    return acc


def g2_psi(tr, Pt):
    return ((Pt[0].conj() * const_fp2(tr, PSI_CX)).mat(), (Pt[1].conj() * const_fp2(tr, PSI_CY)).mat(),
            Pt[2].conj().mat())


def iso_proj(tr, x, y):
    """3-isogeny E2' -> E2 (RFC 9380 App. E.3) to projective: (xn yd : y yn xd : xd yd)."""
    def poly(cs):
        acc = const_fp2(tr, cs[-1])
        for c in reversed(cs[:-1]):
            acc = (acc * x + const_fp2(tr, c)).mat()
        return acc
    xn, xd, yn, yd = poly(ISO_XNUM), poly(ISO_XDEN), poly(ISO_YNUM), poly(ISO_YDEN)
    return ((xn * yd).mat(), ((y * yn).mat() * xd).mat(), (xd * yd).mat())


def h2c_program(tr):
    """hash_to_G2 after the two SSWU maps (inputs: the affine E2' points of u0, u1): isogeny, add,
    clear_cofactor (RFC 9380 App. G.3: [x^2-x-1]P + [x-1]psi(P) + psi^2(2P)), to affine."""
    q = [iso_proj(tr, in_fp2(tr, f"m{m}x"), in_fp2(tr, f"m{m}y")) for m in range(2)]
    Pt = g2_add_c(q[0], q[1])
    t1 = g2_neg(g2_mul_xabs(Pt))
    t2 = g2_psi(tr, Pt)
    t3 = g2_psi(tr, g2_psi(tr, g2_dbl_c(Pt)))
    t3 = g2_add_c(t3, g2_neg(t2))
    t2 = g2_add_c(t1, t2)
    t2 = g2_neg(g2_mul_xabs(t2))
    t3 = g2_add_c(t3, t2)
    t3 = g2_add_c(t3, g2_neg(t1))
    Q = g2_add_c(t3, g2_neg(Pt))
    zi = Q[2].inv().mat()
    return Q[0] * zi, Q[1] * zi, Q[2]


def g2sub_program(tr):
    """Signature subgroup check psi(P) == [x]P (Scott) with complete formulas: e1 = px Z - X,
    e2 = py Z + Y for T = [|x|]P = (X : Y : Z) ([x]P = -T); P in G2 iff Z != 0, e1 = e2 = 0."""
    x, y = in_fp2(tr, "sx"), in_fp2(tr, "sy")
    T = g2_mul_xabs((x, y, Fp2(tr.one(), tr.const(0))))
    px = (x.conj() * const_fp2(tr, PSI_CX)).mat()
    py = (y.conj() * const_fp2(tr, PSI_CY)).mat()
    return px * T[2] - T[0], py * T[2] + T[1], T[2]


# ============================================================================ scheduling + allocation
class Program:
    def __init__(self, name, tr, outputs, team, state_slots, policy="cp", slack=2, cap=96):
        self.name, self.tr, self.team, self.policy, self.slack, self.cap = name, tr, team, policy, slack, cap
        self.outputs = outputs            # list of (name, F)
        self.state_slots = state_slots    # name -> slot for inputs/outputs sharing storage
        if 0 not in tr.consts:            # the record padding term reads a zero constant
            tr.consts[0] = tr._new("const", const=0)
        self.zero = tr.consts[0]
        self.build()

    def build(self):
        tr, T = self.tr, self.team
        # output ops: one LIN per output (writes its state slot)
        self.out_ops = []
        for name, f in self.outputs:
            self.out_ops.append(tr.lin(f, name="out:" + name))
        ops = [v for v in tr.vals if v.kind in ("mul", "lin", "inv")]
        # dependencies
        deps = {}
        for v in ops:
            terms = list(v.a.items()) if isinstance(v.a, dict) else list(v.a)
            if v.b:
                terms += list(v.b.items())
            deps[v] = {u for u, _ in terms if u.kind in ("mul", "lin", "inv")}
            for u, _ in terms:
                u.readers.append(v)
        # WAR: an output written into an input's slot waits for every reader of that input
        name_to_input = tr.inputs
        for v in self.out_ops:
            nm = v.name[4:]
            if nm in name_to_input:
                deps[v] |= {r for r in name_to_input[nm].readers if r is not v}
        # critical-path priority
        succ = defaultdict(list)
        for v, ds in deps.items():
            for u in ds:
                succ[u].append(v)
        prio = {}
        for v in reversed(ops):
            prio[v] = 1 + max((prio[s] for s in succ[v]), default=0)
        if self.policy == "fifo":  # trace order: follows the sequential program, keeps few values live
            prio = {v: -v.id for v in ops}
        elif self.policy == "mix":  # trace order, but within a window the critical path first
            prio = {v: -(v.id // 400) * 100000 + prio[v] for v in ops}
        # ALAP release: an op becomes eligible only `SLACK` levels before the latest level it can run
        # at without lengthening the critical path, so off-critical work does not run far ahead and
        # hold LDS slots (the schedule lag is tracked so eligibility keeps pace with the real rounds)
        cp_len = max(prio.values()) if prio else 0
        asap = {}
        for v in ops:
            asap[v] = 1 + max((asap[u] for u in deps[v]), default=0)
        operand_vals = {}
        readers_of = defaultdict(int)
        for v in ops:
            terms = list(v.a.items()) if isinstance(v.a, dict) else list(v.a)
            if v.b:
                terms += list(v.b.items())
            operand_vals[v] = {u for u, _ in terms if u.kind in ("mul", "lin", "inv")}
            for u in operand_vals[v]:
                readers_of[u] += 1
        remaining = {}
        live = [0]
        indeg = {v: len(deps[v]) for v in ops}
        waiting = [(cp_len - prio[v], v.id, v) for v in ops if indeg[v] == 0]
        heapq.heapify(waiting)
        ready = []
        rounds = []
        r = 0
        lag = 0
        while ready or waiting:
            level = r - lag
            while waiting and waiting[0][0] - self.slack <= level:
                _, _, v = heapq.heappop(waiting)
                heapq.heappush(ready, (-prio[v], v.id, v))
            if not ready:  # nothing eligible: advance the level to the next waiting op
                lag = r - (waiting[0][0] - self.slack)
                continue
            cur, deferred = [], []
            while ready and len(cur) < T:
                item = heapq.heappop(ready)
                v = item[2]
                ins = {u for u in operand_vals[v] if u in remaining}
                frees = sum(1 for u in ins if remaining[u] == 1)
                if cur and live[0] + 1 - frees > self.cap and frees == 0:
                    deferred.append(item)  # register (LDS slot) pressure: wait for values to die
                    continue
                cur.append(v)
                live[0] += 1 - frees
                for u in ins:
                    remaining[u] -= 1
                    if remaining[u] == 0:
                        del remaining[u]
                if readers_of[v]:
                    remaining[v] = readers_of[v]
                else:
                    live[0] -= 1
            for item in deferred:
                heapq.heappush(ready, item)
            for v in cur:
                v.round = r
            rounds.append(cur)
            for v in cur:
                for s in succ[v]:
                    indeg[s] -= 1
                    if indeg[s] == 0:
                        heapq.heappush(waiting, (cp_len - prio[s], s.id, s))
            r += 1
            # critical-path ops still queued: the schedule is behind the ideal levels
            if ready and min(-p for p, _, _ in ready) >= cp_len - level:
                lag += 1
        self.rounds = rounds
        # last use of every value (round of its last reader)
        for v in tr.vals:
            v.last_use = max((u.round for u in v.readers if u.round is not None), default=-1)
        # slot allocation
        nxt = 0
        for name, v in tr.inputs.items():
            v.slot = self.state_slots[name]
            nxt = max(nxt, v.slot + 1)
        self.consts = [v.const for v in tr.consts.values()]
        free = []
        heapq.heapify(free)
        nxt = max(nxt, max(self.state_slots.values()) + 1)
        base_free = nxt
        release = defaultdict(list)
        for v in tr.inputs.values():  # inputs whose slots are not reused by outputs may be freed after last use
            pass
        peak = nxt
        for r, cur in enumerate(rounds):
            for s in release.pop(r, []):
                heapq.heappush(free, s)
            for v in cur:
                if v.name and v.name.startswith("out:"):
                    v.slot = self.state_slots[v.name[4:]]
                    continue
                if free:
                    v.slot = heapq.heappop(free)
                else:
                    v.slot = base_free
                    base_free += 1
                    peak = max(peak, base_free)
                release[max(v.last_use, r) + 1].append(v.slot)
        self.nslots = peak
        for k, v in enumerate(tr.consts.values()):  # constants are copied into LDS after the slots
            v.slot = self.nslots + k
        assert self.nslots + len(self.consts) < SLOT_NONE

    def max_abs_sum(self):
        """max over all combinations of sum |coef| (bounds the unreduced accumulator: < sum * p)"""
        m = 1
        for cur in self.rounds:
            for v in cur:
                for terms in (v.a, v.b):
                    if terms:
                        items = terms.items() if isinstance(terms, dict) else terms
                        m = max(m, sum(abs(c) for _, c in items))
        return m

    def stats(self):
        muls = sum(1 for cur in self.rounds for v in cur if v.kind == "mul")
        lins = sum(1 for cur in self.rounds for v in cur if v.kind == "lin")
        invs = sum(1 for cur in self.rounds for v in cur if v.kind == "inv")
        lanes = len(self.rounds) * self.team
        return (f"{self.name}: team {self.team}, {len(self.rounds)} rounds, {muls} mul, {lins} lin, {invs} inv, "
                f"lane use {100.0 * (muls + lins + invs) / lanes:.1f}%, {self.nslots} LDS slots "
                f"({self.nslots * 48} B/item), {len(self.consts)} constants")

    # ---------------------------------------------------------------- encoding
    def encode(self):
        """Fixed-size records, so the device can prefetch round r+1 while it executes round r.

        hdr: two uint32 per round (wave-uniform):
          hdr[2r]   = nA | mA << 4 | kA << 8 | fullA << 11 | nB << 12 | mB << 16 | kB << 20
          hdr[2r+1] = used | any_mul << 8 | any_inv << 9
        (n terms, max |coef|, reduction bits k with 2^k > sum |coef|, full reduction of A).
        rec: REC_HW uint16 per lane per round, T lanes per round (lanes >= used: dst = SLOT_NONE):
          rec[0] = dst | MUL << 12 | INV << 13;  A terms at rec[1 .. 1+nA);  B terms at rec[B_AT ..]
          term = slot | coef << 12 (signed 4-bit); padding = slot 0, coef 0 (adds nothing).
        Slots >= nslots are the constant table (copied into LDS by the kernel prologue)."""
        hdr, rec = [], []
        T = self.team
        for cur in self.rounds:
            ents = []
            for v in cur:
                a = list(v.a.items()) if isinstance(v.a, dict) else list(v.a)
                b = list(v.b.items()) if v.b else []
                ents.append((v, a, b))
            nA = max(len(a) for _, a, _ in ents)
            nB = max(len(b) for _, _, b in ents)
            mA = max((abs(c) for _, a, _ in ents for _, c in a), default=1)
            mB = max((abs(c) for _, _, b in ents for _, c in b), default=1)
            # reduction of the unreduced accumulator (< S p, S = sum |c|): conditional subtraction of
            # 2^s p for s = k-1 .. lo with 2^k > S; lo = 0 (< p: LIN results are stored) or 1
            # (<= 2p suffices for a Montgomery operand: a, b <= 2p -> ab < R p)
            kA = max(sum(abs(c) for _, c in a).bit_length() for _, a, _ in ents)
            fullA = any(v.kind != "mul" for v, _, _ in ents)
            anymul = any(v.kind == "mul" for v, _, _ in ents)
            anyinv = any(v.kind == "inv" for v, _, _ in ents)
            kB = max((sum(abs(c) for _, c in b).bit_length() for v, _, b in ents if v.kind == "mul"), default=0)
            assert kA <= 6 and kB <= 6 and mA <= 7 and mB <= 7 and nA <= B_AT - 1 and nB <= REC_HW - B_AT
            assert not anymul or nA <= B_AT - 1
            hdr += [nA | (mA << 4) | (kA << 8) | ((1 if fullA else 0) << 11) | (nB << 12) | (mB << 16) | (kB << 20),
                    len(ents) | ((1 if anymul else 0) << 8) | ((1 if anyinv else 0) << 9)]
            for lane in range(T):
                # unused term positions: the zero constant at coefficient +1 (adds nothing, and the
                # device's |c| = 1 path needs no mask)
                w = [0] + [self.zero.slot | (1 << 12)] * (REC_HW - 1)
                if lane < len(ents):
                    v, a, b = ents[lane]
                    flags = (1 << 12) if v.kind == "mul" else (1 << 13) if v.kind == "inv" else 0
                    w[0] = v.slot | flags
                    for k, (u, c) in enumerate(a):
                        assert -8 <= c <= 7 and c != 0, c
                        w[1 + k] = u.slot | ((c & 0xF) << 12)
                    for k, (u, c) in enumerate(b):
                        assert -8 <= c <= 7 and c != 0, c
                        w[B_AT + k] = u.slot | ((c & 0xF) << 12)
                else:
                    w[0] = SLOT_NONE
                rec += w
        return hdr, rec

    # ---------------------------------------------------------------- emulation (round semantics)
    def emulate(self, inputs):
        """Execute the ENCODED program with Python integers (the device's round semantics)."""
        mem = {}
        for name, v in self.tr.inputs.items():
            mem[v.slot] = inputs[name] % P
        consts = {self.nslots + k: c for k, c in enumerate(self.consts)}
        hdr, rec = self.encode()
        T = self.team
        for r in range(len(hdr) // 2):
            h0, h1 = hdr[2 * r], hdr[2 * r + 1]
            nA, nB, used = h0 & 0xF, (h0 >> 12) & 0xF, h1 & 0xFF
            writes = []
            for lane in range(T):
                e = rec[(r * T + lane) * REC_HW:(r * T + lane + 1) * REC_HW]
                dst = e[0]
                if lane >= used:
                    assert dst == SLOT_NONE
                    continue

                def ev(ts):
                    acc = 0
                    for t in ts:
                        s, c = t & 0xFFF, (t >> 12) & 0xF
                        c = c - 16 if c >= 8 else c
                        if c == 0:
                            continue
                        val = consts[s] if s >= self.nslots else mem[s]
                        acc = (acc + c * val) % P
                    return acc
                A = ev(e[1:1 + nA])
                if dst & (1 << 12):
                    res = A * ev(e[B_AT:B_AT + nB]) % P
                elif dst & (1 << 13):
                    res = pow(A, P - 2, P)
                else:
                    res = A
                writes.append((dst & 0xFFF, res))
            for s, x in writes:
                mem[s] = x
        return mem


# ============================================================================ checks against the oracle
def check_miller(prog, team):
    from oracle import bls12_381 as B
    rnd = random.Random(7)
    for trial in range(2):
        a, b = rnd.randrange(1, 1 << 60), rnd.randrange(1, 1 << 60)
        Pp = B.g1_mul(B.G1_GEN, a)
        Q1 = B.g2_mul(B.G2_GEN, b)
        Q2 = B.g2_mul(B.G2_GEN, b + 7)
        inp = {"q1x0": Q1[0][0], "q1x1": Q1[0][1], "q1y0": Q1[1][0], "q1y1": Q1[1][1],
               "q2x0": Q2[0][0], "q2x1": Q2[0][1], "q2y0": Q2[1][0], "q2y1": Q2[1][1],
               "p1nx": (-Pp[0]) % P, "p1y": Pp[1], "p2nx": (-B.G1_GEN[0]) % P, "p2y": (-B.G1_GEN[1]) % P}
        mem = prog.emulate(inp)
        g = [(mem[prog.state_slots[f"f{i}_0"]], mem[prog.state_slots[f"f{i}_1"]]) for i in range(6)]
        got = B.final_exponentiation(B.f12_from_coeffs(g))
        e1 = B.pairing(Pp, Q1)
        e2 = B.pairing(B.g1_neg(B.G1_GEN), Q2)
        exp = B.f12_mul(e1, e2)
        assert got == exp, "miller program mismatch"
    print(f"  miller program checked against oracle pairings ({prog.name})")


def check_fexp(prog):
    from oracle import bls12_381 as B
    rnd = random.Random(9)
    f = tuple(tuple((rnd.randrange(P), rnd.randrange(P)) for _ in range(3)) for _ in range(2))
    g = B.f12_coeffs(f)
    inp = {}
    for i in range(6):
        inp[f"f{i}_0"], inp[f"f{i}_1"] = g[i]
    mem = prog.emulate(inp)
    out = [(mem[prog.state_slots[f"r{i}_0"]], mem[prog.state_slots[f"r{i}_1"]]) for i in range(6)]
    e = B.final_exponentiation(f)
    assert B.f12_from_coeffs(out) == B.f12_mul(B.f12_mul(e, e), e), "fexp program mismatch"
    print(f"  fexp program checked against oracle final exponentiation ({prog.name})")


# ============================================================================ main
def make_miller(team, policy="cp"):
    tr = Tracer()
    f = miller_program(tr)
    names = [f"f{i}_{j}" for i in range(6) for j in range(2)]
    outs = []
    for i, g in enumerate(f.coeffs()):
        outs += [(f"f{i}_0", g.c0), (f"f{i}_1", g.c1)]
    inputs = ["q1x0", "q1x1", "q1y0", "q1y1", "q2x0", "q2x1", "q2y0", "q2y1", "p1nx", "p1y", "p2nx", "p2y"]
    slots = {n: k for k, n in enumerate(inputs + names)}
    return Program("miller", tr, outs, team, slots, policy)


def make_fexp(team, policy="cp"):
    tr = Tracer()
    r = fexp_program(tr)
    outs = []
    for i, g in enumerate(r.coeffs()):
        outs += [(f"r{i}_0", g.c0), (f"r{i}_1", g.c1)]
    ins = [f"f{i}_{j}" for i in range(6) for j in range(2)]
    slots = {n: k for k, n in enumerate(ins + [o for o, _ in outs])}
    return Program("fexp", tr, outs, team, slots, policy)


def make_h2c(team, policy="cp"):
    tr = Tracer()
    hx, hy, hz = h2c_program(tr)
    outs = [("hx0", hx.c0), ("hx1", hx.c1), ("hy0", hy.c0), ("hy1", hy.c1), ("hz0", hz.c0), ("hz1", hz.c1)]
    ins = [f"m{m}{c}{j}" for m in range(2) for c in "xy" for j in range(2)]
    slots = {n: k for k, n in enumerate(ins + [o for o, _ in outs])}
    return Program("h2c", tr, outs, team, slots, policy)


def make_g2sub(team, policy="cp"):
    tr = Tracer()
    e1, e2, z = g2sub_program(tr)
    outs = [("e10", e1.c0), ("e11", e1.c1), ("e20", e2.c0), ("e21", e2.c1), ("z0", z.c0), ("z1", z.c1)]
    ins = ["sx0", "sx1", "sy0", "sy1"]
    slots = {n: k for k, n in enumerate(ins + [o for o, _ in outs])}
    return Program("g2sub", tr, outs, team, slots, policy)


def check_h2c(prog):
    from oracle import bls12_381 as B
    rnd = random.Random(11)
    for _ in range(2):
        msg = rnd.randbytes(32)
        u = B.hash_to_field_fp2(msg, 2, B.DST_POP)
        inp = {}
        for m in range(2):
            x, y = B.sswu_g2(u[m])
            inp[f"m{m}x0"], inp[f"m{m}x1"], inp[f"m{m}y0"], inp[f"m{m}y1"] = x[0], x[1], y[0], y[1]
        mem = prog.emulate(inp)
        got = ((mem[prog.state_slots["hx0"]], mem[prog.state_slots["hx1"]]),
               (mem[prog.state_slots["hy0"]], mem[prog.state_slots["hy1"]]))
        assert got == B.hash_to_g2(msg), "h2c program mismatch"
    print(f"  h2c program checked against oracle hash_to_g2 ({prog.name})")


def check_g2sub(prog):
    from oracle import bls12_381 as B
    rnd = random.Random(13)
    cases = [(B.g2_mul(B.G2_GEN, rnd.randrange(1, B.R)), True)]
    x = 1
    while len(cases) < 3:  # points of E2 outside G2
        x += 1
        X = (x, 5)
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(X), X), B.B2))
        if y is not None:
            cases.append(((X, y), False))
    for pt, want in cases:
        (x0, x1), (y0, y1) = pt
        mem = prog.emulate({"sx0": x0, "sx1": x1, "sy0": y0, "sy1": y1})
        e = [mem[prog.state_slots[k]] for k in ("e10", "e11", "e20", "e21")]
        z = [mem[prog.state_slots[k]] for k in ("z0", "z1")]
        got = any(z) and not any(e)
        assert got == want == B.g2_in_subgroup(pt), "g2sub program mismatch"
    print(f"  g2sub program checked against oracle subgroup membership ({prog.name})")


def emit(progs, path):
    lines = ["// GENERATED by tools/gen_programs.py — do not edit.  Team programs (see lcv_engine.hpp).",
             "#pragma once", "#include <stdint.h>", "",
             f"#define LCV_PROG_REC_HW {REC_HW}", f"#define LCV_PROG_B_AT {B_AT}", f"#define LCV_PROG_KLIN {KLIN}", ""]
    for p in progs:
        hdr, rec = p.encode()
        N = p.name.upper()
        lines.append(f"// {p.stats()}")
        lines.append(f"#define LCV_PROG_{N}_TEAM {p.team}")
        lines.append(f"#define LCV_PROG_{N}_ROUNDS {len(hdr) // 2}")
        lines.append(f"#define LCV_PROG_{N}_SLOTS {p.nslots}")
        lines.append(f"#define LCV_PROG_{N}_NCONST {len(p.consts)}")
        lines.append(f"#define LCV_PROG_{N}_MAXSUM {p.max_abs_sum()}")
        lines.append(f"#define LCV_PROG_{N}_ZERO {p.zero.slot}")
        for nm, s in sorted(p.state_slots.items(), key=lambda kv: kv[1]):
            lines.append(f"#define LCV_PROG_{N}_SLOT_{nm.upper()} {s}")
        lines.append(f"static const uint32_t kProg_{p.name}_hdr[{len(hdr)}] = {{")
        for i in range(0, len(hdr), 16):
            lines.append("  " + ",".join(str(w) for w in hdr[i:i + 16]) + ",")
        lines.append("};")
        lines.append(f"static const uint16_t kProg_{p.name}_rec[{len(rec)}] __attribute__((aligned(16))) = {{")
        for i in range(0, len(rec), 32):
            lines.append("  " + ",".join(str(w) for w in rec[i:i + 32]) + ",")
        lines.append("};")
        # constants: Montgomery form, 12 little-endian 32-bit limbs each
        lines.append(f"static const uint32_t kProg_{p.name}_consts[{max(1, len(p.consts)) * 12}] = {{")
        for c in p.consts or [0]:
            m = c * RM % P
            lines.append("  " + ",".join(f"0x{(m >> (32 * k)) & 0xffffffff:08x}u" for k in range(12)) + ",")
        lines.append("};")
        lines.append("")
    open(path, "w").write("\n".join(lines) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--team", type=int, default=32, help="Miller team (32: 720 rounds vs 1,070 at 16; r01_v12)")
    ap.add_argument("--fexp-team", type=int, default=16)
    ap.add_argument("--g2-team", type=int, default=16)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "light-client-consensus-specs_amd", "csrc", "lcv_programs.inc"))
    args = ap.parse_args()
    progs = [make_miller(args.team), make_fexp(args.fexp_team), make_h2c(args.g2_team), make_g2sub(args.g2_team)]
    for p in progs:
        print(p.stats())
    if args.check:
        check_miller(progs[0], args.team)
        check_fexp(progs[1])
        check_h2c(progs[2])
        check_g2sub(progs[3])
    emit(progs, args.out)


if __name__ == "__main__":
    main()
