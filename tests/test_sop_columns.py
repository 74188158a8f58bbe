"""CPU model of the SOP engine's 28-bit column arithmetic (csrc/lcv_sop.hpp sop_products / sop_kara_mac /
sop_kara_join / sop_redc28), checked two ways:
  * exactness: the thirteen 28-bit + one 20-bit quotient digits give (T + M p) / 2^384 with the unique
    M < 2^384, T + M p = 0 mod 2^384 — the 32-bit engine's result, so the programs' Montgomery
    representatives are unchanged (tools/gen_sop.py emulates with that formula);
  * bounds: for every distinct op shape of the four programs, with every term at its largest value (p,
    a shadow of 0), no unsigned column / reduction intermediate reaches 2^64 and no signed Karatsuba
    middle column reaches 2^63, and tools/gen_sop.py's Program.col_bound / kara_bound (which set the
    round flags the device trusts) are at least the exact maxima.
The host simulation runs the C++ itself on real data (test_tools_hostsim.py, the parity tests); this
test covers the extreme operands the data never reaches."""
import os
import random
import sys

import helpers as H

sys.path.insert(0, os.path.join(H.ROOT, "tools"))
import gen_sop as GS  # noqa: E402

P = GS.P
R = 1 << 384
M28 = (1 << 28) - 1
NP28 = (-pow(P, -1, 1 << 28)) % (1 << 28)
PL = [(P >> (28 * j)) & M28 for j in range(14)]


def limbs(v, n):
    return [(v >> (28 * i)) & M28 for i in range(n - 1)] + [v >> (28 * (n - 1))]


class Track:
    def __init__(self):
        self.u = 0   # largest unsigned intermediate
        self.s = 0   # largest |signed| intermediate

    def uu(self, v):
        assert v >= 0
        self.u = max(self.u, v)
        return v

    def ss(self, v):
        self.s = max(self.s, abs(v))
        return v


def device_columns(prods, kara, x15, tr):
    """prods: [(X, Y)] operand values as the device forms them (X = m (t0 + t1), Y = t0 + t1)."""
    nx = 15 if x15 else 14
    col = [0] * 28
    if kara:
        p0, p2, pd = [0] * 13, [0] * 13, [0] * 13
        for X, Y in prods:
            x, y = limbs(X, 14), limbs(Y, 14)
            xd = [x[i] - x[i + 7] for i in range(7)]
            yd = [y[j + 7] - y[j] for j in range(7)]
            for i in range(7):
                for j in range(7):
                    p0[i + j] = tr.uu(p0[i + j] + x[i] * y[j])
                    p2[i + j] = tr.uu(p2[i + j] + x[i + 7] * y[j + 7])
                    pd[i + j] = tr.ss(pd[i + j] + xd[i] * yd[j])
        for c in range(28):
            v = p0[c] if c < 13 else 0
            if 7 <= c < 20:
                v += p0[c - 7] + p2[c - 7] + pd[c - 7]
            if 14 <= c < 27:
                v += p2[c - 14]
            col[c] = tr.uu(v)
    else:
        for X, Y in prods:
            x, y = limbs(X, nx), limbs(Y, 14)
            for i in range(nx):
                for j in range(14):
                    col[i + j] = tr.uu(col[i + j] + x[i] * y[j])
    return col


def device_redc(col, tr):
    col = list(col)
    carry = 0
    for i in range(13):
        v = tr.uu(col[i] + carry)
        q = ((v & 0xFFFFFFFF) * NP28) & M28
        carry = tr.uu(v + q * PL[0]) >> 28
        for j in range(1, 14):
            col[i + j] = tr.uu(col[i + j] + q * PL[j])
    v = tr.uu(col[13] + carry)
    q = ((v & 0xFFFFFFFF) * NP28) & 0xFFFFF
    v = tr.uu(v + q * PL[0])
    assert v & 0xFFFFF == 0
    for j in range(1, 14):
        col[13 + j] = tr.uu(col[13 + j] + q * PL[j])
    L = [v & M28]
    carry = v >> 28
    for c in range(14, 28):
        t = tr.uu(col[c] + carry)
        L.append(t & M28)
        carry = t >> 28
    L.append(carry)
    bits = sum(l << (28 * k) for k, l in enumerate(L))
    assert bits & 0xFFFFF == 0
    return bits >> 20


def test_redc_digits_exact():
    rng = random.Random(7)
    tr = Track()
    for _ in range(300):
        prods = [(rng.randrange(2 * P), rng.randrange(2 * P)) for _ in range(rng.randrange(1, 8))]
        T = sum(x * y for x, y in prods)
        expect = (T + ((-T * pow(P, -1, R)) % R) * P) // R
        for kara in (False, True):
            got = device_redc(device_columns(prods, kara, False, tr), tr)
            assert got == expect


def test_columns_below_the_generator_bounds():
    shapes = {}
    for p in GS.build():
        p.finalize()
        for ops in p.rounds:
            x15, kara = p.round_flags(ops)
            for o in ops:
                key = (tuple((m, len(x), len(y)) for x, y, m in o.prods), x15, kara)
                shapes.setdefault(key, (p, o))
    assert shapes
    for (prods, x15, kara), (p, o) in shapes.items():
        if not prods:
            continue
        tr = Track()
        vals = [(m * nx * P, ny * P) for m, nx, ny in prods]   # every term = p
        device_redc(device_columns(vals, kara, x15, tr), tr)
        assert tr.u < 1 << 64 and tr.s < 1 << 63, (p.name, prods)
        assert p.col_bound(o, x15) >= tr.u, (p.name, prods)
        if kara:
            assert p.kara_bound(o) >= tr.s, (p.name, prods)
