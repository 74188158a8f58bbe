"""The fan engine's row tail (csrc/lcv_sop_row.hpp) as an algorithm, on the CPU: a lane-by-lane emulation of its
16-lane row steps (DPP row_shr / row_shl / row_newbcast, row ballots) checked against the plain integer definitions —
r' = (T + M p) / 2^384 with M = T (-p^-1) mod 2^384 (sop_redc28's value), v = (r' + sum |c| (u or p - u)) mod p, the
stored words and the shadow p - v.  The emulation follows the device code step for step (same carry rounds, same
lookahead, same FP64 quotient estimate and exactness test), so a change to the row math that breaks its bounds
shows up here without a GPU; tests/test_row_tail_gpu.py runs the device code itself against the one-lane tail."""
import random

import pytest

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
M28 = (1 << 28) - 1
NP392 = (-pow(P, -1, 1 << 392)) % (1 << 392)
PL = [(P >> (28 * j)) & M28 for j in range(14)] + [0, 0]
NQ = [(NP392 >> (28 * j)) & M28 for j in range(14)] + [0, 0]
PW = [(P >> (32 * j)) & 0xFFFFFFFF for j in range(12)] + [0] * 4
U64 = (1 << 64) - 1


# row primitives (16 lanes)
def shr(x, k=1):
    return [0] * k + x[:16 - k]


def shl(x, k):
    return x[k:] + [0] * k


def bcast(x, k):
    return [x[k]] * 16


def norm2(x):  # rw_norm2: two unsigned carry rounds (64-bit lanes)
    for _ in range(2):
        c = [v >> 28 for v in x]
        x = [((v & M28) + cin) & U64 for v, cin in zip(x, shr(c))]
    return x


def lookahead(x, low):  # rw_norm_exact(_s): limbs < 2^29 - 1 on lanes 0..13
    g = sum(1 << j for j in range(16) if low[j] and x[j] > M28)
    p = sum(1 << j for j in range(16) if low[j] and x[j] == M28)
    a = g | p
    cy = (a + g) ^ a ^ g
    return [((x[j] + ((cy >> j) & 1)) & M28) if low[j] else x[j] + ((cy >> j) & 1) for j in range(16)]


def norm_exact(x):
    assert all(0 <= v < (1 << 29) - 1 for v in x[:14]), "rw_norm_exact precondition"
    return [v & M28 for v in lookahead(x, [True] * 16)]


LOW = [j < 14 for j in range(16)]


def norm_exact_s(x):
    assert all(0 <= v < (1 << 29) - 1 for v in x[:14]), "rw_norm_exact_s precondition"
    return lookahead(x, LOW)


def carry1s(x):  # one signed carry round over lanes 0..13 into lane 14
    c = [(x[j] >> 28) if LOW[j] else 0 for j in range(16)]
    return [((x[j] & M28) if LOW[j] else x[j]) + cin for j, cin in zip(range(16), shr(c))]


def biased_sub(u, v):
    return [u[j] - v[j] + ((1 << 28) if j < 14 else 0) - (1 if 1 <= j <= 14 else 0) for j in range(16)]


def limbs_of(v):
    return [(v >> (28 * j)) & M28 for j in range(14)] + [0, 0]


def value_of(x):
    return sum(v << (28 * j) for j, v in enumerate(x))


def word(L):  # rw_word: canonical limbs -> word j on lane j < 13
    a1, a2 = shl(L, 1), shl(L, 2)
    out = []
    for j in range(16):
        hiw = j >= 7
        x0, x1 = (a1[j], a2[j]) if hiw else (L[j], a1[j])
        sh = 4 * j - 28 if hiw else 4 * j
        out.append(((x0 >> sh) | (x1 << (28 - sh))) & 0xFFFFFFFF if j < 13 else 0)
    return out


def redc_limbs(lo, hi):  # rw_redc_limbs
    t = norm2(lo)
    hi = [(h + v) & U64 for h, v in zip(hi, shl([v & 0xFFFFFFFF for v in t], 14))]
    t32 = [t[j] & 0xFFFFFFFF if j < 14 else 0 for j in range(16)]
    nq = [[NQ[j - i] if i <= j < 14 else 0 for j in range(16)] for i in range(14)]
    pl = [[PL[j - i] if i <= j < 14 else 0 for j in range(16)] for i in range(14)]
    ph = [[PL[j + 14 - i] if j < i else 0 for j in range(16)] for i in range(14)]
    c = [0] * 16
    for i in range(14):
        s = bcast(t32, i)
        c = [(cv + sv * n) & U64 for cv, sv, n in zip(c, s, nq[i])]
    m = [v & 0xFFFFFFFF if j < 14 else 0 for j, v in enumerate(norm2(c))]
    m = norm_exact(m)
    m[13] &= 0xFFFFF
    l, h = list(t32), list(hi)
    for i in range(14):
        s = bcast(m, i)
        l = [(lv + sv * q) & U64 for lv, sv, q in zip(l, s, pl[i])]
        h = [(hv + sv * q) & U64 for hv, sv, q in zip(h, s, ph[i])]
    u = [v & 0xFFFFFFFF for v in norm2(l)]
    e = 1 if any(u[j] for j in range(13)) else 0
    hn = [((v & M28) + cin) & U64 for v, cin in zip(h, shr([v >> 28 for v in h]))]
    R = [(v << 8) & U64 for v in hn]
    R[0] += ((u[13] + e) >> 20) + (u[14] << 8)
    R[1] += u[15] << 8
    return [((v & M28) + cin) & 0xFFFFFFFF for v, cin in zip(R, shr([v >> 28 for v in R]))], m


def row_value(rl, adds, red):  # rw_value; adds: [(coef, limbs of u)]
    x = list(rl)
    for c, t in adds:
        mag = abs(c)
        term = biased_sub(PL, t) if c < 0 else t
        x = [xv + mag * tv for xv, tv in zip(x, term)]
    if red:
        if adds:
            x = carry1s(x)
        top = ((float(x[14]) * 268435456.0 + float(x[13])) * 268435456.0 + float(x[12])) * 268435456.0 + float(x[11])
        e = top * float.fromhex("0x1.3b06ba5e7993dp-73") - 2.0 ** -30
        qi = int(e)
        q = max(qi, 0)
        exact = e - qi <= 1.0 - 2.0 ** -29
        y = [x[j] - q * PL[j] + ((q << 28) if j < 14 else 0) - (q if 1 <= j <= 14 else 0) for j in range(16)]
        y = norm_exact_s(carry1s(y))
        if not exact:
            z = norm_exact_s(biased_sub([v & 0xFFFFFFFF for v in y], PL))
            if z[14] == 0:
                y = z
        x = y
    elif adds:
        x = norm_exact_s(carry1s(x))
    else:
        x = norm_exact(x)
    return [v if j < 14 else 0 for j, v in enumerate(x)]


def neg_word(vw):  # rw_neg_word
    g = sum(1 << j for j in range(12) if PW[j] < vw[j])
    p = sum(1 << j for j in range(12) if PW[j] == vw[j])
    a = g | p
    cy = (a + g) ^ a ^ g
    return [(PW[j] - vw[j] - ((cy >> j) & 1)) & 0xFFFFFFFF if j < 12 else 0 for j in range(16)]


def columns(prods):
    """28 column sums of sum m X Y (normalised 28-bit limbs, m X < 2^392), lane j: columns j and j + 14."""
    col = [0] * 28
    for x, y, m in prods:
        X, Y = limbs_of(m * x)[:14], limbs_of(y)[:14]
        for i in range(14):
            for j in range(14):
                col[i + j] += X[i] * Y[j]
    assert max(col) < 1 << 64
    return col[:14] + [0, 0], col[14:28] + [0, 0]


def words_of(v):
    return [(v >> (32 * j)) & 0xFFFFFFFF for j in range(12)]


@pytest.mark.parametrize("seed", range(6))
def test_row_tail_matches_integer_definitions(seed):
    rng = random.Random(1000 + seed)
    for case in range(40):
        nk = rng.randrange(0, 5)
        edge = case % 7
        val = (lambda: P - 1 - rng.randrange(8)) if edge == 3 else (lambda: rng.randrange(8)) if edge == 5 \
            else (lambda: rng.randrange(P))
        prods = [(val(), val(), rng.choice([1, 1, 2, 3, rng.randrange(1, 1024)])) for _ in range(nk)]
        T = sum(m * x * y for x, y, m in prods)
        adds = [(rng.choice([-1, 1]) * rng.randrange(1, 40), val()) for _ in range(rng.randrange(0, 3))]
        # the header's reduction bound: r' + sum |c| p < 2^red p
        bound = T // (1 << 384) + P + sum(abs(c) for c, _ in adds) * P
        red = 0
        while (P << red) <= bound:
            red += 1
        red += rng.randrange(0, 2)
        # reference (sop_redc28's value, sop_tail_value, sop_tail_store)
        M = (T * NP392) % (1 << 384)
        r_ref = (T + M * P) >> 384
        assert (T + M * P) % (1 << 384) == 0
        v_ref = (r_ref + sum((c * u) for c, u in adds)) % P
        # the row
        if nk:
            lo, hi = columns(prods)
            rl, m = redc_limbs(lo, hi)
            assert value_of(m[:14]) == M, "the row's quotient is the canonical one"
            assert value_of(rl) == r_ref and all(0 <= v < (1 << 28) + (1 << 17) for v in rl[:14])
        else:
            rl = [0] * 16
        vl = row_value(rl, [(c, limbs_of(u)) for c, u in adds], red)
        assert all(0 <= v <= M28 for v in vl[:14]) and value_of(vl) == v_ref
        vw = word(vl)
        assert vw[:12] == words_of(v_ref)
        assert neg_word(vw)[:12] == words_of(P - v_ref)
