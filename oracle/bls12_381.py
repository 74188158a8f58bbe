"""CPU restatement of BLS12-381 as used by `bls.FastAggregateVerify` — TEST INFRASTRUCTURE ONLY.

This module is the *oracle* (checker) for the MI355X HIP path. Only `tests/`,
`__graft_entry__.smoke()`, `bench.py`'s `cpu_baseline` leg and the golden-vector generator
may import it. The product path (`lcv`) never routes through it.

What it restates (none of this lives in /root/reference):
  * the call site `bls.FastAggregateVerify(participant_pubkeys, signing_root, signature)`
    at reference `sync-protocol.md:464`;
  * upstream `eth2spec.utils.bls` -> py_ecc `G2ProofOfPossession.FastAggregateVerify`
    semantics (IETF draft-irtf-cfrg-bls-signature-05 §3.3.4, POP ciphersuite
    `BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_`): KeyValidate every pubkey
    (decode, non-identity, subgroup), aggregate, decode + subgroup-check the signature,
    hash_to_G2 (RFC 9380 §8.8.2 BLS12381G2_XMD:SHA-256_SSWU_RO_), pairing check;
    any decoding error -> False.  No module/version of py_ecc/blst is pinned anywhere in the
    reference (and none is installed here); the algorithm is restated from the published
    standards and py_ecc's documented decoding rules.

Everything is written for clarity, not speed: affine points, Python ints, a textbook affine
Miller loop and a *definitional* final exponentiation (f ** ((p^12-1)/r), with only the
easy part done via Frobenius).  Pinned by: curve/subgroup identities, generator encodings,
bilinearity, and RFC 9380 / eth2 vectors recalled in tests/test_oracle_bls.py.
"""
from __future__ import annotations

import functools
import hashlib
from typing import Optional, Sequence, Tuple

# ----------------------------------------------------------------------------- constants
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X = -0xD201000000010000  # BLS parameter x (negative)
X_ABS = 0xD201000000010000

G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
G2_X = (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E)
G2_Y = (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE)

# RFC 9380 §8.8.2: effective cofactor for G2
H_EFF_G2 = 0xBC69F08F2EE75B3584C6A0EA91B352888E2A8E9145AD7689986FF031508FFE1329C2F178731DB956D82BF015D1212B02EC0EC69D7477C1AE954CBC06689F6A359894C0ADEBBF6B4E8020005AAA95551

DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"


# ----------------------------------------------------------------------------- Fp
def fp_inv(a: int) -> int:
    return pow(a, -1, P)


def fp_sqrt(a: int) -> Optional[int]:
    """p = 3 mod 4: candidate a^((p+1)/4); None if a is a non-residue."""
    a %= P
    y = pow(a, (P + 1) // 4, P)
    return y if (y * y - a) % P == 0 else None


def fp_is_square(a: int) -> bool:
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


# ----------------------------------------------------------------------------- Fp2 = Fp[u]/(u^2+1)
Fp2 = Tuple[int, int]
F2_ZERO: Fp2 = (0, 0)
F2_ONE: Fp2 = (1, 0)


def f2(a0: int, a1: int = 0) -> Fp2:
    return (a0 % P, a1 % P)


def f2_add(a: Fp2, b: Fp2) -> Fp2:
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a: Fp2, b: Fp2) -> Fp2:
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a: Fp2) -> Fp2:
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a: Fp2, b: Fp2) -> Fp2:
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a: Fp2) -> Fp2:
    return f2_mul(a, a)


def f2_muls(a: Fp2, s: int) -> Fp2:
    return ((a[0] * s) % P, (a[1] * s) % P)


def f2_conj(a: Fp2) -> Fp2:
    return (a[0], (-a[1]) % P)


def f2_inv(a: Fp2) -> Fp2:
    n = (a[0] * a[0] + a[1] * a[1]) % P
    ni = fp_inv(n)
    return ((a[0] * ni) % P, (-a[1] * ni) % P)


def f2_pow(a: Fp2, e: int) -> Fp2:
    r = F2_ONE
    b = a
    while e:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_sqr(b)
        e >>= 1
    return r


def f2_is_zero(a: Fp2) -> bool:
    return a[0] == 0 and a[1] == 0


def f2_is_square(a: Fp2) -> bool:
    # a is a square in Fp2 iff its norm a0^2 + a1^2 is a square in Fp
    return fp_is_square((a[0] * a[0] + a[1] * a[1]) % P)


def f2_sqrt(a: Fp2) -> Optional[Fp2]:
    """Some square root of a (either one), or None.  Norm-based ("complex") method."""
    a0, a1 = a[0] % P, a[1] % P
    if a1 == 0:
        r = fp_sqrt(a0)
        if r is not None:
            return (r, 0)
        r = fp_sqrt((-a0) % P)
        return (0, r) if r is not None else None
    alpha = fp_sqrt((a0 * a0 + a1 * a1) % P)
    if alpha is None:
        return None
    inv2 = (P + 1) // 2
    delta = ((a0 + alpha) * inv2) % P
    x0 = fp_sqrt(delta)
    if x0 is None:
        delta = ((a0 - alpha) * inv2) % P
        x0 = fp_sqrt(delta)
        if x0 is None:
            return None
    x1 = (a1 * fp_inv(2 * x0)) % P
    y = (x0, x1)
    return y if f2_sqr(y) == (a0, a1) else None


def sgn0_fp2(a: Fp2) -> int:
    """RFC 9380 §4.1 sgn0 for m = 2."""
    sign_0 = a[0] & 1
    zero_0 = a[0] == 0
    sign_1 = a[1] & 1
    return int(sign_0 or (zero_0 and sign_1))


XI: Fp2 = (1, 1)  # non-residue for the sextic tower: v^3 = xi = 1 + u

# ----------------------------------------------------------------------------- Fp6 = Fp2[v]/(v^3 - xi)
Fp6 = Tuple[Fp2, Fp2, Fp2]
F6_ZERO: Fp6 = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE: Fp6 = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a: Fp6, b: Fp6) -> Fp6:
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a: Fp6, b: Fp6) -> Fp6:
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a: Fp6) -> Fp6:
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a: Fp6, b: Fp6) -> Fp6:
    # schoolbook; v^3 = xi
    a0, a1, a2 = a
    b0, b1, b2 = b
    c0 = f2_add(f2_mul(a0, b0), f2_mul(XI, f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul(XI, f2_mul(a2, b2)))
    c2 = f2_add(f2_add(f2_mul(a0, b2), f2_mul(a1, b1)), f2_mul(a2, b0))
    return (c0, c1, c2)


def f6_mul_by_v(a: Fp6) -> Fp6:
    return (f2_mul(XI, a[2]), a[0], a[1])


def f6_inv(a: Fp6) -> Fp6:
    a0, a1, a2 = a
    t0 = f2_sub(f2_sqr(a0), f2_mul(XI, f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul(XI, f2_sqr(a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    d = f2_add(f2_mul(a0, t0), f2_mul(XI, f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    di = f2_inv(d)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


# ----------------------------------------------------------------------------- Fp12 = Fp6[w]/(w^2 - v)
Fp12 = Tuple[Fp6, Fp6]
F12_ONE: Fp12 = (F6_ONE, F6_ZERO)


def f12_mul(a: Fp12, b: Fp12) -> Fp12:
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c0 = f6_add(t0, f6_mul_by_v(t1))
    c1 = f6_add(f6_mul(a0, b1), f6_mul(a1, b0))
    return (c0, c1)


def f12_sqr(a: Fp12) -> Fp12:
    return f12_mul(a, a)


def f12_conj(a: Fp12) -> Fp12:
    return (a[0], f6_neg(a[1]))


def f12_inv(a: Fp12) -> Fp12:
    a0, a1 = a
    d = f6_sub(f6_mul(a0, a0), f6_mul_by_v(f6_mul(a1, a1)))
    di = f6_inv(d)
    return (f6_mul(a0, di), f6_neg(f6_mul(a1, di)))


def f12_pow(a: Fp12, e: int) -> Fp12:
    r = F12_ONE
    b = a
    while e:
        if e & 1:
            r = f12_mul(r, b)
        b = f12_sqr(b)
        e >>= 1
    return r


def f12_coeffs(a: Fp12):
    """Fp12 as 6 Fp2 coefficients of w^0..w^5 (w^2 = v): c0=(g0,g2,g4), c1=(g1,g3,g5)."""
    (g0, g2, g4), (g1, g3, g5) = a
    return [g0, g1, g2, g3, g4, g5]


def f12_from_coeffs(g) -> Fp12:
    return ((g[0], g[2], g[4]), (g[1], g[3], g[5]))


# Frobenius: (sum g_i w^i)^p = sum conj(g_i) * w^(i p) = sum conj(g_i) * gamma_i * w^i,
# gamma_i = w^(i(p-1)) = xi^(i(p-1)/6)   (w^6 = xi)
GAMMA1 = [f2_pow(XI, i * (P - 1) // 6) for i in range(6)]


def f12_frob(a: Fp12) -> Fp12:
    g = f12_coeffs(a)
    return f12_from_coeffs([f2_mul(f2_conj(g[i]), GAMMA1[i]) for i in range(6)])


# ----------------------------------------------------------------------------- curves (affine, None = infinity)
B1 = 4
B2: Fp2 = (4, 4)  # twist E2: y^2 = x^3 + 4(1+u)

G1Point = Optional[Tuple[int, int]]
G2Point = Optional[Tuple[Fp2, Fp2]]

G1_GEN: G1Point = (G1_X, G1_Y)
G2_GEN: G2Point = (G2_X, G2_Y)


def g1_on_curve(p: G1Point) -> bool:
    if p is None:
        return True
    x, y = p
    return (y * y - x * x * x - B1) % P == 0


def g1_neg(p: G1Point) -> G1Point:
    return None if p is None else (p[0], (-p[1]) % P)


def g1_add(a: G1Point, b: G1Point) -> G1Point:
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1) * fp_inv(2 * y1) % P
    else:
        lam = (y2 - y1) * fp_inv(x2 - x1) % P
    x3 = (lam * lam - x1 - x2) % P
    y3 = (lam * (x1 - x3) - y1) % P
    return (x3, y3)


def g1_mul(p: G1Point, k: int) -> G1Point:
    if k < 0:
        return g1_mul(g1_neg(p), -k)
    r = None
    q = p
    while k:
        if k & 1:
            r = g1_add(r, q)
        q = g1_add(q, q)
        k >>= 1
    return r


def g2_on_curve(p: G2Point) -> bool:
    if p is None:
        return True
    x, y = p
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO


def g2_neg(p: G2Point) -> G2Point:
    return None if p is None else (p[0], f2_neg(p[1]))


def g2_add(a: G2Point, b: G2Point) -> G2Point:
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if f2_add(y1, y2) == F2_ZERO:
            return None
        lam = f2_mul(f2_muls(f2_sqr(x1), 3), f2_inv(f2_muls(y1, 2)))
    else:
        lam = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
    x3 = f2_sub(f2_sub(f2_sqr(lam), x1), x2)
    y3 = f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1)
    return (x3, y3)


def g2_mul(p: G2Point, k: int) -> G2Point:
    if k < 0:
        return g2_mul(g2_neg(p), -k)
    r = None
    q = p
    while k:
        if k & 1:
            r = g2_add(r, q)
        q = g2_add(q, q)
        k >>= 1
    return r


# #E2(Fp2) = H2 * R; H2 = 13^2 * 23^2 * 2713 * 11953 * 262069 * (a 448-bit prime)
H2 = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5
H2_SMALL_PRIMES = (13, 23, 2713, 11953, 262069)
H2_BIG = H2 // (13 ** 2 * 23 ** 2 * 2713 * 11953 * 262069)


def _g2_order_dividing(t: G2Point, m: int, primes) -> int:
    """The order of t, given that it divides m (whose prime factors are `primes`)."""
    for q in primes:
        while m % q == 0 and g2_mul(t, m // q) is None:
            m //= q
    return m


def g2_point_of_order(ell: int, start: int = 2) -> G2Point:
    """A point of E2(Fp2) of order exactly `ell`, a divisor of H2 built from its primes: a deterministic
    curve point times #E2 / (ell's primes' full part of #E2), then times primes until the order is ell.
    Test inputs for the G2 membership test's exceptional cases (tests/test_oracle_bls.py,
    tests/test_gpu_intermediates.py, tools/gen_sop.py --check)."""
    n = H2 * R
    primes = [q for q in H2_SMALL_PRIMES + (H2_BIG,) if ell % q == 0]
    full = 1
    for q in primes:
        while n % (full * q) == 0:
            full *= q
    assert full % ell == 0 and ell > 1
    x = start
    while x < start + 200:  # (E2's 13- and 23-parts have exponent 13 / 23: no point of order 169 or 529)
        X = (x, 1)
        x += 1
        y = f2_sqrt(f2_add(f2_mul(f2_sqr(X), X), B2))
        if y is None:
            continue
        t = g2_mul((X, y), n // full)
        if t is None:
            continue
        o = _g2_order_dividing(t, full, primes)
        if o % ell:
            continue
        t = g2_mul(t, o // ell)
        if t is not None and _g2_order_dividing(t, ell, primes) == ell:
            return t
    raise ValueError(f"no point of order {ell} found on E2")


def g1_in_subgroup(p: G1Point) -> bool:
    return g1_on_curve(p) and g1_mul(p, R) is None


def g2_in_subgroup(p: G2Point) -> bool:
    """Definitional: r * P == O."""
    return g2_on_curve(p) and g2_mul(p, R) is None


# psi = untwist-Frobenius-twist endomorphism on E2
PSI_CX = f2_inv(f2_pow(XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(XI, (P - 1) // 2))


def g2_psi(p: G2Point) -> G2Point:
    if p is None:
        return None
    return (f2_mul(f2_conj(p[0]), PSI_CX), f2_mul(f2_conj(p[1]), PSI_CY))


G1_BETA = 0x5F19672FDF76CE51BA69C6076A0F77EADDB3A93BE6F89688DE17D813620A00022E01FFFFFFFEFFFE
H1 = 0x396C8C005555E1568C00AAAB0000AAAB  # #E1(Fp) / r = 3 * 11^2 * 10177^2 * 859267^2 * 52437899^2


def g1_in_subgroup_phi(p: G1Point) -> bool:
    """Scott's test phi(P) == [-x^2]P with phi(x, y) = (beta x, y) (the GPU's KeyValidate test);
    cross-checked against r*P in tests."""
    if p is None or not g1_on_curve(p):
        return False
    return (G1_BETA * p[0] % P, p[1]) == g1_neg(g1_mul(p, X * X))


def g2_in_subgroup_psi(p: G2Point) -> bool:
    """Scott's test psi(P) == [x]P (the GPU's test); cross-checked against r*P in tests."""
    return g2_on_curve(p) and g2_psi(p) == g2_mul(p, X)


# ----------------------------------------------------------------------------- serialization (ZCash format)
class DecodeError(ValueError):
    pass


def g1_compress(p: G1Point) -> bytes:
    if p is None:
        return bytes([0xC0]) + bytes(47)
    x, y = p
    a_flag = (y * 2) // P
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80 | (0x20 if a_flag else 0)
    return bytes(b)


def g1_decompress(data: bytes) -> G1Point:
    """py_ecc `decompress_G1` rules: c_flag must be 1; b_flag must equal (x == 0); the
    identity must have a_flag == 0; x < p; x^3 + 4 must be a square; a_flag selects y."""
    if len(data) != 48:
        raise DecodeError("length")
    z = int.from_bytes(data, "big")
    c_flag = (z >> 383) & 1
    b_flag = (z >> 382) & 1
    a_flag = (z >> 381) & 1
    if not c_flag:
        raise DecodeError("c_flag")
    x = z & ((1 << 381) - 1)
    is_inf = x == 0
    if b_flag != is_inf:
        raise DecodeError("b_flag")
    if is_inf:
        if a_flag:
            raise DecodeError("infinity a_flag")
        return None
    if x >= P:
        raise DecodeError("x >= p")
    y = fp_sqrt((x * x * x + B1) % P)
    if y is None:
        raise DecodeError("not on curve")
    if (y * 2) // P != a_flag:
        y = P - y
    return (x, y)


def g2_compress(p: G2Point) -> bytes:
    if p is None:
        return bytes([0xC0]) + bytes(95)
    x, y = p
    if y[1] != 0:
        a_flag = (y[1] * 2) // P
    else:
        a_flag = (y[0] * 2) // P
    b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    b[0] |= 0x80 | (0x20 if a_flag else 0)
    return bytes(b)


def g2_decompress(data: bytes) -> G2Point:
    """py_ecc `decompress_G2` rules (x_im || x_re, flags in the top 3 bits of x_im)."""
    if len(data) != 96:
        raise DecodeError("length")
    z1 = int.from_bytes(data[:48], "big")
    z2 = int.from_bytes(data[48:], "big")
    c_flag = (z1 >> 383) & 1
    b_flag = (z1 >> 382) & 1
    a_flag = (z1 >> 381) & 1
    if not c_flag:
        raise DecodeError("c_flag")
    x1 = z1 & ((1 << 381) - 1)
    x0 = z2
    is_inf = x1 == 0 and x0 == 0
    if b_flag != is_inf:
        raise DecodeError("b_flag")
    if is_inf:
        if a_flag:
            raise DecodeError("infinity a_flag")
        return None
    if x1 >= P or x0 >= P:
        raise DecodeError("x >= p")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise DecodeError("not on curve")
    if y[1] != 0:
        flag = (y[1] * 2) // P
    else:
        flag = (y[0] * 2) // P
    if flag != a_flag:
        y = f2_neg(y)
    return (x, y)


# ----------------------------------------------------------------------------- hash_to_G2 (RFC 9380)
SHA_COMPRESSIONS = [0]  # op counter (oracle/canonical.py): compressions of expand_message_xmd's SHA-256 calls


def _sha256(data: bytes) -> bytes:
    SHA_COMPRESSIONS[0] += (len(data) + 8) // 64 + 1
    return hashlib.sha256(data).digest()


def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    """RFC 9380 §5.3.1 with SHA-256 (b_in_bytes = 32, s_in_bytes = 64)."""
    b_in, s_in = 32, 64
    ell = (len_in_bytes + b_in - 1) // b_in
    if ell > 255 or len_in_bytes > 65535 or len(dst) > 255:
        raise ValueError("expand_message_xmd bounds")
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(s_in)
    l_i_b = len_in_bytes.to_bytes(2, "big")
    b0 = _sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime)
    bi = _sha256(b0 + b"\x01" + dst_prime)
    out = bytearray(bi)
    for i in range(2, ell + 1):
        bi = _sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime)
        out += bi
    return bytes(out[:len_in_bytes])


def hash_to_field_fp2(msg: bytes, count: int, dst: bytes):
    """RFC 9380 §5.2, m = 2, L = 64."""
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(ub[off:off + L], "big") % P)
        out.append((e[0], e[1]))
    return out


# 3-isogenous curve E2': y^2 = x^3 + A' x + B'  (RFC 9380 §8.8.2)
ISO_A: Fp2 = (0, 240)
ISO_B: Fp2 = (1012, 1012)
SSWU_Z: Fp2 = f2(-2, -1)

# RFC 9380 Appendix E.3 isogeny map constants (entry j multiplies x'^j)
_XNUM = [
    (0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
     0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
    (0,
     0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
    (0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1, 0),
]
_XDEN = [
    (0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63),
    (0xC, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F),
    (1, 0),
]
_YNUM = [
    (0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
     0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
    (0,
     0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
    (0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10, 0),
]
_YDEN = [
    (0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB,
     0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB),
    (0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3),
    (0x12, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99),
    (1, 0),
]
ISO_XNUM = [f2(*c) for c in _XNUM]
ISO_XDEN = [f2(*c) for c in _XDEN]
ISO_YNUM = [f2(*c) for c in _YNUM]
ISO_YDEN = [f2(*c) for c in _YDEN]


def _poly(coeffs, x: Fp2) -> Fp2:
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_on_curve(pt) -> bool:
    x, y = pt
    return f2_sqr(y) == f2_add(f2_add(f2_mul(f2_sqr(x), x), f2_mul(ISO_A, x)), ISO_B)


def iso_map_g2(pt: Tuple[Fp2, Fp2]) -> G2Point:
    xp, yp = pt
    xd = _poly(ISO_XDEN, xp)
    yd = _poly(ISO_YDEN, xp)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    x = f2_mul(_poly(ISO_XNUM, xp), f2_inv(xd))
    y = f2_mul(yp, f2_mul(_poly(ISO_YNUM, xp), f2_inv(yd)))
    return (x, y)


def sswu_g2(u: Fp2) -> Tuple[Fp2, Fp2]:
    """RFC 9380 §6.6.2 simplified SWU onto E2' (straight-line description)."""
    A, B, Z = ISO_A, ISO_B, SSWU_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    den = f2_add(f2_sqr(zu2), zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(den):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, f2_inv(den)))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    x2 = f2_mul(zu2, x1)
    gx2 = f2_add(f2_add(f2_mul(f2_sqr(x2), x2), f2_mul(A, x2)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x, y = x2, f2_sqrt(gx2)
    assert y is not None
    if sgn0_fp2(u) != sgn0_fp2(y):
        y = f2_neg(y)
    return (x, y)


def map_to_curve_g2(u: Fp2) -> G2Point:
    return iso_map_g2(sswu_g2(u))


def clear_cofactor_g2(p: G2Point) -> G2Point:
    return g2_mul(p, H_EFF_G2)


def hash_to_g2(msg: bytes, dst: bytes = DST_POP) -> G2Point:
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0 = map_to_curve_g2(u0)
    q1 = map_to_curve_g2(u1)
    return clear_cofactor_g2(g2_add(q0, q1))


# ----------------------------------------------------------------------------- pairing
def _line_twist(T: Tuple[Fp2, Fp2], lam: Fp2, p: Tuple[int, int]) -> Fp12:
    """Line through T (on the twist, slope lam) evaluated at P, scaled by w^3 (an Fp4 factor,
    killed by the final exponentiation).  With psi(x', y') = (x' w^-2, y' w^-3):
        l * w^3 = (lam x' - y') - lam xP w^2 + yP w^3,   w^2 = v, w^3 = v w.
    """
    xT, yT = T
    xP, yP = p
    c00 = f2_sub(f2_mul(lam, xT), yT)
    c01 = f2_neg(f2_muls(lam, xP))
    c11 = (yP % P, 0)
    return ((c00, c01, F2_ZERO), (F2_ZERO, c11, F2_ZERO))


def miller_loop(p: G1Point, q: G2Point) -> Fp12:
    """Textbook affine Miller loop f_{|x|,Q}(P) for the optimal ate pairing, conjugated at the end
    because x < 0 (result equals f_{x,Q}(P) up to factors killed by the final exponentiation)."""
    if p is None or q is None:
        return F12_ONE
    f = F12_ONE
    T = q
    bits = bin(X_ABS)[3:]
    for b in bits:
        xT, yT = T
        lam = f2_mul(f2_muls(f2_sqr(xT), 3), f2_inv(f2_muls(yT, 2)))
        f = f12_mul(f12_sqr(f), _line_twist(T, lam, p))
        x3 = f2_sub(f2_sqr(lam), f2_muls(xT, 2))
        y3 = f2_sub(f2_mul(lam, f2_sub(xT, x3)), yT)
        T = (x3, y3)
        if b == "1":
            xT, yT = T
            xQ, yQ = q
            lam = f2_mul(f2_sub(yQ, yT), f2_inv(f2_sub(xQ, xT)))
            f = f12_mul(f, _line_twist(T, lam, p))
            x3 = f2_sub(f2_sub(f2_sqr(lam), xT), xQ)
            y3 = f2_sub(f2_mul(lam, f2_sub(xT, x3)), yT)
            T = (x3, y3)
    return f12_conj(f)  # x < 0


HARD_EXP = (P ** 4 - P ** 2 + 1) // R


def final_exponentiation(f: Fp12) -> Fp12:
    """f ** ((p^12 - 1) / r), exactly: easy part (p^6-1)(p^2+1) via conj/Frobenius, hard part
    (p^4 - p^2 + 1)/r by plain square-and-multiply."""
    f1 = f12_mul(f12_conj(f), f12_inv(f))  # f^(p^6 - 1)
    f2_ = f12_mul(f12_frob(f12_frob(f1)), f1)  # ^(p^2 + 1)
    return f12_pow(f2_, HARD_EXP)


def pairing(p: G1Point, q: G2Point) -> Fp12:
    return final_exponentiation(miller_loop(p, q))


# ----------------------------------------------------------------------------- IETF BLS (POP ciphersuite)
def sk_to_pk(sk: int) -> bytes:
    return g1_compress(g1_mul(G1_GEN, sk))


def sign(sk: int, msg: bytes, dst: bytes = DST_POP) -> bytes:
    return g2_compress(g2_mul(hash_to_g2(msg, dst), sk))


@functools.lru_cache(maxsize=8192)
def key_validate(pk: bytes) -> bool:
    """KeyValidate (memoised: the result is a pure function of the 48 bytes)."""
    try:
        p = g1_decompress(pk)
    except DecodeError:
        return False
    if p is None:
        return False
    return g1_in_subgroup(p)


@functools.lru_cache(maxsize=8192)
def _decode_pk(pk: bytes) -> G1Point:
    return g1_decompress(pk)


def aggregate_pubkeys(pks: Sequence[bytes]) -> G1Point:
    acc = None
    for pk in pks:
        acc = g1_add(acc, _decode_pk(bytes(pk)))
    return acc


def core_verify_point(pk_point: G1Point, msg: bytes, sig: bytes, dst: bytes = DST_POP) -> bool:
    if pk_point is None:
        return False  # KeyValidate(aggregate): identity
    try:
        s = g2_decompress(sig)
    except DecodeError:
        return False
    if not g2_in_subgroup(s):
        return False
    h = hash_to_g2(msg, dst)
    f = f12_mul(miller_loop(pk_point, h), miller_loop(g1_neg(G1_GEN), s))
    return final_exponentiation(f) == F12_ONE


def fast_aggregate_verify(pks: Sequence[bytes], msg: bytes, sig: bytes, dst: bytes = DST_POP) -> bool:
    """IETF FastAggregateVerify (py_ecc semantics: every pubkey KeyValidated; [] -> False)."""
    if len(pks) < 1:
        return False
    for pk in pks:
        if not key_validate(bytes(pk)):
            return False
    agg = aggregate_pubkeys(pks)
    return core_verify_point(agg, bytes(msg), bytes(sig), dst)


def aggregate_signatures(sigs: Sequence[bytes]) -> bytes:
    acc = None
    for s in sigs:
        acc = g2_add(acc, g2_decompress(s))
    return g2_compress(acc)
