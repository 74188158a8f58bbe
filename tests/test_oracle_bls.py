"""CPU checks of the oracle itself (oracle/bls12_381.py, oracle/ssz.py) before it is trusted as the
checker of the HIP path: recalled known-answer vectors, group-order and curve identities,
bilinearity, sign/verify round trips and hypothesis properties of Fp / Fp2 against Python integers.

The BLS arithmetic lives upstream (py_ecc / blst, RFC 9380, the IETF BLS draft) and none of it is in
/root/reference, so these vectors are *recalled*: each was written down from
memory before the oracle was run on it, and the oracle reproduced it byte for byte.
  * eth2 BLS `sign` vectors (consensus-spec-tests general/bls/sign): pubkeys of the secret keys
    0x263d..40e3 and 0x47b8..5138, the signature of 0x263d..40e3 over 32 zero bytes and of
    0x47b8..5138 over 32 bytes of 0x56 (all 96 bytes);
  * RFC 9380 appendix J.10.1 (BLS12381G2_XMD:SHA-256_SSWU_RO_, msg = ""): the x coordinate of P;
  * RFC 9380 appendix K.1 (expand_message_xmd SHA-256, msg = "", len_in_bytes = 0x20).
"""
import hashlib

import pytest
from hypothesis import given, settings, strategies as st

from oracle import bls12_381 as B
from oracle import ssz

SK1 = 0x263DBD792F5B1BE47ED85F8938C0F29586AF0D3AC7B977F21C278FE1462040E3
SK2 = 0x47B8192D77BF871B62E87859D653922725724A5C031AFEABC60BCEF5FF665138
PK1 = "a491d1b0ecd9bb917989f0e74f0dea0422eac4a873e5e2644f368dffb9a6e20fd6e10c1b77654d067c0618f6e5a7f79a"
PK2 = "b301803f8b5ac4a1133581fc676dfedc60d891dd5fa99028805e5ea5b08d3491af75d0707adab3b70c6a6a580217bf81"
SIG1_ZERO = ("b6ed936746e01f8ecf281f020953fbf1f01debd5657c4a383940b020b26507f6076334f91e2366c96e9ab279fb515809"
             "0352ea1c5b0c9274504f4f0e7053af24802e51e4568d164fe986834f41e55c8e850ce1f98458c0cfc9ab380b55285a55")
SIG2_56 = ("af1390c3c47acdb37131a51216da683c509fce0e954328a59f93aebda7e4ff974ba208d9a4a2a2389f892a9d418d6184"
           "18dd7f7a6bc7aa0da999a9d3a5b815bc085e14fd001f6a1948768a3f4afefc8b8240dda329f984cb345c6363272ba4fe")

fp = st.integers(min_value=0, max_value=B.P - 1)


def test_eth2_sign_kats():
    assert B.sk_to_pk(SK1).hex() == PK1
    assert B.sk_to_pk(SK2).hex() == PK2
    assert B.sign(SK1, bytes(32)).hex() == SIG1_ZERO
    assert B.sign(SK2, b"\x56" * 32).hex() == SIG2_56
    assert B.fast_aggregate_verify([bytes.fromhex(PK1)], bytes(32), bytes.fromhex(SIG1_ZERO))
    assert B.fast_aggregate_verify([bytes.fromhex(PK2)], b"\x56" * 32, bytes.fromhex(SIG2_56))
    assert not B.fast_aggregate_verify([bytes.fromhex(PK2)], bytes(32), bytes.fromhex(SIG2_56))


def test_rfc9380_vectors():
    assert B.expand_message_xmd(b"", b"QUUX-V01-CS02-with-expander-SHA256-128", 0x20).hex() == \
        "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"
    x, _ = B.hash_to_g2(b"", b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_")
    assert x == (0x0141EBFBDCA40EB85B87142E130AB689C673CF60F1A3E98D69335266F30D9B8D4AC44C1038E9DCDD5393FAF5C41FB78A,
                 0x05CB8437535E20ECFFAEF7752BADDF98034139C38452458BAEEFAB379BA13DFF5BF5DD71B72418717047F5B0F37DA03D)


def test_curve_identities():
    x = B.X
    assert B.R == x ** 4 - x ** 2 + 1
    assert B.P == (x - 1) ** 2 * B.R // 3 + x
    assert B.P % 4 == 3
    assert B.g1_on_curve(B.G1_GEN) and B.g2_on_curve(B.G2_GEN)
    assert B.g1_mul(B.G1_GEN, B.R) is None  # r * G1 = O
    assert B.g2_mul(B.G2_GEN, B.R) is None  # r * G2 = O
    assert B.g1_compress(B.G1_GEN).hex().startswith("97f1d3a73197d794")
    assert B.g2_compress(B.G2_GEN).hex().startswith("93e02b6052719f60")
    # the psi-based subgroup test agrees with the definitional one (members and a non-member)
    Q = B.g2_mul(B.G2_GEN, 0x1234567)
    assert B.g2_in_subgroup(Q) and B.g2_in_subgroup_psi(Q)
    xx = 1
    while True:
        xx += 1
        X = (xx, 3)
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(X), X), B.B2))
        if y is not None:
            break
    assert not B.g2_in_subgroup((X, y)) and not B.g2_in_subgroup_psi((X, y))


def test_g1_membership_phi_matches_definition():
    """KeyValidate's G1 membership test on the device is phi(P) == [-x^2]P: it agrees with r*P == O on
    members, on points whose order has each prime factor of the cofactor h1, and on mixed points."""
    import random
    rng = random.Random(7)
    assert B.H1 == 3 * 11 ** 2 * 10177 ** 2 * 859267 ** 2 * 52437899 ** 2
    assert pow(B.G1_BETA, 3, B.P) == 1

    def curve_point():
        while True:
            x = rng.randrange(B.P)
            y = B.fp_sqrt((x ** 3 + B.B1) % B.P)
            if y is not None:
                return (x, y)
    seen = set()
    for _ in range(3):
        g = B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))
        assert B.g1_in_subgroup(g) and B.g1_in_subgroup_phi(g)
        q = curve_point()
        for ell in (3, 11, 10177, 859267, 52437899, B.H1):
            # E1(Fp)'s ell-part is Z/ell x Z/ell for the squared primes: [h1 r / ell^2]Q has order ell
            t = B.g1_mul(q, B.H1 * B.R // (ell if ell in (3, B.H1) else ell * ell))
            if t is None:
                continue
            if ell != B.H1:
                assert B.g1_mul(t, ell) is None
            seen.add(ell)
            assert not B.g1_in_subgroup(t) and not B.g1_in_subgroup_phi(t), ell
            m = B.g1_add(g, t)
            assert not B.g1_in_subgroup(m) and not B.g1_in_subgroup_phi(m), ell
        assert B.g1_in_subgroup(q) == B.g1_in_subgroup_phi(q)
    assert seen >= {3, 11, 10177, 859267, 52437899}


def test_bilinearity():
    a, b = 0x1D5E7, 0x2B9F3
    e = B.pairing(B.G1_GEN, B.G2_GEN)
    assert e != B.f12_pow(e, 0)  # non-degenerate
    lhs = B.pairing(B.g1_mul(B.G1_GEN, a), B.g2_mul(B.G2_GEN, b))
    assert lhs == B.f12_pow(e, a * b)
    assert B.f12_pow(e, B.R) == B.f12_pow(e, 0)  # e has order r


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sign_verify_round_trip(seed):
    import random
    rnd = random.Random(seed)
    sks = [rnd.randrange(1, B.R) for _ in range(3)]
    msg = rnd.randbytes(32)
    pks = [B.sk_to_pk(k) for k in sks]
    sig = B.aggregate_signatures([B.sign(k, msg) for k in sks])
    assert B.fast_aggregate_verify(pks, msg, sig)
    assert sig == B.sign(sum(sks) % B.R, msg)  # aggregate of signatures = signature of summed keys
    assert not B.fast_aggregate_verify(pks[:2], msg, sig)
    assert not B.fast_aggregate_verify(pks, bytes(32) if msg != bytes(32) else b"\x01" * 32, sig)
    assert not B.fast_aggregate_verify([], msg, sig)


def test_sha_and_merkle_vs_hashlib():
    for n in (0, 1, 55, 56, 63, 64, 65, 119, 128, 1000):
        data = bytes(range(256)) * 4
        assert ssz.sha256(data[:n]) == hashlib.sha256(data[:n]).digest()
    chunks = [hashlib.sha256(bytes([i])).digest() for i in range(5)]
    z = bytes(32)
    h = lambda a, b: hashlib.sha256(a + b).digest()  # noqa: E731
    want = h(h(h(chunks[0], chunks[1]), h(chunks[2], chunks[3])), h(h(chunks[4], z), h(z, z)))
    assert ssz.merkleize(chunks) == want


@settings(max_examples=60, deadline=None)
@given(fp, fp, fp, fp)
def test_fp2_field_properties(a0, a1, b0, b1):
    a, b = (a0, a1), (b0, b1)
    ab = B.f2_mul(a, b)
    assert ab == ((a0 * b0 - a1 * b1) % B.P, (a0 * b1 + a1 * b0) % B.P)
    assert B.f2_sqr(a) == B.f2_mul(a, a)
    if a != (0, 0):
        assert B.f2_mul(a, B.f2_inv(a)) == (1, 0)
    s = B.f2_sqrt(B.f2_sqr(a))
    assert s is not None and (s == a or s == B.f2_neg(a))
    r = B.f2_sqrt(b)
    assert (r is not None) == B.f2_is_square(b)
    if r is not None:
        assert B.f2_sqr(r) == b


@settings(max_examples=60, deadline=None)
@given(fp)
def test_fp_sqrt_and_inverse(a):
    if a:
        assert a * B.fp_inv(a) % B.P == 1
    s = B.fp_sqrt(a * a % B.P)
    assert s is not None and s * s % B.P == a * a % B.P
    assert (B.fp_sqrt(a) is not None) == B.fp_is_square(a)


def test_point_encoding_round_trip():
    import random
    rnd = random.Random(4)
    for _ in range(4):
        k = rnd.randrange(1, B.R)
        p1, p2 = B.g1_mul(B.G1_GEN, k), B.g2_mul(B.G2_GEN, k)
        assert B.g1_decompress(B.g1_compress(p1)) == p1
        assert B.g2_decompress(B.g2_compress(p2)) == p2


def test_g2_torsion_points():
    """The E2 points of tests/g2_edge_points.py: on the curve, of the stated order, outside G2 by r*P and
    by the psi test; order 13 puts the |x| walk at T = -Q before its second addition; no point of E2
    reaches T = +Q at an addition (gcd(k - 1, #E2) = 1 for every addition prefix k)."""
    from math import gcd
    import g2_edge_points as E
    n = B.H2 * B.R
    k, prefixes = 1, []
    for bit in bin(B.X_ABS)[3:]:
        k *= 2
        if bit == "1":
            prefixes.append(k)
            k += 1
    assert tuple(prefixes) == E.ADD_PREFIXES and k == B.X_ABS
    assert all(gcd(p - 1, n) == 1 for p in prefixes)
    assert [p for p in prefixes if gcd(p + 1, n) > 1] == [12]  # 13 | 12 + 1: only T = -Q is reachable
    for name, p in E.edge_points().items():
        assert B.g2_on_curve(p) and p is not None, name
        assert not B.g2_in_subgroup(p) and not B.g2_in_subgroup_psi(p), name
        assert B.g2_decompress(B.g2_compress(p)) == p, name
    o13 = B.g2_point_of_order(13)
    assert B.g2_mul(o13, 12) == B.g2_neg(o13) and B.g2_mul(o13, 13) is None
    for ell in (23, 2713, 11953, 262069):
        q = B.g2_point_of_order(ell)
        assert B.g2_mul(q, ell) is None and B.g2_mul(q, ell // ell) is not None
