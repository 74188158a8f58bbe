"""GPU parity of INTERMEDIATE values (north star: verdicts and intermediate points bit-exact):
the windowed sqrt exponentiations, decoded signature points, masked aggregate pubkeys (including
committees with duplicate members, which drive the doubling branch of the mixed addition), G1 key
decode/KeyValidate edge cases, and FastAggregateVerify over such committees — liblcv.so through the
C ABI vs the CPU oracle (oracle/bls12_381.py).  Reference call site: sync-protocol.md:456-464.

LCV_TEST_HOSTSIM=1 runs the same tests on the host simulation of the device code (CPU dry run).
"""
import random

import numpy as np
import pytest

from oracle import bls12_381 as B

pytestmark = pytest.mark.gpu

P = B.P


def _be48(x: int) -> bytes:
    return x.to_bytes(48, "big")


def _ints(row, k):
    b = bytes(row)
    return [int.from_bytes(b[48 * i:48 * i + 48], "big") for i in range(k)]


def _non_subgroup_g1(start: int):
    """A point of E1(Fp) outside G1 (the cofactor is > 1, so almost every curve point is)."""
    x = start
    while True:
        x += 1
        y = B.fp_sqrt((x * x * x + B.B1) % P)
        if y is not None and not B.g1_in_subgroup((x, y)):
            return (x, y)


def _non_subgroup_g2(start: int):
    x = start
    while True:
        x += 1
        X = (x, 7)
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(X), X), B.B2))
        if y is not None and not B.g2_in_subgroup((X, y)):
            return (X, y)


def _oracle_sig(sig: bytes):
    """(status, affine point) with the device's status codes: 0 ok, 1 identity, 2 invalid."""
    try:
        pt = B.g2_decompress(sig)
    except B.DecodeError:
        return 2, None
    if pt is None:
        return 1, None
    return (0, pt) if B.g2_in_subgroup(pt) else (2, pt)


@pytest.mark.parametrize("latency_rows", [64, 0])
def test_fp_pow_windowed(gpu_verifier, latency_rows):
    """fp_pow_p1d4 / fp_pow_p3d4 (sliding window) vs pow() on edge and random inputs: latency mode (64) runs
    the latency twins' chains (one value per wave, each product spread over the wave: lcv_wave.hpp), 0 the
    batch kernels' one-lane chains."""
    rng = random.Random(21)
    xs = [0, 1, 2, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 4, 5, (1 << 380) % P, P - (1 << 370)]
    while len(xs) < 40:
        a = rng.randrange(P)
        xs.append(a)
        xs.append(a * a % P)  # a residue
    prev = getattr(gpu_verifier, "latency_mode", 64)
    gpu_verifier.set_latency_mode(latency_rows)
    try:
        out = gpu_verifier.debug_fp_pow(np.frombuffer(b"".join(_be48(x) for x in xs), np.uint8))
    finally:
        gpu_verifier.set_latency_mode(prev)
    for i, x in enumerate(xs):
        got = _ints(out[i], 2)
        assert got == [pow(x, (P + 1) // 4, P), pow(x, (P - 3) // 4, P)], x


def test_g2_decompress_points(gpu_verifier):
    """Decoded signature point and status (flags, x >= p, off-curve, outside G2, identity)."""
    rng = random.Random(22)
    sigs = [B.g2_compress(B.g2_mul(B.G2_GEN, rng.randrange(1, B.R))) for _ in range(6)]
    sigs.append(B.sign(0x1234, b"\x42" * 32))
    sigs.append(bytes([0xC0]) + bytes(95))                      # identity: valid encoding
    sigs.append(bytes([0xE0]) + bytes(95))                      # identity with a_flag
    sigs.append(bytes([0x40]) + bytes(95))                      # no compression flag
    ok = bytearray(sigs[0])
    ok[0] &= 0x7F
    sigs.append(bytes(ok))                                      # c_flag cleared on a real point
    ok = bytearray(sigs[1])
    ok[0] |= 0x40
    sigs.append(bytes(ok))                                      # b_flag set on a finite point
    sigs.append(bytes([0x80 | 0x1A]) + bytes([0xFF]) * 47 + bytes(48))  # x_im >= p
    sigs.append(bytes([0x80]) + bytes(47) + _be48(P))           # x_re == p
    x = 3
    while True:  # off curve: x^3 + b is not a square in Fp2
        x += 1
        X = (x, 1)
        if B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(X), X), B.B2)) is None:
            break
    sigs.append(_be48((1 << 383) | 1) + _be48(x))                # x = x + 1 u (c_flag on x_im)
    sigs.append(B.g2_compress(_non_subgroup_g2(10)))          # on the curve, outside G2
    sigs.append(B.g2_compress(_non_subgroup_g2(1000)))
    out, st = gpu_verifier.debug_g2_decompress(np.frombuffer(b"".join(sigs), np.uint8))
    for i, s in enumerate(sigs):
        want_st, pt = _oracle_sig(s)
        assert int(st[i]) == want_st, (i, s.hex())
        if want_st == 0:
            g = _ints(out[i], 4)
            assert ((g[0], g[1]), (g[2], g[3])) == pt, i


def _committee(seed: int, dup_pairs=()):
    rng = random.Random(seed)
    sks = [rng.randrange(1, B.R) for _ in range(512)]
    for a, b in dup_pairs:  # member b duplicates member a (sampling with replacement on mainnet)
        sks[b] = sks[a]
    pks = [B.sk_to_pk(k) for k in sks]
    return sks, pks


def _bits(idx):
    b = bytearray(64)
    for j in idx:
        b[j // 8] |= 1 << (j % 8)
    return bytes(b)


def test_aggregate_points_with_duplicates(gpu_verifier):
    """Masked aggregate (both the direct sum and the > 256 complement trick) vs the oracle, on a
    committee with adjacent and distant duplicate members."""
    dups = [(3, 4), (10, 300), (511, 0), (100, 101), (101, 102)]
    sks, pks = _committee(23, dups)
    table = np.frombuffer(b"".join(pks), np.uint8)
    rng = random.Random(24)
    sets = [
        [3, 4],                                   # P + P through the mixed addition
        [10, 300, 5],
        [100, 101, 102],                          # 3P
        list(range(512)),                         # everything (complement with no removals)
        [j for j in range(512) if j not in (4, 101)],  # complement removing one copy of a duplicate
        sorted(rng.sample(range(512), 200)),
        sorted(rng.sample(range(512), 400)) + [],
        [0, 511],
        [7],
    ]
    bits = np.frombuffer(b"".join(_bits(s) for s in sets), np.uint8)
    out, st = gpu_verifier.debug_aggregate(table, np.zeros(len(sets), np.uint32), bits)
    for i, s in enumerate(sets):
        want = B.aggregate_pubkeys([pks[j] for j in s])
        assert int(st[i]) == (1 if want is None else 0), i
        if want is not None:
            assert tuple(_ints(out[i], 2)) == want, i


def test_aggregate_cancelling_to_identity(gpu_verifier):
    """Members P and -P: the aggregate is the identity (KeyValidate(aggregate) fails -> status 1)."""
    rng = random.Random(25)
    sks = [rng.randrange(1, B.R) for _ in range(512)]
    sks[9] = B.R - sks[8]
    pks = [B.sk_to_pk(k) for k in sks]
    out, st = gpu_verifier.debug_aggregate(np.frombuffer(b"".join(pks), np.uint8), np.zeros(2, np.uint32),
                                           np.frombuffer(_bits([8, 9]) + _bits([8, 9, 10]), np.uint8))
    assert list(st) == [1, 0]
    assert tuple(_ints(out[1], 2)) == B.g1_decompress(pks[10])


def _bad_keys():
    gen = B.g1_compress(B.G1_GEN)
    ns = _non_subgroup_g1(5)
    x = 0
    while True:  # x^3 + 4 not a square: off the curve
        x += 1
        if B.fp_sqrt((x ** 3 + B.B1) % P) is None:
            break
    return {
        "identity": bytes([0xC0]) + bytes(47),
        "identity_a_flag": bytes([0xE0]) + bytes(47),
        "no_c_flag": bytes([gen[0] & 0x7F]) + gen[1:],
        "b_flag_on_point": bytes([gen[0] | 0x40]) + gen[1:],
        "x_eq_p": bytes([0x80 | (P >> 376)]) + _be48(P)[1:],
        "x_max": bytes([0x9F]) + bytes([0xFF]) * 47,
        "off_curve": bytes([0x80 | (x >> 376)]) + _be48(x)[1:],
        "non_subgroup": B.g1_compress(ns),
        "all_zero": bytes(48),
        # points whose order is a cofactor prime (3, 11, 10177) and a G1 point plus an order-11 point:
        # each exercises the device's phi(P) == [-x^2]P membership test against r*P == O
        "order3": B.g1_compress(_cofactor_point(3)),
        "order11": B.g1_compress(_cofactor_point(11)),
        "order10177": B.g1_compress(_cofactor_point(10177)),
        "g1_plus_order11": B.g1_compress(B.g1_add(B.g1_mul(B.G1_GEN, 12345), _cofactor_point(11))),
    }


def _cofactor_point(ell: int):
    """A point of E1(Fp) of order ell (a prime factor of the cofactor h1; ell^2 divides h1 for ell > 3,
    and E1(Fp)'s ell-part is then Z/ell x Z/ell, of exponent ell)."""
    k = B.H1 * B.R // (ell if ell == 3 else ell * ell)
    x = 1
    while True:
        x += 1
        y = B.fp_sqrt((x * x * x + B.B1) % P)
        if y is None:
            continue
        t = B.g1_mul((x, y), k)
        if t is not None:
            assert B.g1_mul(t, ell) is None
            return t


def test_g1_key_validate_edges(gpu_verifier):
    """KeyValidate of every committee member (lcv_set_store's key status) vs the oracle, and the
    aggregate status when an invalid key participates (FastAggregateVerify -> False)."""
    bad = _bad_keys()
    sks, pks = _committee(26)
    pos = {}
    for k, (name, kb) in enumerate(bad.items()):
        j = 17 + 37 * k
        pks[j] = kb
        pos[name] = j
    cur = b"".join(pks) + bytes(48)
    ks = gpu_verifier.set_store(0, cur, bytes(24624))
    for j in range(512):
        assert (ks[j] == 0) == B.key_validate(pks[j]), (j, pks[j].hex())
    for name, j in pos.items():
        assert ks[j] == 2, name
    # aggregate status: 2 when a bad key participates (direct and complement paths), else the sum
    table = np.frombuffer(b"".join(pks), np.uint8)
    good = [j for j in range(512) if j not in pos.values()]
    sets = [[pos["non_subgroup"], 1, 2], [j for j in range(512) if j != pos["identity"]], good[:300], good[:20]]
    out, st = gpu_verifier.debug_aggregate(table, np.zeros(len(sets), np.uint32),
                                           np.frombuffer(b"".join(_bits(s) for s in sets), np.uint8))
    assert list(st[:2]) == [2, 2]
    for i in (2, 3):
        assert int(st[i]) == 0
        assert tuple(_ints(out[i], 2)) == B.aggregate_pubkeys([pks[j] for j in sets[i]])


def test_fast_aggregate_verify_batch_duplicates(gpu_verifier):
    """lcv_fast_aggregate_verify_batch over two committee tables (one with duplicate members and
    an invalid key) vs the oracle's FastAggregateVerify, item by item."""
    sksA, pksA = _committee(27, [(1, 2), (50, 400)])
    sksB, pksB = _committee(28)
    pksB[5] = _bad_keys()["non_subgroup"]
    rng = random.Random(29)
    items = []
    for t in range(10):
        c = t % 2
        sks, pks = (sksA, pksA) if c == 0 else (sksB, pksB)
        if t == 0:
            idx = [1, 2]
        elif t == 2:
            idx = [j for j in range(512) if j != 2]
        elif t == 4:
            idx = [50, 400] + list(range(60, 200))
        elif t == 5:
            idx = [5, 6, 7]  # bad key participates
        else:
            idx = sorted(rng.sample([j for j in range(512) if not (c == 1 and j == 5)], rng.randrange(1, 512)))
        msg = rng.randbytes(32)
        sk = sum(sks[j] for j in idx) % B.R
        sig = B.sign(sk, msg if t != 6 else b"\x00" * 32)  # item 6: signature over another message
        if t == 8:
            sig = bytes([0xC0]) + bytes(95)  # identity signature
        items.append((c, idx, msg, sig, pks))
    committees = np.frombuffer(b"".join(pksA) + b"".join(pksB), np.uint8)
    got = gpu_verifier.fast_aggregate_verify_batch(
        committees, np.array([c for c, *_ in items], np.uint32),
        np.frombuffer(b"".join(_bits(i) for _, i, *_ in items), np.uint8),
        np.frombuffer(b"".join(m for _, _, m, _, _ in items), np.uint8),
        np.frombuffer(b"".join(s for *_, s, _ in items), np.uint8))
    want = [B.fast_aggregate_verify([pks[j] for j in idx], msg, sig) for c, idx, msg, sig, pks in items]
    assert list(got) == want
    assert want[0] and want[2] and want[4] and not want[5] and not want[6] and not want[8]
