"""The canonical-algorithm op counter (oracle/canonical.py; SURVEY.md §8(d)'s roofline numerator):
every textbook algorithm it counts computes the definitional oracle's values, and the committed counts
in profiles/opcounts.json["canonical"] are what the counter produces (so every per-kernel frac in the
bench line recomputes from profiles/ by hand)."""
import json
import os
import random

import pytest

import helpers as H
from oracle import bls12_381 as B
from oracle import canonical as K


@pytest.mark.parametrize("tower", ["karatsuba", "schoolbook"])
def test_tower_and_cyclotomic_ops_match_oracle(tower):
    rnd = random.Random(7)
    f = tuple(tuple((rnd.randrange(B.P), rnd.randrange(B.P)) for _ in range(3)) for _ in range(2))
    g = tuple(tuple((rnd.randrange(B.P), rnd.randrange(B.P)) for _ in range(3)) for _ in range(2))
    m = B.f12_mul(B.f12_frob(B.f12_frob(B.f12_mul(B.f12_conj(f), B.f12_inv(f)))), B.f12_mul(B.f12_conj(f), B.f12_inv(f)))
    K.MODE["tower"] = tower
    try:
        F, G, M = K.f12_from_oracle(f), K.f12_from_oracle(g), K.f12_from_oracle(m)
        assert K.f12_to_oracle(K.f12_mul(F, G)) == B.f12_mul(f, g)
        assert K.f12_to_oracle(K.f12_sqr(F)) == B.f12_sqr(f)
        assert K.f12_to_oracle(K.f12_inv(F)) == B.f12_inv(f)
        assert K.f12_to_oracle(K.f12_frob(F, 1)) == B.f12_frob(f)
        assert K.f12_to_oracle(K.f12_frob(F, 2)) == B.f12_frob(B.f12_frob(f))
        assert K.f12_to_oracle(K.f12_cyc_sqr(M)) == B.f12_sqr(m)  # Granger-Scott on the cyclotomic subgroup
    finally:
        K.MODE["tower"] = "karatsuba"


def test_curve_formulas_match_oracle():
    Q = B.g2_mul(B.G2_GEN, 12345)
    R = B.g2_mul(B.G2_GEN, 777)
    one = K.f2c((1, 0))
    T = (K.f2c(Q[0]), K.f2c(Q[1]), one)
    aff = lambda t: tuple(c.t() for c in K.g2_to_affine(t))  # noqa: E731
    T2, _ = K.g2_dbl(T)
    assert aff(T2) == B.g2_add(Q, Q)
    T3, _ = K.g2_add_mixed(T2, (K.f2c(R[0]), K.f2c(R[1])))
    assert aff(T3) == B.g2_add(B.g2_add(Q, Q), R)
    assert aff(K.g2_add(T2, T3)) == B.g2_add(B.g2_add(Q, Q), aff(T3))
    assert aff(K.g2_psi(T)) == B.g2_psi(Q)
    assert aff(K.g2_mul_abs_x(T)) == B.g2_mul(Q, B.X_ABS)
    # subgroup test: members pass, a non-member (random curve point, cofactor component) fails
    assert K.g2_subgroup_psi((K.f2c(Q[0]), K.f2c(Q[1])))
    x = (5, 1)
    while True:
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B2))
        if y is not None:
            break
        x = (x[0] + 1, 1)
    assert not B.g2_in_subgroup((x, y)) and not K.g2_subgroup_psi((K.f2c(x), K.f2c(y)))
    # G1 Jacobian sums
    pts = [B.g1_mul(B.G1_GEN, k) for k in (3, 5, 11, 17)]
    acc = (K.Fp(pts[0][0]), K.Fp(pts[0][1]), K.Fp(1))
    for p in pts[1:]:
        acc = K.g1_madd(acc, (K.Fp(p[0]), K.Fp(p[1])))
    a = K.g1_to_affine(acc)
    assert (a[0].v, a[1].v) == B.g1_mul(B.G1_GEN, 36)


def test_hash_to_g2_and_pairing_match_oracle():
    msg = bytes(range(32))
    us = K.hash_to_field(msg)
    assert [u.t() for u in us] == B.hash_to_field_fp2(msg, 2, B.DST_POP)
    maps = [K.sswu(u) for u in us]
    assert [(x.t(), y.t()) for x, y in maps] == [B.sswu_g2(u.t()) for u in us]
    H2 = K.g2_to_affine(K.clear_cofactor(K.g2_add(*(K.iso_map_projective(m) for m in maps))))
    assert (H2[0].t(), H2[1].t()) == B.hash_to_g2(msg)
    # one pairing: canonical Miller loop + HHT final exponentiation == oracle pairing ^ 3
    P1, Q = B.g1_mul(B.G1_GEN, 99), B.g2_mul(B.G2_GEN, 5)
    lines = K.miller_lines((K.Fp(P1[0]), K.Fp(P1[1])), (K.f2c(Q[0]), K.f2c(Q[1])))
    unit = ((K.f2c((1, 0)), K.FP0, K.FP0), (K.FP0, K.FP0, K.FP0))
    e = K.final_exponentiation(K._densify(K.miller_acc(lines, [unit] * len(lines))))
    eo = B.pairing(P1, Q)
    assert K.f12_to_oracle(e) == B.f12_mul(B.f12_mul(eo, eo), eo)


def test_committed_canonical_counts_reproduce():
    """profiles/opcounts.json["canonical"] == a fresh count (deterministic: fixed seeds, fixed algorithms)."""
    import sys
    sys.path.insert(0, os.path.join(H.ROOT, "tools"))
    import canonical_count
    oc = json.load(open(os.path.join(H.ROOT, "profiles", "opcounts.json")))["canonical"]
    fresh = canonical_count.count(2, "full", "karatsuba")
    assert fresh["per_update"] == oc["per_update"] and fresh["per_committee"] == oc["per_committee"]
    assert oc["per_committee"]["nsc_htr"]["sha"] == 2050  # HTR(SyncCommittee): 1,025 SHA-256 calls
    # the canonical numerator is never below the device's executed count for the pairing kernels
    ex = json.load(open(os.path.join(H.ROOT, "profiles", "opcounts.json")))["per_update"]
    for st in ("miller_loop", "final_exp"):
        assert oc["per_update"][st]["int32_ops"] >= 0.95 * ex[st]["int32_ops"]
