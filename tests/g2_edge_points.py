"""Signatures on E2 outside G2 that drive the fused G2 membership check (psi(Q) == [x]Q, folded into the
signature pairing's line walk, tools/gen_sop.py line_program) into its exceptional cases.

* Points of each small prime order of the cofactor H2 (13, 23, 2713, 11953, 262069), composite orders,
  and of the 448-bit prime H2_BIG.
* Order 13: the walk's T reaches -Q at its second addition step ([12]Q = -Q), so T + Q = O there and the
  walk continues from the identity (the exceptional case the design argues leaves Z = 0 for good).
* G2 + small-torsion sums: members of no subgroup the test could accept.
* T = +Q at an addition step needs ord(Q) | k - 1 for an addition prefix k of |x| (2, 12, 104, 53760,
  230901736800256); gcd(k - 1, #E2) = 1 for each, so no point of E2(Fp2) reaches it
  (tests/test_oracle_bls.py::test_g2_torsion_points checks this)."""
from oracle import bls12_381 as B

ADD_PREFIXES = (2, 12, 104, 53760, 230901736800256)  # [k]Q held by T before each addition of the |x| walk


def edge_points():
    g = B.g2_mul(B.G2_GEN, 0x1234567)
    h = B.hash_to_g2(b"\x07" * 32)
    o13 = B.g2_point_of_order(13)
    pts = {f"order_{ell}": B.g2_point_of_order(ell) for ell in (13, 23, 299, 2713, 11953, 262069, 13 * 2713)}
    pts["order_h2big"] = B.g2_point_of_order(B.H2_BIG)
    pts["neg_order_13"] = B.g2_neg(o13)
    pts["g2_plus_order_13"] = B.g2_add(g, o13)
    pts["g2_plus_order_23"] = B.g2_add(g, B.g2_point_of_order(23))
    pts["g2_plus_order_2713"] = B.g2_add(g, B.g2_point_of_order(2713))
    pts["g2_plus_order_h2big"] = B.g2_add(g, pts["order_h2big"])
    pts["hash_plus_order_13"] = B.g2_add(h, o13)
    return pts


def edge_signatures():
    """name -> 96-byte compressed signature (every one decodes to a curve point outside G2)."""
    return {k: B.g2_compress(p) for k, p in edge_points().items()}
