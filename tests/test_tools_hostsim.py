"""CPU checks of the build tooling and of device arithmetic through the host simulation:
  * tools/gen_sop.py emulates every SOP program (line walk + fused G2 subgroup check, Miller
    accumulation, final exponentiation, hash_to_G2 tail) with Python integers against the oracle;
  * tools/opcount.py (the roofline numerator) attributes work to every BLS stage, one mark per kernel;
  * the windowed sqrt exponentiations of lcv_field.hpp vs pow() (host simulation of the device code).
"""
import os
import sys

import numpy as np
import pytest

import helpers as H

sys.path.insert(0, os.path.join(H.ROOT, "tools"))

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def test_sop_programs_match_oracle():
    """tools/gen_sop.py emulates every SOP program with Python integers (exact device semantics:
    Montgomery representatives, unreduced accumulators, REDC, the header's subtraction count) against
    the oracle's pairing, final exponentiation and hash_to_G2; the committed kernel header is what the
    generator emits now (no stale program ships)."""
    import gen_sop as GS
    progs = GS.build()
    for p in progs:
        p.finalize()
    GS.check_miller(progs[0], progs[1])
    GS.check_miller_fused(progs[0], progs[1], progs[4])  # latency mode's walks + accumulation in one program
    GS.check_fexp(progs[2])
    GS.check_h2c(progs[3])
    text = open(os.path.join(H.PKG, "csrc", "lcv_sop_programs.inc")).read()
    schoolbook = False
    for p in progs:
        hdr, _ = p.encode()
        assert f"#define LCV_SOP_{p.name.upper()}_ROUNDS {len(hdr) // 4}" in text
        assert f"#define LCV_SOP_{p.name.upper()}_SLOTS {p.nslots}" in text
        schoolbook |= any((w0 & 15) and not (w0 >> 22) & 1 for w0 in hdr[0::4])
    # the device compiles the schoolbook scans out when no product round needs them (lcv_sop.hpp)
    assert f"#define LCV_SOP_SCHOOLBOOK {int(schoolbook)}" in text
    assert not schoolbook, "every product round is Karatsuba since the line walk's 48 C' operand"


def test_opcount_every_stage():
    ops = os.path.join(H.PKG, "build", "liblcv_hostsim_ops.so")
    if not os.path.exists(ops):
        import subprocess
        subprocess.check_call(["make", "-s", "hostsim"], cwd=H.PKG)
    import opcount
    c = opcount.count(2)
    per = c["per_update"]
    for st in ("h2c_sswu", "hash_to_g2", "sig_decode", "miller_lines_sig", "g1_aggregate", "miller_lines",
               "miller_loop", "final_exp"):
        assert per.get(st, {}).get("fp_mul", 0) > 0, st
    assert per["pre_checks"]["sha"] > 0
    # HTR(SyncCommittee) is charged per distinct committee: 1,025 SHA-256 calls = 2,050 compressions
    assert "nsc_htr" not in per and c["per_committee"]["nsc_htr"]["sha"] == 2050
    # the SOP programs' products and reductions are what the op counter sees (padding products excluded):
    # each is half of a reduced Fp multiplication
    import gen_sop as GS
    lp, ap, fp = GS.build()[:3]
    for p in (lp, ap, fp):
        p.finalize()  # the negated-shadow pass may add a first round

    def half_muls(p):  # products + one reduction per op of a round with products (K = 0 rounds skip it)
        return sum(len(o.prods) + (1 if max(len(q.prods) for q in r) else 0) for r in p.rounds for o in r) / 2
    assert per["final_exp"]["fp_mul"] == half_muls(fp) + 1  # + the inversion's Montgomery correction (y R^3)
    assert per["miller_loop"]["fp_mul"] == half_muls(ap)
    assert per["miller_lines"]["fp_mul"] == half_muls(lp) == per["miller_lines_sig"]["fp_mul"]
    tot = c["total_per_update"]
    assert abs(sum(d["fp_mul"] for d in per.values()) - tot["fp_mul"]) < 1e-6


def test_windowed_pow_hostsim(sim_verifier):
    rng = np.random.default_rng(5)
    xs = [0, 1, 2, P - 1, P - 2, (P - 1) // 2] + [int.from_bytes(rng.bytes(48), "big") % P for _ in range(20)]
    xs += [x * x % P for x in xs[6:12]]
    out = sim_verifier.debug_fp_pow(np.frombuffer(b"".join(x.to_bytes(48, "big") for x in xs), np.uint8))
    for i, x in enumerate(xs):
        b = out[i].tobytes()
        assert int.from_bytes(b[:48], "big") == pow(x, (P + 1) // 4, P)
        assert int.from_bytes(b[48:], "big") == pow(x, (P - 3) // 4, P)


def test_fp_inverse_hostsim(sim_verifier):
    """Bernstein-Yang inversion (lcv_field.hpp fp_inv_by) against pow(a, p - 2, p): 0 (inv0), 1, p - 1,
    powers of two and p minus powers of two (long runs of equal bits), limb-boundary values, random."""
    rng = np.random.default_rng(6)
    xs = [0, 1, 2, 3, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, (1 << 30) - 1, 1 << 30, 1 << 32, (1 << 360) - 1]
    xs += [(1 << k) % P for k in range(0, 384, 11)] + [P - (1 << k) for k in range(0, 380, 17)]
    xs += [int.from_bytes(rng.bytes(48), "big") % P for _ in range(400)]
    a = np.frombuffer(b"".join(x.to_bytes(48, "big") for x in xs), np.uint8)
    out, _ = sim_verifier.debug_fp(a, a)
    for i, x in enumerate(xs):
        assert int.from_bytes(out[i].tobytes()[144:192], "big") == pow(x, P - 2, P), hex(x)
