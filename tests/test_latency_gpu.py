"""Latency mode (lcv_set_latency_mode(max_rows); default 64): batches of at most max_rows rows run the SOP
programs — Miller lines and accumulation, final exponentiation, hash_to_G2's tail — on the fan engine, an
op's K products on K lanes and one item per block (csrc/lcv_k_fan.hip, lcv_sop_fan.hpp).  Its results must
equal the batch engine's bit for bit and the oracle's: verdicts and reasons on adversarial rows, decoded
signatures, hash_to_G2 points and pairing values."""
import random

import numpy as np
import pytest

import helpers as H
from oracle import bls12_381 as B

pytestmark = pytest.mark.gpu


def _both(v, fn):
    """(fan engine, batch engine) results of fn; restores the mode it found."""
    prev = getattr(v, "latency_mode", 64)
    v.set_latency_mode(64)
    try:
        fan = fn()
        v.set_latency_mode(0)
        batch = fn()
    finally:
        v.set_latency_mode(prev)
    return fan, batch


def test_latency_engine_verdicts(gpu_verifier):
    from lcv import synth
    v = gpu_verifier
    n = 24
    kinds = synth.adversarial_kinds(n, seed=51, bad_fraction=0.5)
    sb = synth.generate(v, n, seed=51, participation="random", kinds=kinds)
    v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    (okw, rw), (okn, rn) = _both(v, lambda: v.validate(sb.updates, sb.current_slot, sb.genesis_validators_root))
    assert np.array_equal(rw, sb.expected_reason) and np.array_equal(rn, rw) and np.array_equal(okw, okn)
    # one update at a time (the reference's per-update call, sync-protocol.md:512), on the fan engine
    prev = getattr(v, "latency_mode", 64)
    v.set_latency_mode(64)
    try:
        for i in (0, int(np.argmax(sb.expected_reason == 14)) if (sb.expected_reason == 14).any() else 1):
            ok1, r1 = v.validate(sb.updates.slice(i, i + 1), sb.current_slot, sb.genesis_validators_root)
            assert int(r1[0]) == int(sb.expected_reason[i])
    finally:
        v.set_latency_mode(prev)


def test_latency_engine_intermediates(gpu_verifier):
    v = gpu_verifier
    rng = random.Random(52)
    # pairing values e(P, Q)^3 after the final exponentiation
    ps = [B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)) for _ in range(3)]
    qs = [B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)) for _ in range(3)]
    p96 = np.frombuffer(b"".join(x.to_bytes(48, "big") + y.to_bytes(48, "big") for x, y in ps), np.uint8)
    q192 = np.frombuffer(b"".join(q[0][0].to_bytes(48, "big") + q[0][1].to_bytes(48, "big") + q[1][0].to_bytes(48, "big")
                                  + q[1][1].to_bytes(48, "big") for q in qs), np.uint8)
    ew, en = _both(v, lambda: v.debug_pairing(p96, q192))
    assert np.array_equal(ew, en)
    for i in range(3):
        e = B.pairing(ps[i], qs[i])
        e3 = B.f12_coeffs(B.f12_mul(B.f12_mul(e, e), e))
        got = [int.from_bytes(ew[i][48 * k:48 * k + 48].tobytes(), "big") for k in range(12)]
        assert got == [c for g in e3 for c in g]
    # hash_to_G2 and signature decoding (incl. an invalid and a non-subgroup encoding)
    msgs = np.frombuffer(bytes(rng.randrange(256) for _ in range(32 * 3)), np.uint8)
    (hw, iw), (hn, inn) = _both(v, lambda: v.debug_hash_to_g2(msgs))
    assert np.array_equal(hw, hn) and np.array_equal(iw, inn)
    for i in range(3):
        h = B.hash_to_g2(msgs[32 * i:32 * i + 32].tobytes())
        got = [int.from_bytes(hw[i][48 * k:48 * k + 48].tobytes(), "big") for k in range(4)]
        assert got == [h[0][0], h[0][1], h[1][0], h[1][1]]
    import g2_edge_points as E
    sigs = [B.sign(0x77, b"\x01" * 32), bytes([0xC0]) + bytes(95), E.edge_signatures()["order_13"],
            bytes([0x80]) + bytes(47) + bytes([0xFF]) * 48]
    (dw, sw), (dn, sn) = _both(v, lambda: v.debug_g2_decompress(np.frombuffer(b"".join(sigs), np.uint8)))
    assert np.array_equal(dw, dn) and np.array_equal(sw, sn) and list(sw) == [0, 1, 2, 2]


def test_latency_engine_fast_aggregate_verify(gpu_verifier):
    v = gpu_verifier
    sks = [3 + k for k in range(40)]
    pks = [B.sk_to_pk(k) for k in sks]
    msg = b"\x42" * 32
    sig = B.aggregate_signatures([B.sign(k, msg) for k in sks])
    (a, b) = _both(v, lambda: (v.fast_aggregate_verify(pks, msg, sig), v.fast_aggregate_verify(pks, b"\x43" * 32, sig)))
    assert a == b == (True, False)


def _knob_verifier(monkeypatch, env):
    """A fresh context (LCV_SOP_ITEMS_* are read at lcv_init) in latency mode 0, so that every SOP launch
    takes the batch engine — the only engine that reads the knob."""
    import os
    from lcv.device import Verifier
    for k, val in env.items():
        monkeypatch.setenv(k, str(val))
    v = H.hostsim_verifier() if os.environ.get("LCV_TEST_HOSTSIM") == "1" else Verifier(0)
    v.set_latency_mode(0)
    v.engine_log(reset=True)
    return v


@pytest.mark.parametrize("items", [1, 5, 6])
def test_h2c_items_per_wave(engine_verifier, items, monkeypatch):
    """hash_to_G2's tail on the batch engine with fewer items per wave (LCV_SOP_ITEMS_H2C, read at lcv_init): a
    ragged batch (37 messages: partial last wave) gives both engines' default launches' points bit for bit,
    and the oracle's; the engine log proves the batch engine ran h2c at `items` per wave."""
    rng = random.Random(60 + items)
    msgs = np.frombuffer(bytes(rng.randrange(256) for _ in range(32 * 37)), np.uint8)
    h_ref, i_ref = engine_verifier.debug_hash_to_g2(msgs)  # default launch of the parametrized engine
    v = _knob_verifier(monkeypatch, {"LCV_SOP_ITEMS_H2C": items})
    h, inf = v.debug_hash_to_g2(msgs)
    log = v.engine_log()
    assert log["fan"] == 0 and log["batch"] > 0 and log["items"]["h2c"] == items, log
    assert np.array_equal(h, h_ref) and np.array_equal(inf, i_ref)
    for i in (0, 36):
        e = B.hash_to_g2(msgs[32 * i:32 * i + 32].tobytes())
        got = [int.from_bytes(h[i][48 * k:48 * k + 48].tobytes(), "big") for k in range(4)]
        assert got == [e[0][0], e[0][1], e[1][0], e[1][1]]
    v.close()


@pytest.mark.parametrize("items", [3, 4])
def test_pairing_items_per_wave(engine_verifier, items, monkeypatch):
    """The pairing's SOP kernels on the batch engine (line walk, Miller accumulation, final exponentiation) with
    fewer items per wave (LCV_SOP_ITEMS_LINES / _ACC / _FEXP): pairing values of a ragged batch (7 items) equal
    both engines' default launches'; the engine log proves each program ran at `items` per wave."""
    rng = random.Random(70 + items)
    ps = [B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)) for _ in range(7)]
    qs = [B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)) for _ in range(7)]
    p96 = np.frombuffer(b"".join(x.to_bytes(48, "big") + y.to_bytes(48, "big") for x, y in ps), np.uint8)
    q192 = np.frombuffer(b"".join(q[0][0].to_bytes(48, "big") + q[0][1].to_bytes(48, "big") + q[1][0].to_bytes(48, "big")
                                  + q[1][1].to_bytes(48, "big") for q in qs), np.uint8)
    ref = engine_verifier.debug_pairing(p96, q192)
    v = _knob_verifier(monkeypatch, {f"LCV_SOP_ITEMS_{name}": items for name in ("LINES", "ACC", "FEXP")})
    assert np.array_equal(v.debug_pairing(p96, q192), ref)
    log = v.engine_log()
    assert log["fan"] == 0 and log["items"] == {"lines": items, "miller_acc": items, "fexp": items, "h2c": 0}, log
    e = B.pairing(ps[6], qs[6])
    e3 = B.f12_coeffs(B.f12_mul(B.f12_mul(e, e), e))
    assert [int.from_bytes(ref[6][48 * k:48 * k + 48].tobytes(), "big") for k in range(12)] == [c for g in e3 for c in g]
    v.close()
