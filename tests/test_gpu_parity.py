"""GPU parity: liblcv.so on the MI355X vs the CPU oracle (oracle/), bit-exact, through the C ABI."""
import numpy as np
import pytest

import helpers as H
from oracle import bls12_381 as B

pytestmark = pytest.mark.gpu

KAT_SK = 0x263DBD792F5B1BE47ED85F8938C0F29586AF0D3AC7B977F21C278FE1462040E3


def _ints(row, k):
    b = row.tobytes()
    return [int.from_bytes(b[48 * i:48 * i + 48], "big") for i in range(k)]


def test_fp_ops(gpu_verifier):
    rng = np.random.default_rng(1)
    n = 256
    A = [int.from_bytes(rng.bytes(48), "big") % B.P for _ in range(n)]
    Bv = [int.from_bytes(rng.bytes(48), "big") % B.P for _ in range(n)]
    A[0], Bv[0] = 0, 0
    A[1], Bv[1] = B.P - 1, B.P - 1
    a = np.frombuffer(b"".join(x.to_bytes(48, "big") for x in A), np.uint8)
    b = np.frombuffer(b"".join(x.to_bytes(48, "big") for x in Bv), np.uint8)
    out, ok = gpu_verifier.debug_fp(a, b)
    for i in range(n):
        g = _ints(out[i], 6)
        assert g[:4] == [A[i] * Bv[i] % B.P, (A[i] + Bv[i]) % B.P, (A[i] - Bv[i]) % B.P, pow(A[i], B.P - 2, B.P)]
        s = B.f2_sqrt((A[i], Bv[i]))
        assert bool(ok[i]) == (s is not None)
        if s is not None:
            assert B.f2_sqr((g[4], g[5])) == (A[i], Bv[i])


def test_hash_to_g2(gpu_verifier):
    rng = np.random.default_rng(2)
    msgs = [bytes(32), b"\xff" * 32] + [rng.bytes(32) for _ in range(6)]
    out, inf = gpu_verifier.debug_hash_to_g2(np.frombuffer(b"".join(msgs), np.uint8))
    for i, m in enumerate(msgs):
        g = _ints(out[i], 4)
        assert ((g[0], g[1]), (g[2], g[3])) == B.hash_to_g2(m)
        assert inf[i] == 0


def test_sign_kat(gpu_verifier):
    """eth2 BLS sign KAT (recalled: sk 0x263d..40e3, message 0x00*32)."""
    sk = np.frombuffer(KAT_SK.to_bytes(32, "big"), np.uint8)
    pk = gpu_verifier.sk_to_pk_batch(sk).tobytes()
    sig = gpu_verifier.sign_batch(sk, np.zeros(32, np.uint8)).tobytes()
    assert pk.hex() == ("a491d1b0ecd9bb917989f0e74f0dea0422eac4a873e5e2644f368dffb9a6e20f"
                        "d6e10c1b77654d067c0618f6e5a7f79a")
    assert sig.hex().startswith("b6ed936746e01f8ecf281f020953fbf1f01debd5657c4a383940b020b26507f6")
    assert sig == B.sign(KAT_SK, bytes(32))
    assert gpu_verifier.fast_aggregate_verify([pk], bytes(32), sig)
    assert not gpu_verifier.fast_aggregate_verify([pk], b"\x01" * 32, sig)


def test_pairing_value(engine_verifier):
    rng = np.random.default_rng(3)
    ps, qs, exp = [], [], []
    for _ in range(2):
        a, b = int(rng.integers(1, 2 ** 62)), int(rng.integers(1, 2 ** 62))
        P, Q = B.g1_mul(B.G1_GEN, a), B.g2_mul(B.G2_GEN, b)
        ps.append(P[0].to_bytes(48, "big") + P[1].to_bytes(48, "big"))
        qs.append(b"".join(c.to_bytes(48, "big") for c in (Q[0][0], Q[0][1], Q[1][0], Q[1][1])))
        e = B.pairing(P, Q)
        exp.append(B.f12_mul(B.f12_mul(e, e), e))  # device returns e^3
    out = engine_verifier.debug_pairing(np.frombuffer(b"".join(ps), np.uint8), np.frombuffer(b"".join(qs), np.uint8))
    for i in range(2):
        g = _ints(out[i], 12)
        coeffs = [(g[2 * k], g[2 * k + 1]) for k in range(6)]
        assert B.f12_from_coeffs(coeffs) == exp[i]


def test_validate_adversarial_vs_oracle(engine_verifier):
    from lcv import synth
    kinds = np.array([0, 1, 2, 3, 4, 5, 6, 7, 0, 1, 2, 0])
    sb = synth.generate(engine_verifier, len(kinds), seed=7, participation="random", kinds=kinds)
    engine_verifier.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    ok, reason = engine_verifier.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    store = H.store_from(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    exp = [H.O.validate_light_client_update(store, H.update_from(sb.updates, i), sb.current_slot,
                                            sb.genesis_validators_root) for i in range(len(kinds))]
    assert list(reason) == exp
    assert list(reason) == list(sb.expected_reason)
    assert list(ok) == [e == 0 for e in exp]


def test_validate_large_batch_properties(gpu_verifier):
    """Full-size property check (no per-row oracle): 4096 adversarial rows, verdict == construction."""
    from lcv import synth
    n = 4096
    kinds = synth.adversarial_kinds(n, seed=5, bad_fraction=0.10)
    sb = synth.generate(gpu_verifier, n, seed=5, participation="random", kinds=kinds)
    gpu_verifier.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    ok, reason = gpu_verifier.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    assert np.array_equal(reason, sb.expected_reason)
    # idempotence + resident path gives the same verdicts
    rb = gpu_verifier.upload(sb.updates)
    v2, r2 = gpu_verifier.validate_resident(rb, sb.current_slot, sb.genesis_validators_root)
    assert np.array_equal(r2, reason) and np.array_equal(v2.astype(bool), ok)
    # every execution shape (serial stages; slices over 2..4 streams, ragged last slice) agrees
    try:
        for shape in [(1, 1), (2, 3), (4, 7), (4, 32)]:
            gpu_verifier.set_pipeline(*shape)
            v3, r3 = gpu_verifier.validate_resident(rb, sb.current_slot, sb.genesis_validators_root)
            assert np.array_equal(r3, reason), shape
    finally:
        gpu_verifier.set_pipeline(1, 1)


def test_store_sequence_on_gpu(engine_verifier):
    """lcv.store over liblcv.so reproduces the reference's exec'd process_light_client_update
    sequence (tests/golden/store_sequence.npz) step by step and in the batched form."""
    import store_cases
    store_cases.run(engine_verifier)


def test_validate_non_subgroup_signature(engine_verifier):
    """Signatures that decode to curve points outside G2 (or to the identity) fail at :464 on the
    validate path, where the G2 subgroup check is fused into the signature pairing's line walk."""
    from lcv import synth
    sb = synth.generate(engine_verifier, 6, seed=9)
    sigs = sb.updates.sync_signature
    x, bad = 1, []
    while len(bad) < 3:
        x += 1
        X = (x, 11)
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(X), X), B.B2))
        if y is not None and not B.g2_in_subgroup((X, y)):
            bad.append(B.g2_compress((X, y)))
    for row, s in zip((1, 3, 4), bad):
        sigs[row] = np.frombuffer(s, np.uint8)
    sigs[5] = np.frombuffer(bytes([0xC0]) + bytes(95), np.uint8)  # identity signature
    engine_verifier.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    ok, reason = engine_verifier.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    store = H.store_from(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    exp = [H.O.validate_light_client_update(store, H.update_from(sb.updates, i), sb.current_slot,
                                            sb.genesis_validators_root) for i in range(6)]
    assert exp == [0, 14, 0, 14, 14, 14]
    assert list(reason) == exp
