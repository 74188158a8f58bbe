"""The Python drop-ins with the reference's names (lcv.bls.FastAggregateVerify, lcv.merkle.
is_valid_merkle_branch / hash_tree_root_sync_committee, lcv.sync_protocol.validate_light_client_update)
and the batched C entries behind them (lcv_merkle_branch_batch, lcv_htr_sync_committee_batch,
lcv_fast_aggregate_verify_batch), each against the CPU oracle.  Reference call sites:
sync-protocol.md:234, 356, 428, 443 (Merkle), :444 (HTR), :464 (FastAggregateVerify), :386-465.
"""
import hashlib
import random

import numpy as np
import pytest

import golden_cases as G
import helpers as H
from oracle import bls12_381 as B
from oracle import spec as S
from oracle import ssz

pytestmark = pytest.mark.gpu


def _fold(leaf, branch, index):
    v = leaf
    for i, b in enumerate(branch):
        v = hashlib.sha256(b + v if (index >> i) & 1 else v + b).digest()
    return v


def test_is_valid_merkle_branch_dropin(gpu_verifier):
    from lcv.merkle import is_valid_merkle_branch
    rng = random.Random(31)
    for depth, index in ((4, 9), (5, 22), (5, 23), (6, 41), (1, 0), (0, 0)):
        leaf = rng.randbytes(32)
        branch = [rng.randbytes(32) for _ in range(depth)]
        root = _fold(leaf, branch, index)
        assert is_valid_merkle_branch(leaf, branch, depth, index, root, verifier=gpu_verifier)
        assert S.is_valid_merkle_branch(leaf, branch, depth, index, root)
        bad = bytes([root[0] ^ 1]) + root[1:]
        assert not is_valid_merkle_branch(leaf, branch, depth, index, bad, verifier=gpu_verifier)
        if depth:
            assert not is_valid_merkle_branch(leaf, branch, depth, index ^ 1, root, verifier=gpu_verifier)
    with pytest.raises(IndexError):  # the spec indexes branch[i] for i < depth
        is_valid_merkle_branch(bytes(32), [bytes(32)] * 3, 4, 9, bytes(32), verifier=gpu_verifier)


def test_merkle_branch_batch_entry(gpu_verifier):
    """lcv_merkle_branch_batch: n rows, one depth/index per call, ~1/3 corrupted."""
    rng = np.random.default_rng(32)
    for depth, index in ((4, 9), (5, 23), (6, 41)):
        n = 300
        leaves = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        br = rng.integers(0, 256, (n, depth * 32), dtype=np.uint8)
        roots = np.stack([np.frombuffer(_fold(leaves[i].tobytes(), [br[i, 32 * k:32 * k + 32].tobytes()
                                                                   for k in range(depth)], index), np.uint8)
                          for i in range(n)])
        bad = rng.random(n) < 0.33
        br[bad, rng.integers(0, depth * 32)] ^= 0x10
        got = gpu_verifier.merkle_branch_batch(leaves, br, depth, index, roots)
        assert np.array_equal(got, ~bad)


def test_htr_sync_committee_dropin_and_batch(gpu_verifier):
    from lcv.merkle import hash_tree_root_sync_committee
    rng = np.random.default_rng(33)
    comms = [rng.integers(0, 256, 24624, dtype=np.uint8).tobytes() for _ in range(5)] + [bytes(24624)]
    want = [ssz.hash_tree_root(H.committee_from(c)) for c in comms]
    got = gpu_verifier.htr_sync_committee_batch(np.frombuffer(b"".join(comms), np.uint8))
    assert [bytes(r) for r in got] == want
    assert hash_tree_root_sync_committee(comms[2], verifier=gpu_verifier) == want[2]
    assert hash_tree_root_sync_committee(H.committee_from(comms[3]), verifier=gpu_verifier) == want[3]


def test_fast_aggregate_verify_dropin(gpu_verifier):
    from lcv import bls
    rng = random.Random(34)
    sks = [rng.randrange(1, B.R) for _ in range(600)]
    pks = [B.sk_to_pk(k) for k in sks]
    msg = rng.randbytes(32)

    def fav(p, m, s):
        return bls.FastAggregateVerify(p, m, s, verifier=gpu_verifier)

    sig3 = B.sign(sum(sks[:3]) % B.R, msg)
    assert fav(pks[:3], msg, sig3) and B.fast_aggregate_verify(pks[:3], msg, sig3)
    assert not fav(pks[:2], msg, sig3)
    assert not fav(pks[:3], bytes(32), sig3)
    assert not fav([], msg, sig3)                       # empty key list -> False
    assert not fav(pks[:3], msg, sig3[:95])              # malformed signature length -> False
    assert not fav(pks[:2] + [b"\x00" * 48], msg, sig3)  # undecodable key -> False
    # more keys than one 512-key table: the slices' aggregates are summed on the device
    sig600 = B.sign(sum(sks) % B.R, msg)
    assert fav(pks, msg, sig600)
    assert not fav(pks[:599], msg, sig600)
    sig513 = B.sign(sum(sks[:513]) % B.R, msg)
    assert fav(pks[:513], msg, sig513)
    # a message that is not a 32-byte signing root (expand_message_xmd streamed on the device)
    for m in (b"", b"abc", rng.randbytes(31), rng.randbytes(33), rng.randbytes(200)):
        s = B.sign(sum(sks[:2]) % B.R, m)
        assert fav(pks[:2], m, s), len(m)
        assert not fav(pks[:2], m + b"x", s)


def test_fast_aggregate_verify_batch_entry(gpu_verifier):
    b = G.load_bls()
    pks = [b["fav_pks"][k].tobytes() for k in range(3)]
    table = np.frombuffer(b"".join(pks) + bytes(48 * 509), np.uint8)
    m, s = b["fav_msg"].tobytes(), b["fav_sig"].tobytes()
    bits = [bytes([0b111]) + bytes(63), bytes([0b011]) + bytes(63), bytes([0b111]) + bytes(63)]
    msgs = [m, m, bytes(32)]
    got = gpu_verifier.fast_aggregate_verify_batch(table, np.zeros(3, np.uint32),
                                                   np.frombuffer(b"".join(bits), np.uint8),
                                                   np.frombuffer(b"".join(msgs), np.uint8),
                                                   np.frombuffer(s * 3, np.uint8))
    assert list(got) == [True, False, False]


def test_validate_light_client_update_dropin(gpu_verifier):
    """The single-update drop-in returns None for a valid update and raises AssertionError naming
    the reference's failing assert otherwise (the golden cases' expected reasons come from the
    reference's exec'd blocks)."""
    from lcv import sync_protocol as SP
    from lcv.device import PackedUpdates
    g = G.load_updates()
    cur, nxt, zero = (g["nsc_pool"][k].tobytes() for k in range(3))
    gvr = g["genesis_validators_root"].tobytes()
    p = PackedUpdates(nsc_pool=g["nsc_pool"], nsc_index=g["nsc_index"].copy(),
                      signature_slot=g["signature_slot"].copy(), **{k: np.ascontiguousarray(g[k]) for k in G.COLS})
    seen = set()
    for i, want in enumerate(g["expected_reason"]):
        want = int(want)
        if want in seen and want != 0:
            continue
        seen.add(want)
        store = H.store_from(int(g["store_finalized_slot"][i]), cur, nxt if int(g["store_next_known"][i]) else zero)
        upd = H.update_from(p, i)
        cs = int(g["current_slot"][i])
        if want == 0:
            assert SP.validate_light_client_update(store, upd, cs, gvr, verifier=gpu_verifier) is None
        else:
            with pytest.raises(AssertionError, match=f"reason {want}\\)"):
                SP.validate_light_client_update(store, upd, cs, gvr, verifier=gpu_verifier)
    assert len(seen) >= 10
