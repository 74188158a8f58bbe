"""Drop-in `validate_light_client_update` (reference sync-protocol.md:386-465) and its batched form.

    validate_light_client_update(store, update, current_slot, genesis_validators_root) -> None
        raises AssertionError on an invalid update, exactly when the reference's asserts would
        (the message names the failing assert: sync-protocol.md line + reason code).
    validate_light_client_updates(store, updates, current_slot, genesis_validators_root)
        -> (verdict: np.ndarray[bool], reason: np.ndarray[uint8])
        semantics: [validate_light_client_update(store, u, ...) for u in updates] against ONE
        immutable store snapshot; `updates` is a sequence of update objects or a PackedUpdates
        batch (the throughput path: no per-update Python work).

Every check — Merkle branches, SSZ hash_tree_root, committee selection, signing root and
`bls.FastAggregateVerify` — runs in the HIP kernels of liblcv.so; this module only packs bytes.
There is no CPU fallback: without liblcv.so / a GPU, `LcvUnavailable` is raised.
"""
from __future__ import annotations

import hashlib
from typing import Optional, Sequence, Tuple, Union

import numpy as np

from . import layout as L
from . import runtime
from .device import PackedUpdates, Verifier

# reason code -> (reference line, description); reason k = the k-th assert of the function
REASONS = {
    0: ("", "valid"),
    1: ("sync-protocol.md:392", "sum(sync_committee_bits) >= MIN_SYNC_COMMITTEE_PARTICIPANTS"),
    2: ("sync-protocol.md:395", "is_valid_light_client_header(update.attested_header)"),
    3: ("sync-protocol.md:398", "current_slot >= signature_slot > attested slot >= finalized slot"),
    4: ("sync-protocol.md:402", "signature_period in (store_period, store_period + 1)"),
    5: ("sync-protocol.md:404", "signature_period == store_period"),
    6: ("sync-protocol.md:411-414", "update is relevant"),
    7: ("sync-protocol.md:420", "finalized_header == LightClientHeader()"),
    8: ("sync-protocol.md:423", "genesis finalized_header == LightClientHeader()"),
    9: ("sync-protocol.md:426", "is_valid_light_client_header(update.finalized_header)"),
    10: ("sync-protocol.md:428-434", "is_valid_merkle_branch(finality_branch)"),
    11: ("sync-protocol.md:439", "next_sync_committee == SyncCommittee()"),
    12: ("sync-protocol.md:442", "next_sync_committee == store.next_sync_committee"),
    13: ("sync-protocol.md:443-449", "is_valid_merkle_branch(next_sync_committee_branch)"),
    14: ("sync-protocol.md:464", "bls.FastAggregateVerify(participant_pubkeys, signing_root, signature)"),
}


def pack_updates(updates: Sequence) -> PackedUpdates:
    """Spec `LightClientUpdate` objects -> packed batch; identical next_sync_committee values are
    stored once in the pool (HTR(SyncCommittee) is then computed once per distinct value)."""
    n = len(updates)
    cols = {k: np.zeros((n, w), np.uint8) for k, w in (
        ("att_beacon", L.BEACON_BYTES), ("att_exec", L.EXEC_BYTES), ("att_branch", L.EXEC_BRANCH_BYTES),
        ("fin_beacon", L.BEACON_BYTES), ("fin_exec", L.EXEC_BYTES), ("fin_branch", L.EXEC_BRANCH_BYTES),
        ("nsc_branch", L.NSC_BRANCH_BYTES), ("finality_branch", L.FINALITY_BRANCH_BYTES),
        ("sync_bits", L.BITS_BYTES), ("sync_signature", L.SIGNATURE_BYTES))}
    sig_slot = np.zeros(n, np.uint64)
    pool, pool_ix = [], {}
    nsc_index = np.zeros(n, np.uint32)

    def put(name, i, b):
        cols[name][i] = np.frombuffer(b, np.uint8)

    for i, u in enumerate(updates):
        for pre, h in (("att", u.attested_header), ("fin", u.finalized_header)):
            b, e, br = L.pack_header(h)
            put(pre + "_beacon", i, b)
            put(pre + "_exec", i, e)
            put(pre + "_branch", i, br)
        sc = L.pack_sync_committee(u.next_sync_committee)
        key = hashlib.sha256(sc).digest()
        if key not in pool_ix:
            pool_ix[key] = len(pool)
            pool.append(sc)
        nsc_index[i] = pool_ix[key]
        put("nsc_branch", i, L.pack_branch(u.next_sync_committee_branch, 5))
        put("finality_branch", i, L.pack_branch(u.finality_branch, 6))
        put("sync_bits", i, L.pack_bits(u.sync_aggregate.sync_committee_bits))
        sig = bytes(u.sync_aggregate.sync_committee_signature)
        if len(sig) != L.SIGNATURE_BYTES:
            raise ValueError("sync_committee_signature must be 96 bytes")
        put("sync_signature", i, sig)
        sig_slot[i] = int(u.signature_slot)
    if not pool:
        pool.append(bytes(L.SYNC_COMMITTEE_BYTES))
    nsc_pool = np.frombuffer(b"".join(pool), np.uint8).reshape(len(pool), L.SYNC_COMMITTEE_BYTES).copy()
    return PackedUpdates(nsc_pool=nsc_pool, nsc_index=nsc_index, signature_slot=sig_slot, **cols)


def _store_args(store) -> Tuple[int, bytes, bytes]:
    return (int(store.finalized_header.beacon.slot), L.pack_sync_committee(store.current_sync_committee),
            L.pack_sync_committee(store.next_sync_committee))


def validate_light_client_updates(store, updates: Union[Sequence, PackedUpdates], current_slot: int,
                                  genesis_validators_root: bytes, verifier: Optional[Verifier] = None
                                  ) -> Tuple[np.ndarray, np.ndarray]:
    """Batched validate_light_client_update against one store snapshot -> (verdicts, reason codes)."""
    v = verifier if verifier is not None else runtime.default_verifier()
    batch = updates if isinstance(updates, PackedUpdates) else pack_updates(updates)
    if batch.n == 0:
        return np.zeros(0, bool), np.zeros(0, np.uint8)
    runtime.ensure_store(v, *_store_args(store))
    return v.validate(batch, int(current_slot), bytes(genesis_validators_root))


def validate_light_client_update(store, update, current_slot: int, genesis_validators_root: bytes,
                                 verifier: Optional[Verifier] = None) -> None:
    """Reference sync-protocol.md:386-465: returns None, raises AssertionError if invalid."""
    ok, reason = validate_light_client_updates(store, [update], current_slot, genesis_validators_root, verifier)
    if not ok[0]:
        line, what = REASONS.get(int(reason[0]), ("?", "?"))
        raise AssertionError(f"validate_light_client_update: assert {what} failed ({line}, reason {int(reason[0])})")
