"""Light-client store state machine over GPU-verified batches.

Host restatement of the reference's store logic, driven by the batched HIP verifier:

    get_safety_threshold                    sync-protocol.md:323-327
    is_better_update                        sync-protocol.md:260-311
    apply_light_client_update               sync-protocol.md:470-486
    process_light_client_store_force_update sync-protocol.md:490-503
    process_light_client_update             sync-protocol.md:508-553
    process_light_client_finality_update    sync-protocol.md:559-573
    process_light_client_optimistic_update  sync-protocol.md:578-592
    initialize_light_client_store           sync-protocol.md:351-373 (its three asserts run in the
                                            HIP kernel F_bootstrap)

plus `process_light_client_updates(store, updates, current_slot, gvr)`: the reference's sequential
loop `for u in updates: process_light_client_update(store, u, ...)` (an AssertionError rejects the
update and leaves the store unchanged: validation runs before any mutation), returning the accept
flags.  Validation is speculative and batched: every pending update is validated on the GPU against
the current store snapshot in ONE call; the host then applies the store logic in order, and only
when `apply_light_client_update` changes what validation reads (finalized slot, current / next
sync committee) are the remaining updates re-validated, again as one batch.  The store mutation
itself is scalar and order-dependent, so it stays on the host.

Store / update objects are duck-typed: any objects with the reference's field names (the spec
containers, or the lightweight defaults below for the finality / optimistic conversions).
"""
from __future__ import annotations

from dataclasses import dataclass
from types import SimpleNamespace
from typing import Any, Optional, Sequence

import numpy as np

from . import config
from . import layout as L
from . import runtime
from .device import Verifier
from .sync_protocol import REASONS, validate_light_client_updates

# SLOTS_PER_EPOCH * EPOCHS_PER_SYNC_COMMITTEE_PERIOD and UPDATE_TIMEOUT (sync-protocol.md:89) come from the
# active network configuration (lcv.config.active(); mainnet unless set)


# ------------------------------------------------------------------ predicates (sync-protocol.md:246-341)
def _zero(b: bytes) -> bool:
    return not any(b)


def compute_sync_committee_period_at_slot(slot) -> int:
    return config.active().compute_sync_committee_period_at_slot(slot)


def is_sync_committee_update(update) -> bool:
    return not _zero(L.pack_branch(update.next_sync_committee_branch, 5))


def is_finality_update(update) -> bool:
    return not _zero(L.pack_branch(update.finality_branch, 6))


def is_next_sync_committee_known(store) -> bool:
    return not _zero(L.pack_sync_committee(store.next_sync_committee))


def get_safety_threshold(store) -> int:
    return max(int(store.previous_max_active_participants), int(store.current_max_active_participants)) // 2


def _participants(update) -> int:
    return int(sum(bool(b) for b in update.sync_aggregate.sync_committee_bits))


def _slot(header) -> int:
    return int(header.beacon.slot)


# ------------------------------------------------------------------ store logic
def is_better_update(new_update, old_update) -> bool:
    """sync-protocol.md:260-311."""
    max_active = len(new_update.sync_aggregate.sync_committee_bits)
    new_n, old_n = _participants(new_update), _participants(old_update)
    new_super, old_super = new_n * 3 >= max_active * 2, old_n * 3 >= max_active * 2
    if new_super != old_super:
        return new_super > old_super
    if not new_super and new_n != old_n:
        return new_n > old_n

    def relevant_sc(u):
        return is_sync_committee_update(u) and (compute_sync_committee_period_at_slot(_slot(u.attested_header))
                                                == compute_sync_committee_period_at_slot(u.signature_slot))
    new_rel, old_rel = relevant_sc(new_update), relevant_sc(old_update)
    if new_rel != old_rel:
        return new_rel
    new_fin, old_fin = is_finality_update(new_update), is_finality_update(old_update)
    if new_fin != old_fin:
        return new_fin
    if new_fin:
        def sc_finality(u):
            return (compute_sync_committee_period_at_slot(_slot(u.finalized_header))
                    == compute_sync_committee_period_at_slot(_slot(u.attested_header)))
        new_scf, old_scf = sc_finality(new_update), sc_finality(old_update)
        if new_scf != old_scf:
            return new_scf
    if new_n != old_n:
        return new_n > old_n
    if _slot(new_update.attested_header) != _slot(old_update.attested_header):
        return _slot(new_update.attested_header) < _slot(old_update.attested_header)
    return int(new_update.signature_slot) < int(old_update.signature_slot)


def apply_light_client_update(store, update) -> None:
    """sync-protocol.md:470-486."""
    store_period = compute_sync_committee_period_at_slot(_slot(store.finalized_header))
    update_finalized_period = compute_sync_committee_period_at_slot(_slot(update.finalized_header))
    if not is_next_sync_committee_known(store):
        assert update_finalized_period == store_period
        store.next_sync_committee = update.next_sync_committee
    elif update_finalized_period == store_period + 1:
        store.current_sync_committee = store.next_sync_committee
        store.next_sync_committee = update.next_sync_committee
        store.previous_max_active_participants = store.current_max_active_participants
        store.current_max_active_participants = 0
    if _slot(update.finalized_header) > _slot(store.finalized_header):
        store.finalized_header = update.finalized_header
        if _slot(store.finalized_header) > _slot(store.optimistic_header):
            store.optimistic_header = store.finalized_header


def process_light_client_store_force_update(store, current_slot: int) -> None:
    """sync-protocol.md:490-503 (the best update's finalized header is replaced on a copy, so the
    caller's update object is not mutated)."""
    if int(current_slot) > _slot(store.finalized_header) + config.active().UPDATE_TIMEOUT and store.best_valid_update is not None:
        best = store.best_valid_update
        if _slot(best.finalized_header) <= _slot(store.finalized_header):
            best = SimpleNamespace(**{k: getattr(best, k) for k in _UPDATE_FIELDS})
            best.finalized_header = best.attested_header
        apply_light_client_update(store, best)
        store.best_valid_update = None


def _apply_valid(store, update) -> None:
    """process_light_client_update (sync-protocol.md:508-553) after validation succeeded."""
    n = _participants(update)
    if store.best_valid_update is None or is_better_update(update, store.best_valid_update):
        store.best_valid_update = update
    store.current_max_active_participants = max(int(store.current_max_active_participants), n)
    if n > get_safety_threshold(store) and _slot(update.attested_header) > _slot(store.optimistic_header):
        store.optimistic_header = update.attested_header
    has_finalized_next = (not is_next_sync_committee_known(store) and is_sync_committee_update(update)
                          and is_finality_update(update)
                          and compute_sync_committee_period_at_slot(_slot(update.finalized_header))
                          == compute_sync_committee_period_at_slot(_slot(update.attested_header)))
    if n * 3 >= len(update.sync_aggregate.sync_committee_bits) * 2 and (
            _slot(update.finalized_header) > _slot(store.finalized_header) or has_finalized_next):
        apply_light_client_update(store, update)
        store.best_valid_update = None


def _validation_key(store):
    """What validate_light_client_update reads from the store."""
    return (_slot(store.finalized_header), L.pack_sync_committee(store.current_sync_committee),
            L.pack_sync_committee(store.next_sync_committee))


def process_light_client_updates(store, updates: Sequence, current_slot: int, genesis_validators_root: bytes,
                                 verifier: Optional[Verifier] = None, reasons_out: Optional[list] = None
                                 ) -> np.ndarray:
    """Sequential `process_light_client_update` over `updates` (in order) with batched GPU
    validation; returns accept flags.  `reasons_out` (optional list) receives each update's
    validation reason code (0 = valid, REASONS in lcv.sync_protocol) under the store it met."""
    v = verifier if verifier is not None else runtime.default_verifier()
    if v.config != config.active():
        # the host-side periods / UPDATE_TIMEOUT read config.active(); the device checks read v.config
        raise ValueError(f"process_light_client_updates: the verifier validates under network configuration "
                         f"{v.config.name!r} but lcv.config.active() is {config.active().name!r}; call "
                         f"lcv.config.set_active() (or Verifier.set_config) so both sides agree")
    verifier = v
    n = len(updates)
    accepted = np.zeros(n, bool)
    reasons = np.zeros(n, np.uint8)
    start = 0
    while start < n:
        key = _validation_key(store)
        ok, rs = validate_light_client_updates(store, updates[start:], current_slot, genesis_validators_root, verifier)
        k = start
        while k < n:
            reasons[k] = rs[k - start]
            if ok[k - start]:
                accepted[k] = True
                _apply_valid(store, updates[k])
            k += 1
            if _validation_key(store) != key:
                break  # the store moved: re-validate what is left against the new snapshot
        start = k
    if reasons_out is not None:
        reasons_out.extend(int(r) for r in reasons)
    return accepted


def process_light_client_update(store, update, current_slot: int, genesis_validators_root: bytes,
                                verifier: Optional[Verifier] = None) -> None:
    """sync-protocol.md:508-553: raises AssertionError (store unchanged) on an invalid update."""
    rs: list = []
    if not process_light_client_updates(store, [update], current_slot, genesis_validators_root, verifier, rs)[0]:
        line, what = REASONS.get(rs[0], ("?", "?"))
        raise AssertionError(f"validate_light_client_update: assert {what} failed ({line}, reason {rs[0]})")


# ------------------------------------------------------------------ finality / optimistic updates
_UPDATE_FIELDS = ("attested_header", "next_sync_committee", "next_sync_committee_branch", "finalized_header",
                  "finality_branch", "sync_aggregate", "signature_slot")


def _default_sync_committee():
    return SimpleNamespace(pubkeys=[bytes(L.PUBKEY_BYTES)] * L.SYNC_COMMITTEE_SIZE, aggregate_pubkey=bytes(L.PUBKEY_BYTES))


def _default_header():
    """LightClientHeader() (all-zero beacon header, execution header and branch)."""
    beacon = SimpleNamespace(slot=0, proposer_index=0, parent_root=bytes(32), state_root=bytes(32), body_root=bytes(32))
    execution = SimpleNamespace(logs_bloom=bytes(256), extra_data=b"")
    return SimpleNamespace(beacon=beacon, execution=execution, execution_branch=[bytes(32)] * 4)


def _finality_as_update(fu):
    return SimpleNamespace(attested_header=fu.attested_header, next_sync_committee=_default_sync_committee(),
                           next_sync_committee_branch=[bytes(32)] * 5, finalized_header=fu.finalized_header,
                           finality_branch=fu.finality_branch, sync_aggregate=fu.sync_aggregate,
                           signature_slot=fu.signature_slot)


def _optimistic_as_update(ou):
    return SimpleNamespace(attested_header=ou.attested_header, next_sync_committee=_default_sync_committee(),
                           next_sync_committee_branch=[bytes(32)] * 5, finalized_header=_default_header(),
                           finality_branch=[bytes(32)] * 6, sync_aggregate=ou.sync_aggregate,
                           signature_slot=ou.signature_slot)


def process_light_client_finality_update(store, finality_update, current_slot: int, genesis_validators_root: bytes,
                                         verifier: Optional[Verifier] = None) -> None:
    """sync-protocol.md:559-573."""
    process_light_client_update(store, _finality_as_update(finality_update), current_slot, genesis_validators_root,
                                verifier)


def process_light_client_optimistic_update(store, optimistic_update, current_slot: int,
                                           genesis_validators_root: bytes, verifier: Optional[Verifier] = None) -> None:
    """sync-protocol.md:578-592."""
    process_light_client_update(store, _optimistic_as_update(optimistic_update), current_slot,
                                genesis_validators_root, verifier)


# ------------------------------------------------------------------ bootstrap (sync-protocol.md:164-179, :351-373)
@dataclass
class LightClientStore:
    """sync-protocol.md:164-179 (field names and meaning as the reference's dataclass)."""
    finalized_header: Any
    current_sync_committee: Any
    next_sync_committee: Any
    best_valid_update: Optional[Any]
    optimistic_header: Any
    previous_max_active_participants: int
    current_max_active_participants: int


BOOTSTRAP_REASONS = {
    0: ("", "valid"),
    1: ("sync-protocol.md:353", "is_valid_light_client_header(bootstrap.header)"),
    2: ("sync-protocol.md:354", "hash_tree_root(bootstrap.header.beacon) == trusted_block_root"),
    3: ("sync-protocol.md:356-362", "is_valid_merkle_branch(current_sync_committee_branch)"),
}


def initialize_light_client_store(trusted_block_root: bytes, bootstrap, verifier: Optional[Verifier] = None
                                  ) -> LightClientStore:
    """sync-protocol.md:351-373: the header-validity, trusted-root and committee-branch asserts run on the
    device (lcv_bootstrap_check_batch); raises AssertionError naming the failing assert."""
    v = verifier if verifier is not None else runtime.default_verifier()
    beacon, execution, branch = L.pack_header(bootstrap.header)
    root = bytes(trusted_block_root)
    if len(root) != 32:
        raise ValueError("trusted_block_root must be 32 bytes")
    u8 = lambda b: np.frombuffer(b, np.uint8)  # noqa: E731
    r = int(v.bootstrap_check_batch(u8(beacon), u8(execution), u8(branch),
                                    u8(L.pack_sync_committee(bootstrap.current_sync_committee)),
                                    u8(L.pack_branch(bootstrap.current_sync_committee_branch, 5)), u8(root))[0])
    if r:
        line, what = BOOTSTRAP_REASONS[r]
        raise AssertionError(f"initialize_light_client_store: assert {what} failed ({line}, reason {r})")
    return LightClientStore(finalized_header=bootstrap.header, current_sync_committee=bootstrap.current_sync_committee,
                            next_sync_committee=_default_sync_committee(), best_valid_update=None,
                            optimistic_header=bootstrap.header, previous_max_active_participants=0,
                            current_max_active_participants=0)
