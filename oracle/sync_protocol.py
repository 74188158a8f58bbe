"""CPU restatement of the light-client update validation path — TEST INFRASTRUCTURE ONLY.

Restates reference `sync-protocol.md` (Inspector-Butters/light-client-consensus-specs @ 2025-04-04):
  * containers `LightClientHeader` (:96-101), `LightClientUpdate` (:120-133),
    `LightClientStore` (:165-179);
  * helpers `get_lc_execution_root` (:186-214), `is_valid_light_client_header` (:220-240),
    `is_sync_committee_update` (:246-247), `is_finality_update` (:253-254),
    `is_next_sync_committee_known` (:316-317), `get_subtree_index` (:333-334),
    `compute_sync_committee_period_at_slot` (:340-341);
  * `validate_light_client_update` (:386-465), returning a *reason code* instead of raising:
    reason k = the k-th `assert` of that function in source order (1..14), 0 = valid.
    The numbering is derived mechanically from the reference text by
    tests/golden/make_golden.py, which also exec's the reference's own blocks and checks that
    both agree on every golden case.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

from . import spec as S
from .ssz import Bytes32, Container, hash_tree_root

REASONS = {
    0: "valid",
    1: "participants",                 # :392
    2: "attested header invalid",      # :395
    3: "slot ordering",                # :398
    4: "signature period (next known)",    # :402
    5: "signature period (next unknown)",  # :404
    6: "update not relevant",          # :411-414
    7: "finalized header not empty",   # :420
    8: "finalized genesis header not empty",  # :423
    9: "finalized header invalid",     # :426
    10: "finality branch",             # :428-434
    11: "next sync committee not empty",  # :439
    12: "next sync committee != store",   # :442
    13: "next sync committee branch",  # :443-449
    14: "sync committee signature",    # :464
}


class LightClientHeader(Container):
    beacon: S.BeaconBlockHeader
    execution: S.ExecutionPayloadHeader
    execution_branch: S.ExecutionBranch


class LightClientUpdate(Container):
    attested_header: LightClientHeader
    next_sync_committee: S.SyncCommittee
    next_sync_committee_branch: S.NextSyncCommitteeBranch
    finalized_header: LightClientHeader
    finality_branch: S.FinalityBranch
    sync_aggregate: S.SyncAggregate
    signature_slot: S.Slot


class LightClientFinalityUpdate(Container):
    attested_header: LightClientHeader
    finalized_header: LightClientHeader
    finality_branch: S.FinalityBranch
    sync_aggregate: S.SyncAggregate
    signature_slot: S.Slot


class LightClientOptimisticUpdate(Container):
    attested_header: LightClientHeader
    sync_aggregate: S.SyncAggregate
    signature_slot: S.Slot


@dataclass
class LightClientStore:
    finalized_header: LightClientHeader
    current_sync_committee: S.SyncCommittee
    next_sync_committee: S.SyncCommittee
    best_valid_update: Optional[LightClientUpdate]
    optimistic_header: LightClientHeader
    previous_max_active_participants: int
    current_max_active_participants: int


def get_lc_execution_root(header: LightClientHeader) -> bytes:
    epoch = S.compute_epoch_at_slot(header.beacon.slot)
    if epoch >= S.DENEB_FORK_EPOCH:
        return hash_tree_root(header.execution)
    if epoch >= S.CAPELLA_FORK_EPOCH:
        e = header.execution
        capella_hdr = S.CapellaExecutionPayloadHeader(**{n: getattr(e, n) for n, _ in S.CapellaExecutionPayloadHeader._fields})
        return hash_tree_root(capella_hdr)
    return Bytes32()


def is_valid_light_client_header(header: LightClientHeader) -> bool:
    epoch = S.compute_epoch_at_slot(header.beacon.slot)
    if epoch < S.DENEB_FORK_EPOCH:
        if header.execution.blob_gas_used != 0 or header.execution.excess_blob_gas != 0:
            return False
    if epoch < S.CAPELLA_FORK_EPOCH:
        return header.execution == S.ExecutionPayloadHeader() and header.execution_branch == S.ExecutionBranch()
    return S.is_valid_merkle_branch(
        leaf=get_lc_execution_root(header),
        branch=header.execution_branch,
        depth=S.floorlog2(S.EXECUTION_PAYLOAD_GINDEX),
        index=get_subtree_index(S.EXECUTION_PAYLOAD_GINDEX),
        root=header.beacon.body_root,
    )


def is_sync_committee_update(update: LightClientUpdate) -> bool:
    return update.next_sync_committee_branch != S.NextSyncCommitteeBranch()


def is_finality_update(update: LightClientUpdate) -> bool:
    return update.finality_branch != S.FinalityBranch()


def is_next_sync_committee_known(store: LightClientStore) -> bool:
    return store.next_sync_committee != S.SyncCommittee()


def get_subtree_index(gindex: int) -> int:
    return gindex % 2 ** S.floorlog2(gindex)


def compute_sync_committee_period_at_slot(slot) -> int:
    return S.compute_sync_committee_period(S.compute_epoch_at_slot(slot))


def validate_light_client_update(store: LightClientStore, update: LightClientUpdate,
                                 current_slot: int, genesis_validators_root: bytes) -> int:
    """Reason code of the first failing check (0 = valid), reference `sync-protocol.md:386-465`."""
    agg = update.sync_aggregate
    if not sum(agg.sync_committee_bits) >= S.MIN_SYNC_COMMITTEE_PARTICIPANTS:
        return 1
    if not is_valid_light_client_header(update.attested_header):
        return 2
    att_slot = update.attested_header.beacon.slot
    fin_slot = update.finalized_header.beacon.slot
    if not (current_slot >= update.signature_slot > att_slot >= fin_slot):
        return 3
    store_period = compute_sync_committee_period_at_slot(store.finalized_header.beacon.slot)
    sig_period = compute_sync_committee_period_at_slot(update.signature_slot)
    next_known = is_next_sync_committee_known(store)
    if next_known:
        if sig_period not in (store_period, store_period + 1):
            return 4
    else:
        if sig_period != store_period:
            return 5
    att_period = compute_sync_committee_period_at_slot(att_slot)
    has_next = (not next_known) and (is_sync_committee_update(update) and att_period == store_period)
    if not (att_slot > store.finalized_header.beacon.slot or has_next):
        return 6
    if not is_finality_update(update):
        if update.finalized_header != LightClientHeader():
            return 7
    else:
        if fin_slot == S.GENESIS_SLOT:
            if update.finalized_header != LightClientHeader():
                return 8
            finalized_root = Bytes32()
        else:
            if not is_valid_light_client_header(update.finalized_header):
                return 9
            finalized_root = hash_tree_root(update.finalized_header.beacon)
        if not S.is_valid_merkle_branch(
                leaf=finalized_root, branch=update.finality_branch,
                depth=S.floorlog2(S.FINALIZED_ROOT_GINDEX), index=get_subtree_index(S.FINALIZED_ROOT_GINDEX),
                root=update.attested_header.beacon.state_root):
            return 10
    if not is_sync_committee_update(update):
        if update.next_sync_committee != S.SyncCommittee():
            return 11
    else:
        if att_period == store_period and next_known:
            if update.next_sync_committee != store.next_sync_committee:
                return 12
        if not S.is_valid_merkle_branch(
                leaf=hash_tree_root(update.next_sync_committee), branch=update.next_sync_committee_branch,
                depth=S.floorlog2(S.NEXT_SYNC_COMMITTEE_GINDEX), index=get_subtree_index(S.NEXT_SYNC_COMMITTEE_GINDEX),
                root=update.attested_header.beacon.state_root):
            return 13
    if sig_period == store_period:
        committee = store.current_sync_committee
    else:
        committee = store.next_sync_committee
    pks = [pk for bit, pk in zip(agg.sync_committee_bits, committee.pubkeys) if bit]
    fork_version_slot = max(int(update.signature_slot), 1) - 1
    fork_version = S.compute_fork_version(S.compute_epoch_at_slot(fork_version_slot))
    domain = S.compute_domain(S.DOMAIN_SYNC_COMMITTEE, fork_version, genesis_validators_root)
    signing_root = S.compute_signing_root(update.attested_header.beacon, domain)
    if not S.bls.FastAggregateVerify(pks, signing_root, agg.sync_committee_signature):
        return 14
    return 0


def signing_root_of(update: LightClientUpdate, genesis_validators_root: bytes) -> bytes:
    fork_version_slot = max(int(update.signature_slot), 1) - 1
    fork_version = S.compute_fork_version(S.compute_epoch_at_slot(fork_version_slot))
    domain = S.compute_domain(S.DOMAIN_SYNC_COMMITTEE, fork_version, genesis_validators_root)
    return S.compute_signing_root(update.attested_header.beacon, domain)
