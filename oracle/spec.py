"""Upstream consensus-specs names the reference's light-client blocks depend on — TEST INFRA ONLY.

`sync-protocol.md` uses 36 free names that are defined upstream.  This module
restates them (mainnet preset/config) so that (a) the oracle restatement in
`oracle/sync_protocol.py` can run and (b) the reference's own python blocks can be exec'd
against them to pin the restatement (tests/golden/make_golden.py).

Sources restated (upstream ethereum/consensus-specs, not in /root/reference):
  phase0 beacon-chain: compute_epoch_at_slot, compute_domain, compute_fork_data_root,
    compute_signing_root, is_valid_merkle_branch, ForkData, SigningData, BeaconBlockHeader;
  altair: SyncCommittee, SyncAggregate, compute_sync_committee_period, DOMAIN_SYNC_COMMITTEE;
  deneb/capella: ExecutionPayloadHeader, compute_fork_version (deneb form);
  ssz: floorlog2, GeneralizedIndex, uint64 aliases.
"""
from __future__ import annotations

from dataclasses import dataclass
from types import SimpleNamespace
from typing import Optional, Sequence

from . import bls12_381 as _bls
from .ssz import (Bitvector, ByteList, ByteVector, Bytes4, Bytes20, Bytes32, Bytes48, Bytes96, Container, SSZList,
                  Vector, boolean, compute_merkle_proof, hash_tree_root, sha256, uint8, uint64, uint256)

# ----------------------------------------------------------------------------- mainnet preset/config
SLOTS_PER_EPOCH = 32
EPOCHS_PER_SYNC_COMMITTEE_PERIOD = 256
SYNC_COMMITTEE_SIZE = 512
MAX_EXTRA_DATA_BYTES = 32
BYTES_PER_LOGS_BLOOM = 256
GENESIS_SLOT = 0
GENESIS_FORK_VERSION = bytes.fromhex("00000000")
ALTAIR_FORK_VERSION = bytes.fromhex("01000000")
BELLATRIX_FORK_VERSION = bytes.fromhex("02000000")
CAPELLA_FORK_VERSION = bytes.fromhex("03000000")
DENEB_FORK_VERSION = bytes.fromhex("04000000")
ALTAIR_FORK_EPOCH = 74240
BELLATRIX_FORK_EPOCH = 144896
CAPELLA_FORK_EPOCH = 194048
DENEB_FORK_EPOCH = 269568
DOMAIN_SYNC_COMMITTEE = bytes.fromhex("07000000")
MIN_SYNC_COMMITTEE_PARTICIPANTS = 1
UPDATE_TIMEOUT = SLOTS_PER_EPOCH * EPOCHS_PER_SYNC_COMMITTEE_PERIOD

_CONFIG_NAMES = ("SLOTS_PER_EPOCH", "EPOCHS_PER_SYNC_COMMITTEE_PERIOD", "GENESIS_FORK_VERSION", "ALTAIR_FORK_VERSION",
                 "BELLATRIX_FORK_VERSION", "CAPELLA_FORK_VERSION", "DENEB_FORK_VERSION", "ALTAIR_FORK_EPOCH",
                 "BELLATRIX_FORK_EPOCH", "CAPELLA_FORK_EPOCH", "DENEB_FORK_EPOCH", "DOMAIN_SYNC_COMMITTEE")


class use_config:
    """Context manager: run the oracle (and reference blocks exec'd over reference_namespace(), which
    reads these globals when it is built) under another network configuration: keyword values for the
    names in _CONFIG_NAMES; UPDATE_TIMEOUT follows."""

    def __init__(self, **values):
        bad = set(values) - set(_CONFIG_NAMES)
        assert not bad, bad
        self.values = values

    def __enter__(self):
        g = globals()
        self.saved = {k: g[k] for k in _CONFIG_NAMES + ("UPDATE_TIMEOUT",)}
        g.update(self.values)
        g["UPDATE_TIMEOUT"] = g["SLOTS_PER_EPOCH"] * g["EPOCHS_PER_SYNC_COMMITTEE_PERIOD"]
        return self

    def __exit__(self, *exc):
        globals().update(self.saved)
        return False


# generalized indices (reference sync-protocol.md:78-81, pre-Electra values)
FINALIZED_ROOT_GINDEX = 105
CURRENT_SYNC_COMMITTEE_GINDEX = 54
NEXT_SYNC_COMMITTEE_GINDEX = 55
EXECUTION_PAYLOAD_GINDEX = 25

Slot = uint64
Epoch = uint64
ValidatorIndex = uint64
Gwei = uint64
GeneralizedIndex = int
Root = Bytes32
Hash32 = Bytes32
Version = Bytes4
DomainType = Bytes4
Domain = Bytes32
BLSPubkey = Bytes48
BLSSignature = Bytes96
ExecutionAddress = Bytes20


def floorlog2(x: int) -> int:
    if x < 1:
        raise ValueError("floorlog2 of < 1")
    return int(x).bit_length() - 1


# custom types from the reference's table (sync-protocol.md:67-72)
FinalityBranch = Vector[Bytes32, floorlog2(FINALIZED_ROOT_GINDEX)]
CurrentSyncCommitteeBranch = Vector[Bytes32, floorlog2(CURRENT_SYNC_COMMITTEE_GINDEX)]
NextSyncCommitteeBranch = Vector[Bytes32, floorlog2(NEXT_SYNC_COMMITTEE_GINDEX)]
ExecutionBranch = Vector[Bytes32, floorlog2(EXECUTION_PAYLOAD_GINDEX)]


class BeaconBlockHeader(Container):
    slot: Slot
    proposer_index: ValidatorIndex
    parent_root: Root
    state_root: Root
    body_root: Root


class SyncCommittee(Container):
    pubkeys: Vector[BLSPubkey, SYNC_COMMITTEE_SIZE]
    aggregate_pubkey: BLSPubkey


class SyncAggregate(Container):
    sync_committee_bits: Bitvector[SYNC_COMMITTEE_SIZE]
    sync_committee_signature: BLSSignature


LogsBloom = ByteVector[BYTES_PER_LOGS_BLOOM]
ExtraData = ByteList[MAX_EXTRA_DATA_BYTES]


class ExecutionPayloadHeader(Container):  # deneb (17 fields)
    parent_hash: Hash32
    fee_recipient: ExecutionAddress
    state_root: Bytes32
    receipts_root: Bytes32
    logs_bloom: LogsBloom
    prev_randao: Bytes32
    block_number: uint64
    gas_limit: uint64
    gas_used: uint64
    timestamp: uint64
    extra_data: ExtraData
    base_fee_per_gas: uint256
    block_hash: Hash32
    transactions_root: Root
    withdrawals_root: Root
    blob_gas_used: uint64
    excess_blob_gas: uint64


class CapellaExecutionPayloadHeader(Container):  # capella (15 fields)
    parent_hash: Hash32
    fee_recipient: ExecutionAddress
    state_root: Bytes32
    receipts_root: Bytes32
    logs_bloom: LogsBloom
    prev_randao: Bytes32
    block_number: uint64
    gas_limit: uint64
    gas_used: uint64
    timestamp: uint64
    extra_data: ExtraData
    base_fee_per_gas: uint256
    block_hash: Hash32
    transactions_root: Root
    withdrawals_root: Root


capella = SimpleNamespace(ExecutionPayloadHeader=CapellaExecutionPayloadHeader)


# ----------------------------------------------------------------------------- Deneb beacon chain (producer side)
# The containers full-node.md's producer functions read (BeaconState, SignedBeaconBlock, ...), restated
# from upstream deneb/beacon-chain.md with the mainnet preset limits.  Operation lists the fixtures keep
# empty use an opaque composite element (an empty list's root depends only on its limit).
class Fork(Container):
    previous_version: Version
    current_version: Version
    epoch: Epoch


class Checkpoint(Container):
    epoch: Epoch
    root: Root


class Eth1Data(Container):
    deposit_root: Root
    deposit_count: uint64
    block_hash: Hash32


class Validator(Container):
    pubkey: BLSPubkey
    withdrawal_credentials: Bytes32
    effective_balance: Gwei
    slashed: boolean
    activation_eligibility_epoch: Epoch
    activation_epoch: Epoch
    exit_epoch: Epoch
    withdrawable_epoch: Epoch


class HistoricalSummary(Container):
    block_summary_root: Root
    state_summary_root: Root


class Withdrawal(Container):
    index: uint64
    validator_index: ValidatorIndex
    address: ExecutionAddress
    amount: Gwei


class _Opaque(Container):
    root: Root


Transaction = ByteList[2 ** 30]


class ExecutionPayload(Container):  # deneb
    parent_hash: Hash32
    fee_recipient: ExecutionAddress
    state_root: Bytes32
    receipts_root: Bytes32
    logs_bloom: LogsBloom
    prev_randao: Bytes32
    block_number: uint64
    gas_limit: uint64
    gas_used: uint64
    timestamp: uint64
    extra_data: ExtraData
    base_fee_per_gas: uint256
    block_hash: Hash32
    transactions: SSZList[Transaction, 2 ** 20]
    withdrawals: SSZList[Withdrawal, 16]
    blob_gas_used: uint64
    excess_blob_gas: uint64


class BeaconBlockBody(Container):  # deneb (12 fields -> 16 leaves; execution_payload = gindex 25)
    randao_reveal: BLSSignature
    eth1_data: Eth1Data
    graffiti: Bytes32
    proposer_slashings: SSZList[_Opaque, 16]
    attester_slashings: SSZList[_Opaque, 2]
    attestations: SSZList[_Opaque, 128]
    deposits: SSZList[_Opaque, 16]
    voluntary_exits: SSZList[_Opaque, 16]
    sync_aggregate: SyncAggregate
    execution_payload: ExecutionPayload
    bls_to_execution_changes: SSZList[_Opaque, 16]
    blob_kzg_commitments: SSZList[Bytes48, 4096]


class BeaconBlock(Container):
    slot: Slot
    proposer_index: ValidatorIndex
    parent_root: Root
    state_root: Root
    body: BeaconBlockBody


class SignedBeaconBlock(Container):
    message: BeaconBlock
    signature: BLSSignature


class BeaconState(Container):  # deneb (28 fields -> 32 leaves)
    genesis_time: uint64
    genesis_validators_root: Root
    slot: Slot
    fork: Fork
    latest_block_header: BeaconBlockHeader
    block_roots: Vector[Root, 8192]
    state_roots: Vector[Root, 8192]
    historical_roots: SSZList[Root, 2 ** 24]
    eth1_data: Eth1Data
    eth1_data_votes: SSZList[Eth1Data, 2048]
    eth1_deposit_index: uint64
    validators: SSZList[Validator, 2 ** 40]
    balances: SSZList[Gwei, 2 ** 40]
    randao_mixes: Vector[Bytes32, 65536]
    slashings: Vector[Gwei, 8192]
    previous_epoch_participation: SSZList[uint8, 2 ** 40]
    current_epoch_participation: SSZList[uint8, 2 ** 40]
    justification_bits: Bitvector[4]
    previous_justified_checkpoint: Checkpoint
    current_justified_checkpoint: Checkpoint
    finalized_checkpoint: Checkpoint
    inactivity_scores: SSZList[uint64, 2 ** 40]
    current_sync_committee: SyncCommittee
    next_sync_committee: SyncCommittee
    latest_execution_payload_header: ExecutionPayloadHeader
    next_withdrawal_index: uint64
    next_withdrawal_validator_index: ValidatorIndex
    historical_summaries: SSZList[HistoricalSummary, 2 ** 24]


class ForkData(Container):
    current_version: Version
    genesis_validators_root: Root


class SigningData(Container):
    object_root: Root
    domain: Domain


def compute_epoch_at_slot(slot) -> int:
    return uint64(int(slot) // SLOTS_PER_EPOCH)


def compute_sync_committee_period(epoch) -> int:
    return uint64(int(epoch) // EPOCHS_PER_SYNC_COMMITTEE_PERIOD)


def compute_fork_version(epoch) -> bytes:
    epoch = int(epoch)
    if epoch >= DENEB_FORK_EPOCH:
        return Version(DENEB_FORK_VERSION)
    if epoch >= CAPELLA_FORK_EPOCH:
        return Version(CAPELLA_FORK_VERSION)
    if epoch >= BELLATRIX_FORK_EPOCH:
        return Version(BELLATRIX_FORK_VERSION)
    if epoch >= ALTAIR_FORK_EPOCH:
        return Version(ALTAIR_FORK_VERSION)
    return Version(GENESIS_FORK_VERSION)


def compute_fork_data_root(current_version, genesis_validators_root) -> bytes:
    return hash_tree_root(ForkData(current_version=current_version,
                                   genesis_validators_root=genesis_validators_root))


def compute_domain(domain_type, fork_version=None, genesis_validators_root=None) -> bytes:
    if fork_version is None:
        fork_version = GENESIS_FORK_VERSION
    if genesis_validators_root is None:
        genesis_validators_root = bytes(32)
    fdr = compute_fork_data_root(fork_version, genesis_validators_root)
    return Domain(bytes(domain_type) + bytes(fdr)[:28])


def compute_signing_root(ssz_object, domain) -> bytes:
    return hash_tree_root(SigningData(object_root=hash_tree_root(ssz_object), domain=domain))


def is_valid_merkle_branch(leaf, branch: Sequence[bytes], depth: int, index: int, root) -> bool:
    """phase0 beacon-chain `is_valid_merkle_branch`."""
    value = bytes(leaf)
    for i in range(int(depth)):
        if int(index) // (2 ** i) % 2:
            value = sha256(bytes(branch[i]) + value)
        else:
            value = sha256(value + bytes(branch[i]))
    return value == bytes(root)


class _BlsNamespace:
    """`eth2spec.utils.bls` wrapper semantics: any exception -> False."""

    bls_active = True

    @staticmethod
    def FastAggregateVerify(pubkeys, message, signature) -> bool:
        try:
            return _bls.fast_aggregate_verify([bytes(p) for p in pubkeys], bytes(message), bytes(signature))
        except Exception:
            return False


bls = _BlsNamespace()


def reference_namespace() -> dict:
    """Namespace supplying the 36 free names of the reference's sync-protocol.md blocks."""
    ns = dict(
        BeaconBlockHeader=BeaconBlockHeader, Bytes32=Bytes32, CAPELLA_FORK_EPOCH=CAPELLA_FORK_EPOCH,
        CURRENT_SYNC_COMMITTEE_GINDEX=CURRENT_SYNC_COMMITTEE_GINDEX, Container=Container,
        CurrentSyncCommitteeBranch=CurrentSyncCommitteeBranch, DENEB_FORK_EPOCH=DENEB_FORK_EPOCH,
        DOMAIN_SYNC_COMMITTEE=DomainType(DOMAIN_SYNC_COMMITTEE),
        EXECUTION_PAYLOAD_GINDEX=EXECUTION_PAYLOAD_GINDEX, ExecutionBranch=ExecutionBranch,
        ExecutionPayloadHeader=ExecutionPayloadHeader, FINALIZED_ROOT_GINDEX=FINALIZED_ROOT_GINDEX,
        FinalityBranch=FinalityBranch, GENESIS_SLOT=GENESIS_SLOT, GeneralizedIndex=GeneralizedIndex,
        MIN_SYNC_COMMITTEE_PARTICIPANTS=MIN_SYNC_COMMITTEE_PARTICIPANTS,
        NEXT_SYNC_COMMITTEE_GINDEX=NEXT_SYNC_COMMITTEE_GINDEX, NextSyncCommitteeBranch=NextSyncCommitteeBranch,
        Optional=Optional, Root=Root, Slot=Slot, SyncAggregate=SyncAggregate, SyncCommittee=SyncCommittee,
        UPDATE_TIMEOUT=UPDATE_TIMEOUT, bls=bls, capella=capella, compute_domain=compute_domain,
        compute_epoch_at_slot=compute_epoch_at_slot, compute_fork_version=compute_fork_version,
        compute_signing_root=compute_signing_root, compute_sync_committee_period=compute_sync_committee_period,
        dataclass=dataclass, floorlog2=floorlog2, hash_tree_root=hash_tree_root,
        is_valid_merkle_branch=is_valid_merkle_branch, uint64=uint64,
    )
    return ns
