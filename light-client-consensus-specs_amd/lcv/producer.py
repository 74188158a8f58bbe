"""Producer side of the light-client data: full-node.md's helper and
derivation functions over a sparse view of the beacon state and blocks.

    compute_merkle_proof                    full-node.md:35-38 (declared there without a body)
    block_to_light_client_header            full-node.md:43-89
    create_light_client_bootstrap           full-node.md:105-121
    create_light_client_update              full-node.md:138-188
    create_light_client_finality_update     full-node.md:197-205
    create_light_client_optimistic_update   full-node.md:213-219

A full node holds whole BeaconStates (28 fields, millions of validators); light-client data reads
five of them.  `BeaconStateView` keeps those five explicitly (slot, latest_block_header,
finalized_checkpoint, current / next sync committee) and every other field by its hash_tree_root, so
hash_tree_root(state) and the three state proofs (gindices 54, 55, 105) are exact for the real
state.  `BeaconBlockView` likewise keeps a block's header fields, its body's sync_aggregate and
execution payload (as the 832-byte execution record of include/lcv.h, i.e. the payload's header form:
transactions_root / withdrawals_root in place of the lists, which is what its hash_tree_root and
block_to_light_client_header use) and the other body fields by root.  Outputs are the packed rows of
include/lcv.h (`UpdateRow`, `BootstrapRow`; `pack_updates` -> PackedUpdates for the verifier and
lcv.wire.encode_updates / encode_bootstrap for the wire).  The asserts are the reference's.

Host code (hashlib SHA-256): deriving data is a per-block full-node task off the verifier's hot path;
the 10^4-row synthetic batches of lcv.synth are built here too (pinned against the reference's exec'd
full-node.md blocks: tests/golden/producer.npz).

Views are treated as immutable once their roots are first used (roots are memoised per instance;
`dataclasses.replace` makes a fresh view).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import config as _config
from . import layout as L
from .config import NetworkConfig

# generalized indices (sync-protocol.md:78-81)
FINALIZED_ROOT_GINDEX = 105
CURRENT_SYNC_COMMITTEE_GINDEX = 54
NEXT_SYNC_COMMITTEE_GINDEX = 55
EXECUTION_PAYLOAD_GINDEX = 25
GENESIS_SLOT = 0
MIN_SYNC_COMMITTEE_PARTICIPANTS = 1

STATE_FIELDS = 28        # Deneb BeaconState (Altair 24 .. Deneb 28: one 32-leaf tree either way)
BODY_FIELDS = 12         # Deneb BeaconBlockBody (16-leaf tree)
F_SLOT, F_LATEST_BLOCK_HEADER, F_FINALIZED_CHECKPOINT, F_CURRENT_SC, F_NEXT_SC = 2, 4, 20, 22, 23
B_SYNC_AGGREGATE, B_EXECUTION_PAYLOAD = 8, 9


def sha256(b: bytes, _h=hashlib.sha256) -> bytes:
    return _h(b).digest()


ZERO_HASHES = [bytes(32)]
for _ in range(40):
    ZERO_HASHES.append(sha256(ZERO_HASHES[-1] + ZERO_HASHES[-1]))


# ------------------------------------------------------------------ SSZ merkleization (host)
def merkleize(chunks: Sequence[bytes], depth: int) -> bytes:
    layer = list(chunks)
    assert len(layer) <= 1 << depth
    if not layer:
        return ZERO_HASHES[depth]
    for d in range(depth):
        if len(layer) % 2:
            layer.append(ZERO_HASHES[d])
        layer = [sha256(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def merkle_layers(chunks: Sequence[bytes], depth: int) -> List[List[bytes]]:
    """Every layer of merkleize(chunks, depth), leaves first (odd layers padded with the zero subtree)."""
    layers, layer = [], list(chunks)
    for d in range(depth):
        if len(layer) % 2:
            layer.append(ZERO_HASHES[d])
        layers.append(layer)
        layer = [sha256(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
    layers.append(layer)
    return layers


def layers_path(layers: List[List[bytes]], index: int) -> List[bytes]:
    out = []
    for d, layer in enumerate(layers[:-1]):
        sib = index ^ 1
        out.append(layer[sib] if sib < len(layer) else ZERO_HASHES[d])
        index >>= 1
    return out


def merkle_path(chunks: Sequence[bytes], depth: int, index: int) -> List[bytes]:
    """Sibling roots from leaf `index` of merkleize(chunks, depth) up to the root (bottom-up)."""
    return layers_path(merkle_layers(chunks, depth), index)


def fold_branch(leaf: bytes, branch: Sequence[bytes], index: int) -> bytes:
    v = leaf
    for i, b in enumerate(branch):
        v = sha256(b + v) if (index >> i) & 1 else sha256(v + b)
    return v


def u64_chunk(v: int) -> bytes:
    return int(v).to_bytes(8, "little") + bytes(24)


def htr_beacon(b112: bytes) -> bytes:
    """hash_tree_root(BeaconBlockHeader) of its 112-byte SSZ."""
    chunks = [b112[0:8] + bytes(24), b112[8:16] + bytes(24), b112[16:48], b112[48:80], b112[80:112]]
    return merkleize(chunks, 3)


def htr_exec_record(rec: bytes, deneb: bool) -> bytes:
    """hash_tree_root of the ExecutionPayloadHeader (= of its ExecutionPayload) held in an 832-byte
    execution record (Deneb 17 fields, Capella 15)."""
    bloom = rec[L.EXEC_BLOOM_OFF:L.EXEC_BLOOM_OFF + 256]
    bloom_root = merkleize([bloom[32 * k:32 * k + 32] for k in range(8)], 3)
    ext_len = int.from_bytes(rec[L.EXEC_EXTRALEN_OFF:L.EXEC_EXTRALEN_OFF + 4], "little")
    extra_root = sha256(rec[320:352] + ext_len.to_bytes(8, "little") + bytes(24))
    nf = 17 if deneb else 15
    leaves = [bloom_root if k == 4 else extra_root if k == 10 else rec[32 * k:32 * k + 32] for k in range(nf)]
    return merkleize(leaves, 5 if deneb else 4)


def htr_pubkey(pk: bytes) -> bytes:
    return sha256(pk[:32] + pk[32:48] + bytes(16))


def htr_sync_committee(sc: bytes) -> bytes:
    roots = [htr_pubkey(sc[48 * j:48 * j + 48]) for j in range(L.SYNC_COMMITTEE_SIZE)]
    return sha256(merkleize(roots, 9) + htr_pubkey(sc[L.SYNC_COMMITTEE_SIZE * 48:]))


def htr_sync_aggregate(bits64: bytes, sig96: bytes) -> bytes:
    return sha256(sha256(bits64[:32] + bits64[32:64]) + merkleize([sig96[0:32], sig96[32:64], sig96[64:96]], 2))


def beacon_header(slot: int, proposer_index: int, parent_root: bytes, state_root: bytes, body_root: bytes) -> bytes:
    """112-byte SSZ BeaconBlockHeader."""
    b = (int(slot).to_bytes(8, "little") + int(proposer_index).to_bytes(8, "little") + bytes(parent_root)
         + bytes(state_root) + bytes(body_root))
    assert len(b) == L.BEACON_BYTES
    return b


# ------------------------------------------------------------------ sparse views
_SC_ROOTS: Dict[bytes, bytes] = {}


def _committee_root(sc: bytes) -> bytes:
    """hash_tree_root(SyncCommittee), memoised by content (a committee serves a whole period)."""
    key = sha256(sc)
    r = _SC_ROOTS.get(key)
    if r is None:
        if len(_SC_ROOTS) > (1 << 16):
            _SC_ROOTS.clear()
        r = _SC_ROOTS[key] = htr_sync_committee(sc)
    return r


@dataclass
class BeaconStateView:
    """BeaconState: the fields light-client data reads, plus every field's hash_tree_root.

    field_roots: (28, 32) roots of all fields in BeaconState order; the entries of the explicit fields
    (slot 2, latest_block_header 4, finalized_checkpoint 20, current / next_sync_committee 22 / 23)
    are recomputed from them."""
    slot: int
    latest_block_header: bytes                 # 112 B SSZ
    finalized_checkpoint_epoch: int
    finalized_checkpoint_root: bytes
    current_sync_committee: bytes              # 24,624 B SSZ
    next_sync_committee: bytes
    field_roots: np.ndarray = field(default_factory=lambda: np.zeros((STATE_FIELDS, 32), np.uint8))
    _memo: Optional[list] = field(default=None, init=False, repr=False, compare=False)  # tree layers

    def chunks(self) -> List[bytes]:
        return list(self._layers()[0][:STATE_FIELDS])

    def _layers(self) -> List[List[bytes]]:
        if self._memo is None:
            self._memo = merkle_layers(self._chunks(), 5)
        return self._memo

    def _chunks(self) -> List[bytes]:
        roots = [bytes(r) for r in np.asarray(self.field_roots, np.uint8).reshape(-1, 32)]
        assert len(roots) == STATE_FIELDS
        roots[F_SLOT] = u64_chunk(self.slot)
        roots[F_LATEST_BLOCK_HEADER] = htr_beacon(self.latest_block_header)
        roots[F_FINALIZED_CHECKPOINT] = sha256(u64_chunk(self.finalized_checkpoint_epoch)
                                               + bytes(self.finalized_checkpoint_root))
        roots[F_CURRENT_SC] = _committee_root(bytes(self.current_sync_committee))
        roots[F_NEXT_SC] = _committee_root(bytes(self.next_sync_committee))
        return roots

    def hash_tree_root(self) -> bytes:
        return self._layers()[-1][0]

    def merkle_proof(self, gindex: int) -> List[bytes]:
        layers = self._layers()
        if gindex in (CURRENT_SYNC_COMMITTEE_GINDEX, NEXT_SYNC_COMMITTEE_GINDEX):
            return layers_path(layers, gindex - 32)
        if gindex == FINALIZED_ROOT_GINDEX:  # finalized_checkpoint (field 20) -> its `root` (child 1)
            return [u64_chunk(self.finalized_checkpoint_epoch)] + layers_path(layers, F_FINALIZED_CHECKPOINT)
        raise ValueError(f"no proof for generalized index {gindex} of BeaconState")


@dataclass
class BeaconBlockView:
    """SignedBeaconBlock: the header fields, the body's sync_aggregate and execution payload, and
    every body field's hash_tree_root.

    execution: the payload's 832-byte execution record (header form), needed from Capella on;
    execution_deneb: whether it is a Deneb payload (17 fields) or Capella (15).  body_roots: (12, 32)
    roots of the body fields in BeaconBlockBody order; sync_aggregate (8) and, with an execution
    record, execution_payload (9) are recomputed."""
    slot: int
    proposer_index: int
    parent_root: bytes
    state_root: bytes
    sync_committee_bits: bytes                 # 64 B
    sync_committee_signature: bytes            # 96 B
    execution: Optional[bytes] = None
    execution_deneb: bool = True
    body_roots: np.ndarray = field(default_factory=lambda: np.zeros((BODY_FIELDS, 32), np.uint8))
    _memo: Optional[tuple] = field(default=None, init=False, repr=False, compare=False)  # (body layers, header)

    def _body(self) -> tuple:
        if self._memo is None:
            layers = merkle_layers(self._body_chunks(), 4)
            self._memo = (layers, beacon_header(self.slot, self.proposer_index, self.parent_root, self.state_root,
                                                layers[-1][0]))
        return self._memo

    def body_chunks(self) -> List[bytes]:
        return list(self._body()[0][0][:BODY_FIELDS])

    def _body_chunks(self) -> List[bytes]:
        roots = [bytes(r) for r in np.asarray(self.body_roots, np.uint8).reshape(-1, 32)]
        assert len(roots) == BODY_FIELDS
        roots[B_SYNC_AGGREGATE] = htr_sync_aggregate(bytes(self.sync_committee_bits), bytes(self.sync_committee_signature))
        if self.execution is not None:
            roots[B_EXECUTION_PAYLOAD] = htr_exec_record(bytes(self.execution), self.execution_deneb)
        return roots

    def body_root(self) -> bytes:
        return self.header()[80:112]

    def header(self) -> bytes:
        """BeaconBlockHeader of the block (state_root as the block carries it)."""
        return self._body()[1]

    def hash_tree_root(self) -> bytes:
        """hash_tree_root(block.message) == hash_tree_root of its BeaconBlockHeader."""
        return htr_beacon(self.header())

    def body_merkle_proof(self, gindex: int) -> List[bytes]:
        if gindex != EXECUTION_PAYLOAD_GINDEX:
            raise ValueError(f"no proof for generalized index {gindex} of BeaconBlockBody")
        return layers_path(self._body()[0], gindex - 16)


def compute_merkle_proof(obj, index: int) -> List[bytes]:
    """full-node.md:35-38: the Merkle proof of the node at generalized index `index` (bottom-up)."""
    if isinstance(obj, BeaconStateView):
        return obj.merkle_proof(int(index))
    if isinstance(obj, BeaconBlockView):   # a block's body (the call site passes block.message.body)
        return obj.body_merkle_proof(int(index))
    raise TypeError(f"compute_merkle_proof: unsupported object {type(obj).__name__}")


# ------------------------------------------------------------------ outputs (packed rows)
@dataclass
class HeaderRow:
    """LightClientHeader as include/lcv.h rows."""
    beacon: bytes       # 112
    execution: bytes    # 832
    execution_branch: bytes  # 128


EMPTY_HEADER = HeaderRow(bytes(L.BEACON_BYTES), bytes(L.EXEC_BYTES), bytes(L.EXEC_BRANCH_BYTES))
EMPTY_SYNC_COMMITTEE = bytes(L.SYNC_COMMITTEE_BYTES)


@dataclass
class UpdateRow:
    """LightClientUpdate (sync-protocol.md:120-133); defaults = the reference's LightClientUpdate()."""
    attested_header: HeaderRow = EMPTY_HEADER
    next_sync_committee: bytes = EMPTY_SYNC_COMMITTEE
    next_sync_committee_branch: bytes = bytes(L.NSC_BRANCH_BYTES)
    finalized_header: HeaderRow = EMPTY_HEADER
    finality_branch: bytes = bytes(L.FINALITY_BRANCH_BYTES)
    sync_committee_bits: bytes = bytes(L.BITS_BYTES)
    sync_committee_signature: bytes = bytes(L.SIGNATURE_BYTES)
    signature_slot: int = 0


@dataclass
class BootstrapRow:
    """LightClientBootstrap (sync-protocol.md:109-115)."""
    header: HeaderRow
    current_sync_committee: bytes
    current_sync_committee_branch: bytes  # 160


def block_to_light_client_header(block: BeaconBlockView, cfg: Optional[NetworkConfig] = None) -> HeaderRow:
    """full-node.md:43-89."""
    cfg = cfg or _config.active()
    epoch = cfg.compute_epoch_at_slot(block.slot)
    if epoch >= cfg.CAPELLA_FORK_EPOCH:
        if block.execution is None:
            raise ValueError("a Capella-or-later block needs its execution payload")
        rec = bytearray(block.execution)
        if epoch < cfg.DENEB_FORK_EPOCH:   # the Deneb blob fields exist only from Deneb on
            rec[480:488] = bytes(8)
            rec[512:520] = bytes(8)
        branch = b"".join(compute_merkle_proof(block, EXECUTION_PAYLOAD_GINDEX))
        execution = bytes(rec)
    else:   # pre-Capella: no execution data in light-client headers
        execution, branch = bytes(L.EXEC_BYTES), bytes(L.EXEC_BRANCH_BYTES)
    return HeaderRow(block.header(), execution, branch)


def _state_header_root(state: BeaconStateView) -> bytes:
    """hash_tree_root of state.latest_block_header with state_root = hash_tree_root(state)."""
    h = state.latest_block_header
    return htr_beacon(h[:48] + state.hash_tree_root() + h[80:])


def create_light_client_bootstrap(state: BeaconStateView, block: BeaconBlockView,
                                  cfg: Optional[NetworkConfig] = None) -> BootstrapRow:
    """full-node.md:105-121."""
    cfg = cfg or _config.active()
    assert cfg.compute_epoch_at_slot(state.slot) >= cfg.ALTAIR_FORK_EPOCH
    assert state.slot == int.from_bytes(state.latest_block_header[:8], "little")
    assert _state_header_root(state) == block.hash_tree_root()
    return BootstrapRow(header=block_to_light_client_header(block, cfg),
                        current_sync_committee=bytes(state.current_sync_committee),
                        current_sync_committee_branch=b"".join(
                            compute_merkle_proof(state, CURRENT_SYNC_COMMITTEE_GINDEX)))


def create_light_client_update(state: BeaconStateView, block: BeaconBlockView, attested_state: BeaconStateView,
                               attested_block: BeaconBlockView, finalized_block: Optional[BeaconBlockView],
                               cfg: Optional[NetworkConfig] = None) -> UpdateRow:
    """full-node.md:138-188."""
    cfg = cfg or _config.active()
    assert cfg.compute_epoch_at_slot(attested_state.slot) >= cfg.ALTAIR_FORK_EPOCH
    assert sum(bin(b).count("1") for b in bytes(block.sync_committee_bits)) >= MIN_SYNC_COMMITTEE_PARTICIPANTS

    assert state.slot == int.from_bytes(state.latest_block_header[:8], "little")
    assert _state_header_root(state) == block.hash_tree_root()
    update_signature_period = cfg.compute_sync_committee_period_at_slot(block.slot)

    assert attested_state.slot == int.from_bytes(attested_state.latest_block_header[:8], "little")
    att_root = attested_block.hash_tree_root()
    assert _state_header_root(attested_state) == att_root == bytes(block.parent_root)
    update_attested_period = cfg.compute_sync_committee_period_at_slot(attested_block.slot)

    update = UpdateRow()
    update.attested_header = block_to_light_client_header(attested_block, cfg)

    # next_sync_committee is only useful if the message is signed by the current sync committee
    if update_attested_period == update_signature_period:
        update.next_sync_committee = bytes(attested_state.next_sync_committee)
        update.next_sync_committee_branch = b"".join(compute_merkle_proof(attested_state, NEXT_SYNC_COMMITTEE_GINDEX))

    # indicate finality whenever possible
    if finalized_block is not None:
        if finalized_block.slot != GENESIS_SLOT:
            update.finalized_header = block_to_light_client_header(finalized_block, cfg)
            assert htr_beacon(update.finalized_header.beacon) == bytes(attested_state.finalized_checkpoint_root)
        else:
            assert bytes(attested_state.finalized_checkpoint_root) == bytes(32)
        update.finality_branch = b"".join(compute_merkle_proof(attested_state, FINALIZED_ROOT_GINDEX))

    update.sync_committee_bits = bytes(block.sync_committee_bits)
    update.sync_committee_signature = bytes(block.sync_committee_signature)
    update.signature_slot = int(block.slot)
    return update


def create_light_client_finality_update(update: UpdateRow) -> UpdateRow:
    """full-node.md:197-205: the finality fields of `update` (as an UpdateRow whose next-committee
    fields are the defaults, the form sync-protocol.md:563-571 converts a LightClientFinalityUpdate to)."""
    return UpdateRow(attested_header=update.attested_header, finalized_header=update.finalized_header,
                     finality_branch=update.finality_branch, sync_committee_bits=update.sync_committee_bits,
                     sync_committee_signature=update.sync_committee_signature, signature_slot=update.signature_slot)


def create_light_client_optimistic_update(update: UpdateRow) -> UpdateRow:
    """full-node.md:213-219 (as an UpdateRow with default finality / next-committee fields,
    sync-protocol.md:582-590)."""
    return UpdateRow(attested_header=update.attested_header, sync_committee_bits=update.sync_committee_bits,
                     sync_committee_signature=update.sync_committee_signature, signature_slot=update.signature_slot)


def pack_updates(rows: Sequence[UpdateRow]):
    """UpdateRows -> PackedUpdates (include/lcv.h layouts; next_sync_committee values deduplicated
    into the pool, so HTR(SyncCommittee) runs once per distinct committee on the device)."""
    from .device import PackedUpdates
    n = len(rows)
    pool: Dict[bytes, int] = {}
    idx = np.zeros(n, np.uint32)
    for i, r in enumerate(rows):
        idx[i] = pool.setdefault(bytes(r.next_sync_committee), len(pool))
    pool_arr = np.zeros((max(1, len(pool)), L.SYNC_COMMITTEE_BYTES), np.uint8)
    for sc, k in pool.items():
        pool_arr[k] = np.frombuffer(sc, np.uint8)

    def col(get, width):
        a = np.zeros((n, width), np.uint8)
        for i, r in enumerate(rows):
            a[i] = np.frombuffer(get(r), np.uint8)
        return a
    return PackedUpdates(
        att_beacon=col(lambda r: r.attested_header.beacon, L.BEACON_BYTES),
        att_exec=col(lambda r: r.attested_header.execution, L.EXEC_BYTES),
        att_branch=col(lambda r: r.attested_header.execution_branch, L.EXEC_BRANCH_BYTES),
        fin_beacon=col(lambda r: r.finalized_header.beacon, L.BEACON_BYTES),
        fin_exec=col(lambda r: r.finalized_header.execution, L.EXEC_BYTES),
        fin_branch=col(lambda r: r.finalized_header.execution_branch, L.EXEC_BRANCH_BYTES),
        nsc_branch=col(lambda r: r.next_sync_committee_branch, L.NSC_BRANCH_BYTES),
        finality_branch=col(lambda r: r.finality_branch, L.FINALITY_BRANCH_BYTES),
        sync_bits=col(lambda r: r.sync_committee_bits, L.BITS_BYTES),
        sync_signature=col(lambda r: r.sync_committee_signature, L.SIGNATURE_BYTES),
        nsc_pool=pool_arr, nsc_index=idx,
        signature_slot=np.array([r.signature_slot for r in rows], np.uint64))
