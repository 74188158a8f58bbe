"""Byte layouts of the packed (structure-of-arrays) update batch, and packing of spec objects.

The drop-ins (`lcv.sync_protocol.validate_light_client_update`, ...) accept the reference's own
container objects (`LightClientUpdate`, `LightClientHeader`, `SyncCommittee`,
reference sync-protocol.md:96-133) by duck typing: anything with the same attribute names and
SSZ-serialisable values works (eth2spec/remerkleable objects, or the test oracle's containers).
They are packed here into the row layouts of include/lcv.h:

  beacon      112 B  SSZ BeaconBlockHeader (slot u64, proposer_index u64, parent_root, state_root,
                     body_root)
  execution   832 B  17 leaf chunks of ExecutionPayloadHeader in field order (leaf 4 = logs_bloom
                     is unused/zero, leaf 10 = extra_data zero padded), logs_bloom at 544,
                     extra_data length u32 at 800; all-zero <=> ExecutionPayloadHeader()
  branch      n x 32 B (execution 4, next_sync_committee 5, finality 6)
  bits        64 B   SSZ Bitvector[512]
  signature   96 B   compressed G2
  committee   24624 B SSZ SyncCommittee (512 x 48 B pubkeys, 48 B aggregate_pubkey)

No BLS or SHA arithmetic happens here: packing is pure byte plumbing (the device hashes).
"""
from __future__ import annotations

from typing import Iterable, List, Sequence, Tuple

import numpy as np

SYNC_COMMITTEE_SIZE = 512
PUBKEY_BYTES = 48
SIGNATURE_BYTES = 96
SYNC_COMMITTEE_BYTES = SYNC_COMMITTEE_SIZE * PUBKEY_BYTES + PUBKEY_BYTES  # 24624
BEACON_BYTES = 112
EXEC_BYTES = 832
EXEC_BLOOM_OFF = 544
EXEC_EXTRALEN_OFF = 800
EXEC_BRANCH_BYTES = 128
NSC_BRANCH_BYTES = 160
FINALITY_BRANCH_BYTES = 192
BITS_BYTES = 64
MAX_EXTRA_DATA_BYTES = 32

# ExecutionPayloadHeader field order (Deneb: 17 fields; Capella: the first 15)
EXEC_FIELDS = ("parent_hash", "fee_recipient", "state_root", "receipts_root", "logs_bloom", "prev_randao",
               "block_number", "gas_limit", "gas_used", "timestamp", "extra_data", "base_fee_per_gas",
               "block_hash", "transactions_root", "withdrawals_root", "blob_gas_used", "excess_blob_gas")
_U64_FIELDS = {"block_number", "gas_limit", "gas_used", "timestamp", "blob_gas_used", "excess_blob_gas"}


def _b(x) -> bytes:
    return bytes(x)


def pack_beacon(beacon) -> bytes:
    """SSZ serialisation of BeaconBlockHeader (fixed 112 bytes)."""
    out = (int(beacon.slot).to_bytes(8, "little") + int(beacon.proposer_index).to_bytes(8, "little")
           + _b(beacon.parent_root) + _b(beacon.state_root) + _b(beacon.body_root))
    if len(out) != BEACON_BYTES:
        raise ValueError("malformed BeaconBlockHeader")
    return out


def pack_execution(execution) -> bytes:
    """Execution record (832 B) of a Deneb or Capella ExecutionPayloadHeader (missing Deneb blob
    fields of a Capella header read as 0)."""
    rec = bytearray(EXEC_BYTES)
    for k, name in enumerate(EXEC_FIELDS):
        v = getattr(execution, name, 0)
        if name == "logs_bloom":
            bloom = _b(v)
            if len(bloom) != 256:
                raise ValueError("logs_bloom must be 256 bytes")
            rec[EXEC_BLOOM_OFF:EXEC_BLOOM_OFF + 256] = bloom
        elif name == "extra_data":
            ed = _b(v)
            if len(ed) > MAX_EXTRA_DATA_BYTES:
                raise ValueError("extra_data longer than 32 bytes")
            rec[32 * k:32 * k + len(ed)] = ed
            rec[EXEC_EXTRALEN_OFF:EXEC_EXTRALEN_OFF + 4] = len(ed).to_bytes(4, "little")
        elif name in _U64_FIELDS:
            rec[32 * k:32 * k + 8] = int(v).to_bytes(8, "little")
        elif name == "base_fee_per_gas":
            rec[32 * k:32 * k + 32] = int(v).to_bytes(32, "little")
        else:
            b = _b(v)
            if len(b) > 32:
                raise ValueError(f"{name} longer than 32 bytes")
            rec[32 * k:32 * k + len(b)] = b
    return bytes(rec)


def pack_branch(branch, depth: int) -> bytes:
    items = [_b(x) for x in branch]
    if len(items) != depth or any(len(x) != 32 for x in items):
        raise ValueError(f"branch must be {depth} x 32 bytes")
    return b"".join(items)


def pack_header(header) -> Tuple[bytes, bytes, bytes]:
    """LightClientHeader (reference sync-protocol.md:96-101) -> (beacon, execution, branch) rows."""
    return pack_beacon(header.beacon), pack_execution(header.execution), pack_branch(header.execution_branch, 4)


def pack_sync_committee(sc) -> bytes:
    pks = [_b(p) for p in sc.pubkeys]
    if len(pks) != SYNC_COMMITTEE_SIZE or any(len(p) != PUBKEY_BYTES for p in pks):
        raise ValueError("SyncCommittee must hold 512 x 48-byte pubkeys")
    agg = _b(sc.aggregate_pubkey)
    if len(agg) != PUBKEY_BYTES:
        raise ValueError("aggregate_pubkey must be 48 bytes")
    return b"".join(pks) + agg


def pack_bits(bits: Sequence) -> bytes:
    """SSZ Bitvector[512]: bit i -> byte i // 8, bit i % 8."""
    arr = np.asarray([bool(x) for x in bits], dtype=np.uint8)
    if arr.shape != (SYNC_COMMITTEE_SIZE,):
        raise ValueError("sync_committee_bits must have 512 entries")
    return np.packbits(arr, bitorder="little").tobytes()


def unpack_bits(b64: bytes) -> List[bool]:
    return [bool(x) for x in np.unpackbits(np.frombuffer(bytes(b64), np.uint8), bitorder="little")]
