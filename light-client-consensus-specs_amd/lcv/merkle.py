"""Drop-in `is_valid_merkle_branch` (upstream phase0; reference call sites sync-protocol.md:234,
356, 428, 443) and `hash_tree_root(SyncCommittee)` (call site :444), on the SHA-256 kernels of
liblcv.so.  Batched forms take numpy rows and run one lane per branch / committee.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import layout as L
from . import runtime
from .device import Verifier


def is_valid_merkle_branch(leaf: bytes, branch: Sequence[bytes], depth: int, index: int, root: bytes,
                           verifier: Optional[Verifier] = None) -> bool:
    leaf, root = bytes(leaf), bytes(root)
    items = [bytes(b) for b in branch]
    depth, index = int(depth), int(index)
    if len(leaf) != 32 or len(root) != 32 or any(len(b) != 32 for b in items) or depth < 0:
        raise ValueError("is_valid_merkle_branch: leaf/root/branch entries must be 32 bytes")
    if len(items) < depth:
        raise IndexError("is_valid_merkle_branch: branch shorter than depth")  # the spec's branch[i] would raise
    v = verifier if verifier is not None else runtime.default_verifier()
    br = np.frombuffer(b"".join(items[:depth]), np.uint8) if depth else np.zeros(0, np.uint8)
    return bool(v.merkle_branch_batch(np.frombuffer(leaf, np.uint8), br, depth, index,
                                      np.frombuffer(root, np.uint8))[0])


def is_valid_merkle_branch_batch(leaves: np.ndarray, branches: np.ndarray, depth: int, index: int, roots: np.ndarray,
                                 verifier: Optional[Verifier] = None) -> np.ndarray:
    v = verifier if verifier is not None else runtime.default_verifier()
    return v.merkle_branch_batch(leaves, branches, depth, index, roots)


def hash_tree_root_sync_committee(sync_committee, verifier: Optional[Verifier] = None) -> bytes:
    """HTR of one SyncCommittee (object with .pubkeys/.aggregate_pubkey, or its 24624 SSZ bytes)."""
    raw = sync_committee if isinstance(sync_committee, (bytes, bytearray)) else L.pack_sync_committee(sync_committee)
    v = verifier if verifier is not None else runtime.default_verifier()
    return v.htr_sync_committee_batch(np.frombuffer(bytes(raw), np.uint8))[0].tobytes()
