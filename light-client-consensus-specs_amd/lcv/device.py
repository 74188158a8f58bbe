"""`Verifier`: one device context of liblcv.so and numpy-level wrappers around the C ABI."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, fields
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

from . import config as _config
from ._native import Lib, LcvError, UpdateBatch, HeaderCols, as_u8, load, ptr

SYNC_COMMITTEE_BYTES = 24624
EXEC_RECORD_BYTES = 832


@dataclass
class PackedUpdates:
    """Structure-of-arrays batch of LightClientUpdates (row i = update i); layouts in include/lcv.h."""
    att_beacon: np.ndarray       # (n, 112) u8
    att_exec: np.ndarray         # (n, 832) u8
    att_branch: np.ndarray       # (n, 128) u8
    fin_beacon: np.ndarray       # (n, 112) u8
    fin_exec: np.ndarray         # (n, 832) u8
    fin_branch: np.ndarray       # (n, 128) u8
    nsc_pool: np.ndarray         # (npool, 24624) u8
    nsc_index: np.ndarray        # (n,) u32
    nsc_branch: np.ndarray       # (n, 160) u8
    finality_branch: np.ndarray  # (n, 192) u8
    sync_bits: np.ndarray        # (n, 64) u8
    sync_signature: np.ndarray   # (n, 96) u8
    signature_slot: np.ndarray   # (n,) u64

    @property
    def n(self) -> int:
        return int(self.att_beacon.shape[0])

    def check(self) -> None:
        n = self.n
        shapes = dict(att_beacon=112, att_exec=832, att_branch=128, fin_beacon=112, fin_exec=832, fin_branch=128,
                      nsc_branch=160, finality_branch=192, sync_bits=64, sync_signature=96)
        for name, w in shapes.items():
            a = getattr(self, name)
            if a.dtype != np.uint8 or a.shape != (n, w) or not a.flags.c_contiguous:
                raise ValueError(f"{name}: need C-contiguous uint8 ({n}, {w}), got {a.dtype} {a.shape}")
        if self.nsc_pool.dtype != np.uint8 or self.nsc_pool.ndim != 2 or self.nsc_pool.shape[1] != SYNC_COMMITTEE_BYTES:
            raise ValueError("nsc_pool: need uint8 (npool, 24624)")
        if self.nsc_index.dtype != np.uint32 or self.nsc_index.shape != (n,):
            raise ValueError("nsc_index: need uint32 (n,)")
        if self.signature_slot.dtype != np.uint64 or self.signature_slot.shape != (n,):
            raise ValueError("signature_slot: need uint64 (n,)")
        if n and int(self.nsc_index.max()) >= self.nsc_pool.shape[0]:
            raise ValueError("nsc_index out of range")

    def slice(self, lo: int, hi: int) -> "PackedUpdates":
        kw = {}
        for f in fields(self):
            a = getattr(self, f.name)
            kw[f.name] = a if f.name == "nsc_pool" else np.ascontiguousarray(a[lo:hi])
        return PackedUpdates(**kw)

    def to_c(self) -> Tuple[UpdateBatch, list]:
        self.check()
        keep = []

        def P(a, t=C.c_uint8):
            a = np.ascontiguousarray(a)
            keep.append(a)
            return ptr(a, t)

        b = UpdateBatch()
        b.attested = HeaderCols(P(self.att_beacon), P(self.att_exec), P(self.att_branch))
        b.finalized = HeaderCols(P(self.fin_beacon), P(self.fin_exec), P(self.fin_branch))
        b.nsc_pool = P(self.nsc_pool)
        b.nsc_index = P(self.nsc_index, C.c_uint32)
        b.nsc_branch = P(self.nsc_branch)
        b.finality_branch = P(self.finality_branch)
        b.sync_bits = P(self.sync_bits)
        b.sync_signature = P(self.sync_signature)
        b.signature_slot = P(self.signature_slot, C.c_uint64)
        b.n = self.n
        b.npool = int(self.nsc_pool.shape[0])
        return b, keep


class ResidentBatch:
    def __init__(self, verifier: "Verifier", handle: C.c_void_p, n: int):
        self.v = verifier
        self.handle = handle
        self.n = n

    def free(self):
        if self.handle:
            self.v.lib.lcv_batch_free(self.v.ctx, self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Verifier:
    """A liblcv context on one device.  `lib` defaults to the product HIP library."""

    def __init__(self, device: int = 0, lib: Optional[Lib] = None):
        self.lib = lib if lib is not None else load()
        self.ctx = C.c_void_p()
        rc = self.lib.lcv_init(device, C.byref(self.ctx))
        if rc != 0:
            raise LcvError(f"lcv_init(device={device}) failed with status {rc}")
        self.device = device
        self.config = _config.MAINNET  # the context's network configuration (lcv_init: mainnet)
        self.latency_mode = 64  # lcv_set_latency_mode's value (lcv_init's default: the fan engine up to 64 rows)

    # ------------------------------------------------------------------ plumbing
    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self.lib.lcv_last_error(self.ctx)
            raise LcvError(f"{what}: status {rc}: {msg.decode() if msg else ''}")

    def close(self):
        if self.ctx:
            self.lib.lcv_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_config(self, cfg: "_config.NetworkConfig") -> None:
        """The network configuration this context validates under (lcv_set_config; mainnet after init)."""
        epochs = np.array(cfg.fork_epochs(), np.uint64)
        versions = np.frombuffer(b"".join(cfg.fork_versions()), np.uint8).copy()
        dom = np.frombuffer(cfg.DOMAIN_SYNC_COMMITTEE, np.uint8).copy()
        self._check(self.lib.lcv_set_config(self.ctx, int(cfg.SLOTS_PER_EPOCH), int(cfg.EPOCHS_PER_SYNC_COMMITTEE_PERIOD),
                                            ptr(epochs, C.c_uint64), ptr(versions), ptr(dom)), "lcv_set_config")
        self.config = cfg

    def set_pipeline(self, streams: int, chunks: int) -> None:
        """Run validate's per-update stage chain on `chunks` slices over `streams` HIP streams
        (overlapping stages of different slices); (1, 1) = serial stages with per-stage timings."""
        self._check(self.lib.lcv_set_pipeline(self.ctx, int(streams), int(chunks)), "lcv_set_pipeline")

    def set_latency_mode(self, max_rows: int) -> None:
        """Latency mode for small batches (lcv_set_latency_mode): batches of at most max_rows rows run the SOP
        programs (hash_to_G2's tail, final exponentiation) on the fan engine (an op's K products on K lanes, its
        reduction and tail on a 16-lane row, one item per block), both Miller walks and the accumulation as one fan-engine program, and the SSWU
        maps / signature decoding one item per wave (square-root chains spread over the wave) — one update
        6.0 ms on the batch engine -> 2.8 ms.  Results are identical to the batch engine's.  Default 64;
        0 = the batch engine always."""
        self._check(self.lib.lcv_set_latency_mode(self.ctx, int(max_rows)), "lcv_set_latency_mode")
        self.latency_mode = int(max_rows)

    def engine_log(self, reset: bool = False) -> Dict[str, object]:
        """Which engines ran since the last reset (lcv_debug_engine_log): SOP launches on the fan / batch
        engine, SSWU + signature launches on the one-item-per-wave twins / one lane per item, and the items
        per wave of each SOP program's last batch-engine launch (0 = not launched)."""
        out = np.zeros(8, np.uint64)
        self._check(self.lib.lcv_debug_engine_log(self.ctx, ptr(out, C.c_uint64), 1 if reset else 0),
                    "lcv_debug_engine_log")
        return {"fan": int(out[0]), "batch": int(out[1]), "twin": int(out[2]), "lane": int(out[3]),
                "items": dict(zip(("lines", "miller_acc", "fexp", "h2c"), (int(x) for x in out[4:8])))}

    def last_timings(self) -> Dict[str, float]:
        ms = (C.c_float * 16)()
        n = C.c_int()
        self._check(self.lib.lcv_last_timings(self.ctx, ms, 16, C.byref(n)), "lcv_last_timings")
        return {self.lib.lcv_stage_name(i).decode(): float(ms[i]) for i in range(n.value)}

    # ------------------------------------------------------------------ validation
    def set_store(self, finalized_slot: int, current_sync_committee: bytes, next_sync_committee: bytes) -> np.ndarray:
        cur = as_u8(bytes(current_sync_committee))
        nxt = as_u8(bytes(next_sync_committee))
        if cur.size != SYNC_COMMITTEE_BYTES or nxt.size != SYNC_COMMITTEE_BYTES:
            raise ValueError("committees must be 24624-byte SSZ SyncCommittee values")
        ks = np.zeros(1024, np.uint8)
        self._check(self.lib.lcv_set_store(self.ctx, int(finalized_slot), ptr(cur), ptr(nxt), ptr(ks)), "lcv_set_store")
        return ks

    def validate(self, batch: PackedUpdates, current_slot: int, genesis_validators_root: bytes):
        b, keep = batch.to_c()
        gvr = as_u8(bytes(genesis_validators_root))
        v = np.zeros(batch.n, np.uint8)
        r = np.zeros(batch.n, np.uint8)
        self._check(self.lib.lcv_validate_updates(self.ctx, C.byref(b), int(current_slot), ptr(gvr), ptr(v), ptr(r)),
                    "lcv_validate_updates")
        return v.astype(bool), r

    def upload(self, batch: PackedUpdates) -> ResidentBatch:
        b, keep = batch.to_c()
        h = C.c_void_p()
        self._check(self.lib.lcv_batch_upload(self.ctx, C.byref(b), C.byref(h)), "lcv_batch_upload")
        return ResidentBatch(self, h, batch.n)

    def validate_resident(self, rb: ResidentBatch, current_slot: int, genesis_validators_root: bytes,
                          verdict: Optional[np.ndarray] = None, reason: Optional[np.ndarray] = None):
        gvr = as_u8(bytes(genesis_validators_root))
        v = verdict if verdict is not None else np.zeros(rb.n, np.uint8)
        r = reason if reason is not None else np.zeros(rb.n, np.uint8)
        self._check(self.lib.lcv_validate_resident(self.ctx, rb.handle, int(current_slot), ptr(gvr), ptr(v), ptr(r)),
                    "lcv_validate_resident")
        return v, r

    def validate_resident_dev(self, rb: ResidentBatch, current_slot: int, genesis_validators_root: bytes,
                              verdict_dev_ptr: int):
        gvr = as_u8(bytes(genesis_validators_root))
        self._check(self.lib.lcv_validate_resident_dev(self.ctx, rb.handle, int(current_slot), ptr(gvr),
                                                       C.c_void_p(verdict_dev_ptr)), "lcv_validate_resident_dev")

    def validate_resident_async(self, rb: ResidentBatch, current_slot: int, genesis_validators_root: bytes,
                                slot: int) -> None:
        """Enqueue the whole pipeline for rb on work-space slot 0..7 and return at once (up to eight
        batches in flight); collect the verdicts with slot_wait(slot)."""
        gvr = as_u8(bytes(genesis_validators_root))
        self._keep_gvr = getattr(self, "_keep_gvr", {})
        self._keep_gvr[slot] = gvr  # the call reads it before returning; kept for symmetry with the slot
        self._check(self.lib.lcv_validate_resident_async(self.ctx, rb.handle, int(current_slot), ptr(gvr), int(slot)),
                    "lcv_validate_resident_async")

    def validate_async(self, batch: PackedUpdates, current_slot: int, genesis_validators_root: bytes,
                       slot: int) -> None:
        """Host-input serving entry (lcv_validate_async): the batch is staged into slot 0..7's pinned buffer,
        uploaded, validated and its verdicts copied back, all enqueued; collect them with slot_wait(slot).
        The batch's arrays may be reused as soon as this returns."""
        b, keep = batch.to_c()
        gvr = as_u8(bytes(genesis_validators_root))
        self._check(self.lib.lcv_validate_async(self.ctx, C.byref(b), int(current_slot), ptr(gvr), int(slot)),
                    "lcv_validate_async")
        del keep

    def event_pool(self) -> int:
        """HIP events held for stage timings (test hook: must stay bounded under asynchronous calls)."""
        n = C.c_uint64()
        self._check(self.lib.lcv_debug_event_pool(self.ctx, C.byref(n)), "lcv_debug_event_pool")
        return int(n.value)

    def slot_wait(self, slot: int, n: int, verdict: Optional[np.ndarray] = None, reason: Optional[np.ndarray] = None):
        """Wait for the batch of `slot`; its first n verdicts (bool) and reason codes."""
        v = verdict if verdict is not None else np.zeros(n, np.uint8)
        r = reason if reason is not None else np.zeros(n, np.uint8)
        self._check(self.lib.lcv_slot_wait(self.ctx, int(slot), int(n), ptr(v), ptr(r)), "lcv_slot_wait")
        return v, r

    # ------------------------------------------------------------------ BLS / SSZ primitives
    def fast_aggregate_verify(self, pubkeys: Sequence[bytes], message: bytes, signature: bytes) -> bool:
        pks = as_u8(b"".join(bytes(p) for p in pubkeys)) if len(pubkeys) else np.zeros(1, np.uint8)
        if any(len(bytes(p)) != 48 for p in pubkeys):
            return False
        msg, sig = bytes(message), bytes(signature)
        if len(sig) != 96:
            return False
        m = as_u8(msg) if msg else np.zeros(1, np.uint8)
        res = C.c_int()
        self._check(self.lib.lcv_fast_aggregate_verify(self.ctx, ptr(pks), len(pubkeys), ptr(m), len(msg),
                                                       ptr(as_u8(sig)), C.byref(res)), "lcv_fast_aggregate_verify")
        return bool(res.value)

    def fast_aggregate_verify_batch(self, committees: np.ndarray, committee_id: np.ndarray, bits: np.ndarray,
                                    msgs: np.ndarray, sigs: np.ndarray) -> np.ndarray:
        committees = np.ascontiguousarray(committees, np.uint8).reshape(-1, 512 * 48)
        cid = np.ascontiguousarray(committee_id, np.uint32)
        bits = np.ascontiguousarray(bits, np.uint8).reshape(-1, 64)
        msgs = np.ascontiguousarray(msgs, np.uint8).reshape(-1, 32)
        sigs = np.ascontiguousarray(sigs, np.uint8).reshape(-1, 96)
        n = cid.shape[0]
        out = np.zeros(n, np.uint8)
        self._check(self.lib.lcv_fast_aggregate_verify_batch(self.ctx, ptr(committees), committees.shape[0],
                                                             ptr(cid, C.c_uint32), ptr(bits), ptr(msgs), ptr(sigs), n,
                                                             ptr(out)), "lcv_fast_aggregate_verify_batch")
        return out.astype(bool)

    def merkle_branch_batch(self, leaves: np.ndarray, branches: np.ndarray, depth: int, index: int,
                            roots: np.ndarray) -> np.ndarray:
        leaves = np.ascontiguousarray(leaves, np.uint8).reshape(-1, 32)
        n = leaves.shape[0]
        branches = np.ascontiguousarray(branches, np.uint8).reshape(n, 32 * depth) if depth else np.zeros((n, 0), np.uint8)
        roots = np.ascontiguousarray(roots, np.uint8).reshape(n, 32)
        out = np.zeros(n, np.uint8)
        br = branches if depth else np.zeros(32, np.uint8)
        self._check(self.lib.lcv_merkle_branch_batch(self.ctx, ptr(leaves), ptr(np.ascontiguousarray(br)), int(depth),
                                                     int(index), ptr(roots), n, ptr(out)), "lcv_merkle_branch_batch")
        return out.astype(bool)

    def htr_sync_committee_batch(self, committees: np.ndarray) -> np.ndarray:
        committees = np.ascontiguousarray(committees, np.uint8).reshape(-1, SYNC_COMMITTEE_BYTES)
        n = committees.shape[0]
        out = np.zeros((n, 32), np.uint8)
        self._check(self.lib.lcv_htr_sync_committee_batch(self.ctx, ptr(committees), n, ptr(out)),
                    "lcv_htr_sync_committee_batch")
        return out

    def bootstrap_check_batch(self, beacon: np.ndarray, execution: np.ndarray, exec_branch: np.ndarray,
                              committees: np.ndarray, committee_branch: np.ndarray, trusted_roots: np.ndarray
                              ) -> np.ndarray:
        """initialize_light_client_store's asserts (sync-protocol.md:353-362) per row -> reason codes
        (0 ok, 1 header, 2 trusted root, 3 current_sync_committee branch)."""
        beacon = np.ascontiguousarray(beacon, np.uint8).reshape(-1, 112)
        n = beacon.shape[0]
        cols = [beacon, np.ascontiguousarray(execution, np.uint8).reshape(n, EXEC_RECORD_BYTES),
                np.ascontiguousarray(exec_branch, np.uint8).reshape(n, 128),
                np.ascontiguousarray(committees, np.uint8).reshape(n, SYNC_COMMITTEE_BYTES),
                np.ascontiguousarray(committee_branch, np.uint8).reshape(n, 160),
                np.ascontiguousarray(trusted_roots, np.uint8).reshape(n, 32)]
        out = np.zeros(n, np.uint8)
        self._check(self.lib.lcv_bootstrap_check_batch(self.ctx, *[ptr(c) for c in cols], n, ptr(out)),
                    "lcv_bootstrap_check_batch")
        return out

    def sk_to_pk_batch(self, sks: np.ndarray) -> np.ndarray:
        sks = np.ascontiguousarray(sks, np.uint8).reshape(-1, 32)
        out = np.zeros((sks.shape[0], 48), np.uint8)
        self._check(self.lib.lcv_sk_to_pk_batch(self.ctx, ptr(sks), sks.shape[0], ptr(out)), "lcv_sk_to_pk_batch")
        return out

    def sign_batch(self, sks: np.ndarray, msgs: np.ndarray) -> np.ndarray:
        sks = np.ascontiguousarray(sks, np.uint8).reshape(-1, 32)
        msgs = np.ascontiguousarray(msgs, np.uint8).reshape(-1, 32)
        out = np.zeros((sks.shape[0], 96), np.uint8)
        self._check(self.lib.lcv_sign_batch(self.ctx, ptr(sks), ptr(msgs), sks.shape[0], ptr(out)), "lcv_sign_batch")
        return out

    # ------------------------------------------------------------------ parity-test entry points
    def debug_fp(self, a: np.ndarray, b: np.ndarray):
        a = np.ascontiguousarray(a, np.uint8).reshape(-1, 48)
        b = np.ascontiguousarray(b, np.uint8).reshape(-1, 48)
        n = a.shape[0]
        out = np.zeros((n, 288), np.uint8)
        ok = np.zeros(n, np.uint8)
        self._check(self.lib.lcv_debug_fp(self.ctx, ptr(a), ptr(b), n, ptr(out), ptr(ok)), "lcv_debug_fp")
        return out, ok

    def debug_fp_pow(self, a: np.ndarray) -> np.ndarray:
        """(n, 96): a^((p+1)/4) || a^((p-3)/4), canonical big-endian."""
        a = np.ascontiguousarray(a, np.uint8).reshape(-1, 48)
        out = np.zeros((a.shape[0], 96), np.uint8)
        self._check(self.lib.lcv_debug_fp_pow(self.ctx, ptr(a), a.shape[0], ptr(out)), "lcv_debug_fp_pow")
        return out

    def debug_hash_to_g2(self, msgs: np.ndarray):
        msgs = np.ascontiguousarray(msgs, np.uint8).reshape(-1, 32)
        n = msgs.shape[0]
        out = np.zeros((n, 192), np.uint8)
        inf = np.zeros(n, np.uint8)
        self._check(self.lib.lcv_debug_hash_to_g2(self.ctx, ptr(msgs), n, ptr(out), ptr(inf)), "lcv_debug_hash_to_g2")
        return out, inf

    def debug_g2_decompress(self, sigs: np.ndarray):
        sigs = np.ascontiguousarray(sigs, np.uint8).reshape(-1, 96)
        n = sigs.shape[0]
        out = np.zeros((n, 192), np.uint8)
        st = np.zeros(n, np.uint8)
        self._check(self.lib.lcv_debug_g2_decompress(self.ctx, ptr(sigs), n, ptr(out), ptr(st)),
                    "lcv_debug_g2_decompress")
        return out, st

    def debug_aggregate(self, committees: np.ndarray, committee_id: np.ndarray, bits: np.ndarray):
        committees = np.ascontiguousarray(committees, np.uint8).reshape(-1, 512 * 48)
        cid = np.ascontiguousarray(committee_id, np.uint32)
        bits = np.ascontiguousarray(bits, np.uint8).reshape(-1, 64)
        n = cid.shape[0]
        out = np.zeros((n, 96), np.uint8)
        st = np.zeros(n, np.uint8)
        self._check(self.lib.lcv_debug_aggregate(self.ctx, ptr(committees), committees.shape[0], ptr(cid, C.c_uint32),
                                                 ptr(bits), n, ptr(out), ptr(st)), "lcv_debug_aggregate")
        return out, st

    def debug_pairing(self, p96: np.ndarray, q192: np.ndarray) -> np.ndarray:
        p96 = np.ascontiguousarray(p96, np.uint8).reshape(-1, 96)
        q192 = np.ascontiguousarray(q192, np.uint8).reshape(-1, 192)
        n = p96.shape[0]
        out = np.zeros((n, 576), np.uint8)
        self._check(self.lib.lcv_debug_pairing(self.ctx, ptr(p96), ptr(q192), n, ptr(out)), "lcv_debug_pairing")
        return out
