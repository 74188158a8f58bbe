"""SSZ wire decode of light-client messages straight into the packed batch.

Light-client data reaches a client as SSZ bytes (Req/Resp `LightClientUpdatesByRange` chunks,
`light_client_finality_update` / `light_client_optimistic_update` gossip, `LightClientBootstrap`;
p2p-interface.md).  Upstream, each message is deserialised into Python containers
(sync-protocol.md:109-115, :120-133, :138-148, :153-160) and then validated one at a time.  Here a
whole batch of messages is decoded by the native decoder of liblcv.so (`lcv_ssz_decode_updates`,
csrc/lcv_wire.cpp: host C++, strict SSZ offset rules) directly into the `PackedUpdates` rows the
device verifier consumes; no per-update Python objects are built.

    decode_updates(messages, kind="update", fork="deneb")  -> PackedUpdates   (ValueError if malformed)
        fork: "deneb" | "capella" | "altair" for every message, or one per message (a Req/Resp
        response's chunks each carry a ForkDigest context: p2p-interface.md:189-200; `fork_of_digest_version`
        maps a chunk's fork version to its name under the network configuration)
    decode_updates_status(messages, kind, fork)             -> (PackedUpdates, ok: np.ndarray[bool])
    decode_bootstrap(data, fork="deneb")                    -> Bootstrap (header rows, committee, branch)
    encode_updates(batch, kind="update", fork="deneb")      -> [bytes]  (serving side; inverse of decode)

`kind` "finality" / "optimistic" rows are the LightClientUpdate the reference builds from those
messages (sync-protocol.md:563-571 / :582-590).  `messages` is a sequence of `bytes`, or a tuple
(buf: uint8 array, offsets: uint64 array, lengths: uint64 array) describing messages inside one
buffer (e.g. a received Req/Resp payload, without copying).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple, Union

import numpy as np

from . import layout as L
from ._native import HeaderCols, Lib, UpdateBatch, load, ptr
from .device import PackedUpdates

KINDS = {"update": 0, "finality": 1, "optimistic": 2}
FORKS = {"deneb": 0, "capella": 1, "altair": 2}  # altair: LightClientHeader = {beacon}; rows = its Capella upgrade


def fork_of_digest_version(version: bytes, cfg=None) -> str:
    """The light-client container namespace of a message whose ForkDigest context is `version`
    (p2p-interface.md:82-85 / 112-115 / 157-160 / 197-200): ALTAIR..BELLATRIX -> "altair",
    CAPELLA -> "capella", DENEB and later -> "deneb"."""
    from . import config as _config
    cfg = cfg or _config.active()
    v = bytes(version)
    if v in (cfg.ALTAIR_FORK_VERSION, cfg.BELLATRIX_FORK_VERSION):
        return "altair"
    if v == cfg.CAPELLA_FORK_VERSION:
        return "capella"
    if v == cfg.DENEB_FORK_VERSION:
        return "deneb"
    raise ValueError(f"no light-client data for fork version {v.hex()}")


def _fork_codes(fork, n: int):
    """One fork code for the call, or a per-message uint8 array."""
    if isinstance(fork, str):
        if fork not in FORKS:
            raise ValueError(f"fork must be one of {list(FORKS)}")
        return FORKS[fork], None
    forks = list(fork)
    if len(forks) != n or any(f not in FORKS for f in forks):
        raise ValueError(f"fork must be a name or one of {list(FORKS)} per message")
    return None, np.array([FORKS[f] for f in forks], np.uint8)

Messages = Union[Sequence[bytes], Tuple[np.ndarray, np.ndarray, np.ndarray]]


def _lib(lib: Optional[Lib]) -> Lib:
    return lib if lib is not None else load()


def _flatten(messages: Messages) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    if isinstance(messages, tuple) and len(messages) == 3 and isinstance(messages[0], np.ndarray):
        buf, offs, lens = messages
        buf = np.ascontiguousarray(buf, np.uint8).reshape(-1)
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint64)
        if offs.shape != lens.shape or (offs.size and int((offs + lens).max()) > buf.size):
            raise ValueError("offsets/lengths do not describe messages inside buf")
        return buf, offs, lens
    parts = [bytes(m) for m in messages]
    lens = np.array([len(p) for p in parts], np.uint64)
    offs = np.zeros(len(parts), np.uint64)
    if len(parts):
        offs[1:] = np.cumsum(lens)[:-1]
    buf = np.frombuffer(b"".join(parts), np.uint8) if parts else np.zeros(0, np.uint8)
    return buf, offs, lens


def decode_updates_status(messages: Messages, kind: str = "update", fork="deneb",
                          lib: Optional[Lib] = None) -> Tuple[PackedUpdates, np.ndarray]:
    """Decode n SSZ messages -> (PackedUpdates, ok); malformed messages give all-zero rows, ok False."""
    if kind not in KINDS:
        raise ValueError(f"kind must be one of {list(KINDS)}")
    buf, offs, lens = _flatten(messages)
    n = int(offs.size)
    fcode, forks = _fork_codes(fork, n)
    cols = {k: np.zeros((n, w), np.uint8) for k, w in (
        ("att_beacon", L.BEACON_BYTES), ("att_exec", L.EXEC_BYTES), ("att_branch", L.EXEC_BRANCH_BYTES),
        ("fin_beacon", L.BEACON_BYTES), ("fin_exec", L.EXEC_BYTES), ("fin_branch", L.EXEC_BRANCH_BYTES),
        ("nsc_branch", L.NSC_BRANCH_BYTES), ("finality_branch", L.FINALITY_BRANCH_BYTES),
        ("sync_bits", L.BITS_BYTES), ("sync_signature", L.SIGNATURE_BYTES))}
    nsc_index = np.zeros(n, np.uint32)
    sig_slot = np.zeros(n, np.uint64)
    pool_src = np.zeros(n + 1, np.uint64)
    npool = C.c_uint64(0)
    status = np.zeros(max(n, 1), np.uint8)
    b = UpdateBatch()
    b.attested = HeaderCols(ptr(cols["att_beacon"]), ptr(cols["att_exec"]), ptr(cols["att_branch"]))
    b.finalized = HeaderCols(ptr(cols["fin_beacon"]), ptr(cols["fin_exec"]), ptr(cols["fin_branch"]))
    b.nsc_index = ptr(nsc_index, C.c_uint32)
    b.nsc_branch = ptr(cols["nsc_branch"])
    b.finality_branch = ptr(cols["finality_branch"])
    b.sync_bits = ptr(cols["sync_bits"])
    b.sync_signature = ptr(cols["sync_signature"])
    b.signature_slot = ptr(sig_slot, C.c_uint64)
    b.n = n
    b.npool = 0
    src = buf if buf.size else np.zeros(1, np.uint8)
    if forks is None:
        rc = _lib(lib).lcv_ssz_decode_updates(ptr(src), ptr(offs, C.c_uint64), ptr(lens, C.c_uint64), n,
                                             KINDS[kind], fcode, C.byref(b), ptr(pool_src, C.c_uint64),
                                             C.byref(npool), ptr(status))
    else:
        fk = forks if forks.size else np.zeros(1, np.uint8)
        rc = _lib(lib).lcv_ssz_decode_updates_mixed(ptr(src), ptr(offs, C.c_uint64), ptr(lens, C.c_uint64), n,
                                                   KINDS[kind], ptr(fk), C.byref(b), ptr(pool_src, C.c_uint64),
                                                   C.byref(npool), ptr(status))
    if rc != 0:
        raise ValueError(f"lcv_ssz_decode_updates: status {rc}")
    k = int(npool.value)
    pool = np.zeros((max(k, 1), L.SYNC_COMMITTEE_BYTES), np.uint8)
    for j in range(k):  # distinct committees only: a handful per batch
        s = int(pool_src[j])
        if s != 0xFFFFFFFFFFFFFFFF:
            pool[j] = buf[s:s + L.SYNC_COMMITTEE_BYTES]
    batch = PackedUpdates(nsc_pool=pool, nsc_index=nsc_index, signature_slot=sig_slot, **cols)
    return batch, status[:n] == 0


def decode_updates(messages: Messages, kind: str = "update", fork="deneb",
                   lib: Optional[Lib] = None) -> PackedUpdates:
    """Strict decode: raises ValueError (as upstream SSZ deserialisation does) if any message is malformed."""
    batch, ok = decode_updates_status(messages, kind, fork, lib)
    if not ok.all():
        bad = np.flatnonzero(~ok)
        raise ValueError(f"malformed SSZ {kind} message(s) at index {bad[:8].tolist()}")
    return batch


@dataclass
class Bootstrap:
    """LightClientBootstrap (sync-protocol.md:109-115) as packed rows (layouts of include/lcv.h)."""
    beacon: np.ndarray                 # (112,) u8
    execution: np.ndarray              # (832,) u8 execution record
    execution_branch: np.ndarray       # (128,) u8
    current_sync_committee: np.ndarray  # (24624,) u8
    current_sync_committee_branch: np.ndarray  # (160,) u8


def decode_bootstrap(data: bytes, fork: str = "deneb", lib: Optional[Lib] = None) -> Bootstrap:
    if fork not in FORKS:
        raise ValueError(f"fork must be one of {list(FORKS)}")
    buf = np.frombuffer(bytes(data), np.uint8) if len(data) else np.zeros(1, np.uint8)
    out = Bootstrap(np.zeros(L.BEACON_BYTES, np.uint8), np.zeros(L.EXEC_BYTES, np.uint8),
                    np.zeros(L.EXEC_BRANCH_BYTES, np.uint8), np.zeros(L.SYNC_COMMITTEE_BYTES, np.uint8),
                    np.zeros(L.NSC_BRANCH_BYTES, np.uint8))
    st = np.zeros(1, np.uint8)
    rc = _lib(lib).lcv_ssz_decode_bootstrap(ptr(buf), len(data), FORKS[fork], ptr(out.beacon), ptr(out.execution),
                                           ptr(out.execution_branch), ptr(out.current_sync_committee),
                                           ptr(out.current_sync_committee_branch), ptr(st))
    if rc != 0:
        raise ValueError(f"lcv_ssz_decode_bootstrap: status {rc}")
    if st[0]:
        raise ValueError("malformed SSZ LightClientBootstrap")
    return out


# ------------------------------------------------------------------ encode (serving side)
_EXEC_SPANS = ((0, 32), (32, 52), (64, 96), (96, 128), (544, 800), (160, 192), (192, 200), (224, 232), (256, 264),
               (288, 296), None, (352, 384), (384, 416), (416, 448), (448, 480), (480, 488), (512, 520))


def _encode_header(beacon: np.ndarray, rec: np.ndarray, branch: np.ndarray, fork: str) -> bytes:
    if fork == "altair":  # LightClientHeader = {beacon}: the execution data must be empty
        if np.asarray(rec).any() or np.asarray(branch).any():
            raise ValueError("an Altair-format header carries no execution data")
        return np.asarray(beacon).tobytes()
    elen = int.from_bytes(rec[800:804].tobytes(), "little")
    spans = _EXEC_SPANS if fork == "deneb" else _EXEC_SPANS[:15]
    fixed = 584 if fork == "deneb" else 568
    ex = b"".join(fixed.to_bytes(4, "little") if s is None else rec[s[0]:s[1]].tobytes() for s in spans)
    return (beacon.tobytes() + (L.BEACON_BYTES + 4 + L.EXEC_BRANCH_BYTES).to_bytes(4, "little") + branch.tobytes()
            + ex + rec[320:320 + elen].tobytes())


def encode_updates(batch: PackedUpdates, kind: str = "update", fork: str = "deneb") -> list:
    """Packed rows -> SSZ wire bytes of LightClientUpdate / FinalityUpdate / OptimisticUpdate (the
    inverse of decode_updates for rows that came from such messages; a full node serves these)."""
    if kind not in KINDS or fork not in FORKS:
        raise ValueError(f"kind must be one of {list(KINDS)}, fork one of {list(FORKS)}")
    out = []
    for i in range(batch.n):
        att = _encode_header(batch.att_beacon[i], batch.att_exec[i], batch.att_branch[i], fork)
        tail = batch.sync_bits[i].tobytes() + batch.sync_signature[i].tobytes() + int(batch.signature_slot[i]).to_bytes(8, "little")
        if fork == "altair":  # every container fixed-size: fields in order, no offsets
            fin = _encode_header(batch.fin_beacon[i], batch.fin_exec[i], batch.fin_branch[i], fork)
            if kind == "optimistic":
                out.append(att + tail)
            elif kind == "finality":
                out.append(att + fin + batch.finality_branch[i].tobytes() + tail)
            else:
                out.append(att + batch.nsc_pool[int(batch.nsc_index[i])].tobytes() + batch.nsc_branch[i].tobytes()
                           + fin + batch.finality_branch[i].tobytes() + tail)
            continue
        if kind == "optimistic":
            fixed = 4 + len(tail)
            out.append(fixed.to_bytes(4, "little") + tail + att)
            continue
        fin = _encode_header(batch.fin_beacon[i], batch.fin_exec[i], batch.fin_branch[i], fork)
        mid = batch.finality_branch[i].tobytes() + tail
        if kind == "finality":
            fixed = 8 + len(mid)
            out.append(fixed.to_bytes(4, "little") + (fixed + len(att)).to_bytes(4, "little") + mid + att + fin)
            continue
        sc = batch.nsc_pool[int(batch.nsc_index[i])].tobytes() + batch.nsc_branch[i].tobytes()
        fixed = 4 + len(sc) + 4 + len(mid)
        out.append(fixed.to_bytes(4, "little") + sc + (fixed + len(att)).to_bytes(4, "little") + mid + att + fin)
    return out


def encode_bootstrap(beacon: bytes, execution: bytes, execution_branch: bytes, committee: bytes,
                     committee_branch: bytes, fork: str = "deneb") -> bytes:
    """LightClientBootstrap rows (sync-protocol.md:109-115) -> SSZ wire bytes (inverse of decode_bootstrap)."""
    if fork not in FORKS:
        raise ValueError(f"fork must be one of {list(FORKS)}")
    u8 = lambda b: np.frombuffer(bytes(b), np.uint8)  # noqa: E731
    if len(committee) != L.SYNC_COMMITTEE_BYTES or len(committee_branch) != 160:
        raise ValueError("committee must be 24,624 bytes and its branch 5 x 32 bytes")
    hdr = _encode_header(u8(beacon), u8(execution), u8(execution_branch), fork)
    if fork == "altair":
        return hdr + bytes(committee) + bytes(committee_branch)
    fixed = 4 + L.SYNC_COMMITTEE_BYTES + 160
    return fixed.to_bytes(4, "little") + bytes(committee) + bytes(committee_branch) + hdr
