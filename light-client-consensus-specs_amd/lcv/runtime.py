"""Process-wide device contexts for the drop-in functions (one `Verifier` per device).

`default_verifier()` opens liblcv.so on device 0 (or the device chosen with `use_device`).
`set_default_verifier(v)` lets a caller (or the test-suite's host-simulation harness) supply its own
context.  The store snapshot last sent to a context is remembered, so repeated single-update calls
against one store (the reference's per-update usage, sync-protocol.md:512) decode and KeyValidate
the two committees only once.
"""
from __future__ import annotations

import hashlib
import threading
from typing import Dict, Optional

from . import config
from .device import Verifier

_lock = threading.Lock()
_default: Optional[Verifier] = None
_device = 0
_store_key: Dict[int, bytes] = {}


def use_device(device: int) -> None:
    global _device, _default
    with _lock:
        _device = int(device)
        _default = None


def set_default_verifier(v: Optional[Verifier]) -> None:
    global _default
    with _lock:
        _default = v


def default_verifier() -> Verifier:
    """The process-wide context (opened on first use, with the active network configuration)."""
    global _default
    with _lock:
        if _default is None:
            v = Verifier(_device)
            if config.active() != config.MAINNET:
                v.set_config(config.active())
            _default = v
        return _default


def current_default() -> Optional[Verifier]:
    return _default


def ensure_store(v: Verifier, finalized_slot: int, current: bytes, nxt: bytes) -> None:
    key = hashlib.sha256(finalized_slot.to_bytes(8, "little") + current + nxt).digest()
    if _store_key.get(id(v)) == key and getattr(v, "_store_key", None) == key:
        return
    v.set_store(finalized_slot, current, nxt)
    v._store_key = key
    _store_key[id(v)] = key
