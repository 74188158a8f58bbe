"""lcv — MI355X (gfx950) batched verifier for the light-client sync-protocol hot path.

Drop-ins for the reference's call surface (Inspector-Butters/light-client-consensus-specs):
    lcv.bls.FastAggregateVerify                    sync-protocol.md:464
    lcv.merkle.is_valid_merkle_branch              sync-protocol.md:234,356,428,443
    lcv.sync_protocol.validate_light_client_update sync-protocol.md:386-465
plus the batched `lcv.sync_protocol.validate_light_client_updates` (packed SoA batches), the store
state machine over verified batches (`lcv.store`: process_light_client_update(s), sync-protocol.md:470-592) and
`lcv.device.Verifier` (one liblcv.so context per GPU).  All arithmetic runs in the HIP kernels of
liblcv.so (loaded through ctypes); there is no CPU fallback.
"""
from . import bls, layout, merkle, runtime, store, sync_protocol
from ._native import LcvError, LcvUnavailable
from .device import PackedUpdates, Verifier
from .merkle import is_valid_merkle_branch
from .sync_protocol import validate_light_client_update, validate_light_client_updates

__all__ = ["bls", "layout", "merkle", "runtime", "store", "sync_protocol", "LcvError", "LcvUnavailable", "PackedUpdates",
           "Verifier", "is_valid_merkle_branch", "validate_light_client_update", "validate_light_client_updates"]
