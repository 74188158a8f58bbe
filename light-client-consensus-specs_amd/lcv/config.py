"""Network configuration of the light-client path (the consensus-specs preset / config values that
sync-protocol.md reads), applied at run time instead of being compiled into the kernels.

    SLOTS_PER_EPOCH, EPOCHS_PER_SYNC_COMMITTEE_PERIOD   periods, UPDATE_TIMEOUT (sync-protocol.md:89)
    ALTAIR / BELLATRIX / CAPELLA / DENEB _FORK_EPOCH    is_valid_light_client_header (:220-240),
                                                        get_lc_execution_root (:186-214),
                                                        compute_fork_version (:461)
    GENESIS .. DENEB _FORK_VERSION                      compute_fork_version (:461)
    DOMAIN_SYNC_COMMITTEE                               compute_domain (:462)

`active()` is the process-wide configuration (as the pyspec's module-level config is): the store state
machine and the synthetic producer read it, and `runtime.default_verifier()` applies it to its device
context.  A `Verifier` carries its own copy (`Verifier.set_config`).  SYNC_COMMITTEE_SIZE is fixed at the
mainnet preset's 512 (the packed layouts of include/lcv.h).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, replace
from typing import Tuple


@dataclass(frozen=True)
class NetworkConfig:
    name: str = "mainnet"
    SLOTS_PER_EPOCH: int = 32
    EPOCHS_PER_SYNC_COMMITTEE_PERIOD: int = 256
    ALTAIR_FORK_EPOCH: int = 74240
    BELLATRIX_FORK_EPOCH: int = 144896
    CAPELLA_FORK_EPOCH: int = 194048
    DENEB_FORK_EPOCH: int = 269568
    GENESIS_FORK_VERSION: bytes = bytes.fromhex("00000000")
    ALTAIR_FORK_VERSION: bytes = bytes.fromhex("01000000")
    BELLATRIX_FORK_VERSION: bytes = bytes.fromhex("02000000")
    CAPELLA_FORK_VERSION: bytes = bytes.fromhex("03000000")
    DENEB_FORK_VERSION: bytes = bytes.fromhex("04000000")
    DOMAIN_SYNC_COMMITTEE: bytes = bytes.fromhex("07000000")

    def __post_init__(self):
        if self.SLOTS_PER_EPOCH < 1 or self.EPOCHS_PER_SYNC_COMMITTEE_PERIOD < 1:
            raise ValueError("SLOTS_PER_EPOCH and EPOCHS_PER_SYNC_COMMITTEE_PERIOD must be >= 1")
        e = self.fork_epochs()
        if any(e[k] > e[k + 1] for k in range(3)):
            raise ValueError("fork epochs must be non-decreasing (altair <= bellatrix <= capella <= deneb)")
        if any(len(v) != 4 for v in self.fork_versions()) or len(self.DOMAIN_SYNC_COMMITTEE) != 4:
            raise ValueError("fork versions and DOMAIN_SYNC_COMMITTEE are 4 bytes")

    # --------------------------------------------------------------- derived
    @property
    def SLOTS_PER_PERIOD(self) -> int:
        return self.SLOTS_PER_EPOCH * self.EPOCHS_PER_SYNC_COMMITTEE_PERIOD

    @property
    def UPDATE_TIMEOUT(self) -> int:  # sync-protocol.md:89
        return self.SLOTS_PER_PERIOD

    def fork_epochs(self) -> Tuple[int, int, int, int]:
        return (self.ALTAIR_FORK_EPOCH, self.BELLATRIX_FORK_EPOCH, self.CAPELLA_FORK_EPOCH, self.DENEB_FORK_EPOCH)

    def fork_versions(self) -> Tuple[bytes, ...]:
        return (self.GENESIS_FORK_VERSION, self.ALTAIR_FORK_VERSION, self.BELLATRIX_FORK_VERSION,
                self.CAPELLA_FORK_VERSION, self.DENEB_FORK_VERSION)

    def compute_epoch_at_slot(self, slot: int) -> int:
        return int(slot) // self.SLOTS_PER_EPOCH

    def compute_sync_committee_period_at_slot(self, slot: int) -> int:
        return int(slot) // self.SLOTS_PER_PERIOD

    def compute_fork_version(self, epoch: int) -> bytes:
        v = self.GENESIS_FORK_VERSION
        for e, ver in zip(self.fork_epochs(), self.fork_versions()[1:]):
            if int(epoch) >= e:
                v = ver
        return v

    def with_(self, **kw) -> "NetworkConfig":
        return replace(self, **kw)


MAINNET = NetworkConfig()

# A non-mainnet configuration for tests and examples: a Sepolia-style testnet (its own fork versions
# and fork epochs; the values are this repository's test choice, not a statement about any network).
TESTNET = NetworkConfig(name="testnet", ALTAIR_FORK_EPOCH=50, BELLATRIX_FORK_EPOCH=100, CAPELLA_FORK_EPOCH=56832,
                        DENEB_FORK_EPOCH=132608, GENESIS_FORK_VERSION=bytes.fromhex("90000069"),
                        ALTAIR_FORK_VERSION=bytes.fromhex("90000070"),
                        BELLATRIX_FORK_VERSION=bytes.fromhex("90000071"),
                        CAPELLA_FORK_VERSION=bytes.fromhex("90000072"),
                        DENEB_FORK_VERSION=bytes.fromhex("90000073"))

_lock = threading.Lock()
_active = MAINNET


def active() -> NetworkConfig:
    return _active


def set_active(cfg: NetworkConfig) -> None:
    """Make `cfg` the process-wide configuration (and apply it to the default device context, if open)."""
    global _active
    if not isinstance(cfg, NetworkConfig):
        raise TypeError("cfg must be a NetworkConfig")
    with _lock:
        _active = cfg
    from . import runtime
    v = runtime.current_default()
    if v is not None:
        v.set_config(cfg)
