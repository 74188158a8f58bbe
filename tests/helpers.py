"""Test helpers: locate the libraries, and convert packed rows <-> oracle containers.

Converting a packed row back into the oracle's `LightClientUpdate` lets the CPU oracle
(oracle/sync_protocol.py, restating reference sync-protocol.md:386-465) judge exactly the bytes
the device judged.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "light-client-consensus-specs_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

HOSTSIM = os.path.join(PKG, "build", "liblcv_hostsim.so")
PRODUCT = os.path.join(PKG, "lcv", "liblcv.so")

from oracle import spec as S  # noqa: E402
from oracle import sync_protocol as O  # noqa: E402
from oracle.ssz import uint64  # noqa: E402


def ensure_hostsim() -> str:
    if not os.path.exists(HOSTSIM):
        import subprocess
        subprocess.check_call(["make", "-s", "hostsim"], cwd=PKG)
    return HOSTSIM


def hostsim_verifier():
    from lcv._native import Lib
    from lcv.device import Verifier
    return Verifier(lib=Lib(ensure_hostsim()))


def beacon_from(b: bytes) -> S.BeaconBlockHeader:
    return S.BeaconBlockHeader(slot=int.from_bytes(b[0:8], "little"), proposer_index=int.from_bytes(b[8:16], "little"),
                               parent_root=b[16:48], state_root=b[48:80], body_root=b[80:112])


def exec_from(rec: bytes) -> S.ExecutionPayloadHeader:
    elen = int.from_bytes(rec[800:804], "little")
    u = lambda k: int.from_bytes(rec[32 * k:32 * k + 8], "little")  # noqa: E731
    return S.ExecutionPayloadHeader(
        parent_hash=rec[0:32], fee_recipient=rec[32:52], state_root=rec[64:96], receipts_root=rec[96:128],
        logs_bloom=rec[544:800], prev_randao=rec[160:192], block_number=u(6), gas_limit=u(7), gas_used=u(8),
        timestamp=u(9), extra_data=rec[320:320 + elen], base_fee_per_gas=int.from_bytes(rec[352:384], "little"),
        block_hash=rec[384:416], transactions_root=rec[416:448], withdrawals_root=rec[448:480],
        blob_gas_used=u(15), excess_blob_gas=u(16))


def header_from(beacon: bytes, rec: bytes, branch: bytes) -> O.LightClientHeader:
    return O.LightClientHeader(beacon=beacon_from(beacon), execution=exec_from(rec),
                               execution_branch=[branch[32 * k:32 * k + 32] for k in range(4)])


def committee_from(sc: bytes) -> S.SyncCommittee:
    return S.SyncCommittee(pubkeys=[sc[48 * j:48 * j + 48] for j in range(512)], aggregate_pubkey=sc[512 * 48:])


def update_from(p, i: int) -> O.LightClientUpdate:
    t = lambda a: bytes(np.asarray(a[i]).tobytes())  # noqa: E731
    bits = [bool(x) for x in np.unpackbits(p.sync_bits[i], bitorder="little")]
    return O.LightClientUpdate(
        attested_header=header_from(t(p.att_beacon), t(p.att_exec), t(p.att_branch)),
        next_sync_committee=committee_from(p.nsc_pool[int(p.nsc_index[i])].tobytes()),
        next_sync_committee_branch=[t(p.nsc_branch)[32 * k:32 * k + 32] for k in range(5)],
        finalized_header=header_from(t(p.fin_beacon), t(p.fin_exec), t(p.fin_branch)),
        finality_branch=[t(p.finality_branch)[32 * k:32 * k + 32] for k in range(6)],
        sync_aggregate=S.SyncAggregate(sync_committee_bits=bits, sync_committee_signature=t(p.sync_signature)),
        signature_slot=int(p.signature_slot[i]))


def store_from(fin_slot: int, cur: bytes, nxt: bytes) -> O.LightClientStore:
    fin = O.LightClientHeader()
    fin.beacon.slot = uint64(fin_slot)
    return O.LightClientStore(finalized_header=fin, current_sync_committee=committee_from(cur),
                              next_sync_committee=committee_from(nxt), best_valid_update=None,
                              optimistic_header=O.LightClientHeader(), previous_max_active_participants=0,
                              current_max_active_participants=0)
