"""The fused G2 membership check on its exceptional path: signatures that decode to
E2 points of small cofactor orders, G2 + torsion sums and the order-13 point whose |x| walk meets T = -Q
(tests/g2_edge_points.py) are rejected — through lcv_debug_g2_decompress (status 2, as the oracle's
r * P == O test says) and through lcv_validate_updates (reason 14, the signature assert at
sync-protocol.md:464, as the oracle's FastAggregateVerify says) — on the host simulation of the kernel
code (CPU) and on the MI355X."""
import numpy as np
import pytest

import g2_edge_points as E
import helpers as H
from oracle import bls12_381 as B


def _status(sig: bytes) -> int:
    try:
        pt = B.g2_decompress(sig)
    except B.DecodeError:
        return 2
    if pt is None:
        return 1
    return 0 if B.g2_in_subgroup(pt) else 2


def check_g2_edge(v):
    from lcv import synth
    sigs = E.edge_signatures()
    names = list(sigs)
    good = B.g2_compress(B.g2_mul(B.G2_GEN, 987654321))
    allsig = [sigs[k] for k in names] + [good]
    _, st = v.debug_g2_decompress(np.frombuffer(b"".join(allsig), np.uint8))
    want = [_status(s) for s in allsig]
    assert want == [2] * len(names) + [0]
    assert [int(x) for x in st] == want, dict(zip(names + ["g2"], [int(x) for x in st]))
    # the same signatures inside full updates: every other check passes, the signature assert fails
    n = len(names) + 2
    sb = synth.generate(v, n, seed=41)
    v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    u = sb.updates
    for i, k in enumerate(names):
        u.sync_signature[i] = np.frombuffer(sigs[k], np.uint8)
    ok, reason = v.validate(u, sb.current_slot, sb.genesis_validators_root)
    store = H.store_from(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    exp = [H.O.validate_light_client_update(store, H.update_from(u, i), sb.current_slot, sb.genesis_validators_root)
           for i in range(n)]
    assert exp == [14] * len(names) + [0, 0]
    assert [int(r) for r in reason] == exp
    assert list(ok) == [e == 0 for e in exp]


def test_g2_edge_hostsim(sim_verifier):
    check_g2_edge(sim_verifier)


@pytest.mark.gpu
def test_g2_edge_gpu(gpu_verifier):
    check_g2_edge(gpu_verifier)
