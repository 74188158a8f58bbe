"""Two batches in flight on the MI355X (lcv_validate_resident_async / lcv_slot_wait): each slot's
verdicts and reasons equal the synchronous call's and the rows' construction."""
import numpy as np
import pytest

from test_pipeline_hostsim import check_async_slots, check_host_async

pytestmark = pytest.mark.gpu


def test_async_slots_gpu(gpu_verifier):
    check_async_slots(gpu_verifier)


def test_host_async_gpu(gpu_verifier):
    """lcv_validate_async (pinned staging, DMA upload, pinned verdicts) on eight slots, plus the bounded
    stage-timing event pool under 50 asynchronous batches."""
    v = gpu_verifier
    check_host_async(v, cycles=3)
    from test_pipeline_hostsim import _two_batches
    a, _ = _two_batches(v, 64)
    v.set_store(a.store_finalized_slot, a.current.ssz, a.next.ssz)
    rb = v.upload(a.updates)
    before = v.event_pool()
    for k in range(50):
        v.validate_resident_async(rb, a.current_slot, a.genesis_validators_root, k % 8)
        if k >= 7:
            v.slot_wait((k + 1) % 8, a.updates.n)
    for s in range(8):
        v.slot_wait(s, a.updates.n)
    assert v.event_pool() == before


def test_async_slots_full_batches_gpu(gpu_verifier):
    """configs[1]-sized batches (10^4 rows each, 10% adversarial), alternated over the two slots four
    times with the host waiting for a slot only before reusing it, as bench.py's serving loop does."""
    from lcv import synth
    v = gpu_verifier
    n = 10000
    bs = [synth.generate(v, n, seed=s, participation="random",
                         kinds=synth.adversarial_kinds(n, seed=s, bad_fraction=0.10)) for s in (21, 22)]
    v.set_store(bs[0].store_finalized_slot, bs[0].current.ssz, bs[0].next.ssz)
    rbs = [v.upload(b.updates) for b in bs]
    for k in range(4):
        s = k % 2
        if k >= 2:
            _, r = v.slot_wait(s, n)
            assert np.array_equal(r, bs[s].expected_reason)
        v.validate_resident_async(rbs[s], bs[s].current_slot, bs[s].genesis_validators_root, s)
    for s in (0, 1):
        ok, r = v.slot_wait(s, n)
        assert np.array_equal(r, bs[s].expected_reason) and np.array_equal(ok.astype(bool), r == 0)
