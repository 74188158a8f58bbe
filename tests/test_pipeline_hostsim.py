"""The slice pipeline of validate (lcv_set_pipeline) on the host simulation: the slicing of the batch
and of the work space (work_view) must not change any verdict or reason (CPU, no GPU)."""
import copy

import numpy as np
import pytest

import helpers as H


def test_slices_match_serial():
    from lcv import synth
    v = H.hostsim_verifier()
    n = 300  # 3 slices of 128 (whole waves): the last one ragged
    kinds = synth.adversarial_kinds(n, seed=9, bad_fraction=0.2)
    sb = synth.generate(v, n, seed=9, participation="random", kinds=kinds)
    v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    v.set_pipeline(1, 1)
    ok1, r1 = v.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    assert np.array_equal(r1, sb.expected_reason)
    v.set_pipeline(4, 2)
    ok2, r2 = v.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    assert np.array_equal(r2, r1) and np.array_equal(ok2, ok1)


def test_set_pipeline_rejects_bad_shapes():
    from lcv._native import LcvError
    v = H.hostsim_verifier()
    with pytest.raises(LcvError):
        v.set_pipeline(0, 1)
    with pytest.raises(LcvError):
        v.set_pipeline(2, 0)


def _two_batches(v, n=96):
    from lcv import synth
    kinds = synth.adversarial_kinds(n, seed=4, bad_fraction=0.25)
    a = synth.generate(v, n, seed=4, participation="random", kinds=kinds)
    b = synth.generate(v, n, seed=5, participation="random", kinds=synth.adversarial_kinds(n, seed=5, bad_fraction=0.25))
    return a, b


def check_async_slots(v):
    """lcv_validate_resident_async / lcv_slot_wait: two batches in flight on slots 0 and 1, reused
    twice each; every batch's verdicts and reasons equal the synchronous call's and its construction."""
    a, b = _two_batches(v)
    v.set_store(a.store_finalized_slot, a.current.ssz, a.next.ssz)
    ra, rb = v.upload(a.updates), v.upload(b.updates)
    sync_a = v.validate_resident(ra, a.current_slot, a.genesis_validators_root)
    assert np.array_equal(sync_a[1], a.expected_reason)
    for rep in range(2):
        v.validate_resident_async(ra, a.current_slot, a.genesis_validators_root, 0)
        v.validate_resident_async(rb, b.current_slot, b.genesis_validators_root, 1)
        va, za = v.slot_wait(0, len(a.expected_reason))
        vb, zb = v.slot_wait(1, len(b.expected_reason))
        assert np.array_equal(za, a.expected_reason) and np.array_equal(va, sync_a[0])
        assert np.array_equal(zb, b.expected_reason) and np.array_equal(vb.astype(bool), zb == 0)
    # eight batches in flight: every slot of the context, a and b alternating
    for s in range(8):
        x = (a, ra) if s % 2 == 0 else (b, rb)
        v.validate_resident_async(x[1], x[0].current_slot, x[0].genesis_validators_root, s)
    for s in range(8):
        exp = a.expected_reason if s % 2 == 0 else b.expected_reason
        assert np.array_equal(v.slot_wait(s, len(exp))[1], exp)
    # a synchronous call after async ones still uses slot 0 and agrees
    again = v.validate_resident(ra, a.current_slot, a.genesis_validators_root)
    assert np.array_equal(again[1], sync_a[1])


def check_host_async(v, cycles=3):
    """lcv_validate_async (host batch in, verdicts out, eight in flight): every batch's verdicts and
    reasons equal its construction and the synchronous call's; the caller's arrays are reusable when the
    call returns (overwritten before the slot is waited for); mixing with resident async calls on the
    same slot keeps each call's results; the stage-timing event pool stays bounded."""
    a, b = _two_batches(v)
    v.set_store(a.store_finalized_slot, a.current.ssz, a.next.ssz)
    sync_a = v.validate(a.updates, a.current_slot, a.genesis_validators_root)
    pool0 = v.event_pool()
    for rep in range(cycles):
        for s in range(8):
            x = a if (s + rep) % 2 == 0 else b
            if rep == 1 and s == 3:  # the call copied the batch: clobbering the caller's arrays is harmless
                tmp = copy.deepcopy(x.updates)
                v.validate_async(tmp, x.current_slot, x.genesis_validators_root, s)
                tmp.sync_signature[:] = 0
                tmp.att_beacon[:] = 0xFF
            else:
                v.validate_async(x.updates, x.current_slot, x.genesis_validators_root, s)
        for s in range(8):
            x = a if (s + rep) % 2 == 0 else b
            ok, r = v.slot_wait(s, x.updates.n)
            assert np.array_equal(r, x.expected_reason) and np.array_equal(ok.astype(bool), r == 0)
            if x is a:
                assert np.array_equal(r, sync_a[1])
    # a resident async batch on a slot after a host-input one (and back) reports its own results
    rb = v.upload(b.updates)
    v.validate_async(a.updates, a.current_slot, a.genesis_validators_root, 2)
    assert np.array_equal(v.slot_wait(2, a.updates.n)[1], a.expected_reason)
    v.validate_resident_async(rb, b.current_slot, b.genesis_validators_root, 2)
    assert np.array_equal(v.slot_wait(2, b.updates.n)[1], b.expected_reason)
    v.validate_async(a.updates, a.current_slot, a.genesis_validators_root, 2)
    assert np.array_equal(v.slot_wait(2, a.updates.n)[1], a.expected_reason)
    # asynchronous calls take no stage-timing events (the pool grew ~24 events per batch)
    assert v.event_pool() <= max(pool0, 64)


def test_async_slots_hostsim():
    check_async_slots(H.hostsim_verifier())


def test_host_async_hostsim():
    check_host_async(H.hostsim_verifier(), cycles=2)


def test_async_rejects_bad_slot():
    from lcv._native import LcvError
    v = H.hostsim_verifier()
    a, _ = _two_batches(v, 8)
    v.set_store(a.store_finalized_slot, a.current.ssz, a.next.ssz)
    ra = v.upload(a.updates)
    with pytest.raises(LcvError):
        v.validate_resident_async(ra, a.current_slot, a.genesis_validators_root, 8)
    with pytest.raises(LcvError):
        v.slot_wait(1, 10 ** 6)


def test_chunks_rotate_over_slots_hostsim():
    """A batch of several chunks (64-row chunks here, 65,536 in production): chunks rotate over the eight
    work-space slots, each slot's first chunk hashing the committee pool; every verdict and reason equals
    the one-chunk call's and the construction (ragged last chunk, more chunks than slots)."""
    import ctypes as C
    from lcv import synth
    v = H.hostsim_verifier()
    n = 64 * 10 + 17
    kinds = synth.adversarial_kinds(n, seed=12, bad_fraction=0.2)
    sb = synth.generate(v, n, seed=12, participation="random", kinds=kinds, npool=3)
    v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    ok1, r1 = v.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    assert np.array_equal(r1, sb.expected_reason)
    v._check(v.lib.lcv_debug_set_chunk(v.ctx, C.c_uint64(64)), "lcv_debug_set_chunk")
    try:
        ok2, r2 = v.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
        rb = v.upload(sb.updates)
        ok3, r3 = v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root)
    finally:
        v._check(v.lib.lcv_debug_set_chunk(v.ctx, C.c_uint64(65536)), "lcv_debug_set_chunk")
    assert np.array_equal(r2, r1) and np.array_equal(ok2, ok1)
    assert np.array_equal(r3, r1) and np.array_equal(ok3.astype(bool), ok1)
