"""The slice pipeline of validate (lcv_set_pipeline) on the host simulation: the slicing of the batch
and of the work space (work_view) must not change any verdict or reason (CPU, no GPU)."""
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
