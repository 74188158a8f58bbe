"""GPU: liblcv.so on the MI355X against the golden fixtures (reference-exec'd expected reasons)."""
import numpy as np
import pytest

import golden_cases as G

pytestmark = pytest.mark.gpu


def test_update_cases_gpu(engine_verifier):
    got, exp = G.run_update_cases(engine_verifier)
    assert list(got) == list(exp)


def test_testnet_config_gpu(engine_verifier):
    """lcv_set_config on the device: non-mainnet fork versions / epochs (reference-exec'd reasons)."""
    got_t, exp_t, got_m, exp_m = G.run_testnet_cases(engine_verifier)
    assert list(got_t) == list(exp_t)
    assert list(got_m) == list(exp_m)


def test_bls_vectors_gpu(engine_verifier):
    b = G.load_bls()
    out, inf = engine_verifier.debug_hash_to_g2(b["h2c_msg"])
    assert np.array_equal(out, b["h2c_out"]) and not inf.any()
    _, st = engine_verifier.debug_g2_decompress(b["sig"])
    assert list(st) == list(b["sig_status"])
    pks = [b["fav_pks"][k].tobytes() for k in range(3)]
    m, s = b["fav_msg"].tobytes(), b["fav_sig"].tobytes()
    assert engine_verifier.fast_aggregate_verify(pks, m, s)
    assert not engine_verifier.fast_aggregate_verify(pks[:2], m, s)
    assert not engine_verifier.fast_aggregate_verify(pks + [bytes([0xC0]) + bytes(47)], m, s)
