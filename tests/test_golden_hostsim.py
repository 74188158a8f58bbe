"""CPU: the device per-item code (host-simulation build) against the golden fixtures, whose expected
reasons come from exec'ing the reference's own sync-protocol.md blocks (and the oracle)."""
import json
import os

import numpy as np

import golden_cases as G


def test_fixture_covers_every_assert():
    meta = json.load(open(os.path.join(G.GOLDEN, "lc_updates.json")))
    assert set(meta["expected_reason"]) == set(range(15))  # valid + each of the 14 asserts


def test_update_cases_hostsim(sim_verifier):
    got, exp = G.run_update_cases(sim_verifier)
    assert list(got) == list(exp)


def test_bls_vectors_hostsim(sim_verifier):
    b = G.load_bls()
    out, inf = sim_verifier.debug_hash_to_g2(b["h2c_msg"])
    assert np.array_equal(out, b["h2c_out"]) and not inf.any()
    pts, st = sim_verifier.debug_g2_decompress(b["sig"])
    assert list(st) == list(b["sig_status"])
    pks = [b["fav_pks"][k].tobytes() for k in range(3)]
    m, s = b["fav_msg"].tobytes(), b["fav_sig"].tobytes()
    assert sim_verifier.fast_aggregate_verify(pks, m, s)
    assert not sim_verifier.fast_aggregate_verify(pks[:2], m, s)
    assert not sim_verifier.fast_aggregate_verify(pks + [bytes([0xC0]) + bytes(47)], m, s)


def test_testnet_config_hostsim(sim_verifier):
    """lcv_set_config: the same rows are valid under the configuration they were signed under and
    fail (signing domain / header fork rules) under mainnet, as the reference's exec'd blocks say."""
    got_t, exp_t, got_m, exp_m = G.run_testnet_cases(sim_verifier)
    assert list(got_t) == list(exp_t)
    assert list(got_m) == list(exp_m)
    assert list(exp_t) != list(exp_m)


def test_config_validation(sim_verifier):
    import pytest
    from lcv._native import LcvError
    from lcv.config import MAINNET, NetworkConfig
    with pytest.raises(ValueError):
        NetworkConfig(CAPELLA_FORK_EPOCH=10, BELLATRIX_FORK_EPOCH=20)
    bad = MAINNET.with_(name="x")
    object.__setattr__(bad, "DENEB_FORK_EPOCH", 5)  # bypass the dataclass check: the C ABI checks too
    with pytest.raises(LcvError):
        sim_verifier.set_config(bad)
    assert MAINNET.compute_fork_version(MAINNET.DENEB_FORK_EPOCH) == bytes.fromhex("04000000")
    assert MAINNET.compute_fork_version(MAINNET.CAPELLA_FORK_EPOCH - 1) == bytes.fromhex("02000000")
    assert MAINNET.UPDATE_TIMEOUT == 8192
