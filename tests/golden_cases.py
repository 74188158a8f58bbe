"""Shared runner for the committed golden fixtures (tests/golden/*.npz, made by make_golden.py)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
COLS = ("att_beacon", "att_exec", "att_branch", "fin_beacon", "fin_exec", "fin_branch", "nsc_branch",
        "finality_branch", "sync_bits", "sync_signature")


def load_updates(name="lc_updates"):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def testnet_config():
    """The non-mainnet NetworkConfig the testnet fixture was made under (values from its JSON)."""
    import json
    from lcv.config import NetworkConfig
    c = json.load(open(os.path.join(GOLDEN, "lc_updates_testnet.json")))["config"]
    return NetworkConfig(**{k: (bytes.fromhex(v) if isinstance(v, str) and k != "name" else v) for k, v in c.items()})


def load_bls():
    return dict(np.load(os.path.join(GOLDEN, "bls_vectors.npz"), allow_pickle=False))


def run_update_cases(verifier, name="lc_updates", expected="expected_reason"):
    """Validate every golden case through the C ABI, grouped by (store snapshot, current_slot);
    returns the device reason codes in case order."""
    from lcv.device import PackedUpdates
    g = load_updates(name)
    n = len(g[expected])
    gvr = g["genesis_validators_root"].tobytes()
    cur, nxt, zero = (g["nsc_pool"][k].tobytes() for k in range(3))
    out = np.full(n, 255, np.uint8)
    keys = sorted({(int(g["store_finalized_slot"][i]), int(g["store_next_known"][i]), int(g["current_slot"][i]))
                   for i in range(n)})
    for fin, nk, cs in keys:
        rows = [i for i in range(n) if (int(g["store_finalized_slot"][i]), int(g["store_next_known"][i]),
                                        int(g["current_slot"][i])) == (fin, nk, cs)]
        verifier.set_store(fin, cur, nxt if nk else zero)
        p = PackedUpdates(nsc_pool=g["nsc_pool"], nsc_index=g["nsc_index"][rows].copy(),
                          signature_slot=g["signature_slot"][rows].copy(),
                          **{k: np.ascontiguousarray(g[k][rows]) for k in COLS})
        ok, reason = verifier.validate(p, cs, gvr)
        assert np.array_equal(ok, reason == 0)
        out[rows] = reason
    return out, g[expected]


def run_testnet_cases(verifier):
    """The testnet fixture under its own configuration, then under mainnet (the configuration is
    restored to mainnet afterwards): (got_testnet, expected_testnet, got_mainnet, expected_mainnet)."""
    from lcv.config import MAINNET
    verifier.set_config(testnet_config())
    try:
        got_t, exp_t = run_update_cases(verifier, "lc_updates_testnet", "expected_reason_testnet")
    finally:
        verifier.set_config(MAINNET)
    got_m, exp_m = run_update_cases(verifier, "lc_updates_testnet", "expected_reason_mainnet")
    return got_t, exp_t, got_m, exp_m
