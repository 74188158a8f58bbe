"""Shared runner for the committed golden fixtures (tests/golden/*.npz, made by make_golden.py)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
COLS = ("att_beacon", "att_exec", "att_branch", "fin_beacon", "fin_exec", "fin_branch", "nsc_branch",
        "finality_branch", "sync_bits", "sync_signature")


def load_updates():
    return dict(np.load(os.path.join(GOLDEN, "lc_updates.npz"), allow_pickle=False))


def load_bls():
    return dict(np.load(os.path.join(GOLDEN, "bls_vectors.npz"), allow_pickle=False))


def run_update_cases(verifier):
    """Validate every golden case through the C ABI, grouped by (store snapshot, current_slot);
    returns the device reason codes in case order."""
    from lcv.device import PackedUpdates
    g = load_updates()
    n = len(g["expected_reason"])
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
    return out, g["expected_reason"]
