"""Shared driver of the store-sequence parity tests: the committed fixture
tests/golden/store_sequence.npz was produced by the reference's own exec'd
`process_light_client_update` / `process_light_client_store_force_update`
(tests/golden/make_golden.py); lcv.store must reproduce every accept flag, reason and store summary."""
import os
import sys

import numpy as np

import helpers as H

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
COLS = ("att_beacon", "att_exec", "att_branch", "fin_beacon", "fin_exec", "fin_branch", "nsc_branch",
        "finality_branch", "sync_bits", "sync_signature")


def load():
    from lcv.device import PackedUpdates
    z = np.load(os.path.join(HERE, "golden", "store_sequence.npz"))
    p = PackedUpdates(nsc_pool=z["nsc_pool"], nsc_index=z["nsc_index"], signature_slot=z["signature_slot"],
                      **{k: z[k] for k in COLS})
    return z, p


def summary(store) -> list:
    import hashlib
    from lcv import layout as L

    def dig(sc):
        return int.from_bytes(hashlib.sha256(L.pack_sync_committee(sc)).digest()[:7], "little")
    best = store.best_valid_update
    return [int(store.finalized_header.beacon.slot), int(store.optimistic_header.beacon.slot),
            -1 if best is None else int(best.signature_slot), -1 if best is None else int(best.attested_header.beacon.slot),
            dig(store.current_sync_committee), dig(store.next_sync_committee),
            int(store.previous_max_active_participants), int(store.current_max_active_participants)]


def run(verifier):
    from lcv import store as LS
    z, p = load()
    n = len(z["kinds"])
    cur, nxt = z["current_committee"].tobytes(), z["next_committee"].tobytes()
    cs, gvr = int(z["current_slot"]), z["genesis_validators_root"].tobytes()
    for case, next_known in enumerate((1, 0)):
        ups = [H.update_from(p, i) for i in range(n)]
        nb = nxt if next_known else bytes(24624)
        # one update at a time (process_light_client_update, raising on invalid updates)
        st = H.store_from(int(z["store_finalized_slot"]), cur, nb)
        for i in range(n):
            try:
                LS.process_light_client_update(st, ups[i], cs, gvr, verifier)
                ok = 1
            except AssertionError:
                ok = 0
            assert ok == z["accepted"][case][i], (case, i)
            assert summary(st) == list(z["summary"][case][i]), (case, i, summary(st), list(z["summary"][case][i]))
        # the batched form: one speculative GPU validation + re-validation after each store move
        st = H.store_from(int(z["store_finalized_slot"]), cur, nb)
        reasons: list = []
        acc = LS.process_light_client_updates(st, ups, cs, gvr, verifier, reasons)
        assert list(acc.astype(np.uint8)) == list(z["accepted"][case])
        assert reasons == list(z["reason"][case])
        assert summary(st) == list(z["summary"][case][n - 1])
        force = int(st.finalized_header.beacon.slot) + LS.config.active().UPDATE_TIMEOUT + 1
        LS.process_light_client_store_force_update(st, force)
        assert summary(st) == list(z["summary"][case][n])
