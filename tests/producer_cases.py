"""Shared runner for the producer fixture (tests/golden/producer.npz, made by make_golden.py producer):
the reference's exec'd full-node.md outputs for random Deneb-shaped states and blocks."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    z = dict(np.load(os.path.join(GOLDEN, "producer.npz"), allow_pickle=False))
    meta = json.load(open(os.path.join(GOLDEN, "producer.json")))
    return z, meta["cases"]


def state_view(z, k):
    from lcv.producer import BeaconStateView
    return BeaconStateView(slot=int(z["state_slot"][k]), latest_block_header=z["state_header"][k].tobytes(),
                           finalized_checkpoint_epoch=int(z["state_fin_epoch"][k]),
                           finalized_checkpoint_root=z["state_fin_root"][k].tobytes(),
                           current_sync_committee=z["state_cur"][k].tobytes(), next_sync_committee=z["state_nxt"][k].tobytes(),
                           field_roots=z["state_roots"][k])


def block_view(z, k):
    from lcv.producer import BeaconBlockView
    return BeaconBlockView(slot=int(z["block_slot"][k]), proposer_index=int(z["block_proposer"][k]),
                           parent_root=z["block_parent"][k].tobytes(), state_root=z["block_state_root"][k].tobytes(),
                           sync_committee_bits=z["block_bits"][k].tobytes(), sync_committee_signature=z["block_sig"][k].tobytes(),
                           execution=z["block_exec"][k].tobytes(), execution_deneb=True, body_roots=z["block_roots"][k])


def expected(z, kind, i):
    o = z[f"out_{kind}_offsets"]
    return z[f"out_{kind}"][int(o[i]):int(o[i + 1])].tobytes()


def produce(z, case):
    """Run lcv.producer on one fixture case: (update, finality, optimistic, bootstrap) rows."""
    from lcv import producer as PR
    fb = block_view(z, case["finalized_block"]) if case["finalized_block"] >= 0 else None
    upd = PR.create_light_client_update(state_view(z, case["state"]), block_view(z, case["block"]),
                                        state_view(z, case["attested_state"]), block_view(z, case["attested_block"]), fb)
    boot = PR.create_light_client_bootstrap(state_view(z, case["attested_state"]), block_view(z, case["attested_block"]))
    return upd, PR.create_light_client_finality_update(upd), PR.create_light_client_optimistic_update(upd), boot
