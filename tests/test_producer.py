"""Producer side (full-node.md): lcv.producer over sparse state / block views
reproduces, byte for byte, the light-client data the reference's own exec'd full-node.md functions
derive from the full Deneb-shaped objects (tests/golden/producer.npz), and the derived updates pass
validation (host simulation of the device code here; the MI355X in test_producer_gpu)."""
import numpy as np
import pytest

import producer_cases as PC


def test_producer_bytes_match_reference():
    from lcv import wire
    from lcv.producer import pack_updates
    z, cases = PC.load()
    for i, c in enumerate(cases):
        upd, fu, ou, boot = PC.produce(z, c)
        assert wire.encode_updates(pack_updates([upd]), "update")[0] == PC.expected(z, "update", i), c["name"]
        assert wire.encode_updates(pack_updates([fu]), "finality")[0] == PC.expected(z, "finality", i), c["name"]
        assert wire.encode_updates(pack_updates([ou]), "optimistic")[0] == PC.expected(z, "optimistic", i), c["name"]
        h = boot.header
        got = wire.encode_bootstrap(h.beacon, h.execution, h.execution_branch, boot.current_sync_committee,
                                    boot.current_sync_committee_branch)
        assert got == PC.expected(z, "bootstrap", i), c["name"]


def test_producer_asserts():
    """The reference's asserts: a block whose parent is not the attested block, a state whose header
    does not match its block, a sync aggregate with no participants."""
    from dataclasses import replace
    from lcv import producer as PR
    z, cases = PC.load()
    c = cases[0]
    st, blk = PC.state_view(z, c["state"]), PC.block_view(z, c["block"])
    ast, ablk = PC.state_view(z, c["attested_state"]), PC.block_view(z, c["attested_block"])
    fb = PC.block_view(z, c["finalized_block"])
    with pytest.raises(AssertionError):
        PR.create_light_client_update(st, replace(blk, parent_root=bytes(32)), ast, ablk, fb)
    with pytest.raises(AssertionError):
        PR.create_light_client_update(st, blk, ast, replace(ablk, proposer_index=ablk.proposer_index + 1), fb)
    with pytest.raises(AssertionError):
        PR.create_light_client_update(st, replace(blk, sync_committee_bits=bytes(64)), ast, ablk, fb)
    with pytest.raises(AssertionError):
        PR.create_light_client_bootstrap(ast, blk)


def _validate(v, z, cases):
    from lcv.producer import pack_updates
    cur, nxt = z["current_committee"].tobytes(), z["next_committee"].tobytes()
    gvr = z["genesis_validators_root"].tobytes()
    out = []
    for c in cases:
        upd = PC.produce(z, c)[0]
        v.set_store(c["store_finalized_slot"], cur, nxt)
        ok, reason = v.validate(pack_updates([upd]), c["current_slot"], gvr)
        out.append(int(reason[0]))
    return out


def test_produced_updates_validate_hostsim(sim_verifier):
    z, cases = PC.load()
    assert _validate(sim_verifier, z, cases) == [c["reason"] for c in cases]


@pytest.mark.gpu
def test_produced_updates_validate_gpu(engine_verifier):
    z, cases = PC.load()
    assert _validate(engine_verifier, z, cases) == [c["reason"] for c in cases]
