"""Store state machine (lcv.store) against the reference's own exec'd
process_light_client_update sequence (tests/golden/store_sequence.npz), validation on the host
simulation of the device code (CPU, no GPU)."""
import helpers as H
import store_cases


def test_store_sequence_matches_reference():
    store_cases.run(H.hostsim_verifier())


def test_is_better_update_prefers_supermajority_and_older_data():
    from types import SimpleNamespace as NS
    from lcv import store as LS

    def upd(n, att, sig, fin=True):
        hdr = lambda s: NS(beacon=NS(slot=s))  # noqa: E731
        return NS(sync_aggregate=NS(sync_committee_bits=[1] * n + [0] * (512 - n)), attested_header=hdr(att),
                  finalized_header=hdr(att - 10), signature_slot=sig,
                  next_sync_committee_branch=[bytes(32)] * 5,
                  finality_branch=[b"\x01" * 32] * 6 if fin else [bytes(32)] * 6)
    assert LS.is_better_update(upd(400, 100, 101), upd(300, 100, 101))      # supermajority wins
    assert not LS.is_better_update(upd(300, 100, 101), upd(400, 100, 101))
    assert LS.is_better_update(upd(200, 100, 101), upd(100, 100, 101))      # more participants below 2/3
    assert LS.is_better_update(upd(400, 100, 101), upd(400, 100, 101, False))  # finality present
    assert LS.is_better_update(upd(400, 90, 101), upd(400, 100, 101))       # older attested data
    assert LS.is_better_update(upd(400, 100, 101), upd(400, 100, 102))      # older signature slot


def test_store_refuses_config_mismatch():
    """the host-side store logic reads lcv.config.active(), the device checks the verifier's
    configuration; a verifier set to another network than the active one is refused, not half-applied."""
    import pytest
    from lcv import config
    from lcv import store as LS
    v = H.hostsim_verifier()
    v.set_config(config.TESTNET)
    with pytest.raises(ValueError, match="network configuration"):
        LS.process_light_client_updates(None, [], 0, bytes(32), verifier=v)
