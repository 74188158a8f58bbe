"""SSZ wire decode (lcv.wire, csrc/lcv_wire.cpp) and the bootstrap checks (lcv_bootstrap_check_batch).

Fixtures: tests/golden/wire.npz — SSZ bytes serialised by the reference's OWN exec'd containers
(sync-protocol.md:109-160) from the golden update rows, and bootstraps whose expected reason is the
failing assert of the reference's exec'd initialize_light_client_store (:351-373); made by
tests/golden/make_golden.py wire.  The decoder is host code, so the CPU tests run the real decoder of
both libraries (host simulation and, when built, the product liblcv.so); the device bootstrap check
runs on the host simulation here and on the MI355X in the gpu test.
"""
import os

import numpy as np
import pytest

import helpers as H
from golden_cases import COLS, GOLDEN, load_updates

from lcv import layout as L
from lcv import wire
from lcv._native import Lib
from oracle import spec as S
from oracle import sync_protocol as O
from oracle.ssz import Container, serialize


def load_wire():
    return dict(np.load(os.path.join(GOLDEN, "wire.npz"), allow_pickle=False))


def libs():
    out = [Lib(H.ensure_hostsim())]
    if os.path.exists(H.PRODUCT):
        out.append(Lib(H.PRODUCT))
    return out


def expected_rows(g, rows, kind):
    """Golden packed rows as the reference converts them for finality / optimistic updates
    (sync-protocol.md:563-571, :582-590)."""
    exp = {k: g[k][rows].copy() for k in COLS}
    committees = g["nsc_pool"][g["nsc_index"][rows]].copy()
    if kind >= 1:
        exp["nsc_branch"][:] = 0
        committees[:] = 0
    if kind == 2:
        for k in ("fin_beacon", "fin_exec", "fin_branch", "finality_branch"):
            exp[k][:] = 0
    return exp, committees


def messages(w, sel):
    return [w["buf"][int(w["offsets"][i]):int(w["offsets"][i] + w["lengths"][i])].tobytes() for i in sel]


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_decode_reference_wire_bytes(kind):
    w, g = load_wire(), load_updates()
    sel = np.flatnonzero(w["kind"] == kind)
    rows = w["row"][sel]
    exp, committees = expected_rows(g, rows, kind)
    for lib in libs():
        batch = wire.decode_updates(messages(w, sel), kind=["update", "finality", "optimistic"][kind], lib=lib)
        for k in COLS:
            assert np.array_equal(getattr(batch, k), exp[k]), k
        assert np.array_equal(batch.signature_slot, g["signature_slot"][rows])
        assert np.array_equal(batch.nsc_pool[batch.nsc_index], committees)
        batch.check()


def test_decode_from_one_buffer_and_dedup():
    """(buf, offsets, lengths) input; repeated committees are pooled once, SyncCommittee() once."""
    w = load_wire()
    sel = np.flatnonzero(w["kind"] == 0)
    msgs = messages(w, sel) * 5
    buf = np.frombuffer(b"".join(msgs), np.uint8)
    lens = np.array([len(m) for m in msgs], np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    batch = wire.decode_updates((buf, offs, lens), lib=libs()[0])
    distinct = {bytes(r) for r in batch.nsc_pool[batch.nsc_index]}
    assert batch.nsc_pool.shape[0] == len(distinct) <= 3
    assert batch.n == len(msgs)


def test_malformed_messages_rejected():
    w = load_wire()
    full = messages(w, [int(np.flatnonzero(w["kind"] == 0)[0])])[0]
    fin = messages(w, [int(np.flatnonzero(w["kind"] == 1)[0])])[0]

    def with_u32(b, pos, v):
        return b[:pos] + int(v).to_bytes(4, "little") + b[pos + 4:]
    fixed_off = int.from_bytes(fin[0:4], "little")
    bad = [b"", fin[:100], with_u32(fin, 0, 369), with_u32(fin, 4, 300),  # truncated / first offset / order
           with_u32(fin, 4, len(fin) + 1), fin + bytes(33),                  # out of bounds / extra_data > 32
           full[:25151]]
    cases = [fin] + bad[:-1]
    for lib in libs():
        batch, ok = wire.decode_updates_status(cases, kind="finality", lib=lib)
        assert ok.tolist() == [True] + [False] * (len(cases) - 1)
        assert not batch.att_beacon[1:].any() and not batch.sync_signature[1:].any()
        _, ok = wire.decode_updates_status([full, bad[-1]], kind="update", lib=lib)
        assert ok.tolist() == [True, False]
        with pytest.raises(ValueError):
            wire.decode_updates(cases, kind="finality", lib=lib)
    assert fixed_off == 368


class CapellaHeader(Container):
    beacon: S.BeaconBlockHeader
    execution: S.CapellaExecutionPayloadHeader
    execution_branch: S.ExecutionBranch


class CapellaUpdate(Container):
    attested_header: CapellaHeader
    next_sync_committee: S.SyncCommittee
    next_sync_committee_branch: S.NextSyncCommitteeBranch
    finalized_header: CapellaHeader
    finality_branch: S.FinalityBranch
    sync_aggregate: S.SyncAggregate
    signature_slot: S.Slot


def test_decode_capella_wire():
    g = load_updates()
    from lcv.device import PackedUpdates
    p = PackedUpdates(nsc_pool=g["nsc_pool"], nsc_index=g["nsc_index"], signature_slot=g["signature_slot"],
                      **{k: g[k] for k in COLS})
    rows = [28, 30]  # capella_valid, bellatrix_valid (no blob gas fields)

    def cap(h):
        e = h.execution
        ce = S.CapellaExecutionPayloadHeader(**{n: getattr(e, n) for n, _ in S.CapellaExecutionPayloadHeader._fields})
        return CapellaHeader(beacon=h.beacon, execution=ce, execution_branch=h.execution_branch)
    msgs = []
    for i in rows:
        u = H.update_from(p, i)
        msgs.append(serialize(CapellaUpdate(attested_header=cap(u.attested_header), next_sync_committee=u.next_sync_committee,
                                            next_sync_committee_branch=u.next_sync_committee_branch,
                                            finalized_header=cap(u.finalized_header), finality_branch=u.finality_branch,
                                            sync_aggregate=u.sync_aggregate, signature_slot=u.signature_slot)))
    exp, committees = expected_rows(g, np.array(rows), 0)
    for lib in libs():
        batch = wire.decode_updates(msgs, fork="capella", lib=lib)
        for k in COLS:
            assert np.array_equal(getattr(batch, k), exp[k]), k
        assert np.array_equal(batch.nsc_pool[batch.nsc_index], committees)
        # a Capella message is malformed under the Deneb layout (17-field fixed part)
        _, ok = wire.decode_updates_status(msgs, fork="deneb", lib=lib)
        assert not ok.any()


class Bootstrap(Container):
    header: O.LightClientHeader
    current_sync_committee: S.SyncCommittee
    current_sync_committee_branch: S.CurrentSyncCommitteeBranch


def boots(w):
    return [w["boot_buf"][int(o):int(o + n)].tobytes() for o, n in zip(w["boot_offsets"], w["boot_lengths"])]


def test_decode_bootstrap_matches_oracle_deserialisation():
    w = load_wire()
    for lib in libs():
        for b in boots(w):
            d = wire.decode_bootstrap(b, lib=lib)
            o = Bootstrap.de(b)
            beacon, execution, branch = L.pack_header(o.header)
            assert d.beacon.tobytes() == beacon and d.execution.tobytes() == execution
            assert d.execution_branch.tobytes() == branch
            assert d.current_sync_committee.tobytes() == L.pack_sync_committee(o.current_sync_committee)
            assert d.current_sync_committee_branch.tobytes() == L.pack_branch(o.current_sync_committee_branch, 5)
            with pytest.raises(ValueError):
                wire.decode_bootstrap(b[:-1] if len(b) == 24788 + 244 + 584 else b[:200], lib=lib)


def run_bootstrap_cases(v):
    w = load_wire()
    ds = [wire.decode_bootstrap(b, lib=v.lib) for b in boots(w)]
    st = lambda name: np.stack([getattr(d, name) for d in ds])  # noqa: E731
    got = v.bootstrap_check_batch(st("beacon"), st("execution"), st("execution_branch"), st("current_sync_committee"),
                                  st("current_sync_committee_branch"), w["boot_trusted"])
    return got, w["boot_reason"], ds, w


def test_bootstrap_checks_hostsim_match_reference():
    got, exp, _, _ = run_bootstrap_cases(H.hostsim_verifier())
    assert got.tolist() == exp.tolist()


def test_initialize_light_client_store_hostsim():
    from lcv.store import initialize_light_client_store
    v = H.hostsim_verifier()
    w = load_wire()
    bs = [Bootstrap.de(b) for b in boots(w)]
    for b, trusted, r in zip(bs, w["boot_trusted"], w["boot_reason"]):
        if r == 0:
            store = initialize_light_client_store(trusted.tobytes(), b, verifier=v)
            assert store.finalized_header is b.header and store.optimistic_header is b.header
            assert store.best_valid_update is None and not any(bytes(store.next_sync_committee.aggregate_pubkey))
        else:
            with pytest.raises(AssertionError, match=f"reason {int(r)}"):
                initialize_light_client_store(trusted.tobytes(), b, verifier=v)


def validate_decoded(v, batch, rows, g):
    """Validate decoded rows against the golden store snapshot of their source row; device reasons
    and the oracle's reasons for the same (converted) updates."""
    from lcv.device import PackedUpdates  # noqa: F401
    gvr = g["genesis_validators_root"].tobytes()
    cur, nxt, zero = (g["nsc_pool"][k].tobytes() for k in range(3))
    got = np.full(len(rows), 255, np.uint8)
    exp = np.full(len(rows), 255, np.uint8)
    keys = sorted({(int(g["store_finalized_slot"][r]), int(g["store_next_known"][r]), int(g["current_slot"][r]))
                   for r in rows})
    for fin, nk, cs in keys:
        sel = [j for j, r in enumerate(rows) if (int(g["store_finalized_slot"][r]), int(g["store_next_known"][r]),
                                                   int(g["current_slot"][r])) == (fin, nk, cs)]
        v.set_store(fin, cur, nxt if nk else zero)
        sub = batch.slice(0, batch.n)
        for f in COLS + ("nsc_index", "signature_slot"):
            setattr(sub, f, np.ascontiguousarray(getattr(batch, f)[sel]))
        ok, reason = v.validate(sub, cs, gvr)
        got[sel] = reason
        store = H.store_from(fin, cur, nxt if nk else zero)
        for j in sel:
            exp[j] = H.O.validate_light_client_update(store, H.update_from(batch, j), cs, gvr)
    return got, exp


@pytest.mark.gpu
@pytest.mark.no_sop
def test_bootstrap_checks_gpu(engine_verifier):
    got, exp, _, _ = run_bootstrap_cases(engine_verifier)
    assert got.tolist() == exp.tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [0, 1, 2])
def test_decode_then_validate_gpu(engine_verifier, kind):
    """SSZ bytes (serialised by the reference's containers) -> native decode -> device validation."""
    w, g = load_wire(), load_updates()
    sel = np.flatnonzero(w["kind"] == kind)
    rows = w["row"][sel]
    batch = wire.decode_updates(messages(w, sel), kind=["update", "finality", "optimistic"][kind], lib=engine_verifier.lib)
    got, exp = validate_decoded(engine_verifier, batch, rows, g)
    assert got.tolist() == exp.tolist()
    if kind == 0:
        assert got.tolist() == g["expected_reason"][rows].tolist()


def test_dedup_exact_on_sampled_key_collision():
    """Committees equal in the sampled bytes (first + aggregate pubkey) but different elsewhere stay
    distinct pool rows; identical ones share a row; a large batch takes the threaded path."""
    w = load_wire()
    full = messages(w, [int(np.flatnonzero(w["kind"] == 0)[0])])[0]
    other = bytearray(full)
    other[4 + 48 * 100 + 5] ^= 0x01   # committee starts at byte 4: pubkey 100 differs
    msgs = ([full, bytes(other)] * 700)[:1400]
    for lib in libs():
        batch = wire.decode_updates(msgs, lib=lib)
        assert batch.nsc_pool.shape[0] == 2
        assert batch.nsc_index[0::2].tolist() == [0] * 700 and batch.nsc_index[1::2].tolist() == [1] * 700
        assert batch.nsc_pool[1].tobytes() == bytes(other[4:4 + 24624])


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_encode_reproduces_reference_bytes(kind):
    """encode_updates(decode_updates(x)) == x for the reference-serialised messages."""
    w = load_wire()
    msgs = messages(w, np.flatnonzero(w["kind"] == kind))
    k = ["update", "finality", "optimistic"][kind]
    batch = wire.decode_updates(msgs, kind=k, lib=libs()[0])
    assert wire.encode_updates(batch, kind=k) == msgs


class AltairHeader(Container):  # upstream altair LightClientHeader: beacon only (fixed-size)
    beacon: S.BeaconBlockHeader


class AltairUpdate(Container):
    attested_header: AltairHeader
    next_sync_committee: S.SyncCommittee
    next_sync_committee_branch: S.NextSyncCommitteeBranch
    finalized_header: AltairHeader
    finality_branch: S.FinalityBranch
    sync_aggregate: S.SyncAggregate
    signature_slot: S.Slot


def test_mixed_fork_response():
    """A LightClientUpdatesByRange response straddling fork boundaries (per-chunk ForkDigest context,
    p2p-interface.md:189-200): a Deneb, a Capella and an Altair-format chunk decoded in one pass with a
    fork per message.  The Altair chunk is serialised by the oracle's SSZ from upstream altair
    containers (not in the reference) and decodes to the golden row's Capella upgrade (empty execution);
    encode_updates(fork="altair") reproduces the same bytes."""
    from lcv.config import MAINNET, TESTNET
    from lcv.device import PackedUpdates
    w, g = load_wire(), load_updates()
    p = PackedUpdates(nsc_pool=g["nsc_pool"], nsc_index=g["nsc_index"], signature_slot=g["signature_slot"],
                      **{k: g[k] for k in COLS})
    sel_deneb = [int(np.flatnonzero((w["kind"] == 0) & (w["row"] == 0))[0])]
    u = H.update_from(p, 30)  # bellatrix_valid: pre-Capella, empty execution
    alt = serialize(AltairUpdate(attested_header=AltairHeader(beacon=u.attested_header.beacon),
                                 next_sync_committee=u.next_sync_committee,
                                 next_sync_committee_branch=u.next_sync_committee_branch,
                                 finalized_header=AltairHeader(beacon=u.finalized_header.beacon),
                                 finality_branch=u.finality_branch, sync_aggregate=u.sync_aggregate,
                                 signature_slot=u.signature_slot))
    assert wire.encode_updates(p.slice(30, 31), "update", "altair")[0] == alt
    cap = wire.encode_updates(p.slice(28, 29), "update", "capella")[0]
    msgs = messages(w, sel_deneb) + [cap, alt]
    rows = np.array([0, 28, 30])
    exp, committees = expected_rows(g, rows, 0)
    for lib in libs():
        batch = wire.decode_updates(msgs, fork=["deneb", "capella", "altair"], lib=lib)
        for k in COLS:
            assert np.array_equal(getattr(batch, k), exp[k]), k
        assert np.array_equal(batch.nsc_pool[batch.nsc_index], committees)
        # the fork decides the layout: the Altair chunk under the Capella layout is malformed
        _, ok = wire.decode_updates_status(msgs, fork=["deneb", "capella", "capella"], lib=lib)
        assert list(ok) == [True, True, False]
    # the finality / optimistic Altair forms and the bootstrap round-trip too
    for kind in ("finality", "optimistic"):
        m = wire.encode_updates(p.slice(30, 31), kind, "altair")
        b = wire.decode_updates(m, kind=kind, fork="altair")
        assert wire.encode_updates(b, kind, "altair") == m
    bt = wire.encode_bootstrap(p.att_beacon[30], p.att_exec[30], p.att_branch[30], g["nsc_pool"][0].tobytes(),
                               bytes(range(160)), fork="altair")
    d = wire.decode_bootstrap(bt, fork="altair")
    assert d.beacon.tobytes() == p.att_beacon[30].tobytes() and not d.execution.any()
    assert d.current_sync_committee_branch.tobytes() == bytes(range(160))
    # ForkDigest context -> container namespace, under the network configuration
    assert wire.fork_of_digest_version(MAINNET.BELLATRIX_FORK_VERSION, MAINNET) == "altair"
    assert wire.fork_of_digest_version(MAINNET.CAPELLA_FORK_VERSION, MAINNET) == "capella"
    assert wire.fork_of_digest_version(TESTNET.DENEB_FORK_VERSION, TESTNET) == "deneb"
    with pytest.raises(ValueError):
        wire.fork_of_digest_version(MAINNET.GENESIS_FORK_VERSION, MAINNET)
