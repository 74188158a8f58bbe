#!/usr/bin/env python3
"""Generate the committed golden fixtures (run in the build container only; needs /root/reference).

    python tests/golden/make_golden.py

lc_updates.npz — light-client update cases (packed rows, include/lcv.h layouts) with the reason code
    of the first failing assert of `validate_light_client_update`.  The expected reason of every case
    is computed TWICE and must agree:
      (1) by exec'ing the reference's OWN python blocks from /root/reference/sync-protocol.md
          (compiled with their markdown line numbers; the failing assert's line is mapped to its
          index among the function's asserts), over the oracle's restatement of the 36 upstream
          names (oracle/spec.py: SSZ, compute_*, bls = oracle FastAggregateVerify);
      (2) by the oracle restatement oracle/sync_protocol.py.
    Nothing from the reference is stored: only inputs and the expected reason codes.
store_sequence.npz — a sequence of updates run through the reference's OWN exec'd
    `process_light_client_update` (and one `process_light_client_store_force_update`) from two
    starting stores (next committee known / unknown): per step the accept flag, the validation
    reason and a summary of the store (finalized / optimistic slot, best update, committees, max
    participants).  `python tests/golden/make_golden.py store` regenerates only this file.
wire.npz — SSZ wire bytes produced by the reference's OWN exec'd containers (LightClientUpdate,
    LightClientFinalityUpdate, LightClientOptimisticUpdate, LightClientBootstrap) from golden rows, and
    bootstrap cases whose expected reason is the failing assert of the reference's exec'd
    `initialize_light_client_store`.  `python tests/golden/make_golden.py wire` regenerates only this.
bls_vectors.npz — hash_to_G2 outputs, G1/G2 decompression cases (valid, identity, bad flags, x >= p,
    not on curve, not in the subgroup) and FastAggregateVerify verdicts, all from oracle/bls12_381.py.
"""
from __future__ import annotations

import ast
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import helpers as H  # noqa: E402

from lcv import synth  # noqa: E402
from lcv.config import MAINNET, TESTNET  # noqa: E402
from oracle import bls12_381 as B  # noqa: E402
from oracle import spec as S  # noqa: E402
from oracle.ssz import serialize  # noqa: E402

REF = "/root/reference/sync-protocol.md"
COLS = ("att_beacon", "att_exec", "att_branch", "fin_beacon", "fin_exec", "fin_branch", "nsc_branch",
        "finality_branch", "sync_bits", "sync_signature")


# ----------------------------------------------------------------------------- reference exec
def load_reference():
    text = open(REF).read()
    ns = S.reference_namespace()
    assert_lines = None
    for m in re.finditer(r"```python\n(.*?)```", text, re.S):
        start_line = text[:m.start(1)].count("\n") + 1
        code = m.group(1)
        exec(compile("\n" * (start_line - 1) + code, "sync-protocol.md", "exec", dont_inherit=True), ns)
        if code.startswith("def validate_light_client_update"):
            tree = ast.parse("\n" * (start_line - 1) + code)
            assert_lines = [(n.lineno, n.end_lineno) for n in ast.walk(tree) if isinstance(n, ast.Assert)]
    assert_lines = sorted(assert_lines)
    assert len(assert_lines) == 14, assert_lines
    return ns, assert_lines


def reference_reason(ns, assert_lines, store, update, current_slot, gvr) -> int:
    import traceback
    try:
        ns["validate_light_client_update"](store, update, current_slot, gvr)
        return 0
    except AssertionError:
        tb = traceback.extract_tb(sys.exc_info()[2])
        lines = [f.lineno for f in tb if f.filename == "sync-protocol.md"]
        return next(k for k, (a, b) in enumerate(assert_lines) if a <= lines[-1] <= b) + 1


def to_reference_objects(ns, p, i, fin_slot, cur, nxt):
    """The same bytes as the reference's own container classes (exec'd from the markdown)."""
    ou = H.update_from(p, i)
    LCH, LCU = ns["LightClientHeader"], ns["LightClientUpdate"]

    def hdr(h):
        return LCH(beacon=h.beacon, execution=h.execution, execution_branch=h.execution_branch)

    u = LCU(attested_header=hdr(ou.attested_header), next_sync_committee=ou.next_sync_committee,
            next_sync_committee_branch=ou.next_sync_committee_branch, finalized_header=hdr(ou.finalized_header),
            finality_branch=ou.finality_branch, sync_aggregate=ou.sync_aggregate, signature_slot=ou.signature_slot)
    fin = LCH()
    fin.beacon.slot = fin_slot
    store = ns["LightClientStore"](finalized_header=fin, current_sync_committee=H.committee_from(cur),
                                   next_sync_committee=H.committee_from(nxt), best_valid_update=None,
                                   optimistic_header=LCH(), previous_max_active_participants=0,
                                   current_max_active_participants=0)
    return store, u


# ----------------------------------------------------------------------------- cases
class Cases:
    def __init__(self):
        self.rows = {k: [] for k in COLS}
        self.sig_slot, self.pool_row, self.store_fin, self.next_known, self.current_slot, self.name = [], [], [], [], [], []

    def add(self, p, i, name, store_fin, next_known, current_slot, pool_row, **over):
        for k in COLS:
            self.rows[k].append(bytes(over.get(k, p.__dict__[k][i].tobytes())))
        self.sig_slot.append(int(over.get("signature_slot", p.signature_slot[i])))
        self.pool_row.append(pool_row)
        self.store_fin.append(store_fin)
        self.next_known.append(next_known)
        self.current_slot.append(current_slot)
        self.name.append(name)


def flip(b: bytes, j: int, mask: int = 1) -> bytes:
    return b[:j] + bytes([b[j] ^ mask]) + b[j + 1:]


def build_cases(v):
    cur, nxt = synth.make_committee(v, 0), synth.make_committee(v, 1)
    comms = (cur, nxt)
    C = Cases()
    SPP = MAINNET.SLOTS_PER_PERIOD
    P = synth.DENEB_PERIOD * SPP
    # A: Deneb, next committee known; every corruption kind once (+ 2 valid)
    kinds = np.array([0, 0, 1, 2, 3, 4, 5, 6, 7])
    a = synth.generate(v, len(kinds), seed=21, participation="random", kinds=kinds, committees=comms)
    for i, k in enumerate(kinds):
        C.add(a.updates, i, f"deneb_kind{k}", P, 1, a.current_slot, 1)
    pa = a.updates
    big = P + 4 * SPP
    # mutations of the valid row 0
    C.add(pa, 0, "slot_order_current", P, 1, int(pa.signature_slot[0]) - 1, 1)
    C.add(pa, 0, "sig_period_skip", P, 1, big, 1, signature_slot=P + 2 * SPP + 5)
    att_slot = int.from_bytes(pa.att_beacon[0][:8].tobytes(), "little")
    C.add(pa, 0, "not_relevant", att_slot, 1, a.current_slot, 1)
    C.add(pa, 0, "finalized_not_empty", P, 1, a.current_slot, 1, finality_branch=bytes(192))
    fb = bytearray(pa.fin_beacon[0].tobytes())
    fb[0:8] = bytes(8)
    C.add(pa, 0, "finalized_genesis_not_empty", P, 1, a.current_slot, 1, fin_beacon=bytes(fb))
    C.add(pa, 0, "finalized_header_invalid", P, 1, a.current_slot, 1, fin_branch=flip(pa.fin_branch[0].tobytes(), 3))
    C.add(pa, 0, "nsc_not_empty", P, 1, a.current_slot, 1, nsc_branch=bytes(160))
    C.add(pa, 0, "nsc_mismatch_store", P, 1, a.current_slot, 0)  # pool row 0 = current committee != store.next
    C.add(pa, 0, "bad_sig_bitflip", P, 1, a.current_slot, 1, sync_signature=flip(pa.sync_signature[0].tobytes(), 95))
    sig_inf = bytes([0xC0]) + bytes(95)
    C.add(pa, 0, "sig_identity", P, 1, a.current_slot, 1, sync_signature=sig_inf)
    sig_noflag = bytes([pa.sync_signature[0][0] & 0x7F]) + pa.sync_signature[0][1:].tobytes()
    C.add(pa, 0, "sig_c_flag_clear", P, 1, a.current_slot, 1, sync_signature=sig_noflag)
    bits_one = bytearray(64)
    bits_one[0] = 1
    C.add(pa, 0, "single_participant_wrong_sig", P, 1, a.current_slot, 1, sync_bits=bytes(bits_one))
    # B: no finality / no next committee (valid), Deneb
    b1 = synth.generate(v, 1, seed=22, with_finality=False, committees=comms)
    C.add(b1.updates, 0, "no_finality", P, 1, b1.current_slot, 1)
    b2 = synth.generate(v, 1, seed=23, with_next=False, committees=comms)
    C.add(b2.updates, 0, "no_next_committee", P, 1, b2.current_slot, 2)
    # C: signature by the next committee (signature period = store + 1)
    c = synth.generate(v, 2, seed=24, sign_next=True, committees=comms)
    C.add(c.updates, 0, "next_period_signature", P, 1, c.current_slot, 1)
    C.add(c.updates, 1, "next_period_signature_store_next_unknown", P, 0, c.current_slot, 1)
    # D: next committee unknown at the store: valid, and relevance via has_next (att slot <= store slot)
    d = synth.generate(v, 1, seed=25, committees=comms)
    C.add(d.updates, 0, "store_next_unknown", P, 0, d.current_slot, 1)
    att_d = int.from_bytes(d.updates.att_beacon[0][:8].tobytes(), "little")
    C.add(d.updates, 0, "relevant_via_next_committee", att_d, 0, d.current_slot, 1)
    C.add(d.updates, 0, "not_relevant_next_known", att_d, 1, d.current_slot, 1)
    # E: Capella update (BASELINE config 1 substitute) and a Capella header carrying blob gas
    PC = synth.CAPELLA_PERIOD * SPP
    e = synth.generate(v, 1, seed=26, period=synth.CAPELLA_PERIOD, committees=comms)
    C.add(e.updates, 0, "capella_valid", PC, 1, e.current_slot, 1)
    ex = bytearray(e.updates.att_exec[0].tobytes())
    ex[480] = 1
    C.add(e.updates, 0, "capella_blob_gas", PC, 1, e.current_slot, 1, att_exec=bytes(ex))
    # F: pre-Capella (Bellatrix) update: empty execution is valid, a non-empty one is not
    f = synth.generate(v, 1, seed=27, period=600, committees=comms)
    PB = 600 * SPP
    C.add(f.updates, 0, "bellatrix_valid", PB, 1, f.current_slot, 1)
    exb = bytearray(832)
    exb[0] = 7
    C.add(f.updates, 0, "bellatrix_nonempty_execution", PB, 1, f.current_slot, 1, att_exec=bytes(exb))
    return C, cur, nxt, a.genesis_validators_root


def main():
    v = H.hostsim_verifier()
    ns, assert_lines = load_reference()
    C, cur, nxt, gvr = build_cases(v)
    n = len(C.name)
    pool = np.stack([np.frombuffer(x, np.uint8) for x in (cur.ssz, nxt.ssz, bytes(24624))])
    arrays = {k: np.stack([np.frombuffer(r, np.uint8) for r in C.rows[k]]) for k in COLS}
    from lcv.device import PackedUpdates
    p = PackedUpdates(nsc_pool=pool, nsc_index=np.array(C.pool_row, np.uint32),
                      signature_slot=np.array(C.sig_slot, np.uint64), **arrays)
    reasons = []
    for i in range(n):
        nk = C.next_known[i]
        nxt_bytes = nxt.ssz if nk else bytes(24624)
        store_o = H.store_from(C.store_fin[i], cur.ssz, nxt_bytes)
        r_oracle = H.O.validate_light_client_update(store_o, H.update_from(p, i), C.current_slot[i], gvr)
        store_r, u_r = to_reference_objects(ns, p, i, C.store_fin[i], cur.ssz, nxt_bytes)
        r_ref = reference_reason(ns, assert_lines, store_r, u_r, C.current_slot[i], gvr)
        assert r_oracle == r_ref, (C.name[i], r_oracle, r_ref)
        reasons.append(r_ref)
        print(f"{i:3d} {C.name[i]:45s} reason {r_ref}", flush=True)
    np.savez_compressed(os.path.join(HERE, "lc_updates.npz"), **arrays, nsc_pool=pool,
                        nsc_index=np.array(C.pool_row, np.uint32), signature_slot=np.array(C.sig_slot, np.uint64),
                        store_finalized_slot=np.array(C.store_fin, np.uint64),
                        store_next_known=np.array(C.next_known, np.uint8),
                        current_slot=np.array(C.current_slot, np.uint64), expected_reason=np.array(reasons, np.uint8),
                        genesis_validators_root=np.frombuffer(gvr, np.uint8))
    json.dump({"cases": C.name, "expected_reason": reasons, "reference_assert_lines": assert_lines},
              open(os.path.join(HERE, "lc_updates.json"), "w"), indent=1)
    make_bls_vectors()


# ----------------------------------------------------------------------------- store sequences
STORE_KINDS = [synth.K_LOW_PARTICIPATION, synth.K_LOW_PARTICIPATION, synth.K_VALID, synth.K_BAD_SIG_MESSAGE,
               synth.K_LOW_PARTICIPATION, synth.K_VALID, synth.K_BAD_FINALITY_BRANCH, synth.K_VALID,
               synth.K_LOW_PARTICIPATION, synth.K_VALID, synth.K_BAD_NSC_BRANCH, synth.K_VALID]


def store_summary(store) -> list:
    """Everything process_light_client_update can change, as integers (committees as a digest)."""
    import hashlib
    from lcv import layout as L

    def dig(sc):
        return int.from_bytes(hashlib.sha256(L.pack_sync_committee(sc)).digest()[:7], "little")
    best = store.best_valid_update
    return [int(store.finalized_header.beacon.slot), int(store.optimistic_header.beacon.slot),
            -1 if best is None else int(best.signature_slot), -1 if best is None else int(best.attested_header.beacon.slot),
            dig(store.current_sync_committee), dig(store.next_sync_committee),
            int(store.previous_max_active_participants), int(store.current_max_active_participants)]


def make_store_sequence():
    v = H.hostsim_verifier()
    ns, assert_lines = load_reference()
    cur, nxt = synth.make_committee(v, 0), synth.make_committee(v, 1)
    kinds = np.array(STORE_KINDS)
    sb = synth.generate(v, len(kinds), seed=31, participation="random", kinds=kinds, committees=(cur, nxt))
    p = sb.updates
    n = len(kinds)
    gvr = sb.genesis_validators_root
    out = {"accepted": [], "reason": [], "summary": []}
    for next_known in (1, 0):
        nxt_bytes = nxt.ssz if next_known else bytes(24624)
        store_r, _ = to_reference_objects(ns, p, 0, sb.store_finalized_slot, cur.ssz, nxt_bytes)
        acc, rea, summ = [], [], []
        for i in range(n):
            _, u_r = to_reference_objects(ns, p, i, sb.store_finalized_slot, cur.ssz, nxt_bytes)
            rea.append(reference_reason(ns, assert_lines, store_r, u_r, sb.current_slot, gvr))
            try:
                ns["process_light_client_update"](store_r, u_r, sb.current_slot, gvr)
                acc.append(1)
            except AssertionError:
                acc.append(0)
            assert acc[-1] == (rea[-1] == 0)
            summ.append(store_summary(store_r))
            print(f"next_known={next_known} step {i:2d} kind {kinds[i]} reason {rea[-1]} store {summ[-1]}", flush=True)
        force_slot = int(store_r.finalized_header.beacon.slot) + ns["UPDATE_TIMEOUT"] + 1
        ns["process_light_client_store_force_update"](store_r, force_slot)
        summ.append(store_summary(store_r))
        print(f"next_known={next_known} force update at {force_slot}: store {summ[-1]}", flush=True)
        out["accepted"].append(acc)
        out["reason"].append(rea)
        out["summary"].append(summ)
    np.savez_compressed(os.path.join(HERE, "store_sequence.npz"), **{k: p.__dict__[k] for k in COLS},
                        nsc_pool=p.nsc_pool, nsc_index=p.nsc_index, signature_slot=p.signature_slot,
                        store_finalized_slot=np.uint64(sb.store_finalized_slot), current_slot=np.uint64(sb.current_slot),
                        genesis_validators_root=np.frombuffer(gvr, np.uint8), kinds=kinds,
                        current_committee=np.frombuffer(cur.ssz, np.uint8), next_committee=np.frombuffer(nxt.ssz, np.uint8),
                        accepted=np.array(out["accepted"], np.uint8), reason=np.array(out["reason"], np.uint8),
                        summary=np.array(out["summary"], np.int64))


def make_bls_vectors():
    rng = np.random.default_rng(99)
    msgs = [bytes(32), b"\xff" * 32] + [rng.bytes(32) for _ in range(6)]
    h2c = [b"".join(c.to_bytes(48, "big") for c in (q[0][0], q[0][1], q[1][0], q[1][1]))
           for q in (B.hash_to_g2(m) for m in msgs)]
    # G2 signature decoding cases: status 0 ok, 1 identity, 2 invalid (py_ecc rules + subgroup)
    sigs, st = [], []
    good = B.sign(12345, msgs[2])
    sigs += [good]; st += [0]
    sigs += [bytes([0xC0]) + bytes(95)]; st += [1]
    sigs += [bytes([0xE0]) + bytes(95)]; st += [2]                       # identity with a_flag
    sigs += [bytes([good[0] & 0x7F]) + good[1:]]; st += [2]              # c_flag clear
    sigs += [bytes([good[0] | 0x40]) + good[1:]]; st += [2]              # b_flag on a non-identity
    sigs += [bytes([0x9A]) + b"\xff" * 47 + bytes(48)]; st += [2]        # x1 >= p
    xp = (B.P + 5).to_bytes(48, "big")
    sigs += [bytes([0x80]) + bytes(47) + xp]; st += [2]                  # x0 >= p
    # on the twist curve but outside G2, and not on the curve at all
    x = 1
    while True:
        x += 1
        X = (x, 1)
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(X), X), B.B2))
        if y is not None and not B.g2_in_subgroup((X, y)):
            sigs += [B.g2_compress((X, y))]; st += [2]
            break
    x = 1
    while True:
        x += 1
        X = (x, 3)
        if B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(X), X), B.B2)) is None:
            enc = bytearray((3).to_bytes(48, "big") + x.to_bytes(48, "big"))
            enc[0] |= 0x80
            sigs += [bytes(enc)]
            st += [2]
            break
    # FastAggregateVerify: (pubkeys, msg, sig) -> verdict
    sks = [7, 11, 13]
    pks = [B.sk_to_pk(k) for k in sks]
    m = msgs[3]
    agg = B.aggregate_signatures([B.sign(k, m) for k in sks])
    fav = [(pks, m, agg), (pks[:2], m, agg), (pks, msgs[4], agg), ([], m, agg),
           (pks + [bytes([0xC0]) + bytes(47)], m, agg)]
    fav_expect = [B.fast_aggregate_verify(a, b_, c) for a, b_, c in fav]
    assert fav_expect == [True, False, False, False, False]
    np.savez_compressed(os.path.join(HERE, "bls_vectors.npz"),
                        h2c_msg=np.frombuffer(b"".join(msgs), np.uint8).reshape(-1, 32),
                        h2c_out=np.frombuffer(b"".join(h2c), np.uint8).reshape(-1, 192),
                        sig=np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 96), sig_status=np.array(st, np.uint8),
                        fav_pks=np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 48),
                        fav_msg=np.frombuffer(m, np.uint8), fav_sig=np.frombuffer(agg, np.uint8))
    print("bls vectors:", len(msgs), "h2c,", len(sigs), "signature decodings")


# ----------------------------------------------------------------------------- SSZ wire + bootstrap
WIRE_UPDATE_ROWS = (0, 6, 21, 22, 28, 30)   # full updates: Deneb, bad nsc branch, no finality, no nsc, capella, bellatrix


def _bootstrap_assert_lines():
    text = open(REF).read()
    for m in re.finditer(r"```python\n(.*?)```", text, re.S):
        if m.group(1).startswith("def initialize_light_client_store"):
            start_line = text[:m.start(1)].count("\n") + 1
            tree = ast.parse("\n" * (start_line - 1) + m.group(1))
            return sorted((n.lineno, n.end_lineno) for n in ast.walk(tree) if isinstance(n, ast.Assert))
    raise RuntimeError("initialize_light_client_store not found")


def make_wire():
    import hashlib
    from oracle.ssz import serialize
    from golden_cases import load_updates
    from lcv.device import PackedUpdates
    ns, _ = load_reference()
    g = load_updates()
    p = PackedUpdates(nsc_pool=g["nsc_pool"], nsc_index=g["nsc_index"], signature_slot=g["signature_slot"],
                      **{k: g[k] for k in COLS})
    n = len(g["expected_reason"])
    LCH, LCU = ns["LightClientHeader"], ns["LightClientUpdate"]
    LCF, LCO, LCB = ns["LightClientFinalityUpdate"], ns["LightClientOptimisticUpdate"], ns["LightClientBootstrap"]
    msgs, kind, row = [], [], []

    def put(obj, k, i):
        b = serialize(obj)
        assert serialize(type(obj).de(b)) == b  # the reference container round-trips its own bytes
        msgs.append(b); kind.append(k); row.append(i)

    for i in range(n):
        _, u = to_reference_objects(ns, p, i, 0, bytes(24624), bytes(24624))
        if i in WIRE_UPDATE_ROWS:
            put(u, 0, i)
        put(LCF(attested_header=u.attested_header, finalized_header=u.finalized_header, finality_branch=u.finality_branch,
                sync_aggregate=u.sync_aggregate, signature_slot=u.signature_slot), 1, i)
        put(LCO(attested_header=u.attested_header, sync_aggregate=u.sync_aggregate, signature_slot=u.signature_slot), 2, i)
    # bootstraps: header = a golden attested header whose state_root commits to a committee at
    # CURRENT_SYNC_COMMITTEE_GINDEX (54: depth 5, subtree index 22) through a synthetic branch
    rng = np.random.default_rng(54)
    cur, nxt = g["nsc_pool"][0].tobytes(), g["nsc_pool"][1].tobytes()
    lines = _bootstrap_assert_lines()
    assert len(lines) == 3, lines
    B_cases = [("deneb_valid", 0, {}), ("capella_valid", 28, {}), ("bellatrix_valid", 30, {}),
               ("bad_execution_branch", 0, {"exec_branch": True}), ("capella_blob_gas", 29, {}),
               ("wrong_trusted_root", 0, {"trusted": True}), ("bad_committee_branch", 0, {"branch": True}),
               ("other_committee", 28, {"committee": True}), ("bellatrix_bad_committee_branch", 30, {"branch": True})]
    bmsgs, btrusted, breason, bnames = [], [], [], []
    sha = lambda b: hashlib.sha256(b).digest()  # noqa: E731
    for name, i, over in B_cases:
        _, u = to_reference_objects(ns, p, i, 0, bytes(24624), bytes(24624))
        h = u.attested_header
        branch = [rng.bytes(32) for _ in range(5)]
        node = bytes(S.hash_tree_root(H.committee_from(cur)))
        for d in range(5):
            node = sha(branch[d] + node) if (22 >> d) & 1 else sha(node + branch[d])
        h.beacon.state_root = node
        if over.get("exec_branch"):
            eb = list(h.execution_branch); eb[2] = flip(bytes(eb[2]), 7); h.execution_branch = eb
        if over.get("branch"):
            branch[3] = flip(branch[3], 30)
        trusted = bytes(S.hash_tree_root(h.beacon))
        if over.get("trusted"):
            trusted = flip(trusted, 0)
        bs = LCB(header=h, current_sync_committee=H.committee_from(nxt if over.get("committee") else cur),
                 current_sync_committee_branch=branch)
        import traceback
        try:
            ns["initialize_light_client_store"](trusted, bs)
            r = 0
        except AssertionError:
            tb = [f.lineno for f in traceback.extract_tb(sys.exc_info()[2]) if f.filename == "sync-protocol.md"]
            r = next(k for k, (a, b) in enumerate(lines) if a <= tb[-1] <= b) + 1
        b = serialize(bs)
        assert serialize(LCB.de(b)) == b
        bmsgs.append(b); btrusted.append(trusted); breason.append(r); bnames.append(name)
        print(f"bootstrap {name:32s} reason {r}", flush=True)
    offs = np.cumsum([0] + [len(m) for m in msgs])
    boffs = np.cumsum([0] + [len(m) for m in bmsgs])
    np.savez_compressed(os.path.join(HERE, "wire.npz"),
                        buf=np.frombuffer(b"".join(msgs), np.uint8), offsets=offs[:-1].astype(np.uint64),
                        lengths=np.diff(offs).astype(np.uint64), kind=np.array(kind, np.uint8), row=np.array(row, np.uint32),
                        boot_buf=np.frombuffer(b"".join(bmsgs), np.uint8), boot_offsets=boffs[:-1].astype(np.uint64),
                        boot_lengths=np.diff(boffs).astype(np.uint64),
                        boot_trusted=np.frombuffer(b"".join(btrusted), np.uint8).reshape(-1, 32),
                        boot_reason=np.array(breason, np.uint8))
    json.dump({"bootstrap_cases": bnames, "bootstrap_reason": breason, "reference_assert_lines": lines,
               "messages": len(msgs)}, open(os.path.join(HERE, "wire.json"), "w"), indent=1)
    print("wire:", len(msgs), "messages,", len(bmsgs), "bootstraps")


# ----------------------------------------------------------------------------- producer side (full-node.md)
FULL_NODE = "/root/reference/full-node.md"


def load_full_node(ns):
    """exec the reference's full-node.md blocks into `ns` (after sync-protocol.md's), with the oracle's
    compute_merkle_proof for the helper the reference declares without a body (full-node.md:35-38)."""
    from oracle.ssz import compute_merkle_proof
    from typing import Sequence
    ns.update(BeaconState=S.BeaconState, SignedBeaconBlock=S.SignedBeaconBlock, ALTAIR_FORK_EPOCH=S.ALTAIR_FORK_EPOCH,
              Sequence=Sequence, SSZObject=object)
    text = open(FULL_NODE).read()
    for m in re.finditer(r"```python\n(.*?)```", text, re.S):
        start_line = text[:m.start(1)].count("\n") + 1
        exec(compile("\n" * (start_line - 1) + m.group(1), "full-node.md", "exec", dont_inherit=True), ns)
    ns["compute_merkle_proof"] = compute_merkle_proof
    return ns


def _payload(rng, deneb=True):
    return S.ExecutionPayload(
        parent_hash=rng.bytes(32), fee_recipient=rng.bytes(20), state_root=rng.bytes(32), receipts_root=rng.bytes(32),
        logs_bloom=rng.bytes(256), prev_randao=rng.bytes(32), block_number=int(rng.integers(0, 2 ** 40)),
        gas_limit=int(rng.integers(0, 2 ** 40)), gas_used=int(rng.integers(0, 2 ** 40)),
        timestamp=int(rng.integers(0, 2 ** 40)), extra_data=rng.bytes(int(rng.integers(0, 33))),
        base_fee_per_gas=int(rng.integers(0, 2 ** 62)), block_hash=rng.bytes(32),
        transactions=[rng.bytes(int(rng.integers(1, 200))) for _ in range(int(rng.integers(0, 4)))],
        withdrawals=[S.Withdrawal(index=int(rng.integers(0, 2 ** 30)), validator_index=int(rng.integers(0, 2 ** 20)),
                                  address=rng.bytes(20), amount=int(rng.integers(0, 2 ** 40))) for _ in range(2)],
        blob_gas_used=int(rng.integers(0, 2 ** 20)) if deneb else 0,
        excess_blob_gas=int(rng.integers(0, 2 ** 20)) if deneb else 0)


def _block_state(rng, slot, parent_root, fin_cp, cur, nxt, bits, sig, gvr):
    """A (post-state, signed block) pair at `slot` with random contents (Deneb containers)."""
    body = S.BeaconBlockBody(randao_reveal=rng.bytes(96),
                             eth1_data=S.Eth1Data(deposit_root=rng.bytes(32), deposit_count=int(rng.integers(0, 2 ** 20)),
                                                  block_hash=rng.bytes(32)),
                             graffiti=rng.bytes(32),
                             sync_aggregate=S.SyncAggregate(sync_committee_bits=list(bits), sync_committee_signature=sig),
                             execution_payload=_payload(rng), blob_kzg_commitments=[rng.bytes(48) for _ in range(2)])
    proposer = int(rng.integers(0, 2 ** 20))
    st = S.BeaconState(
        genesis_time=1606824023, genesis_validators_root=gvr, slot=slot,
        fork=S.Fork(previous_version=rng.bytes(4), current_version=rng.bytes(4), epoch=int(rng.integers(0, 2 ** 20))),
        latest_block_header=S.BeaconBlockHeader(slot=slot, proposer_index=proposer, parent_root=parent_root,
                                                state_root=bytes(32), body_root=S.hash_tree_root(body)),
        historical_roots=[rng.bytes(32) for _ in range(3)],
        eth1_data=S.Eth1Data(deposit_root=rng.bytes(32), deposit_count=7, block_hash=rng.bytes(32)),
        eth1_deposit_index=int(rng.integers(0, 2 ** 20)),
        validators=[S.Validator(pubkey=rng.bytes(48), withdrawal_credentials=rng.bytes(32), effective_balance=32 * 10 ** 9,
                                slashed=k == 1, activation_eligibility_epoch=k, activation_epoch=k + 1,
                                exit_epoch=2 ** 64 - 1, withdrawable_epoch=2 ** 64 - 1) for k in range(3)],
        balances=[int(rng.integers(0, 2 ** 40)) for _ in range(3)],
        previous_epoch_participation=[7, 3, 0], current_epoch_participation=[1, 7, 7],
        justification_bits=[1, 1, 0, 1],
        previous_justified_checkpoint=S.Checkpoint(epoch=int(rng.integers(0, 2 ** 20)), root=rng.bytes(32)),
        current_justified_checkpoint=S.Checkpoint(epoch=int(rng.integers(0, 2 ** 20)), root=rng.bytes(32)),
        finalized_checkpoint=fin_cp, inactivity_scores=[0, 5, 9],
        current_sync_committee=H.committee_from(cur), next_sync_committee=H.committee_from(nxt),
        next_withdrawal_index=int(rng.integers(0, 2 ** 30)), next_withdrawal_validator_index=int(rng.integers(0, 2 ** 20)),
        historical_summaries=[S.HistoricalSummary(block_summary_root=rng.bytes(32), state_summary_root=rng.bytes(32))])
    blk = S.BeaconBlock(slot=slot, proposer_index=proposer, parent_root=parent_root, state_root=S.hash_tree_root(st),
                        body=body)
    return st, S.SignedBeaconBlock(message=blk, signature=rng.bytes(96))


def _state_view_arrays(st):
    """The sparse producer view of an oracle BeaconState: explicit fields + every field's root."""
    roots = np.stack([np.frombuffer(bytes(t.htr(getattr(st, n))), np.uint8) for n, t in type(st)._fields])
    return dict(slot=int(st.slot), header=np.frombuffer(serialize(st.latest_block_header), np.uint8),
                fin_epoch=int(st.finalized_checkpoint.epoch), fin_root=np.frombuffer(bytes(st.finalized_checkpoint.root), np.uint8),
                cur=np.frombuffer(serialize(st.current_sync_committee), np.uint8),
                nxt=np.frombuffer(serialize(st.next_sync_committee), np.uint8), roots=roots)


def _block_view_arrays(sb):
    from types import SimpleNamespace
    from lcv import layout as LL
    m = sb.message
    b = m.body
    roots = np.stack([np.frombuffer(bytes(t.htr(getattr(b, n))), np.uint8) for n, t in type(b)._fields])
    pl = b.execution_payload
    hdr = SimpleNamespace(**{n: getattr(pl, n) for n in LL.EXEC_FIELDS if n not in ("transactions_root", "withdrawals_root")},
                          transactions_root=S.hash_tree_root(pl.transactions), withdrawals_root=S.hash_tree_root(pl.withdrawals))
    return dict(slot=int(m.slot), proposer=int(m.proposer_index), parent=np.frombuffer(bytes(m.parent_root), np.uint8),
                state_root=np.frombuffer(bytes(m.state_root), np.uint8),
                bits=np.frombuffer(S.SyncAggregate._fields[0][1].ser(b.sync_aggregate.sync_committee_bits), np.uint8),
                sig=np.frombuffer(bytes(b.sync_aggregate.sync_committee_signature), np.uint8),
                exec=np.frombuffer(LL.pack_execution(hdr), np.uint8), roots=roots)


def make_producer():
    """producer.npz: light-client data derived by the reference's OWN exec'd full-node.md functions
    (block_to_light_client_header, create_light_client_bootstrap / _update / _finality_update /
    _optimistic_update; compute_merkle_proof = the oracle's SSZ proof) from random Deneb-shaped
    beacon states and blocks (oracle/spec.py containers), with each update's validation reason from the
    exec'd validate_light_client_update.  Stored: the producer views of every state / block (explicit
    fields + field roots, what lcv.producer consumes) and the expected SSZ bytes of every output."""
    from oracle.ssz import serialize
    v = H.hostsim_verifier()
    ns, assert_lines = load_reference()
    load_full_node(ns)
    cur, nxt = synth.make_committee(v, 0), synth.make_committee(v, 1)
    gvr = synth.sha256(b"lcv-producer-genesis-validators-root")
    SPP = MAINNET.SLOTS_PER_PERIOD
    rng = np.random.default_rng(77)
    states, blocks, cases = [], [], []
    outs = {"update": [], "finality": [], "optimistic": [], "bootstrap": []}
    meta = []

    def add_view(lst, arrays):
        lst.append(arrays)
        return len(lst) - 1

    scenarios = [("deneb_full", 1100, "same", "fin", "full"),
                 ("deneb_next_period_signature", 1100, "next", "fin", "random"),
                 ("deneb_no_finalized_block", 1101, "same", None, "random"),
                 ("deneb_genesis_finalized", 1102, "same", "genesis", "full"),
                 ("bellatrix", 600, "same", "fin", "random")]
    for name, period, sigp, fin_kind, part in scenarios:
        base = period * SPP
        F = base + int(rng.integers(1, 64))
        A = F + 64 + int(rng.integers(0, 512))
        Ssl = A + 1 + int(rng.integers(0, 16)) if sigp == "same" else base + SPP + int(rng.integers(0, 32))
        zero_bits = [True] * 512
        fin_state, fin_block = _block_state(rng, F, rng.bytes(32), S.Checkpoint(epoch=0, root=bytes(32)), cur.ssz, nxt.ssz,
                                            zero_bits, rng.bytes(96), gvr)
        if fin_kind == "fin":
            fin_cp = S.Checkpoint(epoch=F // 32, root=S.hash_tree_root(fin_block.message))
            fb = fin_block
        elif fin_kind == "genesis":
            fin_block.message.slot = 0
            fin_cp = S.Checkpoint(epoch=0, root=bytes(32))
            fb = fin_block
        else:
            fin_cp = S.Checkpoint(epoch=F // 32, root=rng.bytes(32))
            fb = None
        att_state, att_block = _block_state(rng, A, rng.bytes(32), fin_cp, cur.ssz, nxt.ssz, zero_bits, rng.bytes(96), gvr)
        # the sync aggregate over the attested header, signed by the committee of the signature period
        if part == "full":
            bits = [True] * 512
        else:
            bits = [bool(x) for x in rng.integers(0, 2, 512)]
            bits[0] = True
        signer = cur if sigp == "same" else nxt
        sk = sum(k for k, b_ in zip(signer.sks, bits) if b_) % synth.R_ORDER
        att_hdr = S.BeaconBlockHeader(slot=A, proposer_index=att_block.message.proposer_index,
                                      parent_root=att_block.message.parent_root, state_root=att_block.message.state_root,
                                      body_root=S.hash_tree_root(att_block.message.body))
        msg = synth.signing_root(serialize(att_hdr), Ssl, gvr, MAINNET)
        sig = v.sign_batch(np.frombuffer(sk.to_bytes(32, "big"), np.uint8), np.frombuffer(msg, np.uint8))[0].tobytes()
        sig_state, sig_block = _block_state(rng, Ssl, S.hash_tree_root(att_block.message), fin_cp, cur.ssz, nxt.ssz,
                                            bits, sig, gvr)
        upd = ns["create_light_client_update"](sig_state, sig_block, att_state, att_block, fb)
        fu = ns["create_light_client_finality_update"](upd)
        ou = ns["create_light_client_optimistic_update"](upd)
        boot = ns["create_light_client_bootstrap"](att_state, att_block)
        for k, obj in (("update", upd), ("finality", fu), ("optimistic", ou), ("bootstrap", boot)):
            outs[k].append(serialize(obj))
        # the update validated by the reference against a store finalized at the start of the period
        store = ns["LightClientStore"](finalized_header=ns["LightClientHeader"](), current_sync_committee=H.committee_from(cur.ssz),
                                       next_sync_committee=H.committee_from(nxt.ssz), best_valid_update=None,
                                       optimistic_header=ns["LightClientHeader"](), previous_max_active_participants=0,
                                       current_max_active_participants=0)
        store.finalized_header.beacon.slot = base
        r = reference_reason(ns, assert_lines, store, upd, Ssl, gvr)
        ids = [add_view(states, _state_view_arrays(st)) for st in (sig_state, att_state)]
        bids = [add_view(blocks, _block_view_arrays(b_)) for b_ in (sig_block, att_block, fin_block)]
        cases.append(dict(name=name, state=ids[0], block=bids[0], attested_state=ids[1], attested_block=bids[1],
                          finalized_block=bids[2] if fb is not None else -1, store_finalized_slot=base, current_slot=Ssl,
                          reason=r))
        print(f"producer {name:30s} update {len(outs['update'][-1])} B, reason {r}", flush=True)
    arrays = {}
    for prefix, lst in (("state", states), ("block", blocks)):
        for k in lst[0]:
            arrays[f"{prefix}_{k}"] = np.stack([np.asarray(x[k]) for x in lst])
    for k, lst in outs.items():
        offs = np.cumsum([0] + [len(m) for m in lst])
        arrays[f"out_{k}"] = np.frombuffer(b"".join(lst), np.uint8)
        arrays[f"out_{k}_offsets"] = offs.astype(np.uint64)
    arrays["current_committee"] = np.frombuffer(cur.ssz, np.uint8)
    arrays["next_committee"] = np.frombuffer(nxt.ssz, np.uint8)
    arrays["genesis_validators_root"] = np.frombuffer(gvr, np.uint8)
    np.savez_compressed(os.path.join(HERE, "producer.npz"), **arrays)
    json.dump({"cases": cases}, open(os.path.join(HERE, "producer.json"), "w"), indent=1)


# ----------------------------------------------------------------------------- non-mainnet configuration
def _oracle_config(cfg):
    """oracle/spec.use_config keywords for a lcv NetworkConfig."""
    from oracle.spec import _CONFIG_NAMES
    return {k: getattr(cfg, k) for k in _CONFIG_NAMES}


def make_testnet_cases():
    """lc_updates_testnet.npz: rows built and signed under a non-mainnet configuration (lcv.config.TESTNET:
    its own fork versions and fork epochs), with the expected reason under that configuration AND under
    mainnet, each from the reference's exec'd blocks (over oracle/spec.py switched to the configuration)
    and the oracle restatement.  Row kinds: Deneb valid / bad signature / corrupted finality branch
    (period 1100: Deneb on both networks, so only the signing domain differs), and a period-600 row
    (Deneb on the testnet, Bellatrix on mainnet: is_valid_light_client_header differs too)."""
    v = H.hostsim_verifier()
    cur, nxt = synth.make_committee(v, 0), synth.make_committee(v, 1)
    comms = (cur, nxt)
    C = Cases()
    SPP = TESTNET.SLOTS_PER_PERIOD
    kinds = np.array([synth.K_VALID, synth.K_BAD_SIG_MESSAGE, synth.K_BAD_FINALITY_BRANCH, synth.K_LOW_PARTICIPATION])
    a = synth.generate(v, len(kinds), seed=41, participation="random", kinds=kinds, committees=comms, cfg=TESTNET)
    for i, k in enumerate(kinds):
        C.add(a.updates, i, f"testnet_deneb_kind{k}", synth.DENEB_PERIOD * SPP, 1, a.current_slot, 1)
    m = synth.generate(v, 1, seed=42, committees=comms, cfg=MAINNET)
    C.add(m.updates, 0, "mainnet_signed_deneb", synth.DENEB_PERIOD * SPP, 1, m.current_slot, 1)
    b = synth.generate(v, 2, seed=43, period=600, committees=comms, cfg=TESTNET)
    C.add(b.updates, 0, "testnet_period600_deneb", 600 * SPP, 1, b.current_slot, 1)
    C.add(b.updates, 1, "testnet_period600_no_next", 600 * SPP, 0, b.current_slot, 1)
    gvr = a.genesis_validators_root
    n = len(C.name)
    pool = np.stack([np.frombuffer(x, np.uint8) for x in (cur.ssz, nxt.ssz, bytes(24624))])
    arrays = {k: np.stack([np.frombuffer(r, np.uint8) for r in C.rows[k]]) for k in COLS}
    from lcv.device import PackedUpdates
    p = PackedUpdates(nsc_pool=pool, nsc_index=np.array(C.pool_row, np.uint32),
                      signature_slot=np.array(C.sig_slot, np.uint64), **arrays)
    expected = {}
    for cfg in (TESTNET, MAINNET):
        with S.use_config(**_oracle_config(cfg)):
            ns, assert_lines = load_reference()
            rs = []
            for i in range(n):
                nxt_bytes = nxt.ssz if C.next_known[i] else bytes(24624)
                store_o = H.store_from(C.store_fin[i], cur.ssz, nxt_bytes)
                r_oracle = H.O.validate_light_client_update(store_o, H.update_from(p, i), C.current_slot[i], gvr)
                store_r, u_r = to_reference_objects(ns, p, i, C.store_fin[i], cur.ssz, nxt_bytes)
                r_ref = reference_reason(ns, assert_lines, store_r, u_r, C.current_slot[i], gvr)
                assert r_oracle == r_ref, (cfg.name, C.name[i], r_oracle, r_ref)
                rs.append(r_ref)
                print(f"{cfg.name:8s} {i:2d} {C.name[i]:32s} reason {r_ref}", flush=True)
            expected[cfg.name] = rs
    assert expected["testnet"] != expected["mainnet"]
    cfgj = {k: (v_.hex() if isinstance(v_, bytes) else v_) for k, v_ in vars(TESTNET).items()}
    np.savez_compressed(os.path.join(HERE, "lc_updates_testnet.npz"), **arrays, nsc_pool=pool,
                        nsc_index=np.array(C.pool_row, np.uint32), signature_slot=np.array(C.sig_slot, np.uint64),
                        store_finalized_slot=np.array(C.store_fin, np.uint64),
                        store_next_known=np.array(C.next_known, np.uint8),
                        current_slot=np.array(C.current_slot, np.uint64),
                        expected_reason_testnet=np.array(expected["testnet"], np.uint8),
                        expected_reason_mainnet=np.array(expected["mainnet"], np.uint8),
                        genesis_validators_root=np.frombuffer(gvr, np.uint8))
    json.dump({"cases": C.name, "config": cfgj, "expected_reason": expected},
              open(os.path.join(HERE, "lc_updates_testnet.json"), "w"), indent=1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "store":
        make_store_sequence()
    elif len(sys.argv) > 1 and sys.argv[1] == "testnet":
        make_testnet_cases()
    elif len(sys.argv) > 1 and sys.argv[1] == "producer":
        make_producer()
    elif len(sys.argv) > 1 and sys.argv[1] == "wire":
        make_wire()
    else:
        main()
        make_store_sequence()
        make_wire()
        make_testnet_cases()
        make_producer()
