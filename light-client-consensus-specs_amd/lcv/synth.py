"""Synthetic light-client updates for the benchmark and tests, DERIVED by the producer.

Every row is what a full node would serve: lcv.producer.create_light_client_update (the reference's
full-node.md:138-188, pinned byte-for-byte against the reference's exec'd blocks in
tests/test_producer.py) over a chain finalized block <- attested block <- signature block, each with a
sparse random BeaconState view (every state field but the five light clients read is a random root).
So the finality branch (gindex 105), next-sync-committee branch (gindex 55), execution branches
(gindex 25) and signing root are all consistent with real state / block trees.

The sync aggregate signature is (sum of participant secret keys) * H(signing_root), computed by the
device signer (`Verifier.sign_batch`), so generating 10^4..10^6 validly signed updates is cheap.
SHA-256 for the trees runs on the host (hashlib): this is input generation, outside every timed
region, and is never the verified path.

Corruption kinds (BASELINE.json config 5): each row has a `kind`; the expected verdict follows.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, replace
from typing import Optional

import numpy as np

from . import config as _config
from . import layout as L
from . import producer as PR
from .producer import fold_branch, htr_beacon, htr_exec_record, htr_pubkey, htr_sync_committee, merkleize  # noqa: F401
from .config import NetworkConfig
from .device import PackedUpdates, Verifier

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
# network values come from a NetworkConfig (lcv.config; the active one unless given)
DENEB_PERIOD = 1100    # slot 9,011,200: a Deneb-era sync-committee period
CAPELLA_PERIOD = 1000  # slot 8,192,000: a Capella-era period

# row kinds
K_VALID = 0
K_LOW_PARTICIPATION = 1    # popcount in [1, 341]: VALID (2/3 only gates apply, sync-protocol.md:545)
K_BAD_SIG_MESSAGE = 2      # signature over a different message          -> reason 14
K_BAD_SIG_ENCODING = 3     # undecodable signature (x >= p)              -> reason 14
K_BAD_FINALITY_BRANCH = 4  # corrupted finality branch byte              -> reason 10
K_BAD_NSC_BRANCH = 5       # corrupted next-sync-committee branch byte   -> reason 13
K_BAD_EXEC_BRANCH = 6      # corrupted attested execution branch byte    -> reason 2
K_NO_PARTICIPANTS = 7      # all bits zero                               -> reason 1
EXPECTED_REASON = {K_VALID: 0, K_LOW_PARTICIPATION: 0, K_BAD_SIG_MESSAGE: 14, K_BAD_SIG_ENCODING: 14,
                   K_BAD_FINALITY_BRANCH: 10, K_BAD_NSC_BRANCH: 13, K_BAD_EXEC_BRANCH: 2, K_NO_PARTICIPANTS: 1}


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def signing_root(att_beacon: bytes, signature_slot: int, gvr: bytes, cfg: Optional[NetworkConfig] = None) -> bytes:
    """compute_signing_root(attested beacon, compute_domain(DOMAIN_SYNC_COMMITTEE, fork_version, gvr))
    (sync-protocol.md:460-463) under `cfg` (the active configuration by default)."""
    cfg = cfg or _config.active()
    fslot = max(int(signature_slot), 1) - 1
    fdr = sha256(cfg.compute_fork_version(cfg.compute_epoch_at_slot(fslot)) + bytes(28) + gvr)
    domain = cfg.DOMAIN_SYNC_COMMITTEE + fdr[:28]
    return sha256(htr_beacon(att_beacon) + domain)


def derive_secret_keys(seed: int, n: int = 512):
    out = []
    for j in range(n):
        k = int.from_bytes(sha256(b"lcv-synthetic-sk" + seed.to_bytes(8, "little") + j.to_bytes(4, "little")), "big")
        out.append(k % (R_ORDER - 1) + 1)
    return out


@dataclass
class Committee:
    sks: list
    pubkeys: bytes  # 512 x 48
    aggregate_pubkey: bytes

    @property
    def ssz(self) -> bytes:
        return self.pubkeys + self.aggregate_pubkey


def make_committee(verifier: Verifier, seed: int) -> Committee:
    sks = derive_secret_keys(seed)
    skb = np.frombuffer(b"".join(k.to_bytes(32, "big") for k in sks), np.uint8)
    pks = verifier.sk_to_pk_batch(skb).tobytes()
    agg = verifier.sk_to_pk_batch(np.frombuffer((sum(sks) % R_ORDER).to_bytes(32, "big"), np.uint8)).tobytes()
    return Committee(sks, pks, agg)


@dataclass
class SyntheticBatch:
    updates: PackedUpdates
    kinds: np.ndarray            # (n,) row kind
    expected_reason: np.ndarray  # (n,) u8
    store_finalized_slot: int
    current: Committee
    next: Committee
    current_slot: int
    genesis_validators_root: bytes

    @property
    def expected_verdict(self) -> np.ndarray:
        return self.expected_reason == 0


def _rand_exec(rng: np.random.Generator, deneb: bool) -> bytes:
    """A random execution record (include/lcv.h layout) from one draw of random bytes."""
    r = rng.bytes(7 * 32 + 20 + 4 * 8 + 1 + 32 + 8 + 256 + 16)
    rec = bytearray(L.EXEC_BYTES)
    for j, k in enumerate((0, 2, 3, 5, 12, 13, 14)):
        rec[32 * k:32 * k + 32] = r[32 * j:32 * j + 32]
    o = 224
    rec[32:52] = r[o:o + 20]                                                 # fee_recipient
    o += 20
    for k in (6, 7, 8, 9):                                                   # u64 fields (< 2^62)
        rec[32 * k:32 * k + 8] = r[o:o + 7] + bytes([r[o + 7] & 0x3F])
        o += 8
    elen = r[o] % 33
    o += 1
    rec[320:320 + elen] = r[o:o + elen]                                      # extra_data
    o += 32
    rec[L.EXEC_EXTRALEN_OFF:L.EXEC_EXTRALEN_OFF + 4] = elen.to_bytes(4, "little")
    rec[352:352 + 8] = r[o:o + 7] + bytes([r[o + 7] & 0x3F])                 # base_fee_per_gas
    o += 8
    rec[L.EXEC_BLOOM_OFF:L.EXEC_BLOOM_OFF + 256] = r[o:o + 256]
    o += 256
    if deneb:                                                                # blob gas (< 2^20)
        rec[480:483] = r[o:o + 2] + bytes([r[o + 2] & 0x0F])
        rec[512:515] = r[o + 8:o + 10] + bytes([r[o + 10] & 0x0F])
    return bytes(rec)


def _header(rng, slot: int, cfg: NetworkConfig):
    """Random LightClientHeader at `slot` with a valid execution branch (body root derived); before
    Capella the execution header and branch are empty (as upgraded Altair headers are)."""
    epoch = cfg.compute_epoch_at_slot(slot)
    if epoch < cfg.CAPELLA_FORK_EPOCH:
        return slot, bytes(L.EXEC_BYTES), bytes(128), rng.bytes(32)
    deneb = epoch >= cfg.DENEB_FORK_EPOCH
    ex = _rand_exec(rng, deneb)
    br = [rng.bytes(32) for _ in range(4)]
    body = fold_branch(htr_exec_record(ex, deneb), br, 9)
    return slot, ex, b"".join(br), body


def _rand_body_roots(rng) -> np.ndarray:
    return np.frombuffer(rng.bytes(32 * PR.BODY_FIELDS), np.uint8).reshape(PR.BODY_FIELDS, 32)


def _rand_state_roots(rng) -> np.ndarray:
    return np.frombuffer(rng.bytes(32 * PR.STATE_FIELDS), np.uint8).reshape(PR.STATE_FIELDS, 32)


def _block(rng, slot: int, cfg: NetworkConfig, parent_root: Optional[bytes] = None, bits: bytes = b"\xff" * 64,
           sig: bytes = bytes(96), payload: bool = True) -> PR.BeaconBlockView:
    """A block view at `slot` with random body contents (an execution payload from Capella on; a block
    whose light-client header is never taken, payload=False, keeps its payload by root only)."""
    epoch = cfg.compute_epoch_at_slot(slot)
    ex = _rand_exec(rng, epoch >= cfg.DENEB_FORK_EPOCH) if payload and epoch >= cfg.CAPELLA_FORK_EPOCH else None
    return PR.BeaconBlockView(slot=slot, proposer_index=int(rng.integers(0, 2 ** 20)),
                              parent_root=parent_root if parent_root is not None else rng.bytes(32),
                              state_root=bytes(32), sync_committee_bits=bits, sync_committee_signature=sig,
                              execution=ex, execution_deneb=epoch >= cfg.DENEB_FORK_EPOCH,
                              body_roots=_rand_body_roots(rng))


def _with_state(rng, blk: PR.BeaconBlockView, fin_epoch: int, fin_root: bytes, cur: bytes, nxt: bytes):
    """(post-state view, block view with its state_root) for `blk`: the state's latest_block_header is
    the block's header with a zero state_root (as a state holds it)."""
    hdr = blk.header()
    st = PR.BeaconStateView(slot=blk.slot, latest_block_header=hdr[:48] + bytes(32) + hdr[80:],
                            finalized_checkpoint_epoch=fin_epoch, finalized_checkpoint_root=fin_root,
                            current_sync_committee=cur, next_sync_committee=nxt, field_roots=_rand_state_roots(rng))
    return st, replace(blk, state_root=st.hash_tree_root())


def generate(verifier: Verifier, n: int, seed: int = 2, period: int = DENEB_PERIOD, participation: str = "full",
             kinds: Optional[np.ndarray] = None, with_next: bool = True, with_finality: bool = True,
             committees=None, gvr: Optional[bytes] = None, sign_next: bool = False, npool: int = 1,
             cfg: Optional[NetworkConfig] = None) -> SyntheticBatch:
    """n synthetic updates against one store (finalized at the first slot of `period`, both
    committees known), each DERIVED by the producer (lcv.producer.create_light_client_update, the
    reference's full-node.md:138-188) from a chain finalized block <- ... attested block <- signature
    block with sparse random states.  participation: "full" (512/512) or "random" (popcount uniform in
    [342,512]).  kinds: optional per-row corruption kinds (see K_*), applied to the derived rows.
    sign_next: signature slots in the next period, signed by the next committee (sync-protocol.md:452-455
    selects it; the producer then leaves out next_sync_committee, full-node.md:165-168).  with_next=False
    clears the next-committee fields of same-period rows (a provider that omits them); with_finality=False
    derives without a finalized block.  npool > 1 (BASELINE configs[3], the SHA-256-heavy form): update i
    carries next_sync_committee number i % npool out of npool distinct committees (HTR(SyncCommittee),
    1,025 SHA-256 calls, then runs once per distinct value); the store's next committee is then unknown,
    as :441-442 would otherwise demand equality with it.
    cfg: the network configuration the rows are built and signed under (default: lcv.config.active())."""
    cfg = cfg or _config.active()
    spp, spe = cfg.SLOTS_PER_PERIOD, cfg.SLOTS_PER_EPOCH
    rng = np.random.default_rng(seed)
    cur, nxt = committees if committees is not None else (make_committee(verifier, 0), make_committee(verifier, 1))
    gvr = gvr if gvr is not None else sha256(b"lcv-synthetic-genesis-validators-root")
    kinds = np.zeros(n, np.int64) if kinds is None else np.asarray(kinds, np.int64)
    store_fin = period * spp
    if npool > 1:
        if sign_next:
            raise ValueError("npool > 1 needs the store's next committee unknown (no next-period signing)")
        prng = np.random.default_rng(seed + 1000)
        pool_bytes = prng.integers(0, 256, (npool, L.SYNC_COMMITTEE_BYTES), dtype=np.uint8)
        for k, r in enumerate(verifier.htr_sync_committee_batch(pool_bytes)):  # device HTR, seeds the memo
            PR._SC_ROOTS[sha256(pool_bytes[k].tobytes())] = bytes(r)
        store_next = Committee([], bytes(512 * 48), bytes(48))  # is_next_sync_committee_known: False
    signer = nxt if sign_next else cur
    total_sk = sum(signer.sks) % R_ORDER

    # pass 1: finalized and attested blocks + states, the participation and the message to sign
    pending, msgs, sk_sums, bitss = [], bytearray(32 * n), bytearray(32 * n), []
    for i in range(n):
        kind = int(kinds[i])
        att_slot = store_fin + 64 + int(rng.integers(0, spp - 256))
        ss = att_slot + 1 + int(rng.integers(0, 64))
        if sign_next:
            ss = store_fin + spp + int(rng.integers(0, 64))
        fin_blk = None
        if with_finality:
            fin_slot = store_fin + int(rng.integers(0, att_slot - store_fin - 32))
            fin_blk = _block(rng, fin_slot, cfg)
            fin_epoch, fin_root = fin_slot // spe, fin_blk.hash_tree_root()
        else:
            fin_epoch, fin_root = int(rng.integers(0, store_fin // spe)), rng.bytes(32)
        nsc = pool_bytes[i % npool].tobytes() if npool > 1 else nxt.ssz
        att_state, att_blk = _with_state(rng, _block(rng, att_slot, cfg), fin_epoch, fin_root, cur.ssz, nsc)
        if kind == K_NO_PARTICIPANTS:
            bits = np.zeros(512, np.uint8)
        elif kind == K_LOW_PARTICIPATION:
            bits = np.zeros(512, np.uint8)
            bits[rng.choice(512, int(rng.integers(1, 342)), replace=False)] = 1
        elif participation == "random":
            bits = np.zeros(512, np.uint8)
            bits[rng.choice(512, int(rng.integers(342, 513)), replace=False)] = 1
        else:
            bits = np.ones(512, np.uint8)
        sks = total_sk if bits.all() else (total_sk - sum(signer.sks[j] for j in np.flatnonzero(bits == 0))) % R_ORDER
        m = signing_root(att_blk.header(), ss, gvr, cfg)
        if kind == K_BAD_SIG_MESSAGE:
            m = sha256(b"not-the-signing-root" + m)
        msgs[32 * i:32 * i + 32] = m
        sk_sums[32 * i:32 * i + 32] = (sks or 1).to_bytes(32, "big")
        bitss.append(np.packbits(bits, bitorder="little").tobytes())
        pending.append((ss, fin_blk, att_state, att_blk))
    sigs = verifier.sign_batch(np.frombuffer(bytes(sk_sums), np.uint8), np.frombuffer(bytes(msgs), np.uint8))
    for i in np.flatnonzero(kinds == K_BAD_SIG_ENCODING):
        sigs[i, 0] = 0x9a  # compression flag set, x1 >= p
        sigs[i, 1:48] = 0xff

    # pass 2: the signature blocks (carrying the sync aggregates), their states, the derived updates
    rows = []
    for i, (ss, fin_blk, att_state, att_blk) in enumerate(pending):
        kind = int(kinds[i])
        # (a block without participants cannot be derived from, full-node.md:146: K_NO_PARTICIPANTS rows are
        # derived with one bit and then cleared, a corruption like the others)
        bits = b"\x01" + bytes(63) if kind == K_NO_PARTICIPANTS else bitss[i]
        blk = _block(rng, ss, cfg, parent_root=att_blk.hash_tree_root(), bits=bits, sig=sigs[i].tobytes(),
                     payload=False)
        st, blk = _with_state(rng, blk, att_state.finalized_checkpoint_epoch, att_state.finalized_checkpoint_root,
                              cur.ssz, att_state.next_sync_committee)
        u = PR.create_light_client_update(st, blk, att_state, att_blk, fin_blk, cfg)
        if kind == K_NO_PARTICIPANTS:
            u.sync_committee_bits = bytes(64)
        if not with_next:
            u.next_sync_committee = PR.EMPTY_SYNC_COMMITTEE
            u.next_sync_committee_branch = bytes(L.NSC_BRANCH_BYTES)
        if kind == K_BAD_FINALITY_BRANCH and with_finality:
            u.finality_branch = _flip(u.finality_branch, int(rng.integers(0, 192)), 0x01)
        if kind == K_BAD_NSC_BRANCH and with_next and not sign_next:
            u.next_sync_committee_branch = _flip(u.next_sync_committee_branch, int(rng.integers(0, 160)), 0x80)
        if kind == K_BAD_EXEC_BRANCH:
            h = u.attested_header
            u.attested_header = PR.HeaderRow(h.beacon, h.execution, _flip(h.execution_branch, int(rng.integers(0, 128)), 0x10))
        rows.append(u)
    upd = PR.pack_updates(rows)
    expected = np.array([EXPECTED_REASON[int(k)] for k in kinds], np.uint8)
    current_slot = int(upd.signature_slot.max()) if n else store_fin + 1
    return SyntheticBatch(upd, kinds, expected, store_fin, cur, store_next if npool > 1 else nxt, current_slot, gvr)


def _flip(b: bytes, j: int, mask: int) -> bytes:
    return b[:j] + bytes([b[j] ^ mask]) + b[j + 1:]


def tile(sb: SyntheticBatch, reps: int) -> SyntheticBatch:
    """`reps` copies of a generated batch back to back (the 10^6-row configs: rows are independent,
    so a tiled batch has the same per-row verdicts; generating 10^6 distinct rows on the host would
    dominate a test's time).  The next-committee pool is shared, not copied."""
    u = sb.updates
    cols = {k: np.ascontiguousarray(np.tile(getattr(u, k), (reps, 1))) for k in (
        "att_beacon", "att_exec", "att_branch", "fin_beacon", "fin_exec", "fin_branch", "nsc_branch",
        "finality_branch", "sync_bits", "sync_signature")}
    upd = PackedUpdates(nsc_pool=u.nsc_pool, nsc_index=np.tile(u.nsc_index, reps),
                        signature_slot=np.tile(u.signature_slot, reps), **cols)
    return SyntheticBatch(upd, np.tile(sb.kinds, reps), np.tile(sb.expected_reason, reps), sb.store_finalized_slot,
                          sb.current, sb.next, sb.current_slot, sb.genesis_validators_root)


def adversarial_kinds(n: int, seed: int = 5, bad_fraction: float = 0.10) -> np.ndarray:
    """BASELINE.json config 5: `bad_fraction` of rows bad, in equal thirds: bad signatures (message /
    encoding), corrupted branches (finality / next-committee / execution), sub-2/3 participation."""
    rng = np.random.default_rng(seed)
    kinds = np.zeros(n, np.int64)
    nbad = int(round(n * bad_fraction))
    rows = rng.choice(n, nbad, replace=False)
    pool = [K_BAD_SIG_MESSAGE, K_BAD_SIG_ENCODING, K_BAD_FINALITY_BRANCH, K_BAD_NSC_BRANCH, K_BAD_EXEC_BRANCH,
            K_LOW_PARTICIPATION]
    weights = np.array([1 / 6, 1 / 6, 1 / 9, 1 / 9, 1 / 9, 1 / 3])
    kinds[rows] = rng.choice(pool, nbad, p=weights / weights.sum())
    return kinds
