"""Synthetic mainnet-preset light-client updates (producer side), for the benchmark and tests.

Follows the producer semantics of `create_light_client_update` (reference full-node.md:138-182):
every update carries an attested header, a finalized header with its finality branch (gindex 105),
the next sync committee with its branch (gindex 55) and Deneb execution branches (gindex 25), all
consistent with ONE sparse BeaconState tree per update:

    state root = node 1;  finality branch  = [n104, n53, n27, n12, n7, n2]   (leaf n105)
                          next-SC branch   = [n54, n26, n12, n7, n2]          (leaf n55)
    n27 = H(n54 = HTR(current_sync_committee), n55 = HTR(next_sync_committee))
    body root: execution branch = [n24, n13, n7, n2] (leaf n25 = HTR(execution header))

The sync aggregate signature is (sum of participant secret keys) * H(signing_root), computed by the
device signer (`Verifier.sign_batch`), so generating 10^4..10^6 validly signed updates is cheap.
SHA-256 for the synthetic trees runs on the host (hashlib): this is input generation, outside every
timed region, and is never the verified path.

Corruption kinds (BASELINE.json config 5): each row has a `kind`; the expected verdict follows.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import config as _config
from . import layout as L
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


def _zero_hashes(n: int = 8):
    z = [bytes(32)]
    for _ in range(n):
        z.append(sha256(z[-1] + z[-1]))
    return z


ZH = _zero_hashes()


def merkleize(chunks, depth: int) -> bytes:
    layer = list(chunks)
    for d in range(depth):
        if len(layer) % 2:
            layer.append(ZH[d])
        layer = [sha256(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def htr_beacon(b112: bytes) -> bytes:
    chunks = [b112[0:8] + bytes(24), b112[8:16] + bytes(24), b112[16:48], b112[48:80], b112[80:112]]
    return merkleize(chunks, 3)


def htr_exec_record(rec: bytes, deneb: bool) -> bytes:
    """hash_tree_root of the ExecutionPayloadHeader held in an 832-byte execution record."""
    bloom = rec[L.EXEC_BLOOM_OFF:L.EXEC_BLOOM_OFF + 256]
    bloom_root = merkleize([bloom[32 * k:32 * k + 32] for k in range(8)], 3)
    ext_len = int.from_bytes(rec[L.EXEC_EXTRALEN_OFF:L.EXEC_EXTRALEN_OFF + 4], "little")
    extra_root = sha256(rec[320:352] + ext_len.to_bytes(8, "little") + bytes(24))
    nf = 17 if deneb else 15
    leaves = []
    for k in range(nf):
        if k == 4:
            leaves.append(bloom_root)
        elif k == 10:
            leaves.append(extra_root)
        else:
            leaves.append(rec[32 * k:32 * k + 32])
    return merkleize(leaves, 5 if deneb else 4)


def fold_branch(leaf: bytes, branch, index: int) -> bytes:
    v = leaf
    for i, b in enumerate(branch):
        v = sha256(b + v) if (index >> i) & 1 else sha256(v + b)
    return v


def htr_pubkey(pk: bytes) -> bytes:
    return sha256(pk[:32] + pk[32:48] + bytes(16))


def htr_sync_committee(sc: bytes) -> bytes:
    roots = [htr_pubkey(sc[48 * j:48 * j + 48]) for j in range(512)]
    return sha256(merkleize(roots, 9) + htr_pubkey(sc[512 * 48:]))


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
    rec = bytearray(L.EXEC_BYTES)
    for k in (0, 2, 3, 5, 12, 13, 14):
        rec[32 * k:32 * k + 32] = rng.bytes(32)
    rec[32:52] = rng.bytes(20)                                              # fee_recipient
    for k in (6, 7, 8, 9):
        rec[32 * k:32 * k + 8] = int(rng.integers(0, 2 ** 62)).to_bytes(8, "little")
    elen = int(rng.integers(0, 33))
    rec[320:320 + elen] = rng.bytes(elen)                                   # extra_data
    rec[L.EXEC_EXTRALEN_OFF:L.EXEC_EXTRALEN_OFF + 4] = elen.to_bytes(4, "little")
    rec[352:352 + 32] = int(rng.integers(0, 2 ** 62)).to_bytes(32, "little")  # base_fee_per_gas
    rec[L.EXEC_BLOOM_OFF:L.EXEC_BLOOM_OFF + 256] = rng.bytes(256)
    if deneb:
        rec[480:488] = int(rng.integers(0, 2 ** 20)).to_bytes(8, "little")
        rec[512:520] = int(rng.integers(0, 2 ** 20)).to_bytes(8, "little")
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


def generate(verifier: Verifier, n: int, seed: int = 2, period: int = DENEB_PERIOD, participation: str = "full",
             kinds: Optional[np.ndarray] = None, with_next: bool = True, with_finality: bool = True,
             committees=None, gvr: Optional[bytes] = None, sign_next: bool = False, npool: int = 1,
             cfg: Optional[NetworkConfig] = None) -> SyntheticBatch:
    """n synthetic updates against one store (finalized at the first slot of `period`, both
    committees known).  participation: "full" (512/512) or "random" (popcount uniform in [342,512]).
    kinds: optional per-row corruption kinds (see K_*).  sign_next: signature slots in the next period,
    signed by the next committee (sync-protocol.md:452-455 selects it).  npool > 1 (BASELINE configs[3],
    the SHA-256-heavy form): update i carries next_sync_committee number i % npool out of npool
    distinct committees (HTR(SyncCommittee), 1,025 SHA-256 calls, then runs once per distinct value);
    the store's next committee is then unknown, as :441-442 would otherwise demand equality with it.
    cfg: the network configuration the rows are built and signed under (default: lcv.config.active())."""
    cfg = cfg or _config.active()
    SLOTS_PER_PERIOD = cfg.SLOTS_PER_PERIOD
    rng = np.random.default_rng(seed)
    cur, nxt = committees if committees is not None else (make_committee(verifier, 0), make_committee(verifier, 1))
    gvr = gvr if gvr is not None else sha256(b"lcv-synthetic-genesis-validators-root")
    kinds = np.zeros(n, np.int64) if kinds is None else np.asarray(kinds, np.int64)
    store_fin = period * SLOTS_PER_PERIOD
    if npool > 1:
        if sign_next:
            raise ValueError("npool > 1 needs the store's next committee unknown (no next-period signing)")
        prng = np.random.default_rng(seed + 1000)
        pool_bytes = prng.integers(0, 256, (npool, L.SYNC_COMMITTEE_BYTES), dtype=np.uint8)
        pool_roots = [bytes(r) for r in verifier.htr_sync_committee_batch(pool_bytes)]
        store_next = Committee([], bytes(512 * 48), bytes(48))  # is_next_sync_committee_known: False
    nsc_root = htr_sync_committee(nxt.ssz)
    cur_root = htr_sync_committee(cur.ssz)
    signer = nxt if sign_next else cur
    total_sk = sum(signer.sks) % R_ORDER

    cols = {k: np.zeros((n, w), np.uint8) for k, w in (("att_beacon", 112), ("att_exec", 832), ("att_branch", 128),
                                                       ("fin_beacon", 112), ("fin_exec", 832), ("fin_branch", 128),
                                                       ("nsc_branch", 160), ("finality_branch", 192),
                                                       ("sync_bits", 64), ("sync_signature", 96))}
    sig_slot = np.zeros(n, np.uint64)
    msgs = bytearray(32 * n)
    sk_sums = bytearray(32 * n)
    for i in range(n):
        kind = int(kinds[i])
        att_slot = store_fin + 64 + int(rng.integers(0, SLOTS_PER_PERIOD - 256))
        ss = att_slot + 1 + int(rng.integers(0, 64))
        if sign_next:
            ss = store_fin + SLOTS_PER_PERIOD + int(rng.integers(0, 64))
        fin_slot = store_fin + int(rng.integers(0, att_slot - store_fin - 32)) if with_finality else 0
        a_slot, a_ex, a_br, a_body = _header(rng, att_slot, cfg)
        # sparse state tree (see module docstring)
        if with_finality:
            f_slot, f_ex, f_br, f_body = _header(rng, fin_slot, cfg)
            f_beacon = (f_slot.to_bytes(8, "little") + int(rng.integers(0, 2 ** 20)).to_bytes(8, "little")
                        + rng.bytes(32) + rng.bytes(32) + f_body)
            fin_leaf = htr_beacon(f_beacon)
        else:
            f_ex, f_br, f_beacon, fin_leaf = bytes(832), bytes(128), bytes(112), None
        n104, n53, n12, n7, n2 = (rng.bytes(32) for _ in range(5))
        n55 = (pool_roots[i % npool] if npool > 1 else nsc_root) if with_next else rng.bytes(32)
        n27 = sha256(cur_root + n55)
        if with_finality:
            n52 = sha256(n104 + fin_leaf)
        else:
            n52 = rng.bytes(32)
        n26 = sha256(n52 + n53)
        n13 = sha256(n26 + n27)
        n6 = sha256(n12 + n13)
        n3 = sha256(n6 + n7)
        state_root = sha256(n2 + n3)
        a_beacon = (a_slot.to_bytes(8, "little") + int(rng.integers(0, 2 ** 20)).to_bytes(8, "little")
                    + rng.bytes(32) + state_root + a_body)
        fin_branch = n104 + n53 + n27 + n12 + n7 + n2 if with_finality else bytes(192)
        nsc_branch = cur_root + n26 + n12 + n7 + n2 if with_next else bytes(160)
        # participation
        if kind == K_NO_PARTICIPANTS:
            bits = np.zeros(512, np.uint8)
        elif kind == K_LOW_PARTICIPATION:
            pc = int(rng.integers(1, 342))
            bits = np.zeros(512, np.uint8)
            bits[rng.choice(512, pc, replace=False)] = 1
        elif participation == "random":
            pc = int(rng.integers(342, 513))
            bits = np.zeros(512, np.uint8)
            bits[rng.choice(512, pc, replace=False)] = 1
        else:
            bits = np.ones(512, np.uint8)
        if bits.all():
            sks = total_sk
        else:
            sks = (total_sk - sum(signer.sks[j] for j in np.flatnonzero(bits == 0))) % R_ORDER
        m = signing_root(a_beacon, ss, gvr, cfg)
        if kind == K_BAD_SIG_MESSAGE:
            m = sha256(b"not-the-signing-root" + m)
        # corruptions of the byte records
        if kind == K_BAD_FINALITY_BRANCH and with_finality:
            j = int(rng.integers(0, 192))
            fin_branch = fin_branch[:j] + bytes([fin_branch[j] ^ 0x01]) + fin_branch[j + 1:]
        if kind == K_BAD_NSC_BRANCH and with_next:
            j = int(rng.integers(0, 160))
            nsc_branch = nsc_branch[:j] + bytes([nsc_branch[j] ^ 0x80]) + nsc_branch[j + 1:]
        if kind == K_BAD_EXEC_BRANCH:
            j = int(rng.integers(0, 128))
            a_br = a_br[:j] + bytes([a_br[j] ^ 0x10]) + a_br[j + 1:]
        cols["att_beacon"][i] = np.frombuffer(a_beacon, np.uint8)
        cols["att_exec"][i] = np.frombuffer(a_ex, np.uint8)
        cols["att_branch"][i] = np.frombuffer(a_br, np.uint8)
        cols["fin_beacon"][i] = np.frombuffer(f_beacon, np.uint8)
        cols["fin_exec"][i] = np.frombuffer(f_ex, np.uint8)
        cols["fin_branch"][i] = np.frombuffer(f_br, np.uint8)
        cols["nsc_branch"][i] = np.frombuffer(nsc_branch, np.uint8)
        cols["finality_branch"][i] = np.frombuffer(fin_branch, np.uint8)
        cols["sync_bits"][i] = np.packbits(bits, bitorder="little")
        sig_slot[i] = ss
        msgs[32 * i:32 * i + 32] = m
        sk_sums[32 * i:32 * i + 32] = (sks or 1).to_bytes(32, "big")
    sigs = verifier.sign_batch(np.frombuffer(bytes(sk_sums), np.uint8), np.frombuffer(bytes(msgs), np.uint8))
    for i in np.flatnonzero(kinds == K_BAD_SIG_ENCODING):
        sigs[i, 0] = 0x9a  # compression flag set, x1 >= p
        sigs[i, 1:48] = 0xff
    cols["sync_signature"][:] = sigs
    if npool > 1 and with_next:
        nsc_pool, nsc_index = pool_bytes, (np.arange(n) % npool).astype(np.uint32)
    else:
        nsc_pool = np.frombuffer(nxt.ssz if with_next else bytes(L.SYNC_COMMITTEE_BYTES), np.uint8).reshape(1, -1).copy()
        nsc_index = np.zeros(n, np.uint32)
    upd = PackedUpdates(nsc_pool=nsc_pool, nsc_index=nsc_index, signature_slot=sig_slot, **cols)
    expected = np.array([EXPECTED_REASON[int(k)] for k in kinds], np.uint8)
    current_slot = int(sig_slot.max()) if n else store_fin + 1
    return SyntheticBatch(upd, kinds, expected, store_fin, cur, store_next if npool > 1 else nxt, current_slot, gvr)


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
