"""BASELINE.json configs[2], [3] and [4] at full size on one GPU, through size-independent properties
(every verdict equals its construction, idempotence of the resident path) plus sampled rows checked
against the CPU oracle (oracle/sync_protocol.py, restating sync-protocol.md:386-465).

  configs[2]: 10^6 updates, random participation 342..512 (the 8-GPU config's whole batch, on one GPU)
  configs[3]: updates with all three branches and a DISTINCT next_sync_committee each (npool = n:
              HTR(SyncCommittee), 1,025 SHA-256 calls, per update: the SHA-256-heavy form)
  configs[4]: 10^6 updates, 10% bad in the SURVEY §8(d) C5 thirds (bad signature message / encoding,
              corrupted finality / next-committee / execution branch, sub-2/3 participation = VALID)

10^6 rows = 16 chunks of 65,536 (the driver's kChunk), so every chunk boundary is crossed.  Rows are
generated on the host (tiled: rows are independent, so copies have identical verdicts).
"""
import os

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu

# LCV_TEST_FULL_N shrinks the batches for a host-simulation dry run (LCV_TEST_HOSTSIM=1)
N_FULL = int(os.environ.get("LCV_TEST_FULL_N", 1 << 20))


def _oracle_rows(sb, rows):
    store = H.store_from(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    return [H.O.validate_light_client_update(store, H.update_from(sb.updates, int(i)), sb.current_slot,
                                             sb.genesis_validators_root) for i in rows]


def _sample(n, k, seed):
    rng = np.random.default_rng(seed)
    chunk = 65536
    # one row per chunk (every chunk of the 10^6 batch), plus random rows, plus the chunk edges
    rows = {int(c * chunk + rng.integers(0, chunk)) for c in range(max(1, n // chunk))}
    rows |= {0, n - 1, chunk - 1, chunk, n // 2}
    rows |= {int(x) for x in rng.integers(0, n, k)}
    return sorted(r for r in rows if r < n)


def test_config4_adversarial_million(gpu_verifier):
    from lcv import synth
    base_n = 16384 if N_FULL >= 16384 else N_FULL
    kinds = synth.adversarial_kinds(base_n, seed=5, bad_fraction=0.10)
    sb0 = synth.generate(gpu_verifier, base_n, seed=5, participation="random", kinds=kinds)
    sb = synth.tile(sb0, N_FULL // base_n)
    assert sb.updates.n == N_FULL
    gpu_verifier.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    rb = gpu_verifier.upload(sb.updates)
    try:
        v, r = gpu_verifier.validate_resident(rb, sb.current_slot, sb.genesis_validators_root)
        assert np.array_equal(r, sb.expected_reason)
        assert np.array_equal(v.astype(bool), sb.expected_reason == 0)
        bad = (sb.expected_reason != 0).mean()
        assert 0.05 < bad < 0.09  # the sub-2/3 third of the 10% stays VALID (only :545 gates it)
        v2, r2 = gpu_verifier.validate_resident(rb, sb.current_slot, sb.genesis_validators_root)
        assert np.array_equal(r2, r)
    finally:
        rb.free()
    rows = _sample(N_FULL, 48, 41)
    assert len(rows) >= min(64, N_FULL // 64)
    assert [int(r[i]) for i in rows] == _oracle_rows(sb, rows)


def test_config2_random_participation_million(gpu_verifier):
    from lcv import synth
    base_n = min(8192, N_FULL)
    sb = synth.tile(synth.generate(gpu_verifier, base_n, seed=3, participation="random"), N_FULL // base_n)
    gpu_verifier.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    pc = np.unpackbits(sb.updates.sync_bits[:base_n], axis=1).sum(1)
    assert pc.min() >= 342 and pc.max() <= 512
    v, r = gpu_verifier.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    assert v.all() and not r.any()
    rows = _sample(N_FULL, 8, 42)
    assert _oracle_rows(sb, rows) == [0] * len(rows)


def test_config3_distinct_next_committees(gpu_verifier):
    from lcv import synth
    n = min(4096, N_FULL)
    kinds = np.zeros(n, np.int64)
    kinds[::97] = synth.K_BAD_NSC_BRANCH
    kinds[5::101] = synth.K_BAD_FINALITY_BRANCH
    sb = synth.generate(gpu_verifier, n, seed=4, kinds=kinds, npool=n)
    assert sb.updates.nsc_pool.shape[0] == n and len(np.unique(sb.updates.nsc_index)) == n
    gpu_verifier.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    v, r = gpu_verifier.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    assert np.array_equal(r, sb.expected_reason)
    rows = sorted({0, 97, 5, 106, n - 1} | set(range(1, n, 509)))
    assert [int(r[i]) for i in rows] == _oracle_rows(sb, rows)
