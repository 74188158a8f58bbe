"""N > 1 path on CPU: world_size-2 gloo processes shard one batch, validate their shards on the host
simulation of the kernels, and all-gather the verdicts (lcv/multi.py, the same code bench.py's
sharding follows on RCCL)."""
import os
import socket

import numpy as np
import pytest

import helpers as H


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lcv import multi, synth
        v = H.hostsim_verifier()
        kinds = np.array([0, 2, 4, 1, 5, 0, 6])
        sb = synth.generate(v, len(kinds), seed=31, kinds=kinds)  # identical on every rank (seeded)
        v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
        full = multi.validate_sharded(v, sb.updates, sb.current_slot, sb.genesis_validators_root, world, rank)
        q.put((rank, full.tolist(), sb.expected_verdict.tolist()))
    finally:
        dist.destroy_process_group()


def test_shard_bounds():
    from lcv.multi import shard_bounds
    for n in (0, 1, 7, 8, 1000001):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[r][1] == b[r + 1][0] for r in range(w - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1


@pytest.mark.timeout(600)
def test_two_rank_gloo():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=500) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, full, exp in res:
        assert full == exp
