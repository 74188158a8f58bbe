"""N > 1 path on CPU: world_size-2 processes shard one batch, validate their shards on the host
simulation of the kernels and all-gather the verdicts through lcv/multi.py's Comm — the same code and
C ABI (lcv_comm_init, lcv_validate_sharded, lcv_slot_allgather, lcv_comm_allreduce_max) bench.py runs over RCCL on the
GPUs; the host simulation's stand-in collective exchanges files.  A gloo run (torch.distributed) of
the same shards checks the gathered verdicts independently."""
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
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lcv import multi, synth
        v = H.hostsim_verifier()
        # 7 rows over 2 ranks; 8 k + 5 = 21 rows over 8 ranks (north_star's width): uneven shards, padded slices
        kinds = np.array([0, 2, 4, 1, 5, 0, 6] * (1 if world <= 2 else 3))
        sb = synth.generate(v, len(kinds), seed=31, kinds=kinds)  # identical on every rank (seeded)
        v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
        comm = multi.Comm(v, world, rank, key=f"test_{port}")
        full = multi.validate_sharded(v, sb.updates, sb.current_slot, sb.genesis_validators_root, comm)
        t = comm.allreduce_max(float(rank + 1))
        # independent check: gloo all-gather of the same shards' verdicts
        lo, hi = multi.shard_bounds(sb.updates.n, world, rank)
        # two batches in flight (bench.py's serving loop): the shard in both work-space slots, the
        # verdicts gathered per slot (lcv_slot_allgather)
        rb = v.upload(sb.updates.slice(lo, hi))
        per_rank = -(-sb.updates.n // world)
        for s in (0, 1):
            v.validate_resident_async(rb, sb.current_slot, sb.genesis_validators_root, s)
        slots = [multi.unshard(comm.slot_allgather(s, hi - lo, per_rank), sb.updates.n, world).astype(bool).tolist()
                 for s in (0, 1)]
        ok, _ = v.validate(sb.updates.slice(lo, hi), sb.current_slot, sb.genesis_validators_root)
        per = -(-sb.updates.n // world)
        buf = torch.zeros(per, dtype=torch.uint8)
        buf[:hi - lo] = torch.from_numpy(ok.astype(np.uint8))
        parts = [torch.zeros(per, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, buf)
        gloo = multi.unshard(torch.cat(parts).numpy(), sb.updates.n, world).astype(bool)
        comm.close()
        q.put((rank, full.tolist(), gloo.tolist(), sb.expected_verdict.tolist(), t, slots))
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


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 8])
def test_two_rank_gloo(world):
    """world 2, and world 8 (the north_star's 8-GPU split) with 8 k + 5 rows: every rank's gathered verdicts
    (validate_sharded and the per-slot all-gathers) equal the construction, the gloo all-gather of the same
    shards and the single-rank result."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=800) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert sorted(r[0] for r in res) == list(range(world))
    for rank, full, gloo, exp, t, slots in res:
        assert full == exp == gloo == slots[0] == slots[1]
        assert t == float(world)


def _inject_failure(multi, dead, mode):
    """Failure injection for the worker of original rank `dead` (a monkeypatch inside that process, so
    the product code carries no test hook): at its first collective (recovery epoch 0) the rank exits
    ("exit", status 17) or stops itself with SIGSTOP ("hang": it stays alive, holds its files and never
    answers, so the survivors' bounded wait is what fires)."""
    import signal
    orig = multi.Comm.validate_sharded

    def validate_sharded(self, *a, **k):
        if self.ranks[self.rank] == dead and self.epoch == 0:
            if mode == "exit":
                os._exit(17)
            os.kill(os.getpid(), signal.SIGSTOP)
        return orig(self, *a, **k)

    multi.Comm.validate_sharded = validate_sharded


def _fail_worker(rank, world, dead, port, q, recovery="reinit", mode="exit"):
    """Rank `dead` dies (or hangs) before its collective; the survivors' collective times out
    (communicator timeout 3 s), they agree on who is left and move onto a new communicator — recovery
    "reinit" (abort + a fresh communicator among themselves, the path RCCL 2.27 takes) or "shrink" — and
    re-validate the batch over themselves."""
    from lcv import multi, synth
    _inject_failure(multi, dead, mode)
    v = H.hostsim_verifier()
    kinds = np.array([0, 2, 4, 1, 5, 0, 6, 3, 0, 1, 0])
    sb = synth.generate(v, len(kinds), seed=33, kinds=kinds)
    v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    comm = multi.Comm(v, world, rank, key=f"fail_{port}", timeout=3.0, recovery=recovery)
    full = multi.validate_sharded(v, sb.updates, sb.current_slot, sb.genesis_validators_root, comm, grace=3.0)
    single, _ = v.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    t = comm.allreduce_max(float(rank + 1))  # the new communicator keeps working
    q.put((rank, full.tolist(), single.astype(bool).tolist(), sb.expected_verdict.tolist(), comm.world, comm.ranks, t,
           comm.last_recovery))
    comm.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,dead,recovery,mode", [(2, 1, "reinit", "exit"), (4, 2, "reinit", "exit"),
                                                      (4, 1, "shrink", "exit"), (3, 1, "reinit", "hang")])
def test_rank_failure_recovery(world, dead, recovery, mode):
    """SURVEY.md §5 (a GPU failing in a shard -> rerun the shard): with one rank dead — or hung, stopped
    by SIGSTOP, so that only the bounded collective wait can notice it — mid-batch the survivors return,
    and their verdicts equal the single-rank result."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, dead, port, q, recovery, mode)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=500) for _ in range(world - 1)]
        for r, p in enumerate(procs):
            if r == dead and mode == "hang":
                continue
            p.join(120)
            assert p.exitcode == (17 if r == dead else 0), (r, p.exitcode)
    finally:
        for p in procs:  # the stopped rank (and anything left after a failure) is killed by its own handle
            if p.is_alive():
                p.kill()
                p.join(30)
    survivors = [r for r in range(world) if r != dead]
    assert sorted(x[0] for x in res) == survivors
    for rank, full, single, exp, w, ranks, t, how in res:
        assert full == single == exp
        assert w == world - 1 and ranks == survivors
        assert t == float(max(survivors) + 1)  # the all-reduce over the survivors (original rank + 1)
        assert how.startswith(recovery)
