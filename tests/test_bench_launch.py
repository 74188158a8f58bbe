"""bench.py's multi-GPU launch on CPU (a SCALE run must not be able to report a 1-GPU number
under an N-GPU label).  `bench.py --gpus 2` without a launcher spawns two rank processes itself; the ranks
rendezvous, build the communicator (the host simulation's stand-in for RCCL), validate their own batches,
all-gather the verdicts and report n_gpus = rccl_ranks = 2.  A launcher whose WORLD_SIZE disagrees with
--gpus is refused.  LCV_BENCH_HOSTSIM=1 runs the kernels' host simulation (test-only)."""
import json
import os
import subprocess
import sys

import pytest

import helpers as H

BENCH = os.path.join(H.ROOT, "bench.py")
ARGS = ["--n", "64", "--steps", "2", "--warmup", "1", "--depth", "2", "--quick"]


def _run(extra_env, args, timeout=600):
    H.ensure_hostsim()
    env = dict(os.environ, LCV_BENCH_HOSTSIM="1")
    env.setdefault("OMP_NUM_THREADS", "2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LCV_RDZV_KEY"):
        env.pop(k, None)
    env.update(extra_env)
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True,
                          timeout=timeout, cwd=H.ROOT)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_gpus_n_spawns_n_ranks(world):
    p = _run({"OMP_NUM_THREADS": "1" if world > 2 else "2"}, ["--gpus", str(world)] + ARGS)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["rccl_ranks"] == world
    assert d["all_valid"] and d["pcie_inclusive_serving"]["all_valid"]
    assert d["value"] > 0 and "host simulation" in d["library"]
    assert all(f"[rank {r}]" in p.stderr for r in range(world))


@pytest.mark.timeout(300)
def test_bench_refuses_mismatched_world():
    p = _run({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, ["--gpus", "2"] + ARGS)
    assert p.returncode == 2
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert "refusing" in p.stderr


def test_launch_tag_is_per_launch(monkeypatch):
    from lcv import multi
    monkeypatch.delenv("LCV_RDZV_KEY", raising=False)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    t1 = multi.launch_tag()
    assert t1.startswith("ppid:") and t1.count(":") == 2 and t1.split(":")[2]  # parent pid + its start time
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "abc")
    assert multi.launch_tag() == "run:abc"
    monkeypatch.setenv("LCV_RDZV_KEY", "k1")
    assert multi.launch_tag() == "k1"


def test_rendezvous_ignores_stale_file(tmp_path, monkeypatch):
    """A file left by an earlier launch on the same address and port (another tag) is never accepted."""
    from lcv import multi
    monkeypatch.setenv("LCV_RENDEZVOUS_DIR", str(tmp_path))
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "12345")
    monkeypatch.setenv("LCV_RDZV_KEY", "old-launch")
    lib = H.hostsim_verifier().lib
    old = multi.rendezvous(lib, 0, 2)
    monkeypatch.setenv("LCV_RDZV_KEY", "new-launch")
    from lcv._native import LcvError
    with pytest.raises(LcvError):
        multi.rendezvous(lib, 1, 2, timeout=0.3)
    new = multi.rendezvous(lib, 0, 2)
    assert multi.rendezvous(lib, 1, 2, timeout=5) == new != old
