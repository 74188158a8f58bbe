"""Multi-GPU sharding of a batch of updates: one process and one liblcv context per GPU, no PyTorch.

Updates are independent given one store snapshot, so a batch is split into
contiguous index ranges, one per rank; each rank validates its shard on its own GPU and the only
collective is one all-gather of the per-update verdict bytes — RCCL over xGMI, device buffer to
device buffer, inside liblcv.so (`lcv_validate_sharded`).  No data-path exchange.

Rendezvous: rank 0 creates the 128-byte RCCL unique id (`lcv_comm_unique_id`) and publishes it in a
file keyed on the launch's MASTER_ADDR:MASTER_PORT (all ranks on one node), tagged with a token unique
to the launch (`launch_tag`), which the other ranks poll for.  The test suite runs the same code on the host simulation, whose stand-in collective
exchanges files (tests/test_multi.py).
"""
from __future__ import annotations

import ctypes as C
import os
import tempfile
import time
from typing import Optional, Tuple

import numpy as np

from ._native import LcvError, as_u8, ptr


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous shard [lo, hi) of rank `rank`; shard sizes differ by at most one."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _proc_start(pid: int) -> str:
    """Start time of process `pid` in clock ticks since boot (/proc/<pid>/stat field 22), '' if unknown."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[19]
    except (OSError, IndexError):
        return ""


def launch_tag() -> str:
    """A token that every rank of ONE launch computes identically and no other launch does:
    LCV_RDZV_KEY (set by bench.py's own spawner or by a caller), else the launcher's run id
    (TORCHELASTIC_RUN_ID, when not the static default "none"), else the shared parent process's pid and
    start time (the ranks of torch.distributed.run / bench.py --gpus are children of one launcher)."""
    tag = os.environ.get("LCV_RDZV_KEY")
    if tag:
        return tag
    run = os.environ.get("TORCHELASTIC_RUN_ID", "")
    if run and run != "none":
        return f"run:{run}"
    ppid = os.getppid()
    return f"ppid:{ppid}:{_proc_start(ppid)}"


def _id_path(key: Optional[str]) -> str:
    """Rendezvous file: keyed on the launch's MASTER_ADDR:MASTER_PORT (not on the parent pid)."""
    if key is None:
        key = f"{os.environ.get('MASTER_ADDR', '127.0.0.1')}_{os.environ.get('MASTER_PORT', '0')}"
    d = os.environ.get("LCV_RENDEZVOUS_DIR", tempfile.gettempdir())
    safe = "".join(c if c.isalnum() or c in "._-" else "_" for c in key)
    return os.path.join(d, f"lcv_rccl_id_{safe}")


def rendezvous(lib, rank: int, world: int, key: Optional[str] = None, timeout: float = 300.0) -> bytes:
    """The communicator id, made by rank 0 and read by every other rank of this launch.  The file holds
    the id and this launch's tag (launch_tag()); a rank accepts only a file carrying its own tag, so a
    file left behind by an earlier launch on the same address and port is never used."""
    path = _id_path(key)
    tag = launch_tag().encode()
    if rank == 0:
        uid = np.zeros(128, np.uint8)
        rc = lib.lcv_comm_unique_id(ptr(uid))
        if rc != 0:
            raise LcvError(f"lcv_comm_unique_id failed with status {rc}")
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(uid.tobytes() + tag)
        os.replace(tmp, path)  # atomic: readers see the whole id or nothing
        return uid.tobytes()
    t0 = time.monotonic()
    while True:
        try:
            with open(path, "rb") as f:
                b = f.read()
            if len(b) == 128 + len(tag) and b[128:] == tag:
                return b[:128]
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise LcvError(f"rendezvous: no communicator id for launch {tag.decode()} at {path} after {timeout:.0f} s")
        time.sleep(0.01)


class CommFailed(LcvError):
    """A collective failed or timed out (a peer rank died or hangs); the communicator must be shrunk to
    the surviving ranks (Comm.recover) before the next collective."""


class Comm:
    """The RCCL communicator of one rank (on `verifier`'s device).  `timeout`: every collective completes
    within it or fails with CommFailed (lcv_comm_set_timeout); `recover()` then agrees on the surviving
    ranks and moves them onto a new communicator.

    `recovery`: "reinit" (default) aborts the failed communicator and the survivors initialise a fresh one
    through the rendezvous directory — the path that works on the RCCL the MI355X image ships (2.27
    refuses ncclCommShrink); "shrink" first tries lcv_comm_shrink (ncclCommShrink with
    NCCL_SHRINK_ABORT) and falls back to "reinit" when RCCL refuses it."""

    def __init__(self, verifier, world: int, rank: int, key: Optional[str] = None, timeout: float = 60.0,
                 recovery: str = "reinit"):
        if recovery not in ("reinit", "shrink"):
            raise ValueError(f"recovery must be 'reinit' or 'shrink', not {recovery!r}")
        self.v, self.world, self.rank = verifier, int(world), int(rank)
        self.key = key
        self.recovery = recovery
        self.epoch = 0          # recoveries so far
        self.ranks = list(range(self.world))  # original rank ids of the current members, by new rank
        uid = rendezvous(verifier.lib, self.rank, self.world, key)
        self.v._check(self.v.lib.lcv_comm_init(self.v.ctx, self.world, self.rank, ptr(as_u8(uid))), "lcv_comm_init")
        self.set_timeout(timeout)

    def set_timeout(self, seconds: float) -> None:
        self.v._check(self.v.lib.lcv_comm_set_timeout(self.v.ctx, float(seconds)), "lcv_comm_set_timeout")
        self.timeout = float(seconds)

    def abort(self) -> None:
        """Abort this rank's communicator (lcv_comm_abort: outstanding collectives are terminated, the
        streams drain); the rank takes no further part in collectives until a new communicator."""
        self.v.lib.lcv_comm_abort(self.v.ctx)

    def _coll(self, rc: int, what: str) -> None:
        """Collective status: LCV_EDEVICE (-2) from a collective = the communicator failed."""
        if rc == -2:
            msg = self.v.lib.lcv_last_error(self.v.ctx)
            raise CommFailed(f"{what}: {msg.decode() if msg else 'collective failed'}")
        self.v._check(rc, what)

    # ---- failure containment: membership agreement through the rendezvous directory
    def _fail_path(self, what: str) -> str:
        return f"{_id_path(self.key)}.{launch_tag_safe()}.fail{self.epoch}.{what}"

    def agree_survivors(self, grace: float = 10.0) -> list:
        """After a failed collective: every live member announces itself, waits until all members did or
        `grace` seconds passed, and the first to publish a decision (exclusive create) fixes the survivor
        list everyone then uses; a member left out of the decision (it announced too late) aborts its
        communicator — so none of its streams stays behind the failed collective — and raises.

        The grace period is at least the communicator timeout: survivors detect the failure when their
        own collective times out, which starts when each enters its wait, so a slower survivor announces
        up to one timeout after the first.  It is counted from the FIRST announcement (the earliest alive
        marker), not from this rank's own, so every survivor decides at the same moment.  Recovery latency:
        a dead rank never announces itself, so a recovery takes one communicator timeout to detect the
        failure (the bounded collective wait) plus up to max(grace, timeout) here — with the default 60 s
        timeout about two minutes; lower it with Comm(timeout=...) / set_timeout where peers are fast."""
        grace = max(float(grace), getattr(self, "timeout", 0.0))
        me = self.ranks[self.rank]
        open(self._fail_path(f"alive.{me}"), "w").close()

        def first_announcement() -> float:
            ts = []
            for r in self.ranks:
                try:
                    ts.append(os.stat(self._fail_path(f"alive.{r}")).st_mtime)
                except FileNotFoundError:
                    pass
            return min(ts) if ts else time.time()

        while time.time() - first_announcement() < grace:
            if all(os.path.exists(self._fail_path(f"alive.{r}")) for r in self.ranks):
                break
            if os.path.exists(self._fail_path("decision")):
                break
            time.sleep(0.01)
        alive = [r for r in self.ranks if os.path.exists(self._fail_path(f"alive.{r}"))]
        dec = self._fail_path("decision")
        try:
            fd = os.open(dec + ".tmp." + str(me), os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
            os.write(fd, (",".join(map(str, alive))).encode())
            os.close(fd)
            os.link(dec + ".tmp." + str(me), dec)  # atomic exclusive publish: the first link wins
        except FileExistsError:
            pass
        finally:
            try:
                os.remove(dec + ".tmp." + str(me))
            except OSError:
                pass
        for _ in range(1000):
            try:
                txt = open(dec).read()
                if txt:
                    break
            except FileNotFoundError:
                pass
            time.sleep(0.01)
        survivors = [int(x) for x in txt.split(",")]
        if me not in survivors:
            self.abort()
            raise CommFailed(f"rank {me} was excluded by the survivors' decision {survivors}")
        return survivors

    def recover(self, grace: float = 10.0) -> list:
        """Move the survivors of a failed communicator (same decision on every survivor) onto a new one;
        returns the survivors' original rank ids.  Afterwards self.rank / self.world are the new ones.
        recovery "reinit" (the default): the failed communicator is aborted and the survivors initialise
        a fresh one through the rendezvous directory (a key per recovery epoch; the lowest surviving rank
        publishes the id).  recovery "shrink": ncclCommShrink (lcv_comm_shrink) first, "reinit" where the
        RCCL build refuses it."""
        survivors = self.agree_survivors(grace)
        exclude = [k for k, r in enumerate(self.ranks) if r not in survivors]
        me = self.ranks[self.rank]
        ex = (C.c_int * max(1, len(exclude)))(*exclude)
        nr, nn = C.c_int(), C.c_int()
        rc = -1
        if self.recovery == "shrink":
            rc = self.v.lib.lcv_comm_shrink(self.v.ctx, ex, len(exclude), C.byref(nr), C.byref(nn))
        self.ranks = [r for r in self.ranks if r in survivors]
        self.last_recovery = "shrink" if rc == 0 else "reinit"
        if rc not in (0, -1):
            msg = self.v.lib.lcv_last_error(self.v.ctx)
            self.last_recovery += f" (lcv_comm_shrink: {msg.decode() if msg else rc})"
        if rc == 0:
            self.rank, self.world = int(nr.value), int(nn.value)
        else:
            self.abort()
            self.rank, self.world = self.ranks.index(me), len(self.ranks)
            base = self.key if self.key is not None else \
                f"{os.environ.get('MASTER_ADDR', '127.0.0.1')}_{os.environ.get('MASTER_PORT', '0')}"
            key = f"{base}.epoch{self.epoch + 1}"
            uid = rendezvous(self.v.lib, self.rank, self.world, key)
            self.v._check(self.v.lib.lcv_comm_init(self.v.ctx, self.world, self.rank, ptr(as_u8(uid))),
                          "lcv_comm_init (recovery)")
            self._epoch_keys = getattr(self, "_epoch_keys", []) + [key]
        if self.world != len(self.ranks):
            raise CommFailed(f"shrunk communicator has {self.world} ranks, the survivors' decision {len(self.ranks)}")
        self.epoch += 1
        return survivors

    def validate_sharded(self, rb, current_slot: int, genesis_validators_root: bytes, per_rank: int,
                         out: Optional[np.ndarray] = None) -> np.ndarray:
        """Validate this rank's resident shard (rb.n <= per_rank) and all-gather every rank's verdict
        bytes: (world * per_rank,) uint8, rank-major, each slice zero padded."""
        gvr = as_u8(bytes(genesis_validators_root))
        buf = out if out is not None else np.zeros(self.world * per_rank, np.uint8)
        self._coll(self.v.lib.lcv_validate_sharded(self.v.ctx, rb.handle, int(current_slot), ptr(gvr),
                                                   int(per_rank), ptr(buf)), "lcv_validate_sharded")
        return buf

    def slot_allgather(self, slot: int, n: int, per_rank: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        """After this rank's batch in work-space slot `slot` (Verifier.validate_resident_async), all-gather
        every rank's verdict bytes: (world * per_rank,) uint8, rank-major, each slice zero padded."""
        buf = out if out is not None else np.zeros(self.world * per_rank, np.uint8)
        self._coll(self.v.lib.lcv_slot_allgather(self.v.ctx, int(slot), int(n), int(per_rank), ptr(buf)),
                   "lcv_slot_allgather")
        return buf

    def count(self) -> int:
        """Ranks in the communicator as RCCL reports them (ncclCommCount)."""
        c = C.c_int()
        self.v._check(self.v.lib.lcv_comm_count(self.v.ctx, C.byref(c)), "lcv_comm_count")
        return int(c.value)

    def allreduce_max(self, x: float) -> float:
        d = C.c_double(float(x))
        self._coll(self.v.lib.lcv_comm_allreduce_max(self.v.ctx, C.byref(d)), "lcv_comm_allreduce_max")
        return d.value

    def barrier(self) -> None:
        self.allreduce_max(0.0)

    def close(self) -> None:
        if self.v is not None:
            try:
                self.barrier()
            except LcvError:
                pass  # a failed (or already aborted) communicator: lcv_comm_destroy aborts / skips it
            if self.rank == 0:
                import glob
                keys = [self.key] + getattr(self, "_epoch_keys", [])
                for f in [_id_path(k) for k in keys] + glob.glob(f"{_id_path(self.key)}.*.fail*"):
                    try:
                        os.remove(f)
                    except OSError:
                        pass
            self.v.lib.lcv_comm_destroy(self.v.ctx)
            self.v = None


def unshard(gathered: np.ndarray, n_total: int, world: int) -> np.ndarray:
    """Rank-major padded slices -> the n_total verdicts in batch order."""
    per = gathered.size // world
    parts = [gathered[r * per:r * per + (shard_bounds(n_total, world, r)[1] - shard_bounds(n_total, world, r)[0])]
             for r in range(world)]
    return np.concatenate(parts) if parts else gathered[:0]


def validate_sharded(verifier, batch, current_slot: int, genesis_validators_root: bytes, comm: Comm,
                     recover: bool = True, grace: float = 10.0) -> np.ndarray:
    """This rank validates its shard of `batch` (the full PackedUpdates, identical on every rank);
    returns the full verdict array (bool) on every rank.  The store must already be set on `verifier`.

    Failure containment: when a peer dies or hangs, the collective fails within the
    communicator's timeout on every surviving rank (CommFailed); with `recover` the survivors agree on
    who is left (Comm.recover), shrink the communicator to themselves and the batch is re-sharded over
    them — the failed rank's shard is validated on the survivors — until a pass completes.  The result
    equals the single-rank verdicts."""
    while True:
        world, rank = comm.world, comm.rank
        lo, hi = shard_bounds(batch.n, world, rank)
        per = -(-batch.n // world)
        if hi > lo:
            rb = verifier.upload(batch.slice(lo, hi))
        else:  # an empty shard still joins the collective (a one-row dummy batch, verdict overwritten)
            rb = verifier.upload(batch.slice(0, 1))
        try:
            g = comm.validate_sharded(rb, current_slot, genesis_validators_root, max(per, 1))
            return unshard(g, batch.n, world).astype(bool)
        except CommFailed:
            if not recover or world == 1:
                raise
            comm.recover(grace)
        finally:
            rb.free()


def launch_tag_safe() -> str:
    return "".join(c if c.isalnum() or c in "._-" else "_" for c in launch_tag())
