#!/usr/bin/env python3
"""Benchmark: verified LightClientUpdates/sec (512-member committee) on 1..8 MI355X.

One step = `validate_light_client_updates` over this rank's resident batch of synthetic
mainnet-preset Deneb updates (BASELINE.json configs[1]: 10,000 updates per GPU, full 512/512
participation, every update carrying next_sync_committee + finality + execution branches), i.e.
every kernel of the hot path (SSZ/SHA-256, hash_to_G2, signature decode + subgroup check, masked G1
aggregation, Miller loop, final exponentiation, verdicts).  Inputs are resident in HBM (uploaded
once, outside the timed region); for N > 1 each step ends with an RCCL all-gather of the per-rank
verdict bytes (the only collective of the design).  Weak scaling: every rank owns `--n` updates.

Default shape (--depth 8): the serving loop keeps eight batches in flight — eight resident batches of
`--n` updates rotate over the work-space slots of the context (lcv_validate_resident_async), so later
batches' latency-bound early stages (SSWU, hash_to_G2) share the GPU with earlier batches' Miller loop
and final exponentiation; each timed step is one whole batch, waited for and its verdicts read (or
all-gathered) inside the timed region.  --depth 1 times one batch at a time; both rates are reported.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n UPDATES_PER_GPU] [--participation full|random]
                    [--depth 1..8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "light-client-consensus-specs_amd"))

import numpy as np  # noqa: E402

DEFAULT_DEPTH = 8
# one HIP stream pair per work-space slot: with HIP's default of 4 hardware queues per process the
# streams of several slots would share queues (ordering more than the events require); gpurun allows <= 32
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

# Roofline denominators.  The op model W = 600 N_fpmul + 24 N_fpadd +
# 2100 N_sha prices a Montgomery product at 600 INT32 ops, i.e. 2 ops per multiply-add
# of a 288-mad product, so its natural peak is the chip's multiply-add issue rate, MEASURED: the
# v_mad_u64_u32 rate of tools/microbench/peakbench.hip (inline asm, 128 independent mads per iteration,
# no other instruction; wall time over the whole chip) at the SOP kernels' residency of 3 waves per SIMD,
# committed in profiles/r05_cal/peakbench.txt, x 2 ops per mad.
PEAK_FILE = os.path.join(ROOT, "profiles", "r05_cal", "peakbench.txt")
PEAK_WAVES_PER_SIMD = 3


def measured_peaks(path: str = PEAK_FILE) -> dict:
    """Rows of the committed peakbench output: {(kernel, W): {"ms", "ginstr", "cyc_clock", "cyc_24",
    "mad_T", "op_T"}}."""
    rows = {}
    for line in open(path):
        if line.startswith("#") or "|" not in line:
            continue
        head, *cols = [c.strip() for c in line.split("|")]
        name, w = head.rsplit(None, 1)
        vals = [float(c) for c in cols]
        rows[(name.split()[0], int(w))] = dict(zip(("ms", "ginstr", "cyc_clock", "cyc_24", "mad_T", "op_T"), vals))
    return rows


def mac_peak_tops(w: int = PEAK_WAVES_PER_SIMD) -> float:
    """2 ops x the measured v_mad_u64_u32 rate (T/s) at w waves per SIMD (profiles/r05_cal/peakbench.txt)."""
    return measured_peaks()[("mad", w)]["op_T"]


PEAK_MAC_TOPS = mac_peak_tops()
# the full-rate INT32 VALU lane rate (4 x SIMD-32 per CU x 2 ops per multiply-add, MI355X_MICROARCH.md):
# every fraction is also reported against it
PEAK_INT32_VALU_TOPS = 78.6
# stages whose canonical (textbook) numerator counts the algorithm class the device runs; elsewhere the
# canonical counter charges Fermat inversions / square-root chains / a separate psi check the device does
# not run (Bernstein-Yang inversion, windowed chains, the check fused into the line walk), so only the
# executed numerator is a statement about the hardware there
CANONICAL_MATCHED = ("pre_checks", "signing_root", "nsc_htr", "hash_to_g2", "miller_lines", "miller_loop", "final_exp")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


PKG_DIR = os.path.join(ROOT, "light-client-consensus-specs_amd")
CPU_LIB = os.path.join(PKG_DIR, "build", "liblcv_cpu.so")


def physical_cores() -> dict:
    """Host core counts: physical cores (unique (core, socket) pairs of `lscpu -p`) and logical CPUs."""
    import subprocess
    out = {"logical_cpus": os.cpu_count()}
    try:
        rows = subprocess.run(["lscpu", "-p=Core,Socket"], capture_output=True, text=True, timeout=10).stdout
        out["physical_cores_lscpu"] = len({l for l in rows.splitlines() if l and not l.startswith("#")})
        model = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        out["model"] = next((l.split(":", 1)[1].strip() for l in model.splitlines() if l.startswith("Model name")), None)
    except Exception as e:  # reported, never fatal
        out["lscpu_error"] = repr(e)
    return out


def cpu_library():
    """The CPU-baseline library: rebuilt with -O3 -march=native for THIS host (`make cpu-native`, always
    recompiled into TMPDIR, ~20 s), else the prebuilt portable -march=x86-64-v3 build."""
    import subprocess
    import tempfile
    out = os.path.join(tempfile.gettempdir(), f"liblcv_cpu_native_{os.getpid()}.so")
    try:
        subprocess.run(["make", "-s", "-C", PKG_DIR, "cpu-native", f"CPU_NATIVE_OUT={out}"], check=True,
                       capture_output=True, timeout=240)
        return out, "-O3 -march=native, built on this host"
    except Exception as e:
        log(f"cpu baseline: native build failed ({e!r}); using the prebuilt x86-64-v3 library")
        return CPU_LIB, "-O3 -march=x86-64-v3 -madx (prebuilt, portable)"


def _omp_threads(n: int | None = None) -> int:
    """Set (n) / read the OpenMP pool of this process (libgomp, shared with liblcv_cpu.so)."""
    import ctypes
    try:
        g = ctypes.CDLL("libgomp.so.1")
        if n is not None:
            g.omp_set_num_threads(ctypes.c_int(n))
        return int(g.omp_get_max_threads())
    except OSError:
        return int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)


def cpu_baseline(target_s: float = 15.0, seed: int = 3):
    """The CPU baseline: the build's own C++ verifier — the same
    per-update field/tower/curve code as the device, compiled for the host (-O3 -march=native, 64-bit limb
    Montgomery products, direct per-update pairing code instead of the team-program interpreter;
    liblcv_cpu.so) — on a bounded sample of the same workload (~`target_s` seconds), over the host CPU
    share of the lease: the CPUs this process may run on (os.sched_getaffinity), capped by the pool's
    per-GPU share (OMP_NUM_THREADS, which the GPU pool sets to its 16-CPU share of a one-GPU lease: worker
    pools must stay within it).  Beside it: the rate on ONE thread (a short sample) and the linear
    per-core extrapolation to the host's physical cores, labelled as such; for scale only, the
    pure-Python oracle on one core."""
    from lcv import synth
    from lcv._native import Lib
    from lcv.device import Verifier
    path, flags = cpu_library()
    if not os.path.exists(path):
        return None
    v = Verifier(lib=Lib(path))
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0")) or affinity
    threads = _omp_threads(min(affinity, share))
    base = synth.generate(v, 512, seed=seed)
    v.set_store(base.store_finalized_slot, base.current.ssz, base.next.ssz)
    t0 = time.perf_counter()
    ok, _ = v.validate(base.updates, base.current_slot, base.genesis_validators_root)
    rate0 = 512 / (time.perf_counter() - t0)
    reps = max(1, int(rate0 * target_s / 512))
    sb = synth.tile(base, reps)
    t0 = time.perf_counter()
    ok, _ = v.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    dt = time.perf_counter() - t0
    assert ok.all()
    # one thread, ~target_s / 4 of work: the per-core rate
    _omp_threads(1)
    one = base.updates.slice(0, 64)
    t1 = time.perf_counter()
    ok1, _ = v.validate(one, base.current_slot, base.genesis_validators_root)
    dt1 = time.perf_counter() - t1
    reps1 = max(1, int(64 / dt1 * target_s / 4 / 64))
    sb1 = synth.tile(base, (64 * reps1 + 511) // 512).updates.slice(0, 64 * reps1)
    t1 = time.perf_counter()
    ok1, _ = v.validate(sb1, base.current_slot, base.genesis_validators_root)
    dt1 = time.perf_counter() - t1
    assert ok1.all()
    _omp_threads(threads)
    host = physical_cores()
    per_core = sb1.n / dt1
    out = {"value": round(sb.updates.n / dt, 1), "unit": "updates/s", "cores": threads, "kind": "port",
           "sample": f"{sb.updates.n} synthetic Deneb updates (512/512, all branches; 512 generated rows tiled "
                     f"x{reps}), validated by liblcv_cpu (C++ port of the device path, {flags}, "
                     f"64-bit-limb Montgomery, OpenMP over {threads} threads), {dt:.1f} s",
           "cores_used": threads, "cpus_in_affinity_mask": affinity,
           "cpu_share_of_lease": share,
           "cores_note": ("the GPU pool's one-GPU lease gives this process a CPU share of "
                          f"{share} (OMP_NUM_THREADS set by the pool; worker pools are to stay within it) out of "
                          f"{affinity} CPUs in its affinity mask; the baseline runs {threads} threads"),
           "per_core_value": round(per_core, 1),
           "per_core_sample": f"{sb1.n} updates on 1 thread, {dt1:.1f} s",
           "whole_host_linear_extrapolation": (round(per_core * host["physical_cores_lscpu"], 1)
                                               if host.get("physical_cores_lscpu") else None),
           "whole_host_extrapolation_is": "per_core_value x physical_cores_lscpu (not measured: the lease's "
                                          "CPU share does not allow a whole-host run)",
           "host": host, "compile_flags": flags}
    if path != CPU_LIB:
        try:
            os.remove(path)
        except OSError:
            pass
    # for scale only: the pure-Python oracle (oracle/sync_protocol.py), one core, a few updates
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import helpers as H
    store = H.store_from(base.store_finalized_slot, base.current.ssz, base.next.ssz)
    ups = [H.update_from(base.updates, i) for i in range(4)]
    H.O.validate_light_client_update(store, ups[0], base.current_slot, base.genesis_validators_root)  # key cache
    t0 = time.perf_counter()
    for u in ups:
        assert H.O.validate_light_client_update(store, u, base.current_slot, base.genesis_validators_root) == 0
    out["python_oracle_scale_only"] = {"value": round(len(ups) / (time.perf_counter() - t0), 2),
                                       "unit": "updates/s", "cores": 1}
    return out


def _free_port() -> int:
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, one GPU each, a launch token for the RCCL rendezvous)
    before this process touches any GPU, and return the first non-zero exit code (0 if all succeed).
    Rank 0 prints the JSON line."""
    import subprocess
    import uuid
    port, tag = str(_free_port()), uuid.uuid4().hex
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, LCV_RDZV_KEY=tag)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                log(f"bench: rank {procs.index(p)} exited with {code}; stopping the other ranks")
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--n", type=int, default=10000, help="updates per GPU (configs[1]: 10,000)")
    ap.add_argument("--participation", default="full", choices=["full", "random"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline sample size in seconds")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the configs[2]/[3]/[4] lines")
    ap.add_argument("--quick", action="store_true",
                    help="only the timed configs[1] measurements (no configs / wire / latency / CPU-baseline lines)")
    ap.add_argument("--pipeline", default="1,1", help="STREAMS,SLICES of the timed run (1,1 = serial stages)")
    ap.add_argument("--depth", type=int, default=DEFAULT_DEPTH, choices=range(1, 9),
                    help="batches in flight: D > 1 = serving loop over D work-space slots "
                         "(lcv_validate_resident_async), 1 = one batch at a time")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: this process becomes the launcher (it never touches a GPU itself)
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks; refusing to report "
            f"a {world}-rank measurement under a {args.gpus}-GPU label")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from lcv import multi, synth
    from lcv.device import Verifier
    from lcv._native import Lib, load
    import ctypes
    # test-only: LCV_BENCH_HOSTSIM=1 runs the same script on the host simulation of the kernels (CPU, every
    # rank on "device 0"; tests/test_bench_launch.py); the JSON line then names that library
    hostsim = os.environ.get("LCV_BENCH_HOSTSIM") == "1"
    lib = Lib(os.path.join(PKG_DIR, "build", "liblcv_hostsim.so")) if hostsim else load()
    device = 0 if hostsim else local
    nd = ctypes.c_int(0)
    lib.lcv_device_count(ctypes.byref(nd))
    if device >= nd.value:
        log(f"bench: rank {rank} needs GPU {local} but {nd.value} are visible")
        sys.exit(3)

    v = Verifier(device, lib=lib)
    # N > 1: one process per GPU, RCCL (over xGMI) inside liblcv.so for the verdict all-gather, the
    # barrier and the max-over-ranks of the timed region; no PyTorch anywhere on the path
    comm = multi.Comm(v, world, rank) if world > 1 else None
    rccl_ranks = comm.count() if comm is not None else 1
    if rccl_ranks != world:
        log(f"bench: RCCL communicator has {rccl_ranks} ranks, WORLD_SIZE is {world}")
        sys.exit(4)
    t0 = time.perf_counter()
    sb = synth.generate(v, args.n, seed=2 + rank, participation=args.participation)
    log(f"[rank {rank}] generated {args.n} updates in {time.perf_counter() - t0:.1f}s")
    v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    rb = v.upload(sb.updates)
    # depth D > 1: D different resident batches of the same shape (same store), one per work-space slot
    D = args.depth
    sbs = [sb] + [synth.generate(v, args.n, seed=1000 * k + 2 + rank, participation=args.participation)
                  for k in range(1, D)]
    rbs = [rb] + [v.upload(b.updates) for b in sbs[1:]]
    pipe = tuple(int(x) for x in args.pipeline.split(","))
    v.set_pipeline(*pipe)
    verdict = np.zeros(args.n, np.uint8)
    reason = np.zeros(args.n, np.uint8)

    gathered = np.zeros(world * args.n, np.uint8)

    def step():  # every lcv call returns after its stream work is complete (device synchronised)
        if comm is None:
            v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root, verdict, reason)
        else:
            comm.validate_sharded(rb, sb.current_slot, sb.genesis_validators_root, args.n, gathered)

    def sync():
        if comm is not None:
            comm.barrier()

    slot_ok = [True] * D
    per_slot_v = [np.zeros(args.n, np.uint8) for _ in range(D)]
    per_slot_r = [np.zeros(args.n, np.uint8) for _ in range(D)]
    per_slot_g = [np.zeros(world * args.n, np.uint8) for _ in range(D)]

    def collect(s):  # wait for slot s's batch; its verdicts (all-gathered over RCCL when N > 1)
        if comm is None:
            v.slot_wait(s, args.n, per_slot_v[s], per_slot_r[s])
            slot_ok[s] = slot_ok[s] and bool((per_slot_v[s] == 1).all())
        else:
            comm.slot_allgather(s, args.n, args.n, per_slot_g[s])
            slot_ok[s] = slot_ok[s] and bool((per_slot_g[s] == 1).all())

    def stream_steps(k_steps):
        # serving loop: batch k runs in slot k % D while batches k - D + 1 .. k - 1 are still on the GPU;
        # the host waits for a slot (and reads its verdicts) only before reusing it, and drains them all
        for k in range(k_steps):
            s = k % D
            if k >= D:
                collect(s)
            v.validate_resident_async(rbs[s], sbs[s].current_slot, sbs[s].genesis_validators_root, s)
        for k in range(max(0, k_steps - D), k_steps):
            collect(k % D)

    for _ in range(args.warmup):
        step()
    if D > 1:
        stream_steps(max(D, args.warmup))
    # correctness of what is timed: every synthetic update is valid
    if comm is None:
        v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root, verdict, reason)
        ok_all = bool((verdict == 1).all())
    else:
        step()
        ok_all = bool((gathered == 1).all())
    serial = pipe == (1, 1) and args.depth == 1
    stage_ms = {k: 0.0 for k in v.last_timings()}
    sync()
    t0 = time.perf_counter()
    if D > 1:
        stream_steps(args.steps)
    else:
        for _ in range(args.steps):
            step()
            if serial:  # stage kernel times: HIP events on each stage's stream, inside the timed region
                for k, ms in v.last_timings().items():
                    stage_ms[k] += ms
    sync()
    dt = time.perf_counter() - t0
    if comm is not None:
        dt = comm.allreduce_max(dt)
    if D > 1:
        ok_all = ok_all and all(slot_ok)

    serial_ms, serial_ok = 1000 * dt / args.steps, ok_all
    if not serial:
        # a multi-stream pipeline overlaps stages, so per-stage kernel times come from the serial
        # shape (no other kernel sharing the GPU), run after the timed region
        v.set_pipeline(1, 1)
        sync()
        ts = time.perf_counter()
        for _ in range(args.steps):
            step()
            for k, ms in v.last_timings().items():
                stage_ms[k] += ms
        sync()
        serial_ms = 1000 * (time.perf_counter() - ts) / args.steps
        if comm is not None:
            serial_ms = 1000 * comm.allreduce_max(serial_ms / 1000)
        serial_ok = bool((verdict == 1).all()) if comm is None else bool((gathered == 1).all())
        v.set_pipeline(*pipe)

    # PCIe-inclusive rates (host batch -> device each time), reported beside `value`, never as it:
    # one batch at a time through lcv_validate_updates, and the serving loop from host buffers
    t1 = time.perf_counter()
    v.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    pcie_rate = args.n / (time.perf_counter() - t1)
    serving = serving_from_host(v, sbs, D, args.steps, comm)

    if rank != 0:
        if comm is not None:
            comm.close()
        return
    wire_out = None if args.quick else wire_path(v, sb, args.n)
    try:
        latency = None if args.quick else latency_lines(v, sb)
    except Exception as e:  # reported, never fatal to the throughput measurement
        latency = {"error": repr(e)}
    total = world * args.n * args.steps
    stage_avg = {k: round(ms / args.steps, 3) for k, ms in stage_ms.items() if ms > 0}
    kernel_ms = sum(stage_avg.values())
    npool = int(sb.updates.nsc_pool.shape[0])
    roof = roofline(stage_avg, args.n, npool)
    if roof is not None:  # the whole pipeline's rate against the same peaks (all stages, all kernels)
        for sec in ("executed", "canonical"):
            if sec != "executed" and sec not in _opcounts():
                continue
            ops = total_ops_per_update(args.n, npool, sec)
            rate = ops * total / dt / world / 1e12
            roof[f"pipeline_ops_per_update_{sec}"] = round(ops, 1)
            if sec == "executed":
                roof["pipeline_frac_executed"] = round(rate / PEAK_MAC_TOPS, 4)
                roof["pipeline_frac_executed_vs_int32_valu_peak"] = round(rate / PEAK_INT32_VALU_TOPS, 4)
            else:
                # the textbook algorithms' op count at the measured update rate: a work-equivalent rate,
                # NOT a fraction of any peak (it charges Fermat inversions / square roots and a textbook
                # Miller loop the device does not run, so it can exceed the hardware's rate)
                roof["pipeline_canonical_equivalent_T_ops_per_s"] = round(rate, 3)
        roof["pipeline_frac"] = roof["pipeline_frac_executed"]  # headline: the executed numerator
    configs = None if (args.no_configs or args.quick or world > 1) else config_lines(v)
    distinct = None if configs is None else distinct_serving(v, args.n, D, args.steps)
    out = {
        "metric": "verified LightClientUpdates/sec (512-member committee)",
        "value": round(total / dt, 1),
        "unit": "updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * dt / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (381-bit Montgomery Fp on 12x32-bit limbs; SHA-256 words)",
        "data": "synthetic (mainnet preset, Deneb, device-signed)",
        "config": {"workload": f"configs[1]: {args.n} updates/GPU, {args.participation} participation, "
                               f"next_sync_committee + finality + execution branches; the {args.n} updates of a "
                               f"batch share ONE next_sync_committee value ({npool} distinct per batch, so "
                               f"HTR(SyncCommittee) runs {npool}x per batch; configs[3] with a distinct committee "
                               f"per update: value_distinct_committees)",
                   "updates_per_gpu": args.n, "committee": 512, "parallelism": f"dp{world} (independent updates)"},
        # SURVEY 8(d)'s timed region from host buffers (H2D of the packed batch + kernels + verdicts D2H),
        # the same serving loop: beside `value`, which the bench contract defines on HBM-resident inputs
        "value_h2d_inclusive": serving["updates_per_s"],
        # configs[3]'s shape (a distinct next_sync_committee per update, HTR(SyncCommittee) per update) in
        # the same serving loop as `value`; configs["configs[3]"] has it one batch at a time
        "value_distinct_committees": None if distinct is None else distinct["updates_per_s"],
        "distinct_committees_serving": distinct,
        "all_valid": ok_all and serial_ok,
        "pipeline": {"streams": pipe[0], "slices": pipe[1]},
        "batches_in_flight": args.depth,
        "serial_ms_per_step": round(serial_ms, 3),
        # one batch at a time (the latency-bound shape: every stage's launch waits for the previous)
        "value_one_batch_at_a_time": round(world * args.n / (serial_ms / 1000), 1),
        # per-kernel HIP-event times (one mark per kernel); the signature chain runs on a second
        # stream beside the message chain, so their sum exceeds the wall time of a step
        "stage_kernel_ms_per_step": stage_avg,
        "sum_of_stage_kernel_ms": round(kernel_ms, 3),
        "value_is": ("inputs resident in HBM when the timed region starts (the bench contract); every kernel, "
                     "the verdict read-back and (N > 1) the RCCL all-gather are inside it; " +
                     (f"{D} batches in flight (serving loop over {D} work-space slots, "
                      "lcv_validate_resident_async): later batches' stages overlap earlier ones', every batch's "
                      "verdicts are waited for and copied out (all-gathered over RCCL for N > 1) inside the "
                      "timed region; " if D > 1 else "") +
                     "pcie_inclusive_* copies the packed batch host->device and the verdicts back in every call"),
        "rccl_ranks": rccl_ranks,
        # SURVEY §8(d)'s timed region (host batch in, kernels, verdicts out) with D batches in flight
        "pcie_inclusive_serving": serving,
        "pcie_inclusive_one_batch_at_a_time_1gpu": round(pcie_rate, 1),
        "roofline": roof,
        "configs": configs,
        "wire": wire_out,
        "latency": latency,
    }
    if hostsim:
        out["library"] = "liblcv_hostsim.so (TEST-ONLY host simulation: not a GPU measurement)"
    if not (args.no_cpu_baseline or args.quick) and world == 1:
        try:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        except Exception as e:  # reported, never fatal to the GPU measurement
            out["cpu_baseline"] = {"error": repr(e)}
        pc = out["cpu_baseline"].get("per_core_value") if isinstance(out["cpu_baseline"], dict) else None
        if pc and isinstance(latency, dict) and "validate_one_update_ms" in latency:
            # the reference's call shape (one update per call) on one CPU core of the same host, beside the GPU's
            latency["cpu_one_core_ms"] = round(1000.0 / pc, 3)
    print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()


def distinct_serving(v, n: int, D: int, steps: int) -> dict:
    """configs[3]-shaped batches (a DISTINCT next_sync_committee per update, so HTR(SyncCommittee) runs once
    per update) in the serving loop `value` uses: D batches in flight on the work-space slots, inputs
    resident, the host waiting for a slot only before reusing it.  Two generated batches alternate over the
    slots (each ~0.27 GB resident); every verdict must be VALID as constructed."""
    from lcv import synth
    bs = [synth.generate(v, n, seed=4 + 40 * k, npool=n) for k in range(2)]
    v.set_store(bs[0].store_finalized_slot, bs[0].current.ssz, bs[0].next.ssz)
    rbs = [v.upload(b.updates) for b in bs]
    outs = [np.zeros(n, np.uint8) for _ in range(D)]
    ok = [True]

    def run(k_steps):
        for k in range(k_steps):
            s = k % D
            if k >= D:
                v.slot_wait(s, n, outs[s])
                ok[0] = ok[0] and bool((outs[s] == 1).all())
            b = bs[s % 2]
            v.validate_resident_async(rbs[s % 2], b.current_slot, b.genesis_validators_root, s)
        for k in range(max(0, k_steps - D), k_steps):
            v.slot_wait(k % D, n, outs[k % D])
            ok[0] = ok[0] and bool((outs[k % D] == 1).all())

    try:
        run(D)
        t0 = time.perf_counter()
        run(steps)
        dt = time.perf_counter() - t0
    finally:
        for rb in rbs:
            rb.free()
    return {"updates_per_s": round(n * steps / dt, 1), "batches_in_flight": D, "steps": steps,
            "ms_per_batch": round(1000 * dt / steps, 3), "all_valid": ok[0],
            "workload": f"{n} updates per batch, a distinct next_sync_committee each (configs[3]), inputs resident"}


def serving_from_host(v, sbs, D: int, steps: int, comm=None) -> dict:
    """The serving loop from HOST buffers (SURVEY §8(d)'s timed region: H2D of the packed batch + all
    kernels + D2H of the verdicts): batch k is handed to lcv_validate_async on slot k % D — staged into
    the slot's pinned buffer, uploaded by DMA on the slot's stream while the other slots' kernels run,
    validated, verdicts copied back — and the host waits for a slot only before reusing it.  Max over
    ranks for N > 1 (each rank serves its own batches)."""
    n = sbs[0].updates.n
    out_v = [np.zeros(n, np.uint8) for _ in range(D)]
    ok = [True]

    def run(k_steps):
        for k in range(k_steps):
            s = k % D
            if k >= D:
                v.slot_wait(s, n, out_v[s])
                ok[0] = ok[0] and bool((out_v[s] == 1).all())
            b = sbs[s]
            v.validate_async(b.updates, b.current_slot, b.genesis_validators_root, s)
        for k in range(max(0, k_steps - D), k_steps):
            v.slot_wait(k % D, n, out_v[k % D])
            ok[0] = ok[0] and bool((out_v[k % D] == 1).all())

    run(D)  # warm: pinned staging and device copies allocated
    if comm is not None:
        comm.barrier()
    t0 = time.perf_counter()
    run(steps)
    dt = time.perf_counter() - t0
    if comm is not None:
        dt = comm.allreduce_max(dt)
    world = comm.world if comm is not None else 1
    return {"updates_per_s": round(world * n * steps / dt, 1), "batches_in_flight": D, "steps": steps,
            "ms_per_batch": round(1000 * dt / steps, 3), "all_valid": ok[0],
            "bytes_h2d_per_update": int(sum(getattr(sbs[0].updates, f).nbytes for f in (
                "att_beacon", "att_exec", "att_branch", "fin_beacon", "fin_exec", "fin_branch", "nsc_index",
                "nsc_branch", "finality_branch", "sync_bits", "sync_signature", "signature_slot")) / n),
            "timed_region": "host PackedUpdates (pageable numpy) -> pinned staging (host memcpy) -> H2D DMA -> "
                            "every kernel -> verdict + reason D2H to pinned memory -> host; lcv_validate_async / "
                            "lcv_slot_wait"}


def latency_lines(v, sb, calls: int = 20) -> dict:
    """Single-call latency of the reference-shaped drop-ins (the per-update usage at sync-protocol.md:512
    and :464): one update validated against the resident store through the C ABI, and
    FastAggregateVerify over the 512-key committee (first call decodes and KeyValidates the keys; later
    calls with the same keys reuse the decoded table).  Medians over `calls` calls, ms."""
    from lcv import synth
    gvr = sb.genesis_validators_root
    one = sb.updates.slice(0, 1)
    v.validate(one, sb.current_slot, gvr)
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        ok, _ = v.validate(one, sb.current_slot, gvr)
        ts.append(time.perf_counter() - t0)
    pks = [sb.current.pubkeys[48 * j:48 * j + 48] for j in range(512)]
    msg = synth.signing_root(sb.updates.att_beacon[0].tobytes(), int(sb.updates.signature_slot[0]), gvr)
    sig = sb.updates.sync_signature[0].tobytes()
    pks_first = pks[1:] + pks[:1]  # a different table (order) than the later calls: a cold decode
    t0 = time.perf_counter()
    v.fast_aggregate_verify(pks_first, msg, sig)
    first = time.perf_counter() - t0
    fav_ok = v.fast_aggregate_verify(pks, msg, sig)
    tf = []
    for _ in range(calls):
        t0 = time.perf_counter()
        fav_ok &= v.fast_aggregate_verify(pks, msg, sig)
        tf.append(time.perf_counter() - t0)
    # the same single-update call on the batch engine (lcv_set_latency_mode(0)), for comparison
    prev = getattr(v, "latency_mode", 64)
    v.set_latency_mode(0)
    try:
        v.validate(one, sb.current_slot, gvr)
        tb = []
        for _ in range(calls):
            t0 = time.perf_counter()
            v.validate(one, sb.current_slot, gvr)
            tb.append(time.perf_counter() - t0)
    finally:
        v.set_latency_mode(prev)
    return {"validate_one_update_ms": round(1000 * float(np.median(ts)), 3), "validate_one_update_valid": bool(ok[0]),
            "validate_one_update_batch_engine_ms": round(1000 * float(np.median(tb)), 3),
            "fast_aggregate_verify_512_ms": round(1000 * float(np.median(tf)), 3),
            "fast_aggregate_verify_512_cold_ms": round(1000 * first, 3), "fast_aggregate_verify_valid": bool(fav_ok),
            "note": "default latency mode (lcv_set_latency_mode 64: the SOP programs of batches <= 64 rows on the "
                    "fan engine, an op's K products on K lanes, one update per block; DESIGN.md 3.5); "
                    "*_batch_engine_ms: the same call with latency mode off"}


def wire_path(v, sb, n: int) -> dict:
    """SSZ wire path, beside `value`: the batch serialised to LightClientUpdate
    SSZ bytes, decoded by the native decoder (host threads) and validated from host buffers; the
    decoded rows must reproduce the packed batch exactly (full-size round trip)."""
    from lcv import wire
    msgs = wire.encode_updates(sb.updates)
    buf = np.frombuffer(b"".join(msgs), np.uint8)
    lens = np.array([len(m) for m in msgs], np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    wire.decode_updates(msgs[:1])  # binds the library outside the timed decode
    t0 = time.perf_counter()
    wb = wire.decode_updates((buf, offs, lens))
    t_dec = time.perf_counter() - t0
    ok, _ = v.validate(wb, sb.current_slot, sb.genesis_validators_root)
    t_all = time.perf_counter() - t0
    u = sb.updates
    same = all(np.array_equal(getattr(wb, k), getattr(u, k)) for k in (
        "att_beacon", "att_exec", "att_branch", "fin_beacon", "fin_exec", "fin_branch", "nsc_branch",
        "finality_branch", "sync_bits", "sync_signature", "signature_slot"))
    pairs = np.unique(np.stack([wb.nsc_index, u.nsc_index], 1), axis=0)
    same = same and all(np.array_equal(wb.nsc_pool[a], u.nsc_pool[b]) for a, b in pairs)
    return {"bytes": int(buf.nbytes), "decode_updates_per_s": round(n / t_dec, 1),
            "decode_gb_per_s": round(buf.nbytes / t_dec / 1e9, 2),
            "decode_plus_validate_updates_per_s_1gpu": round(n / t_all, 1),
            "roundtrip_exact": bool(same), "all_valid": bool(ok.all()),
            "host_threads": min(16, os.cpu_count() or 1)}


def _opcounts():
    return json.load(open(os.path.join(ROOT, "profiles", "opcounts.json")))


def _ops(c) -> float:
    return 600 * c["fp_mul"] + 24 * c["fp_add"] + 2100 * c["sha"]


def total_ops_per_update(n: int, npool: int, section: str = "executed") -> float:
    """INT32 ops per update of the whole pipeline for a batch of n updates over npool distinct next
    committees: the per-update stages plus npool / n of the per-committee ones (HTR(SyncCommittee))."""
    c = _opcounts() if section == "executed" else _opcounts()[section]
    per = sum(_ops(d) for d in c["per_update"].values())
    return per + sum(_ops(d) for d in c.get("per_committee", {}).values()) * npool / n


# the kernels of each stage (HBM traffic and counters from profiles/<round>/pmc_*.json)
STAGE_KERNELS = {"miller_lines": "k_sop<F_sop_lines>", "miller_lines_sig": "k_sop<F_sop_lines>",
                 "miller_loop": "k_sop<F_sop_acc>",
                 "final_exp": "k_sop<F_sop_fexp>",
                 "hash_to_g2": "k_sop<F_sop_h2c>", "h2c_sswu": "k_items<F_h2c_map>",
                 "sig_decode": "k_items<F_sig>",
                 "g1_aggregate": "k_items<F_agg>", "pre_checks": "k_items<F_pre>", "signing_root": "k_items<F_sigroot>",
                 "nsc_htr": "k_team<F_nsc_team>"}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_latest.json")


def stage_pmc(stage: str):
    """rocprofv3 counters of the stage's kernel from the committed PMC summary (tools/pmc_collect.sh,
    tools/pmc_summary.py): HBM bytes per launch (FETCH_SIZE x2 on gfx950 per MI355X_MICROARCH.md, +
    WRITE_SIZE), VALU utilisation, occupancy, LDS bank conflicts."""
    if not os.path.exists(PMC_FILE) or stage not in STAGE_KERNELS:
        return None
    return json.load(open(PMC_FILE)).get("kernels", {}).get(STAGE_KERNELS[stage])


def pmc_pipe(stage: str):
    """The VALU-pipe block of the stage's kernel: the committed PMC counters (tools/pmc_summary.py) priced
    by tools/valu_model.py with the peakbench cycle costs (the same measurement as the roofline peak):
    the SIMD cycles its instruction stream needs / the SIMD cycles of the launch."""
    pmc = stage_pmc(stage)
    if not pmc or "raw" not in pmc:
        return None
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import valu_model
    return valu_model.pipe(STAGE_KERNELS[stage], pmc["raw"])


def roofline(stage_ms: dict, n: int, npool: int = 1):
    """The dominant kernel against the VALU.  Work per launch = per-update ops x n for the per-update
    stages, per-committee ops x npool for HTR(next_sync_committee) (one 64-lane tree per DISTINCT
    committee).  Op model W = 600 N_fpmul + 24 N_fpadd + 2100 N_sha; numerators
    (profiles/opcounts.json):
      * executed  — the device's own operations (tools/opcount.py over the host-simulation build of the
                    same kernel code; an SOP op of K products and one reduction = (K + 1) / 2 Fp mul):
                    the headline `frac`, every per-kernel `frac` and `pipeline_frac`;
      * canonical — the oracle's op counter on the textbook algorithms (oracle/canonical.py), reported
                    only for the stages whose device algorithm is of the same class (CANONICAL_MATCHED).
    Two denominators: the multiply-add issue peak (39.3 T = 2 x the v_mad_u64_u32 rate, `peak`) and the
    full-rate INT32 VALU peak (78.6 T).  Beside them the hardware's own statement, `valu_pipe`: the SIMD
    cycles the kernel's VALU instruction stream needs (rocprofv3 instruction counts x measured cycles per
    instruction class) over the SIMD cycles of the launch (tools/valu_model.py)."""
    path = os.path.join(ROOT, "profiles", "opcounts.json")
    if not os.path.exists(path) or not stage_ms:
        return None
    oc = _opcounts()
    canon = oc.get("canonical")

    def work(sec, stage):
        if sec is None:
            return None
        if stage in sec.get("per_committee", {}):
            return _ops(sec["per_committee"][stage]) * npool, "per committee", _ops(sec["per_committee"][stage])
        if stage in sec["per_update"]:
            return _ops(sec["per_update"][stage]) * n, "per update", _ops(sec["per_update"][stage])
        return None

    def one(stage):
        ex = work(oc, stage)
        if ex is None or stage_ms.get(stage, 0) <= 0:
            return None
        sec = stage_ms[stage] * 1e-3
        ach = ex[0] / sec / 1e12
        d = {"ms_per_launch": stage_ms[stage], "unit_of_work": ex[1], "units_per_launch": npool if ex[1] == "per committee" else n,
             "ops_executed_per_unit": ex[2], "achieved": round(ach, 3),
             "frac": round(ach / PEAK_MAC_TOPS, 4), "frac_vs_int32_valu_peak": round(ach / PEAK_INT32_VALU_TOPS, 4)}
        ca = work(canon, stage) if stage in CANONICAL_MATCHED else None
        if ca is not None:
            d["ops_canonical_per_unit"] = ca[2]
            d["frac_canonical"] = round(ca[0] / sec / 1e12 / PEAK_MAC_TOPS, 4)
        else:
            d["frac_canonical"] = None  # the textbook count is of another algorithm class (docstring)
        pp = pmc_pipe(stage)
        if pp is not None:
            # counter-only (the profiled launch's instructions x measured cycles / its GRBM cycles), and
            # live: the same cycle need over this run's event time at the nominal 2.4 GHz (the DVFS clock
            # is lower under load, so the live figure understates)
            d["valu_pipe_busy"] = pp["issue_fraction"]
            d["mad_share_of_pipe_cycles"] = pp["mad_share_of_pipe_cycles"]
            d["valu_pipe_busy_live_2p4ghz"] = round(pp["pipe_cycles_per_launch"] / (sec * 2.4e9 * 1024), 4)
        return d
    per = {k: one(k) for k in stage_ms if one(k) is not None}
    if not per:
        return None
    if any(d["frac"] > 1.0 for d in per.values()):  # an op-model or timing error: reported, not hidden
        log("bench: a per-kernel roofline fraction above 1: " + str({k: d["frac"] for k, d in per.items()}))
    stage = max(per, key=lambda k: per[k]["ms_per_launch"])
    d = per[stage]
    pmc = stage_pmc(stage) or {}
    return {"bound": "valu", "kernel": STAGE_KERNELS.get(stage, stage), "stage": stage,
            "achieved": d["achieved"], "peak": PEAK_MAC_TOPS, "unit": "T INT32 op/s", "frac": d["frac"],
            "numerator": "executed (the device's own operations, op model W of SURVEY.md 8(d))",
            "peak_is": (f"measured multiply-add issue peak: 2 ops x the v_mad_u64_u32 rate of an all-mad stream "
                        f"(tools/microbench/peakbench.hip, inline asm, wall time over all 1,024 SIMDs) at "
                        f"{PEAK_WAVES_PER_SIMD} waves/SIMD, profiles/r05_cal/peakbench.txt"),
            "peak_by_waves_per_simd": {w: measured_peaks()[("mad", w)]["op_T"] for w in (1, 2, 3, 4, 8)},
            "peak_int32_valu": PEAK_INT32_VALU_TOPS, "frac_vs_int32_valu_peak": d["frac_vs_int32_valu_peak"],
            "frac_canonical": d.get("frac_canonical"),
            "valu_pipe_busy": d.get("valu_pipe_busy"),
            "mad_share_of_pipe_cycles": d.get("mad_share_of_pipe_cycles"),
            "valu_pipe_busy_live_2p4ghz": d.get("valu_pipe_busy_live_2p4ghz"),
            "valu_pipe": pmc_pipe(stage),
            "valu_pipe_is": "the launch's VALU instructions priced by class (v_mad_u64_u32 C_MAD, other 64-bit "
                            "C_64, 32-bit C_32: peakbench cycles at 3 waves/SIMD, tools/valu_model.py) over its "
                            "SIMD cycles (GRBM_GUI_ACTIVE / 8 x 1024); rocprofv3 counters of profiles/pmc_latest.json",
            "instruction_classes": "profiles/r05_iclass/iclass.md (tools/sop_iclass.py)",
            "valu_busy_pmc": pmc.get("valu_busy"),
            "valu_busy_pmc_is": "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: one quad-cycle per VALU instruction "
                                "issued, whatever its rate (a quarter-rate v_mad_u64_u32 counts once): an issue "
                                "count per wave, not the pipe's occupancy (valu_pipe_busy)",
            "traffic": pmc.get("hbm_bytes_per_launch"), "traffic_unit": "B per launch (rocprofv3 PMC)",
            "ops_per_update_executed": d["ops_executed_per_unit"],
            "ops_per_update_canonical": d.get("ops_canonical_per_unit"),
            "ms_per_launch": d["ms_per_launch"],
            "counters": pmc or None, "per_kernel": per}


def config_lines(v) -> dict:
    """BASELINE.json configs[2], [3], [4] on this GPU (one timed pass each, inputs resident), so the
    bench line carries them beside configs[1].  10^6-row batches tile 65,536 generated rows (rows are
    independent); every verdict must equal its construction."""
    from lcv import synth
    out = {}

    def timed(sb, label, reps=2, tiled=None):
        v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
        rb = v.upload(sb.updates)
        try:
            vv, rr = v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root)  # warm + check
            ok = bool(np.array_equal(rr, sb.expected_reason))
            t0 = time.perf_counter()
            for _ in range(reps):
                v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root, vv, rr)
            dt = (time.perf_counter() - t0) / reps
            stages = {k: round(ms, 3) for k, ms in v.last_timings().items() if ms > 0}
        finally:
            rb.free()
        return {"workload": label, "n": sb.updates.n, "updates_per_s": round(sb.updates.n / dt, 1),
                "ms_per_pass": round(1000 * dt, 3), "verdicts_match_construction": ok,
                "valid_fraction": round(float((sb.expected_reason == 0).mean()), 4), "stage_kernel_ms": stages,
                "rows": tiled or "every row generated"}
    t0 = time.perf_counter()
    base = synth.generate(v, 15625, seed=3, participation="random")
    sb2 = synth.tile(base, 8)
    out["configs[2]"] = timed(sb2, "125,000 updates (the 1M / 8-GPU batch's per-GPU shard), "
                                   "random participation 342..512",
                              tiled="15,625 generated rows tiled x8 (rows are independent)")
    # the masked pubkey gather of g1_aggregate (north star: HBM GB/s of the gather): a lane reads the
    # affine points (96 B) of the non-participants (> 256 participants: subtracted from the committee's
    # precomputed sum) or of the participants (<= 256) from the resident 49 KB committee table
    # measured on one 15,625-row chunk validated alone (the multi-chunk passes above overlap their
    # chunks on the work-space slots, so their per-stage event times include other chunks' kernels)
    pc = np.unpackbits(base.updates.sync_bits, axis=1).sum(axis=1)
    gathered = np.where(pc > 256, 512 - pc, pc).astype(np.float64) * 96
    v.set_store(base.store_finalized_slot, base.current.ssz, base.next.ssz)
    rb = v.upload(base.updates)
    try:
        for _ in range(2):
            v.validate_resident(rb, base.current_slot, base.genesis_validators_root)
        agg_ms = v.last_timings().get("g1_aggregate", 0.0)
    finally:
        rb.free()
    out["configs[2]"]["pubkey_gather"] = {
        "rows": base.updates.n, "bytes_per_update": round(float(gathered.mean()), 1),
        "g1_aggregate_ms": round(agg_ms, 3),
        "GB_per_s": round(float(gathered.sum()) / (agg_ms * 1e-3) / 1e9, 1) if agg_ms else None,
        "note": "algorithmic bytes / g1_aggregate kernel time (k_team<F_agg_team>, 4 lanes per update); the "
                "2 x 512-point table stays in L2/MALL, so this is gather bandwidth from cache, far below "
                "the 8 TB/s HBM roofline (each lane runs a chain of mixed additions)"}
    sb3 = synth.generate(v, 10000, seed=4, npool=10000)
    out["configs[3]"] = timed(sb3, "10,000 Deneb updates, all branches, a DISTINCT next_sync_committee each "
                                   "(HTR(SyncCommittee) per update)")
    kinds = synth.adversarial_kinds(16384, seed=5, bad_fraction=0.10)
    b4 = synth.generate(v, 16384, seed=5, participation="random", kinds=kinds)
    out["configs[4]"] = timed(synth.tile(b4, 64), "1,048,576 adversarial updates on one GPU: 10% bad (bad "
                                                  "signature message/encoding, corrupted branch, sub-2/3 "
                                                  "participation = VALID)", reps=1,
                                tiled="16,384 generated rows tiled x64 (rows are independent)")
    # the kernels with a full chip of work: one 65,536-row chunk validated alone (serial stages, one launch
    # per kernel), so each launch has 6.5x the waves of a configs[1] launch
    t1 = time.perf_counter()
    full = synth.tile(synth.generate(v, 8192, seed=6), 8)  # configs[1]'s row shape: valid, 512/512
    v.set_store(full.store_finalized_slot, full.current.ssz, full.next.ssz)
    rb = v.upload(full.updates)
    try:
        v.validate_resident(rb, full.current_slot, full.genesis_validators_root)
        v.validate_resident(rb, full.current_slot, full.genesis_validators_root)
        st = {k: ms for k, ms in v.last_timings().items() if ms > 0}
    finally:
        rb.free()
    rf = roofline(st, full.updates.n, int(full.updates.nsc_pool.shape[0]))
    if rf is not None:
        out["roofline_full_chip"] = {
            "workload": f"{full.updates.n} configs[1]-shaped rows (valid, full participation) in one chunk, "
                        "one batch at a time (6.5x the waves of a configs[1] launch)",
            "per_kernel": {k: {"ms_per_launch": round(d["ms_per_launch"], 3), "frac": d["frac"],
                               "frac_vs_int32_valu_peak": d["frac_vs_int32_valu_peak"],
                               "frac_canonical": d["frac_canonical"]}
                           for k, d in rf["per_kernel"].items()},
            "note": "miller_loop and final_exp run alone on the chip; the two line walks run concurrently "
                    "(one per stream) as do pre_checks/sig_decode beside signing_root/h2c_sswu/hash_to_g2, "
                    "so their event-timed durations overlap and their fractions are lower bounds.  nsc_htr "
                    "hashes the batch's one distinct committee (a single 64-lane tree)"}
    log(f"configs[2..4] lines in {time.perf_counter() - t0:.1f}s (full-chip roofline {time.perf_counter() - t1:.1f}s)")
    return out


if __name__ == "__main__":
    main()
