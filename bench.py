#!/usr/bin/env python3
"""Benchmark: verified LightClientUpdates/sec (512-member committee) on 1..8 MI355X.

One step = `validate_light_client_updates` over this rank's resident batch of synthetic
mainnet-preset Deneb updates (BASELINE.json configs[1]: 10,000 updates per GPU, full 512/512
participation, every update carrying next_sync_committee + finality + execution branches), i.e.
every kernel of the hot path (SSZ/SHA-256, hash_to_G2, signature decode + subgroup check, masked G1
aggregation, Miller loop, final exponentiation, verdicts).  Inputs are resident in HBM (uploaded
once, outside the timed region); for N > 1 each step ends with an RCCL all-gather of the per-rank
verdict bytes (the only collective of the design).  Weak scaling: every rank owns `--n` updates.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n UPDATES_PER_GPU] [--participation full|random]
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

PEAK_INT32_TOPS = 39.3  # 256 CU x 64 lanes x 2.4 GHz; the box-measured mad rate is reported beside it


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(sample: int, seed: int = 3):
    """The CPU oracle (oracle/, a pure-Python restatement of the path) timed on this host, one core,
    on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import helpers as H
    from lcv import synth
    v = H.hostsim_verifier() if os.path.exists(H.HOSTSIM) else None
    if v is None:
        return None
    sb = synth.generate(v, sample, seed=seed)
    store = H.store_from(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    ups = [H.update_from(sb.updates, i) for i in range(sample)]
    # warm the per-key KeyValidate cache (a per-store cost, like the device's lcv_set_store)
    H.O.validate_light_client_update(store, ups[0], sb.current_slot, sb.genesis_validators_root)
    t0 = time.perf_counter()
    for u in ups:
        r = H.O.validate_light_client_update(store, u, sb.current_slot, sb.genesis_validators_root)
        assert r == 0
    dt = time.perf_counter() - t0
    return {"value": round(sample / dt, 3), "unit": "updates/s", "cores": 1, "kind": "port",
            "sample": f"{sample} synthetic Deneb updates (512/512, all branches), oracle/sync_protocol.py "
                      f"single process; committee KeyValidate cache warmed first"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=10000, help="updates per GPU (configs[1]: 10,000)")
    ap.add_argument("--participation", default="full", choices=["full", "random"])
    ap.add_argument("--cpu-sample", type=int, default=12)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipeline", default="1,1", help="STREAMS,SLICES of the timed run (1,1 = serial stages)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    from lcv import synth
    from lcv.device import Verifier

    v = Verifier(local)
    t0 = time.perf_counter()
    sb = synth.generate(v, args.n, seed=2 + rank, participation=args.participation)
    log(f"[rank {rank}] generated {args.n} updates in {time.perf_counter() - t0:.1f}s")
    v.set_store(sb.store_finalized_slot, sb.current.ssz, sb.next.ssz)
    rb = v.upload(sb.updates)
    pipe = tuple(int(x) for x in args.pipeline.split(","))
    v.set_pipeline(*pipe)
    verdict = np.zeros(args.n, np.uint8)
    reason = np.zeros(args.n, np.uint8)

    if dist is not None:
        import torch
        vdev = torch.zeros(args.n, dtype=torch.uint8, device=f"cuda:{local}")
        gathered = torch.zeros(world * args.n, dtype=torch.uint8, device=f"cuda:{local}")

    def step():
        if dist is None:
            v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root, verdict, reason)
        else:
            v.validate_resident_dev(rb, sb.current_slot, sb.genesis_validators_root, vdev.data_ptr())
            dist.all_gather_into_tensor(gathered, vdev)

    def sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        step()
    # correctness of what is timed: every synthetic update is valid
    if dist is None:
        v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root, verdict, reason)
        ok_all = bool((verdict == 1).all())
    else:
        step()
        import torch
        torch.cuda.synchronize()
        ok_all = bool((gathered == 1).all().item())
    serial = pipe == (1, 1)
    stage_ms = {k: 0.0 for k in v.last_timings()}
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if serial:  # stage kernel times: HIP events on each stage's stream, inside the timed region
            for k, ms in v.last_timings().items():
                stage_ms[k] += ms
    sync()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    serial_ms, serial_ok = 1000 * dt / args.steps, ok_all
    if not serial:
        # a multi-stream pipeline overlaps stages, so per-stage kernel times come from the serial
        # shape (no other kernel sharing the GPU), run after the timed region
        v.set_pipeline(1, 1)
        ts = time.perf_counter()
        for _ in range(args.steps):
            v.validate_resident(rb, sb.current_slot, sb.genesis_validators_root, verdict, reason)
            for k, ms in v.last_timings().items():
                stage_ms[k] += ms
        serial_ms = 1000 * (time.perf_counter() - ts) / args.steps
        serial_ok = bool((verdict == 1).all())
        v.set_pipeline(*pipe)

    # PCIe-inclusive rate (host batch -> device each time), reported beside `value`, never as it
    t1 = time.perf_counter()
    v.validate(sb.updates, sb.current_slot, sb.genesis_validators_root)
    pcie_rate = args.n / (time.perf_counter() - t1)

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return
    wire_out = wire_path(v, sb, args.n)
    total = world * args.n * args.steps
    stage_avg = {k: round(ms / args.steps, 3) for k, ms in stage_ms.items()}
    kernel_ms = sum(stage_avg.values())
    roof = roofline(stage_avg, args.n)
    if roof is not None:  # the whole pipeline's rate against the same peak (all stages, all kernels)
        roof["pipeline_ops_per_update"] = total_ops_per_update()
        roof["pipeline_achieved"] = round(roof["pipeline_ops_per_update"] * total / dt / world / 1e12, 3)
        roof["pipeline_frac"] = round(roof["pipeline_achieved"] / PEAK_INT32_TOPS, 4)
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
                               f"next_sync_committee + finality + execution branches",
                   "updates_per_gpu": args.n, "committee": 512, "parallelism": f"dp{world} (independent updates)"},
        "all_valid": ok_all and serial_ok,
        "pipeline": {"streams": pipe[0], "slices": pipe[1]},
        "serial_ms_per_step": round(serial_ms, 3),
        "serial_kernel_ms_per_step": round(kernel_ms, 3),
        "serial_stage_ms_per_step": stage_avg,
        "pcie_inclusive_updates_per_s_1gpu": round(pcie_rate, 1),
        "roofline": roof,
        "wire": wire_out,
    }
    if not args.no_cpu_baseline and world == 1:
        try:
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample)
        except Exception as e:  # reported, never fatal to the GPU measurement
            out["cpu_baseline"] = {"error": repr(e)}
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


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


def total_ops_per_update():
    c = json.load(open(os.path.join(ROOT, "profiles", "opcounts.json")))["total_per_update"]
    return 600 * c["fp_mul"] + 24 * c["fp_add"] + 2100 * c["sha"]


# stages whose kernels merged into another stage's kernel (the Miller team program computes the lines
# and the accumulation: its op count is the sum of both host-simulation stages)
MERGED = {"miller_accumulate": ["miller_lines"], "sig_decode": ["miller_lines_sig"]}
# the kernels of each stage (HBM traffic from profiles/traffic_pmc.json, tools/pmc_traffic.sh)
STAGE_KERNELS = {"miller_accumulate": ["k_eng<F_eng_miller>"], "final_exp": ["k_eng<F_eng_fexp>"],
                 "hash_to_g2": ["k_items<F_h2c_map>", "k_eng<F_eng_h2c>"],
                 "sig_decode": ["k_items<F_sig>", "k_eng<F_eng_g2sub>"]}


def stage_traffic(stage: str):
    """HBM bytes per launch of a stage's kernels from the committed rocprofv3 PMC passes (FETCH_SIZE
    doubled for gfx950 per MI355X_MICROARCH.md, + WRITE_SIZE), or None."""
    path = os.path.join(ROOT, "profiles", "traffic_pmc.json")
    if not os.path.exists(path) or stage not in STAGE_KERNELS:
        return None
    t = json.load(open(path))
    tot = 0.0
    for k in STAGE_KERNELS[stage]:
        if k not in t:
            return None
        tot += 2 * t[k]["FETCH_SIZE_KB_per_launch"] + t[k]["WRITE_SIZE_KB_per_launch"]
    return round(tot * 1024)


def roofline(stage_ms: dict, n: int):
    """Dominant kernel stage vs the INT32 VALU peak.  Algorithmic work per update per stage comes from
    profiles/opcounts.json (counted by the host-simulation build of the same kernels, tools/opcount.py):
    W = 600 N_fpmul + 24 N_fpadd + 2100 N_sha (SURVEY.md §8(d) op model)."""
    path = os.path.join(ROOT, "profiles", "opcounts.json")
    if not os.path.exists(path) or not stage_ms:
        return None
    counts = json.load(open(path))["per_update"]
    stage = max(stage_ms, key=lambda k: stage_ms[k])
    if stage not in counts or stage_ms[stage] <= 0:
        return None
    ops = 0.0
    for st in [stage] + MERGED.get(stage, []):
        c = counts.get(st, {"fp_mul": 0, "fp_add": 0, "sha": 0})
        ops += 600 * c["fp_mul"] + 24 * c["fp_add"] + 2100 * c["sha"]
    achieved = ops * n / (stage_ms[stage] * 1e-3) / 1e12
    return {"bound": "valu", "kernel": stage, "achieved": round(achieved, 3), "peak": PEAK_INT32_TOPS,
            "unit": "T INT32 op/s", "frac": round(achieved / PEAK_INT32_TOPS, 4),
            "traffic": stage_traffic(stage), "traffic_unit": "B per launch (rocprofv3 PMC)",
            "ops_per_update": ops, "ms_per_launch": stage_ms[stage]}


if __name__ == "__main__":
    main()
