#!/bin/bash
# Pipeline-shape sweep: bench at several (streams, slices) shapes of lcv_set_pipeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for p in ${SHAPES:-2,2 3,3 4,4}; do
  timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-configs --pipeline $p > gpurun_out/sweep_$p.json 2> gpurun_out/sweep_$p.err || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_$p.json')); print('$p', d['value'], d['ms_per_step'], d['serial_ms_per_step'])" | tee -a gpurun_out/sweep.txt
done
