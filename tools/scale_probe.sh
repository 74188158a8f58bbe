#!/bin/bash
# Stage times vs updates per GPU (latency- vs throughput-bound probe): one bench line per n.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in ${NS:-2500 5000 10000 20000 40000}; do
  timeout -k 10 240 python -u bench.py --n $n --steps 3 --warmup 1 --no-cpu-baseline --no-configs > gpurun_out/scale_$n.json 2> gpurun_out/scale_$n.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/scale_$n.json'))
print($n, 'value', round(d['value']), 'ms', d['ms_per_step'], {k: v for k, v in d['stage_kernel_ms_per_step'].items() if v > 0.3})"
done
