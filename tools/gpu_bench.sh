#!/bin/bash
# GPU call for a quick performance check: smoke, then one short bench (no CPU baseline / config lines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-configs > gpurun_out/bench.json 2> gpurun_out/bench.err &&
python -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'valid', d['all_valid'])
print(d['stage_kernel_ms_per_step'])"
