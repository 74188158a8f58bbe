#!/bin/bash
# configs[1] throughput by batches in flight (bench.py --depth D), ROUNDS passes over DEPTHS on one box.
#   OUT=gpurun_out/<tag> tools/depth_sweep.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/depth}
mkdir -p $OUT
for i in ${ROUNDS:-1 2}; do
  for D in ${DEPTHS:-1 2 3 4 6 8}; do
    timeout -k 10 240 python -u bench.py --depth $D --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline --no-configs --quick \
      > $OUT/d${D}_$i.json 2> $OUT/d${D}_$i.err || exit 1
    python -c "
import json; d=json.load(open('$OUT/d${D}_$i.json')); print('depth', $D, 'pass', $i, d['value'], d['ms_per_step'])" | tee -a $OUT/depth_sweep.txt
  done
done
