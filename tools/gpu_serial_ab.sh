#!/bin/bash
# One-batch-at-a-time A/B of liblcv.so builds on ONE box: abp/liblcv_<V>.so for V in $VARIANTS, bench.py
# --quick (serial stage times, HIP events), ROUNDS passes; prints the stage times of the pairing kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/serial_ab}
mkdir -p $OUT
LIB=light-client-consensus-specs_amd/lcv/liblcv.so
cp $LIB $OUT/.liblcv_orig.so
trap 'cp $OUT/.liblcv_orig.so $LIB' EXIT
for i in ${ROUNDS:-1 2}; do
  for v in ${VARIANTS:-A B}; do
    cp abp/liblcv_$v.so $LIB &&
    timeout -k 10 200 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --quick ${BENCH_ARGS:-} \
      > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || exit 1
    python -c "
import json; d=json.load(open('$OUT/b_${v}_$i.json')); s=d['stage_kernel_ms_per_step']
print('$v', $i, round(d['value']), d['serial_ms_per_step'], {k: s.get(k) for k in (${KEYS:-'miller_loop', 'miller_lines', 'miller_lines_sig', 'final_exp', 'hash_to_g2', 'g1_aggregate'})})"
  done
done
