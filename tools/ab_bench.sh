#!/bin/bash
# A/B of two liblcv.so builds on ONE box (box-to-box spread is ~2 %): alternates ab/liblcv_A.so and
# ab/liblcv_B.so into lcv/liblcv.so, short configs[1] bench each (no CPU baseline / config lines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
LIB=light-client-consensus-specs_amd/lcv/liblcv.so
cp $LIB gpurun_out/.liblcv_orig.so
trap 'cp gpurun_out/.liblcv_orig.so $LIB' EXIT  # the original library is back whatever happens
for i in ${ROUNDS:-1 2}; do
  for v in A B; do
    cp ab/liblcv_$v.so $LIB &&
    timeout -k 10 240 python -u bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-configs \
      > gpurun_out/ab_${v}_$i.json 2> gpurun_out/ab_${v}_$i.err || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/ab_${v}_$i.json'))
print('$v', $i, d['value'], d['value_one_batch_at_a_time'], d['stage_kernel_ms_per_step'])"
  done
done
cp gpurun_out/.liblcv_orig.so $LIB
