#!/bin/bash
# Bench A/B of liblcv.so builds on ONE box (box-to-box spread is ~2-4 %): abp/liblcv_<V>.so for V in
# $VARIANTS copied into lcv/liblcv.so in turn; full bench line (configs included, no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/bench_ab}
mkdir -p $OUT
LIB=light-client-consensus-specs_amd/lcv/liblcv.so
cp $LIB $OUT/.liblcv_orig.so
trap 'cp $OUT/.liblcv_orig.so $LIB' EXIT
for i in ${ROUNDS:-1 2}; do
  for v in ${VARIANTS:-A B}; do
    cp abp/liblcv_$v.so $LIB &&
    timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline \
      > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit 1
    python -c "
import json; d=json.load(open('$OUT/bench_${v}_$i.json')); c=d['configs']
print('$v', $i, round(d['value']), round(d['value_h2d_inclusive']), {k: round(c[k]['updates_per_s']) for k in ('configs[2]','configs[3]','configs[4]')}, d['latency']['validate_one_update_ms'])"
  done
done
