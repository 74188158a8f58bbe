#!/bin/bash
# Latency A/B of liblcv.so builds on ONE box: ab/liblcv_<V>.so for V in $VARIANTS (default "A B") copied
# into lcv/liblcv.so in turn, tools/latency_breakdown.py on the fan engine (one update), ROUNDS passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/lat_ab}
mkdir -p $OUT
LIB=light-client-consensus-specs_amd/lcv/liblcv.so
cp $LIB $OUT/.liblcv_orig.so
trap 'cp $OUT/.liblcv_orig.so $LIB' EXIT
for i in ${ROUNDS:-1 2}; do
  for v in ${VARIANTS:-A B}; do
    cp ${ABDIR:-abp}/liblcv_$v.so $LIB &&
    LCV_LAT_MODES=64 LCV_LAT_NS=1 LCV_LAT_REPS=20 timeout -k 10 200 python -u tools/latency_breakdown.py \
      > $OUT/lat_${v}_$i.json 2> $OUT/lat_${v}_$i.err || exit 1
    if [ -n "${POW:-}" ]; then
      timeout -k 10 120 python -u tools/pow_timing.py > $OUT/pow_${v}_$i.json 2> $OUT/pow_${v}_$i.err || exit 1
      echo "$v $i pow $(cat $OUT/pow_${v}_$i.json)"
    fi
    python -c "
import json; d=json.load(open('$OUT/lat_${v}_$i.json'))['latency_engine_n1']
s=d['stage_ms']; print('$v', $i, d['wall_ms_median'], {k: s[k] for k in ('nsc_htr','pre_checks','sig_decode','h2c_sswu','hash_to_g2','miller_loop','final_exp') if k in s})"
  done
done
