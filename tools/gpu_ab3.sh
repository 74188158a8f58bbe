#!/bin/bash
# Same-box A/B of liblcv.so variants (round 6): abp/liblcv_<V>.so for V in $VARIANTS, copied into lcv/liblcv.so
# in turn; a short configs[1] bench each (serving rate, one batch at a time, per-stage kernel ms, one-update
# latency).  First the GPU parity tests named by $TESTS on the tree's own library (the candidate).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab3}
mkdir -p $OUT
LIB=light-client-consensus-specs_amd/lcv/liblcv.so
cp $LIB $OUT/.liblcv_orig.so
trap 'cp $OUT/.liblcv_orig.so $LIB' EXIT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for i in ${ROUNDS:-1 2 3}; do
  for v in ${VARIANTS:-A B}; do
    cp abp/liblcv_$v.so $LIB &&
    timeout -k 10 240 python -u bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-configs \
      > $OUT/ab_${v}_$i.json 2> $OUT/ab_${v}_$i.err || exit 1
    python -c "
import json; d=json.load(open('$OUT/ab_${v}_$i.json')); s=d.get('stage_kernel_ms_per_step', {})
print('$v', $i, round(d['value']), round(d['value_one_batch_at_a_time']), {k: round(s[k], 3) for k in ('final_exp', 'miller_loop', 'miller_lines', 'hash_to_g2') if k in s}, d['latency']['validate_one_update_ms'])"
  done
done
