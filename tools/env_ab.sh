#!/bin/bash
# Same-box A/B of an environment knob read at lcv_init: short configs[1] benches alternating the values
# of $VAR over $VALUES ("-" = unset), ROUNDS times.   VAR=LCV_SOP_ITEMS_FEXP VALUES="- 4 3" tools/env_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in ${ROUNDS:-1 2}; do
  for val in ${VALUES}; do
    if [ "$val" = "-" ]; then unset $VAR; else export $VAR=$val; fi
    timeout -k 10 240 python -u bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-configs \
      > gpurun_out/env_${val}_$i.json 2> gpurun_out/env_${val}_$i.err || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/env_${val}_$i.json'))
pk=d['roofline']['per_kernel']['final_exp']
print('$VAR=$val', $i, d['value'], d['value_one_batch_at_a_time'], 'final_exp ms', pk.get('ms_per_launch'), 'frac', pk.get('frac'), d['stage_kernel_ms_per_step'])"
  done
done
unset $VAR
