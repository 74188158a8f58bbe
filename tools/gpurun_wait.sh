#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool has no box or slot for it (nothing ran,
# nothing charged: gpurun's transient answers).  Any call that ran — pass or fail — is final.
#   tools/gpurun_wait.sh TIMEOUT 'command'   (log: gpurun_out/.wait.log)
T=$1; shift
mkdir -p gpurun_out
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > gpurun_out/.wait.log 2>&1
  rc=$?
  if grep -q "status=transient" gpurun_out/.wait.log && grep -qE "nothing was charged|no free box|retry in|stopped responding" gpurun_out/.wait.log; then
    sleep 90
    continue
  fi
  cat gpurun_out/.wait.log
  exit $rc
done
cat gpurun_out/.wait.log
exit 3
