#!/bin/bash
# HBM traffic of every kernel of one serial bench step (FETCH_SIZE and WRITE_SIZE in separate passes,
# as MI355X_MICROARCH.md prescribes; FETCH_SIZE is doubled for gfx950 when it is reported).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/traffic/fetch -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 1,1 > gpurun_out/traffic/fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/traffic/write -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 1,1 > gpurun_out/traffic/write.log 2>&1 &&
echo traffic ok
