set -o pipefail
mkdir -p gpurun_out/r04_q2
timeout -k 10 60 tools/microbench/quadtrace > gpurun_out/r04_q2/quadtrace.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_latency_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04_q2/pytest_latency.txt 2>&1 &&
timeout -k 10 200 python -u tools/latency_breakdown.py > gpurun_out/r04_q2/latency.json 2> gpurun_out/r04_q2/latency.err
