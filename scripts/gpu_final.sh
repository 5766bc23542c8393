#!/bin/bash
# Round-end rehearsal on one box: the GPU suite, smoke(), the driver's default bench and a
# 20-step bench (what the driver runs, in its order).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/final_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/final_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/final_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
grep -E '^\{' gpurun_out/final_bench.log | cut -c1-600
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench20.log 2>&1 || { tail -20 gpurun_out/final_bench20.log; exit 1; }
grep -E '^\{' gpurun_out/final_bench20.log | cut -c1-600
