#!/bin/bash
# One gpurun call: GPU numerics tests, headline bench (bf16), fp8-KV exploration bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 300 --warmup 200 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
if [ -n "$FP8KV" ]; then
  timeout -k 10 600 python bench.py --steps 300 --warmup 200 --kv-cache-dtype fp8 > gpurun_out/bench_fp8kv.log 2>&1 || { tail -20 gpurun_out/bench_fp8kv.log; exit 1; }
  tail -2 gpurun_out/bench_fp8kv.log
fi
