#!/bin/bash
# One gpurun call: build, GPU numerics tests, short bench, rocprof summary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m ome_amd.build > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  rc=$?
  tail -5 gpurun_out/bench.log
  exit $rc
fi
