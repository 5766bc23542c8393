#!/bin/bash
# One gpurun call: selected GPU tests (PYTEST_FILES) then optional bench (BENCH_ARGS) and an
# optional rocprof summary (PROF=1).  Every GPU step has its own time limit; the first failure ends
# the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$PYTEST_FILES" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread $PYTEST_FILES \
      > gpurun_out/pytest_step.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_step.log | tail -40
  [ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_step.log; exit $rc; }
fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py $BENCH_ARGS > gpurun_out/bench_step.log 2> gpurun_out/bench_step.err
  rc=$?
  tail -3 gpurun_out/bench_step.log; grep -v amdgpu.ids gpurun_out/bench_step.err | tail -8
  [ $rc -ne 0 ] && exit $rc
fi
exit 0
