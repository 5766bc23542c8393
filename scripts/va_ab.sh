#!/bin/bash
# varlen attention A/B on one GPU: encoder GPU tests with the default and the SUB=2 fast body,
# then scripts/varlen_attn_bench.py for generic / fast SUB 1 / fast SUB 2 (one process each:
# the launcher reads the variables once).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/va.txt
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encoder_gpu.py > gpurun_out/va_test.log 2>&1 || exit $?
OME_VARLEN_SUB=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encoder_gpu.py >> gpurun_out/va_test.log 2>&1 || exit $?
for f in "0 1" "1 1" "1 2"; do
  set -- $f
  OME_VARLEN_FAST=$1 OME_VARLEN_SUB=$2 timeout -k 10 200 python -u scripts/varlen_attn_bench.py > gpurun_out/va_one.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/va_one.txt | sed "s/^/fast $1 sub $2 /" >> gpurun_out/va.txt
done
