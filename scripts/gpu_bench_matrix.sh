#!/bin/bash
# GPU tests + a matrix of bench variants (each its own time limit; stop at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m ome_amd.build > gpurun_out/build.log 2>&1 || exit 1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
run() {  # name, args...
  local name=$1; shift
  echo "== $name $*"
  timeout -k 10 420 python bench.py "$@" > "gpurun_out/b_${name}.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "gpurun_out/b_${name}.log" | tail -2 | cut -c1-330
  return $rc
}
IFS=';' read -ra VARIANTS <<< "${VARIANTS:-default:;nooverlap:--no-overlap}"
for v in "${VARIANTS[@]}"; do
  name=${v%%:*}; args=${v#*:}
  run "$name" $args || exit $?
done
cp -f ome_amd/_tuned/*.csv gpurun_out/ 2>/dev/null
exit 0
