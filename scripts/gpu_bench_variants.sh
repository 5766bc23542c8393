#!/bin/bash
# Bench variants on one MI355X: baseline / mixed-chunk / TunableOp-tuned decode GEMMs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m ome_amd.build > gpurun_out/build.log 2>&1 || exit 1
run() {  # name, env..., -- args
  local name=$1; shift
  echo "== $name" ; date
  env "$@" > "gpurun_out/b_${name}.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/b_${name}.log"
  return $rc
}
run base OME_TUNE_GEMM=0 timeout -k 10 420 python bench.py --steps 400 --warmup 200 &&
run mixed OME_TUNE_GEMM=0 timeout -k 10 420 python bench.py --steps 400 --warmup 200 --mixed-chunk &&
run tuned_mixed OME_TUNE_GEMM=1 timeout -k 10 600 python bench.py --steps 400 --warmup 200 --mixed-chunk &&
run tuned_mixed2 OME_TUNE_GEMM=1 timeout -k 10 420 python bench.py --steps 400 --warmup 200 --mixed-chunk
rc=$?
cp -f ome_amd/_tuned/*.csv gpurun_out/ 2>/dev/null
exit $rc
