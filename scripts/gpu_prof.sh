#!/bin/bash
# rocprofv3 kernel-trace + stats of a bench run; summarised on the box (the raw trace is too
# big to ship back) into gpurun_out/${PROF_NAME:-prof}/summary.md.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/${PROF_NAME:-prof}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
python -m ome_amd.build > gpurun_out/build.log 2>&1 || exit 1
STEPS=${PROF_STEPS:-200}
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${PROF_NAME:-prof} -o run --output-format csv -- python3 $R/bench.py --steps $STEPS --warmup ${PROF_WARMUP:-200} ${BENCH_ARGS} > $R/gpurun_out/${PROF_NAME:-prof}_bench.log 2>&1
rc=$?
cd $R
grep -v amdgpu.ids gpurun_out/${PROF_NAME:-prof}_bench.log | tail -2 | cut -c1-300
[ $rc -eq 0 ] || exit $rc
python scripts/prof_summary.py gpurun_out/${PROF_NAME:-prof} $((STEPS * 8)) > gpurun_out/${PROF_NAME:-prof}/summary.md && head -40 gpurun_out/${PROF_NAME:-prof}/summary.md
find gpurun_out/${PROF_NAME:-prof} -name "*kernel_trace.csv" -delete
exit 0
