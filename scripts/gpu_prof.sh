#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
python -m ome_amd.build > gpurun_out/build.log 2>&1 || exit 1
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py ${BENCH_ARGS:---steps 100 --warmup 50} > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
