#!/bin/bash
# PP=2 rehearsal (Llama-3-8B, both stages sharing GPU 0, IPC hand-offs) under a rocprofv3 kernel
# trace, decode graphs off (OME_PP_GRAPHS=0) then on: one rocprofv3 per rank (each rank is its own
# process, started from this shell -- no launcher in between), per-kernel stats per rank.
#   bash scripts/pp_trace.sh  -> gpurun_out/pp_trace/g{0,1}/r{0,1}/…kernel_stats.csv + bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/pp_trace
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 OME_BENCH_SHARE_GPU=1 OME_TUNE_GEMM=0 MASTER_ADDR=127.0.0.1 \
  WORLD_SIZE=2 LOCAL_WORLD_SIZE=2
port=29611
for g in ${PP_MODES:-0 1}; do
  pids=()
  for r in 0 1; do
    if [ "${NOPROF:-0}" = 1 ]; then   # plain timing run (same launch, no profiler)
      (cd /tmp && RANK=$r LOCAL_RANK=$r MASTER_PORT=$port OME_PP_GRAPHS=$g timeout -k 10 500 \
        python3 $R/bench.py --gpus 2 --pp 2 --steps ${STEPS:-6} --warmup 2 --no-e2e-block \
        > $O/g$g.r$r.log 2>&1) &
    else
      (cd /tmp && RANK=$r LOCAL_RANK=$r MASTER_PORT=$port OME_PP_GRAPHS=$g timeout -k 10 500 \
        rocprofv3 --kernel-trace --stats -d $O/g$g/r$r -o run --output-format csv -- \
        python3 $R/bench.py --gpus 2 --pp 2 --steps ${STEPS:-6} --warmup 2 --no-e2e-block \
        > $O/g$g.r$r.log 2>&1) &
    fi
    pids+=($!)
  done
  rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  [ $rc -eq 0 ] || { echo "mode $g failed rc=$rc"; exit $rc; }
  echo "OME_PP_GRAPHS=$g $(grep -h '"metric"' $O/g$g.r0.log)" | tee -a $O/bench_lines.txt
  [ -d $O/g$g ] && find $O/g$g -name "*kernel_trace.csv" -size +20M -delete
  port=$((port + 1))
done
exit 0
