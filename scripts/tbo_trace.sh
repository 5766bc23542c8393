#!/bin/bash
# Two-batch overlap under a rocprofv3 kernel trace: 2 ranks sharing GPU 0 (DP attention + EP over
# the IPC low-latency exchange), TBO off then on, one rocprofv3 per rank started from this shell
# (no launcher, no re-exec), then scripts/tbo_trace.py summarises each rank's trace.
#   bash scripts/tbo_trace.sh  -> gpurun_out/tbo_trace/{off,on}/r{0,1}/... + summary_{off,on}.md
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/tbo_trace
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MASTER_ADDR=127.0.0.1
port=29631
for m in ${TBO_MODES:-off on}; do
  pids=()
  for r in 0 1; do
    (cd /tmp && MASTER_PORT=$port timeout -k 10 400 \
      rocprofv3 --kernel-trace -d $O/$m/r$r -o run --output-format csv -- \
      python3 $R/scripts/tbo_bench.py --rank $r --modes $m ${TBO_ARGS} > $O/$m.r$r.log 2>&1) &
    pids+=($!)
  done
  rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  [ $rc -eq 0 ] || { echo "mode $m failed rc=$rc"; tail -n 5 $O/$m.r0.log $O/$m.r1.log; exit $rc; }
  echo "TBO $m: $(grep -h '"tok_s"' $O/$m.r0.log)"
  python3 $R/scripts/tbo_trace.py $O/$m > $O/summary_$m.md || exit 1
  find $O/$m -name "*kernel_trace.csv" -size +20M -delete
  port=$((port + 1))
done
exit 0
