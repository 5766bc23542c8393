#!/bin/bash
# Prefill-batching sweep on the headline bench (tok/s vs p50 TTFT).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "0 50" "1024 40" "2048 60" "4096 100"; do
  set -- $cfg
  OME_PREFILL_BATCH_TOKENS=$1 OME_PREFILL_MAX_WAIT_MS=$2 timeout -k 10 300 python bench.py --steps 300 --warmup 200 \
    > gpurun_out/pb_$1.log 2>&1 || { tail -5 gpurun_out/pb_$1.log; exit 1; }
  echo "tokens=$1 wait=$2 $(grep -o '"value": [0-9.]*' gpurun_out/pb_$1.log) $(grep -o '"p50_ttft_ms": [0-9.]*' gpurun_out/pb_$1.log)"
done
