#!/bin/bash
# Engine headline A/B over the chunked-prefill budget (interleaved, one box): bench.py at
# 2048 / 4096 / 8192 prefill tokens per step, twice each.  Results -> gpurun_out/r04/chunk_ab.txt
set -o pipefail
mkdir -p gpurun_out/r04
for c in 2048 4096 8192 2048 4096 8192; do
  timeout -k 10 240 python -u bench.py --no-e2e-block --steps 20 --warmup 5 --chunked-prefill-size $c \
    > gpurun_out/r04/chunk_$c.log 2>&1 || exit 1
  grep '^{' gpurun_out/r04/chunk_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk $c', d['value'], d['p50_ttft_ms'])" >> gpurun_out/r04/chunk_ab.txt || exit 1
done
