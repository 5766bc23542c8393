#!/bin/bash
# varlen attention timing probes (wrong results by design): 0 normal, 1 no V image writes,
# 2 no global K/V loads.  One process each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/va_probe.txt
for p in 0 1 2; do
  OME_VARLEN_PROBE=$p timeout -k 10 200 python -u scripts/varlen_attn_bench.py > gpurun_out/va_one.txt 2>&1 || exit $?
  grep -E "long 8k|qwen" gpurun_out/va_one.txt | sed "s/^/probe $p /" >> gpurun_out/va_probe.txt
done
