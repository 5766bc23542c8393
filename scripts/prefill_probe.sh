#!/bin/bash
# Paged prefill timing probes (OME_PREFILL_PROBE: 0 normal, 1 no V image stores, 2 no K/V global
# loads, 3 identity pages); wrong results by design for 1-3.  One process each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/pf_probe.txt
for p in 0 1 2 3; do
  OME_PREFILL_PROBE=$p timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/pf_one.txt 2>&1 || exit $?
  grep -E "causal" gpurun_out/pf_one.txt | sed "s/^/probe $p /" >> gpurun_out/pf_probe.txt
done
