#!/bin/bash
# Same-box A/B of one environment switch: "$1" = the switch (e.g. OME_PREFILL_ROWS=64), run
# against the default on the prefill probe and the headline bench, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SW=${1:?env switch}
mkdir -p gpurun_out
out=gpurun_out/ab_env.txt
: > $out
for e in "" "$SW" "" "$SW"; do
  echo "== ${e:-default}: prefill probe" >> $out
  env $e timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/ab_x.txt 2>&1 || exit $?
  grep -E "causal" gpurun_out/ab_x.txt >> $out
done
for e in "" "$SW" "" "$SW"; do
  echo "== ${e:-default}: bench" >> $out
  env $e timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ab_bench.txt 2>&1 || exit $?
  grep -E '^\{' gpurun_out/ab_bench.txt | cut -c1-330 >> $out
done
cat $out
