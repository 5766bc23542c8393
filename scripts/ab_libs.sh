#!/bin/bash
# Same-box A/B of two builds of ome_kernels (default ome_amd/_lib vs $1, e.g. ome_amd/_lib_noslp
# from scripts/build_variant.py): prefill attention probe, then the headline bench, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VAR=${1:?variant lib dir}
mkdir -p gpurun_out
out=gpurun_out/ab_libs.txt
: > $out
for lib in "" "$VAR"; do
  echo "== lib ${lib:-default}: prefill probe" >> $out
  OME_LIB_DIR=$lib timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/ab_pf.txt 2>&1 || exit $?
  grep -E "causal" gpurun_out/ab_pf.txt >> $out
done
for lib in "" "$VAR" "" "$VAR"; do
  echo "== lib ${lib:-default}: bench" >> $out
  OME_LIB_DIR=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ab_bench.txt 2>&1 || exit $?
  grep -E '^\{' gpurun_out/ab_bench.txt | cut -c1-400 >> $out
done
cat $out
