#!/bin/bash
# Same-box A/B of the attention kernels in two builds of ome_kernels: $1 = baseline lib dir
# (scripts/build_variant.py), default ome_amd/_lib = candidate.  Correctness first (GPU tests of
# every attention kernel against fp32 references, candidate build), then prefill / decode / MLA /
# varlen microbenchmarks and the headline bench, alternating builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BASE=${1:?baseline lib dir}
EXTRA=${2:-}   # optional third build (e.g. ome_amd/_lib_prio)
mkdir -p gpurun_out
out=gpurun_out/ab_attn.txt
: > $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_encoder_gpu.py -m gpu > gpurun_out/ab_tests.txt 2>&1 || { tail -30 gpurun_out/ab_tests.txt; exit 1; }
tail -2 gpurun_out/ab_tests.txt >> $out
for lib in "$BASE" "" $EXTRA "$BASE" "" $EXTRA; do
  tag=${lib:-candidate}
  echo "== $tag: prefill probe" >> $out
  OME_LIB_DIR=$lib timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/ab_x.txt 2>&1 || exit $?
  grep -E "causal" gpurun_out/ab_x.txt >> $out
  echo "== $tag: decode attention" >> $out
  OME_LIB_DIR=$lib timeout -k 10 200 python -u scripts/attn_bench.py > gpurun_out/ab_x.txt 2>&1 || exit $?
  tail -12 gpurun_out/ab_x.txt >> $out
  echo "== $tag: mla" >> $out
  OME_LIB_DIR=$lib timeout -k 10 200 python -u scripts/mla_bench.py > gpurun_out/ab_x.txt 2>&1 || exit $?
  tail -8 gpurun_out/ab_x.txt >> $out
  echo "== $tag: varlen" >> $out
  OME_LIB_DIR=$lib timeout -k 10 200 python -u scripts/varlen_attn_bench.py > gpurun_out/ab_x.txt 2>&1 || exit $?
  tail -8 gpurun_out/ab_x.txt >> $out
done
for lib in "$BASE" "" $EXTRA "$BASE" "" $EXTRA; do
  echo "== ${lib:-candidate}: bench" >> $out
  OME_LIB_DIR=$lib timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ab_bench.txt 2>&1 || exit $?
  grep -E '^\{' gpurun_out/ab_bench.txt | cut -c1-330 >> $out
done
cat $out
