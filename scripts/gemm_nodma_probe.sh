#!/bin/bash
# Timing probe: the stream-K kernel with and without its in-loop DMA (SK_FLAGS=1: results wrong,
# timing only) -- separates the staging wait from the loop's own MFMA / LDS / barrier cost.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/nodma
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for cfg in gate_up:2048:256:224 gate_up:2048:256:256 gate_up:256:128:224 qkv:256:128:192; do
  IFS=: read -r shape m bn nwg <<< "$cfg"
  for fl in 0 1; do
    tag=${shape}_${m}_${bn}_${nwg}_f$fl
    SK_FLAGS=$fl timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o run --output-format csv -- python3 $R/scripts/gemm_sk_one.py $shape $m $bn $nwg 40 > $OUT/$tag.log 2>&1 || { echo FAILED $tag; exit 1; }
    python3 - "$OUT/$tag" "$tag" <<'PY'
import csv, glob, sys
for p in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "gemm_sk" in r["Name"]:
            print(f'{sys.argv[2]:32s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"]) / 1000:8.1f} us')
PY
  done
done
