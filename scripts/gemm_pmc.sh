#!/bin/bash
# PMC counter passes (one rocprofv3 run per configuration, <= 8 SQ + 2 GRBM counters) over
# scripts/gemm_sk_one.py; summarised by scripts/pmc_summary.py into gpurun_out/pmc/summary.txt.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
CNT=${PMC_COUNTERS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"}
cd /tmp
CONFIGS=${PMC_CONFIGS:-gate_up:256:128:224 gate_up:2048:256:224 gate_up:2048:0:0 qkv:256:128:192}
for cfg in $CONFIGS; do
  IFS=: read -r shape m bn nwg <<< "$cfg"
  tag=${shape}_${m}_${bn}_${nwg}
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d $OUT/$tag -o run --output-format csv -- python3 $R/scripts/gemm_sk_one.py $shape $m $bn $nwg 30 > $OUT/$tag.log 2>&1 || { echo "FAILED $tag"; tail -n 5 $OUT/$tag.log; exit 1; }
done
cd $R && python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
