#!/bin/bash
# Ping-pong GEMM diagnostics: probe builds (scripts/gemm_pp_probe.py) + one PMC pass.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/pp
mkdir -p $OUT
export TMPDIR=/tmp
for p in 0 1 2; do
  OME_PP_PROBE=$p timeout -k 10 120 python3 $R/scripts/gemm_pp_probe.py || exit 1
done
CNT=${PMC_COUNTERS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"}
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc $CNT -d $OUT/pmc -o run --output-format csv -- python3 $R/scripts/gemm_pp_probe.py > $OUT/pmc.log 2>&1 || { echo "PMC FAILED"; tail -n 5 $OUT/pmc.log; exit 1; }
cd $R && python3 scripts/pmc_summary.py $OUT/pmc > $OUT/summary.txt && cat $OUT/summary.txt
