#!/bin/bash
# Round-4 GPU measurements: (1) Llama-3-70B TP=2 rehearsal with 2 ranks sharing GPU 0 (custom
# all-reduce over IPC, 32 MiB two-shot messages at the 2048-token prefill budget); (2) DeepSeek-V3
# shaped fp8 serving, 6 of 61 layers, with a kernel summary (MLA glue fused into mla_prep).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "${RUN_TP2:-1}" = 1 ]; then
  OME_BENCH_SHARE_GPU=1 OME_TUNE_GEMM=0 timeout -k 10 700 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --tp 2 \
    --model llama-3-70b --steps 3 --warmup 1 --no-e2e-block > gpurun_out/r04/tp2_70b.log 2>&1 || exit $?
fi
if [ "${RUN_DS:-1}" = 1 ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r04_dsv3 -o run --output-format csv -- \
    python3 $R/bench.py --model deepseek-v3 --layers 6 --concurrency 128 --context-length 4096 --steps 5 --warmup 2 \
    --quantization fp8 --no-e2e-block > $R/gpurun_out/r04_dsv3_bench.log 2>&1
  rc=$?
  cd $R
  [ $rc -eq 0 ] || exit $rc
  python scripts/prof_summary.py gpurun_out/r04_dsv3 40 > gpurun_out/r04_dsv3/summary.md
  find gpurun_out/r04_dsv3 -name "*kernel_trace.csv" -delete
fi
exit 0
