#!/bin/bash
# Other model families / precisions through the same BenchmarkJob-style bench (exploration, not
# the headline): DeepSeek-V2-Lite (MLA + MoE, random init), Llama-3-8B FP8 W8A8; plus a
# rocprofv3 kernel summary of the DeepSeek run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m ome_amd.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --model deepseek-v2-lite --steps 100 --warmup 60 --concurrency 128 \
    > gpurun_out/b_dsv2lite.log 2>&1 || { tail -20 gpurun_out/b_dsv2lite.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b_dsv2lite.log | tail -2 | cut -c1-400
timeout -k 10 400 python bench.py --quantization fp8 --steps 200 --warmup 100 > gpurun_out/b_fp8.log 2>&1 \
    || { tail -20 gpurun_out/b_fp8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b_fp8.log | tail -2 | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ds" -o ds -- \
    python "$GRAFT_REPO_ROOT/bench.py" --model deepseek-v2-lite --steps 40 --warmup 40 --concurrency 128 \
    > "$GRAFT_REPO_ROOT/gpurun_out/prof_ds.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_ds.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/prof_ds -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/ds_kernel_stats.csv && head -25 gpurun_out/ds_kernel_stats.csv | cut -c1-200
find gpurun_out/prof_ds -name "*kernel_trace.csv" -delete
exit 0
