#!/bin/bash
# MoE / MLA model GPU tests, then the DeepSeek-V3 6-layer fp8 bench (one MI355X).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_moe_gpu.py \
  tests/test_moe_gpu.py tests/test_deepseek_gpu.py tests/test_minicpm3_gpu.py tests/test_kimi_vl_gpu.py \
  tests/test_new_families_gpu.py tests/test_bailing_gpu.py > gpurun_out/ds_test.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model deepseek-v3 --layers 6 --concurrency 128 --context-length 4096 \
  --steps 5 --warmup 2 --quantization fp8 --no-e2e-block > gpurun_out/dsv3_bench2.log 2>&1
