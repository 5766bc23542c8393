set -o pipefail
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gemm_xl_gpu.py tests/test_glm4v_gpu.py tests/test_deepseek_gpu.py tests/test_encoder_gpu.py tests/test_kernels_gpu.py tests/test_load_exchange_gpu.py -k "xl or glm or mla or deepseek or varlen or encoder or blocksparse or prefill or exchange" -s > gpurun_out/t6a.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t6a.log; exit 1; }
timeout -k 10 120 python3 scripts/mla_bench.py > gpurun_out/mla_a.log 2>&1 && OME_MLA_ALL_MIN_T=0 timeout -k 10 120 python3 scripts/mla_bench.py > gpurun_out/mla_b.log 2>&1 || exit 1
timeout -k 10 60 python3 scripts/blocksparse_bench.py > gpurun_out/bsb.log 2>&1 && timeout -k 10 60 python3 scripts/blocksparse_bench.py --dense >> gpurun_out/bsb.log 2>&1 && OME_BS_SKIP=0 OME_PREFILL_FAST=0 timeout -k 10 60 python3 scripts/blocksparse_bench.py >> gpurun_out/bsb.log 2>&1 && OME_BS_SKIP=0 timeout -k 10 60 python3 scripts/blocksparse_bench.py >> gpurun_out/bsb.log 2>&1 || exit 1
tail -4 gpurun_out/t6a.log; cat gpurun_out/bsb.log gpurun_out/mla_a.log gpurun_out/mla_b.log | grep -v amdgpu.ids
OME_AR_ORDER_PROBE=1 timeout -k 10 200 python3 scripts/comm_latency_bench.py 2 > gpurun_out/comm6.log 2>&1 || { tail -20 gpurun_out/comm6.log; exit 1; }
grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/comm6.log
timeout -k 10 300 python3 scripts/loader_bench.py --layers 2 --tp 8 --concurrent > gpurun_out/loader6.log 2>&1 || { tail -20 gpurun_out/loader6.log; exit 1; }
grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/loader6.log
