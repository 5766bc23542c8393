#!/bin/bash
# Single-GPU serving throughput of the larger model families (bf16, random-init weights,
# BenchmarkJob scenario N(480,240)/(300,150)): one MI355X holds Llama-3-70B (141 GB) and
# Llama-4-Scout (218 GB) whole.  Each run is time-limited; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
run() {
  local name=$1; shift
  echo "== $name $*"
  timeout -k 10 ${T:-420} python -u bench.py "$@" > gpurun_out/bench_$name.log 2>&1
  local rc=$?
  tail -2 gpurun_out/bench_$name.log
  return $rc
}
run 70b --model llama-3-70b --steps 100 --warmup 100 --concurrency 128 &&
run dsv2lite --model deepseek-v2-lite --steps 200 --warmup 150 &&
run mixtral --model mixtral-8x7b --steps 200 --warmup 150 &&
T=600 run scout --model llama-4-scout-17b-16e --steps 100 --warmup 100 --concurrency 128
