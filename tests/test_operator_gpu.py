"""The operator -> GPU -> BenchmarkJob slice on a real MI355X: ClusterBaseModel
``random://llama-3-8b`` + ClusterServingRuntime requesting ``amd.com/gpu: 1`` + InferenceService
reconcile to Ready; the node executor starts ``ome_amd.runtime.server`` on GPU 0 (HIP graphs,
native kernels); a BenchmarkJob (D(100,100), concurrency 1 / 4 / 16, short limits) completes and
writes results (reference: pkg/controller/v1beta1/benchmark/controller.go:499-557)."""
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_isvc_on_gpu_serves_a_benchmarkjob(tmp_path):
    from ome_amd.bench import operator_slice

    assert torch.cuda.device_count() >= 1
    res = operator_slice.run(tmp_path, preset="llama-3-8b", scenarios=("D(100,100)",), concurrency=(1, 4, 16),
                             max_time=4, max_requests=16,
                             log=lambda m: print(m, file=sys.stderr, flush=True))
    assert res["gpu_ids"] == "0"
    summary = res["summary"]
    assert [s["concurrency"] for s in summary] == [1, 4, 16]
    for s in summary:
        assert s["num_completed"] >= 1 and s["output_tokens"]["mean"] == 100
        assert s["output_throughput_tokens_per_s"] > 0 and s["ttft_s"]["p50"] > 0
    # more concurrency, more throughput: the engine batches the requests on the GPU
    assert summary[2]["output_throughput_tokens_per_s"] > 2 * summary[0]["output_throughput_tokens_per_s"]
