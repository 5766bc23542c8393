"""bench.py --e2e plumbing on CPU: a real server child (tiny random Llama), the closed-loop
streaming client counting tokens from the per-chunk usage, TTFT, and a clean shutdown."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_e2e_client_counts_streamed_tokens():
    from ome_amd.bench import e2e

    r = e2e.run("tiny-llama", "D(20,12)", concurrency=4, context_length=256, steps=2, warmup=1, step_s=2.0,
                vocab=1024, server_args=["--device", "cpu", "--disable-cuda-graph"])
    assert r["tokens"] > 0 and r["value"] > 0
    assert r["p50_ttft_ms"] is not None and r["p50_ttft_ms"] > 0
