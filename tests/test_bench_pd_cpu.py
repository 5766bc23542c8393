"""bench.py --pd plumbing on CPU: a prefill server, a decode server and the PD router as separate
processes (tiny random Llama), the streaming client counting tokens that went router -> prefill
-> KV hand-off (TCP blob path on CPU) -> decode."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_pd_bench_end_to_end_cpu(tmp_path):
    from ome_amd.bench import pd

    r = pd.run("tiny-llama", "D(24,10)", concurrency=3, context_length=256, steps=2, warmup=1, step_s=3.0,
               n_prefill=1, n_decode=1, max_total_tokens=4096, decode_total_tokens=4096, log_dir=str(tmp_path),
               extra=["--device", "cpu", "--disable-cuda-graph"])
    assert r["errors"] == 0 and r["tokens"] > 0, (r, open(tmp_path / "decode0.log").read()[-3000:])
    assert r["p50_ttft_ms"] is not None
