"""Tensor parallelism for the hybrid (recurrent + attention) families on CPU: 2 gloo ranks must
generate exactly what 1 rank generates from the same Hugging Face checkpoint.

* Qwen3-Next: Gated-DeltaNet layers split by key-head groups (q/k/v/z/b/a rows, conv channels,
  A_log / dt_bias, out_proj columns), gated attention by query heads, MoE by intermediate dim;
* NemotronH: Mamba-2 layers split by SSM heads / groups, attention by heads, MLP / MoE by
  intermediate dim."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

transformers = pytest.importorskip("transformers")

PROMPTS = [[3 + (i * 37 + j) % 500 for j in range(7 + 9 * i)] for i in range(3)]


def _worker(rank, world, port, path, q):
    import traceback

    torch.set_num_threads(2)   # two ranks inside an xdist worker share the container's cores
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    try:
        from ome_amd.runtime.engine import Engine, EngineArgs
        from ome_amd.runtime.request import SamplingParams

        eng = Engine(EngineArgs(model_path=path, tp_size=world, device="cpu", max_running_requests=8,
                                context_length=256, dtype="float32", chunked_prefill_size=16))
        if rank == 0:
            out = [r.output_ids for r in eng.generate(PROMPTS, SamplingParams(max_new_tokens=6, ignore_eos=True))]
            eng.stop_group()
            q.put(out)
        else:
            eng.run_forever()
    except Exception:  # noqa: BLE001 -- surface a rank's failure instead of a queue timeout
        q.put(("error", rank, traceback.format_exc()))


def _tp2(path):
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    single = Engine(EngineArgs(model_path=str(path), device="cpu", max_running_requests=8, context_length=256,
                               dtype="float32", chunked_prefill_size=16))
    want = [r.output_ids for r in single.generate(PROMPTS, SamplingParams(max_new_tokens=6, ignore_eos=True))]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, str(path), q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=400)
    assert not (isinstance(got, tuple) and got[0] == "error"), got
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got, want


@pytest.mark.timeout(500)
def test_qwen3_next_tp2_matches_tp1(tmp_path):
    if not hasattr(transformers, "Qwen3NextConfig"):
        pytest.skip("transformers without Qwen3-Next")
    from tests.test_qwen3_next_cpu import _hf_model

    _hf_model(tmp_path)
    got, want = _tp2(tmp_path)
    assert got == want


@pytest.mark.timeout(500)
@pytest.mark.parametrize("pattern,kw", [
    ("M-M*-M", {}),
    ("M*E-ME", dict(n_routed_experts=8, num_experts_per_tok=2, moe_intermediate_size=64,
                    moe_shared_expert_intermediate_size=96, n_group=1, topk_group=1)),
])
def test_nemotron_h_tp2_matches_tp1(tmp_path, pattern, kw):
    if not hasattr(transformers, "NemotronHConfig"):
        pytest.skip("transformers without NemotronH")
    from tests.test_nemotron_h_cpu import _hf_model

    _hf_model(tmp_path, pattern, **kw)
    got, want = _tp2(tmp_path)
    assert got == want
