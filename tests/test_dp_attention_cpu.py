"""DP attention + expert parallelism on CPU (gloo): 2 ranks, each scheduling its own requests
with full attention / dense weights and half of the experts, MoE tokens exchanged by
all-to-all (``ome_amd.parallel.ep``), tokens relayed to rank 0 -- must generate what a single
rank generates from the same HF checkpoint (Qwen3-MoE and DeepSeek-V3 layouts)."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from ome_amd.io.safetensors import save_file
from ome_amd.models import build_model
from ome_amd.models.config import PRESETS, ModelConfig
from tests.test_deepseek_cpu import _hf_weights
from tests.test_moe_cpu import _export_hf

PROMPTS = [[3 + (i * 37 + j) % 1000 for j in range(5 + 7 * i)] for i in range(5)]


def _worker(rank, world, port, path, q, relay_cap=None, overlap=None, prompts=PROMPTS):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model_path=path, tp_size=world, dp_size=world, enable_dp_attention=True, device="cpu",
                            max_running_requests=8, context_length=256, dtype="float32", overlap_schedule=overlap))
    assert eng.dp_overlap == bool(overlap)
    if relay_cap is not None:   # force the two-phase relay fallback on every step
        eng._dp_cap = relay_cap
    m = eng.runner.model
    assert m.E_local == m.E // world and m.e0 == rank * m.E_local
    if rank == 0:
        reqs = eng.generate(prompts, SamplingParams(max_new_tokens=8, ignore_eos=True))
        owners = {r.dp_rank for r in reqs}
        eng.stop_group()
        q.put(([r.output_ids for r in reqs], owners))
    else:
        eng.run_forever()


def _checkpoint(tmp_path, kind):
    if kind == "gpt-oss":   # biased experts, sinks, sliding windows
        from tests.test_gpt_oss_cpu import _hf_model

        _hf_model(tmp_path)
        return
    if kind in ("olmoe", "dbrx", "minimax_m2"):   # spec-driven decoder MoE families
        from tests.test_decoder_families_cpu import _hf_model

        _hf_model(kind, tmp_path)
        return
    if kind == "qwen3-moe":
        hf = dict(PRESETS["tiny-moe"])
        m = build_model(ModelConfig.from_hf(hf), "cpu", torch.float32, load_format="dummy", seed=5)
        _export_hf(m, tmp_path, "qwen3")
    else:
        hf = dict(PRESETS["tiny-deepseek"])
        w = _hf_weights(ModelConfig.from_hf(hf), seed=2)
        save_file({k: v.contiguous() for k, v in w.items()}, tmp_path / "model.safetensors")
    (tmp_path / "config.json").write_text(json.dumps(hf))


@pytest.mark.timeout(400)
@pytest.mark.parametrize("kind,relay_cap,overlap", [
    ("qwen3-moe", None, None), ("deepseek-v3", None, None), ("qwen3-moe", 3, None), ("gpt-oss", None, None),
    ("olmoe", None, None), ("dbrx", None, None), ("minimax_m2", None, None),
    # overlapped DP steps (the GPU default): step k+1 enqueued before step k's tokens are read back
    ("qwen3-moe", None, True), ("deepseek-v3", None, True), ("qwen3-moe", 3, True)])
def test_dp_attention_ep_matches_single(tmp_path, kind, relay_cap, overlap, world=2, prompts=PROMPTS):
    _checkpoint(tmp_path, kind)
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    single = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", max_running_requests=8, context_length=256,
                               dtype="float32"))
    want = [r.output_ids for r in single.generate(prompts, SamplingParams(max_new_tokens=8, ignore_eos=True))]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), q, relay_cap, overlap, prompts))
          for r in range(world)]
    for p in ps:
        p.start()
    got, owners = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert owners == set(range(world))  # every rank served requests
    assert got == want


@pytest.mark.timeout(400)
def test_dp_relay_mixed_overflow_keeps_every_rank(tmp_path):
    """4 ranks (2 of the 8 experts each), 6 prompts -> ranks own {0, 4}, {1, 5}, {2}, {3}; relay
    capacity 12 floats: follower 1's two-request update overflows (13 floats) while followers 2
    and 3 fit theirs (7 floats).  The two-phase fallback must carry EVERY follower's update --
    the non-overflowing ranks already took theirs out of the pending list, so dropping them
    would leave their proxy requests hanging on rank 0."""
    prompts = [[3 + (i * 37 + j) % 1000 for j in range(5 + 3 * i)] for i in range(6)]
    test_dp_attention_ep_matches_single(tmp_path, "qwen3-moe", 12, None, world=4, prompts=prompts)


def test_dp_relay_unknown_finish_reason_is_an_abort():
    """The DP-attention token relay packs finish reasons as codes: a reason outside the table
    (e.g. a PD transfer failure) must reach the client as an abort, never as a normal stop."""
    from ome_amd.runtime import engine as E

    assert E._unknown_code("abort:something_new") == E._REASON_CODE["abort"]
    assert E._REASONS[E._REASON_CODE["abort:kv_layout_mismatch"]] == "abort:kv_layout_mismatch"
    packed = [1.0, 7.0, 1.0, 1.0, 99.0, 42.0, -0.5]   # one update: handle 7, 1 token, finished, code 99
    (h, toks, lps, fin, reason), = E._unpack_updates(packed)
    assert (h, toks, fin, reason) == (7, [42], True, "abort")
