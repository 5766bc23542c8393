"""DeciLM / Llama-Nemotron NAS (``models/decilm.py``) against an fp32 transcription of the block
semantics (per-layer GQA group, no-op / linear-replaced attention and FFN, per-layer FFN width,
Llama-3 RoPE) on a tiny random checkpoint written with the reference's weight names; logits and
greedy decode through the engine, including per-layer KV-head pages and layers without KV.
(The remote modeling code is not importable offline: parity with it is unpinned.)"""
import json

import pytest
import torch
from safetensors.torch import save_file

from ome_amd.models.decilm import ffn_mult_to_intermediate
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams

H, NH, D, V, L = 256, 4, 64, 300, 5   # head dim 64: also served on the gfx950 kernels
BLOCKS = [
    {"attention": {"n_heads_in_group": 2, "no_op": False, "replace_with_linear": False},
     "ffn": {"ffn_mult": 1.5, "no_op": False, "replace_with_linear": False}},
    {"attention": {"n_heads_in_group": None, "no_op": True, "replace_with_linear": False},
     "ffn": {"ffn_mult": 2.0, "no_op": False, "replace_with_linear": False}},
    {"attention": {"n_heads_in_group": 4, "no_op": False, "replace_with_linear": False},
     "ffn": {"ffn_mult": None, "no_op": True, "replace_with_linear": False}},
    {"attention": {"n_heads_in_group": None, "no_op": False, "replace_with_linear": True},
     "ffn": {"ffn_mult": None, "no_op": False, "replace_with_linear": True}},
    {"attention": {"n_heads_in_group": 1, "no_op": False, "replace_with_linear": False},
     "ffn": {"ffn_mult": 1.0, "no_op": False, "replace_with_linear": False}},
]


def _weights():
    g = torch.Generator().manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g) * 0.08  # noqa: E731
    w = {"model.embed_tokens.weight": r(V, H), "model.norm.weight": 1 + r(H), "lm_head.weight": r(V, H)}
    for i, b in enumerate(BLOCKS):
        p = f"model.layers.{i}."
        a, f = b["attention"], b["ffn"]
        if not a["no_op"]:
            w[p + "input_layernorm.weight"] = 1 + r(H)
            if a["replace_with_linear"]:
                w[p + "self_attn.linear_attn.weight"] = r(H, H)
            else:
                kv = NH // a["n_heads_in_group"]
                w.update({p + "self_attn.q_proj.weight": r(NH * D, H), p + "self_attn.k_proj.weight": r(kv * D, H),
                          p + "self_attn.v_proj.weight": r(kv * D, H), p + "self_attn.o_proj.weight": r(H, NH * D)})
        if not f["no_op"]:
            w[p + "post_attention_layernorm.weight"] = 1 + r(H)
            if f["replace_with_linear"]:
                w[p + "mlp.linear_mlp.weight"] = r(H, H)
            else:
                inter = ffn_mult_to_intermediate(f["ffn_mult"], H)
                w.update({p + "mlp.gate_proj.weight": r(inter, H), p + "mlp.up_proj.weight": r(inter, H),
                          p + "mlp.down_proj.weight": r(H, inter)})
    return w


def _ref_logits(w, ids, theta=10000.0):
    T = len(ids)
    rms = lambda x, g: x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * g  # noqa: E731
    inv = 1.0 / theta ** (torch.arange(0, D, 2).float() / D)
    ang = torch.arange(T).float()[:, None] * inv[None]
    cos, sin = torch.cat([ang.cos()] * 2, -1), torch.cat([ang.sin()] * 2, -1)
    rot = lambda x: x * cos[:, None] + torch.cat([-x[..., D // 2:], x[..., :D // 2]], -1) * sin[:, None]  # noqa
    h = w["model.embed_tokens.weight"][torch.tensor(ids)]
    for i, b in enumerate(BLOCKS):
        p = f"model.layers.{i}."
        a, f = b["attention"], b["ffn"]
        if not a["no_op"]:
            x = rms(h, w[p + "input_layernorm.weight"])
            if a["replace_with_linear"]:
                h = h + x @ w[p + "self_attn.linear_attn.weight"].T
            else:
                G = a["n_heads_in_group"]
                q = rot((x @ w[p + "self_attn.q_proj.weight"].T).view(T, NH, D))
                k = rot((x @ w[p + "self_attn.k_proj.weight"].T).view(T, NH // G, D)).repeat_interleave(G, 1)
                v = (x @ w[p + "self_attn.v_proj.weight"].T).view(T, NH // G, D).repeat_interleave(G, 1)
                s = torch.einsum("qhd,khd->hqk", q, k) / D ** 0.5
                s = s.masked_fill(torch.ones(T, T, dtype=torch.bool).triu(1), float("-inf"))
                o = torch.einsum("hqk,khd->qhd", s.softmax(-1), v).reshape(T, NH * D)
                h = h + o @ w[p + "self_attn.o_proj.weight"].T
        if not f["no_op"]:
            x = rms(h, w[p + "post_attention_layernorm.weight"])
            if f["replace_with_linear"]:
                h = h + x @ w[p + "mlp.linear_mlp.weight"].T
            else:
                gt, up = x @ w[p + "mlp.gate_proj.weight"].T, x @ w[p + "mlp.up_proj.weight"].T
                h = h + (torch.nn.functional.silu(gt) * up) @ w[p + "mlp.down_proj.weight"].T
    return rms(h, w["model.norm.weight"]) @ w["lm_head.weight"].T


def _checkpoint(tmp_path):
    w = _weights()
    save_file({k: v.contiguous() for k, v in w.items()}, str(tmp_path / "model.safetensors"))
    cfg = {"architectures": ["DeciLMForCausalLM"], "model_type": "nemotron-nas", "hidden_size": H,
           "num_attention_heads": NH, "num_hidden_layers": L, "vocab_size": V, "rms_norm_eps": 1e-5,
           "rope_theta": 10000.0, "max_position_embeddings": 512, "tie_word_embeddings": False,
           "hidden_act": "silu", "block_configs": BLOCKS}
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    return w


def test_decilm_matches_block_semantics(tmp_path):
    w = _checkpoint(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "DeciLMForCausalLM"
    assert m.kv_layers == [0, 2, 4] and eng.runner.kv.k[1] is None and eng.runner.kv.k[3] is None
    assert [eng.runner.kv.k[i].shape[1] for i in (0, 2, 4)] == [2, 1, 4]   # per-layer KV heads
    ids = [(7 * i + 3) % 290 + 5 for i in range(30)]
    from tests.test_engine_gpu import _hidden_prefill

    got = m.compute_logits(_hidden_prefill(eng, ids)).float()
    want = _ref_logits(w, ids)
    assert torch.allclose(got, want, atol=2e-3, rtol=2e-3), (got - want).abs().max()
    # greedy decode through the engine == argmax continuation of the reference
    out = eng.generate([ids], SamplingParams(max_new_tokens=6, ignore_eos=True))[0].output_ids
    seq = list(ids)
    for _ in range(6):
        seq.append(int(_ref_logits(w, seq)[-1].argmax()))
    assert out == seq[len(ids):]


def _pp_worker(rank, world, port, path, q):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    eng = Engine(EngineArgs(model_path=path, pp_size=world, device="cpu", max_running_requests=4,
                            context_length=256, dtype="float32"))
    if rank == 0:
        out = [r.output_ids for r in eng.generate(PP_PROMPTS, SamplingParams(max_new_tokens=6, ignore_eos=True))]
        eng.stop_group()
        q.put(out)
    else:
        eng.run_forever()


PP_PROMPTS = [[(7 * i + 3 * j) % 290 + 5 for j in range(6 + 5 * i)] for i in range(3)]


@pytest.mark.timeout(300)
def test_decilm_pp2_matches_single(tmp_path):
    """PP=2 over the heterogeneous block stack: stage 0 ends on an attention-only block (no-op
    FFN), so the hand-off carries a pending block output; per-stage per-layer KV heads."""
    import socket

    import torch.multiprocessing as mp

    _checkpoint(tmp_path)
    single = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                               context_length=256))
    want = [r.output_ids for r in single.generate(PP_PROMPTS, SamplingParams(max_new_tokens=6, ignore_eos=True))]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_pp_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want
