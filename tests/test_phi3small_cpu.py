"""Phi-3-small (``models/phi3small.py``) on CPU against an independent fp32 restatement of the
published architecture (the remote modelling code is not importable offline: parity with it is
unpinned).  The tiny config makes the block-sparse pattern bite: 4-token blocks, a band of 2 local
blocks and every 3rd block as a per-head rotating vertical stripe, on every other layer; prompts
span 10+ blocks, so dense layers, band-only keys and stripe keys are all exercised -- in one
prefill, in chunked prefill and in decode."""
import json
import math

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.io.safetensors import save_file
from ome_amd.models.common import AttnMeta
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams

CFG = dict(architectures=["Phi3SmallForCausalLM"], model_type="phi3small", vocab_size=300, hidden_size=128,
           num_hidden_layers=4, num_attention_heads=4, num_key_value_heads=2, ff_intermediate_size=192,
           hidden_act="gegelu", gegelu_limit=20.0, layer_norm_epsilon=1e-5, rope_embedding_base=10000.0,
           max_position_embeddings=512, blocksparse_block_size=4, blocksparse_num_local_blocks=2,
           blocksparse_vert_stride=3, blocksparse_homo_head_pattern=False, dense_attention_every_n_layers=2,
           mup_attn_multiplier=1.5, mup_embedding_multiplier=4.0, mup_use_scaling=True, mup_width_multiplier=2.0,
           bos_token_id=1, eos_token_id=2, pad_token_id=0)


def _weights(seed=0):
    g = torch.Generator().manual_seed(seed)
    c = CFG
    H, nh, nkv, ff, L, V = (c["hidden_size"], c["num_attention_heads"], c["num_key_value_heads"],
                            c["ff_intermediate_size"], c["num_hidden_layers"], c["vocab_size"])
    hd = H // nh
    r = lambda *s, std=0.08: torch.randn(*s, generator=g) * std  # noqa: E731
    w = {"model.embed_tokens.weight": r(V, H, std=0.3), "lm_head.weight": r(V, H, std=0.2),
         "model.final_layernorm.weight": 1 + r(H, std=0.1), "model.final_layernorm.bias": r(H, std=0.05)}
    for i in range(L):
        p = f"model.layers.{i}."
        w.update({p + "input_layernorm.weight": 1 + r(H, std=0.1), p + "input_layernorm.bias": r(H, std=0.05),
                  p + "post_attention_layernorm.weight": 1 + r(H, std=0.1),
                  p + "post_attention_layernorm.bias": r(H, std=0.05),
                  p + "self_attn.query_key_value.weight": r((nh + 2 * nkv) * hd, H),
                  p + "self_attn.query_key_value.bias": r((nh + 2 * nkv) * hd, std=0.05),
                  p + "self_attn.dense.weight": r(H, nh * hd), p + "self_attn.dense.bias": r(H, std=0.05),
                  p + "mlp.up_proj.weight": r(2 * ff, H), p + "mlp.up_proj.bias": r(2 * ff, std=0.05),
                  p + "mlp.down_proj.weight": r(H, ff), p + "mlp.down_proj.bias": r(H, std=0.05)})
    return w


def _ref_logits(w, ids):
    """fp32 restatement: LayerNorm pre-norm blocks, kv-grouped biased QKV, NeoX RoPE, muP scales,
    block-sparse causal attention on layers (i + 1) % 2 != 0, interleaved GeGELU."""
    c = CFG
    H, nh, nkv, L = c["hidden_size"], c["num_attention_heads"], c["num_key_value_heads"], c["num_hidden_layers"]
    hd, g = H // nh, nh // nkv
    T = len(ids)
    B, loc, vert = c["blocksparse_block_size"], c["blocksparse_num_local_blocks"], c["blocksparse_vert_stride"]
    step = max(1, vert // nh)
    eps = c["layer_norm_epsilon"]
    x = w["model.embed_tokens.weight"][torch.tensor(ids)] * c["mup_embedding_multiplier"]
    pos = torch.arange(T, dtype=torch.float32)
    inv = 1.0 / (c["rope_embedding_base"] ** (torch.arange(0, hd, 2, dtype=torch.float32) / hd))
    ang = pos[:, None] * inv[None]
    cos, sin = torch.cat([ang.cos()] * 2, -1), torch.cat([ang.sin()] * 2, -1)

    def rope(t):  # [T, n, hd]
        t1, t2 = t[..., :hd // 2], t[..., hd // 2:]
        return t * cos[:, None] + torch.cat([-t2, t1], -1) * sin[:, None]

    qi, ki = torch.arange(T)[:, None], torch.arange(T)[None]
    causal = ki <= qi
    for i in range(L):
        p = f"model.layers.{i}."
        h = F.layer_norm(x, (H,), w[p + "input_layernorm.weight"], w[p + "input_layernorm.bias"], eps)
        qkv = (h @ w[p + "self_attn.query_key_value.weight"].T + w[p + "self_attn.query_key_value.bias"])
        qkv = qkv.view(T, nkv, g + 2, hd)
        q, k, v = qkv[:, :, :g].reshape(T, nh, hd), qkv[:, :, g], qkv[:, :, g + 1]
        q, k = rope(q), rope(k)
        o = torch.empty(T, nh, hd)
        for hh in range(nh):
            s = (q[:, hh] @ k[:, hh // g].T) * (c["mup_attn_multiplier"] / hd)
            m = causal
            if (i + 1) % c["dense_attention_every_n_layers"] != 0:
                qb, kb = qi // B, ki // B
                m = m & (((qb - kb) < loc) | (((kb + hh * step + 1) % vert) == 0))
            s = s.masked_fill(~m, float("-inf"))
            o[:, hh] = torch.softmax(s, -1) @ v[:, hh // g]
        x = x + o.reshape(T, H) @ w[p + "self_attn.dense.weight"].T + w[p + "self_attn.dense.bias"]
        h = F.layer_norm(x, (H,), w[p + "post_attention_layernorm.weight"], w[p + "post_attention_layernorm.bias"], eps)
        up = h @ w[p + "mlp.up_proj.weight"].T + w[p + "mlp.up_proj.bias"]
        a_g, a_l = up[..., ::2].clamp(max=20.0), up[..., 1::2].clamp(-20.0, 20.0)
        x = x + (a_g * torch.sigmoid(1.702 * a_g) * (a_l + 1)) @ w[p + "mlp.down_proj.weight"].T + \
            w[p + "mlp.down_proj.bias"]
    x = F.layer_norm(x, (H,), w["model.final_layernorm.weight"], w["model.final_layernorm.bias"], eps)
    return (x @ w["lm_head.weight"].T) / c["mup_width_multiplier"]


def _checkpoint(tmp_path):
    w = _weights()
    save_file({k: v.contiguous() for k, v in w.items()}, tmp_path / "model.safetensors")
    (tmp_path / "config.json").write_text(json.dumps(CFG))
    return w


def _prefill_logits(eng, ids, chunks):
    run = eng.runner
    slot = run.slots.alloc()
    pages = run.pages.alloc(-(-len(ids) // run.P))
    run.slots.set_pages(slot, 0, pages)
    run.slots.flush()
    t = lambda a: torch.tensor(a, dtype=torch.int32, device=run.device)  # noqa: E731
    outs, s = [], 0
    for n in chunks:
        rng = list(range(s, s + n))
        meta = AttnMeta("prefill", t(rng), t([pages[x // run.P] * run.P + x % run.P for x in rng]),
                        run.slots.table.index_select(0, t([slot])), cu_q=t([0, n]), kv_lens=t([s + n]),
                        items=t(ops.prefill_work_items([n], [s + n])).view(-1, 2))
        outs.append(run.model.compute_logits(run.model.forward(t(ids[s:s + n]), meta, run.kv)).float())
        s += n
    run.pages.free(pages)
    run.slots.free(slot)
    return torch.cat(outs, 0)


IDS = [(11 * i + 5) % 290 + 3 for i in range(45)]


def test_phi3small_logits_match_restatement(tmp_path):
    w = _checkpoint(tmp_path)
    want = _ref_logits(w, IDS)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "Phi3SmallForCausalLM"
    assert m.sparse_layer == [True, False, True, False] and m.bs == (4, 2, 3, 1, 0)
    tol = 2e-3 * max(1.0, want.abs().max().item())
    assert (_prefill_logits(eng, IDS, [45]) - want).abs().max().item() < tol
    assert (_prefill_logits(eng, IDS, [17, 28]) - want).abs().max().item() < tol   # chunked: prefix + sparse


def test_phi3small_generate_matches_restatement(tmp_path):
    w = _checkpoint(tmp_path)
    ids, toks = list(IDS), []
    for _ in range(6):   # greedy decode of the restatement (the engine decodes against its paged cache)
        nxt = int(_ref_logits(w, ids + toks)[-1].argmax())
        toks.append(nxt)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=256))
    assert eng.generate([ids], SamplingParams(max_new_tokens=6, ignore_eos=True))[0].output_ids == toks


def test_blocksparse_pack_roundtrip():
    v = ops.blocksparse_pack((64, 16, 8, 1, 96))
    assert v & 15 == 6 and (v >> 4) & 0xffff == 16 and (v >> 20) & 0xfff == 8 and (v >> 32) & 0xff == 1
    assert (v >> 40) & 0xfff == 96 and ops.blocksparse_pack(None) == 0
    assert math.isclose(1.0, 1.0)
