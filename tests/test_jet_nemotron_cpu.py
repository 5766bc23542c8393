"""Jet-Nemotron (``models/jet_nemotron.py``) on CPU against an independent fp32 restatement of the
published architecture (JetBlock: silu q / k, dynamic causal conv on v with per-token generated
taps, gated delta rule with L2-normalised q / k, gated RMSNorm output; kept full-attention and
sliding-window layers).  The remote modelling code is not importable offline: parity with it is
unpinned.  Greedy generation through the engine (prefill + recurrent decode, one prefill chunk
and several) must match the restatement token for token."""
import json
import math

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.io.safetensors import save_file
from ome_amd.models.jet_nemotron import jet_layer_types
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams

JET = dict(num_heads=2, head_dim=64, expand_v=1.5, conv_size=4, dconv_generator_reduction=4, norm_eps=1e-5)
CFG = dict(architectures=["JetNemotronForCausalLM"], model_type="jet_nemotron", vocab_size=256, hidden_size=128,
           intermediate_size=96, num_hidden_layers=4, num_attention_heads=2, num_key_value_heads=1,
           rms_norm_eps=1e-6, rope_theta=10000.0, max_position_embeddings=512, tie_word_embeddings=False,
           layer_types=["jet", "attn", "jet", "swa"],
           efficient_attention_config={"jet": JET, "swa": {"window_size": 8}}, bos_token_id=1, eos_token_id=2)


def _weights(seed=0):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s, std=0.1: torch.randn(*s, generator=g) * std  # noqa: E731
    H, V, I = CFG["hidden_size"], CFG["vocab_size"], CFG["intermediate_size"]
    nh, nkv = CFG["num_attention_heads"], CFG["num_key_value_heads"]
    hd = H // nh
    Hn, dk = JET["num_heads"], JET["head_dim"]
    dv = int(dk * JET["expand_v"])
    K, R = JET["conv_size"], H // JET["dconv_generator_reduction"]
    w = {"model.embed_tokens.weight": r(V, H, std=0.5), "lm_head.weight": r(V, H, std=0.3),
         "model.norm.weight": 1 + r(H)}
    for i, t in enumerate(CFG["layer_types"]):
        p = f"model.layers.{i}."
        w.update({p + "input_layernorm.weight": 1 + r(H), p + "post_attention_layernorm.weight": 1 + r(H),
                  p + "mlp.gate_proj.weight": r(I, H), p + "mlp.up_proj.weight": r(I, H),
                  p + "mlp.down_proj.weight": r(H, I)})
        a = p + "self_attn."
        if t == "jet":
            w.update({a + "q_proj.weight": r(Hn * dk, H), a + "k_proj.weight": r(Hn * dk, H),
                      a + "v_proj.weight": r(Hn * dv, H), a + "g_proj.weight": r(Hn * dv, H),
                      a + "a_proj.weight": r(Hn, H), a + "b_proj.weight": r(Hn, H),
                      a + "o_proj.weight": r(H, Hn * dv), a + "A_log": torch.log(torch.tensor([2.0, 6.0])),
                      a + "dt_bias": torch.tensor([0.5, -0.3]), a + "o_norm.weight": 1 + r(dv),
                      a + "dynamic_conv1d.kernel_generator.0.weight": r(R, H, std=0.3),
                      a + "dynamic_conv1d.kernel_generator.2.weight": r(Hn * dv * K, R, std=0.3),
                      a + "dynamic_conv1d.kernel_generator.2.bias": r(Hn * dv * K, std=0.3)})
        else:
            w.update({a + "q_proj.weight": r(nh * hd, H), a + "q_proj.bias": r(nh * hd),
                      a + "k_proj.weight": r(nkv * hd, H), a + "k_proj.bias": r(nkv * hd),
                      a + "v_proj.weight": r(nkv * hd, H), a + "v_proj.bias": r(nkv * hd),
                      a + "o_proj.weight": r(H, nh * hd)})
    return w


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def _ref_logits(w, ids):
    H, nh, nkv = CFG["hidden_size"], CFG["num_attention_heads"], CFG["num_key_value_heads"]
    hd, eps = H // nh, CFG["rms_norm_eps"]
    Hn, dk = JET["num_heads"], JET["head_dim"]
    dv, K = int(dk * JET["expand_v"]), JET["conv_size"]
    T = len(ids)
    x = w["model.embed_tokens.weight"][torch.tensor(ids)]
    pos = torch.arange(T, dtype=torch.float32)
    inv = 1.0 / (CFG["rope_theta"] ** (torch.arange(0, hd, 2, dtype=torch.float32) / hd))
    ang = pos[:, None] * inv[None]
    cos, sin = torch.cat([ang.cos()] * 2, -1), torch.cat([ang.sin()] * 2, -1)

    def rope(t):
        t1, t2 = t[..., :hd // 2], t[..., hd // 2:]
        return t * cos[:, None] + torch.cat([-t2, t1], -1) * sin[:, None]

    qi, ki = torch.arange(T)[:, None], torch.arange(T)[None]
    for i, kind in enumerate(CFG["layer_types"]):
        p = f"model.layers.{i}."
        a = p + "self_attn."
        h = _rms(x, w[p + "input_layernorm.weight"], eps)
        if kind == "jet":
            q = F.silu(h @ w[a + "q_proj.weight"].T).view(T, Hn, dk)
            k = F.silu(h @ w[a + "k_proj.weight"].T).view(T, Hn, dk)
            v0 = h @ w[a + "v_proj.weight"].T
            gate = (h @ w[a + "g_proj.weight"].T).view(T, Hn, dv)
            taps = (F.silu(h @ w[a + "dynamic_conv1d.kernel_generator.0.weight"].T)
                    @ w[a + "dynamic_conv1d.kernel_generator.2.weight"].T
                    + w[a + "dynamic_conv1d.kernel_generator.2.bias"]).view(T, Hn * dv, K)
            vp = torch.cat([torch.zeros(K - 1, Hn * dv), v0], 0)
            v = torch.stack([F.silu((taps[t] * vp[t:t + K].T).sum(-1)) for t in range(T)]).view(T, Hn, dv)
            q = q / q.norm(dim=-1, keepdim=True).clamp_min(1e-12) / math.sqrt(dk)
            k = k / k.norm(dim=-1, keepdim=True).clamp_min(1e-12)
            decay = torch.exp(-torch.exp(w[a + "A_log"]) * F.softplus(h @ w[a + "a_proj.weight"].T + w[a + "dt_bias"]))
            beta = torch.sigmoid(h @ w[a + "b_proj.weight"].T)
            S = torch.zeros(Hn, dk, dv)
            o = torch.empty(T, Hn, dv)
            for t in range(T):
                S = S * decay[t][:, None, None]
                delta = (v[t] - torch.einsum("hk,hkv->hv", k[t], S)) * beta[t][:, None]
                S = S + k[t][:, :, None] * delta[:, None, :]
                o[t] = torch.einsum("hk,hkv->hv", q[t], S)
            o = _rms(o, w[a + "o_norm.weight"], JET["norm_eps"]) * F.silu(gate)
            out = o.reshape(T, Hn * dv) @ w[a + "o_proj.weight"].T
        else:
            q = (h @ w[a + "q_proj.weight"].T + w[a + "q_proj.bias"]).view(T, nh, hd)
            k = (h @ w[a + "k_proj.weight"].T + w[a + "k_proj.bias"]).view(T, nkv, hd)
            v = (h @ w[a + "v_proj.weight"].T + w[a + "v_proj.bias"]).view(T, nkv, hd)
            q, k = rope(q), rope(k)
            m = ki <= qi
            if kind == "swa":
                m = m & (ki > qi - 8)
            o = torch.empty(T, nh, hd)
            for hh in range(nh):
                s = (q[:, hh] @ k[:, hh // (nh // nkv)].T) / math.sqrt(hd)
                o[:, hh] = torch.softmax(s.masked_fill(~m, float("-inf")), -1) @ v[:, hh // (nh // nkv)]
            out = o.reshape(T, H) @ w[a + "o_proj.weight"].T
        x = x + out
        h = _rms(x, w[p + "post_attention_layernorm.weight"], eps)
        x = x + (F.silu(h @ w[p + "mlp.gate_proj.weight"].T) * (h @ w[p + "mlp.up_proj.weight"].T)) @ \
            w[p + "mlp.down_proj.weight"].T
    return _rms(x, w["model.norm.weight"], eps) @ w["lm_head.weight"].T


def _checkpoint(tmp_path):
    w = _weights()
    save_file({k: v.contiguous() for k, v in w.items()}, tmp_path / "model.safetensors")
    (tmp_path / "config.json").write_text(json.dumps(CFG))
    return w


IDS = [(13 * i + 7) % 250 + 3 for i in range(23)]


def _greedy_ref(w, ids, n):
    toks = []
    for _ in range(n):
        toks.append(int(_ref_logits(w, ids + toks)[-1].argmax()))
    return toks


def test_jet_nemotron_generate_matches_restatement(tmp_path):
    w = _checkpoint(tmp_path)
    want = _greedy_ref(w, IDS, 6)
    for chunk in (512, 7):   # one prefill chunk / chunked prefill continuing conv + delta-rule state
        eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                                context_length=256, chunked_prefill_size=chunk))
        m = eng.runner.model
        assert type(m).__name__ == "JetNemotronForCausalLM" and m.kv_layers == [1, 3] and m.cpk == 1
        got = eng.generate([IDS], SamplingParams(max_new_tokens=6, ignore_eos=True))[0].output_ids
        assert got == want, (chunk, got, want)


def test_jet_nemotron_batch_of_two_matches_single(tmp_path):
    w = _checkpoint(tmp_path)
    other = [(5 * i + 11) % 250 + 3 for i in range(9)]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    outs = eng.generate([IDS, other], SamplingParams(max_new_tokens=5, ignore_eos=True))
    assert outs[0].output_ids == _greedy_ref(w, IDS, 5)
    assert outs[1].output_ids == _greedy_ref(w, other, 5)


def test_dyn_conv1d_reference_continues_state():
    g = torch.Generator().manual_seed(0)
    T, C, K = 9, 6, 4
    x = torch.randn(T, C, generator=g)
    taps = torch.randn(T, C * K, generator=g)
    st = torch.zeros(2, C, K - 1)
    whole = ops.dyn_conv1d(x, taps, st.clone(), torch.tensor([0, T]), torch.tensor([0]), torch.tensor([1]))
    st2 = torch.zeros(2, C, K - 1)
    a = ops.dyn_conv1d(x[:4], taps[:4], st2, torch.tensor([0, 4]), torch.tensor([1]), torch.tensor([1]))
    b = ops.dyn_conv1d(x[4:], taps[4:], st2, torch.tensor([0, T - 4]), torch.tensor([1]), torch.tensor([0]))
    assert torch.allclose(torch.cat([a, b]), whole, atol=1e-6)
    # per-head taps (cpk = 3): channels of a head share one kernel
    th = torch.randn(T, 2 * K, generator=g)
    o = ops.dyn_conv1d(x, th, torch.zeros(1, C, K - 1), torch.tensor([0, T]), torch.tensor([0]), torch.tensor([1]),
                       cpk=3)
    full = th.view(T, 2, 1, K).expand(-1, -1, 3, -1).reshape(T, C * K)
    assert torch.allclose(o, ops.dyn_conv1d(x, full, torch.zeros(1, C, K - 1), torch.tensor([0, T]),
                                            torch.tensor([0]), torch.tensor([1])), atol=1e-6)


def test_layer_types_defaults():
    assert jet_layer_types({}, 28)[15] == "attn" and jet_layer_types({}, 28)[21] == "swa"
    assert jet_layer_types({}, 28).count("jet") == 24
    assert jet_layer_types({"layer_types": ["linear_attention", "full_attention"]}, 2) == ["jet", "attn"]
