"""Remote-code families of the reference catalog (checkpoints whose modelling code lives in the
model repo, not in transformers: InternLM2 (+ reward head), Qwen (v1), Baichuan-2, EXAONE-3,
Orion, MiniCPM, ChatGLM / GLM-4 (THUDM layout), MiMo) and the sequence-classification heads.

transformers does not ship these classes, so each test builds the transformers model with the
same mathematics (Llama, Qwen2, StableLM-without-qk-norm = Orion, Granite multipliers = MiniCPM
scales, GLM = ChatGLM), re-lays its weights into the family's own checkpoint names / fused
layouts and config spelling, and checks ome_amd's logits (or scores) on that checkpoint against
the transformers forward.  This pins the checkpoint mapping; the equivalence of the remote
modelling code with its transformers counterpart is parity unpinned (the remote code is not
available offline)."""
import json
import math

import pytest
import torch

transformers = pytest.importorskip("transformers")

from safetensors.torch import save_file  # noqa: E402

from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

from test_gemma_cpu import _our_logits  # noqa: E402

V = 512
IDS = [(7 * i + 3) % 500 + 3 for i in range(40)]


def _rand(m):
    torch.manual_seed(0)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n and n.endswith("weight"):
                p.normal_(1.0, 0.2)
            elif p.dim() == 2:
                p.normal_(0.0, 0.08)
            else:
                p.normal_(0.0, 0.05)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    return m


def _llama(**kw):
    T = transformers
    c = dict(vocab_size=V, hidden_size=256, intermediate_size=384, num_hidden_layers=3, num_attention_heads=4,
             num_key_value_heads=2, max_position_embeddings=512, rope_theta=10000.0, rms_norm_eps=1e-5,
             tie_word_embeddings=False)
    c.update(kw)
    return _rand(T.LlamaForCausalLM(T.LlamaConfig(**c)))


def _save(tmp, cfg: dict, sd: dict):
    (tmp / "config.json").write_text(json.dumps(cfg))
    save_file({k: v.contiguous() for k, v in sd.items()}, str(tmp / "model.safetensors"))


def _llama_keys(hf):
    c = hf.config
    return dict(vocab_size=c.vocab_size, hidden_size=c.hidden_size, intermediate_size=c.intermediate_size,
                num_hidden_layers=c.num_hidden_layers, num_attention_heads=c.num_attention_heads,
                num_key_value_heads=c.num_key_value_heads, max_position_embeddings=512, rms_norm_eps=1e-5,
                rope_theta=10000.0, tie_word_embeddings=False)


def _layers(sd):
    n = 1 + max(int(k.split(".")[2]) for k in sd if k.startswith("model.layers."))
    return range(n)


def _convert(kind, tmp):
    """-> (reference transformers model, reference output kind)"""
    if kind in ("internlm2", "internlm2_reward"):
        hf = _llama()
        sd, c = hf.state_dict(), hf.config
        nh, nkv, D = c.num_attention_heads, c.num_key_value_heads, c.hidden_size // c.num_attention_heads
        G = nh // nkv
        out = {"model.tok_embeddings.weight": sd["model.embed_tokens.weight"], "model.norm.weight": sd["model.norm.weight"],
               "output.weight": sd["lm_head.weight"]}
        for i in _layers(sd):
            p = f"model.layers.{i}."
            q = sd[p + "self_attn.q_proj.weight"].view(nkv, G, D, -1)
            k = sd[p + "self_attn.k_proj.weight"].view(nkv, 1, D, -1)
            v = sd[p + "self_attn.v_proj.weight"].view(nkv, 1, D, -1)
            out[p + "attention.wqkv.weight"] = torch.cat([q, k, v], 1).reshape(-1, c.hidden_size)
            out[p + "attention.wo.weight"] = sd[p + "self_attn.o_proj.weight"]
            out[p + "feed_forward.w1.weight"] = sd[p + "mlp.gate_proj.weight"]
            out[p + "feed_forward.w3.weight"] = sd[p + "mlp.up_proj.weight"]
            out[p + "feed_forward.w2.weight"] = sd[p + "mlp.down_proj.weight"]
            out[p + "attention_norm.weight"] = sd[p + "input_layernorm.weight"]
            out[p + "ffn_norm.weight"] = sd[p + "post_attention_layernorm.weight"]
        arch = "InternLM2ForCausalLM"
        if kind == "internlm2_reward":
            arch = "InternLM2ForRewardModel"
            hf.v_head = torch.randn(1, c.hidden_size) * 0.1
            out["v_head.weight"] = hf.v_head
        _save(tmp, {"architectures": [arch], "model_type": "internlm2", "bias": False, **_llama_keys(hf)}, out)
        return hf
    if kind in ("qwen1", "mimo"):
        T = transformers
        hf = _rand(T.Qwen2ForCausalLM(T.Qwen2Config(vocab_size=V, hidden_size=256, intermediate_size=384,
                                                    num_hidden_layers=3, num_attention_heads=4,
                                                    num_key_value_heads=4 if kind == "qwen1" else 2,
                                                    max_position_embeddings=512, rope_theta=10000.0,
                                                    rms_norm_eps=1e-6, tie_word_embeddings=False)))
        sd, c = hf.state_dict(), hf.config
        if kind == "mimo":
            out = dict(sd)
            out["model.mtp_layers.0.input_layernorm.weight"] = torch.ones(c.hidden_size)
            keys = _llama_keys(hf)
            keys["rms_norm_eps"] = 1e-6
            _save(tmp, {"architectures": ["MiMoForCausalLM"], "model_type": "mimo", **keys}, out)
            return hf
        out = {"transformer.wte.weight": sd["model.embed_tokens.weight"], "transformer.ln_f.weight": sd["model.norm.weight"],
               "lm_head.weight": sd["lm_head.weight"]}
        for i in _layers(sd):
            p, q = f"model.layers.{i}.", f"transformer.h.{i}."
            for kd in ("weight", "bias"):
                out[q + f"attn.c_attn.{kd}"] = torch.cat([sd[p + f"self_attn.{x}_proj.{kd}"] for x in "qkv"], 0)
            out[q + "attn.c_proj.weight"] = sd[p + "self_attn.o_proj.weight"]
            out[q + "mlp.w1.weight"] = sd[p + "mlp.up_proj.weight"]
            out[q + "mlp.w2.weight"] = sd[p + "mlp.gate_proj.weight"]
            out[q + "mlp.c_proj.weight"] = sd[p + "mlp.down_proj.weight"]
            out[q + "ln_1.weight"] = sd[p + "input_layernorm.weight"]
            out[q + "ln_2.weight"] = sd[p + "post_attention_layernorm.weight"]
        _save(tmp, {"architectures": ["QWenLMHeadModel"], "model_type": "qwen", "vocab_size": V, "hidden_size": 256,
                    "intermediate_size": 2 * c.intermediate_size, "num_hidden_layers": 3, "num_attention_heads": 4,
                    "kv_channels": 64, "rotary_emb_base": 10000, "rotary_pct": 1.0, "layer_norm_epsilon": 1e-6,
                    "seq_length": 512}, out)
        return hf
    if kind == "baichuan2":  # NormHead: the checkpoint keeps the raw lm_head, logits use normalised rows
        hf = _llama(num_key_value_heads=2, vocab_size=125696, num_hidden_layers=2, hidden_size=128,
                    intermediate_size=256, num_attention_heads=2)
        sd = dict(hf.state_dict())
        out = {k: v.clone() for k, v in sd.items() if ".self_attn.q_proj" not in k and ".self_attn.k_proj" not in k
               and ".self_attn.v_proj" not in k}
        for i in _layers(sd):
            p = f"model.layers.{i}.self_attn."
            out[p + "W_pack.weight"] = torch.cat([sd[p + f"{x}_proj.weight"] for x in "qkv"], 0)
        with torch.no_grad():
            hf.lm_head.weight.copy_(torch.nn.functional.normalize(hf.lm_head.weight, dim=-1))
        keys = _llama_keys(hf)
        keys.pop("max_position_embeddings")
        _save(tmp, {"architectures": ["BaichuanForCausalLM"], "model_type": "baichuan", "model_max_length": 512,
                    **keys}, out)
        return hf
    if kind == "exaone":
        hf = _llama()
        sd = hf.state_dict()
        out = {"transformer.wte.weight": sd["model.embed_tokens.weight"], "transformer.ln_f.weight": sd["model.norm.weight"],
               "lm_head.weight": sd["lm_head.weight"]}
        for i in _layers(sd):
            p, q = f"model.layers.{i}.", f"transformer.h.{i}."
            for x in "qkv":
                out[q + f"attn.attention.{x}_proj.weight"] = sd[p + f"self_attn.{x}_proj.weight"]
            out[q + "attn.attention.out_proj.weight"] = sd[p + "self_attn.o_proj.weight"]
            out[q + "mlp.c_fc_0.weight"] = sd[p + "mlp.gate_proj.weight"]
            out[q + "mlp.c_fc_1.weight"] = sd[p + "mlp.up_proj.weight"]
            out[q + "mlp.c_proj.weight"] = sd[p + "mlp.down_proj.weight"]
            out[q + "ln_1.weight"] = sd[p + "input_layernorm.weight"]
            out[q + "ln_2.weight"] = sd[p + "post_attention_layernorm.weight"]
        keys = _llama_keys(hf)
        _save(tmp, {"architectures": ["ExaoneForCausalLM"], "model_type": "exaone", "num_layers": 3,
                    "layer_norm_epsilon": 1e-5, "activation_function": "silu",
                    **{k: v for k, v in keys.items() if k not in ("num_hidden_layers", "rms_norm_eps")}}, out)
        return hf
    if kind == "orion":  # = StableLM without qk-norm / qkv bias, full rotary, sequential residual
        T = transformers
        hf = _rand(T.StableLmForCausalLM(T.StableLmConfig(vocab_size=V, hidden_size=256, intermediate_size=384,
                                                          num_hidden_layers=3, num_attention_heads=4,
                                                          num_key_value_heads=4, partial_rotary_factor=1.0,
                                                          max_position_embeddings=512, layer_norm_eps=1e-5)))
        _save(tmp, {"architectures": ["OrionForCausalLM"], "model_type": "orion", "vocab_size": V, "hidden_size": 256,
                    "intermediate_size": 384, "num_hidden_layers": 3, "num_attention_heads": 4,
                    "num_key_value_heads": 4, "max_position_embeddings": 512, "rms_norm_eps": 1e-5,
                    "rope_theta": 10000.0, "tie_word_embeddings": False}, hf.state_dict())
        return hf
    if kind == "minicpm":  # MiniCPM scales = Granite multipliers with attention scale 1/sqrt(D)
        T = transformers
        L, H, dmb, se, sdp = 3, 256, 64, 12.0, 1.4
        hf = _rand(T.GraniteForCausalLM(T.GraniteConfig(vocab_size=V, hidden_size=H, intermediate_size=384,
                                                        num_hidden_layers=L, num_attention_heads=4,
                                                        num_key_value_heads=2, max_position_embeddings=512,
                                                        embedding_multiplier=se, residual_multiplier=sdp / math.sqrt(L),
                                                        attention_multiplier=64 ** -0.5, logits_scaling=H / dmb,
                                                        tie_word_embeddings=True, rms_norm_eps=1e-5)))
        keys = _llama_keys(hf)
        keys["tie_word_embeddings"] = True
        _save(tmp, {"architectures": ["MiniCPMForCausalLM"], "model_type": "minicpm", "scale_emb": se,
                    "scale_depth": sdp, "dim_model_base": dmb, **keys},
              {k: v for k, v in hf.state_dict().items() if k != "lm_head.weight"})
        return hf
    if kind == "chatglm":  # THUDM layout of the GLM architecture (transformers' Glm is its port)
        T = transformers
        hf = _rand(T.GlmForCausalLM(T.GlmConfig(vocab_size=V, hidden_size=256, intermediate_size=384,
                                                num_hidden_layers=3, num_attention_heads=4, num_key_value_heads=2,
                                                head_dim=64, partial_rotary_factor=0.5, attention_bias=True,
                                                max_position_embeddings=512, rms_norm_eps=1e-5,
                                                tie_word_embeddings=False, pad_token_id=0)))
        sd = hf.state_dict()
        out = {"transformer.embedding.word_embeddings.weight": sd["model.embed_tokens.weight"],
               "transformer.encoder.final_layernorm.weight": sd["model.norm.weight"],
               "transformer.output_layer.weight": sd["lm_head.weight"]}
        for i in _layers(sd):
            p, q = f"model.layers.{i}.", f"transformer.encoder.layers.{i}."
            for kd in ("weight", "bias"):
                out[q + f"self_attention.query_key_value.{kd}"] = torch.cat(
                    [sd[p + f"self_attn.{x}_proj.{kd}"] for x in "qkv"], 0)
            out[q + "self_attention.dense.weight"] = sd[p + "self_attn.o_proj.weight"]
            out[q + "mlp.dense_h_to_4h.weight"] = sd[p + "mlp.gate_up_proj.weight"]
            out[q + "mlp.dense_4h_to_h.weight"] = sd[p + "mlp.down_proj.weight"]
            out[q + "input_layernorm.weight"] = sd[p + "input_layernorm.weight"]
            out[q + "post_attention_layernorm.weight"] = sd[p + "post_attention_layernorm.weight"]
        _save(tmp, {"architectures": ["ChatGLMModel"], "model_type": "chatglm", "hidden_size": 256, "num_layers": 3,
                    "num_attention_heads": 4, "multi_query_attention": True, "multi_query_group_num": 2,
                    "kv_channels": 64, "ffn_hidden_size": 384, "padded_vocab_size": V, "layernorm_epsilon": 1e-5,
                    "seq_length": 512, "rope_ratio": 1, "add_qkv_bias": True, "rmsnorm": True}, out)
        return hf
    raise KeyError(kind)


@pytest.mark.parametrize("kind", ["internlm2", "qwen1", "mimo", "baichuan2", "exaone", "orion", "minicpm", "chatglm"])
def test_remote_family_checkpoint(tmp_path, kind):
    hf = _convert(kind, tmp_path)
    with torch.no_grad():
        want = hf(torch.tensor([IDS])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    assert type(eng.runner.model).__name__ == "DecoderForCausalLM" and not eng.cfg.is_embedding
    got = _our_logits(eng, IDS)
    err = (got - want).abs().max().item()
    assert err < 2e-3 * max(1.0, want.abs().max().item()), err
    with torch.no_grad():
        want_ids = hf.generate(torch.tensor([IDS]), max_new_tokens=5, do_sample=False)[0, len(IDS):].tolist()
    assert eng.generate([IDS], SamplingParams(max_new_tokens=5, ignore_eos=True))[0].output_ids == want_ids


def _scores(eng, prompts):
    reqs = [eng.make_request(p, SamplingParams(max_new_tokens=0)) for p in prompts]
    for r in reqs:
        r.is_embedding = True
        eng.add_request(r)
    while not all(r.finished for r in reqs):
        eng.step()
    return torch.tensor([r.embedding for r in reqs])


def test_internlm2_reward_head(tmp_path):
    hf = _convert("internlm2_reward", tmp_path)
    prompts = [IDS, IDS[:9]]
    with torch.no_grad():
        want = torch.stack([hf.model(torch.tensor([p])).last_hidden_state[0, -1] @ hf.v_head.T for p in prompts])
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    assert eng.cfg.is_embedding
    got = _scores(eng, prompts)
    assert got.shape == (2, 1) and torch.allclose(got, want, atol=2e-3, rtol=2e-3), (got, want)


def test_llama_sequence_classification_head(tmp_path):
    T = transformers
    hf = _rand(T.LlamaForSequenceClassification(T.LlamaConfig(
        vocab_size=V, hidden_size=256, intermediate_size=384, num_hidden_layers=2, num_attention_heads=4,
        num_key_value_heads=2, max_position_embeddings=512, num_labels=3, pad_token_id=0)))
    hf.save_pretrained(tmp_path, safe_serialization=True)
    prompts = [IDS, IDS[:13]]
    with torch.no_grad():
        want = torch.cat([hf(torch.tensor([p])).logits for p in prompts])
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    got = _scores(eng, prompts)
    assert got.shape == (2, 3) and torch.allclose(got, want, atol=2e-3, rtol=2e-3), (got, want)


def test_embedding_model_batch_matches_hf(tmp_path):
    """--is-embedding (e5-mistral style MistralModel): last-token pooling + L2 norm for a batch of
    prompts of different lengths, one of them a prefix of another (prefix-cache hit)."""
    T = transformers
    hf = _rand(T.MistralModel(T.MistralConfig(vocab_size=V, hidden_size=256, intermediate_size=384,
                                              num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                                              max_position_embeddings=512, pad_token_id=0)))
    hf.config.architectures = ["MistralModel"]
    hf.save_pretrained(tmp_path, safe_serialization=True)
    prompts = [IDS, IDS[:9], IDS[5:30]]
    with torch.no_grad():
        want = torch.stack([torch.nn.functional.normalize(hf(torch.tensor([p])).last_hidden_state[0, -1], dim=-1)
                            for p in prompts])
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    assert eng.cfg.is_embedding
    got = _scores(eng, prompts)
    assert torch.allclose(got, want, atol=2e-4), (got - want).abs().max()
