"""Starcoder2 and GPT-NeoX (LayerNorm families) against Hugging Face transformers: a tiny random
HF model is saved as safetensors, loaded by ome_amd and run on the CPU reference ops; prefill
logits of every position must match HF's eager forward and greedy decoding must agree with
``generate`` -- covering LayerNorm+bias, projection biases, GELU-tanh / exact-GELU MLPs, GQA +
sliding window (Starcoder2), fused per-head QKV, partial rotary and the parallel residual
(GPT-NeoX, both residual forms) and Phi-2 (shared-norm parallel residual, biased lm_head)."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from ome_amd import ops  # noqa: E402
from ome_amd.models.config import preset  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402
from ome_amd.ops import reference as ref  # noqa: E402

from test_gemma_cpu import _our_logits  # noqa: E402


def _hf_model(kind: str, tmp_path):
    torch.manual_seed(0)
    if kind == "starcoder2":
        cfg = transformers.Starcoder2Config(vocab_size=512, hidden_size=128, intermediate_size=384,
                                            num_hidden_layers=3, num_attention_heads=4, num_key_value_heads=2,
                                            max_position_embeddings=512, sliding_window=16, bos_token_id=1,
                                            eos_token_id=2)
        m = transformers.Starcoder2ForCausalLM(cfg)
    elif kind == "phi":
        # head_dim 80 (as Phi-2): exercises the zero-padding to the 128 kernel tile
        cfg = transformers.PhiConfig(vocab_size=512, hidden_size=160, intermediate_size=384, num_hidden_layers=3,
                                     num_attention_heads=2, partial_rotary_factor=0.4, hidden_act="gelu_new",
                                     max_position_embeddings=512, bos_token_id=1, eos_token_id=2)
        m = transformers.PhiForCausalLM(cfg)
    else:
        cfg = transformers.GPTNeoXConfig(vocab_size=512, hidden_size=128, intermediate_size=512,
                                         num_hidden_layers=3, num_attention_heads=2, rotary_pct=0.25,
                                         use_parallel_residual=(kind == "neox"), max_position_embeddings=512,
                                         bos_token_id=1, eos_token_id=2)
        m = transformers.GPTNeoXForCausalLM(cfg)
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
    m.save_pretrained(tmp_path, safe_serialization=True)
    return m


@pytest.mark.parametrize("kind", ["starcoder2", "neox", "neox_sequential", "phi"])
def test_layernorm_family_matches_hf(tmp_path, kind):
    hf = _hf_model(kind, tmp_path)
    ids = [(7 * i + 3) % 500 + 3 for i in range(40)]
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "LayerNormForCausalLM"
    if kind == "starcoder2":
        assert m.window == 16 and m.tp.hkv == 2
    elif kind == "phi":
        assert m.phi and m.parallel_residual and m.lm_head_b is not None
        assert m.cfg.rot_dim == 32 and m.D == 128 and m.Dt == 80
    else:
        assert m.cfg.rot_dim == 16 and m.parallel_residual == (kind == "neox")
    got = _our_logits(eng, ids)
    err = (got - want).abs().max().item()
    assert err < 2e-3 * max(1.0, want.abs().max().item()), err
    with torch.no_grad():
        want_ids = hf.generate(torch.tensor([ids]), max_new_tokens=6, do_sample=False)[0, len(ids):].tolist()
    r = eng.generate([ids], SamplingParams(max_new_tokens=6, ignore_eos=True))[0]
    assert r.output_ids == want_ids


def test_presets_and_config_parsing():
    for name in ("starcoder2-7b", "pythia-1.4b", "tiny-starcoder2", "tiny-neox", "phi-2", "tiny-phi"):
        assert preset(name).rms_norm_eps == 1e-5
    c = preset("pythia-1.4b")
    assert c.rot_dim == 32 and c.head_dim == 128
    c = preset("starcoder2-7b")
    assert c.sliding_window == 4096 and c.attention_bias and c.rope_theta == 1e6
    c = preset("phi-2")
    assert c.rot_dim == 32 and c.head_dim == 128 and c.attn_head_dim == 80 and c.attention_bias and c.hidden_act == "gelu_new"


def test_layernorm_and_act_reference_ops():
    torch.manual_seed(0)
    x = torch.randn(5, 64)
    w, b = torch.randn(64), torch.randn(64)
    want = torch.nn.functional.layer_norm(x, (64,), w, b, 1e-5)
    assert torch.allclose(ops.layernorm(x, w, b, 1e-5), want, atol=1e-5)
    r = torch.randn(5, 64)
    xx, rr = x.clone(), r.clone()
    ops.fused_add_layernorm(xx, rr, w, b, 1e-5)
    assert torch.allclose(rr, x + r) and torch.allclose(xx, ref.layernorm(x + r, w, b, 1e-5), atol=1e-5)
    y = ops.act(x.clone(), 3)
    assert torch.allclose(y, torch.nn.functional.gelu(x), atol=1e-6)


def test_phi2_param_count_uses_checkpoint_head_dim():
    """Phi-2's heads are zero-padded 80 -> 128 for the kernels; the parameter count (memory and
    weight estimates) must still be the checkpoint's 2.78 B."""
    from ome_amd.models.config import preset

    cfg = preset("phi-2")
    assert cfg.head_dim == 128 and cfg.attn_head_dim == 80
    assert abs(cfg.num_params() / 1e9 - 2.78) < 0.02


def test_random_init_zeroes_padded_head_dims():
    """Random-init weights of a padded-head model behave like a padded checkpoint: the pad rows of
    q/k/v (weights and biases) and the pad columns of o_proj are zero."""
    from ome_amd.models.layernorm_lm import LayerNormForCausalLM

    cfg = preset("tiny-phi")
    cfg.head_dim, cfg.attn_head_dim = 128, cfg.head_dim  # pad 64 -> 128 as Phi-2 pads 80 -> 128
    m = LayerNormForCausalLM(cfg, device="cpu", dtype=torch.float32).init_random(seed=1)
    Dt, D, H = 64, 128, cfg.hidden_size
    for i in m.layers:
        assert m.w_qkv[i].view(-1, D, H)[:, Dt:].abs().sum() == 0
        assert m.b_qkv[i].view(-1, D)[:, Dt:].abs().sum() == 0
        assert m.w_o[i].view(H, -1, D)[:, :, Dt:].abs().sum() == 0
        assert m.w_qkv[i].view(-1, D, H)[:, :Dt].abs().sum() > 0
