"""Gemma 2 / Gemma 3 (text) against Hugging Face transformers (installed in the image): a tiny
random HF model is saved as safetensors, loaded by ome_amd, and the prefill logits of every
position must match HF's eager forward (fp32, CPU reference ops) -- covering the (1 + w) norms,
sandwich norms, embedding scaling, GeGLU, query_pre_attn_scalar, attention-logit soft-capping,
per-layer sliding windows, Gemma-3 q/k-norm and local RoPE base, and final-logit soft-capping."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from ome_amd import ops  # noqa: E402
from ome_amd.models.common import AttnMeta  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402


def _hf_model(kind: str, tmp_path):
    torch.manual_seed(0)
    common = dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=4, num_attention_heads=4,
                  num_key_value_heads=2, head_dim=64, max_position_embeddings=512, rms_norm_eps=1e-6,
                  sliding_window=16, query_pre_attn_scalar=64, pad_token_id=0, bos_token_id=1, eos_token_id=2)
    if kind == "gemma2":
        cfg = transformers.Gemma2Config(attn_logit_softcapping=50.0, final_logit_softcapping=30.0, **common)
        m = transformers.Gemma2ForCausalLM(cfg)
    else:
        cfg = transformers.Gemma3TextConfig(rope_theta=1_000_000.0, rope_local_base_freq=10_000.0,
                                            sliding_window_pattern=2, **common)
        m = transformers.Gemma3ForCausalLM(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(0.0, 0.2)  # exercise the (1 + w) fold
            elif p.dim() == 2:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    return m


def _our_logits(eng: Engine, ids: list[int]) -> torch.Tensor:
    run = eng.runner
    slot = run.slots.alloc()
    pages = run.pages.alloc(-(-len(ids) // run.P))
    run.slots.set_pages(slot, 0, pages)
    run.slots.flush()
    T = len(ids)
    t = lambda a: torch.tensor(a, dtype=torch.int32)  # noqa: E731
    meta = AttnMeta("prefill", t(list(range(T))), t([pages[p // run.P] * run.P + p % run.P for p in range(T)]),
                    run.slots.table.index_select(0, t([slot])), cu_q=t([0, T]), kv_lens=t([T]),
                    items=t(ops.prefill_work_items([T], [T])).view(-1, 2))
    h = run.model.forward(t(ids), meta, run.kv)
    out = run.model.compute_logits(h).float()
    run.pages.free(pages)
    run.slots.free(slot)
    return out


@pytest.mark.parametrize("kind", ["gemma2", "gemma3"])
def test_gemma_prefill_logits_match_hf(tmp_path, kind):
    hf = _hf_model(kind, tmp_path)
    ids = [(7 * i + 3) % 500 + 3 for i in range(40)]  # longer than the sliding window
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "GemmaForCausalLM"
    assert m.windows.count(16) >= 1 and m.windows.count(-1) >= 1
    got = _our_logits(eng, ids)
    err = (got - want).abs().max().item()
    assert err < 2e-3 * max(1.0, want.abs().max().item()), err
    # greedy continuation agrees with HF generate
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ids]), max_new_tokens=6, do_sample=False)[0, len(ids):].tolist()
    r = eng.generate([ids], SamplingParams(max_new_tokens=6, ignore_eos=True))[0]
    assert r.output_ids == ref


def test_gemma2_sequence_classification_matches_hf(tmp_path):
    """Gemma2ForSequenceClassification (Skywork-Reward-Gemma-2 style reward model): the score of the
    last token of each prompt matches HF's pooled logits."""
    from tests.test_decoder_remote_families_cpu import _scores

    torch.manual_seed(0)
    cfg = transformers.Gemma2Config(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=4,
                                    num_attention_heads=4, num_key_value_heads=2, head_dim=64,
                                    max_position_embeddings=512, rms_norm_eps=1e-6, sliding_window=16,
                                    query_pre_attn_scalar=64, attn_logit_softcapping=50.0,
                                    final_logit_softcapping=30.0, pad_token_id=0, num_labels=1)
    hf = transformers.Gemma2ForSequenceClassification(cfg)
    with torch.no_grad():
        for n, p in hf.named_parameters():
            if "norm" in n:
                p.normal_(0.0, 0.2)
            elif p.dim() == 2:
                p.normal_(0.0, 0.08)
    hf = hf.float().eval()
    hf.config._attn_implementation = "eager"
    hf.save_pretrained(tmp_path, safe_serialization=True)
    prompts = [[(7 * i + 3) % 500 + 3 for i in range(40)], [(5 * i + 1) % 500 + 3 for i in range(11)]]
    with torch.no_grad():
        want = torch.cat([hf(torch.tensor([p])).logits for p in prompts]).float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    assert eng.cfg.is_embedding
    got = _scores(eng, prompts)
    assert got.shape == (2, 1) and torch.allclose(got, want, atol=2e-3, rtol=2e-3), (got, want)
