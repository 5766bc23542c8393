"""LayerNorm families on gfx950: the ``ome_layernorm`` / ``ome_act`` HIP kernels against fp32
PyTorch references, and Starcoder2 / GPT-NeoX class models through the engine with HIP-graph
decode (graph decode must agree with an eager prefill recompute)."""
import pytest
import torch

from ome_amd import ops
from ome_amd.ops import reference as ref
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_engine_gpu import _hidden_prefill

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H", [128, 2048, 4608, 8192])
@pytest.mark.parametrize("rows", [1, 7, 600])
def test_layernorm_kernel(H, rows):
    torch.manual_seed(H + rows)
    x = (torch.randn(rows, H, device="cuda") * 3 + 1).bfloat16()
    w = torch.randn(H, device="cuda").bfloat16()
    b = torch.randn(H, device="cuda").bfloat16()
    want = torch.nn.functional.layer_norm(x.float(), (H,), w.float(), b.float(), 1e-5)
    got = ops.layernorm(x, w, b, 1e-5)
    assert (got.float() - want).abs().max().item() < 0.05 * max(1.0, want.abs().max().item() / 8)
    got_nb = ops.layernorm(x, w, None, 1e-5)
    want_nb = torch.nn.functional.layer_norm(x.float(), (H,), w.float(), None, 1e-5)
    assert torch.allclose(got_nb.float(), want_nb, atol=0.06, rtol=0.02)
    # fused residual add
    r = torch.randn(rows, H, device="cuda").bfloat16()
    xx, rr = x.clone(), r.clone()
    ops.fused_add_layernorm(xx, rr, w, b, 1e-5)
    s = (x.float() + r.float()).bfloat16()
    assert torch.equal(rr, s)
    assert torch.allclose(xx.float(), ref.layernorm(s.float(), w.float(), b.float(), 1e-5), atol=0.06, rtol=0.02)


@pytest.mark.parametrize("kind", [0, 1, 3])
def test_act_kernel(kind):
    torch.manual_seed(kind)
    x = (torch.randn(3, 8192, device="cuda") * 4).bfloat16()
    want = ref.act(x.float().clone(), kind)
    got = ops.act(x.clone(), kind)
    assert torch.allclose(got.float(), want, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("model", ["tiny-starcoder2", "tiny-neox", "tiny-phi"])
def test_layernorm_family_engine_graph_decode(model):
    eng = Engine(EngineArgs(model=model, device="cuda", max_running_requests=8, context_length=512))
    m = eng.runner.model
    assert type(m).__name__ == "LayerNormForCausalLM" and eng.runner.use_graph
    prompts = [[11 + (i * 13 + j) % 900 for j in range(5 + 70 * i)] for i in range(3)]
    reqs = eng.generate(prompts, SamplingParams(max_new_tokens=16, ignore_eos=True))
    for r in reqs:
        assert len(r.output_ids) == 16
        seq = r.prompt_ids + r.output_ids
        h = _hidden_prefill(eng, seq[:-1])
        top = m.compute_logits(h[-16:]).float().argmax(-1).cpu().tolist()
        assert sum(int(a == b) for a, b in zip(top, r.output_ids)) >= 14, (top, r.output_ids)
