"""Gated DeltaNet kernels on gfx950 vs the fp32 PyTorch reference (strided views of one
projection output, varlen sequences, fresh and continued state, GQA-style k-head sharing), the
norm-then-gate RMSNorm, and a Qwen3-Next-class model served with HIP-graph decode agreeing with
the eager path."""
import pytest
import torch

from ome_amd import ops
from ome_amd.ops import reference as ref
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("v1", [False, True])
@pytest.mark.parametrize("aligned", [True, False])
@pytest.mark.parametrize("dk,dv,Hk,Hv", [(128, 128, 2, 4), (64, 128, 4, 4), (128, 64, 1, 2),
                                         (256, 512, 2, 2), (64, 96, 2, 2)])   # + Jet-Nemotron shapes
def test_gdn_scan_matches_reference(dk, dv, Hk, Hv, aligned, v1):
    if v1 and (dk > 128 or dv > 128):
        pytest.skip("v1 kernel: dk <= 128, dv <= 128")
    torch.manual_seed(0)
    kd, vd = Hk * dk, Hv * dv
    lens = [5, 1, 70]
    T = sum(lens)
    pad = 8 - (2 * Hv) % 8 if aligned else 1   # row stride % 8 == 0 (the model's conv output) or odd
    proj = (torch.randn(T, 2 * kd + vd + 2 * Hv + pad, device=DEV)).to(torch.bfloat16)
    q, k, v = proj[:, :kd], proj[:, kd:2 * kd], proj[:, 2 * kd:2 * kd + vd]
    b, a = proj[:, 2 * kd + vd:2 * kd + vd + Hv], proj[:, 2 * kd + vd + Hv:2 * kd + vd + 2 * Hv]
    A_log = torch.rand(Hv, device=DEV) * 2 - 1
    dtb = torch.randn(Hv, device=DEV) * 0.5
    cu = torch.tensor([0, 5, 6, 76], dtype=torch.int32, device=DEV)
    slot = torch.tensor([2, 0, 3], dtype=torch.int32, device=DEV)
    reset = torch.tensor([1, 0, 0], dtype=torch.int32, device=DEV)
    st0 = torch.randn(4, Hv, dv, dk, device=DEV) * 0.1
    st_k, st_r = st0.clone(), st0.clone().cpu()
    y_k = ops.gdn_scan(q, k, v, a, b, A_log, dtb, st_k, cu, slot, reset, Hv, Hk, v1=v1)
    c = lambda t: t.cpu()  # noqa: E731
    y_r = ref.gdn_scan(c(q), c(k), c(v), c(a), c(b), c(A_log), c(dtb), st_r, c(cu), c(slot), c(reset), Hv, Hk,
                       torch.empty(T, vd, dtype=torch.bfloat16))
    scale = max(1.0, y_r.float().abs().max().item())
    assert (y_k.float().cpu() - y_r.float()).abs().max().item() < 2e-2 * scale
    assert (st_k.cpu() - st_r).abs().max().item() < 1e-3 * max(1.0, st_r.abs().max().item())
    assert torch.equal(st_k[1].cpu(), st0[1].cpu())   # untouched slot


def test_norm_first_gated_rmsnorm():
    torch.manual_seed(0)
    T, H, dv = 37, 8, 128
    y = torch.randn(T, H * dv, device=DEV, dtype=torch.bfloat16)
    zz = torch.randn(T, H * dv + 64, device=DEV, dtype=torch.bfloat16)
    z = zz[:, 64:]
    w = (torch.randn(dv, device=DEV) * 0.2 + 1).to(torch.bfloat16)
    got = ops.gated_rmsnorm(y, z, w, dv, 1e-6, norm_first=True)
    want = ref.gated_rmsnorm(y.cpu(), z.cpu(), w.cpu(), dv, 1e-6, norm_first=True)
    assert (got.float().cpu() - want.float()).abs().max().item() < 3e-2 * max(1.0, want.float().abs().max().item())


def test_qwen3_next_engine_graph_vs_eager():
    outs = []
    for graph in (True, False):
        eng = Engine(EngineArgs(model="tiny-qwen3-next", device="cuda", max_running_requests=8, context_length=512,
                                cuda_graph=graph))
        assert eng.runner.use_graph == graph and eng.runner.model.kv_layers == [3]
        prompts = [[11 + (i * 13 + j) % 900 for j in range(5 + 70 * i)] for i in range(3)]
        reqs = eng.generate(prompts, SamplingParams(max_new_tokens=16, ignore_eos=True))
        outs.append([r.output_ids for r in reqs])
        del eng
        torch.cuda.empty_cache()
    for a, b in zip(*outs):
        assert sum(int(x == y) for x, y in zip(a, b)) >= 14, (a, b)
