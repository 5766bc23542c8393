"""Mamba-2 kernels on gfx950 vs the fp32 PyTorch reference (strided views of one in_proj output,
varlen sequences, fresh and continued state), and a NemotronH-class model served with HIP-graph
decode agreeing with the eager path."""
import pytest
import torch

from ome_amd import ops
from ome_amd.ops import reference as ref
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("P,N", [(64, 128), (64, 64), (32, 128)])
def test_ssm_kernels_match_reference(P, N):
    torch.manual_seed(0)
    H, G, K = 8, 2, 4
    I, cd = H * P, H * P + 2 * G * N
    lens = [5, 1, 40]
    T = sum(lens)
    proj = (torch.randn(T, I + cd + H, device=DEV) * 0.5).to(torch.bfloat16)
    z, xbc, dt = proj[:, :I], proj[:, I:I + cd], proj[:, I + cd:]
    w = (torch.randn(cd, K, device=DEV) * 0.3).to(torch.bfloat16)
    b = (torch.randn(cd, device=DEV) * 0.1).to(torch.bfloat16)
    cu = torch.tensor([0, 5, 6, 46], dtype=torch.int32, device=DEV)
    slot = torch.tensor([2, 0, 3], dtype=torch.int32, device=DEV)
    reset = torch.tensor([1, 0, 0], dtype=torch.int32, device=DEV)
    cs0 = (torch.randn(4, cd, K - 1, device=DEV) * 0.5).to(torch.bfloat16)
    ss0 = torch.randn(4, H, P, N, device=DEV) * 0.1
    A = -torch.rand(H, device=DEV) - 0.2
    D, db = torch.randn(H, device=DEV), torch.randn(H, device=DEV) - 1.0
    gw = (torch.randn(I, device=DEV) * 0.2 + 1).to(torch.bfloat16)

    cs_k, cs_r = cs0.clone(), cs0.cpu().clone()
    conv_k = ops.ssm_conv1d(xbc, w, b, cs_k, cu, slot, reset)
    conv_r = ref.ssm_conv1d(xbc.cpu(), w.cpu(), b.cpu(), cs_r, cu.cpu(), slot.cpu(), reset.cpu(),
                            torch.empty(T, cd, dtype=torch.bfloat16))
    assert (conv_k.float().cpu() - conv_r.float()).abs().max().item() < 2e-2
    assert torch.equal(cs_k.cpu(), cs_r)  # last K-1 raw inputs per touched slot; slot 1 untouched
    xs, B, C = conv_k[:, :I], conv_k[:, I:I + G * N], conv_k[:, I + G * N:]
    ss_k, ss_r = ss0.clone(), ss0.clone().cpu()
    y_k = ops.ssm_scan(xs, dt, B, C, A, D, db, 0.001, ss_k, cu, slot, reset, H, P, N, G)
    y_r = ref.ssm_scan(xs.cpu(), dt.cpu(), B.cpu(), C.cpu(), A.cpu(), D.cpu(), db.cpu(), 0.001, ss_r, cu.cpu(),
                       slot.cpu(), reset.cpu(), H, P, N, G, torch.empty(T, I, dtype=torch.bfloat16))
    scale = max(1.0, y_r.float().abs().max().item())
    assert (y_k.float().cpu() - y_r.float()).abs().max().item() < 3e-2 * scale
    assert (ss_k.cpu() - ss_r).abs().max().item() < 1e-3 * max(1.0, ss_r.abs().max().item())
    assert torch.equal(ss_k[1].cpu(), ss0[1].cpu())  # untouched slot
    g_k = ops.gated_rmsnorm(y_k, z, gw, I // G, 1e-5)
    g_r = ref.gated_rmsnorm(y_k.cpu(), z.cpu(), gw.cpu(), I // G, 1e-5)
    assert (g_k.float().cpu() - g_r.float()).abs().max().item() < 3e-2 * max(1.0, g_r.float().abs().max().item())


def test_relu2_act():
    x = torch.randn(64, 256, device=DEV, dtype=torch.bfloat16)
    want = torch.relu(x.float()).square().to(torch.bfloat16)
    assert torch.equal(ops.act(x.clone(), 4), want)


def test_ungated_relu2_moe_matches_reference():
    torch.manual_seed(0)
    T, H, I, E, k = 37, 256, 128, 16, 4
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    wu = (torch.randn(E, I, H, device=DEV) * 0.05).to(torch.bfloat16)
    wd = (torch.randn(E, H, I, device=DEV) * 0.05).to(torch.bfloat16)
    logits = torch.randn(T, E, device=DEV)
    bias = torch.randn(E, device=DEV) * 0.05
    tw, tid = ops.moe_route(logits, k, True, "sigmoid", bias=bias, n_group=4, topk_group=2, group_mode=2)
    rw, rid = ref.moe_route(logits.cpu(), k, True, "sigmoid", bias.cpu(), 4, 2, 2)
    assert torch.equal(tid.cpu().sort(1)[0], rid.sort(1)[0].to(torch.int32))
    got = ops.fused_moe(x, tw, tid, wu, wd, 4, 2.5, gated=False)
    want = ref.fused_moe(x.cpu(), tw.cpu(), tid.cpu(), wu.cpu(), wd.cpu(), 4, 2.5, gated=False)
    assert (got.float().cpu() - want.float()).abs().max().item() < 3e-2 * max(1.0, want.float().abs().max().item())


@pytest.mark.parametrize("model", ["tiny-nemotron-h", "tiny-nemotron-h-moe"])
def test_nemotron_h_engine_graph_vs_eager(model):
    outs = []
    for graph in (True, False):
        eng = Engine(EngineArgs(model=model, device="cuda", max_running_requests=8, context_length=512,
                                cuda_graph=graph))
        assert eng.runner.use_graph == graph and eng.runner.model.kv_layers == ([3] if model == "tiny-nemotron-h"
                                                                                  else [2])
        prompts = [[11 + (i * 13 + j) % 900 for j in range(5 + 70 * i)] for i in range(3)]
        reqs = eng.generate(prompts, SamplingParams(max_new_tokens=16, ignore_eos=True))
        outs.append([r.output_ids for r in reqs])
        del eng
        torch.cuda.empty_cache()
    for a, b in zip(*outs):
        assert sum(int(x == y) for x, y in zip(a, b)) >= 14, (a, b)
