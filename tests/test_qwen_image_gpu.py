"""Qwen-Image on gfx950 (bf16): the fused per-head RMSNorm + 3-axis RoPE + joint-sequence scatter
kernel (``ome_qk_norm_rope``) against its fp32 reference, and the MMDiT forward (CFG pair as two
packed sequences, an edit-style conditioning image) against the fp32 restatement of
tests/test_qwen_image_cpu.py."""
import pytest
import torch

from ome_amd import ops
from ome_amd.diffusion.qwen_image_dit import QwenImageDiT
from ome_amd.ops import reference as ref
from tests.test_qwen_image_cpu import CFG, _ref_dit

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("norm,rope", [(True, True), (False, False), (True, False)])
def test_qk_norm_rope_kernel(hd, norm, rope):
    torch.manual_seed(0)
    T, H = 77, 6
    x = torch.randn(T, 3 * H * hd + 8, device="cuda").to(torch.bfloat16)[:, H * hd:2 * H * hd]
    w = (1 + 0.1 * torch.randn(hd, device="cuda")).to(torch.bfloat16) if norm else None
    ang = torch.rand(T, hd // 2, device="cuda") * 6.0
    cs = torch.stack([ang.cos(), ang.sin()], -1).contiguous() if rope else None
    dst = torch.randperm(T + 10, device="cuda")[:T].to(torch.int32)
    out = torch.zeros(T + 10, H, hd, device="cuda", dtype=torch.bfloat16)
    ops.qk_norm_rope(x, H, hd, w, cs, 1e-6, out, dst)
    want = torch.zeros(T + 10, H, hd, dtype=torch.bfloat16)
    ref.qk_norm_rope(x.cpu(), H, hd, None if w is None else w.cpu(), None if cs is None else cs.cpu(), 1e-6, want,
                     dst.cpu())
    assert (out.float().cpu() - want.float()).abs().max().item() < 3e-2 * max(1.0, want.float().abs().max().item())
    untouched = torch.ones(T + 10, dtype=torch.bool)
    untouched[dst.long().cpu()] = False
    assert out[untouched.cuda()].abs().max().item() == 0


def test_dit_on_gpu_matches_reference():
    cpu = QwenImageDiT(CFG, "cpu", torch.float32).init_random(3, std=0.08)
    sd = cpu.state_dict()
    dit = QwenImageDiT(CFG, "cuda", torch.bfloat16).load(sd.items())
    shapes = [(1, 4, 6), (1, 2, 4)]
    N = sum(f * h * w for f, h, w in shapes)
    g = torch.Generator().manual_seed(0)
    img = torch.randn(1, N, 64, generator=g).expand(2, N, 64).contiguous()
    txts = [torch.randn(7, 96, generator=g), torch.randn(4, 96, generator=g)]
    t = torch.tensor([0.7, 0.7])
    got = dit.forward(img.cuda(), [u.cuda() for u in txts], t.cuda(), shapes).float().cpu()
    want = _ref_dit(sd, CFG, img, txts, t, shapes)
    cos = torch.nn.functional.cosine_similarity(got.reshape(-1, 64), want.reshape(-1, 64), dim=-1)
    assert cos.min().item() > 0.99, cos.min().item()
