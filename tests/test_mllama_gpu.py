"""Llama 3.2 Vision on gfx950: the tiny HF Mllama of ``test_mllama_cpu`` served in bf16 through the
HIP kernels (vision-token cache written by ``ome_kv_cache_write``, cross attention on the paged
decode kernel with per-row key ranges), against HF's fp32 forward; graph decode of an image
request against an eager recompute; and the per-row ``row_lo`` decode-kernel range vs the fp32
reference."""
import pytest
import torch

from ome_amd import ops
from ome_amd.ops import reference as ref
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_mllama_cpu import CASES, _hf, _hf_inputs, _images, _prefill_logits

pytestmark = pytest.mark.gpu


def test_decode_row_lo():
    P, Hq, Hkv, D = 16, 8, 2, 128
    seq = [1000, 37, 600, 6404]
    lo = [0, 10, 599, 4000]
    npages = sum(-(-x // P) for x in seq) + 4
    kc = torch.randn(npages, Hkv, P, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(npages, Hkv, D, P, device="cuda", dtype=torch.bfloat16)
    perm = torch.randperm(npages, device="cuda").to(torch.int32)
    bt = torch.zeros(len(seq), npages, dtype=torch.int32, device="cuda")
    o = 0
    for b, L in enumerate(seq):
        n = -(-L // P)
        bt[b, :n] = perm[o:o + n]
        o += n
    sl = torch.tensor(seq, dtype=torch.int32, device="cuda")
    rl = torch.tensor(lo, dtype=torch.int32, device="cuda")
    q = torch.randn(len(seq), Hq, D, device="cuda", dtype=torch.bfloat16)
    want = ref.paged_decode(q, kc, vc, bt, sl, D ** -0.5, row_lo=rl)
    for parts in (8192, 512):
        ws = ops.DecodeWorkspace(len(seq), Hq, D, 8192, parts, "cuda")
        got = ops.paged_decode(q, kc, vc, bt, sl, D ** -0.5, ws, row_lo=rl)
        assert (got.float() - want.float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("case", list(CASES))
def test_mllama_on_gpu(tmp_path, case):
    hf = _hf(tmp_path)
    ids, n_img = CASES[case]
    imgs = _images()[:n_img]
    inputs = _hf_inputs(ids, imgs)
    with torch.no_grad():
        want = hf(**inputs).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=8, context_length=512))
    assert eng.runner.use_graph
    p = SamplingParams(max_new_tokens=10, ignore_eos=True)
    req = eng.make_mm_request(ids, imgs, p) if imgs else eng.make_request(ids, p)
    got = _prefill_logits(eng, ids, req.mm).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    # bf16 vision tower + a 15-key cross-attention row (image-token row of the first image) sit
    # at ~0.984; the fp32 CPU test pins the semantics exactly
    assert cos.min().item() > 0.98 and cos.mean().item() > 0.995, cos
    eng.add_request(req)
    while not req.finished:
        eng.step()
    seq = ids + req.output_ids
    full = _prefill_logits(eng, seq[:-1], req.mm).float().argmax(-1).cpu().tolist()[-10:]
    assert sum(int(a == b) for a, b in zip(full, req.output_ids)) >= 8, (full, req.output_ids)
