"""Gemma 3 images on gfx950: the per-row visible-key limit (``row_hi``) of both MFMA prefill
kernels against the fp32 reference (sliding window on and off), and the SigLIP tower (head dim 72
on the varlen kernel) + bidirectional image blocks served in bf16 against transformers fp32."""
import pytest
import torch

from ome_amd import ops
from ome_amd.ops import reference as ref
from tests.test_kernels_gpu import DEV, _block_tables, _cache, _close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D,Hq,Hkv", [(128, 32, 8), (64, 8, 4)])   # prefill v2 (GQA-4, D 128) and v1
@pytest.mark.parametrize("window", [-1, 40])
def test_prefill_row_hi(D, Hq, Hkv, window):
    torch.manual_seed(D + window)
    P = 16
    q_lens, kv_lens = [37, 200, 1, 100], [37, 230, 300, 100]
    npages = sum(-(-L // P) for L in kv_lens) + 8
    kc, vc = _cache(npages, Hkv, D)
    bt = _block_tables(kv_lens, P, npages)
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens), dtype=torch.int32, device=DEV)
    q = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    hi = torch.full((sum(q_lens),), -1, dtype=torch.int32)
    # image-like blocks: rows of a block see up to the block's last key (absolute positions)
    for s, (a, n) in enumerate([(5, 20), (40, 64), (0, 0), (10, 50)]):
        pre = kv_lens[s] - q_lens[s]
        for r in range(a, a + n):
            hi[int(cu[s]) + r] = pre + a + n - 1
    hi = hi.to(DEV)
    got = ops.paged_prefill(q, kc, vc, bt, cu, kl, items, D ** -0.5, window, row_hi=hi)
    want = ref.paged_prefill(q, kc, vc, bt, cu, kl, D ** -0.5, window, row_hi=hi)
    _close(got, want, atol=2e-2)
    causal = ref.paged_prefill(q, kc, vc, bt, cu, kl, D ** -0.5, window)
    assert (want.float() - causal.float()).abs().max().item() > 1e-2   # the limit matters


def test_gemma3_vision_on_gpu(tmp_path):
    from ome_amd.models.gemma3_vision import preprocess_gemma3
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams
    from tests.test_gemma3_vision_cpu import BOI, SOFT, _hf_ids, _hf_model, _image

    hf = _hf_model(tmp_path)
    imgs = [_image(0), _image(1, 120, 60)]
    px = torch.cat([preprocess_gemma3(im, 112) for im in imgs])
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=512))
    m = eng.runner.model
    with torch.no_grad():
        want = hf.get_image_features(pixel_values=px, return_dict=True).pooler_output.reshape(-1, 256).float()
    got = m.encode_images(px).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.99, cos.min().item()
    req = eng.make_mm_request([2, 9, 17, BOI, 33, 41, BOI, 12, 7], imgs, SamplingParams(max_new_tokens=8,
                                                                                       ignore_eos=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    t = torch.tensor([_hf_ids(req)])
    with torch.no_grad():
        ref_ids = hf.generate(t, pixel_values=px, token_type_ids=(t == SOFT).long(), max_new_tokens=8,
                              do_sample=False)[0, t.shape[1]:].tolist()
    assert sum(int(a == b) for a, b in zip(req.output_ids, ref_ids)) >= 6, (req.output_ids, ref_ids)
