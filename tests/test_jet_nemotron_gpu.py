"""Jet-Nemotron on gfx950 (bf16): prefill logits through ome_dyn_conv1d + ome_gdn_scan + the paged
attention kernels track the fp32 restatement of tests/test_jet_nemotron_cpu.py; the dynamic conv
kernel matches its fp32 reference bit-for-bit in structure (per-channel and per-head taps, state
carried across chunks)."""
import pytest
import torch

from ome_amd import ops
from ome_amd.models.common import AttnMeta
from ome_amd.ops import reference as ref
from ome_amd.runtime.engine import Engine, EngineArgs
from tests.test_jet_nemotron_cpu import IDS, _checkpoint, _ref_logits

pytestmark = pytest.mark.gpu


def _prefill_logits(eng, ids):
    run = eng.runner
    slot = run.slots.alloc()
    pages = run.pages.alloc(-(-len(ids) // run.P))
    run.slots.set_pages(slot, 0, pages)
    run.slots.flush()
    t = lambda a: torch.tensor(a, dtype=torch.int32, device=run.device)  # noqa: E731
    n = len(ids)
    rng = list(range(n))
    meta = AttnMeta("prefill", t(rng), t([pages[x // run.P] * run.P + x % run.P for x in rng]),
                    run.slots.table.index_select(0, t([slot])), cu_q=t([0, n]), kv_lens=t([n]),
                    items=t(ops.prefill_work_items([n], [n])).view(-1, 2))
    meta.extra["ssm"] = (t([0, n]), t([slot]), t([1]))
    out = run.model.compute_logits(run.model.forward(t(ids), meta, run.kv)).float()
    run.pages.free(pages)
    run.slots.free(slot)
    return out


def test_jet_nemotron_bf16_on_gpu(tmp_path):
    w = _checkpoint(tmp_path)
    want = _ref_logits(w, IDS)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", dtype="bfloat16", max_running_requests=2,
                            context_length=256, cuda_graph=False))
    got = _prefill_logits(eng, IDS).cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    # bf16 through two recurrences (conv window + delta-rule state) per JetBlock: the worst row of
    # the 23 measured 0.992 against the fp32 restatement
    assert cos.min().item() > 0.985 and cos.mean().item() > 0.995, cos
    assert (got.argmax(-1) == want.argmax(-1)).float().mean().item() > 0.9


@pytest.mark.parametrize("cpk", [1, 64])
def test_dyn_conv1d_kernel(cpk):
    torch.manual_seed(0)
    T, C, K = 77, 384, 4
    x = torch.randn(T, C + 8, device="cuda").to(torch.bfloat16)[:, :C]
    taps = torch.randn(T, (C // cpk) * K, device="cuda").to(torch.bfloat16)
    cu = torch.tensor([0, 5, 6, 77], dtype=torch.int32, device="cuda")
    slot = torch.tensor([2, 0, 3], dtype=torch.int32, device="cuda")
    reset = torch.tensor([1, 0, 0], dtype=torch.int32, device="cuda")
    st0 = (torch.randn(4, C, K - 1, device="cuda") * 0.5).to(torch.bfloat16)
    st_k, st_r = st0.clone(), st0.clone().cpu()
    y = ops.dyn_conv1d(x, taps, st_k, cu, slot, reset, cpk)
    yr = ref.dyn_conv1d(x.cpu(), taps.cpu(), st_r, cu.cpu(), slot.cpu(), reset.cpu(), cpk,
                        torch.empty(T, C, dtype=torch.bfloat16))
    assert (y.float().cpu() - yr.float()).abs().max().item() < 3e-2
    assert torch.equal(st_k.cpu(), st_r) and torch.equal(st_k[1].cpu(), st0[1].cpu())
