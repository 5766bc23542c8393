"""DP attention + expert parallelism on the GPU with the low-latency EP exchange: 2 ranks share
GPU 0 (hipIpc peer mappings stand in for xGMI), each schedules its own requests, MoE rows travel
through the device-only dispatch / combine (csrc/comm/ep_ll.hip) and the decode steps replay
HIP graphs (captured with the exchange inside).  Greedy tokens must match one rank holding every
expert (bf16 tolerance: a token may flip late on a near-tie), for bf16 and fp8 experts."""
import json
import os
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp

from ome_amd.io.safetensors import save_file
from ome_amd.models import build_model
from ome_amd.models.config import PRESETS, ModelConfig

pytestmark = pytest.mark.gpu
PROMPTS = [[3 + (i * 37 + j) % 1000 for j in range(5 + 7 * i)] for i in range(6)]
NEW = 10


def _engine(path, world, quant, tbo=False):
    from ome_amd.runtime.engine import Engine, EngineArgs

    kw = dict(tp_size=world, dp_size=world, enable_dp_attention=True, enable_two_batch_overlap=tbo) \
        if world > 1 else {}
    return Engine(EngineArgs(model_path=path, device="cuda", max_running_requests=8, context_length=256,
                             max_total_tokens=4096, mem_fraction_static=0.3, cuda_graph=True, cuda_graph_max_bs=8,
                             quantization=quant, **kw))


def _worker(rank, world, port, path, quant, q, tbo=False):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(world), OME_DIST_BACKEND="gloo", OME_TUNE_GEMM="0")
        torch.cuda.set_device(0)
        from ome_amd.runtime.request import SamplingParams

        eng = _engine(path, world, quant, tbo)
        st = eng.pstate
        assert st.ep_ll is not None and eng.runner.use_graph and eng.runner.graphs
        assert eng.runner.tbo == tbo and (st.ep_ll_b is not None) == tbo
        if rank == 0:
            reqs = eng.generate(PROMPTS, SamplingParams(max_new_tokens=NEW, ignore_eos=True))
            owners = {r.dp_rank for r in reqs}
            eng.stop_group()
            err = st.ep_ll.error() | (st.ep_ll_b.error() if st.ep_ll_b is not None else 0)
            q.put((rank, [r.output_ids for r in reqs], owners, err, None))
        else:
            eng.run_forever()
            err = st.ep_ll.error() | (st.ep_ll_b.error() if st.ep_ll_b is not None else 0)
            q.put((rank, None, None, err, None))
    except Exception:  # noqa: BLE001
        q.put((rank, None, None, None, traceback.format_exc()))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("quant,tbo", [(None, False), ("fp8", False), (None, True)])
def test_dp_attention_low_latency_ep_graphs(tmp_path, quant, tbo):
    """tbo: two-batch overlap -- each decode step as two half batches on two streams through two
    exchanges (captured in the graphs), prefill / idle steps joining B's exchanges; same tokens."""
    from tests.test_moe_cpu import _export_hf

    hf = dict(PRESETS["tiny-moe"])
    m = build_model(ModelConfig.from_hf(hf), "cpu", torch.float32, load_format="dummy", seed=5)
    _export_hf(m, tmp_path, "qwen3")
    (tmp_path / "config.json").write_text(json.dumps(hf))
    del m
    os.environ["OME_TUNE_GEMM"] = "0"
    from ome_amd.runtime.request import SamplingParams

    single = _engine(str(tmp_path), 1, quant)
    want = [r.output_ids for r in single.generate(PROMPTS, SamplingParams(max_new_tokens=NEW, ignore_eos=True))]
    del single
    torch.cuda.empty_cache()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    env_keep = dict(os.environ)
    ps = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), quant, q, tbo)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(2):
            rank, out, owners, err, tb = q.get(timeout=500)
            assert tb is None, f"rank {rank}:\n{tb}"
            assert err == 0, f"rank {rank}: EP error word {err}"
            res[rank] = (out, owners)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
        os.environ.clear()
        os.environ.update(env_keep)
    got, owners = res[0]
    assert owners == {0, 1}
    matched = total = 0
    for w, g in zip(want, got):
        k = 0
        while k < len(w) and k < len(g) and w[k] == g[k]:
            k += 1
        assert k >= 3, f"diverged at {k}: {g} vs {w}"
        matched += k
        total += len(w)
    assert matched >= 0.8 * total
