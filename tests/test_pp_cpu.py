"""Pipeline parallelism on CPU (gloo): PP=2 and TP=2 x PP=2 engines must generate exactly what a
single rank generates from the same HF checkpoint (layer slicing per stage, stage hand-off of
(hidden, residual), last-stage sampling broadcast back, per-stage KV caches), with the step cut
into micro-batches that flow through the stages back to back (default: one per stage; 3 = an
uneven split; 1 = the whole step as one batch)."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from ome_amd.models import build_model
from ome_amd.models.config import PRESETS, ModelConfig
from tests.test_tp_cpu import PROMPTS, _export_dense


def _worker(rank, world, tp, pp, port, path, q, mb=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model_path=path, tp_size=tp, pp_size=pp, device="cpu", max_running_requests=8,
                            context_length=256, dtype="float32", pp_microbatches=mb))
    assert len(eng.runner.model.layers) == 4 // pp
    assert sum(t is not None for t in eng.runner.kv.k) == 4 // pp
    if rank == 0:
        out = [r.output_ids for r in eng.generate(PROMPTS, SamplingParams(max_new_tokens=10, ignore_eos=True))]
        eng.stop_group()
        q.put(out)
    else:
        eng.run_forever()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("tp,pp,mb", [(1, 2, 0), (2, 2, 0), (1, 2, 3)])
def test_pp_matches_single(tmp_path, tp, pp, mb):
    hf = dict(PRESETS["tiny-llama"], num_hidden_layers=4)
    cfg = ModelConfig.from_hf(hf)
    m = build_model(cfg, "cpu", torch.float32, load_format="dummy", seed=13)
    _export_dense(m, tmp_path)
    (tmp_path / "config.json").write_text(json.dumps(hf))
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    single = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", max_running_requests=8, context_length=256,
                               dtype="float32"))
    want = [r.output_ids for r in single.generate(PROMPTS, SamplingParams(max_new_tokens=10, ignore_eos=True))]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    world = tp * pp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, tp, pp, port, str(tmp_path), q, mb)) for r in range(world)]
    for p in ps:
        p.start()
    got = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want


def test_microbatch_split_keeps_order_and_balances_tokens():
    from ome_amd.runtime.model_runner import _split_balanced

    class C:
        def __init__(self, n):
            self.length = n

    for lens, m in (([1] * 10, 2), ([500, 1, 1, 1], 2), ([1, 1], 4), ([300, 300, 1, 1, 1], 3), ([7], 3)):
        cs = [C(n) for n in lens]
        g = _split_balanced(cs, m)
        assert [c for grp in g for c in grp] == cs and all(g) and len(g) == min(m, len(cs))
    g = _split_balanced([C(1) for _ in range(10)], 2)
    assert [len(x) for x in g] == [5, 5]
