"""Pipeline parallelism on CPU (gloo): PP=2 and TP=2 x PP=2 engines must generate exactly what a
single rank generates from the same HF checkpoint (layer slicing per stage, stage hand-off of
(hidden, residual), last-stage sampling broadcast back, per-stage KV caches)."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from ome_amd.models import build_model
from ome_amd.models.config import PRESETS, ModelConfig
from tests.test_tp_cpu import PROMPTS, _export_dense


def _worker(rank, world, tp, pp, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model_path=path, tp_size=tp, pp_size=pp, device="cpu", max_running_requests=8,
                            context_length=256, dtype="float32"))
    assert len(eng.runner.model.layers) == 4 // pp
    assert sum(t is not None for t in eng.runner.kv.k) == 4 // pp
    if rank == 0:
        out = [r.output_ids for r in eng.generate(PROMPTS, SamplingParams(max_new_tokens=10, ignore_eos=True))]
        eng.stop_group()
        q.put(out)
    else:
        eng.run_forever()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("tp,pp", [(1, 2), (2, 2)])
def test_pp_matches_single(tmp_path, tp, pp):
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
    ps = [ctx.Process(target=_worker, args=(r, world, tp, pp, port, str(tmp_path), q)) for r in range(world)]
    for p in ps:
        p.start()
    got = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want
