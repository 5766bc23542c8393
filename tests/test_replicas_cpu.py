"""A job larger than one engine group holds several independent engine replicas (bench.py
``--gpus N --tp K``): 4 gloo ranks = two TP=2 engines, each must generate what a single engine
generates.  Also: ``bench.py --gpus N`` refuses to report N GPUs it does not have, and a rank
whose lockstep step fails takes its whole group down (fail-fast) instead of desynchronising it."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from ome_amd.models import build_model
from ome_amd.models.config import PRESETS, ModelConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROMPTS = [[3 + (i * 37 + j) % 1000 for j in range(9 + 11 * i)] for i in range(3)]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model_path=path, tp_size=2, device="cpu", max_running_requests=8,
                            context_length=256, dtype="float32"))
    st = eng.pstate
    assert st.world_size == 2 and st.replicas == world // 2 and st.rank == rank % 2
    if st.rank == 0:
        out = [r.output_ids for r in eng.generate(PROMPTS, SamplingParams(max_new_tokens=8, ignore_eos=True))]
        eng.stop_group()
        q.put((st.replica, out))
    else:
        eng.run_forever()


@pytest.mark.timeout(300)
def test_two_tp2_replicas_match_single(tmp_path):
    from tests.test_tp_cpu import _export_dense

    cfg = ModelConfig.from_hf(PRESETS["tiny-llama"])
    m = build_model(cfg, "cpu", torch.float32, load_format="dummy", seed=3)
    _export_dense(m, tmp_path)
    (tmp_path / "config.json").write_text(json.dumps(PRESETS["tiny-llama"]))
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    single = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", max_running_requests=8, context_length=256,
                               dtype="float32"))
    want = [r.output_ids for r in single.generate(PROMPTS, SamplingParams(max_new_tokens=8, ignore_eos=True))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 4, port, str(tmp_path), q)) for r in range(4)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: want, 1: want}


def test_bench_refuses_missing_gpus():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr
    assert '"n_gpus"' not in r.stdout


def _failing_worker(rank, world, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model_path=path, tp_size=2, device="cpu", max_running_requests=8,
                            context_length=256, dtype="float32"))
    if rank == 1:
        def boom(*a, **k):
            raise RuntimeError("injected step failure")
        eng.runner.launch = boom
        def fatal():
            q.put(("fatal", rank))
            q.close()
            q.join_thread()   # flush the queue's feeder thread before the process ends
        eng.on_fatal = fatal
        eng.run_forever()
    else:
        eng.add_request(eng.make_request(PROMPTS[0], SamplingParams(max_new_tokens=4, ignore_eos=True)))
        eng.step()
    os._exit(0)


@pytest.mark.timeout(300)
def test_failed_step_fails_the_group(tmp_path):
    from tests.test_tp_cpu import _export_dense

    cfg = ModelConfig.from_hf(PRESETS["tiny-llama"])
    m = build_model(cfg, "cpu", torch.float32, load_format="dummy", seed=3)
    _export_dense(m, tmp_path)
    (tmp_path / "config.json").write_text(json.dumps(PRESETS["tiny-llama"]))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_failing_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        ev = q.get(timeout=240)
        while ev != ("fatal", 1):
            ev = q.get(timeout=240)
    finally:
        for p in ps:   # the leader may still sit in the collective its peer left: end it here
            p.kill()
            p.join(timeout=30)
