"""PD disaggregation over the same-node xGMI/IPC fast path (csrc/comm/kvlink.hip): a decode engine
in another process exports its landing pool, the prefill engine writes each prompt's KV pages
straight into it from its GPU.  On the one-GPU test box both processes share the device, which
exercises the same hipIpc export / open / remote-store path as two GPUs of one node."""
import multiprocessing as mp
import time

import pytest

pytestmark = pytest.mark.gpu

PROMPTS = [[5 + (i * 7 + j) % 900 for j in range(20 + 37 * i)] for i in range(4)]
NEW = 10


def _decode_proc(q_in, q_out):
    import os

    os.environ.setdefault("OME_PD_LANDING_TOKENS", "4096")
    from ome_amd.runtime.disagg import attach_kv_transfer
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model="tiny-llama", device="cuda", max_running_requests=8, context_length=512, seed=0))
    kt = attach_kv_transfer(eng, "decode", 0)
    assert kt.landing is not None, "landing pool must be exported on a GPU"
    q_out.put(("port", kt.port))
    rooms = q_in.get(timeout=300)
    reqs = []
    for room, p in rooms:
        b = {"room": room, "bootstrap_room": room, "disagg_role": "decode"}
        reqs.append(eng.add_request(eng.make_request(p, SamplingParams(max_new_tokens=NEW, ignore_eos=True),
                                                     bootstrap=b)))
    deadline = time.time() + 120
    while any(not r.finished for r in reqs) and time.time() < deadline:
        eng.step()
        time.sleep(0.001)
    q_out.put(("done", [r.output_ids for r in reqs], kt.ipc_received, eng.metrics.step_prefill.n))


def test_pd_ipc_handoff():
    from ome_amd.runtime.disagg import attach_kv_transfer
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    proc = ctx.Process(target=_decode_proc, args=(q_in, q_out), daemon=True)
    proc.start()
    try:
        tag, port = q_out.get(timeout=240)
        assert tag == "port"
        ref = Engine(EngineArgs(model="tiny-llama", device="cuda", max_running_requests=8, context_length=512, seed=0))
        want = [r.output_ids for r in ref.generate(PROMPTS, SamplingParams(max_new_tokens=NEW, ignore_eos=True))]
        del ref
        pre = Engine(EngineArgs(model="tiny-llama", device="cuda", max_running_requests=8, context_length=512, seed=0))
        kt = attach_kv_transfer(pre, "prefill", 0)
        rooms = [(7000 + i, p) for i, p in enumerate(PROMPTS)]
        q_in.put(rooms)
        preqs = []
        for room, p in rooms:
            b = {"room": room, "bootstrap_room": room, "bootstrap_host": "127.0.0.1", "bootstrap_port": port,
                 "disagg_role": "prefill"}
            preqs.append(pre.add_request(pre.make_request(p, SamplingParams(max_new_tokens=1, ignore_eos=True),
                                                          bootstrap=b)))
        deadline = time.time() + 120
        while any(not r.finished for r in preqs) and time.time() < deadline:
            pre.step()
            time.sleep(0.001)
        res = q_out.get(timeout=240)
        assert res[0] == "done"
        outs, ipc_received, dec_prefills = res[1], res[2], res[3]
        assert ipc_received == len(PROMPTS) and kt.ipc_sent == len(PROMPTS)
        assert dec_prefills == 0  # every prompt token arrived over xGMI, none recomputed
        assert all(len(o) == NEW for o in outs)
        assert [o[0] for o in outs] == [w[0] for w in want]  # first token: sampled by the prefill engine
        agree = sum(a == b for o, w in zip(outs, want) for a, b in zip(o, w))
        assert agree >= 0.8 * NEW * len(PROMPTS), (outs, want)
    finally:
        proc.join(timeout=30)
        if proc.is_alive():
            proc.kill()
