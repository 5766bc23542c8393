"""Low-latency expert parallelism (csrc/comm/ep_ll.hip): N processes share GPU 0 through hipIpc
mappings, each with its own tokens and 1/N of the experts; the device-only dispatch / combine
must reproduce a single process running every expert -- eagerly and replayed from a captured
HIP graph (no host sync on split counts), for bf16 and fp8 experts, with skewed routing."""
import os
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

E, H, I, K, T = 16, 512, 256, 4, 24


def _data(rank, it):
    g = torch.Generator().manual_seed(100 * rank + it)
    x = torch.randn(T, H, generator=g).to(torch.bfloat16)
    logits = torch.randn(T, E, generator=g)
    if it % 2:   # skew: most tokens pick experts of rank 0
        logits[:, :E // 2] += 3.0
    return x, logits


def _weights():
    g = torch.Generator().manual_seed(7)
    w13 = (torch.randn(E, 2 * I, H, generator=g) * H ** -0.5).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, generator=g) * I ** -0.5).to(torch.bfloat16)
    return w13, w2


def _worker(rank, world, port, fp8, q):
    try:
        import torch.distributed as dist

        from ome_amd import ops
        from ome_amd.models.quant import quantize_experts
        from ome_amd.parallel.ep_ll import LowLatencyEP

        dev_i = rank % torch.cuda.device_count() if os.environ.get("OME_TEST_SPREAD") == "1" else 0
        torch.cuda.set_device(dev_i)   # spread: one rank per GPU over xGMI; else all ranks share GPU 0
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        dev = torch.device("cuda", dev_i)
        w13, w2 = (w.to(dev) for w in _weights())
        el = E // world
        loc13, loc2 = w13[rank * el:(rank + 1) * el].contiguous(), w2[rank * el:(rank + 1) * el].contiguous()
        if fp8:
            full13, full2 = quantize_experts(w13), quantize_experts(w2)
            loc13, loc2 = quantize_experts(loc13), quantize_experts(loc2)
        else:
            full13, full2 = w13, w2
        ep = LowLatencyEP(None, H, T, K)
        worst = 0.0
        for it in range(4):
            x, logits = (t.to(dev) for t in _data(rank, it))
            tw, tid = ops.moe_route(logits, K)
            got = ep.forward(x, tw, tid, loc13, loc2, 0, 1.0, el)
            want = ops.fused_moe(x, tw, tid, full13, full2, 0, 1.0)
            worst = max(worst, ((got.float() - want.float()).abs().max() / (want.float().abs().max() + 1e-6)).item())
        # captured: static input buffers, replayed with new contents
        xs = torch.zeros(T, H, dtype=torch.bfloat16, device=dev)
        ls = torch.zeros(T, E, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            tw, tid = ops.moe_route(ls, K)
            ep.forward(xs, tw, tid, loc13, loc2, 0, 1.0, el)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            tw, tid = ops.moe_route(ls, K)
            gout = ep.forward(xs, tw, tid, loc13, loc2, 0, 1.0, el)
        dist.barrier()
        for it in range(4, 7):
            x, logits = (t.to(dev) for t in _data(rank, it))
            xs.copy_(x)
            ls.copy_(logits)
            g.replay()
            torch.cuda.synchronize()
            twr, tidr = ops.moe_route(logits, K)
            want = ops.fused_moe(x, twr, tidr, full13, full2, 0, 1.0)
            worst = max(worst, ((gout.float() - want.float()).abs().max() / (want.float().abs().max() + 1e-6)).item())
            dist.barrier()
        q.put((rank, worst, ep.error(), None))
        dist.barrier()
        ep.close()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        q.put((rank, None, None, traceback.format_exc()))


def _free_port():
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


@pytest.mark.parametrize("world,fp8", [(2, False), (4, False), (2, True)])
def test_low_latency_ep_matches_single_rank(world, fp8):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env_keep = dict(os.environ)
    procs = [ctx.Process(target=_worker, args=(r, world, port, fp8, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(world):
            res.append(q.get(timeout=300))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        os.environ.clear()
        os.environ.update(env_keep)
    for rank, worst, err, tb in res:
        assert tb is None, tb
        assert err == 0, f"rank {rank}: error word {err}"
        assert worst < 2e-2, f"rank {rank}: rel err {worst}"


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs (xGMI peers)")
@pytest.mark.parametrize("fp8", [False, True])
def test_low_latency_ep_across_devices(monkeypatch, fp8):
    """Low-latency EP dispatch / combine with one rank per GPU (peer buffers over xGMI)."""
    monkeypatch.setenv("OME_TEST_SPREAD", "1")
    test_low_latency_ep_matches_single_rank(min(4, torch.cuda.device_count()), fp8)
