#!/usr/bin/env python3
"""Per-call latency of the device-side collectives, N ranks sharing ONE GPU through hipIpc
mappings (the 1-GPU box; across 8 MI355X the same protocol runs over xGMI peers):

* custom all-reduce (csrc/comm/allreduce.hip), 8 KiB .. 16 MiB bf16, one-shot / two-shot by size;
* fused all-reduce + residual add + RMSNorm, input produced straight into the IPC staging
  buffer (rows x 4096, the Llama TP layer epilogue);
* low-latency EP dispatch + expert GEMMs + combine per MoE layer (csrc/comm/ep_ll.hip),
  DeepSeek-like routing (top-8 of 256 experts is scaled down to top-8 of 32 experts, H 2048).

Each number is a HIP-graph replay of 20 back-to-back calls, averaged, max over ranks.
Sharing one GPU means every rank's kernels contend for the same CUs and HBM: the numbers are
protocol + kernel latency on one device, not xGMI link numbers.

Usage: python scripts/comm_latency_bench.py [world] > profiles/...txt
"""
import os
import socket
import sys
import traceback

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REPS = 20


def _graph_time(fn, dist, align=None):
    """us per call of ``fn`` over REPS graph-captured calls, max over ranks.  ``align``: a device-side
    rendezvous (one custom all-reduce) enqueued right before the start event, so every rank's timer
    starts at the same device moment.  Without it the host-side gloo barrier leaves the ranks'
    replays up to ~1 ms apart and the early rank's first collective absorbs that skew (the round
    3-5 "32 KiB outlier", see OME_AR_ORDER_PROBE)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(REPS):
            fn()
    dist.barrier()
    g.replay()  # warm replay (every rank replays: the collectives rendezvous on device flags)
    torch.cuda.synchronize()
    dist.barrier()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if align is not None:
        align()
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    t = a.elapsed_time(b) * 1000 / (3 * REPS)
    out = torch.tensor([t])
    dist.all_reduce(out, op=dist.ReduceOp.MAX)
    return out.item()


def _worker(rank, world, port, q):
    try:
        import torch.distributed as dist

        from ome_amd import ops
        from ome_amd.parallel.comm import CustomAllReduce
        from ome_amd.parallel.ep_ll import LowLatencyEP

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        ar = CustomAllReduce(None, max_bytes=32 << 20)
        tiny = torch.zeros(64, device=dev, dtype=torch.bfloat16)
        align = None if os.environ.get("OME_AR_ALIGN", "1") == "0" else (lambda: ar.all_reduce(tiny))
        rows = []
        if os.environ.get("OME_AR_ORDER_PROBE") == "1":
            # the same sizes at several table positions, with the host-barrier-only start (as rounds
            # 3-5 measured) and with the device-aligned start
            import time as _t
            for mode, al in (("host-barrier start", None), ("device-aligned start", align)):
                for pos, kib in enumerate((8, 32, 128, 32, 8, 32, 2048, 32)):
                    n = kib * 1024 // 2
                    x = torch.randn(n, device=dev).to(torch.bfloat16)
                    t0 = _t.perf_counter()
                    t = _graph_time(lambda: ar.all_reduce(x), dist, al)
                    rows.append(f"order-probe {mode:22s} pos {pos} {kib:6d} KiB  {t:8.1f} us  "
                                f"(rank{rank} host {1e3 * (_t.perf_counter() - t0):.1f} ms)")
        for kib in (8, 32, 128, 512, 2048, 8192, 16384):
            n = kib * 1024 // 2
            x = torch.randn(n, device=dev).to(torch.bfloat16)
            t = _graph_time(lambda: ar.all_reduce(x), dist, align)
            rows.append(f"all_reduce        {kib:6d} KiB  {t:8.1f} us  {2 * (world - 1) / world * kib / 1024 / t * 1e6 / 1024:6.2f} GB/s busbw")
        if os.environ.get("OME_AR_GRID_SWEEP") == "1":   # one-shot grid sizing: vectors per lane
            for vpt in (1, 2, 4):
                ar.vpt = vpt
                for kib in (8, 16, 24, 32, 48, 64, 96, 128, 256, 512):
                    n = kib * 1024 // 2
                    x = torch.randn(n, device=dev).to(torch.bfloat16)
                    t = _graph_time(lambda: ar.all_reduce(x), dist, align)
                    rows.append(f"one-shot vpt={vpt} grid={ar._grid(n, False):3d} {kib:5d} KiB  {t:8.1f} us")
            ar.vpt = 0
        for r in (1, 16, 32, 64):
            H = 4096
            st = ar.staging((r, H))
            st.copy_(torch.randn(r, H, device=dev).to(torch.bfloat16))
            res = torch.randn(r, H, device=dev).to(torch.bfloat16)
            w = torch.ones(H, device=dev, dtype=torch.bfloat16)
            t = _graph_time(lambda: ar.all_reduce_add_rmsnorm(st, res, w, 1e-5), dist, align)
            rows.append(f"ar+add+rmsnorm    {r:4d} x {H}  {t:8.1f} us  ({r * H * 2 // 1024} KiB)")
        E, H, I, K = 32, 2048, 512, 8
        el = E // world
        g = torch.Generator().manual_seed(7)
        w13 = (torch.randn(el, 2 * I, H, generator=g) * H ** -0.5).to(torch.bfloat16).to(dev)
        w2 = (torch.randn(el, H, I, generator=g) * I ** -0.5).to(torch.bfloat16).to(dev)
        for T in (1, 16, 64, 128):
            ep = LowLatencyEP(None, H, T, K)
            x = torch.randn(T, H, device=dev).to(torch.bfloat16)
            logits = torch.randn(T, E, device=dev)
            tw, tid = ops.moe_route(logits, K)
            t = _graph_time(lambda: ep.forward(x, tw, tid, w13, w2, 0, 1.0, el), dist, align)
            rows.append(f"ep_ll layer       T={T:4d} top{K}/{E} H{H}  {t:8.1f} us (dispatch + experts + combine)")
            t = _graph_time(lambda: ep.forward(x, tw, tid, None, None, 0, 1.0, el), dist, align)
            rows.append(f"ep_ll exchange    T={T:4d} top{K}/{E} H{H}  {t:8.1f} us (dispatch + combine, no experts)")
            rt = torch.randn(T * K, H, device=dev).to(torch.bfloat16)
            rid = torch.randint(0, el, (T * K,), device=dev, dtype=torch.int32)
            t = _graph_time(lambda: ops.moe_experts_sorted(rt, rid, w13, w2, 0, el), dist, align)
            rows.append(f"experts only      T={T:4d} top{K}/{E} H{H}  {t:8.1f} us (align + 2 grouped GEMMs + act)")
            dist.barrier()
            ep.close()
        q.put((rank, rows, None))
        dist.barrier()
        ar.close()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        q.put((rank, None, traceback.format_exc()))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    bad = [(rank, tb) for rank, _rows, tb in sorted(res, key=lambda r: r[0]) if tb]
    for rank, tb in bad:
        print(f"rank {rank} failed:\n{tb}")
    if bad:
        sys.exit(1)
    print(f"# world={world} ranks on one MI355X (hipIpc peers), HIP-graph replay of {REPS} calls, max over ranks, "
          f"timers started {'after a device-side rendezvous' if os.environ.get('OME_AR_ALIGN', '1') != '0' else 'after a host barrier only'}")
    for line in res[0][1] if res[0][0] == 0 else sorted(res)[0][1]:
        print(line)


if __name__ == "__main__":
    main()
