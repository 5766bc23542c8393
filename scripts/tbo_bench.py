"""Two-batch overlap on/off: DP attention + expert parallelism over the low-latency IPC exchange,
2 ranks sharing GPU 0 (hipIpc mappings stand in for xGMI), DeepSeek-V2-Lite architecture
(random-init weights, --layers of its 27 decoder layers).  Rank 0 submits the prompts; the DP
engine spreads them over both ranks; decode steps replay HIP graphs (with TBO: each step = two
half batches on two streams through two exchanges).  Prints one line per mode: output tokens/s
of the whole 2-rank job and the mean decode step time.

    python scripts/tbo_bench.py [--layers 8] [--prompts 64] [--new 64]
"""
import argparse
import json
import os
import socket
import sys
import time
import traceback

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, world, port, a, tbo, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(world), OME_DIST_BACKEND="gloo",
                          OME_TUNE_GEMM="0", OME_KV_BUDGET_OWN="1")
        torch.cuda.set_device(0)
        from ome_amd.runtime.engine import Engine, EngineArgs
        from ome_amd.runtime.request import SamplingParams

        eng = Engine(EngineArgs(model=a.model, device="cuda", tp_size=world, dp_size=world, enable_dp_attention=True,
                                enable_two_batch_overlap=tbo, max_running_requests=a.prompts, context_length=1024,
                                mem_fraction_static=0.3, cuda_graph=True, cuda_graph_max_bs=a.prompts,
                                num_layers_override=a.layers))
        if rank == 0:
            prompts = [[3 + (i * 37 + j) % 5000 for j in range(32)] for i in range(a.prompts)]
            sp = SamplingParams(max_new_tokens=8, ignore_eos=True)
            eng.generate(prompts[:8], sp)   # warm-up
            torch.cuda.synchronize()
            t = time.perf_counter()
            reqs = eng.generate(prompts, SamplingParams(max_new_tokens=a.new, ignore_eos=True))
            dt = time.perf_counter() - t
            n = sum(len(r.output_ids) for r in reqs)
            eng.stop_group()
            q.put((rank, {"tbo": tbo, "tok_s": round(n / dt, 1), "seconds": round(dt, 3), "tokens": n,
                          "runner_tbo": eng.runner.tbo, "launches": dict(eng.runner.launch_stats)}, None))
        else:
            eng.run_forever()
            print(json.dumps({"rank": rank, "launches": dict(eng.runner.launch_stats)}), flush=True)
            q.put((rank, None, None))
    except Exception:  # noqa: BLE001
        q.put((rank, None, traceback.format_exc()))


def run(a, tbo):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, a, tbo, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = None
    try:
        for _ in range(2):
            rank, out, tb = q.get(timeout=900)
            if tb:
                raise RuntimeError(f"rank {rank}:\n{tb}")
            if out is not None:
                res = out
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="deepseek-v2-lite")
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--prompts", type=int, default=64)
    ap.add_argument("--new", type=int, default=64)
    ap.add_argument("--modes", default="off,on,off,on", help="comma list of off / on (one engine pair per entry)")
    ap.add_argument("--rank", type=int, default=-1,
                    help="run ONE rank in this process (MASTER_PORT from the env; the first --modes entry): "
                         "scripts/tbo_trace.sh starts each rank under its own rocprofv3")
    a = ap.parse_args()
    if a.rank >= 0:
        import queue

        q = queue.Queue()
        _worker(a.rank, 2, int(os.environ["MASTER_PORT"]), a, a.modes.split(",")[0].strip() == "on", q)
        rank, out, tb = q.get()
        if tb:
            sys.exit(f"rank {rank}:\n{tb}")
        if out is not None:
            print(json.dumps(out), flush=True)
        return
    for tbo in [m.strip() == "on" for m in a.modes.split(",")]:
        r = run(a, tbo)
        r.update(model=a.model, layers=a.layers, prompts=a.prompts, new_tokens=a.new,
                 setup="2 ranks sharing GPU 0, DP attention + EP over the IPC low-latency exchange, HIP graphs")
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
