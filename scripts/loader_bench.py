#!/usr/bin/env python3
"""Native loader throughput (libomeio: pread -> pinned staging -> hipMemcpyAsync into HBM).

Writes a synthetic Llama-3-70B-shaped checkpoint slice (``--layers`` decoder layers, bf16), evicts
it from the page cache (POSIX_FADV_DONTNEED; cold reads come from disk), then loads it
(1) whole, as TP=1 does, and (2) as every rank of TP=--tp with the rank-aware shard plan, and
prints GB/s of bytes read and the bytes each TP rank read relative to the whole checkpoint."""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd.io import native as nio  # noqa: E402
from ome_amd.io.safetensors import save_file  # noqa: E402
from ome_amd.models import build_model  # noqa: E402
from ome_amd.models.config import PRESETS, ModelConfig  # noqa: E402
from ome_amd.parallel import state as pstate  # noqa: E402


def evict(path):
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    finally:
        os.close(fd)


def _rank_load(r, tp, d, cfg_hf, start, q, ready, port=0):
    """One TP rank in its own process: wait for the common start, load its shard onto cuda:0.
    ``port``: join a gloo group of the tp ranks, so the loader's cooperative exchange
    (OME_LOAD_EXCHANGE, ome_amd.io.native.ShardExchange) can run over it."""
    try:
        cfg = ModelConfig.from_hf(cfg_hf)
        grp = None
        if port:
            import torch.distributed as dist

            dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=r, world_size=tp)
            grp = dist.group.WORLD
        pstate.set_state(pstate.ParallelState(tp_size=tp, tp_rank=r, world_size=tp, rank=r, backend="gloo",
                                              tp_cpu_group=grp))
        torch.cuda.init()
        torch.empty(1, device="cuda")
        ready.put(r)
        start.wait()
        b0 = nio.bytes_read()
        t = time.perf_counter()
        m = build_model(cfg, "cuda", torch.bfloat16, model_path=d, load_format="safetensors")
        torch.cuda.synchronize()
        q.put((r, time.perf_counter() - t, nio.bytes_read() - b0, None))
        del m
    except Exception as e:  # noqa: BLE001
        q.put((r, 0.0, 0, repr(e)))


def concurrent(tp, d, hf, shards, total, exchange=False):
    """All tp ranks loading their slices at once (one process each, all on GPU 0 here; one per
    GPU on a node) from a cold page cache: per-rank and aggregate GB/s.  ``exchange``: the ranks
    form a gloo group and read column shards / replicated tensors cooperatively."""
    import multiprocessing as mp
    import socket

    for f in shards:
        evict(f)
    port = 0
    if exchange:
        with socket.socket() as s_:
            s_.bind(("127.0.0.1", 0))
            port = s_.getsockname()[1]
    os.environ["OME_LOAD_EXCHANGE"] = "1" if exchange else "0"
    ctx = mp.get_context("spawn")
    start, q, ready = ctx.Event(), ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_rank_load, args=(r, tp, d, hf, start, q, ready, port)) for r in range(tp)]
    for p in ps:
        p.start()
    for _ in ps:   # every process imported torch and initialised the GPU before the common start
        ready.get(timeout=600)
    t0 = time.perf_counter()
    start.set()
    got = [q.get(timeout=600) for _ in ps]
    wall = time.perf_counter() - t0
    for p in ps:
        p.join(timeout=60)
    errs = [g for g in got if g[3]]
    if errs:
        raise RuntimeError(errs)
    nb = sum(g[2] for g in got)
    per = [g[2] / g[1] / 1e9 for g in got]
    print(f"concurrent tp={tp}{' +exchange' if exchange else ''}: {nb / 1e9:.2f} GB read by {tp} ranks in {wall:.2f}s "
          f"wall = {nb / wall / 1e9:.2f} GB/s "
          f"aggregate; per rank {min(per):.2f}-{max(per):.2f} GB/s (mean {sum(per) / len(per):.2f})", flush=True)
    return {"ranks": tp, "wall_s": round(wall, 3), "aggregate_GBps": round(nb / wall / 1e9, 2),
            "per_rank_GBps": [round(x, 2) for x in per], "bytes_total": int(nb), "checkpoint_bytes": int(total)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--concurrent", action="store_true", help="also load all TP ranks at once, one process each")
    a = ap.parse_args()
    hf = dict(PRESETS["llama-3-70b"])
    hf["num_hidden_layers"] = a.layers
    cfg = ModelConfig.from_hf(hf)
    d = a.dir or tempfile.mkdtemp(prefix="ome_loader_")
    H, D, I, V = cfg.hidden_size, cfg.head_dim, cfg.intermediate_size, cfg.vocab_size
    t0 = time.time()
    shards = []
    w = {"model.embed_tokens.weight": torch.empty(V, H, dtype=torch.bfloat16),
         "model.norm.weight": torch.ones(H, dtype=torch.bfloat16),
         "lm_head.weight": torch.empty(V, H, dtype=torch.bfloat16)}
    save_file(w, os.path.join(d, "model-00000.safetensors"))
    shards.append(os.path.join(d, "model-00000.safetensors"))
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        w = {p + "self_attn.q_proj.weight": torch.empty(cfg.num_heads * D, H, dtype=torch.bfloat16),
             p + "self_attn.k_proj.weight": torch.empty(cfg.num_kv_heads * D, H, dtype=torch.bfloat16),
             p + "self_attn.v_proj.weight": torch.empty(cfg.num_kv_heads * D, H, dtype=torch.bfloat16),
             p + "self_attn.o_proj.weight": torch.empty(H, cfg.num_heads * D, dtype=torch.bfloat16),
             p + "mlp.gate_proj.weight": torch.empty(I, H, dtype=torch.bfloat16),
             p + "mlp.up_proj.weight": torch.empty(I, H, dtype=torch.bfloat16),
             p + "mlp.down_proj.weight": torch.empty(H, I, dtype=torch.bfloat16),
             p + "input_layernorm.weight": torch.ones(H, dtype=torch.bfloat16),
             p + "post_attention_layernorm.weight": torch.ones(H, dtype=torch.bfloat16)}
        f = os.path.join(d, f"model-{i + 1:05d}.safetensors")
        save_file(w, f)
        shards.append(f)
    (open(os.path.join(d, "config.json"), "w")).write(json.dumps(hf))
    total = sum(os.path.getsize(f) for f in shards)
    print(f"# wrote {total / 1e9:.2f} GB ({a.layers} layers of Llama-3-70B) in {time.time() - t0:.1f}s", flush=True)
    res = {"checkpoint_gb": round(total / 1e9, 3), "layers": a.layers}
    for tp in (1, a.tp):
        per = []
        for r in range(tp):
            for f in shards:
                evict(f)
            pstate.set_state(pstate.ParallelState(tp_size=tp, tp_rank=r, world_size=tp, rank=r))
            b0 = nio.bytes_read()
            torch.cuda.synchronize()
            t = time.perf_counter()
            m = build_model(cfg, "cuda", torch.bfloat16, model_path=d, load_format="safetensors")
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            nb = nio.bytes_read() - b0
            per.append((dt, nb))
            del m
            torch.cuda.empty_cache()
            if tp > 1 and r >= 1:
                break   # ranks are symmetric; two cold loads are enough
        dt = sum(x[0] for x in per) / len(per)
        nb = sum(x[1] for x in per) / len(per)
        print(f"tp={tp}: {nb / 1e9:.2f} GB read per rank ({100 * nb / total:.1f}% of checkpoint) in {dt:.2f}s = "
              f"{nb / dt / 1e9:.2f} GB/s", flush=True)
        res[f"tp{tp}"] = {"bytes_per_rank": int(nb), "fraction": round(nb / total, 4), "seconds": round(dt, 3),
                          "GBps": round(nb / dt / 1e9, 2)}
    pstate.set_state(pstate.ParallelState())
    if a.concurrent:
        res[f"concurrent_tp{a.tp}"] = concurrent(a.tp, d, hf, shards, total)
        res[f"concurrent_tp{a.tp}_exchange"] = concurrent(a.tp, d, hf, shards, total, exchange=True)
    print(json.dumps(res))
    if not a.dir:
        for f in shards:
            os.unlink(f)


if __name__ == "__main__":
    main()
