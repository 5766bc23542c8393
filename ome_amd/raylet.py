"""Ray-contract node agent for MultiNodeRayVLLM deployments (reference:
``pkg/controller/v1beta1/inferenceservice/reconcilers/multinodevllm/ray.go``,
``dockerfiles/lws-vllm/ray_init.sh``).

The reference runs vLLM on a KubeRay cluster: the head pod starts ``ray start --head`` and then
``vllm serve ... --distributed-executor-backend ray``; worker pods run ``ray start
--address=<head>:6379 --block`` and the engine places its TP / PP ranks on them through Ray.
Ray is not part of this image, and the serving engine here is multi-process
``torch.distributed`` (one process per GPU, RCCL over xGMI) -- so this module implements the
same *contract* with a rendezvous store instead of a Ray cluster:

* ``python -m ome_amd.raylet start --head [--port=6379]`` holds a TCP key-value store on the
  head (the "GCS"); ``start --address=H:P --block`` on a worker registers the node, waits for
  the head engine's launch record and then runs ``ome_amd.runtime.server`` as node ``r`` of the
  group (``--nnodes / --node-rank / --dist-init-addr``), for as long as the head engine lives;
* ``ome_amd.runtime.server --distributed-executor-backend ray`` on the head (the translated
  ``vllm serve``) sizes the group from TP x PP and the GPUs per node, publishes its arguments
  and the engine rendezvous port in the store, and runs as node 0;
* ``ray_init.sh leader|worker`` (the LWS-vLLM image script) map onto the same commands;
  ``ray stop`` is a no-op (the executor stops the processes).

The executor's command translation (``executor/kubelet.py``) rewrites ``ray start`` / ``ray stop``
/ ``ray_init.sh`` to this module, so reference-style RayCluster pods run unchanged.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from datetime import timedelta

ARGV_KEY, PORT_KEY, ALIVE_KEY, RANK_KEY = "ome/argv", "ome/dist_port", "ome/alive", "ome/rank"
DEFAULT_PORT = 6379


def _store(host: str, port: int, master: bool, timeout_s: float = 300.0):
    from torch.distributed import TCPStore

    return TCPStore(host, port, is_master=master, wait_for_workers=False, timeout=timedelta(seconds=timeout_s))


def _split(addr: str) -> tuple[str, int]:
    host, _, port = addr.rpartition(":")
    return (host or "127.0.0.1"), int(port or DEFAULT_PORT)


def head_address() -> str:
    """Where the Ray head's store listens (``RAY_ADDRESS`` as Ray itself reads it)."""
    a = os.environ.get("OME_RAY_ADDRESS") or os.environ.get("RAY_ADDRESS") or f"127.0.0.1:{DEFAULT_PORT}"
    return a[len("ray://"):] if a.startswith("ray://") else a


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("", 0))
        return s.getsockname()[1]


def connect_or_host(addr: str, timeout_s: float = 300.0):
    """Client of the head's store when ``start --head`` already runs it, else host it here."""
    host, port = _split(addr)
    try:
        return _store(host, port, False, timeout_s=2.0)
    except Exception:  # noqa: BLE001 -- nothing listening: this process becomes the head store
        return _store(host, port, True, timeout_s=timeout_s)


def publish_launch(store, argv: list[str], nnodes: int) -> str:
    """Head engine: record the worker launch (arguments + engine rendezvous port); returns the
    port part of ``--dist-init-addr`` (workers pair it with the head host they already know)."""
    port = _free_port()
    store.set(PORT_KEY, str(port))
    store.set(ARGV_KEY, json.dumps({"argv": argv, "nnodes": nnodes}))
    return str(port)


def wait_for_workers(store, n: int, timeout_s: float) -> bool:
    t0 = time.time()
    while time.time() - t0 < timeout_s:
        if int(store.add(ALIVE_KEY, 0)) >= n:
            return True
        time.sleep(0.5)
    return False


def run_worker(addr: str, block: bool = True, timeout_s: float = 600.0) -> int:
    """Register with the head, wait for the engine's launch record, run this node's ranks."""
    host, port = _split(addr)
    deadline = time.time() + timeout_s
    store = None
    while store is None:
        try:
            store = _store(host, port, False, timeout_s=timeout_s)
        except Exception:  # noqa: BLE001 -- head not up yet: retry like `ray start` does
            if time.time() > deadline:
                print(f"raylet: head {addr} unreachable", file=sys.stderr)
                return 1
            time.sleep(1.0)
    store.add(ALIVE_KEY, 1)
    if not block:
        return 0
    store.wait([ARGV_KEY], timedelta(seconds=max(1.0, deadline - time.time())))
    rec = json.loads(store.get(ARGV_KEY))
    rank = int(store.add(RANK_KEY, 1))   # nodes 1 .. nnodes-1 in arrival order
    if rank >= int(rec["nnodes"]):
        print(f"raylet: node {rank} is beyond the engine's {rec['nnodes']} nodes; idle", file=sys.stderr)
        while True:
            time.sleep(3600)
    dist = f"{host}:{store.get(PORT_KEY).decode()}"
    argv = list(rec["argv"]) + ["--nnodes", str(rec["nnodes"]), "--node-rank", str(rank), "--dist-init-addr", dist]
    if os.environ.get("OME_RAY_WORKER_PORT"):
        argv += ["--port", os.environ["OME_RAY_WORKER_PORT"]]
    return subprocess.call([sys.executable, "-m", "ome_amd.runtime.server", *argv])


def _parse_kv(args: list[str]) -> dict:
    out = {}
    for a in args:
        if a.startswith("--") and "=" in a:
            k, v = a[2:].split("=", 1)
            out[k.replace("-", "_")] = v
    return out


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__)
        return 2
    cmd, rest = argv[0], argv[1:]
    if cmd == "stop":
        return 0
    if cmd == "start":
        ap = argparse.ArgumentParser(prog="ome_amd.raylet start")
        ap.add_argument("--head", action="store_true")
        ap.add_argument("--address", default=None)
        ap.add_argument("--port", type=int, default=DEFAULT_PORT)
        ap.add_argument("--block", action="store_true")
        ns, _unknown = ap.parse_known_args(rest)   # Ray's other start flags (dashboard, resources) don't apply
        if ns.head:
            addr = f"127.0.0.1:{ns.port}"
            if not ns.block:   # hold the store in a detached child, as `ray start --head` leaves daemons
                subprocess.Popen([sys.executable, "-m", "ome_amd.raylet", "start", "--head", f"--port={ns.port}",
                                  "--block"], start_new_session=True, stdout=subprocess.DEVNULL,
                                 stderr=subprocess.DEVNULL)
                for _ in range(100):   # return once the store answers
                    try:
                        _store("127.0.0.1", ns.port, False, timeout_s=1.0)
                        return 0
                    except Exception:  # noqa: BLE001
                        time.sleep(0.1)
                return 1
            st = _store("127.0.0.1", ns.port, True)   # held for the life of this process
            print(f"raylet: head store at {addr}", flush=True)
            while st is not None:
                time.sleep(3600)
            return 0
        if not ns.address:
            print("raylet start: --head or --address required", file=sys.stderr)
            return 2
        return run_worker(ns.address if ":" in ns.address else f"{ns.address}:{ns.port}", ns.block)
    if cmd in ("init", "ray_init.sh"):   # the LWS-vLLM image's ray_init.sh leader|worker contract
        sub, kv = (rest[0] if rest else ""), _parse_kv(rest[1:])
        port = int(kv.get("ray_port", DEFAULT_PORT))
        timeout = float(kv.get("ray_init_timeout", 300))
        if sub == "worker":
            return run_worker(f"{kv['ray_address']}:{port}", True, timeout)
        if sub == "leader":
            rc = main(["start", "--head", f"--port={port}"])
            if rc:
                return rc
            st = _store("127.0.0.1", port, False)
            ok = wait_for_workers(st, int(kv["ray_cluster_size"]) - 1, timeout)
            print("All ray workers are active" if ok else "Ray cluster initialisation timed out", flush=True)
            return 0 if ok else 1
        print(f"raylet init: unknown subcommand {sub!r}", file=sys.stderr)
        return 2
    print(f"raylet: unknown command {cmd!r}", file=sys.stderr)
    return 2


if __name__ == "__main__":
    sys.exit(main())
