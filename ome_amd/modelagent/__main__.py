"""Stand-alone model agent (reference ``cmd/model-agent/main.go``): one per node as a DaemonSet
(``config/model-agent/daemonset.yaml``).  It watches BaseModel / ClusterBaseModel through the
Kubernetes API (informer-backed :class:`~ome_amd.store.kube.KubeStore`), downloads artifacts into
``--models-root-dir``, keeps the node's model ConfigMap and labels, and serves ``/healthz`` and
``/metrics`` on ``--port``.  With ``--store-url`` it talks to an ome-amd manager's REST store
instead (single-node installs and tests)."""
from __future__ import annotations

import argparse
import logging
import os
import signal
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from ome_amd.api import constants as C

log = logging.getLogger("ome_amd.modelagent")

#: kinds the agent reads or writes (ConfigMap: per-node model status; Node: labels; Secret: storage keys)
AGENT_KINDS = [("ome.io/v1beta1", "BaseModel"), ("ome.io/v1beta1", "ClusterBaseModel"), ("v1", "ConfigMap"),
               ("v1", "Node"), ("v1", "Secret")]


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m ome_amd.modelagent", description=__doc__.split("\n")[0])
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME", ""))
    ap.add_argument("--models-root-dir", default=C.DEFAULT_MODEL_LOCAL_MOUNT_PATH)
    ap.add_argument("--port", type=int, default=8080, help="healthz / metrics port")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--num-download-worker", type=int, default=4)
    ap.add_argument("--download-retry", type=int, default=3)
    ap.add_argument("--configmap-heal-interval", type=float, default=300.0, help="seconds (reference: 5 min)")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--in-cluster", action="store_true")
    ap.add_argument("--namespace", default=C.OME_NAMESPACE, help="namespace of the per-node ConfigMaps")
    ap.add_argument("--startup-jitter", type=float, default=30.0,
                    help="spread agent start-up over [0, N) s by a hash of the node name (0 disables)")
    return ap


def make_handler(agent):
    from ome_amd.modelagent import metrics as M

    class H(BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            if self.path.startswith("/healthz") or self.path.startswith("/livez"):
                ok, msg = agent.healthz()
                body, code, ctype = msg.encode(), (200 if ok else 500), "text/plain"
            elif self.path.startswith("/metrics"):
                body, code, ctype = M.render(), 200, "text/plain; version=0.0.4"
            else:
                body, code, ctype = b"not found", 404, "text/plain"
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):  # quiet
            pass

    return H


def startup_jitter_s(node_name: str, span: float = 30.0) -> float:
    """Deterministic per-node start-up delay (reference cmd/model-agent/main.go:229-239: hash =
    hash*31 + c over the node name, delay = hash % 30 s) so a fleet of agents starting together
    does not hit the HF API at the same moment (429 storms)."""
    if span <= 0 or not node_name:
        return 0.0
    h = 0
    for c in node_name:   # Go int64 arithmetic: wraps on overflow
        h = ((h * 31 + ord(c) + (1 << 63)) % (1 << 64)) - (1 << 63)
    r = abs(h) % int(span) * (1 if h >= 0 else -1)   # Go's % truncates toward zero
    return float(max(0, r))                           # a negative delay sleeps for no time in Go


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    if not args.node_name:
        raise SystemExit("--node-name (or NODE_NAME) is required")
    from ome_amd.modelagent.agent import ModelAgent
    from ome_amd.store import kube

    client = kube.KubeClient.in_cluster() if args.in_cluster or not args.kubeconfig else \
        kube.KubeClient.from_kubeconfig(args.kubeconfig)
    delay = startup_jitter_s(args.node_name, args.startup_jitter)
    if delay:
        log.info("start-up jitter %.0f s before initialising the hub clients (rate-limit protection)", delay)
        time.sleep(delay)
    store = kube.KubeStore(client, AGENT_KINDS)
    agent = ModelAgent(store, args.node_name, args.models_root_dir, workers=args.num_download_worker,
                       download_retry=args.download_retry, heal_interval=args.configmap_heal_interval)
    agent.start()
    srv = ThreadingHTTPServer((args.host, args.port), make_handler(agent))
    stop = threading.Event()

    def _term(*_):
        stop.set()
        threading.Thread(target=srv.shutdown, daemon=True).start()

    signal.signal(signal.SIGTERM, _term)
    signal.signal(signal.SIGINT, _term)
    log.info("model agent on node %s, models under %s, healthz on :%d", args.node_name, args.models_root_dir,
             args.port)
    try:
        srv.serve_forever()
    finally:
        agent.stop()
        store.close() if hasattr(store, "close") else None
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
