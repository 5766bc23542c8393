"""Local kubelet + scheduler + service proxy for a single MI355X node.

The reference control plane hands Pods to Kubernetes; this framework also has to *run* them
on a bare 8xMI355X box without a cluster.  The executor therefore plays:

* **scheduler** — binds Pending pods to a registered Node honouring ``nodeSelector``,
  required node affinity and ``amd.com/gpu`` requests; GPUs are allocated as concrete device
  indices (xGMI-adjacent contiguous ranges first) and exported as ``HIP_VISIBLE_DEVICES``;
* **kubelet** — runs init containers then containers as process groups
  (``start_new_session``) with k8s env semantics (``$(VAR)`` expansion, fieldRef, secret /
  configMap refs), volume path mapping (hostPath / emptyDir / configMap / PVC), container-port
  remapping (every pod shares the host network, so ``containerPort`` 8080 becomes a free host
  port substituted into ``--port``), startup / readiness / liveness probes (httpGet, tcpSocket,
  exec), restart policy with back-off and ``restartCount``/``lastState``, graceful termination;
* **kube-proxy + DNS** — every Service gets a local TCP proxy that balances over ready
  endpoints; ``<svc>.<ns>.svc.cluster.local`` names resolve through :mod:`ome_amd.executor.dns`.

Container images are mapped to this framework's entrypoints (``sglang.launch_server`` /
``vllm.entrypoints.openai.api_server`` -> :mod:`ome_amd.runtime.server`, ``genai-bench`` ->
:mod:`ome_amd.bench.loadgen`, ``multinode-prober`` -> :mod:`ome_amd.prober`, ``ome-agent`` ->
:mod:`ome_amd.agent`), so reference-style ClusterServingRuntimes run unchanged.

``simulate=True`` skips process launch (pods become Ready right after binding) for
control-plane tests — the analogue of envtest's fake kubelet.
"""
from __future__ import annotations

import json
import logging
import os
import re
import shlex
import signal
import socket
import subprocess
import sys
import threading
import time
import urllib.request
from dataclasses import dataclass, field

from ome_amd.api import constants as C
from ome_amd.store.store import Conflict, NotFound, Store, match_labels, now_iso
from ome_amd.utils.quantity import parse_quantity

log = logging.getLogger("ome_amd.executor")

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PY = sys.executable

# command / image translation to this framework's entrypoints.  Rewrites use a sentinel for the
# interpreter so later rules never re-match text an earlier rule produced.
_PYS = "\x00PY\x00"
_NB = r"(?<![\w/.\x00-])"
COMMAND_ALIASES = [
    (re.compile(_NB + r"python3?\s+-m\s+sglang\.launch_server\b"), f"{_PYS} -m ome_amd.runtime.server"),
    (re.compile(_NB + r"python3?\s+-m\s+vllm\.entrypoints\.openai\.api_server\b"), f"{_PYS} -m ome_amd.runtime.server"),
    (re.compile(_NB + r"vllm\s+serve\b"), f"{_PYS} -m ome_amd.runtime.server --model-path"),
    # SGLang diffusion CLI (the Qwen-Image runtimes): the diffusion server
    (re.compile(_NB + r"sglang\s+serve\b"), f"{_PYS} -m ome_amd.diffusion.server"),
    (re.compile(_NB + r"python3?\s+-m\s+sglang_router\.launch_router\b"), f"{_PYS} -m ome_amd.router"),
    (re.compile(_NB + r"genai-bench\b"), f"{_PYS} -m ome_amd.bench.loadgen"),
    (re.compile(_NB + r"multinode-prober\b"), f"{_PYS} -m ome_amd.prober"),
    (re.compile(_NB + r"ome-agent\b"), f"{_PYS} -m ome_amd.agent"),
    # Ray contract (MultiNodeRayVLLM): the rendezvous agent in place of a Ray cluster
    (re.compile(_NB + r"ray\s+(start|stop)\b"), f"{_PYS} -m ome_amd.raylet \\1"),
    (re.compile(r"(?:\S*/)?ray_init\.sh\b"), f"{_PYS} -m ome_amd.raylet init"),
    (re.compile(_NB + r"python3?(?=\s|$)"), _PYS),
]
_PEER_PORT_FLAGS = {"--service-discovery-port"}
IMAGE_ENTRYPOINTS = {  # image (substring) -> default argv when the container has no command
    "sglang": [PY, "-m", "ome_amd.runtime.server"],
    "vllm": [PY, "-m", "ome_amd.runtime.server"],
    "ome-runtime": [PY, "-m", "ome_amd.runtime.server"],
    "router": [PY, "-m", "ome_amd.router"],
    "genai-bench": [PY, "-m", "ome_amd.bench.loadgen"],
    "multinode-prober": [PY, "-m", "ome_amd.prober"],
    "ome-agent": [PY, "-m", "ome_amd.agent"],
    "model-agent": [PY, "-m", "ome_amd.modelagent"],
}

_VAR = re.compile(r"\$\(([A-Za-z_][A-Za-z0-9_]*)\)")


def expand_vars(s: str, env: dict) -> str:
    """Kubernetes ``$(VAR)`` expansion (``$$(VAR)`` escapes)."""
    out, i = [], 0
    while i < len(s):
        if s.startswith("$$(", i):
            out.append("$(")
            i += 3
            continue
        m = _VAR.match(s, i)
        if m and m.group(1) in env:
            out.append(str(env[m.group(1)]))
            i = m.end()
            continue
        out.append(s[i])
        i += 1
    return "".join(out)


def translate_command(text: str) -> str:
    for pat, rep in COMMAND_ALIASES:
        text = pat.sub(rep, text)
    return text.replace(_PYS, PY)


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def gpu_request(pod_spec: dict) -> int:
    n = 0
    for c in pod_spec.get("containers") or []:
        res = c.get("resources") or {}
        for part in ("limits", "requests"):
            for name in C.GPU_RESOURCE_NAMES:
                v = (res.get(part) or {}).get(name)
                if v is not None:
                    n = max(n, int(parse_quantity(v)))
    return n


# ------------------------------------------------------------------ node model
@dataclass
class NodeInfo:
    name: str
    gpus: int = 8
    labels: dict = field(default_factory=dict)
    gpu_product: str = "AMD_Instinct_MI355X"
    gpu_memory_gib: int = 288
    cpu: int = 0
    memory_gib: int = 0

    def to_object(self) -> dict:
        labels = {"kubernetes.io/hostname": self.name, C.NODE_INSTANCE_TYPE_LABEL: "BM.GPU.MI355X.8",
                  "amd.com/gpu.product-name": self.gpu_product, "amd.com/gpu.family": "CDNA4",
                  "amd.com/gpu.device-id": "75a3", "amd.com/gpu.vram": f"{self.gpu_memory_gib}G",
                  "amd.com/gpu.count": str(self.gpus), **self.labels}
        cpu = self.cpu or os.cpu_count() or 8
        mem = self.memory_gib or 64
        cap = {"cpu": str(cpu), "memory": f"{mem}Gi", C.AMD_GPU_RESOURCE: str(self.gpus), "pods": "110"}
        return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": self.name, "labels": labels},
                "spec": {}, "status": {"capacity": cap, "allocatable": dict(cap),
                                       "conditions": [{"type": "Ready", "status": "True", "reason": "KubeletReady",
                                                       "lastTransitionTime": now_iso()}],
                                       "addresses": [{"type": "InternalIP", "address": "127.0.0.1"},
                                                     {"type": "Hostname", "address": self.name}]}}


def node_affinity_ok(pod_spec: dict, node: dict) -> bool:
    labels = node["metadata"].get("labels") or {}
    for k, v in (pod_spec.get("nodeSelector") or {}).items():
        if labels.get(k) != v:
            return False
    req = (((pod_spec.get("affinity") or {}).get("nodeAffinity") or {})
           .get("requiredDuringSchedulingIgnoredDuringExecution") or {})
    terms = req.get("nodeSelectorTerms") or []
    if not terms:
        return True

    def expr_ok(e: dict) -> bool:
        op, key, vals = e.get("operator"), e.get("key"), e.get("values") or []
        have = labels.get(key)
        if op == "In":
            return have in vals
        if op == "NotIn":
            return have not in vals
        if op == "Exists":
            return key in labels
        if op == "DoesNotExist":
            return key not in labels
        if op in ("Gt", "Lt"):
            try:
                return (int(have) > int(vals[0])) if op == "Gt" else (int(have) < int(vals[0]))
            except (TypeError, ValueError):
                return False
        return False

    return any(all(expr_ok(e) for e in t.get("matchExpressions") or []) for t in terms)


# ------------------------------------------------------------------ running pod state
@dataclass
class ContainerRun:
    name: str
    argv: list
    env: dict
    cwd: str
    log_path: str
    spec: dict
    proc: subprocess.Popen | None = None
    restarts: int = 0
    started_at: float = 0.0
    last_term: dict | None = None
    ready: bool = False
    started: bool = False  # startup probe passed
    probe_fail: dict = field(default_factory=dict)
    probe_next: dict = field(default_factory=dict)
    next_restart: float = 0.0
    done: bool = False
    exit_code: int | None = None


@dataclass
class PodRun:
    key: tuple
    uid: str
    gpu_ids: list
    ports: dict           # containerPort -> host port
    workdir: str
    inits: list
    containers: list
    restart_policy: str
    phase: str = "Pending"
    init_idx: int = 0
    message: str = ""


class Kubelet:
    def __init__(self, store: Store, node: NodeInfo, state_dir: str, simulate: bool = False,
                 probe_scale: float = 1.0, restart_backoff: float = 1.0):
        self.store, self.node, self.simulate = store, node, simulate
        self.state_dir = os.path.abspath(state_dir)
        os.makedirs(os.path.join(self.state_dir, "pods"), exist_ok=True)
        self.runs: dict[tuple, PodRun] = {}
        self.gpu_owner: dict[int, tuple] = {}
        self.probe_scale = probe_scale
        self.restart_backoff = restart_backoff
        self.api_url: str | None = None  # manager REST API handed to pods (router discovery, agents)
        self._lock = threading.RLock()
        self.proxies = ServiceProxies(store, self, os.path.join(self.state_dir, "dns.json"))
        self.register_node()

    # ------------------------------------------------------------------ node
    def register_node(self) -> None:
        obj = self.node.to_object()
        cur = self.store.try_get("v1", "Node", self.node.name)
        if cur is None:
            self.store.create(obj)
        else:
            cur["metadata"]["labels"] = {**obj["metadata"]["labels"], **(cur["metadata"].get("labels") or {})}
            cur["status"] = obj["status"]
            self.store.update(cur)

    def free_gpus(self) -> list[int]:
        return [g for g in range(self.node.gpus) if g not in self.gpu_owner]

    def allocate_gpus(self, n: int, key: tuple) -> list[int] | None:
        free = self.free_gpus()
        if n > len(free):
            return None
        # prefer an aligned contiguous block (xGMI-adjacent peers), then any contiguous, then any
        aligned = [list(range(s, s + n)) for s in range(0, self.node.gpus - n + 1, n if n & (n - 1) == 0 else 1)]
        contiguous = [list(range(s, s + n)) for s in range(self.node.gpus - n + 1)]
        block = next((b for b in aligned + contiguous if all(g in free for g in b)), free[:n])
        for g in block:
            self.gpu_owner[g] = key
        return block

    # ------------------------------------------------------------------ scheduling
    def schedule(self) -> None:
        node_obj = self.store.try_get("v1", "Node", self.node.name)
        if node_obj is None:
            return
        for p in self.store.list("v1", "Pod"):
            if p["spec"].get("nodeName") or p["metadata"].get("deletionTimestamp"):
                continue
            key = (p["metadata"]["namespace"], p["metadata"]["name"])
            reason = None
            if not node_affinity_ok(p["spec"], node_obj):
                reason = "0/1 nodes are available: node(s) didn't match Pod's node affinity/selector"
            else:
                n = gpu_request(p["spec"])
                with self._lock:
                    ids = self.allocate_gpus(n, key) if n else []
                if ids is None:
                    reason = f"0/1 nodes are available: Insufficient {C.AMD_GPU_RESOURCE}"
            st = p.get("status") or {}
            if reason:
                if st.get("phase") != "Pending" or (st.get("conditions") or [{}])[0].get("message") != reason:
                    p["status"] = {"phase": "Pending", "conditions": [{"type": "PodScheduled", "status": "False",
                                                                      "reason": "Unschedulable", "message": reason}]}
                    self.store.update_status(p)
                continue
            p["spec"]["nodeName"] = self.node.name
            ann = p["metadata"].setdefault("annotations", {})
            ann["ome.io/gpu-ids"] = ",".join(map(str, ids))
            try:
                p = self.store.update(p)
            except Exception:  # noqa: BLE001 — conflict: retry next sync
                with self._lock:
                    for g in ids:
                        self.gpu_owner.pop(g, None)
                continue
            p["status"] = {"phase": "Pending", "conditions": [{"type": "PodScheduled", "status": "True"}],
                           "hostIP": "127.0.0.1", "podIP": "127.0.0.1"}
            self.store.update_status(p)

    # ------------------------------------------------------------------ pod setup
    def _resolve_env(self, pod: dict, c: dict, base: dict) -> dict:
        env = dict(base)
        ns = pod["metadata"]["namespace"]
        for ef in c.get("envFrom") or []:
            if ef.get("configMapRef"):
                cm = self.store.try_get("v1", "ConfigMap", ef["configMapRef"]["name"], ns)
                env.update({(ef.get("prefix") or "") + k: v for k, v in ((cm or {}).get("data") or {}).items()})
            if ef.get("secretRef"):
                sec = self.store.try_get("v1", "Secret", ef["secretRef"]["name"], ns)
                env.update({(ef.get("prefix") or "") + k: _secret_val(sec, k) for k in ((sec or {}).get("data") or {})})
        for e in c.get("env") or []:
            name = e.get("name")
            if "value" in e:
                env[name] = expand_vars(str(e.get("value") or ""), env)
                continue
            vf = e.get("valueFrom") or {}
            if vf.get("fieldRef"):
                fp = vf["fieldRef"].get("fieldPath", "")
                env[name] = {"metadata.name": pod["metadata"]["name"], "metadata.namespace": ns,
                             "status.podIP": "127.0.0.1", "status.hostIP": "127.0.0.1", "spec.nodeName": self.node.name,
                             "metadata.uid": pod["metadata"].get("uid", "")}.get(fp, "")
                m = re.match(r"metadata\.(labels|annotations)\['(.+)'\]", fp)
                if m:
                    env[name] = (pod["metadata"].get(m.group(1)) or {}).get(m.group(2), "")
            elif vf.get("secretKeyRef"):
                ref = vf["secretKeyRef"]
                env[name] = _secret_val(self.store.try_get("v1", "Secret", ref["name"], ns), ref["key"])
            elif vf.get("configMapKeyRef"):
                ref = vf["configMapKeyRef"]
                cm = self.store.try_get("v1", "ConfigMap", ref["name"], ns)
                env[name] = ((cm or {}).get("data") or {}).get(ref["key"], "")
            elif vf.get("resourceFieldRef"):
                env[name] = "1"
        return env

    def _volume_paths(self, pod: dict, workdir: str) -> dict:
        """volume name -> host directory."""
        out = {}
        ns = pod["metadata"]["namespace"]
        for v in pod["spec"].get("volumes") or []:
            name = v["name"]
            if v.get("hostPath"):
                out[name] = v["hostPath"]["path"]
            elif "emptyDir" in v:
                out[name] = os.path.join(workdir, "vol", name)
                os.makedirs(out[name], exist_ok=True)
            elif v.get("persistentVolumeClaim"):
                out[name] = os.path.join(self.state_dir, "pvc", ns, v["persistentVolumeClaim"]["claimName"])
                os.makedirs(out[name], exist_ok=True)
            elif v.get("configMap") or v.get("secret"):
                d = os.path.join(workdir, "vol", name)
                os.makedirs(d, exist_ok=True)
                if v.get("configMap"):
                    src = self.store.try_get("v1", "ConfigMap", v["configMap"]["name"], ns) or {}
                    items = (src.get("data") or {})
                else:
                    src = self.store.try_get("v1", "Secret", v["secret"].get("secretName", ""), ns) or {}
                    items = {k: _secret_val(src, k) for k in (src.get("data") or {})}
                for k, val in items.items():
                    with open(os.path.join(d, k), "w") as f:
                        f.write(val)
                out[name] = d
            else:
                out[name] = os.path.join(workdir, "vol", name)
                os.makedirs(out[name], exist_ok=True)
        return out

    def _container_run(self, pod: dict, c: dict, base_env: dict, vols: dict, ports: dict, workdir: str) -> ContainerRun:
        env = self._resolve_env(pod, c, base_env)
        mounts = {}
        for vm in c.get("volumeMounts") or []:
            host = vols.get(vm["name"])
            if host is None:
                continue
            if vm.get("subPath"):
                host = os.path.join(host, vm["subPath"])
            mounts[vm["mountPath"].rstrip("/") or "/"] = host
        # identity mounts (model hostPath at its own path, /dev/shm) need no rewrite
        remap = {k: v for k, v in mounts.items() if k != v}

        def fix(s: str) -> str:
            s = expand_vars(s, env)
            for mp in sorted(remap, key=len, reverse=True):
                s = re.sub(rf"(?<![\w.-]){re.escape(mp)}(?=/|\b|$)", remap[mp], s)
            for cport, hport in ports.items():
                s = re.sub(rf"(--port[= ])({cport})\b", rf"\g<1>{hport}", s)
            return s

        env = {k: fix(v) for k, v in env.items()}
        for k, v in env.items():  # *_PORT env values naming a container port follow the remap
            if (k == "PORT" or k.endswith("_PORT")) and v.isdigit() and int(v) in ports:
                env[k] = str(ports[int(v)])
        cmd = list(c.get("command") or [])
        args = list(c.get("args") or [])
        if not cmd:
            img = c.get("image", "")
            cmd = next((v for k, v in IMAGE_ENTRYPOINTS.items() if k in img), [])
            if not cmd and not args:
                cmd = [PY, "-c", "import time; time.sleep(1e9)"]  # pause-container stand-in
        argv = [fix(a) for a in cmd + args]
        if len(argv) >= 3 and os.path.basename(argv[0]) in ("bash", "sh") and argv[1] in ("-c", "-lc", "-ec"):
            argv = ["/bin/bash", argv[1], translate_command(argv[2])] + argv[3:]
        else:
            argv = shlex.split(translate_command(shlex.join(argv)))
        for i, a in enumerate(argv[:-1]):  # exec-form "--port", "8080" / "--addr", ":8080" pairs
            nxt = argv[i + 1]
            # (--service-discovery-port names the DISCOVERED pods' container port, not one this pod
            # listens on: the router maps it through each worker pod's own host-port annotation)
            if (a == "--port" or a.endswith("-port")) and a not in _PEER_PORT_FLAGS and nxt.isdigit() and \
                    int(nxt) in ports:
                argv[i + 1] = str(ports[int(nxt)])
            elif a in ("--addr", "--listen", "--metrics-addr") and nxt.rpartition(":")[2].isdigit():
                hp, _, pt = nxt.rpartition(":")
                if int(pt) in ports:
                    argv[i + 1] = f"{hp}:{ports[int(pt)]}"
        if ports and not any("--port" in a for a in argv) and "ome_amd.runtime.server" in " ".join(argv):
            argv += ["--port", str(next(iter(ports.values())))]
        return ContainerRun(c["name"], argv, env, workdir, os.path.join(workdir, f"{c['name']}.log"), c)

    def _prepare(self, pod: dict) -> PodRun:
        ns, name = pod["metadata"]["namespace"], pod["metadata"]["name"]
        key = (ns, name)
        workdir = os.path.join(self.state_dir, "pods", f"{ns}_{name}_{pod['metadata']['uid'][:8]}")
        os.makedirs(workdir, exist_ok=True)
        ids_s = (pod["metadata"].get("annotations") or {}).get("ome.io/gpu-ids", "")
        ids = [int(x) for x in ids_s.split(",") if x != ""]
        with self._lock:
            for g in ids:
                self.gpu_owner[g] = key
        ports = {}
        for c in pod["spec"].get("containers") or []:
            for p in c.get("ports") or []:
                cp = int(p["containerPort"])
                if cp not in ports:
                    ports[cp] = free_port()
        vols = self._volume_paths(pod, workdir)
        base = {k: v for k, v in os.environ.items() if not k.startswith(("LWS_", "OME_TEST_"))}
        base.update({"HOSTNAME": pod["spec"].get("hostname") or name, "POD_NAME": name, "POD_NAMESPACE": ns,
                     "PYTHONPATH": REPO_ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
                     "OME_LOCAL_DNS": self.proxies.dns_path, "OME_POD_PORTS": json.dumps(ports),
                     "OME_API_SERVER": self.api_url or "",
                     "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
        if ids:
            base["HIP_VISIBLE_DEVICES"] = ",".join(map(str, ids))
        elif gpu_request(pod["spec"]) == 0:
            base["HIP_VISIBLE_DEVICES"] = ""  # no GPUs requested -> none visible (device plugin semantics)
        inits = [self._container_run(pod, c, base, vols, ports, workdir) for c in pod["spec"].get("initContainers") or []]
        conts = [self._container_run(pod, c, base, vols, ports, workdir) for c in pod["spec"].get("containers") or []]
        ann = pod["metadata"].setdefault("annotations", {})
        if ports and ann.get("ome.io/host-ports") != json.dumps(ports):
            ann["ome.io/host-ports"] = json.dumps({str(k): v for k, v in ports.items()})
            try:
                self.store.update(pod)
            except Exception:  # noqa: BLE001
                pass
        return PodRun(key, pod["metadata"]["uid"], ids, ports, workdir, inits, conts,
                      pod["spec"].get("restartPolicy") or "Always")

    # ------------------------------------------------------------------ process control
    def _start(self, cr: ContainerRun) -> None:
        logf = open(cr.log_path, "ab")
        try:
            cr.proc = subprocess.Popen(cr.argv, env=cr.env, cwd=cr.cwd, stdout=logf, stderr=subprocess.STDOUT,
                                       stdin=subprocess.DEVNULL, start_new_session=True)
        except OSError as e:
            logf.write(f"exec failed: {e}\n".encode())
            cr.proc = None
            cr.exit_code = 127
        finally:
            logf.close()
        cr.started_at = time.time()
        cr.ready = False
        cr.started = not bool(cr.spec.get("startupProbe"))
        cr.probe_fail.clear()
        cr.probe_next.clear()

    @staticmethod
    def _kill(cr: ContainerRun, grace: float = 5.0) -> None:
        p = cr.proc
        if p is None or p.poll() is not None:
            return
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            return
        try:
            p.wait(timeout=grace)
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait(timeout=5)

    def _tail(self, cr: ContainerRun, n: int = 4000) -> str:
        try:
            with open(cr.log_path, "rb") as f:
                f.seek(0, os.SEEK_END)
                sz = f.tell()
                f.seek(max(0, sz - n))
                return f.read().decode(errors="replace")
        except OSError:
            return ""

    # ------------------------------------------------------------------ probes
    def _probe_once(self, probe: dict, run: PodRun, cr: ContainerRun) -> bool:
        timeout = float(probe.get("timeoutSeconds", 1)) * max(1.0, self.probe_scale)

        def port_of(p):
            if isinstance(p, str) and not p.isdigit():
                for c in [cr.spec]:
                    for cp in c.get("ports") or []:
                        if cp.get("name") == p:
                            p = cp["containerPort"]
            p = int(p)
            return run.ports.get(p, p)

        try:
            if probe.get("httpGet"):
                hg = probe["httpGet"]
                url = f"http://127.0.0.1:{port_of(hg.get('port', 80))}{hg.get('path', '/')}"
                req = urllib.request.Request(url, headers={h["name"]: h["value"] for h in hg.get("httpHeaders") or []})
                with urllib.request.urlopen(req, timeout=timeout) as r:
                    return 200 <= r.status < 400
            if probe.get("tcpSocket"):
                with socket.create_connection(("127.0.0.1", port_of(probe["tcpSocket"]["port"])), timeout=timeout):
                    return True
            if probe.get("exec"):
                argv = [translate_command(a) for a in probe["exec"].get("command") or []]
                return subprocess.run(argv, env=cr.env, cwd=cr.cwd, timeout=timeout, capture_output=True).returncode == 0
            if probe.get("grpc"):
                # a real grpc.health.v1.Health/Check of the probe's service (kubelet semantics:
                # only SERVING passes; the engine's --grpc-mode server answers it)
                from ome_amd.runtime.grpc_server import SERVING, health_check_sync

                g = probe["grpc"]
                return health_check_sync(f"127.0.0.1:{port_of(g['port'])}", g.get("service") or "",
                                         timeout=timeout) == SERVING
        except Exception:  # noqa: BLE001 — any failure is a probe failure
            return False
        return True

    def _run_probe(self, kind: str, run: PodRun, cr: ContainerRun, now: float) -> bool | None:
        """None = not due yet; else the probe verdict after thresholds."""
        probe = cr.spec.get(kind)
        if not probe:
            return True
        delay = float(probe.get("initialDelaySeconds", 0)) * self.probe_scale
        if now - cr.started_at < delay or now < cr.probe_next.get(kind, 0.0):
            return None
        cr.probe_next[kind] = now + float(probe.get("periodSeconds", 10)) * self.probe_scale
        ok = self._probe_once(probe, run, cr)
        if ok:
            cr.probe_fail[kind] = 0
            return True
        cr.probe_fail[kind] = cr.probe_fail.get(kind, 0) + 1
        if cr.probe_fail[kind] >= int(probe.get("failureThreshold", 3)):
            return False
        return None

    # ------------------------------------------------------------------ sync loop
    def sync(self) -> None:
        self.schedule()
        now = time.time()
        pods = {(p["metadata"]["namespace"], p["metadata"]["name"]): p for p in self.store.list("v1", "Pod")
                if p["spec"].get("nodeName") == self.node.name}
        # terminate runs whose pod vanished, was replaced (uid) or is being deleted
        for key, run in list(self.runs.items()):
            p = pods.get(key)
            if p is None or p["metadata"]["uid"] != run.uid or p["metadata"].get("deletionTimestamp"):
                self._teardown(run)
        for key, p in pods.items():
            if p["metadata"].get("deletionTimestamp"):
                continue
            run = self.runs.get(key)
            if run is None:
                if (p.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
                    continue
                try:
                    run = self._prepare(p)
                except Exception as e:  # noqa: BLE001
                    log.exception("pod %s setup failed", key)
                    p["status"] = {**(p.get("status") or {}), "phase": "Failed", "message": f"setup failed: {e}"}
                    self.store.update_status(p)
                    continue
                self.runs[key] = run
            if self.simulate:
                self._simulate(run, p)
            else:
                self._drive(run, now)
                self._publish(run, p)
        self.proxies.sync()

    def _teardown(self, run: PodRun) -> None:
        for cr in run.inits + run.containers:
            self._kill(cr, grace=2.0)
        with self._lock:
            for g in run.gpu_ids:
                if self.gpu_owner.get(g) == run.key:
                    self.gpu_owner.pop(g, None)
            for g, k in list(self.gpu_owner.items()):
                if k == run.key:
                    self.gpu_owner.pop(g, None)
        self.runs.pop(run.key, None)

    def _simulate(self, run: PodRun, p: dict) -> None:
        if run.phase == "Running":
            return
        run.phase = "Running"
        for cr in run.containers:
            cr.ready = cr.started = True
        self._publish(run, p)

    def _drive(self, run: PodRun, now: float) -> None:
        if run.phase in ("Succeeded", "Failed"):
            return
        # init containers: sequential, must succeed
        while run.init_idx < len(run.inits):
            cr = run.inits[run.init_idx]
            if cr.proc is None and cr.exit_code is None:
                self._start(cr)
                run.phase = "Pending"
                return
            rc = cr.proc.poll() if cr.proc else cr.exit_code
            if rc is None:
                return
            if rc == 0:
                cr.done, cr.exit_code = True, 0
                run.init_idx += 1
                continue
            cr.exit_code = rc
            if run.restart_policy == "Never":
                run.phase, run.message = "Failed", f"init container {cr.name} exited {rc}: {self._tail(cr, 800)}"
                return
            if now < cr.next_restart:
                return
            cr.restarts += 1
            cr.next_restart = now + min(300.0, self.restart_backoff * 2 ** min(cr.restarts, 8))
            cr.proc, cr.exit_code = None, None
            return
        run.phase = "Running"
        all_done = True
        any_failed = False
        for cr in run.containers:
            if cr.proc is None and cr.exit_code is None and not cr.done:
                if now >= cr.next_restart:
                    self._start(cr)
                all_done = False
                continue
            if cr.done:
                any_failed |= (cr.exit_code or 0) != 0
                continue
            rc = cr.proc.poll() if cr.proc else cr.exit_code
            if rc is None:
                all_done = False
                # startup -> liveness/readiness
                if not cr.started:
                    v = self._run_probe("startupProbe", run, cr, now)
                    if v is True:
                        cr.started = True
                    elif v is False:
                        self._kill(cr, 2.0)
                        rc = -9
                if cr.started and rc is None:
                    if self._run_probe("livenessProbe", run, cr, now) is False:
                        self._kill(cr, 2.0)
                        rc = -9
                    else:
                        v = self._run_probe("readinessProbe", run, cr, now)
                        if v is not None:
                            cr.ready = bool(v)
                if rc is None:
                    continue
            # container exited
            cr.ready = False
            cr.last_term = {"exitCode": rc, "reason": "Completed" if rc == 0 else "Error",
                            "finishedAt": now_iso(), "message": self._tail(cr, 2000)}
            if run.restart_policy == "Always" or (run.restart_policy == "OnFailure" and rc != 0):
                cr.restarts += 1
                cr.proc, cr.exit_code = None, None
                cr.next_restart = now + min(300.0, self.restart_backoff * 2 ** min(cr.restarts - 1, 8))
                all_done = False
            else:
                cr.done, cr.exit_code = True, rc
                any_failed |= rc != 0
        if all_done and run.containers:
            run.phase = "Failed" if any_failed else "Succeeded"

    def _publish(self, run: PodRun, p: dict) -> None:
        cstat = []
        for cr in run.containers:
            running = cr.proc is not None and cr.proc.poll() is None
            state = ({"running": {"startedAt": now_iso()}} if running or self.simulate else
                     {"terminated": cr.last_term or {"exitCode": cr.exit_code or 0}} if cr.done else
                     {"waiting": {"reason": "CrashLoopBackOff" if cr.restarts else "ContainerCreating"}})
            ent = {"name": cr.name, "ready": cr.ready, "started": cr.started, "restartCount": cr.restarts,
                   "image": cr.spec.get("image", ""), "state": state}
            if cr.last_term and not cr.done:
                ent["lastState"] = {"terminated": cr.last_term}
            cstat.append(ent)
        ready = bool(run.containers) and all(cr.ready for cr in run.containers) and run.phase == "Running"
        old = p.get("status") or {}
        st = {"phase": run.phase, "hostIP": "127.0.0.1", "podIP": "127.0.0.1", "containerStatuses": cstat,
              "conditions": [{"type": "PodScheduled", "status": "True"},
                             {"type": "Initialized", "status": "True" if run.init_idx >= len(run.inits) else "False"},
                             {"type": "ContainersReady", "status": "True" if ready else "False"},
                             {"type": "Ready", "status": "True" if ready else "False"}],
              "startTime": old.get("startTime") or now_iso()}
        if run.inits:
            st["initContainerStatuses"] = [{"name": cr.name, "ready": cr.done, "restartCount": cr.restarts,
                                            "state": {"terminated": {"exitCode": cr.exit_code}} if cr.exit_code is not None
                                            else {"running": {}}} for cr in run.inits]
        if run.message:
            st["message"] = run.message
        if _strip_times(old) != _strip_times(st):
            for _ in range(3):
                try:
                    cur = self.store.get("v1", "Pod", p["metadata"]["name"], p["metadata"]["namespace"])
                    if cur["metadata"]["uid"] != run.uid:
                        return
                    cur["status"] = st
                    self.store.update_status(cur)
                    return
                except NotFound:
                    return
                except Conflict:
                    continue

    # ------------------------------------------------------------------ user-facing helpers
    def logs(self, namespace: str, name: str, container: str | None = None) -> str:
        run = self.runs.get((namespace, name))
        if run is None:
            return ""
        crs = [cr for cr in run.inits + run.containers if container in (None, cr.name)]
        return "".join(self._tail(cr, 1 << 20) for cr in crs)

    def host_port(self, namespace: str, name: str, container_port: int) -> int | None:
        run = self.runs.get((namespace, name))
        return run.ports.get(int(container_port)) if run else None

    def inject_fault(self, namespace: str, name: str, container: str | None = None, sig: int = signal.SIGKILL) -> bool:
        """Chaos hook: signal a running container's process group (e.g. simulate a GPU fault / OOM kill)."""
        run = self.runs.get((namespace, name))
        if run is None:
            return False
        for cr in run.containers:
            if container in (None, cr.name) and cr.proc is not None and cr.proc.poll() is None:
                os.killpg(cr.proc.pid, sig)
                return True
        return False

    def shutdown(self) -> None:
        for run in list(self.runs.values()):
            self._teardown(run)
        self.proxies.shutdown()


def _secret_val(sec: dict | None, key: str) -> str:
    if not sec:
        return ""
    if key in (sec.get("stringData") or {}):
        return sec["stringData"][key]
    v = (sec.get("data") or {}).get(key, "")
    import base64
    import binascii

    try:
        return base64.b64decode(v).decode()
    except (binascii.Error, UnicodeDecodeError):
        return v


def _strip_times(st: dict) -> str:
    s = json.dumps(st, sort_keys=True)
    return re.sub(r'"(startedAt|finishedAt|startTime|lastTransitionTime)": "[^"]*"', "", s)


# ------------------------------------------------------------------ services
class _Proxy:
    """One listening TCP port forwarding to a rotating set of backend host ports."""

    def __init__(self, listen_port: int = 0):
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind(("127.0.0.1", listen_port))
        self.sock.listen(256)
        self.port = self.sock.getsockname()[1]
        self.backends: list[int] = []
        self._rr = 0
        self._stop = False
        threading.Thread(target=self._accept, daemon=True).start()

    def _accept(self) -> None:
        while not self._stop:
            try:
                cli, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(cli,), daemon=True).start()

    def _serve(self, cli: socket.socket) -> None:
        bes = list(self.backends)
        if not bes:
            cli.close()
            return
        self._rr = (self._rr + 1) % len(bes)
        try:
            up = socket.create_connection(("127.0.0.1", bes[self._rr]), timeout=10)
        except OSError:
            cli.close()
            return
        up.settimeout(None)

        def pump(a, b):
            try:
                while True:
                    d = a.recv(65536)
                    if not d:
                        break
                    b.sendall(d)
            except OSError:
                pass
            finally:
                for s in (a, b):
                    try:
                        s.shutdown(socket.SHUT_RDWR)
                    except OSError:
                        pass

        t = threading.Thread(target=pump, args=(up, cli), daemon=True)
        t.start()
        pump(cli, up)
        t.join(timeout=60)
        cli.close()
        up.close()

    def close(self) -> None:
        self._stop = True
        try:
            self.sock.close()
        except OSError:
            pass


class ServiceProxies:
    def __init__(self, store: Store, kubelet: "Kubelet", dns_path: str):
        self.store, self.kubelet, self.dns_path = store, kubelet, dns_path
        self.proxies: dict[tuple, _Proxy] = {}
        self._last_dns = None

    def _endpoints(self, svc: dict, port: dict) -> list[int]:
        sel = (svc.get("spec") or {}).get("selector") or {}
        if not sel:
            return []
        out = []
        target = port.get("targetPort", port.get("port"))
        for p in self.store.list("v1", "Pod", svc["metadata"]["namespace"]):
            if not match_labels(p["metadata"].get("labels") or {}, sel):
                continue
            if not any(c.get("type") == "Ready" and c.get("status") == "True" for c in (p.get("status") or {}).get("conditions") or []):
                continue
            tp = target
            if isinstance(tp, str) and not tp.isdigit():
                tp = next((cp["containerPort"] for c in p["spec"].get("containers") or [] for cp in c.get("ports") or []
                           if cp.get("name") == tp), None)
                if tp is None:
                    continue
            hp = self.kubelet.host_port(p["metadata"]["namespace"], p["metadata"]["name"], int(tp))
            out.append(hp if hp else int(tp))
        return out

    def sync(self) -> None:
        dns: dict[str, dict] = {}
        seen = set()
        for svc in self.store.list("v1", "Service"):
            ns, name = svc["metadata"]["namespace"], svc["metadata"]["name"]
            pm = {}
            for port in (svc.get("spec") or {}).get("ports") or []:
                key = (ns, name, int(port["port"]))
                seen.add(key)
                px = self.proxies.get(key)
                if px is None:
                    px = self.proxies[key] = _Proxy()
                px.backends = self._endpoints(svc, port)
                pm[str(port["port"])] = px.port
            for host in (f"{name}.{ns}.svc.cluster.local", f"{name}.{ns}.svc", f"{name}.{ns}"):
                dns[host] = pm
        for key in list(self.proxies):
            if key not in seen:
                self.proxies.pop(key).close()
        # ingress hosts -> backend service proxy
        for ing in self.store.list("networking.k8s.io/v1", "Ingress"):
            for rule in (ing.get("spec") or {}).get("rules") or []:
                for path in ((rule.get("http") or {}).get("paths") or []):
                    be = (path.get("backend") or {}).get("service") or {}
                    svc_host = f"{be.get('name')}.{ing['metadata']['namespace']}.svc.cluster.local"
                    port = str((be.get("port") or {}).get("number", 80))
                    if rule.get("host") and svc_host in dns and port in dns[svc_host]:
                        dns[rule["host"]] = {"80": dns[svc_host][port], "443": dns[svc_host][port]}
        if dns != self._last_dns:
            tmp = self.dns_path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(dns, f)
            os.replace(tmp, self.dns_path)
            self._last_dns = dns

    def shutdown(self) -> None:
        for px in self.proxies.values():
            px.close()
        self.proxies.clear()
