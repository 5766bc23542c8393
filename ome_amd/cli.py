"""omectl — kubectl-style client for the ome-amd manager REST API.

    python -m ome_amd.cli apply -f config/            # YAML file or directory (server-side apply)
    python -m ome_amd.cli get inferenceservices -n default
    python -m ome_amd.cli get isvc llama-3-8b-instruct -o yaml
    python -m ome_amd.cli describe isvc llama-3-8b-instruct
    python -m ome_amd.cli logs llama-3-8b-instruct-engine-abc-0
    python -m ome_amd.cli wait isvc llama-3-8b-instruct --for Ready --timeout 600
    python -m ome_amd.cli delete isvc llama-3-8b-instruct

Server: ``--server`` or ``$OME_API_SERVER`` (default ``http://127.0.0.1:9443``).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time
import urllib.error
import urllib.parse
import urllib.request

import yaml

from ome_amd.manager import KIND_OF_PLURAL, PLURALS
from ome_amd.store.store import CLUSTER_SCOPED

SHORT = {"isvc": "inferenceservices", "bm": "basemodels", "cbm": "clusterbasemodels", "sr": "servingruntimes",
         "csr": "clusterservingruntimes", "ac": "acceleratorclasses", "bj": "benchmarkjobs", "po": "pods",
         "svc": "services", "cm": "configmaps", "deploy": "deployments", "lws": "leaderworkersets", "no": "nodes",
         "ns": "namespaces", "ftw": "finetunedweights", "ing": "ingresses", "hpa": "horizontalpodautoscalers"}
GROUPS = {"InferenceService": "ome.io/v1beta1", "BaseModel": "ome.io/v1beta1", "ClusterBaseModel": "ome.io/v1beta1",
          "ServingRuntime": "ome.io/v1beta1", "ClusterServingRuntime": "ome.io/v1beta1",
          "AcceleratorClass": "ome.io/v1beta1", "BenchmarkJob": "ome.io/v1beta1", "FineTunedWeight": "ome.io/v1beta1",
          "Deployment": "apps/v1", "Job": "batch/v1", "LeaderWorkerSet": "leaderworkerset.x-k8s.io/v1",
          "Ingress": "networking.k8s.io/v1", "HorizontalPodAutoscaler": "autoscaling/v2",
          "ScaledObject": "keda.sh/v1alpha1", "PodDisruptionBudget": "policy/v1", "RayCluster": "ray.io/v1",
          "Role": "rbac.authorization.k8s.io/v1", "RoleBinding": "rbac.authorization.k8s.io/v1",
          "ClusterRole": "rbac.authorization.k8s.io/v1", "ClusterRoleBinding": "rbac.authorization.k8s.io/v1"}


class Client:
    def __init__(self, server: str):
        self.server = server.rstrip("/")

    def req(self, method: str, path: str, body=None, ctype="application/json"):
        data = None
        if body is not None:
            data = body.encode() if isinstance(body, str) else json.dumps(body).encode()
        r = urllib.request.Request(self.server + path, data=data, method=method, headers={"Content-Type": ctype})
        try:
            with urllib.request.urlopen(r, timeout=60) as resp:
                raw = resp.read()
                ct = resp.headers.get("Content-Type", "")
                return json.loads(raw) if "json" in ct else raw.decode()
        except urllib.error.HTTPError as e:
            try:
                msg = json.loads(e.read()).get("message")
            except Exception:  # noqa: BLE001
                msg = str(e)
            raise SystemExit(f"Error from server ({e.code}): {msg}") from None

    @staticmethod
    def path(kind: str, ns: str | None, name: str | None = None, sub: str | None = None) -> str:
        av = GROUPS.get(kind, "v1")
        base = f"/apis/{av}" if "/" in av else f"/api/{av}"
        group = av.split("/")[0] if "/" in av else ""
        if (group, kind) not in CLUSTER_SCOPED and ns:
            base += f"/namespaces/{ns}"
        base += f"/{PLURALS[kind]}"
        if name:
            base += f"/{name}"
        if sub:
            base += f"/{sub}"
        return base


def resolve_kind(s: str) -> str:
    s = s.lower()
    plural = SHORT.get(s, s if s.endswith("s") else s + "s")
    if plural == "ingresss":
        plural = "ingresses"
    kind = KIND_OF_PLURAL.get(plural)
    if kind is None:
        kind = next((k for k in PLURALS if k.lower() == s), None)
    if kind is None:
        raise SystemExit(f"error: the server doesn't have a resource type \"{s}\"")
    return kind


def _cond(obj: dict, t: str) -> str:
    for c in (obj.get("status") or {}).get("conditions") or []:
        if c.get("type") == t:
            return c.get("status", "")
    return ""


def _age(obj: dict) -> str:
    ts = obj["metadata"].get("creationTimestamp")
    if not ts:
        return ""
    try:
        t = time.mktime(time.strptime(ts, "%Y-%m-%dT%H:%M:%SZ")) - time.timezone
    except ValueError:
        return ""
    s = max(0, int(time.time() - t))
    return f"{s}s" if s < 120 else f"{s // 60}m" if s < 7200 else f"{s // 3600}h"


def row(kind: str, o: dict) -> list[str]:
    st = o.get("status") or {}
    name = o["metadata"]["name"]
    if kind == "InferenceService":
        return [name, st.get("url", ""), _cond(o, "Ready"), _age(o)]
    if kind in ("BaseModel", "ClusterBaseModel"):
        sp = o.get("spec") or {}
        return [name, sp.get("vendor", ""), sp.get("modelArchitecture", ""), sp.get("modelParameterSize", ""),
                st.get("state", ""), _age(o)]
    if kind == "Pod":
        cs = st.get("containerStatuses") or []
        ready = f"{sum(1 for c in cs if c.get('ready'))}/{len(cs)}"
        return [name, ready, st.get("phase", ""), str(sum(c.get("restartCount", 0) for c in cs)), _age(o)]
    if kind == "BenchmarkJob":
        return [name, st.get("state", ""), _age(o)]
    if kind == "Deployment":
        return [name, f"{st.get('readyReplicas', 0)}/{(o.get('spec') or {}).get('replicas', 1)}", _age(o)]
    return [name, _age(o)]


HEADERS = {"InferenceService": ["NAME", "URL", "READY", "AGE"],
           "BaseModel": ["NAME", "VENDOR", "ARCHITECTURE", "SIZE", "STATE", "AGE"],
           "ClusterBaseModel": ["NAME", "VENDOR", "ARCHITECTURE", "SIZE", "STATE", "AGE"],
           "Pod": ["NAME", "READY", "STATUS", "RESTARTS", "AGE"], "BenchmarkJob": ["NAME", "STATE", "AGE"],
           "Deployment": ["NAME", "READY", "AGE"]}


def table(rows: list[list[str]], header: list[str]) -> str:
    w = [max(len(str(x)) for x in col) for col in zip(header, *rows)] if rows else [len(h) for h in header]
    return "\n".join("   ".join(str(x).ljust(n) for x, n in zip(r, w)).rstrip() for r in [header] + rows)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("omectl")
    ap.add_argument("--server", default=os.environ.get("OME_API_SERVER", "http://127.0.0.1:9443"))
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("apply")
    p.add_argument("-f", "--filename", required=True)
    for name in ("get", "describe", "delete", "wait"):
        p = sub.add_parser(name)
        p.add_argument("kind")
        p.add_argument("name", nargs="?")
        p.add_argument("-n", "--namespace", default="default")
        p.add_argument("-A", "--all-namespaces", action="store_true")
        p.add_argument("-o", "--output", default="table", choices=["table", "yaml", "json", "name"])
        p.add_argument("-l", "--selector", default=None)
        p.add_argument("--for", dest="for_", default="Ready")
        p.add_argument("--timeout", type=float, default=300.0)
    p = sub.add_parser("logs")
    p.add_argument("pod")
    p.add_argument("-n", "--namespace", default="default")
    p.add_argument("-c", "--container", default=None)
    a = ap.parse_args(argv)
    c = Client(a.server)

    if a.cmd == "apply":
        files = [a.filename] if os.path.isfile(a.filename) else sorted(
            glob.glob(os.path.join(a.filename, "**", "*.yaml"), recursive=True))
        for f in files:
            with open(f) as fh:
                text = fh.read()
            out = c.req("POST", "/apply", text, ctype="text/plain")
            for o in out.get("items", []):
                print(f"{o['kind'].lower()}/{o['metadata']['name']} configured")
        return 0
    if a.cmd == "logs":
        q = f"?container={urllib.parse.quote(a.container)}" if a.container else ""
        print(c.req("GET", Client.path("Pod", a.namespace, a.pod, "log") + q), end="")
        return 0
    kind = resolve_kind(a.kind)
    ns = None if a.all_namespaces else a.namespace
    if a.cmd == "get":
        if a.name:
            objs = [c.req("GET", Client.path(kind, ns, a.name))]
        else:
            q = f"?labelSelector={urllib.parse.quote(a.selector)}" if a.selector else ""
            objs = c.req("GET", Client.path(kind, ns) + q)["items"]
        if a.output == "yaml":
            print(yaml.safe_dump(objs[0] if a.name else {"items": objs}, sort_keys=False), end="")
        elif a.output == "json":
            print(json.dumps(objs[0] if a.name else {"items": objs}, indent=2))
        elif a.output == "name":
            print("\n".join(f"{kind.lower()}/{o['metadata']['name']}" for o in objs))
        else:
            print(table([row(kind, o) for o in objs], HEADERS.get(kind, ["NAME", "AGE"])))
        return 0
    if a.cmd == "describe":
        o = c.req("GET", Client.path(kind, ns, a.name))
        print(yaml.safe_dump(o, sort_keys=False), end="")
        ev = c.req("GET", Client.path("Event", o["metadata"].get("namespace") or "default"))["items"]
        mine = [e for e in ev if (e.get("involvedObject") or {}).get("uid") == o["metadata"].get("uid")]
        if mine:
            print("Events:")
            for e in mine:
                print(f"  {e.get('type', '')}\t{e.get('reason', '')}\t{e.get('message', '')}")
        return 0
    if a.cmd == "delete":
        c.req("DELETE", Client.path(kind, ns, a.name))
        print(f"{kind.lower()}/{a.name} deleted")
        return 0
    if a.cmd == "wait":
        end = time.time() + a.timeout
        while time.time() < end:
            o = c.req("GET", Client.path(kind, ns, a.name))
            if _cond(o, a.for_) == "True" or (o.get("status") or {}).get("state") == a.for_:
                print(f"{kind.lower()}/{a.name} condition met")
                return 0
            time.sleep(2)
        print(f"error: timed out waiting for {a.for_} on {kind.lower()}/{a.name}", file=sys.stderr)
        return 1
    return 2


if __name__ == "__main__":
    raise SystemExit(main())
