"""Metrics-driven autoscaling for the local executor (stand-in for the HPA controller and the
KEDA Prometheus scaler, ``pkg/controller/v1beta1/inferenceservice/reconcilers/keda``).

The engines expose Prometheus text on ``/metrics``; this module scrapes every ready pod of a
scale target, keeps a short sample history per series (for ``rate``/``avg_over_time``) and
evaluates the ScaledObject's query with a PromQL subset:

    expr   := cmp (('*'|'/'|'+'|'-') cmp)*
    cmp    := unary (('<'|'>'|'<='|'>='|'=='|'!=') ['bool'] number)?
    unary  := number | agg '(' expr ')' | fn '(' selector '[' dur ']' ')' | selector | '(' expr ')'
    agg    := sum | avg | max | min | count
    fn     := rate | irate | increase | avg_over_time | max_over_time | min_over_time

Label matchers inside ``{}`` are parsed but every scraped series belongs to the target by
construction (we only scrape its pods), so they are not needed for scoping.

Replica math follows KEDA's AverageValue target: ``desired = ceil(value / threshold)``; for
HPA CPU utilisation, ``desired = ceil(current * usage% / target%)`` with usage read from the
pods' process trees.
"""
from __future__ import annotations

import math
import re
import time
import urllib.request
from collections import defaultdict, deque

from ome_amd.store.store import Store

_TOK = re.compile(r"\s*(?:(\d+\.?\d*(?:e[+-]?\d+)?)|([A-Za-z_:][A-Za-z0-9_:]*)|(<=|>=|==|!=|[<>*/+\-(){}\[\],])|(\"[^\"]*\"|=~|!~|=))",
                  re.I)


def parse_prom_text(text: str) -> dict[str, float]:
    """Sum samples per metric name (labels dropped — one target's pods)."""
    out: dict[str, float] = defaultdict(float)
    for line in text.splitlines():
        if not line or line.startswith("#"):
            continue
        m = re.match(r"([A-Za-z_:][A-Za-z0-9_:]*)(\{[^}]*\})?\s+([-+0-9.eEinfNa]+)", line)
        if m:
            try:
                out[m.group(1)] += float(m.group(3))
            except ValueError:
                pass
    return dict(out)


class SeriesHistory:
    def __init__(self, horizon: float = 600.0):
        self.h: dict[str, deque] = defaultdict(deque)
        self.horizon = horizon

    def add(self, sample: dict[str, float], t: float | None = None) -> None:
        t = time.time() if t is None else t
        for k, v in sample.items():
            d = self.h[k]
            d.append((t, v))
            while d and d[0][0] < t - self.horizon:
                d.popleft()

    def last(self, name: str) -> float:
        d = self.h.get(name)
        return d[-1][1] if d else 0.0

    def window(self, name: str, secs: float, now: float | None = None) -> list[tuple[float, float]]:
        now = time.time() if now is None else now
        return [(t, v) for t, v in self.h.get(name, ()) if t >= now - secs]


def _dur(s: str) -> float:
    m = re.fullmatch(r"(\d+)(ms|s|m|h|d)", s)
    if not m:
        raise ValueError(f"bad duration {s}")
    return int(m.group(1)) * {"ms": 1e-3, "s": 1, "m": 60, "h": 3600, "d": 86400}[m.group(2)]


class PromQL:
    AGG = {"sum", "avg", "max", "min", "count"}
    RANGE = {"rate", "irate", "increase", "avg_over_time", "max_over_time", "min_over_time"}

    def __init__(self, query: str):
        self.toks = []
        pos = 0
        q = query.strip()
        while pos < len(q):
            m = _TOK.match(q, pos)
            if not m or m.end() == pos:
                raise ValueError(f"cannot tokenize {q[pos:]!r}")
            self.toks.append(next(g for g in m.groups() if g is not None))
            pos = m.end()
            while pos < len(q) and q[pos].isspace():
                pos += 1
        self.i = 0

    def eval(self, hist: SeriesHistory, now: float | None = None) -> float:
        self.i, self.hist, self.now = 0, hist, time.time() if now is None else now
        v = self._expr()
        if self.i != len(self.toks):
            raise ValueError(f"trailing tokens {self.toks[self.i:]}")
        return v

    def _peek(self):
        return self.toks[self.i] if self.i < len(self.toks) else None

    def _take(self, want=None):
        t = self._peek()
        if want is not None and t != want:
            raise ValueError(f"expected {want!r}, got {t!r}")
        self.i += 1
        return t

    def _expr(self) -> float:
        v = self._cmp()
        while self._peek() in ("*", "/", "+", "-"):
            op = self._take()
            r = self._cmp()
            v = v * r if op == "*" else (v / r if r else 0.0) if op == "/" else v + r if op == "+" else v - r
        return v

    def _cmp(self) -> float:
        v = self._unary()
        if self._peek() in ("<", ">", "<=", ">=", "==", "!="):
            op = self._take()
            as_bool = self._peek() == "bool"
            if as_bool:
                self._take()
            r = self._unary()
            ok = {"<": v < r, ">": v > r, "<=": v <= r, ">=": v >= r, "==": v == r, "!=": v != r}[op]
            return (1.0 if ok else 0.0) if as_bool else (v if ok else 0.0)
        return v

    def _selector(self) -> str:
        name = self._take()
        if self._peek() == "{":
            while self._take() != "}":
                pass
        return name

    def _unary(self) -> float:
        t = self._peek()
        if t is None:
            raise ValueError("unexpected end of query")
        if t == "(":
            self._take()
            v = self._expr()
            self._take(")")
            return v
        if re.fullmatch(r"\d+\.?\d*(?:e[+-]?\d+)?", t, re.I):
            self._take()
            return float(t)
        if t in self.AGG:
            self._take()
            if self._peek() in ("by", "without"):
                self._take()
                self._take("(")
                while self._take() != ")":
                    pass
            self._take("(")
            v = self._expr()
            self._take(")")
            if self._peek() in ("by", "without"):
                self._take()
                self._take("(")
                while self._take() != ")":
                    pass
            return v  # one aggregated series per target
        if t in self.RANGE:
            self._take()
            self._take("(")
            name = self._selector()
            self._take("[")
            num = self._take()
            unit = self._take() if self._peek() not in ("]",) else "s"
            secs = _dur(f"{num}{unit}")
            self._take("]")
            self._take(")")
            pts = self.hist.window(name, secs, self.now)
            if t.endswith("over_time"):
                vals = [v for _, v in pts] or [0.0]
                return {"avg_over_time": sum(vals) / len(vals), "max_over_time": max(vals),
                        "min_over_time": min(vals)}[t]
            if len(pts) < 2:
                return 0.0
            if t == "irate":
                (t0, v0), (t1, v1) = pts[-2], pts[-1]
            else:
                (t0, v0), (t1, v1) = pts[0], pts[-1]
            dv = v1 - v0 if v1 >= v0 else v1  # counter reset
            return dv if t == "increase" else dv / max(t1 - t0, 1e-9)
        return self.hist.last(self._selector())


def desired_from_keda(value: float, threshold: float, current: int) -> int:
    if threshold <= 0:
        return current
    return max(0, math.ceil(value / threshold - 1e-9))


class MetricsAutoscaler:
    """Periodically sets ``status.desiredReplicas`` on ScaledObjects / HPAs; the executor's
    HPA controllers then clamp and apply it to the Deployment."""

    def __init__(self, store: Store, kubelet, period: float = 15.0):
        self.store, self.kubelet, self.period = store, kubelet, period
        self.hist: dict[tuple, SeriesHistory] = defaultdict(SeriesHistory)
        self._cpu_prev: dict[int, tuple[float, float]] = {}

    def _target_pods(self, ns: str, deploy: str) -> list[dict]:
        d = self.store.try_get("apps/v1", "Deployment", deploy, ns)
        if d is None:
            return []
        uid = d["metadata"]["uid"]
        return [p for p in self.store.list("v1", "Pod", ns)
                if any(r.get("uid") == uid for r in p["metadata"].get("ownerReferences") or [])
                and any(c.get("type") == "Ready" and c.get("status") == "True"
                        for c in (p.get("status") or {}).get("conditions") or [])]

    def scrape(self, ns: str, pods: list[dict]) -> dict[str, float]:
        total: dict[str, float] = defaultdict(float)
        for p in pods:
            for c in p["spec"].get("containers") or []:
                for cp in c.get("ports") or []:
                    hp = self.kubelet.host_port(ns, p["metadata"]["name"], cp["containerPort"])
                    if not hp:
                        continue
                    try:
                        with urllib.request.urlopen(f"http://127.0.0.1:{hp}/metrics", timeout=2) as r:
                            for k, v in parse_prom_text(r.read().decode()).items():
                                total[k] += v
                    except Exception:  # noqa: BLE001 — unreachable pod contributes nothing
                        pass
                    break
        return dict(total)

    def tick(self) -> None:
        for so in self.store.list("keda.sh/v1alpha1", "ScaledObject"):
            ns, name = so["metadata"]["namespace"], so["metadata"]["name"]
            tgt = so["spec"]["scaleTargetRef"]["name"]
            pods = self._target_pods(ns, tgt)
            h = self.hist[(ns, name)]
            h.add(self.scrape(ns, pods))
            desired = None
            for trig in so["spec"].get("triggers") or []:
                md = trig.get("metadata") or {}
                try:
                    val = PromQL(md.get("query", "0")).eval(h)
                except ValueError:
                    continue
                d = desired_from_keda(val, float(md.get("threshold", 1) or 1), len(pods))
                desired = d if desired is None else max(desired, d)
            if desired is not None:
                st = {**(so.get("status") or {}), "desiredReplicas": desired, "lastEvaluated": time.time()}
                so["status"] = st
                self.store.update_status(so)
        for hpa in self.store.list("autoscaling/v2", "HorizontalPodAutoscaler"):
            ns = hpa["metadata"]["namespace"]
            pods = self._target_pods(ns, hpa["spec"]["scaleTargetRef"]["name"])
            if not pods:
                continue
            util = self._cpu_util(ns, pods)
            tgt = 80
            for m in hpa["spec"].get("metrics") or []:
                tgt = ((m.get("resource") or {}).get("target") or {}).get("averageUtilization", tgt)
            if util is None:
                continue
            desired = max(1, math.ceil(len(pods) * util / max(tgt, 1)))
            hpa["status"] = {**(hpa.get("status") or {}), "desiredReplicas": desired,
                             "currentMetrics": [{"type": "Resource", "resource": {
                                 "name": "cpu", "current": {"averageUtilization": int(util)}}}]}
            self.store.update_status(hpa)

    def _cpu_util(self, ns: str, pods: list[dict]) -> float | None:
        try:
            import psutil
        except ImportError:
            return None
        utils = []
        now = time.time()
        for p in pods:
            run = self.kubelet.runs.get((ns, p["metadata"]["name"]))
            if run is None:
                continue
            for cr in run.containers:
                if cr.proc is None or cr.proc.poll() is not None:
                    continue
                try:
                    pr = psutil.Process(cr.proc.pid)
                    cpu = sum(x.cpu_times().user + x.cpu_times().system for x in [pr] + pr.children(recursive=True))
                except psutil.Error:
                    continue
                prev = self._cpu_prev.get(cr.proc.pid)
                self._cpu_prev[cr.proc.pid] = (now, cpu)
                if prev and now > prev[0]:
                    utils.append(100.0 * (cpu - prev[1]) / (now - prev[0]))
        return sum(utils) / len(utils) if utils else None

    def run(self, stop) -> None:
        while not stop.wait(self.period):
            try:
                self.tick()
            except Exception:  # noqa: BLE001
                import logging

                logging.getLogger("ome_amd.executor").exception("autoscaler tick failed")
