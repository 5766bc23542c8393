"""Engine metrics in Prometheus text format.

Both SGLang-style (``sglang:*``) and vLLM-style (``vllm:*``) names are exported, because the
reference's autoscaling defaults query vLLM names (KEDA default query
``vllm:avg_generation_throughput_toks_per_s`` / ``vllm:request_success_total``,
``pkg/controller/v1beta1/inferenceservice/reconcilers/keda/keda_reconciler.go:197-222``) while
its runtimes are SGLang (``--enable-metrics``).  Plus per-phase step timers.
"""
from __future__ import annotations

import bisect
import threading
import time

_LAT_BUCKETS = (0.001, 0.005, 0.01, 0.02, 0.04, 0.06, 0.08, 0.1, 0.25, 0.5, 0.75, 1.0, 2.5, 5.0, 7.5, 10.0,
                20.0, 40.0, 80.0)


class Histogram:
    def __init__(self, buckets=_LAT_BUCKETS):
        self.buckets = list(buckets)
        self.counts = [0] * (len(self.buckets) + 1)
        self.sum = 0.0
        self.n = 0
        self.values: list[float] = []

    def observe(self, v: float) -> None:
        self.counts[bisect.bisect_left(self.buckets, v)] += 1
        self.sum += v
        self.n += 1
        if len(self.values) < 100000:
            self.values.append(v)

    def quantile(self, q: float) -> float | None:
        if not self.values:
            return None
        s = sorted(self.values)
        return s[min(len(s) - 1, int(q * (len(s) - 1) + 0.5))]

    def render(self, name: str, labels: str) -> list[str]:
        out, acc = [], 0
        for b, c in zip(self.buckets, self.counts):
            acc += c
            out.append(f'{name}_bucket{{{labels}{"," if labels else ""}le="{b}"}} {acc}')
        acc += self.counts[-1]
        out.append(f'{name}_bucket{{{labels}{"," if labels else ""}le="+Inf"}} {acc}')
        out.append(f"{name}_sum{{{labels}}} {self.sum}")
        out.append(f"{name}_count{{{labels}}} {self.n}")
        return out


class EngineMetrics:
    def __init__(self, model_name: str = "model"):
        self.model_name = model_name
        self.lock = threading.Lock()
        self.prompt_tokens = 0
        self.generation_tokens = 0
        self.requests_success = 0
        self.requests_arrived = 0
        self.num_running = 0
        self.num_waiting = 0
        self.kv_usage = 0.0
        self.ttft = Histogram()
        self.tpot = Histogram()
        self.e2e = Histogram()
        self.step_prefill = Histogram()
        self.step_decode = Histogram()
        self._window: list[tuple[float, int]] = []
        self.preemptions = 0
        self.host_times: dict | None = None   # engine's host phase split (schedule / launch / wait / commit)

    def on_arrival(self, req) -> None:
        with self.lock:
            self.requests_arrived += 1
            self.prompt_tokens += len(req.prompt_ids)

    def on_step(self, batch, dt: float, done, sched, pages) -> None:
        now = time.perf_counter()
        with self.lock:
            gen = sum(1 for c in batch.chunks if c.sample)
            self.generation_tokens += gen
            (self.step_prefill if batch.mode == "prefill" else self.step_decode).observe(dt)
            self._window.append((now, gen))
            while self._window and now - self._window[0][0] > 10.0:
                self._window.pop(0)
            for r in done:
                self.requests_success += 1
                if r.ttft is not None:
                    self.ttft.observe(r.ttft)
                e2e = (r.finish_time or now) - r.arrival_time
                self.e2e.observe(e2e)
                if len(r.output_ids) > 1 and r.first_token_time is not None:
                    self.tpot.observe((now - r.first_token_time) / (len(r.output_ids) - 1))
            self.num_running, self.num_waiting = sched.num_running, sched.num_waiting
            self.kv_usage = pages.usage()
            self.preemptions = sched.num_preemptions

    def throughput(self) -> float:
        with self.lock:
            if len(self._window) < 2:
                return 0.0
            span = self._window[-1][0] - self._window[0][0]
            return sum(g for _, g in self._window) / span if span > 0 else 0.0

    def render(self) -> str:
        m = f'model_name="{self.model_name}"'
        thr = self.throughput()
        lines = []
        with self.lock:
            gauges = {
                "sglang:num_running_reqs": self.num_running, "sglang:num_queue_reqs": self.num_waiting,
                "sglang:token_usage": self.kv_usage, "sglang:gen_throughput": thr,
                "vllm:num_requests_running": self.num_running, "vllm:num_requests_waiting": self.num_waiting,
                "vllm:gpu_cache_usage_perc": self.kv_usage, "vllm:avg_generation_throughput_toks_per_s": thr,
            }
            counters = {
                "sglang:prompt_tokens_total": self.prompt_tokens,
                "sglang:generation_tokens_total": self.generation_tokens,
                "sglang:num_requests_total": self.requests_arrived,
                "vllm:prompt_tokens_total": self.prompt_tokens,
                "vllm:generation_tokens_total": self.generation_tokens,
                "vllm:request_success_total": self.requests_success,
                "ome:num_preemptions_total": self.preemptions,
            }
            for k, v in gauges.items():
                lines += [f"# TYPE {k} gauge", f"{k}{{{m}}} {v}"]
            for k, v in counters.items():
                lines += [f"# TYPE {k} counter", f"{k}{{{m}}} {v}"]
            if self.host_times:   # per-phase host time of the serving loop (SURVEY §5.1 step timer)
                lines.append("# TYPE ome:host_phase_seconds_total counter")
                lines += [f'ome:host_phase_seconds_total{{{m},phase="{ph}"}} {self.host_times[ph]}'
                          for ph in ("schedule", "launch", "wait", "commit") if ph in self.host_times]
            for name, h in (("sglang:time_to_first_token_seconds", self.ttft),
                            ("vllm:time_to_first_token_seconds", self.ttft),
                            ("sglang:time_per_output_token_seconds", self.tpot),
                            ("vllm:time_per_output_token_seconds", self.tpot),
                            ("sglang:e2e_request_latency_seconds", self.e2e),
                            ("vllm:e2e_request_latency_seconds", self.e2e),
                            ("ome:prefill_step_seconds", self.step_prefill),
                            ("ome:decode_step_seconds", self.step_decode)):
                lines.append(f"# TYPE {name} histogram")
                lines += h.render(name, m)
        return "\n".join(lines) + "\n"
