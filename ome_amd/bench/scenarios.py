"""Traffic-scenario grammar of the BenchmarkJob protocol (genai-bench compatible).

  N(mu_in,sigma_in)/(mu_out,sigma_out)  normal input/output token lengths
  D(in,out)                             deterministic lengths
  U(min_in,max_in)/(min_out,max_out)    uniform lengths; U(min,max) = uniform input, out = in-range
  E(n)                                  embeddings, n input tokens
  I(w,h) / I(w,h,n)                     image input (w x h, n images) — text-to-image-style tasks

Validation regexes mirror the reference webhook
(``pkg/webhook/admission/benchmark/benchmark_webhook.go:135-140``), with the mid-pattern
anchoring bug noted in SURVEY.md Appendix A fixed (every alternative is fully anchored).
"""
from __future__ import annotations

import random
import re
from dataclasses import dataclass

_NUM = r"\d+(?:\.\d+)?"
PATTERNS = {
    "N": re.compile(rf"^N\(({_NUM}),({_NUM})\)/\(({_NUM}),({_NUM})\)$"),
    "D": re.compile(r"^D\((\d+),(\d+)\)$"),
    "U2": re.compile(r"^U\((\d+),(\d+)\)/\((\d+),(\d+)\)$"),
    "U1": re.compile(r"^U\((\d+),(\d+)\)$"),
    "E": re.compile(r"^E\((\d+)(?:,(\d+))?\)$"),
    "I": re.compile(r"^I\((\d+),(\d+)(?:,(\d+))?\)$"),
}

TASK_SCENARIOS = {
    "text-to-text": ("N", "D", "U2", "U1"),
    "text-to-embeddings": ("E",),
    "image-text-to-text": ("I",),
    "image-to-text": ("I",),
    "image-to-embeddings": ("I",),
    "text-to-rerank": ("E",),
}

DEFAULT_SCENARIOS = {
    "text-to-text": ["N(480,240)/(300,150)", "D(100,100)", "D(100,1000)", "D(2000,200)", "D(7800,200)"],
    "text-to-embeddings": ["E(64)", "E(128)", "E(256)", "E(512)", "E(1024)"],
    "image-text-to-text": ["I(512,512)", "I(1024,512)", "I(2048,2048)"],
    "image-to-text": ["I(512,512)", "I(1024,512)", "I(2048,2048)"],
    "image-to-embeddings": ["I(512,512)", "I(1024,512)", "I(2048,2048)"],
    "text-to-rerank": ["E(64)", "E(128)"],
}
DEFAULT_CONCURRENCY = [1, 2, 4, 8, 16, 32, 64, 128, 256]


def validate(scenario: str, task: str = "text-to-text") -> bool:
    kinds = TASK_SCENARIOS.get(task)
    if kinds is None:
        return False
    s = scenario.replace(" ", "")
    return any(PATTERNS[k].match(s) for k in kinds)


@dataclass
class Scenario:
    text: str
    kind: str
    params: tuple

    @classmethod
    def parse(cls, text: str) -> "Scenario":
        s = text.replace(" ", "")
        for k, pat in PATTERNS.items():
            m = pat.match(s)
            if m:
                return cls(text, k, tuple(float(x) if x is not None else None for x in m.groups()))
        raise ValueError(f"invalid traffic scenario {text!r}")

    def sample(self, rng: random.Random, max_in: int = 1 << 30) -> tuple[int, int]:
        """(input_tokens, output_tokens) for one request."""
        p = self.params
        if self.kind == "N":
            i = int(round(rng.gauss(p[0], p[1])))
            o = int(round(rng.gauss(p[2], p[3])))
        elif self.kind == "D":
            i, o = int(p[0]), int(p[1])
        elif self.kind == "U2":
            i, o = rng.randint(int(p[0]), int(p[1])), rng.randint(int(p[2]), int(p[3]))
        elif self.kind == "U1":
            i = rng.randint(int(p[0]), int(p[1]))
            o = rng.randint(int(p[0]), int(p[1]))
        elif self.kind == "E":
            i, o = int(p[0]), 0
        else:  # image: token cost of a w x h image with 14px patches, 2x2 merge
            n = int(p[2] or 1)
            i, o = n * max(1, int(p[0]) // 28) * max(1, int(p[1]) // 28), 256
        return max(1, min(i, max_in)), max(0 if self.kind == "E" else 1, o)
