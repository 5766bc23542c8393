"""Request / sampling-parameter objects of the first-party serving runtime."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import Any, Callable


@dataclass
class SamplingParams:
    max_new_tokens: int = 128
    temperature: float = 0.0
    top_p: float = 1.0
    top_k: int = -1
    min_p: float = 0.0
    stop_token_ids: list[int] = field(default_factory=list)
    stop: list[str] = field(default_factory=list)
    ignore_eos: bool = False
    seed: int | None = None
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    repetition_penalty: float = 1.0
    logprobs: bool = False
    n: int = 1

    @property
    def has_penalties(self) -> bool:
        return self.repetition_penalty != 1.0 or self.frequency_penalty != 0.0 or self.presence_penalty != 0.0

    def validate(self) -> None:
        if self.max_new_tokens < 0:
            raise ValueError("max_new_tokens must be >= 0")
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if not 0 < self.top_p <= 1:
            raise ValueError("top_p must be in (0, 1]")
        if self.top_k == 0 or self.top_k < -1:
            raise ValueError("top_k must be -1 or >= 1")
        if not 0 <= self.min_p <= 1:
            raise ValueError("min_p must be in [0, 1]")


class ReqState(enum.Enum):
    WAITING = "waiting"
    RUNNING = "running"
    FINISHED = "finished"


_rid = itertools.count()

# Placeholder for a token that was sampled on the GPU by an in-flight step but has not reached
# the host yet (overlapped scheduling); replaced in the step's final commit.
PENDING = -1


@dataclass(eq=False)
class Request:
    prompt_ids: list[int]
    params: SamplingParams = field(default_factory=SamplingParams)
    rid: str = field(default_factory=lambda: f"req-{next(_rid)}")
    output_ids: list[int] = field(default_factory=list)
    output_logprobs: list[float] = field(default_factory=list)
    state: ReqState = ReqState.WAITING
    num_cached: int = 0            # tokens whose K/V is resident in the paged cache
    num_prefix_hit: int = 0        # of those, how many came from the prefix cache
    pages: list[int] = field(default_factory=list)
    req_slot: int = -1             # row of the GPU page-table pool
    finish_reason: str | None = None
    arrival_time: float = field(default_factory=time.perf_counter)
    first_token_time: float | None = None
    finish_time: float | None = None
    token_times: list[float] = field(default_factory=list)
    on_token: Callable[["Request", list[int], bool], None] | None = None
    # PD disaggregation: KV arrives from a prefill engine instead of being computed here
    bootstrap: dict | None = None
    embedding: list[float] | None = None
    is_embedding: bool = False
    preempted: int = 0
    lora: str | None = None
    n_pending: int = 0             # placeholders in output_ids awaiting their sampled token
    pen_init: bool = False         # penalty count row initialised for the current req_slot
    dp_rank: int = 0               # DP attention: the rank whose scheduler owns the request
    pending_row: int = -1          # row of the newest pending token in its step's sampled output
    mm: Any = None                 # multimodal inputs (ome_amd.multimodal.MMInput): images, spans, M-RoPE

    @property
    def all_ids(self) -> list[int]:
        return self.prompt_ids + self.output_ids

    def token_at(self, pos: int) -> int:
        """``all_ids[pos]`` without building the concatenated list (hot in the step packing)."""
        n = len(self.prompt_ids)
        return self.prompt_ids[pos] if pos < n else self.output_ids[pos - n]

    def ids_range(self, a: int, b: int) -> list[int]:
        """``all_ids[a:b]`` without building the concatenated list."""
        n = len(self.prompt_ids)
        if b <= n:
            return self.prompt_ids[a:b]
        if a >= n:
            return self.output_ids[a - n:b - n]
        return self.prompt_ids[a:] + self.output_ids[:b - n]

    @property
    def seq_len(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def prefill_done(self) -> bool:
        # decode-ready: every token except the last one has K/V in cache; the last token is the
        # next decode input (a prompt whose final chunk left exactly one token is finished by a
        # decode step, which is the same computation as a 1-token prefill chunk)
        return self.num_cached >= self.seq_len - 1

    @property
    def ttft(self) -> float | None:
        return None if self.first_token_time is None else self.first_token_time - self.arrival_time

    @property
    def finished(self) -> bool:
        return self.state == ReqState.FINISHED
