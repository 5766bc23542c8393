"""Row-count-aware prefill chunk sizing for mixed steps.

A mixed step (prefill chunk + every running decode as a 1-token row) runs each projection GEMM
once over M = decode rows + prefill tokens.  On MI355X the GEMM time is a staircase in M, not a
line: the 256-row MFMA tiles (stream-K ``gemm_sk`` and hipBLASLt's MT256xN kernels) make M = 1056
cost what M = 1250 costs, and M = 544 cost 36 % more than M = 512 (Llama-3-8B, one layer's four
projections, cold weights: ``profiles/r06_m_staircase.txt``).  A scheduler that packs "whatever
is pending, up to ``chunked_prefill_size``" lands on the expensive side of a step about half the
time.

:class:`StepCost` holds t(M) -- the measured GEMM time of one decoder layer at M rows, on a
16-row grid -- and picks the prefill chunk p for a step with D decode rows and ``avail`` prompt
tokens ready so that the marginal cost per prompt token, (t(D + p) - t(D)) / p, is lowest among
the chunks that leave at most ``slack`` tokens behind (so prefill keeps pace with arrivals and
the leftover is bounded), the leftover priced at what a full-size chunk costs per token.  When everything pending is a small remainder whose best marginal cost
is far above a good chunk's, the prefill is deferred one step (bounded by ``max_defer`` steps,
counted in schedule() calls so TP / PP ranks stay in lockstep) to merge with the next arrivals.

Status (profiles/r06_step_cost_ab.txt): opt-in (``OME_STEP_COST=1``).  In-process the aggressive
form measured +1-2 % tokens/s at +6-12 ms p50 TTFT; over HTTP it cost 2-12 % (more, smaller eager
mixed steps compete with the server threads for the host), so the engine default stays the plain
chunk cap.

This is the MI355X-side complement to the reference runtimes' fixed ``--chunked-prefill-size``
(``config/runtimes/srt/meta/llama-3-8b-instruct-rt.yaml``): the flag still caps the chunk; the
cost table decides where below the cap to cut.  The table is measured by the model runner at
start-up on the model's own layer-0/1 projection weights (``ModelRunner.measure_step_cost``) and,
in lockstep mode, broadcast from rank 0 so every rank cuts identically.
"""
from __future__ import annotations

import os


class StepCost:
    G = 16   # row granularity of the table (the MFMA M tile)

    def __init__(self, table_us: list[float], slack: int | None = None, defer_ratio: float | None = None,
                 max_defer: int | None = None, tie: float = 0.02):
        """``table_us[i]``: GEMM time of one layer at M = (i + 1) * G rows ."""
        if not table_us:
            raise ValueError("empty step-cost table")
        self.t = [float(v) for v in table_us]
        self.slack = int(os.environ.get("OME_STEP_COST_SLACK", "256")) if slack is None else slack
        self.defer_ratio = float(os.environ.get("OME_STEP_COST_DEFER", "1.3")) if defer_ratio is None else defer_ratio
        self.max_defer = int(os.environ.get("OME_STEP_COST_MAX_DEFER", "1")) if max_defer is None else max_defer
        self.tie = tie
        # relative cost slack for preferring a cut on a prompt boundary (TTFT)
        self.ttft_tol = float(os.environ.get("OME_STEP_COST_TTFT_TOL", "0.05"))
        # below this many ready prompt tokens a step takes them all (no cut, no deferral): cutting
        # small prefills makes more, smaller mixed steps -- eager launches whose host cost the HTTP
        # server's threads compete for (profiles/r06_step_cost_ab.txt, HTTP block)
        self.min_avail = int(os.environ.get("OME_STEP_COST_MIN_AVAIL", "768"))

    @property
    def max_rows(self) -> int:
        return len(self.t) * self.G

    def at(self, m: int) -> float:
        """t(m): the table entry of the smallest grid row count >= m (0 rows cost nothing)."""
        if m <= 0:
            return 0.0
        i = min(len(self.t), -(-m // self.G)) - 1
        return self.t[i] if m <= self.max_rows else self.t[-1] * m / self.max_rows

    def marginal(self, d: int, p: int) -> float:
        return (self.at(d + p) - self.at(d)) / p

    def _cands(self, d: int, lo: int, hi: int) -> list[int]:
        """Chunk sizes in [lo, hi] worth evaluating: hi itself and every p that ends M on a grid
        boundary (the cost is flat between boundaries, so the largest p of each cell is the one)."""
        out = {hi}
        g = self.G
        m = -(-(d + lo) // g) * g
        while m - d <= hi:
            if m - d >= lo:
                out.add(m - d)
            m += g
        return sorted(out)

    def reference(self, d: int, cap: int) -> float:
        """What a prompt token left for a later step will cost there: the best marginal cost per
        token of a chunk of at least 2 x ``slack`` tokens (tiny chunks can reach a lower marginal
        cost, but not for every token: prefill has to keep pace with arrivals)."""
        lo = min(cap, max(1, 2 * self.slack))
        return min(self.marginal(d, p) for p in self._cands(d, lo, cap))

    def choose(self, d: int, avail: int, cap: int, deferred: int = 0, bounds: list[int] | None = None) -> int:
        """Prompt tokens to prefill this step (0 = defer).  ``d``: decode rows riding the step,
        ``avail``: prompt tokens ready, ``cap``: the chunked-prefill cap, ``deferred``: how many
        consecutive steps this prefill has been deferred.

        Minimises this step's added GEMM time plus the leftover priced at :meth:`reference`:
        cost(p) = t(d + p) - t(d) + (hi - p) * ref over p in [hi - slack, hi] (and p = 0 when the
        whole remainder is small and the deferral budget allows).  ``bounds``: cumulative token
        counts at which a prompt ends in admission order; a cut there within ``ttft_tol`` of the
        best cost is preferred (a prompt cut mid-way waits a whole extra step for its first token)."""
        hi = min(avail, cap)
        if hi <= 0:
            return 0
        if hi < self.min_avail:
            return hi
        ref = self.reference(d, cap)
        base = self.at(d)
        lo = max(1, hi - self.slack)
        cands = self._cands(d, lo, hi)
        ends = sorted({b for b in (bounds or ()) if lo <= b <= hi})
        cands = sorted(set(cands) | set(ends))
        if deferred < self.max_defer and hi <= self.slack < cap:
            cands = [0] + cands
        best_p, best_c = hi, None
        for p in cands:
            c = self.at(d + p) - base + (hi - p) * ref
            # near-ties go to the larger chunk (earlier first tokens for the same GEMM time)
            if best_c is None or c < best_c - self.tie * ref * self.G or (c <= best_c + self.tie * ref * self.G
                                                                          and p > best_p):
                best_p, best_c = p, c
        if ends and best_p not in ends and best_p != hi:
            # the largest prompt-boundary cut whose cost is within ttft_tol of the best
            slack_us = self.ttft_tol * (self.at(d + max(best_p, 1)) - base + (hi - best_p) * ref)
            for p in reversed(ends):
                if self.at(d + p) - base + (hi - p) * ref <= best_c + slack_us:
                    return p
        return best_p

    # ------------------------------------------------------------------ (de)serialisation
    def to_list(self) -> list[float]:
        return list(self.t)

    @classmethod
    def from_measurements(cls, rows: list[int], us: list[float], max_rows: int, **kw) -> "StepCost":
        """Grid table from (rows, time) samples: each grid cell takes the sample at or just above
        it.  Not smoothed: a row count that costs more than a larger one (a routing plan tuned at
        a neighbouring M) really does cost that at run time, and the chooser should avoid it."""
        pairs = sorted(zip(rows, us))
        n = -(-max_rows // cls.G)
        t = []
        j = 0
        for i in range(n):
            m = (i + 1) * cls.G
            while j < len(pairs) - 1 and pairs[j][0] < m:
                j += 1
            t.append(pairs[j][1])
        return cls(t, **kw)
