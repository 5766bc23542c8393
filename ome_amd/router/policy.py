"""Load-balancing policies for the router."""
from __future__ import annotations

import random
import threading


class Policy:
    name = "base"

    def pick(self, workers: list, text: str = "") -> object:
        raise NotImplementedError

    def on_done(self, worker, text: str = "") -> None:
        pass


class RoundRobinPolicy(Policy):
    name = "round_robin"

    def __init__(self):
        self.i = 0
        self.lock = threading.Lock()

    def pick(self, workers, text=""):
        with self.lock:
            w = workers[self.i % len(workers)]
            self.i += 1
            return w


class RandomPolicy(Policy):
    name = "random"

    def __init__(self, seed: int | None = None):
        self.rng = random.Random(seed)

    def pick(self, workers, text=""):
        return self.rng.choice(workers)


class PowerOfTwoPolicy(Policy):
    name = "power_of_two"

    def __init__(self, seed: int | None = None):
        self.rng = random.Random(seed)

    def pick(self, workers, text=""):
        if len(workers) == 1:
            return workers[0]
        a, b = self.rng.sample(workers, 2)
        return a if a.inflight <= b.inflight else b


class _Node:
    __slots__ = ("children", "owners")

    def __init__(self):
        self.children: dict[str, _Node] = {}
        self.owners: dict[str, float] = {}  # worker url -> last access tick


class PrefixTree:
    """Character-chunk radix approximation of each worker's prompt cache (``chunk`` chars per
    edge), with LRU eviction of a worker's entries beyond ``max_chars``."""

    def __init__(self, chunk: int = 16, max_chars: int = 1 << 22):
        self.root = _Node()
        self.chunk = chunk
        self.max_chars = max_chars
        self.chars: dict[str, int] = {}
        self.tick = 0
        self.lock = threading.Lock()

    def _edges(self, text: str):
        c = self.chunk
        return [text[i:i + c] for i in range(0, len(text), c)]

    def insert(self, text: str, worker: str) -> None:
        with self.lock:
            self.tick += 1
            node = self.root
            for e in self._edges(text):
                node = node.children.setdefault(e, _Node())
                if worker not in node.owners:
                    self.chars[worker] = self.chars.get(worker, 0) + len(e)
                node.owners[worker] = self.tick
            if self.chars.get(worker, 0) > self.max_chars:
                self._evict(worker)

    def match(self, text: str) -> tuple[dict[str, int], int]:
        """-> ({worker: matched chars}, total chars)."""
        out: dict[str, int] = {}
        with self.lock:
            node, depth = self.root, 0
            for e in self._edges(text):
                nxt = node.children.get(e)
                if nxt is None:
                    break
                depth += len(e)
                for w in nxt.owners:
                    out[w] = depth
                node = nxt
        return out, len(text)

    def _evict(self, worker: str) -> None:
        """Drop this worker's least-recently-used leaves until it is under 80% of budget."""
        target = self.max_chars * 0.8
        while self.chars.get(worker, 0) > target:
            leaves = []
            stack = [(self.root, None, None)]
            while stack:
                n, parent, key = stack.pop()
                owned_children = [k for k, ch in n.children.items() if worker in ch.owners]
                if parent is not None and worker in n.owners and not owned_children:
                    leaves.append((n.owners[worker], parent, key, n))
                stack.extend((ch, n, k) for k, ch in n.children.items())
            if not leaves:
                break
            leaves.sort(key=lambda t: t[0])
            for _, parent, key, n in leaves:
                if self.chars.get(worker, 0) <= target:
                    break
                n.owners.pop(worker, None)
                self.chars[worker] -= len(key)
                if not n.owners and not n.children:
                    parent.children.pop(key, None)

    def remove_worker(self, worker: str) -> None:
        with self.lock:
            stack = [self.root]
            while stack:
                n = stack.pop()
                n.owners.pop(worker, None)
                stack.extend(n.children.values())
            self.chars.pop(worker, None)


class CacheAwarePolicy(Policy):
    name = "cache_aware"

    def __init__(self, cache_threshold: float = 0.5, balance_abs_threshold: int = 32,
                 balance_rel_threshold: float = 1.5):
        self.tree = PrefixTree()
        self.th = cache_threshold
        self.abs_th = balance_abs_threshold
        self.rel_th = balance_rel_threshold

    def pick(self, workers, text=""):
        loads = [w.inflight for w in workers]
        mx, mn = max(loads), min(loads)
        imbalanced = mx - mn > self.abs_th and mx > mn * self.rel_th
        least = min(workers, key=lambda w: w.inflight)
        if imbalanced or not text:
            chosen = least
        else:
            matched, total = self.tree.match(text)
            best = max(workers, key=lambda w: (matched.get(w.url, 0), -w.inflight))
            ratio = matched.get(best.url, 0) / max(1, total)
            chosen = best if ratio > self.th else least
        if text:
            self.tree.insert(text, chosen.url)
        return chosen


def make_policy(name: str, **kw) -> Policy:
    return {"round_robin": RoundRobinPolicy, "random": RandomPolicy, "power_of_two": PowerOfTwoPolicy,
            "cache_aware": CacheAwarePolicy}[name](**kw)
