"""Controller runtime: rate-limited work queues, watch -> enqueue mapping, and a manager.

Mirrors controller-runtime's model used by the reference (``cmd/manager/main.go``):
level-triggered ``reconcile(key) -> Result`` per kind, ``For`` / ``Owns`` / ``Watches``
wiring, requeue-after timers, exponential per-key backoff on errors.  The manager can run
controllers in worker threads (production) or drain them synchronously
(:meth:`Manager.run_until_idle`, used by the test-suite as the fake-client harness).
"""
from __future__ import annotations

import heapq
import logging
import threading
import time
import traceback
from dataclasses import dataclass
from typing import Callable, Iterable

from ome_amd.store.store import Store, WatchEvent, controller_of, group_of

log = logging.getLogger("ome_amd.controller")


@dataclass
class Result:
    requeue: bool = False
    requeue_after: float | None = None


Key = tuple[str, str]  # (namespace, name)


class WorkQueue:
    """Deduplicating queue with delayed adds and per-key exponential backoff."""

    def __init__(self, base_delay: float = 0.005, max_delay: float = 60.0):
        self._cv = threading.Condition()
        self._ready: list[Key] = []
        self._in_ready: set[Key] = set()
        self._delayed: list[tuple[float, int, Key]] = []
        self._seq = 0
        self._failures: dict[Key, int] = {}
        self._processing: set[Key] = set()
        self._dirty: set[Key] = set()
        self.base, self.max = base_delay, max_delay
        self.clock = time.monotonic

    def add(self, key: Key) -> None:
        with self._cv:
            if key in self._processing:
                self._dirty.add(key)
                return
            if key not in self._in_ready:
                self._in_ready.add(key)
                self._ready.append(key)
                self._cv.notify()

    def add_after(self, key: Key, delay: float) -> None:
        if delay <= 0:
            return self.add(key)
        with self._cv:
            self._seq += 1
            heapq.heappush(self._delayed, (self.clock() + delay, self._seq, key))
            self._cv.notify()

    def add_rate_limited(self, key: Key) -> None:
        n = self._failures.get(key, 0)
        self._failures[key] = n + 1
        self.add_after(key, min(self.max, self.base * (2 ** n)))

    def forget(self, key: Key) -> None:
        self._failures.pop(key, None)

    def _promote(self, now: float) -> None:
        while self._delayed and self._delayed[0][0] <= now:
            _, _, k = heapq.heappop(self._delayed)
            if k not in self._in_ready and k not in self._processing:
                self._in_ready.add(k)
                self._ready.append(k)
            elif k in self._processing:
                self._dirty.add(k)

    def get(self, timeout: float | None = None) -> Key | None:
        with self._cv:
            end = None if timeout is None else self.clock() + timeout
            while True:
                self._promote(self.clock())
                if self._ready:
                    k = self._ready.pop(0)
                    self._in_ready.discard(k)
                    self._processing.add(k)
                    return k
                wait = None
                if self._delayed:
                    wait = max(0.0, self._delayed[0][0] - self.clock())
                if end is not None:
                    rem = end - self.clock()
                    if rem <= 0:
                        return None
                    wait = rem if wait is None else min(wait, rem)
                self._cv.wait(wait)

    def done(self, key: Key) -> None:
        with self._cv:
            self._processing.discard(key)
            if key in self._dirty:
                self._dirty.discard(key)
                if key not in self._in_ready:
                    self._in_ready.add(key)
                    self._ready.append(key)
                    self._cv.notify()

    def fast_forward(self, horizon: float) -> int:
        """Promote delayed items due within ``horizon`` seconds (test harness)."""
        with self._cv:
            n = 0
            now = self.clock()
            keep = []
            for t, s, k in self._delayed:
                if t <= now + horizon:
                    if k not in self._in_ready and k not in self._processing:
                        self._in_ready.add(k)
                        self._ready.append(k)
                        n += 1
                else:
                    keep.append((t, s, k))
            heapq.heapify(keep)
            self._delayed = keep
            return n

    def __len__(self) -> int:
        return len(self._ready)

    @property
    def pending_delayed(self) -> int:
        return len(self._delayed)


class Controller:
    def __init__(self, name: str, store: Store, reconcile: Callable[[Key], Result | None],
                 for_kind: tuple[str, str], owns: Iterable[tuple[str, str]] = (),
                 watches: Iterable[tuple[str, Callable[[dict], Iterable[Key]]]] = ()):
        self.name, self.store, self.reconcile_fn = name, store, reconcile
        self.api_version, self.kind = for_kind
        self.queue = WorkQueue()
        self.owned_kinds = {k for _, k in owns}
        self.watch_map = list(watches)
        self.errors = 0
        self.reconciles = 0
        store.watch(self._on_primary, [self.kind])
        if self.owned_kinds:
            store.watch(self._on_owned, self.owned_kinds)
        for kind, mapper in self.watch_map:
            store.watch(lambda ev, m=mapper: self._on_mapped(ev, m), [kind])

    @staticmethod
    def key_of(obj: dict) -> Key:
        m = obj["metadata"]
        return (m.get("namespace") or "", m["name"])

    def _on_primary(self, ev: WatchEvent) -> None:
        if group_of(ev.obj.get("apiVersion", "v1")) == group_of(self.api_version):
            self.queue.add(self.key_of(ev.obj))

    def _on_owned(self, ev: WatchEvent) -> None:
        ref = controller_of(ev.obj)
        if ref and ref.get("kind") == self.kind:
            ns = ev.obj["metadata"].get("namespace") or ""
            self.queue.add((ns, ref["name"]))

    def _on_mapped(self, ev: WatchEvent, mapper) -> None:
        try:
            for k in mapper(ev.obj) or []:
                self.queue.add(k)
        except Exception:  # noqa: BLE001
            log.exception("%s: watch mapper failed", self.name)

    def process_one(self, timeout: float | None = 0.0) -> bool:
        key = self.queue.get(timeout=timeout)
        if key is None:
            return False
        try:
            self.reconciles += 1
            res = self.reconcile_fn(key) or Result()
            self.queue.forget(key)
            if res.requeue_after:
                self.queue.add_after(key, res.requeue_after)
            elif res.requeue:
                self.queue.add_rate_limited(key)
        except Exception as e:  # noqa: BLE001 — reconcile errors are retried with backoff
            self.errors += 1
            log.warning("%s reconcile %s failed: %s\n%s", self.name, key, e, traceback.format_exc(limit=4))
            self.last_error = e
            self.queue.add_rate_limited(key)
        finally:
            self.queue.done(key)
        return True

    def enqueue_all(self) -> None:
        for o in self.store.list(self.api_version, self.kind):
            self.queue.add(self.key_of(o))


class Manager:
    """Hosts controllers (ome-manager, ``cmd/manager/main.go``)."""

    def __init__(self, store: Store):
        self.store = store
        self.controllers: list[Controller] = []
        self._threads: list[threading.Thread] = []
        self._stop = threading.Event()
        self.runnables: list[Callable[[threading.Event], None]] = []
        self.leader = True

    def add(self, c: Controller) -> Controller:
        self.controllers.append(c)
        return c

    def add_runnable(self, fn: Callable[[threading.Event], None]) -> None:
        self.runnables.append(fn)

    def run_until_idle(self, max_iters: int = 10000, fast_forward: float = 0.0, rounds: int = 1) -> int:
        """Drain every queue synchronously.  ``fast_forward`` promotes requeue-after items due
        within that many seconds (``rounds`` times) so tests can step through timed requeues."""
        n = 0
        for r in range(max(1, rounds)):
            progressed = True
            while progressed and n < max_iters:
                progressed = False
                for c in self.controllers:
                    while c.process_one(timeout=0.0):
                        n += 1
                        progressed = True
                        if n >= max_iters:
                            break
            if fast_forward <= 0:
                break
            moved = sum(c.queue.fast_forward(fast_forward) for c in self.controllers)
            if not moved:
                break
        return n

    def start(self, workers_per_controller: int = 1) -> None:
        for c in self.controllers:
            c.enqueue_all()
            for i in range(workers_per_controller):
                t = threading.Thread(target=self._worker, args=(c,), name=f"ctrl-{c.name}-{i}", daemon=True)
                t.start()
                self._threads.append(t)
        for fn in self.runnables:
            t = threading.Thread(target=fn, args=(self._stop,), daemon=True)
            t.start()
            self._threads.append(t)

    def _worker(self, c: Controller) -> None:
        while not self._stop.is_set():
            c.process_one(timeout=0.2)

    def stop(self) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout=2)
