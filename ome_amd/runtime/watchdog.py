"""Engine watchdog and collective fault handling.

The reference's DeepSeek runtimes pass ``--watchdog-timeout`` to the engine
(``config/runtimes/srt/deepseek-rdma-pd-rt.yaml:125-126``) and rely on the LeaderWorkerSet
``RecreateGroupOnPodRestart`` policy (``pkg/controller/v1beta1/inferenceservice/reconcilers/lws/
lws_reconciler.go:98``) to rebuild a group once one of its ranks dies.  That only works if a rank
whose peer hung actually DIES: on an 8-GPU node the realistic failure is a rank stuck inside a
captured decode graph, with the others spinning in a peer-to-peer collective.

Three pieces close that loop here:

* the xGMI collectives (``csrc/comm/allreduce.hip``, ``csrc/comm/ep_ll.hip``) bound every flag
  wait (``OME_COMM_SPIN_LIMIT``) and, when a wait expires, also set a host-mapped error word that
  this module polls without any HIP call (a blocking copy could queue behind the hung work);
* :class:`Watchdog` -- a thread that tracks the engine loop's current phase (control broadcast,
  schedule, launch, wait for the GPU, commit).  A phase older than ``--watchdog-timeout`` seconds,
  or a recorded collective expiry, logs the stuck phase, dumps every thread's stack and ends the
  process NON-ZERO with ``os._exit`` (never a re-exec: the GPU may be initialised), so the executor
  / LWS restarts the whole group;
* fault injection: ``OME_COMM_FAULT="rank=R,step=S,stall=N"`` makes rank R's collectives sleep
  N x ``s_sleep 127`` before publishing their flags from engine step S on (the "delay a collective"
  hook of SURVEY §5.3(c)), so the expiry path is exercised by tests.
"""
from __future__ import annotations

import faulthandler
import logging
import os
import sys
import threading
import time
from typing import Callable

log = logging.getLogger("ome_amd.watchdog")

EXIT_COLLECTIVE = 75   # a bounded collective wait expired (a peer stalled or died)
EXIT_STUCK = 76        # an engine phase exceeded --watchdog-timeout

_lock = threading.Lock()
_sources: list[tuple[str, Callable[[], int], Callable[[int], int] | None]] = []


class CommError(RuntimeError):
    """A collective's bounded wait expired: this rank's peers did not arrive."""


def register_comm(name: str, host_error: Callable[[], int], set_fault: Callable[[int], int] | None = None) -> None:
    """Register a communicator's host-side error word (and its fault-injection setter)."""
    with _lock:
        _sources.append((name, host_error, set_fault))


def unregister_all() -> None:
    with _lock:
        _sources.clear()


def comm_errors() -> list[str]:
    """Names of the registered communicators whose bounded waits expired."""
    with _lock:
        srcs = list(_sources)
    bad = []
    for name, fn, _ in srcs:
        try:
            if fn():
                bad.append(name)
        except Exception:   # noqa: BLE001 -- a closed communicator is not a failure
            pass
    return bad


def check_comms() -> None:
    """Raise :class:`CommError` when any registered collective recorded an expired wait."""
    bad = comm_errors()
    if bad:
        raise CommError(f"collective wait expired on {', '.join(bad)} (peer rank stalled or died)")


def parse_fault(spec: str | None = None) -> dict | None:
    """``OME_COMM_FAULT="rank=1,step=20,stall=100000"`` -> {"rank": 1, "step": 20, "stall": 100000}."""
    spec = os.environ.get("OME_COMM_FAULT") if spec is None else spec
    if not spec:
        return None
    out = {"rank": 0, "step": 0, "stall": 100000}
    for part in spec.split(","):
        k, _, v = part.partition("=")
        if k.strip() in out and v.strip():
            out[k.strip()] = int(v)
    return out


def maybe_inject(rank: int, step: int, fault: dict | None) -> bool:
    """Arm the stall on this rank's communicators once ``step`` reaches the configured one."""
    if not fault or rank != fault["rank"] or step != fault["step"]:
        return False
    with _lock:
        srcs = list(_sources)
    n = 0
    for name, _, setter in srcs:
        if setter is not None and setter(int(fault["stall"])) == 0:
            n += 1
    log.warning("fault injection: rank %d stalls its collectives from step %d (%d communicators)", rank, step, n)
    return n > 0


class Watchdog:
    """Phase tracker + monitor thread.  ``enter(phase)`` at each phase boundary, ``idle()`` when the
    loop has nothing in flight; ``on_fire(code, reason)`` defaults to logging + ``os._exit(code)``."""

    def __init__(self, timeout_s: float, rank: int = 0, poll_s: float | None = None,
                 on_fire: Callable[[int, str], None] | None = None):
        self.timeout_s = float(timeout_s)
        self.rank = rank
        self.poll_s = poll_s if poll_s is not None else max(0.05, min(1.0, self.timeout_s / 10))
        self.on_fire = on_fire or self._exit
        self.phase = "idle"
        self.t_phase = time.monotonic()
        self.fired: tuple[int, str] | None = None
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="ome-watchdog", daemon=True)
        self._t.start()

    def enter(self, phase: str) -> None:
        self.t_phase = time.monotonic()
        self.phase = phase

    def idle(self) -> None:
        self.enter("idle")

    def stop(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            bad = comm_errors()
            if bad:
                self._fire(EXIT_COLLECTIVE, f"collective wait expired on {', '.join(bad)} during phase "
                                            f"'{self.phase}'")
                return
            phase, t0 = self.phase, self.t_phase
            age = time.monotonic() - t0
            if phase != "idle" and self.timeout_s > 0 and age > self.timeout_s:
                self._fire(EXIT_STUCK, f"engine phase '{phase}' stuck for {age:.1f} s "
                                       f"(--watchdog-timeout {self.timeout_s:g} s)")
                return

    def _fire(self, code: int, reason: str) -> None:
        self.fired = (code, reason)
        log.critical("watchdog (rank %d): %s; exiting with code %d", self.rank, reason, code)
        try:
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            sys.stderr.flush()
        except Exception:   # noqa: BLE001
            pass
        self.on_fire(code, reason)

    @staticmethod
    def _exit(code: int, reason: str) -> None:
        logging.shutdown()
        os._exit(code)


__all__ = ["CommError", "EXIT_COLLECTIVE", "EXIT_STUCK", "Watchdog", "check_comms", "comm_errors", "maybe_inject",
           "parse_fault", "register_comm", "unregister_all"]
