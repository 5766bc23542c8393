"""Engine watchdog and collective fault handling (verdict r05, missing item 1).

The reference runs DeepSeek with ``--watchdog-timeout`` (``config/runtimes/srt/deepseek-rdma-pd-
rt.yaml:125-126``) and relies on LWS ``RecreateGroupOnPodRestart``
(``pkg/controller/v1beta1/inferenceservice/reconcilers/lws/lws_reconciler.go:98``): a rank whose
peer hangs must die non-zero so the group is rebuilt."""
import os
import subprocess
import sys
import textwrap
import threading
import time

import pytest

from ome_amd.runtime import watchdog as W


@pytest.fixture(autouse=True)
def _clean_sources():
    W.unregister_all()
    yield
    W.unregister_all()


def test_stuck_phase_fires_with_the_phase_name():
    fired = []
    wd = W.Watchdog(0.2, rank=3, poll_s=0.02, on_fire=lambda code, why: fired.append((code, why)))
    wd.enter("wait (decode, 256 rows)")
    t0 = time.monotonic()
    while not fired and time.monotonic() - t0 < 5:
        time.sleep(0.02)
    assert fired and fired[0][0] == W.EXIT_STUCK and "wait (decode, 256 rows)" in fired[0][1]
    wd.stop()


def test_idle_and_fresh_phases_never_fire():
    fired = []
    wd = W.Watchdog(0.3, poll_s=0.02, on_fire=lambda code, why: fired.append(code))
    for _ in range(20):   # a busy loop: every phase is short
        wd.enter("schedule")
        time.sleep(0.01)
        wd.enter("launch")
        time.sleep(0.01)
        wd.idle()
    time.sleep(0.5)       # idle for longer than the timeout: not a hang
    assert not fired
    wd.stop()


def test_collective_expiry_fires_and_check_comms_raises():
    err = {"v": 0}
    W.register_comm("allreduce(rank 0/2)", lambda: err["v"], lambda stall: 0)
    W.check_comms()
    fired = []
    wd = W.Watchdog(100.0, poll_s=0.02, on_fire=lambda code, why: fired.append((code, why)))
    err["v"] = 1
    t0 = time.monotonic()
    while not fired and time.monotonic() - t0 < 5:
        time.sleep(0.02)
    assert fired[0][0] == W.EXIT_COLLECTIVE and "allreduce(rank 0/2)" in fired[0][1]
    with pytest.raises(W.CommError):
        W.check_comms()
    wd.stop()


def test_fault_spec_and_injection():
    assert W.parse_fault("") is None
    f = W.parse_fault("rank=1,step=20,stall=5000")
    assert f == {"rank": 1, "step": 20, "stall": 5000}
    got = []
    W.register_comm("c", lambda: 0, lambda stall: got.append(stall) or 0)
    assert not W.maybe_inject(0, 20, f) and not W.maybe_inject(1, 19, f)
    assert W.maybe_inject(1, 20, f) and got == [5000]


def test_engine_marks_phases_and_a_stuck_step_exits_nonzero(tmp_path):
    """A real engine process whose GPU wait never returns: the watchdog ends it with EXIT_STUCK
    (the executor / LWS then restarts the group) instead of hanging forever."""
    code = textwrap.dedent("""
        import time
        from ome_amd.runtime.engine import Engine, EngineArgs
        from ome_amd.runtime.request import SamplingParams
        eng = Engine(EngineArgs(model="tiny-llama", device="cpu", dtype="float32", max_running_requests=4,
                                context_length=128, watchdog_timeout=1.0))
        phases = []
        orig = eng.watchdog.enter
        eng.watchdog.enter = lambda p: (phases.append(p), orig(p))[1]
        eng.generate([[1, 2, 3]], SamplingParams(max_new_tokens=2, ignore_eos=True))
        assert {"control", "schedule", "launch", "commit"} <= set(phases), phases
        assert any(p.startswith("wait (") for p in phases), phases
        print("PHASES-OK", flush=True)
        # now the device "hangs": the next step's result never arrives
        from ome_amd.runtime import model_runner
        def hang(self):
            time.sleep(3600)
        for cls in vars(model_runner).values():
            if isinstance(cls, type) and hasattr(cls, "result"):
                cls.result = hang
        eng.generate([[4, 5, 6]], SamplingParams(max_new_tokens=2, ignore_eos=True))
        print("UNREACHABLE", flush=True)
    """)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert "PHASES-OK" in p.stdout, p.stderr[-3000:]
    assert "UNREACHABLE" not in p.stdout
    assert p.returncode == W.EXIT_STUCK, (p.returncode, p.stderr[-3000:])
    assert "stuck" in p.stderr and "wait (" in p.stderr   # the stuck phase is named in the log
    assert "Thread" in p.stderr                            # every thread's stack was dumped


def test_watchdog_flag_reaches_engine_args():
    from ome_amd.runtime.server import build_parser, engine_args_from, validate_args

    ns = build_parser().parse_args(["--model-path", "random://tiny-llama", "--watchdog-timeout", "1000000"])
    validate_args(ns)
    assert engine_args_from(ns).watchdog_timeout == 1000000.0
    ns = build_parser().parse_args(["--model-path", "random://tiny-llama"])
    assert engine_args_from(ns).watchdog_timeout == 300.0   # SGLang's default


def test_lockstep_step_failure_on_comm_error_exits(monkeypatch):
    """A recorded collective expiry turns the completed step into an error; a multi-rank engine
    then runs on_fatal (exit 70 in production) instead of serving garbage."""
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model="tiny-llama", device="cpu", dtype="float32", max_running_requests=4,
                            context_length=128, watchdog_timeout=0))
    W.register_comm("allreduce(rank 0/2)", lambda: 1)
    monkeypatch.setattr(eng.pstate, "world_size", 2)   # rank 0 of a TP group, for the step error check
    eng._stop = False
    fatal = []
    eng.on_fatal = lambda: fatal.append(1)
    # straight into the scheduler: no control broadcast (there is no peer rank in this test)
    eng.scheduler.add(eng.make_request([1, 2, 3], SamplingParams(max_new_tokens=2, ignore_eos=True)))
    monkeypatch.setattr(eng, "_drain_inbox", lambda: None)
    t = threading.Thread(target=eng.run_forever, daemon=True)
    t.start()
    t.join(timeout=60)
    eng._stop = True
    W.unregister_all()
    assert fatal == [1] and not t.is_alive()
