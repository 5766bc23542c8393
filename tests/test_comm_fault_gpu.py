"""Collective fault handling on the GPU (verdict r05, missing item 1): two ranks
share GPU 0 through the custom xGMI all-reduce; rank 1 is made to stall before publishing its
barrier flags (the OME_COMM_FAULT hook in csrc/comm/allreduce.hip).  Rank 0's bounded wait expires
(OME_COMM_SPIN_LIMIT), the expiry reaches the host-mapped error word without any HIP call, and
rank 0's watchdog ends the process non-zero (EXIT_COLLECTIVE) within the bound -- so the executor /
LWS can restart the group.  Both processes are gone afterwards (nothing left holding the GPU)."""
import os
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, stall_after, q, done):
    os.environ["OME_COMM_FAULT"] = "rank=1"             # arms the stall word (set_fault below)
    os.environ["OME_COMM_SPIN_LIMIT"] = str(1 << 14)    # ~tens of ms of flag polling per wait
    import torch.distributed as dist

    from ome_amd.parallel.comm import CustomAllReduce
    from ome_amd.runtime import watchdog as W

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    ar = CustomAllReduce(None, max_bytes=1 << 20, one_shot_max=256 << 10, blocks=4)
    x = torch.ones(4096, dtype=torch.bfloat16, device="cuda")
    for _ in range(3):   # healthy calls first: both ranks in step, no error recorded
        y = ar.all_reduce(x.clone())
        torch.cuda.synchronize()
        assert float(y[0]) == 2.0
    assert ar.host_error() == 0
    dist.barrier()
    if rank == 1:
        assert ar.set_fault(stall_after) == 0   # every later barrier: sleep before publishing
        ar.all_reduce(x.clone())
        torch.cuda.synchronize()
        q.put((rank, "stalled-call-done"))
        done.set()   # rank 1 no longer reads rank 0's IPC buffers
        return
    # rank 0: the engine's watchdog thread.  Production on_fire = log + stack dump + os._exit(75);
    # here the exit first waits until the stalled peer's kernel has finished, so no process frees
    # IPC-shared memory a live kernel on the same GPU still reads
    def fire(code, why):
        done.wait(60)
        os._exit(code)

    wd = W.Watchdog(60.0, rank=0, poll_s=0.01, on_fire=fire)
    t0 = time.monotonic()
    q.put((rank, "start"))
    ar.all_reduce(x.clone())   # its start barrier waits for rank 1's flags, which come too late
    torch.cuda.synchronize()
    for _ in range(500):       # the watchdog ends this process; reaching the end of the loop is a failure
        time.sleep(0.01)
    q.put((rank, f"not-killed after {time.monotonic() - t0:.1f}s, host_error={ar.host_error()}"))
    wd.stop()


def test_stalled_peer_makes_the_waiting_rank_exit_nonzero():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    done = ctx.Event()
    port = _port()
    # stall ~ 40000 x s_sleep(127) (~0.1-0.2 s) >> rank 0's 2^14-poll wait limit
    ps = [ctx.Process(target=_worker, args=(r, port, 40000, q, done)) for r in range(2)]
    for p in ps:
        p.start()
    t0 = time.monotonic()
    ps[0].join(timeout=120)
    ps[1].join(timeout=60)
    dt = time.monotonic() - t0
    alive = [p.is_alive() for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
            p.join(timeout=30)
    msgs = []
    while not q.empty():
        msgs.append(q.get_nowait())
    from ome_amd.runtime.watchdog import EXIT_COLLECTIVE

    assert not any(alive), (alive, msgs)
    assert ps[0].exitcode == EXIT_COLLECTIVE, (ps[0].exitcode, msgs)
    assert not any(m.startswith("not-killed") for _, m in msgs), msgs
    assert dt < 120
