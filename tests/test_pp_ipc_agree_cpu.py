"""Pipeline IPC hand-off set-up is agreed across the engine group (parallel/state.py
``_pp_ipc_init``): when one rank fails to build a comm, EVERY rank closes its comms and falls back
to RCCL p2p, so no pair runs IPC against RCCL.  CPU / gloo, 2 ranks, a fake comm class that fails
on rank 1 only."""
import os
import socket

import torch.distributed as dist
import torch.multiprocessing as mp


class _FakeComm:
    closed = 0

    def __init__(self, group, max_bytes=0, cpu_group=None):
        if dist.get_rank() == int(os.environ["FAIL_RANK"]):
            raise RuntimeError("hipIpcOpenMemHandle failed (simulated)")
        self.alive = True

    def close(self):
        _FakeComm.closed += 1
        self.alive = False


def _worker(rank, port, fail_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FAIL_RANK=str(fail_rank))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from ome_amd.parallel import comm, state

    comm.CustomAllReduce = _FakeComm
    st = state.ParallelState()
    st.tp_size, st.tp_rank, st.pp_size, st.pp_rank = 1, 0, 2, rank
    st.cpu_group = dist.new_group([0, 1], backend="gloo")
    pair = dist.new_group([0, 1], backend="gloo")
    state._pp_ipc_init(st, {(0, 0): pair, (0, "all"): pair})
    q.put((rank, st.pp_prev is None and st.pp_next is None and st.pp_bcast is None, _FakeComm.closed))
    dist.destroy_process_group()


def _run(fail_rank):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, port, fail_rank, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_one_rank_failure_disables_ipc_everywhere():
    out = _run(fail_rank=1)
    # rank 0 built both of its comms and must close them; rank 1 built nothing
    assert out == [(0, True, 2), (1, True, 0)]


def test_all_ranks_ok_keeps_ipc():
    out = _run(fail_rank=-1)
    assert [(r, none) for r, none, _ in out] == [(0, False), (1, False)]
    assert all(closed == 0 for _, _, closed in out)
