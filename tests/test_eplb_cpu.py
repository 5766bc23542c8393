"""EPLB (redundant experts + load-driven re-placement, parallel/eplb.py): placement algebra, and
a 2-rank DP-attention / EP engine on gloo with redundant experts and a mid-run rebalance that
must still generate exactly what a single rank generates."""
import json
import os
import random
import socket

import pytest
import torch
import torch.multiprocessing as mp

from ome_amd.parallel.eplb import ExpertPlacement, balance
from tests.test_dp_attention_cpu import PROMPTS, _checkpoint


def test_default_placement_matches_plain_ep():
    p = ExpertPlacement.default(8, 2, 0)
    assert p.phys_to_log == [[0, 1, 2, 3], [4, 5, 6, 7]]
    p = ExpertPlacement.default(8, 2, 2)
    assert p.slots == 5
    for r, row in enumerate(p.phys_to_log):
        assert len(set(row)) == len(row)  # never two copies on one rank
    rank, slot, n = p.tables("cpu")
    assert int(n.sum()) == 10 and all(p.phys_to_log[int(rank[e, j])][int(slot[e, j])] == e
                                      for e in range(8) for j in range(int(n[e])))


def test_balance_replicates_hot_experts_and_evens_ranks():
    rng = random.Random(0)
    E, ep, R = 64, 8, 8
    load = [rng.random() for _ in range(E)]
    load[3] = 40.0  # one very hot expert
    load[17] = 20.0
    p = balance(load, ep, (E + R) // ep)
    reps = p.replicas()
    assert len(reps[3]) >= 4 and len(reps[17]) >= 2
    assert len({r for r, _ in reps[3]}) == len(reps[3])  # replicas on distinct ranks
    assert all(len(row) == p.slots for row in p.phys_to_log)
    before = ExpertPlacement.default(E, ep, R).imbalance(load)
    after = p.imbalance(load)
    assert after < before and after < 1.25


def test_migrate_moves_rows(monkeypatch):
    """Single-process simulation of the all-to-all: every rank's new slots hold its new experts."""
    from ome_amd.parallel.eplb import migrate

    E, ep, R = 8, 2, 2
    old = ExpertPlacement.default(E, ep, R)
    new = balance([1, 1, 9, 1, 1, 1, 7, 1], ep, old.slots)
    weights = {r: torch.tensor([[float(e)] * 3 for e in old.phys_to_log[r]]) for r in range(ep)}
    # route each rank's sends through a mailbox
    box = {}

    def run(rank):
        def a2a(out, inp, out_splits, in_splits, group):
            box[rank] = (inp, in_splits)
            return out
        return a2a

    sends = {}
    for r in range(ep):
        migrate(old, new, weights[r], r, None, a2a=run(r))
        sends[r] = box[r]
    for r in range(ep):
        def a2a(out, inp, out_splits, in_splits, group, r=r):
            o = 0
            for src in range(ep):
                sinp, ssplit = sends[src]
                off = sum(ssplit[:r])
                n = out_splits[src]
                out[o:o + n].copy_(sinp[off:off + n])
                o += n
        got = migrate(old, new, weights[r], r, None, a2a=a2a)
        assert [int(x) for x in got[:, 0]] == new.phys_to_log[r]


def _worker(rank, world, port, path, q, tbo=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model_path=path, tp_size=world, dp_size=world, enable_dp_attention=True, device="cpu",
                            max_running_requests=8, context_length=256, dtype="float32",
                            ep_num_redundant_experts=2, eplb_rebalance_steps=3, enable_two_batch_overlap=tbo))
    assert eng.pstate.tbo == tbo
    m = eng.runner.model
    assert m.eplb is not None and m.E_local == (m.E + 2) // world
    if rank == 0:
        reqs = eng.generate(PROMPTS, SamplingParams(max_new_tokens=8, ignore_eos=True))
        eng.stop_group()
        q.put(([r.output_ids for r in reqs], m.eplb.rounds))
    else:
        eng.run_forever()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("kind,tbo", [("qwen3-moe", False), ("deepseek-v3", False), ("qwen3-moe", True),
                                      ("deepseek-v3", True)])
def test_eplb_engine_matches_single(tmp_path, kind, tbo):
    """(with ``tbo``: two-batch overlap of the EP all-to-alls on top of EPLB)"""
    _checkpoint(tmp_path, kind)
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    single = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", max_running_requests=8, context_length=256,
                               dtype="float32"))
    want = [r.output_ids for r in single.generate(PROMPTS, SamplingParams(max_new_tokens=8, ignore_eos=True))]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), q, tbo)) for r in range(2)]
    for p in ps:
        p.start()
    got, rounds = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert rounds >= 2  # experts were re-placed (and weights migrated) mid-generation
    assert got == want
