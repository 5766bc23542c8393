"""Cooperative TP checkpoint read into HBM (ShardExchange; the host-buffer + gloo form that
ranks sharing one GPU use): every rank's shards equal the plain rank-sliced load."""
import pytest

from tests.test_load_exchange_cpu import run_group

pytestmark = pytest.mark.gpu


def test_exchange_load_into_hbm(tmp_path):
    cfg, res, ckpt = run_group(tmp_path, 2, device="cuda")
    for r in range(2):
        assert all(res[r]["same"].values()), (r, res[r]["same"])
    assert sum(res[r]["ex_bytes"] for r in range(2)) <= ckpt * 1.05
