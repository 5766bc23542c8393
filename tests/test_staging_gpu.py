"""Mapped-memory copy kernel (runtime/staging.py): pinned host <-> device, aligned and unaligned
sizes, on a busy stream; the staging ring's H2D path."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 3, 4, 17, 1024, 4097, 65536 + 5])
def test_copy_h2d_d2h_roundtrip(n):
    from ome_amd.runtime.staging import copy_d2h, copy_h2d

    src = torch.randint(0, 255, (n,), dtype=torch.uint8).pin_memory()
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    big = torch.randn(4096, 4096, device="cuda")
    big @ big                                  # the copy queues behind real work
    copy_h2d(dev, src)
    back = torch.zeros(n, dtype=torch.uint8).pin_memory()
    copy_d2h(back, dev)
    torch.cuda.synchronize()
    assert torch.equal(back, src)
    assert torch.equal(dev.cpu(), src)


def test_staging_ring_values_and_reuse():
    from ome_amd.runtime.staging import H2DStaging

    st = H2DStaging("cuda", slots=2, init_bytes=64)
    outs = []
    for i in range(7):   # more rounds than slots, growing sizes (buffer reallocation)
        a = np.arange(10 * (i + 1), dtype=np.int32) * (i + 1)
        outs.append((a, st.to_device(a)))
    b = np.arange(12, dtype=np.int64).reshape(3, 4)
    d = st.to_device(b)
    torch.cuda.synchronize()
    for a, t in outs:
        assert t.dtype == torch.int32 and np.array_equal(t.cpu().numpy(), a)
    assert d.shape == (3, 4) and np.array_equal(d.cpu().numpy(), b)
