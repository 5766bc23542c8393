"""KV page allocator and the device-resident request page tables.

``PagePool`` hands out page ids of the paged KV cache (a LIFO free list — recently freed
pages are still warm in the 256 MiB Infinity Cache).  When the native runtime library is
built, the free list lives in C++ (``csrc/omeio/runtime.cpp``), otherwise in Python.

``ReqSlotPool`` owns ``req_pages [max_reqs, max_pages]`` int32 on the GPU: each running
request gets a row, newly allocated pages are appended host-side and flushed to the device
in ONE small scatter per step, so attention metadata never re-uploads whole block tables
(the decode HIP graph gathers rows with ``index_select`` on device).
"""
from __future__ import annotations

import torch


class PagePool:
    def __init__(self, num_pages: int, reserved: int = 1):
        # page 0 is reserved as a scratch / padding page
        self.num_pages = num_pages
        self._free = list(range(num_pages - 1, reserved - 1, -1))

    @property
    def num_free(self) -> int:
        return len(self._free)

    def alloc(self, n: int) -> list[int] | None:
        if n > len(self._free):
            return None
        out = self._free[-n:]
        del self._free[-n:]
        out.reverse()
        return out

    def free(self, pages) -> None:
        self._free.extend(reversed(list(pages)))

    def usage(self) -> float:
        return 1.0 - len(self._free) / max(1, self.num_pages - 1)


class ReqSlotPool:
    def __init__(self, max_reqs: int, max_pages: int, device="cpu"):
        self.max_reqs, self.max_pages = max_reqs, max_pages
        self.table = torch.zeros(max_reqs, max_pages, dtype=torch.int32, device=device)
        # the last row is reserved for padded rows of bucketed decode graphs
        self._free = list(range(max_reqs - 2, -1, -1))
        self._rows: list[int] = []
        self._cols: list[int] = []
        self._vals: list[int] = []
        self.staging = None   # runtime.staging.H2DStaging (set by the model runner on a GPU)

    def alloc(self) -> int | None:
        return self._free.pop() if self._free else None

    def free(self, slot: int) -> None:
        self._free.append(slot)

    def set_pages(self, slot: int, start: int, pages: list[int]) -> None:
        if start + len(pages) > self.max_pages:
            raise ValueError("request exceeds max pages per sequence (context length)")
        n = len(pages)
        self._rows.extend([slot] * n)
        self._cols.extend(range(start, start + n))
        self._vals.extend(pages)

    def flush(self) -> None:
        if not self._rows:
            return
        import numpy as np

        host = np.asarray([self._rows, self._cols, self._vals], dtype=np.int64)
        if self.staging is not None:
            dev = self.staging.to_device(host)
        else:
            dev = torch.from_numpy(host).to(self.table.device)
        self.table.index_put_((dev[0], dev[1]), dev[2].to(torch.int32))
        self._rows, self._cols, self._vals = [], [], []
