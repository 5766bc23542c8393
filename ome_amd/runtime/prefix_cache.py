"""Page-granular prefix (radix) cache for the paged KV pool.

Full pages of finished requests stay resident, keyed by a hash chain over their token
content (h_i = BLAKE2b-128(h_{i-1} || tokens of page i): a collision-resistant digest, so a
match can never hand out another prompt's KV pages), so a new request whose prompt shares a prefix
reuses those pages instead of recomputing them (SGLang radix cache, which the reference's
runtimes keep enabled unless ``--disable-radix-cache``).  Pages matched by running requests
are pinned (refcount); unpinned pages are evicted LRU-deepest-first when the allocator runs
dry, and eviction of a page leaves its descendants unreachable so they are evicted next.

Multimodal requests pass a ``salt`` (digest of their images, :func:`ome_amd.multimodal.inputs.
mm_cache_key`) mixed into every page from the first image position on: their KV depends on pixels
the token ids do not capture.
"""
from __future__ import annotations

import hashlib
import heapq
import itertools
from array import array


class PrefixCache:
    def __init__(self, pool, page_size: int):
        self.pool, self.P = pool, page_size
        self.by_hash: dict[bytes, int] = {}        # chain digest -> page
        self.meta: dict[int, list] = {}            # page -> [hash, refcount, last_use, depth]
        self._clock = itertools.count()
        # eviction candidates: (last_use, -depth, page), pushed whenever a page becomes unpinned;
        # stale entries (re-pinned, re-used, evicted) are skipped when popped.  O(log n) per page
        # instead of sorting every cached page on each allocation miss (which stalled the engine
        # for tens of ms per step once the pool was full of cached prefixes).
        self._heap: list[tuple[int, int, int]] = []
        self.hits = 0
        self.queries = 0

    def _chain(self, tokens: list[int], salt: bytes = b"", salt_from: int = 0):
        n, P = len(tokens) // self.P, self.P
        if n == 0:
            return
        raw = array("q", tokens[:n * P]).tobytes()
        step = 8 * P
        h = b""
        for i in range(n):
            extra = salt if salt and (i + 1) * P > salt_from else b""
            h = hashlib.blake2b(h + raw[i * step:(i + 1) * step] + extra, digest_size=16).digest()
            yield i, h

    def match(self, tokens: list[int], salt: bytes = b"", salt_from: int = 0) -> list[int]:
        """Pin and return the cached pages covering the longest full-page prefix of ``tokens``."""
        self.queries += 1
        out = []
        t = next(self._clock)
        for _, h in self._chain(tokens, salt, salt_from):
            p = self.by_hash.get(h)
            if p is None:
                break
            m = self.meta[p]
            m[1] += 1
            m[2] = t
            out.append(p)
        if out:
            self.hits += 1
        return out

    def insert(self, tokens: list[int], pages: list[int], salt: bytes = b"", salt_from: int = 0) -> set[int]:
        """Offer a finished request's pages; returns the pages now owned by the cache (the
        caller frees the rest).  Unpins pages the request had matched."""
        kept: set[int] = set()
        t = next(self._clock)
        for i, h in self._chain(tokens, salt, salt_from):
            if i >= len(pages):
                break
            page = pages[i]
            cur = self.by_hash.get(h)
            if cur is None:
                if page in self.meta:  # page cached under another hash: cannot happen, be safe
                    continue
                self.by_hash[h] = page
                self.meta[page] = [h, 0, t, i]
                heapq.heappush(self._heap, (t, -i, page))
                kept.add(page)
            elif cur == page:
                m = self.meta[page]
                m[1] = max(0, m[1] - 1)
                m[2] = t
                if m[1] == 0:
                    heapq.heappush(self._heap, (t, -m[3], page))
                kept.add(page)
        # pages the request matched beyond its own computed prefix are still pinned: release
        for p in pages:
            if p in self.meta and p not in kept:
                self._unpin(p)
                kept.add(p)
        return kept

    def _unpin(self, p: int) -> None:
        m = self.meta[p]
        m[1] = max(0, m[1] - 1)
        if m[1] == 0:
            heapq.heappush(self._heap, (m[2], -m[3], p))

    def release(self, pages: list[int]) -> None:
        for p in pages:
            if p in self.meta:
                self._unpin(p)

    def owns(self, page: int) -> bool:
        return page in self.meta

    def evict(self, n: int) -> int:
        """Free up to ``n`` unpinned pages, least recently used (deepest first among equals)."""
        if n <= 0:
            return 0
        freed = []
        heap = self._heap
        while heap and len(freed) < n:
            t, negd, p = heapq.heappop(heap)
            m = self.meta.get(p)
            if m is None or m[1] != 0 or m[2] != t:
                continue            # stale: evicted, re-pinned or re-used since this push
            h = self.meta.pop(p)[0]
            self.by_hash.pop(h, None)
            freed.append(p)
        if len(heap) > 4 * max(64, len(self.meta)):   # drop accumulated stale entries
            self._heap = [(m[2], -m[3], p) for p, m in self.meta.items() if m[1] == 0]
            heapq.heapify(self._heap)
        self.pool.free(freed)
        return len(freed)

    @property
    def num_pages(self) -> int:
        return len(self.meta)
