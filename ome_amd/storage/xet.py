"""Xet CAS download client for Hugging Face repositories (reference ``pkg/xet``: ``hf_adapter.rs``,
``xet_integration.rs``, ``xet_downloader.rs``, which drive xet-core's FileDownloader).

Protocol (per file):

1. ``HEAD {endpoint}/{repo}/resolve/{rev}/{path}`` without following redirects: a Xet-backed
   file answers with ``X-Xet-Hash`` (the file's merkle hash) and a ``Link`` header whose
   ``rel="xet-auth"`` target (or ``X-Xet-Refresh-Route``) is the token route.
2. ``GET`` the token route with the hub token: ``X-Xet-Cas-Url``, ``X-Xet-Access-Token``,
   ``X-Xet-Token-Expiration`` (unix seconds).  Tokens are cached per route and refreshed 30 s
   before they expire (``XetTokenManager``).
3. ``GET {cas}/reconstruction/{hash}`` (Bearer CAS token; optional ``Range`` for a byte range of
   the file): ``terms`` (xorb hash + chunk range + unpacked length, in file order),
   ``fetch_info`` (per xorb: chunk ranges with a presigned URL and the inclusive byte range to
   fetch) and ``offset_into_first_range``.
4. Every needed xorb byte range is fetched once (thread pool, shared by all terms that fall in
   it), decoded natively (``csrc/omeio/xet.cpp``: chunk headers, LZ4 frames, byte grouping) and
   the terms' chunk spans are written in order into a part file, which is SHA-256 verified
   against the LFS oid and renamed into place.

Files without ``X-Xet-Hash`` (plain LFS / git files) keep the multipart ranged HTTP path of
:mod:`.hfhub`.  No network in CI: ``tests/test_xet_cpu.py`` runs the whole protocol against a
local fake hub + CAS (parity with the public service unpinned offline).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import threading
import time
import urllib.error
import urllib.request
from dataclasses import dataclass
from pathlib import Path

from ome_amd.io import native
from ome_amd.storage import objstore as O


class XetError(O.ObjectStoreError):
    pass


@dataclass
class XetFileData:
    file_hash: str
    refresh_route: str


@dataclass
class XetConnection:
    endpoint: str
    access_token: str
    expiration: int


def parse_link_xet_auth(link: str) -> str | None:
    """URL of the ``rel="xet-auth"`` entry of a Link header."""
    for part in link.split(","):
        part = part.strip()
        if 'rel="xet-auth"' in part or "rel='xet-auth'" in part:
            a, b = part.find("<"), part.find(">")
            if 0 <= a < b:
                return part[a + 1:b]
    return None


def file_data_from_headers(h: dict) -> XetFileData | None:
    h = {k.lower(): v for k, v in h.items()}
    fh = h.get("x-xet-hash")
    if not fh:
        return None
    route = parse_link_xet_auth(h["link"]) if "link" in h else None
    route = route or h.get("x-xet-refresh-route")
    return XetFileData(fh, route) if route else None


def connection_from_headers(h: dict) -> XetConnection | None:
    h = {k.lower(): v for k, v in h.items()}
    try:
        return XetConnection(h["x-xet-cas-url"].rstrip("/"), h["x-xet-access-token"],
                             int(h["x-xet-token-expiration"]))
    except (KeyError, ValueError):
        return None


class _NoRedirect(urllib.request.HTTPRedirectHandler):
    def redirect_request(self, *a, **k):
        return None


class XetClient:
    def __init__(self, hub, workers: int = 8, refresh_margin_s: float = 30.0, timeout: float = 60.0):
        self.hub = hub                      # storage.hfhub.HfHub (endpoint, token, resolve_url)
        self.workers = workers
        self.prefetch = workers            # xorb ranges fetched / decoded ahead of the write position
        self.margin = refresh_margin_s
        self.timeout = timeout
        self._tokens: dict[str, XetConnection] = {}
        self._lock = threading.Lock()
        self.stats = {"token_fetches": 0, "xorb_ranges": 0, "xorb_bytes": 0, "files": 0}

    # ---------------------------------------------------------------- discovery / auth
    def file_data(self, repo: str, path: str, rev: str = "main") -> XetFileData | None:
        req = urllib.request.Request(self.hub.resolve_url(repo, rev, path), method="HEAD",
                                     headers=self.hub._headers())
        try:
            r = urllib.request.build_opener(_NoRedirect).open(req, timeout=self.timeout)
        except urllib.error.HTTPError as e:
            if e.code not in (301, 302, 307, 308):
                raise XetError(f"HEAD {path}: HTTP {e.code}", e.code) from e
            r = e
        return file_data_from_headers(dict(r.headers.items()))

    def connection(self, route: str) -> XetConnection:
        with self._lock:
            c = self._tokens.get(route)
            if c is not None and c.expiration - self.margin > time.time():
                return c
        req = urllib.request.Request(route, headers=self.hub._headers())
        try:
            r = urllib.request.urlopen(req, timeout=self.timeout)
        except urllib.error.HTTPError as e:
            raise XetError(f"xet token route {route}: HTTP {e.code}", e.code) from e
        c = connection_from_headers(dict(r.headers.items()))
        if c is None:   # some deployments answer in the body
            try:
                body = json.loads(r.read() or b"{}")
                c = XetConnection(body["casUrl"].rstrip("/"), body["accessToken"], int(body["exp"]))
            except (KeyError, ValueError) as e:
                raise XetError(f"xet token route {route}: no CAS connection info") from e
        with self._lock:
            self._tokens[route] = c
            self.stats["token_fetches"] += 1
        return c

    def reconstruction(self, conn: XetConnection, file_hash: str, byte_range: tuple[int, int] | None = None) -> dict:
        h = {"Authorization": f"Bearer {conn.access_token}", "User-Agent": "ome-amd/1.0"}
        if byte_range is not None:
            h["Range"] = f"bytes={byte_range[0]}-{byte_range[1]}"
        req = urllib.request.Request(f"{conn.endpoint}/reconstruction/{file_hash}", headers=h)
        try:
            return json.loads(urllib.request.urlopen(req, timeout=self.timeout).read())
        except urllib.error.HTTPError as e:
            raise XetError(f"reconstruction {file_hash}: HTTP {e.code}", e.code) from e

    # ---------------------------------------------------------------- data
    def _fetch(self, url: str, start: int, end: int) -> bytes:
        req = urllib.request.Request(url, headers={"Range": f"bytes={start}-{end}", "User-Agent": "ome-amd/1.0"})
        last = None
        for attempt in range(3):
            try:
                body = urllib.request.urlopen(req, timeout=self.timeout).read()
                if len(body) != end - start + 1:
                    raise XetError(f"xorb range {start}-{end}: got {len(body)} bytes")
                with self._lock:
                    self.stats["xorb_ranges"] += 1
                    self.stats["xorb_bytes"] += len(body)
                return body
            except (urllib.error.URLError, XetError, OSError) as e:
                last = e
                time.sleep(0.2 * (attempt + 1))
        raise XetError(f"xorb range fetch failed: {last}")

    def reconstruct(self, rec: dict, out) -> int:
        """Write the file described by a reconstruction response into the binary stream ``out``;
        returns the bytes written.

        Streams in file order: the xorb ranges are fetched + decoded by the worker pool at most
        ``self.prefetch`` ahead of the term being written, and a decoded range is dropped right
        after the last term that needs it, so peak memory is a few ranges (a few tens of MB),
        not the whole file (a 5 GB shard must fit the model-agent's memory limit)."""
        terms = rec.get("terms") or []
        fetch = rec.get("fetch_info") or {}
        plan = []
        for t in terms:
            h, cs, ce = t["hash"], t["range"]["start"], t["range"]["end"]
            ent = next((i for i, f in enumerate(fetch.get(h, []))
                        if f["range"]["start"] <= cs and ce <= f["range"]["end"]), None)
            if ent is None:
                raise XetError(f"no fetch range covers chunks {cs}-{ce} of xorb {h}")
            plan.append((h, ent, cs, ce, int(t.get("unpacked_length", -1))))
        # keys in order of first use, and the index of each key's last use
        order, last_use = [], {}
        for i, (h, ent, *_rest) in enumerate(plan):
            k = (h, ent)
            if k not in last_use:
                order.append(k)
            last_use[k] = i

        def fetch_decode(k):
            f = fetch[k[0]][k[1]]
            data, offs = native.xet_decode(self._fetch(f["url"], f["url_range"]["start"], f["url_range"]["end"]))
            return data, offs, f["range"]["start"]

        window = max(1, int(getattr(self, "prefetch", 0) or self.workers))
        skip = int(rec.get("offset_into_first_range", 0))
        written = 0
        live: dict = {}          # key -> future (submitted, not yet dropped)
        nxt = 0                  # next key of `order` to submit
        with cf.ThreadPoolExecutor(max(1, min(self.workers, len(order) or 1))) as ex:
            try:
                for i, (h, ent, cs, ce, ulen) in enumerate(plan):
                    k = (h, ent)
                    # keep `window` ranges in flight or decoded ahead of the write position
                    while nxt < len(order) and (len(live) < window or order[nxt] == k):
                        live[order[nxt]] = ex.submit(fetch_decode, order[nxt])
                        nxt += 1
                    with self._lock:
                        self.stats["peak_live_ranges"] = max(self.stats.get("peak_live_ranges", 0), len(live))
                    data, offs, first = live[k].result()
                    a, b = cs - first, ce - first
                    if b >= len(offs):
                        raise XetError(f"xorb {h}: fetched range holds {len(offs) - 1} chunks, term needs {b}")
                    piece = data[offs[a]:offs[b]]
                    if ulen >= 0 and len(piece) != ulen:
                        raise XetError(f"xorb {h} chunks {cs}-{ce}: {len(piece)} bytes, expected {ulen}")
                    if skip:
                        cut = min(skip, len(piece))
                        piece, skip = piece[cut:], skip - cut
                    out.write(piece)
                    written += len(piece)
                    del piece, data
                    if last_use[k] == i:
                        del live[k]      # the decoded range is no longer referenced
            finally:
                for fut in live.values():
                    fut.cancel()
        return written

    def download(self, repo: str, path: str, dest: str | Path, rev: str = "main", size: int | None = None,
                 sha256_hex: str | None = None, fdata: XetFileData | None = None) -> dict:
        """Download one Xet-backed file; raises XetError if the file is not Xet-backed."""
        fdata = fdata or self.file_data(repo, path, rev)
        if fdata is None:
            raise XetError(f"{path}: not a Xet-backed file")
        conn = self.connection(fdata.refresh_route)
        rec = self.reconstruction(conn, fdata.file_hash)
        dest = Path(dest)
        dest.parent.mkdir(parents=True, exist_ok=True)
        part = dest.with_name(dest.name + ".xet.part")
        try:
            with open(part, "wb") as f:
                n = self.reconstruct(rec, f)
        except BaseException:
            part.unlink(missing_ok=True)   # no half-written part file left behind
            raise
        if size is not None and n != size:
            os.unlink(part)
            raise XetError(f"{path}: reconstructed {n} bytes, expected {size}")
        if sha256_hex:
            h = hashlib.sha256()
            with open(part, "rb") as f:
                for blk in iter(lambda: f.read(8 << 20), b""):
                    h.update(blk)
            if h.hexdigest() != sha256_hex:
                os.unlink(part)
                raise XetError(f"{path}: SHA-256 mismatch after reconstruction")
        os.replace(part, dest)
        self.stats["files"] += 1
        return {"bytes": n, "xet_hash": fdata.file_hash, "verified": bool(sha256_hex)}
