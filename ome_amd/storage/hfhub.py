"""Hugging Face Hub client of our own (``pkg/hfutil/hub``: ``repo.go`` ListRepoFiles /
SnapshotDownload, ``download.go`` GetHfFileMetadata / httpDownload).

* :meth:`HfHub.repo_info` — ``GET /api/models/{repo}/revision/{rev}?blobs=true``: commit sha and
  every file with its size and, for LFS files, the SHA-256 of its content.
* :meth:`HfHub.file_metadata` — ``HEAD /{repo}/resolve/{rev}/{file}`` without following the
  redirect: ``X-Repo-Commit``, ``X-Linked-Etag`` (LFS SHA-256) / ``ETag``, ``X-Linked-Size``.
* :func:`snapshot_download` — allow / ignore glob filters, then every file through the
  multipart ranged parallel downloader of :mod:`.objstore` (part files, resume, stitch), LFS files
  verified against their SHA-256; files already present with the right size and digest are kept.
  Large checkpoints therefore come down as many concurrent range requests per shard (the
  reference's xet / parallel hub downloader plays the same role).
"""
from __future__ import annotations

import fnmatch
import json
import os
import urllib.parse
import urllib.request
from pathlib import Path

from ome_amd.storage import objstore as O

HF_ENDPOINT = "https://huggingface.co"


class HfHubError(O.ObjectStoreError):
    pass


class _NoRedirect(urllib.request.HTTPRedirectHandler):
    def redirect_request(self, *a, **k):
        return None


class HfHub(O.ObjectStoreClient):
    """Also an :class:`~ome_amd.storage.objstore.ObjectStoreClient` (``bucket`` = ``repo@rev``) so
    the generic ranged downloader drives it."""
    provider = "huggingface"

    def __init__(self, endpoint: str | None = None, token: str | None = None, repo_type: str = "model"):
        self.endpoint = (endpoint or os.environ.get("HF_ENDPOINT") or HF_ENDPOINT).rstrip("/")
        self.token = token or os.environ.get("HF_TOKEN") or os.environ.get("HUGGING_FACE_HUB_TOKEN")
        self.repo_type = repo_type
        self.http = O._Http(None)

    def _headers(self) -> dict:
        h = {"User-Agent": "ome-amd/1.0", "Accept-Encoding": "identity"}
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        return h

    def _prefix(self) -> str:
        return "" if self.repo_type == "model" else f"{self.repo_type}s/"

    def resolve_url(self, repo: str, rev: str, path: str) -> str:
        return (f"{self.endpoint}/{self._prefix()}{repo}/resolve/{urllib.parse.quote(rev, safe='')}/"
                f"{urllib.parse.quote(path)}")

    def repo_info(self, repo: str, rev: str = "main") -> dict:
        api = {"model": "models", "dataset": "datasets", "space": "spaces"}[self.repo_type]
        url = f"{self.endpoint}/api/{api}/{repo}/revision/{urllib.parse.quote(rev, safe='')}?blobs=true"
        try:
            _, _, body = self.http("GET", url, self._headers())
        except O.ObjectStoreError as e:
            if e.status in (401, 403):
                raise HfHubError(f"{repo}: gated or private repository (token required)", e.status) from e
            if e.status == 404:
                raise HfHubError(f"{repo}@{rev}: repository or revision not found", 404) from e
            raise
        return json.loads(body)

    def files(self, repo: str, rev: str = "main") -> tuple[str, list[O.ObjectInfo]]:
        info = self.repo_info(repo, rev)
        out = []
        for s in info.get("siblings", []):
            lfs = s.get("lfs") or {}
            out.append(O.ObjectInfo(s["rfilename"], int(lfs.get("size", s.get("size", 0)) or 0),
                                    sha256_hex=lfs.get("sha256") or None, etag=s.get("blobId", "")))
        return info.get("sha", ""), out

    def file_metadata(self, repo: str, path: str, rev: str = "main") -> dict:
        req = urllib.request.Request(self.resolve_url(repo, rev, path), method="HEAD", headers=self._headers())
        opener = urllib.request.build_opener(_NoRedirect)
        try:
            r = opener.open(req, timeout=30)
        except urllib.error.HTTPError as e:
            if e.code not in (301, 302, 307, 308):
                raise HfHubError(f"HEAD {path}: HTTP {e.code}", e.code) from e
            r = e
        h = {k.lower(): v for k, v in r.headers.items()}
        etag = (h.get("x-linked-etag") or h.get("etag") or "").strip('"').removeprefix("W/").strip('"')
        return {"commit": h.get("x-repo-commit", ""), "etag": etag,
                "size": int(h.get("x-linked-size") or h.get("content-length") or 0),
                "location": h.get("location") or self.resolve_url(repo, rev, path)}

    # ObjectStoreClient surface for the ranged downloader: bucket = "<repo>@<rev>"
    def get_range(self, bucket, name, start, end):
        repo, rev = bucket.rsplit("@", 1)
        _, _, body = self.http("GET", self.resolve_url(repo, rev, name), {**self._headers(),
                                                                          "Range": f"bytes={start}-{end}"})
        return body


def _wanted(path: str, allow: list[str] | None, ignore: list[str] | None) -> bool:
    if allow and not any(fnmatch.fnmatch(path, p) for p in allow):
        return False
    return not (ignore and any(fnmatch.fnmatch(path, p) for p in ignore))


def snapshot_download(repo: str, local_dir: str | Path, revision: str = "main", token: str | None = None,
                      endpoint: str | None = None, allow_patterns: list[str] | None = None,
                      ignore_patterns: list[str] | None = None, part_size: int = O.DEFAULT_PART_SIZE,
                      workers: int = O.DEFAULT_WORKERS, progress=None, use_xet: bool = True) -> dict:
    """``use_xet``: LFS files that the hub serves from Xet storage (``X-Xet-Hash``) are rebuilt
    from their CAS xorbs (:mod:`.xet`); everything else goes through ranged HTTP."""
    hub = HfHub(endpoint, token)
    xc = None
    if use_xet and os.environ.get("OME_HF_XET", "1") != "0":
        from ome_amd.storage.xet import XetClient

        xc = XetClient(hub, workers=workers)
    sha, files = hub.files(repo, revision)
    files = [f for f in files if _wanted(f.name, allow_patterns, ignore_patterns)]
    local = Path(local_dir)
    local.mkdir(parents=True, exist_ok=True)
    total = sum(f.size for f in files)
    done = [0]

    def tick(n):
        done[0] += n
        if progress:
            progress({"phase": "Downloading", "totalBytes": total, "completedBytes": done[0],
                      "totalFiles": len(files)})

    stats = {"sha": sha, "files": 0, "bytes": 0, "parts": 0, "fetched_parts": 0, "verified": 0, "xet_files": 0}
    for f in files:
        if f.size == 0:   # small non-LFS files: the API may not report a size
            f.size = hub.file_metadata(repo, f.name, sha or revision)["size"]
        fd = xc.file_data(repo, f.name, sha or revision) if xc is not None and f.sha256_hex else None
        dest = local / f.name
        if fd is not None:
            if not (dest.exists() and dest.stat().st_size == f.size and O._file_sha256(dest) == f.sha256_hex):
                xc.download(repo, f.name, dest, sha or revision, size=f.size, sha256_hex=f.sha256_hex, fdata=fd)
            tick(f.size)
            stats["files"] += 1
            stats["xet_files"] += 1
            stats["bytes"] += f.size
            stats["verified"] += 1
            continue
        r = O.download_object(hub, f"{repo}@{sha or revision}", f, local / f.name, part_size, workers, tick)
        stats["files"] += 1
        stats["bytes"] += f.size
        stats["parts"] += r["parts"]
        stats["fetched_parts"] += r["fetched_parts"]
        stats["verified"] += int(bool(r["md5_verified"]))
    (local / ".ome-hf-commit").write_text(sha)
    stats["rate_limit_waits"] = list(hub.http.rate_limit_waits)
    return stats
