"""Object-store clients + parallel ranged transfers (``pkg/storage``, ``pkg/ociobjectstore``).

The provider-neutral surface mirrors the reference's ``storage.Storage`` interface
(``pkg/storage/interfaces.go:25-48``: list / stat / get / put / delete plus multipart upload),
implemented over each provider's REST API with the standard library:

* :class:`S3Client`  — ListObjectsV2 (continuation tokens), HEAD/GET with ``Range``, PUT,
  multipart upload (Create / UploadPart / Complete / Abort); SigV4-signed (:mod:`.auth`).
* :class:`OciClient` — Object Storage ``/n/{ns}/b/{bucket}/o`` (list with ``start`` paging,
  ``fields=name,size,md5``), ranged GET, PUT, multipart ``/u`` uploads; OCI-signed.
* :class:`GcsClient` — JSON API list (``pageToken``), ``alt=media`` ranged download, media upload.
* :class:`AzureClient` — List Blobs (``marker``), ranged Get Blob (``x-ms-range``), Put Blob /
  Put Block + Put Block List; Shared Key, SAS or managed identity.

:func:`download_object` is the reference's multipart ranged parallel download
(``pkg/ociobjectstore/os_parallel_download.go:58-200``, ``providers/*/parallel.go``): the object
is cut into ``part_size`` ranges fetched by a worker pool into part files (a resumed download
keeps every part already complete), stitched into ``<file>.ome-part``, verified against the
provider's MD5 (hex ETag / base64 ``Content-MD5`` / ``md5Hash``; multipart checksums
``<md5>-<n>`` are not whole-object MD5s and are skipped, ``providers/oci/integrity.go:80-91``)
and atomically renamed.  :func:`upload_file` uses the provider's multipart upload above
``part_size``.
"""
from __future__ import annotations

import base64
import concurrent.futures as cf
import hashlib
import json
import os
import shutil
import threading
import time
import urllib.error
import urllib.parse
import urllib.request
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from pathlib import Path
from typing import Callable

from ome_amd.storage import auth as A

DEFAULT_PART_SIZE = 64 << 20
DEFAULT_WORKERS = 8


class ObjectStoreError(RuntimeError):
    def __init__(self, msg: str, status: int | None = None):
        super().__init__(msg)
        self.status = status


@dataclass
class ObjectInfo:
    name: str
    size: int
    md5_hex: str | None = None      # whole-object MD5 when the provider knows it
    etag: str = ""
    sha256_hex: str | None = None   # content SHA-256 (Hugging Face LFS objects)


def _md5_of(etag_or_md5: str | None, b64: bool) -> str | None:
    """Whole-object MD5 (hex) from a provider checksum, None for multipart composites."""
    if not etag_or_md5:
        return None
    v = etag_or_md5.strip('"')
    if "-" in v and v.rsplit("-", 1)[1].isdigit():
        return None
    try:
        return base64.b64decode(v).hex() if b64 else (v.lower() if len(v) == 32 else None)
    except ValueError:
        return None


class RateLimitError(ObjectStoreError):
    """HTTP 429 after the rate-limit retry budget (``waits``: seconds slept on this request)."""

    def __init__(self, msg: str, waits: list[float]):
        super().__init__(msg, 429)
        self.waits = waits


def retry_after_seconds(value: str | None, default: float) -> float:
    """``Retry-After`` as seconds: delta-seconds or an HTTP-date (RFC 9110 §10.2.3)."""
    if not value:
        return default
    value = value.strip()
    try:
        return max(0.0, float(value))
    except ValueError:
        pass
    try:
        import email.utils

        when = email.utils.parsedate_to_datetime(value)
        return max(0.0, when.timestamp() - time.time())
    except (TypeError, ValueError, OverflowError):
        return default


class _Http:
    """Tiny signed-request helper shared by the clients: retries 5xx / connection errors; HTTP 429
    honours ``Retry-After`` (capped at ``max_wait`` s) for ``rate_limit_retries`` attempts and
    records every wait in ``rate_limit_waits`` (the model agent turns them into
    ``model_agent_rate_limit_*`` metrics; reference ``pkg/modelagent/gopher.go:1134-1136``)."""

    def __init__(self, creds: A.Credentials | None, retries: int = 3, timeout: float = 60.0,
                 rate_limit_retries: int = 5, max_wait: float = 60.0, default_wait: float = 5.0):
        self.creds, self.retries, self.timeout = creds, retries, timeout
        self.rate_limit_retries, self.max_wait, self.default_wait = rate_limit_retries, max_wait, default_wait
        self.requests = 0
        self.rate_limit_waits: list[float] = []
        self._lock = threading.Lock()

    def __call__(self, method: str, url: str, headers: dict | None = None, body: bytes = b"",
                 ok=(200, 201, 204, 206)) -> tuple[int, dict, bytes]:
        last = None
        waits: list[float] = []
        attempt = 0
        while attempt < self.retries:
            h = dict(headers or {})
            u = url
            if isinstance(self.creds, A.AzureSas):
                u = self.creds.apply_url(url)
            elif self.creds is not None:
                h = self.creds.sign(method, url, h, body)
            req = urllib.request.Request(u, data=body if method in ("PUT", "POST") else None, method=method,
                                         headers=h)
            with self._lock:
                self.requests += 1
            try:
                with urllib.request.urlopen(req, timeout=self.timeout) as r:
                    return r.status, {k.lower(): v for k, v in r.headers.items()}, r.read()
            except urllib.error.HTTPError as e:
                data = e.read()
                if e.code in ok:
                    return e.code, {k.lower(): v for k, v in e.headers.items()}, data
                if e.code == 429:
                    if len(waits) >= self.rate_limit_retries:
                        raise RateLimitError(f"{method} {url}: HTTP 429 after {len(waits)} rate-limit waits "
                                             f"({sum(waits):.1f} s)", waits) from e
                    w = min(self.max_wait, retry_after_seconds(e.headers.get("Retry-After"), self.default_wait))
                    waits.append(w)
                    with self._lock:
                        self.rate_limit_waits.append(w)
                    time.sleep(w)
                    continue   # rate-limit waits do not use up the error retries
                if e.code < 500:
                    raise ObjectStoreError(f"{method} {url}: HTTP {e.code} {data[:200]!r}", e.code) from e
                last = ObjectStoreError(f"{method} {url}: HTTP {e.code}", e.code)
            except OSError as e:
                last = ObjectStoreError(f"{method} {url}: {e}")
            time.sleep(min(2.0, 0.1 * 2 ** attempt))
            attempt += 1
        raise last


class ObjectStoreClient:
    provider = ""

    def list(self, bucket: str, prefix: str = "") -> list[ObjectInfo]:
        raise NotImplementedError

    def stat(self, bucket: str, name: str) -> ObjectInfo:
        raise NotImplementedError

    def get_range(self, bucket: str, name: str, start: int, end: int) -> bytes:
        """Bytes [start, end] (inclusive)."""
        raise NotImplementedError

    def put(self, bucket: str, name: str, data: bytes) -> None:
        raise NotImplementedError

    def delete(self, bucket: str, name: str) -> None:
        raise NotImplementedError

    # multipart upload (default: not supported -> single put)
    def mpu_begin(self, bucket: str, name: str) -> str | None:
        return None

    def mpu_part(self, bucket: str, name: str, upload_id: str, number: int, data: bytes) -> str:
        raise NotImplementedError

    def mpu_complete(self, bucket: str, name: str, upload_id: str, parts: list[tuple[int, str]]) -> None:
        raise NotImplementedError

    def mpu_abort(self, bucket: str, name: str, upload_id: str) -> None:
        pass

    @property
    def requests(self) -> int:
        return self.http.requests


def _q(s: str, safe: str = "/") -> str:
    return urllib.parse.quote(s, safe=safe)


def _xml_find_all(root, tag):
    return [el for el in root.iter() if el.tag.rsplit("}", 1)[-1] == tag]


def _xml_text(el, tag, default=""):
    for c in el.iter():
        if c.tag.rsplit("}", 1)[-1] == tag:
            return c.text or default
    return default


# ------------------------------------------------------------------ S3
class S3Client(ObjectStoreClient):
    provider = "s3"

    def __init__(self, endpoint: str, creds: A.Credentials | None = None, region: str = "us-east-1"):
        self.endpoint = endpoint.rstrip("/")
        self.region = region
        if isinstance(creds, A.AwsKeys):
            creds.region = region
        self.http = _Http(creds)

    def _url(self, bucket: str, name: str = "", query: str = "") -> str:
        return f"{self.endpoint}/{bucket}" + (f"/{_q(name)}" if name else "") + (f"?{query}" if query else "")

    def list(self, bucket, prefix=""):
        out, token = [], None
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if token:
                q["continuation-token"] = token
            _, _, body = self.http("GET", self._url(bucket, query=urllib.parse.urlencode(sorted(q.items()))))
            root = ET.fromstring(body)
            for c in _xml_find_all(root, "Contents"):
                etag = _xml_text(c, "ETag")
                out.append(ObjectInfo(_xml_text(c, "Key"), int(_xml_text(c, "Size", "0")), _md5_of(etag, False), etag))
            if _xml_text(root, "IsTruncated", "false").lower() != "true":
                return out
            token = _xml_text(root, "NextContinuationToken")

    def stat(self, bucket, name):
        _, h, _ = self.http("HEAD", self._url(bucket, name))
        etag = h.get("etag", "")
        return ObjectInfo(name, int(h.get("content-length", 0)), _md5_of(etag, False), etag)

    def get_range(self, bucket, name, start, end):
        _, _, body = self.http("GET", self._url(bucket, name), {"Range": f"bytes={start}-{end}"})
        return body

    def put(self, bucket, name, data):
        self.http("PUT", self._url(bucket, name), {"Content-Length": str(len(data))}, data)

    def delete(self, bucket, name):
        self.http("DELETE", self._url(bucket, name), ok=(200, 204, 404))

    def mpu_begin(self, bucket, name):
        _, _, body = self.http("POST", self._url(bucket, name, "uploads="))
        return _xml_text(ET.fromstring(body), "UploadId")

    def mpu_part(self, bucket, name, upload_id, number, data):
        q = urllib.parse.urlencode({"partNumber": number, "uploadId": upload_id})
        _, h, _ = self.http("PUT", self._url(bucket, name, q), {"Content-Length": str(len(data))}, data)
        return h.get("etag", "")

    def mpu_complete(self, bucket, name, upload_id, parts):
        xml = "<CompleteMultipartUpload>" + "".join(
            f"<Part><PartNumber>{n}</PartNumber><ETag>{e}</ETag></Part>" for n, e in parts) + "</CompleteMultipartUpload>"
        self.http("POST", self._url(bucket, name, urllib.parse.urlencode({"uploadId": upload_id})), {}, xml.encode())

    def mpu_abort(self, bucket, name, upload_id):
        self.http("DELETE", self._url(bucket, name, urllib.parse.urlencode({"uploadId": upload_id})),
                  ok=(200, 204, 404))


# ------------------------------------------------------------------ OCI
class OciClient(ObjectStoreClient):
    provider = "oci"

    def __init__(self, endpoint: str, namespace: str, creds: A.Credentials | None = None):
        self.endpoint, self.ns = endpoint.rstrip("/"), namespace
        self.http = _Http(creds)

    def _o(self, bucket, name=""):
        return f"{self.endpoint}/n/{_q(self.ns, '')}/b/{_q(bucket, '')}/o" + (f"/{_q(name, '')}" if name else "")

    def list(self, bucket, prefix=""):
        out, start = [], None
        while True:
            q = {"prefix": prefix, "fields": "name,size,md5"}
            if start:
                q["start"] = start
            _, _, body = self.http("GET", self._o(bucket) + "?" + urllib.parse.urlencode(q))
            d = json.loads(body)
            for o in d.get("objects", []):
                out.append(ObjectInfo(o["name"], int(o.get("size", 0)), _md5_of(o.get("md5"), True), o.get("md5", "")))
            start = d.get("nextStartWith")
            if not start:
                return out

    def stat(self, bucket, name):
        _, h, _ = self.http("HEAD", self._o(bucket, name))
        md5 = h.get("content-md5") or h.get("opc-multipart-md5")
        return ObjectInfo(name, int(h.get("content-length", 0)), _md5_of(md5, True), h.get("etag", ""))

    def get_range(self, bucket, name, start, end):
        _, _, body = self.http("GET", self._o(bucket, name), {"Range": f"bytes={start}-{end}"})
        return body

    def put(self, bucket, name, data):
        self.http("PUT", self._o(bucket, name), {"Content-Type": "application/octet-stream",
                                                 "Content-Length": str(len(data))}, data)

    def delete(self, bucket, name):
        self.http("DELETE", self._o(bucket, name), ok=(200, 204, 404))

    def _u(self, bucket):
        return f"{self.endpoint}/n/{_q(self.ns, '')}/b/{_q(bucket, '')}/u"

    def mpu_begin(self, bucket, name):
        _, _, body = self.http("POST", self._u(bucket), {"Content-Type": "application/json"},
                               json.dumps({"object": name}).encode())
        return json.loads(body)["uploadId"]

    def mpu_part(self, bucket, name, upload_id, number, data):
        q = urllib.parse.urlencode({"uploadId": upload_id, "uploadPartNum": number})
        _, h, _ = self.http("PUT", f"{self._u(bucket)}/{_q(name, '')}?{q}",
                            {"Content-Type": "application/octet-stream", "Content-Length": str(len(data))}, data)
        return h.get("etag", "")

    def mpu_complete(self, bucket, name, upload_id, parts):
        body = json.dumps({"partsToCommit": [{"partNum": n, "etag": e} for n, e in parts]}).encode()
        self.http("POST", f"{self._u(bucket)}/{_q(name, '')}?uploadId={_q(upload_id, '')}",
                  {"Content-Type": "application/json"}, body)

    def mpu_abort(self, bucket, name, upload_id):
        self.http("DELETE", f"{self._u(bucket)}/{_q(name, '')}?uploadId={_q(upload_id, '')}", ok=(200, 204, 404))


# ------------------------------------------------------------------ GCS
class GcsClient(ObjectStoreClient):
    provider = "gcs"

    def __init__(self, endpoint: str = "https://storage.googleapis.com", creds: A.Credentials | None = None):
        self.endpoint = endpoint.rstrip("/")
        self.http = _Http(creds)

    def list(self, bucket, prefix=""):
        out, token = [], None
        while True:
            q = {"prefix": prefix}
            if token:
                q["pageToken"] = token
            _, _, body = self.http("GET", f"{self.endpoint}/storage/v1/b/{_q(bucket, '')}/o?{urllib.parse.urlencode(q)}")
            d = json.loads(body)
            for o in d.get("items", []):
                out.append(ObjectInfo(o["name"], int(o.get("size", 0)), _md5_of(o.get("md5Hash"), True),
                                      o.get("etag", "")))
            token = d.get("nextPageToken")
            if not token:
                return out

    def stat(self, bucket, name):
        _, _, body = self.http("GET", f"{self.endpoint}/storage/v1/b/{_q(bucket, '')}/o/{_q(name, '')}")
        o = json.loads(body)
        return ObjectInfo(o["name"], int(o.get("size", 0)), _md5_of(o.get("md5Hash"), True), o.get("etag", ""))

    def get_range(self, bucket, name, start, end):
        _, _, body = self.http("GET", f"{self.endpoint}/storage/v1/b/{_q(bucket, '')}/o/{_q(name, '')}?alt=media",
                               {"Range": f"bytes={start}-{end}"})
        return body

    def put(self, bucket, name, data):
        q = urllib.parse.urlencode({"uploadType": "media", "name": name})
        self.http("POST", f"{self.endpoint}/upload/storage/v1/b/{_q(bucket, '')}/o?{q}",
                  {"Content-Type": "application/octet-stream"}, data)

    def delete(self, bucket, name):
        self.http("DELETE", f"{self.endpoint}/storage/v1/b/{_q(bucket, '')}/o/{_q(name, '')}", ok=(200, 204, 404))


# ------------------------------------------------------------------ Azure
class AzureClient(ObjectStoreClient):
    provider = "azure"

    def __init__(self, endpoint: str, creds: A.Credentials | None = None):
        self.endpoint = endpoint.rstrip("/")     # https://<account>.blob.core.windows.net
        self.http = _Http(creds)

    def list(self, bucket, prefix=""):
        out, marker = [], None
        while True:
            q = {"restype": "container", "comp": "list", "prefix": prefix}
            if marker:
                q["marker"] = marker
            _, _, body = self.http("GET", f"{self.endpoint}/{bucket}?{urllib.parse.urlencode(q)}",
                                   {"x-ms-version": "2021-08-06"})
            root = ET.fromstring(body)
            for b in _xml_find_all(root, "Blob"):
                md5 = _xml_text(b, "Content-MD5")
                out.append(ObjectInfo(_xml_text(b, "Name"), int(_xml_text(b, "Content-Length", "0")),
                                      _md5_of(md5, True), _xml_text(b, "Etag")))
            marker = _xml_text(root, "NextMarker")
            if not marker:
                return out

    def stat(self, bucket, name):
        _, h, _ = self.http("HEAD", f"{self.endpoint}/{bucket}/{_q(name)}", {"x-ms-version": "2021-08-06"})
        return ObjectInfo(name, int(h.get("content-length", 0)), _md5_of(h.get("content-md5"), True), h.get("etag", ""))

    def get_range(self, bucket, name, start, end):
        _, _, body = self.http("GET", f"{self.endpoint}/{bucket}/{_q(name)}",
                               {"x-ms-range": f"bytes={start}-{end}", "x-ms-version": "2021-08-06"})
        return body

    def put(self, bucket, name, data):
        self.http("PUT", f"{self.endpoint}/{bucket}/{_q(name)}",
                  {"x-ms-blob-type": "BlockBlob", "Content-Length": str(len(data)), "x-ms-version": "2021-08-06",
                   "Content-MD5": base64.b64encode(hashlib.md5(data).digest()).decode()}, data)

    def delete(self, bucket, name):
        self.http("DELETE", f"{self.endpoint}/{bucket}/{_q(name)}", {"x-ms-version": "2021-08-06"}, ok=(200, 202, 404))

    def mpu_begin(self, bucket, name):
        return "blocks"       # Azure stages blocks under the blob name; no upload id

    def mpu_part(self, bucket, name, upload_id, number, data):
        bid = base64.b64encode(f"{number:08d}".encode()).decode()
        q = urllib.parse.urlencode({"comp": "block", "blockid": bid})
        self.http("PUT", f"{self.endpoint}/{bucket}/{_q(name)}?{q}",
                  {"Content-Length": str(len(data)), "x-ms-version": "2021-08-06"}, data)
        return bid

    def mpu_complete(self, bucket, name, upload_id, parts):
        xml = "<?xml version=\"1.0\" encoding=\"utf-8\"?><BlockList>" + "".join(
            f"<Latest>{b}</Latest>" for _, b in parts) + "</BlockList>"
        self.http("PUT", f"{self.endpoint}/{bucket}/{_q(name)}?comp=blocklist",
                  {"x-ms-version": "2021-08-06"}, xml.encode())


# ------------------------------------------------------------------ transfers
Progress = Callable[[int], None]


def _file_md5(path: Path) -> str:
    try:
        from ome_amd.io import native

        if native.available():
            return native.md5_file(path)
    except ImportError:
        pass
    h = hashlib.md5()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(8 << 20), b""):
            h.update(b)
    return h.hexdigest()


def _file_sha256(path: Path) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(8 << 20), b""):
            h.update(b)
    return h.hexdigest()


def _digest_ok(path: Path, obj: ObjectInfo) -> bool | None:
    """None: nothing to verify against; else whether the file matches the known digest."""
    if obj.sha256_hex:
        return _file_sha256(path) == obj.sha256_hex
    if obj.md5_hex:
        return _file_md5(path) == obj.md5_hex
    return None


def download_object(client: ObjectStoreClient, bucket: str, obj: ObjectInfo, dest: str | Path,
                    part_size: int = DEFAULT_PART_SIZE, workers: int = DEFAULT_WORKERS,
                    progress: Progress | None = None, verify: bool = True) -> dict:
    """Multipart ranged parallel download of one object with resumable part files.
    Returns ``{"parts", "fetched_parts", "bytes", "md5_verified"}``."""
    dest = Path(dest)
    dest.parent.mkdir(parents=True, exist_ok=True)
    if dest.exists() and dest.stat().st_size == obj.size and (not verify or _digest_ok(dest, obj) in (None, True)):
        return {"parts": 0, "fetched_parts": 0, "bytes": 0,
                "md5_verified": bool(obj.md5_hex or obj.sha256_hex), "skipped": True}
    pdir = dest.with_name(dest.name + ".ome-parts")
    pdir.mkdir(exist_ok=True)
    ranges = [(i, a, min(a + part_size, obj.size) - 1) for i, a in enumerate(range(0, max(obj.size, 1), part_size))]
    if obj.size == 0:
        ranges = []
    fetched = [0]
    lock = threading.Lock()

    def one(i, a, b):
        p = pdir / f"part-{i:05d}"
        if p.exists() and p.stat().st_size == b - a + 1:
            return                                   # resumed: this range is already on disk
        data = client.get_range(bucket, obj.name, a, b)
        if len(data) != b - a + 1:
            raise ObjectStoreError(f"short range read for {obj.name} [{a}, {b}]: {len(data)} bytes")
        tmp = p.with_name(p.name + ".tmp")
        tmp.write_bytes(data)
        os.replace(tmp, p)
        with lock:
            fetched[0] += 1
        if progress:
            progress(len(data))

    with cf.ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        for f in [ex.submit(one, *r) for r in ranges]:
            f.result()
    part = dest.with_name(dest.name + ".ome-part")
    with open(part, "wb") as out:
        for i, _, _ in ranges:
            with open(pdir / f"part-{i:05d}", "rb") as src:
                shutil.copyfileobj(src, out, 8 << 20)
    ok = _digest_ok(part, obj) if verify else None
    if ok is False:
        part.unlink(missing_ok=True)
        shutil.rmtree(pdir, ignore_errors=True)
        raise ObjectStoreError(f"{'SHA-256' if obj.sha256_hex else 'MD5'} mismatch for {obj.name}")
    os.replace(part, dest)
    shutil.rmtree(pdir, ignore_errors=True)
    return {"parts": len(ranges), "fetched_parts": fetched[0], "bytes": obj.size, "md5_verified": bool(ok)}


def download_prefix(client: ObjectStoreClient, bucket: str, prefix: str, dest_dir: str | Path,
                    part_size: int = DEFAULT_PART_SIZE, workers: int = DEFAULT_WORKERS,
                    progress: Callable[[dict], None] | None = None) -> dict:
    """Every object under ``prefix`` into ``dest_dir`` (paths relative to the prefix)."""
    objs = [o for o in client.list(bucket, prefix) if not o.name.endswith("/")]
    if not objs:
        raise ObjectStoreError(f"no objects under {bucket}/{prefix}")
    total = sum(o.size for o in objs)
    done = [0]
    t0 = time.time()
    lock = threading.Lock()

    def tick(n):
        with lock:
            done[0] += n
            if progress:
                progress({"phase": "Downloading", "totalBytes": total, "completedBytes": done[0],
                          "totalFiles": len(objs), "speedBytesPerSec": done[0] / max(time.time() - t0, 1e-6)})

    stats = {"files": 0, "bytes": 0, "parts": 0, "fetched_parts": 0, "verified": 0}
    for o in objs:
        # a prefix naming one object downloads it as its basename; otherwise paths below the prefix
        rel = o.name.rsplit("/", 1)[-1] if o.name == prefix else o.name[len(prefix):].lstrip("/")
        r = download_object(client, bucket, o, Path(dest_dir) / rel, part_size, workers, tick)
        stats["files"] += 1
        stats["bytes"] += o.size
        stats["parts"] += r["parts"]
        stats["fetched_parts"] += r["fetched_parts"]
        stats["verified"] += int(bool(r["md5_verified"]))
    stats["total_bytes"] = total
    stats["md5_manifest"] = {o.name: o.md5_hex for o in objs}
    return stats


def upload_file(client: ObjectStoreClient, bucket: str, name: str, path: str | Path,
                part_size: int = DEFAULT_PART_SIZE, workers: int = DEFAULT_WORKERS) -> int:
    """Upload one file; multipart (parallel parts) above ``part_size`` where the provider has it."""
    path = Path(path)
    size = path.stat().st_size
    uid = client.mpu_begin(bucket, name) if size > part_size else None
    if uid is None:
        client.put(bucket, name, path.read_bytes())
        return 1
    n_parts = -(-size // part_size)

    def one(i):
        with open(path, "rb") as f:
            f.seek(i * part_size)
            data = f.read(part_size)
        return i + 1, client.mpu_part(bucket, name, uid, i + 1, data)

    try:
        with cf.ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
            parts = sorted(ex.map(one, range(n_parts)))
        client.mpu_complete(bucket, name, uid, parts)
    except Exception:
        client.mpu_abort(bucket, name, uid)
        raise
    return n_parts


def upload_tree(client: ObjectStoreClient, bucket: str, prefix: str, src: str | Path, **kw) -> int:
    src = Path(src)
    n = 0
    for p in sorted(src.rglob("*")):
        if p.is_file() and not p.name.startswith(".ome-"):
            upload_file(client, bucket, (prefix.rstrip("/") + "/" if prefix else "") + str(p.relative_to(src)), p, **kw)
            n += 1
    return n


# ------------------------------------------------------------------ URI -> client
def _auth_config(provider: str, default_type: str) -> A.AuthConfig:
    raw = os.environ.get(f"OME_{provider.upper()}_AUTH") or os.environ.get("OME_STORAGE_AUTH")
    if raw:
        d = json.loads(raw)
        if d.get("provider", provider) == provider:
            return A.AuthConfig.from_dict({"provider": provider, **d})
    return A.AuthConfig(provider, default_type)


def client_for(uri_parts: dict, storage_type: str, creds: A.Credentials | None = None):
    """(client, bucket, prefix) for a parsed object-store URI when a remote endpoint is configured
    (``OME_<S3|OCI|GCS|AZURE>_ENDPOINT``, ``AWS_ENDPOINT_URL``, ``STORAGE_EMULATOR_HOST``, or
    ``OME_OBJECT_STORE_MODE=remote`` for the providers' public endpoints); None otherwise (the
    filesystem object-store root serves the URI)."""
    env = os.environ.get
    remote = env("OME_OBJECT_STORE_MODE") == "remote"
    f = A.DEFAULT_FACTORY

    def cred(provider, typ):
        if creds is not None:
            return creds
        try:
            return f.create(_auth_config(provider, typ))
        except A.AuthError:
            return None      # anonymous (public buckets, emulators)

    if storage_type == "S3":
        ep = env("OME_S3_ENDPOINT") or env("AWS_ENDPOINT_URL")
        region = uri_parts.get("region") or env("AWS_REGION") or "us-east-1"
        if not ep and not remote:
            return None
        ep = ep or f"https://s3.{region}.amazonaws.com"
        return S3Client(ep, cred(A.AWS, "AWSDefault"), region), uri_parts["bucket"], uri_parts["prefix"]
    if storage_type == "OCI":
        ep = env("OME_OCI_ENDPOINT")
        if not ep and not remote:
            return None
        ep = ep or f"https://objectstorage.{env('OCI_REGION', 'us-ashburn-1')}.oraclecloud.com"
        return (OciClient(ep, uri_parts["namespace"], cred(A.OCI, "OCIUserPrincipal")), uri_parts["bucket"],
                uri_parts["prefix"])
    if storage_type == "GCS":
        ep = env("OME_GCS_ENDPOINT") or env("STORAGE_EMULATOR_HOST")
        if not ep and not remote:
            return None
        return GcsClient(ep or "https://storage.googleapis.com", cred(A.GCP, "GCPDefault")), uri_parts["bucket"], \
            uri_parts["object"]
    if storage_type == "AZURE":
        ep = env("OME_AZURE_ENDPOINT")
        if not ep and not remote:
            return None
        ep = ep or f"https://{uri_parts['account']}.blob.core.windows.net"
        return AzureClient(ep, cred(A.AZURE, "AzureAccountKey")), uri_parts["container"], uri_parts["blob_path"]
    return None
