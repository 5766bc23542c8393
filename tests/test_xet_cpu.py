"""Xet CAS downloads (reference pkg/xet): native chunk / LZ4 decoding (csrc/omeio/xet.cpp) and the
whole protocol -- HEAD for X-Xet-Hash + xet-auth Link, token route headers with refresh on expiry,
reconstruction terms over several xorbs with shared fetch ranges, stored / LZ4 / byte-grouped
chunks, offset_into_first_range, SHA-256 verification -- against a local fake hub + CAS server.
The encoders below exist only to build fixtures (no lz4 module in the image); parity with the
public Xet service is unpinned offline."""
import hashlib
import json
import os
import struct
import sys
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd.io import native  # noqa: E402
from ome_amd.storage import hfhub, xet  # noqa: E402

pytestmark = pytest.mark.skipif(not native.available(), reason="libomeio not built")


# ------------------------------------------------------------------ fixture encoders
def lz4_block(data: bytes) -> bytes:
    """Greedy LZ4 block compressor (4-byte hash matches, last 5 bytes literal)."""
    out = bytearray()
    n, i, anchor = len(data), 0, 0
    table = {}

    def lenbytes(x):
        b = bytearray()
        while x >= 255:
            b.append(255)
            x -= 255
        b.append(x)
        return b

    while i + 12 <= n:
        key = data[i:i + 4]
        cand = table.get(key)
        table[key] = i
        if cand is not None and i - cand <= 0xFFFF and data[cand:cand + 4] == key:
            m = 4
            while i + m < n - 5 and data[cand + m] == data[i + m]:
                m += 1
            lit = data[anchor:i]
            tok_l, tok_m = min(len(lit), 15), min(m - 4, 15)
            out.append((tok_l << 4) | tok_m)
            if tok_l == 15:
                out += lenbytes(len(lit) - 15)
            out += lit
            out += struct.pack("<H", i - cand)
            if tok_m == 15:
                out += lenbytes(m - 4 - 15)
            i += m
            anchor = i
        else:
            i += 1
    lit = data[anchor:]
    tok_l = min(len(lit), 15)
    out.append(tok_l << 4)
    if tok_l == 15:
        out += lenbytes(len(lit) - 15)
    out += lit
    return bytes(out)


def lz4_frame(data: bytes, block: int = 1 << 16, content_size: bool = False, stored_tail: bool = False) -> bytes:
    flg = 0x40 | (0x08 if content_size else 0) | 0x20   # version 01, block independence
    hdr = bytearray(struct.pack("<I", 0x184D2204)) + bytes([flg, 0x40])
    if content_size:
        hdr += struct.pack("<Q", len(data))
    hdr.append(0)  # header checksum (not verified by the decoder)
    out = bytearray(hdr)
    for k in range(0, len(data), block):
        part = data[k:k + block]
        comp = lz4_block(part)
        if stored_tail and k + block >= len(data):
            out += struct.pack("<I", len(part) | 0x80000000) + part
        else:
            out += struct.pack("<I", len(comp)) + comp
    out += struct.pack("<I", 0)
    return bytes(out)


def group4(data: bytes) -> bytes:
    return b"".join(data[g::4] for g in range(4))


def chunk(data: bytes, scheme: int) -> bytes:
    payload = data if scheme == 0 else lz4_frame(data if scheme == 1 else group4(data))
    h = bytes([0]) + len(payload).to_bytes(3, "little") + bytes([scheme]) + len(data).to_bytes(3, "little")
    return h + payload


# ------------------------------------------------------------------ native decoding
def test_lz4_block_and_frame_roundtrip():
    rnd = os.urandom(3000)
    samples = [b"", b"a", b"abcd" * 1000, rnd, b"xyz" * 7 + rnd[:100] + b"xyz" * 300,
               bytes(range(256)) * 40 + b"\0" * 5000]
    for s in samples:
        assert native.lz4_decode(lz4_block(s), len(s), frame=False) == s
        assert native.lz4_decode(lz4_frame(s, block=1024), len(s)) == s
        assert native.lz4_decode(lz4_frame(s, content_size=True, stored_tail=True), len(s)) == s
    # overlapping back-reference: literal "ab" then match offset 2 length 10 -> "ab" * 6
    blk = bytes([(2 << 4) | 6]) + b"ab" + struct.pack("<H", 2) + bytes([0x10]) + b"!"
    assert native.lz4_decode(blk, 13, frame=False) == b"ab" * 6 + b"!"
    with pytest.raises(native.OmeIOError):   # offset reaching before the output start
        native.lz4_decode(bytes([0x14]) + b"a" + struct.pack("<H", 9) + bytes([0]), 64, frame=False)
    with pytest.raises(native.OmeIOError):   # output capacity too small
        native.lz4_decode(lz4_block(b"q" * 100), 50, frame=False)


def test_xet_chunk_run_decoding():
    parts = [os.urandom(777), b"hello world " * 400, bytes(range(256)) * 33 + b"tail", b""]
    blob = b"".join(chunk(p, s) for p, s in zip(parts, (0, 1, 2, 1)))
    data, offs = native.xet_decode(blob)
    assert data == b"".join(parts)
    assert offs == [0, 777, 777 + 4800, 777 + 4800 + 8452, 777 + 4800 + 8452]
    with pytest.raises(native.OmeIOError):
        native.xet_decode(blob[:-3])              # truncated payload
    bad = bytearray(chunk(b"abc", 0))
    bad[4] = 7
    with pytest.raises(native.OmeIOError):
        native.xet_decode(bytes(bad))             # unknown scheme


# ------------------------------------------------------------------ fake hub + CAS
class FakeXetHub:
    def __init__(self, token_ttl: int = 3600):
        rnd = os.urandom(20000)
        # file A: 3 xorbs' worth of chunks; file B shares xorb X1 (dedup across files)
        self.chunks = {"X1": [rnd[:4000], b"abc" * 2000, rnd[4000:9000]],
                       "X2": [b"model weights " * 500, rnd[9000:12000], bytes(range(256)) * 20],
                       "X3": [rnd[12000:20000]]}
        self.schemes = {"X1": (0, 1, 2), "X2": (1, 0, 2), "X3": (1,)}
        self.xorbs, self.chunk_bytes = {}, {}
        for h, cs in self.chunks.items():
            enc = [chunk(c, s) for c, s in zip(cs, self.schemes[h])]
            self.chunk_bytes[h] = [0]
            for e in enc:
                self.chunk_bytes[h].append(self.chunk_bytes[h][-1] + len(e))
            self.xorbs[h] = b"".join(enc)
        self.terms = {"hashA": [("X1", 0, 2), ("X2", 0, 3), ("X1", 2, 3), ("X3", 0, 1)],
                      "hashB": [("X2", 1, 3), ("X1", 1, 2)]}
        self.files = {"model.safetensors": self.content("hashA"), "extra.bin": self.content("hashB"),
                      "config.json": b'{"model_type": "llama"}'}
        self.xet = {"model.safetensors": "hashA", "extra.bin": "hashB"}
        self.ttl = token_ttl
        self.token_gets = 0
        self.recon_gets = 0
        self.xorb_gets = 0
        self.cdn_gets = 0
        self.tokens = set()
        hub = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body=b"", headers=None):
                self.send_response(code)
                for k, v in (headers or {}).items():
                    self.send_header(k, v)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                if self.command != "HEAD":
                    self.wfile.write(body)

            def do_HEAD(self):
                self.do_GET()

            def do_GET(self):
                u = urllib.parse.urlsplit(self.path)
                path = urllib.parse.unquote(u.path)
                base = f"http://127.0.0.1:{self.server.server_address[1]}"
                if path.startswith("/api/models/org/x/revision/"):
                    sib = [{"rfilename": k, "lfs": {"sha256": hashlib.sha256(v).hexdigest(), "size": len(v)}}
                           if k in hub.xet else {"rfilename": k, "size": len(v)} for k, v in hub.files.items()]
                    return self._send(200, json.dumps({"sha": "c" * 40, "siblings": sib}).encode())
                if path.startswith("/api/models/org/x/xet-read-token/"):
                    if self.headers.get("Authorization") != "Bearer hf_tok":
                        return self._send(401)
                    hub.token_gets += 1
                    tok = f"cas{hub.token_gets}"
                    hub.tokens.add(tok)
                    return self._send(200, b"{}", {"X-Xet-Cas-Url": base + "/cas", "X-Xet-Access-Token": tok,
                                                   "X-Xet-Token-Expiration": str(int(time.time()) + hub.ttl)})
                if path.startswith("/cas/reconstruction/"):
                    auth = self.headers.get("Authorization", "")
                    if auth.removeprefix("Bearer ") not in hub.tokens:
                        return self._send(401)
                    hub.recon_gets += 1
                    fh = path.rsplit("/", 1)[1]
                    terms = [{"hash": h, "unpacked_length": sum(len(c) for c in hub.chunks[h][a:b]),
                              "range": {"start": a, "end": b}} for h, a, b in hub.terms[fh]]
                    # one fetch range per xorb covering every chunk any term of this file needs
                    fi = {}
                    for h, a, b in hub.terms[fh]:
                        lo, hi = fi.get(h, (a, b))
                        fi[h] = (min(lo, a), max(hi, b))
                    fetch = {h: [{"range": {"start": a, "end": b}, "url": f"{base}/xorb/{h}",
                                  "url_range": {"start": hub.chunk_bytes[h][a], "end": hub.chunk_bytes[h][b] - 1}}]
                             for h, (a, b) in fi.items()}
                    return self._send(200, json.dumps({"offset_into_first_range": 0, "terms": terms,
                                                       "fetch_info": fetch}).encode())
                if path.startswith("/xorb/"):
                    hub.xorb_gets += 1
                    h = path.rsplit("/", 1)[1]
                    a, b = (int(x) for x in self.headers["Range"].split("=")[1].split("-"))
                    return self._send(206, hub.xorbs[h][a:b + 1])
                if path.startswith("/cdn/"):
                    hub.cdn_gets += 1
                    data = hub.files[path[len("/cdn/"):]]
                    rng = self.headers.get("Range")
                    if rng:
                        a, b = (int(x) for x in rng.split("=")[1].split("-"))
                        return self._send(206, data[a:b + 1])
                    return self._send(200, data)
                if "/resolve/" in path:
                    name = path.split("/resolve/", 1)[1].split("/", 1)[1]
                    data = hub.files[name]
                    h = {"X-Repo-Commit": "c" * 40, "X-Linked-Size": str(len(data)), "Location": f"{base}/cdn/{name}"}
                    if name in hub.xet:
                        h["X-Xet-Hash"] = hub.xet[name]
                        h["Link"] = (f'<{base}/api/models/org/x/xet-read-token/{"c" * 40}>; rel="xet-auth", '
                                     f'<{base}/cas/reconstruction/{hub.xet[name]}>; rel="xet-reconstruction-info"')
                    if self.command == "HEAD":
                        return self._send(302, b"", h)
                    return self._send(302, b"", h)
                return self._send(404)

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def content(self, fh):
        return b"".join(b"".join(self.chunks[h][a:b]) for h, a, b in self.terms[fh])

    def close(self):
        self.srv.shutdown()


@pytest.fixture
def hub():
    h = FakeXetHub()
    yield h
    h.close()


def test_header_parsing():
    link = ('<https://huggingface.co/api/models/t/xet-read-token/abc>; rel="xet-auth", '
            '<https://cas/reconstruction/h>; rel="xet-reconstruction-info"')
    assert xet.parse_link_xet_auth(link) == "https://huggingface.co/api/models/t/xet-read-token/abc"
    fd = xet.file_data_from_headers({"X-Xet-Hash": "h1", "X-Xet-Refresh-Route": "https://r"})
    assert fd.file_hash == "h1" and fd.refresh_route == "https://r"
    assert xet.file_data_from_headers({"ETag": "x"}) is None
    c = xet.connection_from_headers({"X-Xet-Cas-Url": "https://cas/", "X-Xet-Access-Token": "t",
                                     "X-Xet-Token-Expiration": "1758055996"})
    assert (c.endpoint, c.access_token, c.expiration) == ("https://cas", "t", 1758055996)


def test_xet_file_download_and_dedup(hub, tmp_path):
    h = hfhub.HfHub(hub.url, token="hf_tok")
    xc = xet.XetClient(h, workers=4)
    fd = xc.file_data("org/x", "model.safetensors")
    assert fd.file_hash == "hashA" and fd.refresh_route.endswith("/xet-read-token/" + "c" * 40)
    want = hub.files["model.safetensors"]
    r = xc.download("org/x", "model.safetensors", tmp_path / "m.st", size=len(want),
                    sha256_hex=hashlib.sha256(want).hexdigest())
    assert (tmp_path / "m.st").read_bytes() == want and r["verified"]
    # X1 is used by two terms but fetched once (one covering range per xorb)
    assert hub.xorb_gets == 3 and hub.token_gets == 1
    xc.download("org/x", "extra.bin", tmp_path / "e.bin")
    assert (tmp_path / "e.bin").read_bytes() == hub.files["extra.bin"]
    assert hub.token_gets == 1, "token reused until close to expiry"
    with pytest.raises(xet.XetError):   # wrong digest: part file removed, nothing renamed
        xc.download("org/x", "extra.bin", tmp_path / "bad.bin", sha256_hex="0" * 64)
    assert not (tmp_path / "bad.bin").exists() and not list(tmp_path.glob("*.part"))
    with pytest.raises(xet.XetError):
        xc.download("org/x", "config.json", tmp_path / "c.json")   # not Xet-backed


def test_token_refresh_and_offset_into_first_range(tmp_path):
    hub = FakeXetHub(token_ttl=10)   # inside the 30 s refresh margin: every call refreshes
    try:
        xc = xet.XetClient(hfhub.HfHub(hub.url, token="hf_tok"))
        fd = xc.file_data("org/x", "extra.bin")
        xc.connection(fd.refresh_route)
        xc.connection(fd.refresh_route)
        assert hub.token_gets == 2
        # a reconstruction for a byte range starts mid-chunk: the first bytes are skipped
        conn = xc.connection(fd.refresh_route)
        rec = xc.reconstruction(conn, "hashB")
        rec["offset_into_first_range"] = 123
        import io

        buf = io.BytesIO()
        n = xc.reconstruct(rec, buf)
        assert buf.getvalue() == hub.files["extra.bin"][123:] and n == len(hub.files["extra.bin"]) - 123
    finally:
        hub.close()


def test_snapshot_download_uses_xet_for_xet_files(hub, tmp_path):
    st = hfhub.snapshot_download("org/x", tmp_path / "snap", token="hf_tok", endpoint=hub.url, workers=4)
    for name, data in hub.files.items():
        assert (tmp_path / "snap" / name).read_bytes() == data
    assert st["xet_files"] == 2 and st["files"] == 3
    assert hub.cdn_gets >= 1 and hub.recon_gets == 2   # config.json over HTTP, the rest from CAS
    again = hfhub.snapshot_download("org/x", tmp_path / "snap", token="hf_tok", endpoint=hub.url)
    assert again["xet_files"] == 2 and hub.recon_gets == 2, "present + verified files are kept"


def test_reconstruct_streams_with_bounded_window():
    """A many-xorb file is written in file order with at most ``prefetch`` decoded ranges alive
    (plus ranges a later term still needs): peak memory does not grow with the file."""
    n = 48
    blobs = [os.urandom(1000) + bytes([i]) * 64000 for i in range(n)]
    xorbs = {f"X{i}": chunk(b, 1 if i % 2 else 0) for i, b in enumerate(blobs)}
    terms = [{"hash": f"X{i}", "unpacked_length": len(blobs[i]), "range": {"start": 0, "end": 1}} for i in range(n)]
    terms.append({"hash": "X0", "unpacked_length": len(blobs[0]), "range": {"start": 0, "end": 1}})  # X0 reused last
    fetch = {h: [{"range": {"start": 0, "end": 1}, "url": h, "url_range": {"start": 0, "end": len(x) - 1}}]
             for h, x in xorbs.items()}
    fetched = []

    class Local(xet.XetClient):
        def _fetch(self, url, start, end):
            fetched.append(url)
            return xorbs[url][start:end + 1]

    xc = Local(hub=None, workers=4)
    xc.prefetch = 3
    import io

    buf = io.BytesIO()
    wrote = xc.reconstruct({"terms": terms, "fetch_info": fetch}, buf)
    want = b"".join(blobs) + blobs[0]
    assert buf.getvalue() == want and wrote == len(want)
    assert sorted(fetched) == sorted(xorbs)                      # every range fetched exactly once
    assert xc.stats["peak_live_ranges"] <= xc.prefetch + 1       # X0 stays alive for its last term
