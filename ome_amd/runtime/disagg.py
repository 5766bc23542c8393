"""Prefill/decode disaggregation: KV-cache hand-off between a prefill engine and a decode engine
(the reference runs SGLang ``--disaggregation-mode prefill|decode`` behind its PD router;
``config/runtimes/srt/*-pd-rt.yaml``).

Flow (one request, room id R chosen by the router — :mod:`ome_amd.router`):

  router --(R, decode addr)--> prefill engine: runs the prompt, samples the first token, then
        pushes {header, K/V pages of the prompt, first token} to the decode engine's receiver;
  router --(R)--> decode engine: holds the request until the KV for R arrives, installs the pages
        into its own paged cache (page ids differ: copied page-by-page) and continues decoding
        from the first token — which it also streams to the client.

Transport: a length-prefixed TCP stream per hand-off (``--disaggregation-bootstrap-port`` + TP
rank, one stream per TP rank since each rank owns its head shard).  The payload is the raw
page images in the cache's own MFMA layouts (K ``[pages, Hkv, P, D]``, V ``[pages, Hkv, D, P]``)
so neither side reformats; on the decode side the bytes land in one pinned buffer and are
uploaded with a single H2D copy, then scattered with ``index_copy_`` per layer.  Arrival order
does not matter: KV that arrives before its request waits in the inbox, and vice versa.

Same-node fast path (``OMEKV2``, :mod:`ome_amd.runtime.kvlink`): when both engines sit on one
MI355X node the prefill engine asks the receiver for landing slots, maps the decode engine's
exported landing pool once (hipIpc), writes the pages over xGMI from its own GPU, then sends a
small DONE record; the decode engine copies landing slots into its cache pages on device.  No
host bounce; the TCP blob path stays as the fallback for other nodes / CPU engines.
"""
from __future__ import annotations

import json
import os
import logging
import socket
import struct
import threading
import time

import numpy as np
import torch

log = logging.getLogger("ome_amd.disagg")

MAGIC = b"OMEKV1\0\0"
MAGIC2 = b"OMEKV2\0\0"   # same-node IPC handshake: RESERVE -> (slots, handles) -> DONE


def _send_msg(sock: socket.socket, obj: dict) -> None:
    b = json.dumps(obj).encode()
    sock.sendall(struct.pack("<I", len(b)) + b)


MAX_HEADER_BYTES = 1 << 20   # a JSON header / handshake record is a few hundred bytes


def _recv_msg(sock: socket.socket) -> dict:
    (n,) = struct.unpack("<I", _recv_exact(sock, 4))
    if n > MAX_HEADER_BYTES:
        raise ConnectionError(f"KV transfer record of {n} bytes exceeds {MAX_HEADER_BYTES}")
    return json.loads(_recv_exact(sock, n))


def default_bind_host() -> str:
    """Address the decode-side receiver listens on: ``OME_PD_BIND_HOST``, else the pod address
    the executor / kubelet exports (``POD_IP``), else loopback -- never every interface by
    default, since the receiver takes page images from whoever connects."""
    return os.environ.get("OME_PD_BIND_HOST") or os.environ.get("POD_IP") or "127.0.0.1"


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], min(n - got, 1 << 24))
        if k == 0:
            raise ConnectionError("peer closed during KV transfer")
        got += k
    return bytes(buf)


class KVTransfer:
    def __init__(self, engine, mode: str, port: int, host: str | None = None):
        assert mode in ("prefill", "decode")
        self.engine, self.mode = engine, mode
        self.rank = engine.pstate.rank if engine.pstate.tp_size > 1 else 0
        self.port = port
        self.lock = threading.Lock()
        self.inbox: dict[int, tuple[dict, bytes]] = {}   # room -> (header, payload) (decode side)
        self.waiting: dict[int, object] = {}              # room -> Request awaiting its KV (decode)
        self.sent = 0
        self.received = 0
        self._sock = None
        self.host = socket.gethostname()
        self.landing = None        # decode side: kvlink.LandingPool (same-node IPC fast path)
        self.peers: dict = {}      # prefill side: (host, port) -> kvlink.PeerMapping
        self.ipc_sent = 0
        self.ipc_received = 0
        self.bytes_sent = 0        # page-image bytes pushed (prefill side)
        self.write_s = 0.0         # seconds inside the device-to-device page writes (IPC path)
        runner = engine.runner
        kv = runner.kv
        shapes = {(tuple(kv.k[i].shape[1:]), tuple(kv.v[i].shape[1:])) for i in kv.local_layers}
        if len(shapes) != 1:
            # the page image format carries one K/V page shape for all layers (DeciLM / Nemotron-NAS
            # vary KV heads per layer): refuse at start-up rather than fail every transfer
            raise ValueError("PD disaggregation needs one KV page shape across layers; this model has "
                             f"{len(shapes)} (per-layer KV heads)")
        use_ipc = os.environ.get("OME_PD_IPC", "1") == "1"
        if mode == "decode" and use_ipc:
            from ome_amd.runtime import kvlink

            if kvlink.available(runner.device):
                try:
                    toks = int(os.environ.get("OME_PD_LANDING_TOKENS", str(min(65536, 4 * engine.max_context))))
                    self.landing = kvlink.LandingPool(runner.kv, max(1, toks // runner.P))
                except Exception as e:  # noqa: BLE001 — no IPC export: TCP path only
                    log.warning("PD landing pool unavailable (%s); using the TCP path", e)
        if mode == "decode":
            self._sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            self._sock.bind((host or default_bind_host(), port + self.rank))
            self._sock.listen(64)
            self.port = self._sock.getsockname()[1] - self.rank
            threading.Thread(target=self._accept_loop, name="kv-recv", daemon=True).start()
        else:
            engine.scheduler.on_finish = self._on_prefill_finish

    # ------------------------------------------------------------------ decode side
    def _accept_loop(self) -> None:
        while True:
            try:
                conn, _ = self._sock.accept()
            except OSError:
                return
            threading.Thread(target=self._recv_one, args=(conn,), daemon=True).start()

    def _recv_one(self, conn: socket.socket) -> None:
        try:
            with conn:
                magic = _recv_exact(conn, 8)
                if magic == MAGIC2:
                    return self._recv_ipc(conn)
                if magic != MAGIC:
                    raise ConnectionError("bad KV transfer magic")
                (hl,) = struct.unpack("<I", _recv_exact(conn, 4))
                if hl > MAX_HEADER_BYTES:
                    raise ConnectionError(f"KV header of {hl} bytes")
                header = json.loads(_recv_exact(conn, hl))
                nbytes, cap = int(header["nbytes"]), self.max_payload_bytes()
                if not 0 <= nbytes <= cap:
                    raise ConnectionError(f"KV payload of {nbytes} bytes exceeds the {cap}-byte bound")
                payload = _recv_exact(conn, nbytes)
                conn.sendall(b"OK")
            with self.lock:
                self.inbox[int(header["room"])] = (header, payload)
            self.received += 1
            self.engine._wake.set()
        except Exception as e:  # noqa: BLE001
            log.warning("KV receive failed: %s", e)

    def max_payload_bytes(self) -> int:
        """Largest legal page image: every local layer's K and V pages of one full context."""
        kv, P = self.engine.runner.kv, self.engine.runner.P
        k0, v0 = kv.k[kv.local_layers[0]], kv.v[kv.local_layers[0]]
        page_bytes = (k0[0].numel() + v0[0].numel()) * k0.element_size()
        pages = -(-self.engine.max_context // P)
        return len(kv.local_layers) * pages * page_bytes

    def _recv_ipc(self, conn: socket.socket) -> None:
        """Same-node handshake: RESERVE {room, n_pages, host, dtype} -> {ok, slots, pool} ->
        the prefill GPU writes the pages -> DONE {header}."""
        req = _recv_msg(conn)
        lp = self.landing
        if lp is None or req.get("host") != self.host or req.get("dtype") != str(lp.kv.dtype):
            _send_msg(conn, {"ok": False, "ipc": False})
            return
        slots = lp.reserve(int(req["n_pages"]))
        if slots is None:
            _send_msg(conn, {"ok": False, "ipc": True, "retry": True})
            return
        _send_msg(conn, {"ok": True, "slots": slots,
                         "pool": lp.describe() if req.get("session") != lp.session else {"session": lp.session}})
        try:
            done = _recv_msg(conn)
            if not done.get("ok"):
                raise ConnectionError(done.get("error", "sender aborted"))
            conn.sendall(b"OK")
        except Exception:
            lp.release(slots)
            raise
        header = done["header"]
        with self.lock:
            self.inbox[int(header["room"])] = (header, ("ipc", slots))
        self.received += 1
        self.ipc_received += 1
        self.engine._wake.set()

    def hold(self, req) -> None:
        """Decode engine: park a request until its KV arrives (called from the engine thread)."""
        self.waiting[int(req.bootstrap["room"])] = req

    def poll(self) -> int:
        """Decode engine, start of every step: install every request whose KV has arrived."""
        if not self.waiting:
            return 0
        with self.lock:
            ready = [r for r in self.waiting if r in self.inbox]
        n = 0
        for room in ready:
            req = self.waiting[room]
            with self.lock:
                header, payload = self.inbox[room]
            if not self._install(req, header, payload):
                break  # out of KV pages: retry next step (decodes finishing free pages)
            with self.lock:
                self.inbox.pop(room, None)
            self.waiting.pop(room)
            n += 1
        return n

    def _install(self, req, header: dict, payload: bytes) -> bool:
        from ome_amd.runtime.request import ReqState

        eng = self.engine
        sch, runner = eng.scheduler, eng.runner
        kv, P = runner.kv, runner.P
        L = int(header["n_tokens"])
        k0, v0 = kv.k[kv.local_layers[0]], kv.v[kv.local_layers[0]]
        n_pages = -(-L // P)
        ok = (list(header["shape_k"][1:]) == list(k0.shape[1:]) and int(header["layers"]) == len(kv.local_layers)
              and header.get("dtype", str(kv.dtype)) == str(kv.dtype) and 0 < L <= eng.max_context)
        if ok and not (isinstance(payload, tuple) and payload[0] == "ipc"):
            # TCP page image: exactly n_pages K and V pages per local layer, nothing else
            sk, sv = list(header["shape_k"]), list(header.get("shape_v", []))
            want = len(kv.local_layers) * n_pages * (k0[0].numel() + v0[0].numel()) * k0.element_size()
            ok = (sk[0] == n_pages and sv == [n_pages, *v0.shape[1:]] and len(payload) == want)
        if not ok:
            req.state, req.finish_reason = ReqState.FINISHED, "abort:kv_layout_mismatch"
            if req.on_token:
                req.on_token(req, [], True)
            return True
        if req.req_slot < 0:
            slot = sch.slots.alloc()
            if slot is None:
                return False
            req.req_slot = slot
        pages = sch.pages.alloc(n_pages)
        if pages is None and sch.prefix_cache is not None:
            # finished decodes leave their pages in the radix cache: reclaim before waiting
            sch.prefix_cache.evict(n_pages - sch.pages.num_free)
            pages = sch.pages.alloc(n_pages)
        if pages is None:
            return False
        req.pages = list(pages)
        sch.slots.set_pages(req.req_slot, 0, pages)
        sch.slots.flush()
        if isinstance(payload, tuple) and payload[0] == "ipc":
            self.landing.install(payload[1][:n_pages], pages)
            if runner.is_cuda:
                torch.cuda.current_stream(runner.device).synchronize()
            self.landing.release(payload[1])
            return self._activate(req, header)
        src = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
        if runner.is_cuda:
            src = src.pin_memory().to(runner.device, non_blocking=True)
        idx = torch.tensor(pages, dtype=torch.long, device=runner.device)
        kbytes = int(np.prod(header["shape_k"])) * k0.element_size()
        vbytes = int(np.prod(header["shape_v"])) * k0.element_size()
        o = 0
        for i in kv.local_layers:
            kk = src[o:o + kbytes].view(kv.dtype).view(header["shape_k"])
            o += kbytes
            vv = src[o:o + vbytes].view(kv.dtype).view(header["shape_v"])
            o += vbytes
            kv.k[i].index_copy_(0, idx, kk)
            kv.v[i].index_copy_(0, idx, vv)
        return self._activate(req, header)

    def _activate(self, req, header: dict) -> bool:
        from ome_amd.runtime.request import ReqState

        eng = self.engine
        sch = eng.scheduler
        L = int(header["n_tokens"])
        now = time.perf_counter()
        req.output_ids.append(int(header["first_token"]))
        req.output_logprobs.append(float(header.get("first_logprob", 0.0)))
        req.token_times.append(now)
        req.first_token_time = now
        req.num_cached = L
        req.state = ReqState.RUNNING
        sch.running.append(req)
        eng.metrics.on_arrival(req)
        if req.on_token is not None:
            finished = req.params.max_new_tokens <= 1
            req.on_token(req, [req.output_ids[-1]], finished)
            if finished:
                sch.finish(req, "length")
        return True

    # ------------------------------------------------------------------ prefill side
    def _on_prefill_finish(self, req) -> None:
        """Scheduler hook (before the pages are released): snapshot the prompt's KV pages and
        push them to the decode engine in the background.  On a GPU the snapshot is an on-device
        copy (the pages are free for reuse right after this hook); the same-node IPC path then
        writes it into the decode GPU over xGMI, the TCP path ships it through the host."""
        b = req.bootstrap or {}
        if b.get("disagg_role") != "prefill" or not req.output_ids or req.finish_reason and \
                req.finish_reason.startswith("abort"):
            return
        runner = self.engine.runner
        kv, P = runner.kv, runner.P
        L = len(req.prompt_ids)
        pages = req.pages[: -(-L // P)]
        idx = torch.tensor(pages, dtype=torch.long, device=runner.device)
        ks = [kv.k[i].index_select(0, idx) for i in kv.local_layers]
        vs = [kv.v[i].index_select(0, idx) for i in kv.local_layers]
        event = None
        if runner.is_cuda:
            event = torch.cuda.Event()
            event.record(torch.cuda.current_stream(runner.device))
        header = {"room": int(b["bootstrap_room"]), "n_tokens": L, "first_token": int(req.output_ids[0]),
                  "first_logprob": float(req.output_logprobs[0]) if req.output_logprobs else 0.0,
                  "layers": len(kv.local_layers), "shape_k": [len(pages), *kv.k[kv.local_layers[0]].shape[1:]],
                  "shape_v": [len(pages), *kv.v[kv.local_layers[0]].shape[1:]], "dtype": str(kv.dtype)}
        host, port = b.get("bootstrap_host") or "127.0.0.1", int(b["bootstrap_port"]) + self.rank
        threading.Thread(target=self._push, args=(host, port, header, ks, vs, event), daemon=True).start()

    def _push(self, host: str, port: int, header: dict, ks: list, vs: list, event) -> None:
        runner = self.engine.runner
        if event is not None:
            event.synchronize()
        if runner.is_cuda and os.environ.get("OME_PD_IPC", "1") == "1":
            try:
                if self._send_ipc(host, port, header, ks, vs):
                    return
            except Exception as e:  # noqa: BLE001 — any IPC trouble: fall back to the TCP blob
                log.warning("KV IPC push to %s:%d failed (%s); falling back to TCP", host, port, e)
        parts = []
        for k, v in zip(ks, vs):
            parts.append(k.reshape(-1).view(torch.uint8))
            parts.append(v.reshape(-1).view(torch.uint8))
        blob = torch.cat(parts).cpu().numpy().tobytes()
        self._send(host, port, {**header, "nbytes": len(blob)}, blob)

    def _send_ipc(self, host: str, port: int, header: dict, ks: list, vs: list, retries: int = 200) -> bool:
        """RESERVE -> write pages over xGMI -> DONE.  False = receiver has no IPC path for us."""
        from ome_amd.executor.dns import resolve_host_port
        from ome_amd.runtime import kvlink

        rhost, rport = resolve_host_port(host, port)
        runner = self.engine.runner
        n = int(header["shape_k"][0])
        key = (rhost, rport)
        for attempt in range(retries):
            peer = self.peers.get(key)
            with socket.create_connection((rhost, rport), timeout=30) as s:
                s.sendall(MAGIC2)
                _send_msg(s, {"room": header["room"], "n_pages": n, "host": self.host, "dtype": header["dtype"],
                              "session": peer.session if peer else None})
                rep = _recv_msg(s)
                if not rep.get("ok"):
                    if not rep.get("ipc", True):
                        return False
                    time.sleep(min(0.05, 0.001 * 2 ** min(attempt, 6)))  # landing pool full: wait
                    continue
                pool = rep["pool"]
                if peer is None or peer.session != pool["session"]:
                    if peer is not None:
                        peer.close()
                    peer = kvlink.PeerMapping(pool, runner.device)
                    self.peers[key] = peer
                try:
                    stream = self._ipc_stream()
                    t0 = time.perf_counter()
                    peer.write(ks, vs, rep["slots"], stream)
                    dt = time.perf_counter() - t0
                    nb = sum(t.numel() * t.element_size() for t in (*ks, *vs))
                    with self.lock:
                        self.write_s += dt
                        self.bytes_sent += nb
                except Exception as e:
                    _send_msg(s, {"ok": False, "error": str(e)})
                    raise
                _send_msg(s, {"ok": True, "header": header})
                if _recv_exact(s, 2) != b"OK":
                    raise ConnectionError("no ack")
            self.sent += 1
            self.ipc_sent += 1
            return True
        raise TimeoutError("decode landing pool stayed full")

    def _ipc_stream(self):
        st = getattr(self, "_stream", None)
        if st is None:
            st = self._stream = torch.cuda.Stream(self.engine.runner.device)
        return st

    def _send(self, host: str, port: int, header: dict, blob: bytes, retries: int = 20) -> None:
        from ome_amd.executor.dns import resolve_host_port

        host, port = resolve_host_port(host, port)
        h = json.dumps(header).encode()
        for attempt in range(retries):
            try:
                with socket.create_connection((host, port), timeout=30) as s:
                    s.sendall(MAGIC + struct.pack("<I", len(h)) + h)
                    s.sendall(blob)
                    if _recv_exact(s, 2) != b"OK":
                        raise ConnectionError("no ack")
                self.sent += 1
                with self.lock:
                    self.bytes_sent += len(blob)
                return
            except OSError as e:
                log.warning("KV push to %s:%d failed (%s), retry %d", host, port, e, attempt + 1)
                time.sleep(min(2.0, 0.1 * 2 ** attempt))
        log.error("KV push for room %s dropped", header["room"])

    def stats(self) -> dict:
        """Transfer counters for ``/get_server_info`` (``bench.py --pd`` reports the kvlink rate:
        page-image bytes over the seconds spent in the device-to-device writes)."""
        with self.lock:
            return {"mode": self.mode, "sent": self.sent, "received": self.received, "ipc_sent": self.ipc_sent,
                    "ipc_received": self.ipc_received, "bytes_sent": self.bytes_sent,
                    "ipc_write_s": round(self.write_s, 6),
                    "ipc_write_gbps": round(self.bytes_sent / self.write_s / 1e9, 3) if self.write_s > 0 else None}

    def close(self) -> None:
        if self._sock is not None:
            self._sock.close()


def attach_kv_transfer(engine, mode: str, port: int) -> KVTransfer:
    kt = KVTransfer(engine, mode, port)
    engine.kv_transfer = kt
    return kt
