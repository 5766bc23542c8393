"""PD disaggregation on CPU: a prefill engine pushes KV pages + first token over TCP to a decode
engine, which must then generate exactly what a single engine generates."""
import time

from ome_amd.runtime.disagg import attach_kv_transfer
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams


def _engine():
    return Engine(EngineArgs(model="tiny-llama", device="cpu", max_running_requests=8, context_length=512, seed=0))


def test_prefill_decode_handoff_matches_single_engine():
    prompts = [[5 + (i * 7 + j) % 900 for j in range(20 + 13 * i)] for i in range(3)]
    ref = _engine()
    want = [r.output_ids for r in ref.generate(prompts, SamplingParams(max_new_tokens=12, ignore_eos=True))]

    pre, dec = _engine(), _engine()
    attach_kv_transfer(pre, "prefill", 0)
    kt = attach_kv_transfer(dec, "decode", 0)
    dreqs = []
    for i, p in enumerate(prompts):
        room = 1000 + i
        b = {"room": room, "bootstrap_room": room, "bootstrap_host": "127.0.0.1", "bootstrap_port": kt.port}
        pr = pre.make_request(p, SamplingParams(max_new_tokens=1, ignore_eos=True),
                              bootstrap={**b, "disagg_role": "prefill"})
        dr = dec.make_request(p, SamplingParams(max_new_tokens=12, ignore_eos=True),
                              bootstrap={**b, "disagg_role": "decode"})
        dec.add_request(dr)  # decode side may see the request before its KV (either order works)
        pre.add_request(pr)
        dreqs.append(dr)
    deadline = time.time() + 60
    while any(not r.finished for r in dreqs) and time.time() < deadline:
        pre.step()
        dec.step()
        time.sleep(0.001)
    assert [r.output_ids for r in dreqs] == want
    assert kt.received == 3 and not kt.waiting
    # the decode engine never ran a prefill forward: every prompt token came over the wire
    assert dec.metrics.step_prefill.n == 0 and dec.metrics.step_decode.n > 0


def test_receiver_rejects_oversized_and_malformed_transfers():
    """The decode-side receiver bounds what a peer can make it allocate, and a page image whose
    shape does not match the prompt aborts that request instead of the engine."""
    import json
    import socket
    import struct

    from ome_amd.runtime.disagg import MAGIC, default_bind_host
    from ome_amd.runtime.request import ReqState

    assert default_bind_host() != "0.0.0.0"
    dec = _engine()
    kt = attach_kv_transfer(dec, "decode", 0)
    assert kt._sock.getsockname()[0] == default_bind_host()
    cap = kt.max_payload_bytes()
    # 1) a header announcing more than one full context of pages is refused before any allocation
    h = json.dumps({"room": 7, "nbytes": cap + 1}).encode()
    with socket.create_connection(("127.0.0.1", kt.port), timeout=10) as s:
        s.sendall(MAGIC + struct.pack("<I", len(h)) + h)
        s.settimeout(10)
        assert s.recv(2) == b""  # closed without the OK ack
    assert kt.received == 0 and 7 not in kt.inbox
    # 2) a page image whose page count disagrees with n_tokens aborts only that request
    kv = dec.runner.kv
    k0, v0 = kv.k[kv.local_layers[0]], kv.v[kv.local_layers[0]]
    req = dec.make_request(list(range(5, 45)), SamplingParams(max_new_tokens=4, ignore_eos=True))
    header = {"room": 8, "n_tokens": 40, "layers": len(kv.local_layers), "first_token": 3,
              "shape_k": [1, *k0.shape[1:]], "shape_v": [1, *v0.shape[1:]], "dtype": str(kv.dtype)}
    payload = bytes(len(kv.local_layers) * (k0[0].numel() + v0[0].numel()) * k0.element_size())
    assert kt._install(req, header, payload) is True
    assert req.state == ReqState.FINISHED and req.finish_reason == "abort:kv_layout_mismatch"
    kt.close()
