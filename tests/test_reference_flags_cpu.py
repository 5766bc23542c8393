"""Every flag the reference runtimes pass (``/root/reference/config/runtimes/**``) is either
implemented or an explicit, documented no-op (``ome_amd/runtime/flags.py``), and the process it goes
to (engine / router / diffusion server) parses the runtime's whole argument list with no leftovers
(verdict r05, missing item 3).  Unknown flags now stop the process instead of being dropped."""
import glob
import os
import re
import shlex

import pytest
import yaml

from ome_amd.runtime import flags as F

REF = "/root/reference/config/runtimes"
# the reference's flag set, frozen here so the test still means something where the reference
# checkout is absent (it only exists in the build container)
FROZEN = {
    "--attention-backend", "--chat-template", "--chunked-prefill-size", "--context-length", "--cuda-graph-bs",
    "--cuda-graph-max-bs", "--cuda-graph-sizes", "--decode-log-interval", "--decode-selector", "--deepep-mode",
    "--disable-cuda-graph", "--disable-fast-image-processor", "--disable-radix-cache",
    "--disable-shared-experts-fusion", "--disaggregation-ib-device", "--disaggregation-mode", "--dist-init-addr",
    "--dp-size", "--enable-auto-tool-choice", "--enable-chunked-prefill", "--enable-deepep-moe",
    "--enable-dp-attention", "--enable-dp-lm-head", "--enable-eplb", "--enable-metrics", "--enable-multimodal",
    "--enable-torch-compile", "--enable-two-batch-overlap", "--enforce-eager", "--ep-dispatch-algorithm",
    "--ep-num-redundant-experts", "--eplb-algorithm", "--gpu-memory-utilization", "--grpc-mode",
    "--health-check-endpoint", "--host", "--is-embedding", "--kv-cache-dtype", "--limit-mm-per-prompt",
    "--load-balance-method", "--log-level", "--log-requests", "--log-requests-level", "--max-log-len",
    "--max-model-len", "--max-num-seqs", "--max-payload-size", "--max-running-requests", "--max-total-tokens",
    "--mem-frac", "--mem-fraction-static", "--middleware", "--mm-attention-backend", "--model", "--model-path",
    "--moe-a2a-backend", "--moe-dense-tp-size", "--nccl-init", "--nnodes", "--node-rank", "--page-size",
    "--pd-disaggregation", "--policy", "--port", "--preemption-mode", "--prefill-round-robin-balance",
    "--prefill-selector", "--quantization", "--reasoning-parser", "--selector", "--served-model-name",
    "--service-discovery", "--service-discovery-namespace", "--service-discovery-port", "--skip-server-warmup",
    "--tensor-parallel-size", "--tokenizer-path", "--tool-call-parser", "--torch-compile-max-bs", "--tp",
    "--tp-size", "--trust-remote-code", "--watchdog-timeout", "--worker-startup-timeout-secs",
}

_ENTRY = [("sglang.launch_server", "engine"), ("vllm.entrypoints.openai.api_server", "engine"),
          ("launch_router", "router")]


def _runners(doc):
    spec = (doc or {}).get("spec") or {}
    for comp in ("engineConfig", "decoderConfig", "routerConfig"):
        c = spec.get(comp) or {}
        for key in ("runner", "leader", "worker"):
            r = c.get(key)
            if key != "runner" and isinstance(r, dict):
                r = r.get("runner")
            if isinstance(r, dict):
                yield r


def _argv(runner):
    """-> (process, argv after the entrypoint) or None."""
    toks = []
    for t in list(runner.get("command") or []) + list(runner.get("args") or []):
        t = str(t)
        toks += shlex.split(t) if ("launch_server" in t or "launch_router" in t or "vllm" in t) and " " in t else [t]
    for i, t in enumerate(toks):
        for mod, proc in _ENTRY:
            if t == mod or t.endswith(mod):
                return proc, toks[i + 1:]
        if t in ("vllm", "sglang") and i + 1 < len(toks) and toks[i + 1] == "serve":
            if t == "sglang":
                return "diffusion", toks[i + 2:]
            rest = toks[i + 2:]
            return "engine", (["--model-path", rest[0]] + rest[1:]) if rest and not rest[0].startswith("-") else rest
    return None


def _clean(argv):
    out = []
    for t in argv:
        if t in ("&&", ";", "|"):
            break
        out.append("2" if re.fullmatch(r"\$[({][A-Za-z_]+[)}]", t) else t)
    return out


def _reference_cases():
    if not os.path.isdir(REF):
        return []
    cases = []
    for f in sorted(glob.glob(os.path.join(REF, "**", "*.yaml"), recursive=True)):
        with open(f) as fh:
            for doc in yaml.safe_load_all(fh):
                for r in _runners(doc if isinstance(doc, dict) else {}):
                    got = _argv(r)
                    if got:
                        cases.append((os.path.relpath(f, REF), got[0], _clean(got[1])))
    return cases


CASES = _reference_cases()


def test_every_reference_flag_is_classified():
    seen = {t.split("=", 1)[0] for _, _, argv in CASES for t in argv if t.startswith("--")} if CASES else FROZEN
    if CASES:
        assert seen <= FROZEN | set(F.REFERENCE_FLAGS), "update FROZEN / flags.py for new reference flags"
    missing = sorted(f for f in seen | FROZEN if f not in F.REFERENCE_FLAGS)
    assert not missing, f"reference flags with no entry in ome_amd/runtime/flags.py: {missing}"
    for flag, (proc, status, note) in F.REFERENCE_FLAGS.items():
        assert proc in (F.ENGINE, F.ROUTER) and status in ("impl", "noop") and len(note) > 10, flag


@pytest.mark.skipif(not CASES, reason="reference checkout not present")
def test_reference_runtimes_parse_completely():
    from ome_amd.diffusion.server import build_parser as diffusion_parser
    from ome_amd.router.server import build_parser as router_parser
    from ome_amd.runtime.server import build_parser as engine_parser, validate_args

    n = {"engine": 0, "router": 0, "diffusion": 0}
    for path, proc, argv in CASES:
        ap = {"engine": engine_parser, "router": router_parser, "diffusion": diffusion_parser}[proc]()
        ns, unknown = ap.parse_known_args(argv)
        assert not unknown, f"{path} ({proc}): unparsed {unknown}"
        if proc == "engine":
            validate_args(ns)   # raises on a value this framework cannot honour
        for t in argv:
            if t.startswith("--") and proc != "diffusion":
                ent = F.REFERENCE_FLAGS[t.split("=", 1)[0]]
                assert ent[0] == proc or t.split("=", 1)[0] in F.SHARED, f"{path}: {t} classified {ent[0]}"
        n[proc] += 1
    assert n["engine"] > 200 and n["router"] > 150 and n["diffusion"] >= 2, n


def test_unknown_engine_and_router_flags_fail_loudly(monkeypatch):
    from ome_amd.router import server as rs
    from ome_amd.runtime import server as es

    monkeypatch.delenv("OME_ALLOW_UNKNOWN_FLAGS", raising=False)
    with pytest.raises(SystemExit) as e:
        es.main(["--model-path", "random://tiny-llama", "--device", "cpu", "--no-such-flag"])
    assert e.value.code == 2
    with pytest.raises(SystemExit) as e:
        rs.main(["--no-such-router-flag", "1"])
    assert e.value.code == 2


def test_flag_semantics():
    from ome_amd.runtime.server import build_parser, engine_args_from, validate_args

    ap = build_parser()

    def args(*a):
        ns = ap.parse_args(list(a))
        validate_args(ns)
        return ns, engine_args_from(ns)

    ns, ea = args("--model-path", "random://tiny-llama", "--enforce-eager", "--cuda-graph-sizes", "1", "8", "32",
                  "--watchdog-timeout", "1000000", "--deepep-mode", "normal", "--prefill-round-robin-balance",
                  "--limit-mm-per-prompt", "image=2", "--tokenizer-path", "/tmp/tok")
    assert ns.disable_cuda_graph and not ea.cuda_graph and ea.cuda_graph_bs == [1, 8, 32]
    assert ea.watchdog_timeout == 1000000 and ea.deepep_mode == "normal" and ea.dp_balance == "round_robin"
    assert ns.mm_limit == 2 and ea.tokenizer_path == "/tmp/tok"
    _, ea = args("--model-path", "random://tiny-llama", "--load-balance-method", "minimum_tokens")
    assert ea.dp_balance == "minimum_tokens"
    ns, _ = args("--model-path", "x", "--limit-mm-per-prompt", '{"image": 0}')
    assert ns.mm_limit == 0
    for bad in (["--enable-dp-lm-head"], ["--moe-dense-tp-size", "2", "--enable-dp-attention"],
                ["--middleware", "some.other.middleware"], ["--limit-mm-per-prompt", "video"]):
        with pytest.raises(ValueError):
            validate_args(ap.parse_args(["--model-path", "x"] + bad))
    ns = ap.parse_args(["--model-path", "x", "--enable-deepep-moe"])
    validate_args(ns)
    assert ns.moe_a2a_backend == "deepep"


def test_cuda_graph_bs_buckets_and_dp_balance():
    """--cuda-graph-bs selects the captured buckets; the DP placement methods place as named."""
    import torch

    from ome_amd.runtime.engine import Engine, EngineArgs

    eng = Engine(EngineArgs(model="tiny-llama", device="cpu", dtype="float32", max_running_requests=64,
                            context_length=256, cuda_graph_bs=[4, 16, 24], watchdog_timeout=0))
    assert eng.runner.buckets == [4, 16, 24] and eng.runner.bmax == 24
    assert torch.is_tensor(eng.runner.out_ids)
