"""OpenAI-images HTTP server for the Qwen-Image pipelines (the ``sglang serve`` diffusion runtime of
``config/runtimes/srt/Qwen/Qwen-Image-rt.yaml``): ``POST /v1/images/generations`` (JSON:
prompt, n, size "WxH", negative_prompt, num_inference_steps, true_cfg_scale / guidance_scale,
seed, response_format b64_json) and ``POST /v1/images/edits`` (the same plus ``image`` /
``images`` as data URLs or base64 -- the edit pipelines), ``/health``, ``/v1/models`` and
Prometheus ``/metrics``.  One request at a time per GPU (a diffusion step already fills the
MI355X); requests queue on an asyncio lock and run in a worker thread.

``python -m ome_amd.diffusion.server --model-path DIR`` (a diffusers directory) or
``--model-path random://qwen-image`` (random-init weights of the architecture).
"""
from __future__ import annotations

import argparse
import asyncio
import base64
import io
import logging
import time

log = logging.getLogger("ome_amd.diffusion.server")


def _png_b64(arr) -> str:
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    return base64.b64encode(buf.getvalue()).decode()


def _decode_image(src: str):
    from ome_amd.multimodal.inputs import load_image

    if src.startswith("data:") or src.startswith(("http://", "https://", "/")):
        return load_image(src)
    return load_image(base64.b64decode(src))


def build_app(pipe, served_name: str):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import PlainTextResponse

    app = FastAPI(title="ome_amd diffusion runtime")
    lock = asyncio.Lock()
    counters = {"requests": 0, "images": 0, "errors": 0, "seconds": 0.0}

    @app.get("/health")
    async def health():
        return {"status": "ok"}

    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": served_name, "object": "model", "owned_by": "ome_amd"}]}

    @app.get("/metrics")
    async def metrics():
        lines = [f"ome_images_requests_total {counters['requests']}", f"ome_images_generated_total {counters['images']}",
                 f"ome_images_errors_total {counters['errors']}",
                 f"ome_images_seconds_total {counters['seconds']:.3f}",
                 f"ome_images_denoise_steps_total {pipe.stats['steps']}"]
        return PlainTextResponse("\n".join(lines) + "\n")

    async def run(body: dict, images: list | None):
        counters["requests"] += 1
        try:
            w, h = (int(v) for v in str(body.get("size", "1024x1024")).lower().split("x"))
        except ValueError as e:
            raise HTTPException(400, f"bad size {body.get('size')!r}") from e
        if not 16 <= w <= 4096 or not 16 <= h <= 4096:
            raise HTTPException(400, "size out of range")
        n = max(1, min(int(body.get("n", 1)), 8))
        kw = dict(negative_prompt=body.get("negative_prompt"), width=w, height=h,
                  steps=int(body.get("num_inference_steps", body.get("steps", 50))),
                  true_cfg_scale=float(body.get("true_cfg_scale", body.get("guidance_scale", 4.0))), images=images)
        seed = int(body.get("seed", int(time.time() * 1000) & 0x7FFFFFFF))
        out = []
        t0 = time.perf_counter()
        async with lock:
            for i in range(n):
                try:
                    arr = await asyncio.to_thread(pipe, str(body.get("prompt", "")), seed=seed + i, **kw)
                except ValueError as e:
                    counters["errors"] += 1
                    raise HTTPException(400, str(e)) from e
                out.append({"b64_json": _png_b64(arr)})
        counters["images"] += n
        counters["seconds"] += time.perf_counter() - t0
        return {"created": int(time.time()), "data": out}

    @app.post("/v1/images/generations")
    async def generations(body: dict):
        if pipe.kind != "t2i":
            raise HTTPException(400, "this runtime serves image edits: POST /v1/images/edits")
        return await run(body, None)

    @app.post("/v1/images/edits")
    async def edits(body: dict):
        srcs = body.get("images") or ([body["image"]] if body.get("image") else [])
        if not srcs:
            raise HTTPException(400, "image required")
        if pipe.kind == "t2i":
            raise HTTPException(400, "this runtime serves text-to-image: POST /v1/images/generations")
        return await run(body, [_decode_image(s) for s in srcs])

    return app


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--model-path", required=True)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--served-model-name", default=None)
    ap.add_argument("--pipeline", default=None, help="random:// only: QwenImagePipeline | QwenImageEditPipeline | ...")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--tp-size", type=int, default=1, help="accepted for runtime-flag compatibility (1 only)")
    ap.add_argument("--enable-metrics", action="store_true")
    ap.add_argument("--log-requests", action="store_true")
    return ap


def main(argv=None) -> int:
    import torch
    import uvicorn

    from ome_amd.diffusion.pipeline import PIPELINES, QwenImagePipeline

    a = build_parser().parse_args(argv)
    if a.tp_size != 1:
        raise SystemExit("the diffusion runtime runs one pipeline per GPU (--tp-size 1)")
    dt = getattr(torch, a.dtype)
    if a.model_path.startswith("random://"):
        kind = PIPELINES.get(a.pipeline or "QwenImagePipeline", "t2i")
        pipe = QwenImagePipeline.random(a.model_path[len("random://"):], kind, a.device, dt)
    else:
        pipe = QwenImagePipeline.from_pretrained(a.model_path, a.device, dt)
    uvicorn.run(build_app(pipe, a.served_model_name or a.model_path), host=a.host, port=a.port, log_level="info")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
