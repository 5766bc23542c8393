"""Qwen-Image text-to-image at the real size on one GPU: random-init 20B MMDiT (60 blocks, 3072
wide), Qwen2.5-VL-7B text encoder and the VAE (``ome_amd.diffusion.pipeline.PRESETS["qwen-image"]``;
synthetic weights, the benchmark rule), 1024 x 1024, true CFG (prompt + negative prompt in one
packed forward).  Prints one JSON line: seconds per image, per denoising step, and the DiT /
VAE / text-encoder split.

    python scripts/qwen_image_bench.py --steps 50
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from ome_amd.diffusion.pipeline import QwenImagePipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="qwen-image")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--warmup-steps", type=int, default=2)
    a = ap.parse_args()
    t0 = time.perf_counter()
    pipe = QwenImagePipeline.random(a.preset, device="cuda")
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    prompt = "A red fox sitting in a snowy forest at dawn, photorealistic, golden light " * 2
    pipe(prompt, negative_prompt=" ", width=a.size, height=a.size, steps=a.warmup_steps)   # warm-up
    torch.cuda.synchronize()
    dit_t = []
    orig = pipe.dit.forward

    def timed(*args, **kw):
        torch.cuda.synchronize()
        s = time.perf_counter()
        out = orig(*args, **kw)
        torch.cuda.synchronize()
        dit_t.append(time.perf_counter() - s)
        return out

    pipe.dit.forward = timed
    t1 = time.perf_counter()
    img = pipe(prompt, negative_prompt=" ", width=a.size, height=a.size, steps=a.steps)
    torch.cuda.synchronize()
    total = time.perf_counter() - t1
    dit = sum(dit_t)
    print(json.dumps({"metric": "Qwen-Image t2i seconds per image", "value": round(total, 3), "unit": "s/image",
                      "size": a.size, "steps": a.steps, "true_cfg": True, "dit_s": round(dit, 3),
                      "dit_ms_per_step": round(1e3 * dit / max(1, len(dit_t)), 1),
                      "other_s (text encoder + VAE + scheduler)": round(total - dit, 3),
                      "dit_params_b": round(pipe.dit.weight_bytes() / 2e9, 2), "build_s": round(build_s, 1),
                      "image_shape": list(img.shape), "dtype": "bf16",
                      "data": "synthetic (random-init weights of the Qwen-Image architecture)"}), flush=True)


if __name__ == "__main__":
    main()
