# One image for every ome-amd process (manager + node executor, model agent, ome-agent jobs,
# first-party runtime, router, multinode prober, metrics aggregator, benchmark load generator).
# The reference ships six images (dockerfiles/*.Dockerfile); here they differ only by command.
#
#   docker build -f dockerfiles/ome-amd.Dockerfile -t ome-amd:latest .
#
# Base: ROCm 7 + PyTorch for gfx950 (MI355X).  The HIP kernels are compiled at build time for
# gfx950 only (no other targets, no CUDA).
ARG BASE=rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.7.1
FROM ${BASE}

ENV OME_OFFLOAD_ARCH=gfx950 \
    PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTHONUNBUFFERED=1 \
    OME_STATE_DIR=/var/lib/ome

RUN pip install --no-cache-dir fastapi uvicorn aiohttp pydantic pyyaml safetensors huggingface_hub \
        transformers tokenizers prometheus_client && \
    apt-get update && apt-get install -y --no-install-recommends libssl-dev && rm -rf /var/lib/apt/lists/*

WORKDIR /opt/ome-amd
COPY ome_amd ./ome_amd
COPY csrc ./csrc
COPY config ./config
COPY bench.py __graft_entry__.py ./
RUN python -m ome_amd.build --force && python -c "import ome_amd, ome_amd.ops; assert ome_amd.ops.available()"

ENV PYTHONPATH=/opt/ome-amd
EXPOSE 9443 8080
ENTRYPOINT ["python", "-m"]
CMD ["ome_amd.manager", "--host", "0.0.0.0", "--port", "9443", "--catalog", "/opt/ome-amd/config/acceleratorclasses", \
     "--catalog", "/opt/ome-amd/config/runtimes", "--catalog", "/opt/ome-amd/config/models"]
