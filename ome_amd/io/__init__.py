"""Artifact I/O: safetensors header parsing, native (C++) parallel loaders, file copy /
verification and AES-GCM for encrypted models (``csrc/omeio``)."""
