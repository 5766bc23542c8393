"""ome-agent: the init-container / sidecar / job toolbox (``cmd/ome-agent``,
``internal/ome-agent/*``).

    python -m ome_amd.agent enigma              # model-init: decrypt weights (AES-256-GCM, native)
    python -m ome_amd.agent encrypt             # the inverse, for publishing encrypted models
    python -m ome_amd.agent hf-download         # snapshot a Hugging Face repo
    python -m ome_amd.agent replica             # storage -> storage replication with checksums
    python -m ome_amd.agent fine-tuned-adapter  # init container: fetch adapter weights
    python -m ome_amd.agent serving-agent       # sidecar: hot-(un)load adapters from a spec file
    python -m ome_amd.agent model-metadata      # job: parse config.json, patch the (Cluster)BaseModel

Every subcommand takes ``--config <yaml>`` (the reference's ``/ome-agent.yaml``) plus flags and
environment variables with the same names the webhooks inject.

Key management (enigma): a model's files are encrypted with a random 256-bit data key (DEK);
the DEK is stored wrapped (AES-256-GCM) by a master key (MEK) in ``<model>/.ome-dek``.  The MEK
comes from the Kubernetes Secret ``$DECRYPTION_SECRET_NAME`` key ``$DECRYPTION_KEY_NAME`` via the
manager API (``$OME_API_SERVER``), or from ``$OME_MEK`` / ``$OME_MEK_FILE`` (base64) — the
stand-in for the reference's OCI KMS / Vault clients.  Bulk crypto runs in ``libomeio``
(OpenSSL EVP, streaming, authenticated).
"""
