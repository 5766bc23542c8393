"""ome-agent CLI entrypoint (see :mod:`ome_amd.agent`)."""
from __future__ import annotations

import argparse
import base64
import json
import logging
import os
import shutil
import sys
import tempfile
import time
import urllib.request
import zipfile
from pathlib import Path

import yaml

log = logging.getLogger("ome_amd.agent")

# files never encrypted (metadata the loaders read before decryption) — ``enigma.go isIgnoredFile``
IGNORED = {"config.json", "generation_config.json", "tokenizer.json", "tokenizer_config.json",
           "special_tokens_map.json", "model.safetensors.index.json", ".ome-dek", ".ome-encrypted", "README.md",
           "LICENSE", ".gitattributes", "tokenizer.model", "vocab.json", "merges.txt"}
MARKER = ".ome-encrypted"


def _cfg(args) -> dict:
    if getattr(args, "config", None) and os.path.exists(args.config):
        with open(args.config) as f:
            return yaml.safe_load(f) or {}
    return {}


def _opt(args, cfg: dict, name: str, env: str | None = None, default=None):
    v = getattr(args, name.replace("-", "_"), None)
    if v not in (None, ""):
        return v
    if env and os.environ.get(env):
        return os.environ[env]
    return cfg.get(name, cfg.get(name.replace("-", "_"), default))


# ------------------------------------------------------------------ key management
def _api_get(path: str) -> dict | None:
    api = os.environ.get("OME_API_SERVER")
    if not api:
        return None
    try:
        with urllib.request.urlopen(api.rstrip("/") + path, timeout=10) as r:
            return json.loads(r.read())
    except Exception as e:  # noqa: BLE001
        log.warning("API %s failed: %s", path, e)
        return None


def master_key(args, cfg) -> bytes:
    for src in (os.environ.get("OME_MEK"), _read(os.environ.get("OME_MEK_FILE"))):
        if src:
            return _key32(src)
    secret, key = _opt(args, cfg, "secret-name", "DECRYPTION_SECRET_NAME"), _opt(args, cfg, "key-name",
                                                                               "DECRYPTION_KEY_NAME")
    ns = os.environ.get("POD_NAMESPACE", "default")
    if secret:
        sec = _api_get(f"/api/v1/namespaces/{ns}/secrets/{secret}")
        if sec:
            data = {**(sec.get("data") or {}), **{k: base64.b64encode(v.encode()).decode()
                                                  for k, v in (sec.get("stringData") or {}).items()}}
            raw = data.get(key or "mek") or next(iter(data.values()), None)
            if raw:
                return _key32(base64.b64decode(raw).decode().strip())
    raise SystemExit("enigma: no master key (set OME_MEK / OME_MEK_FILE or DECRYPTION_SECRET_NAME + OME_API_SERVER)")


def _read(p):
    if p and os.path.exists(p):
        return Path(p).read_text().strip()
    return None


def _key32(b64: str) -> bytes:
    k = base64.b64decode(b64)
    if len(k) != 32:
        raise SystemExit(f"master key must be 32 bytes (AES-256), got {len(k)}")
    return k


def _files(model_dir: Path):
    for p in sorted(model_dir.rglob("*")):
        if p.is_file() and p.name not in IGNORED and not p.name.startswith(".ome-"):
            yield p


def cmd_encrypt(args) -> int:
    """Encrypt a model directory in place: fresh DEK per model, wrapped by the MEK."""
    from ome_amd.io import native

    cfg = _cfg(args)
    d = Path(_opt(args, cfg, "local-path", "LOCAL_PATH"))
    mek = master_key(args, cfg)
    dek = os.urandom(32)
    (d / ".ome-dek").write_bytes(native.aes_gcm_encrypt(dek, mek, os.urandom(12)))
    n = 0
    for p in _files(d):
        native.aes_gcm_encrypt_file(p, p, dek, os.urandom(12))
        n += 1
    (d / MARKER).write_text(json.dumps({"files": n, "algorithm": "AES-256-GCM", "time": time.time()}))
    log.info("encrypted %d files under %s", n, d)
    return 0


def data_key(args, cfg: dict, model_dir: Path) -> bytes:
    """The model's plaintext DEK (enigma.go prepareDecryptionKey): with a key service configured
    (``kms_provider`` oci | vault, :func:`ome_amd.storage.kms.from_config`) the master key id comes
    from the key metadata (``key_metadata``), the wrapped DEK from the vault secret
    (``secret_name`` / ``vault_id``) or the model's ``.ome-dek``, and the key service unwraps
    it; otherwise the local MEK (Secret / file) unwraps ``.ome-dek``."""
    import base64 as _b64

    from ome_amd.io import native
    from ome_amd.storage import kms

    provider, secrets = kms.from_config(cfg)
    if provider is None:
        return native.aes_gcm_decrypt((model_dir / ".ome-dek").read_bytes(), master_key(args, cfg))
    key_id = provider.master_key_id(cfg.get("key_metadata") or {})
    secret = _opt(args, cfg, "secret-name", "DECRYPTION_SECRET_NAME")
    if secrets is not None and secret:
        wrapped = secrets.get(secret, cfg.get("vault_id"))
    else:
        wrapped = (model_dir / ".ome-dek").read_text().strip()
    dek = provider.decrypt(wrapped, key_id)
    if len(dek) != 32:
        dek = _b64.b64decode(dek)   # services that return the key base64-encoded once more
    return dek


def cmd_enigma(args) -> int:
    """Model-init: validate the model store, then decrypt every weight file (``enigma.go:41-174``).
    With ``--temp-path`` the model is first copied there (the reference copies to a temp dir so the
    shared host copy stays encrypted) and decrypted in the copy."""
    from ome_amd.io import native

    cfg = _cfg(args)
    d = Path(_opt(args, cfg, "local-path", "LOCAL_PATH", "/mnt/models"))
    if not d.is_dir() or not any(d.iterdir()):
        log.error("model store %s is missing or empty", d)
        return 1
    if str(_opt(args, cfg, "disable-model-decryption", "DISABLE_MODEL_DECRYPTION", "false")).lower() == "true":
        log.info("model decryption disabled")
        return 0
    if not (d / MARKER).exists():
        log.info("model at %s is not encrypted; nothing to do", d)
        return 0
    tmp = _opt(args, cfg, "temp-path", "TEMP_PATH")
    if tmp:
        shutil.copytree(d, tmp, dirs_exist_ok=True)
        d = Path(tmp)
    try:
        dek = data_key(args, cfg, d)
    except Exception as e:  # noqa: BLE001 -- any key-service failure stops the model-init
        log.error("failed to unwrap the data key with the master key: %s", e)
        return 1
    n = 0
    for p in _files(d):
        native.aes_gcm_decrypt_file(p, p, dek)
        n += 1
    (d / MARKER).unlink()
    (d / ".ome-dek").unlink(missing_ok=True)   # absent when the wrapped DEK lives in a vault secret
    log.info("decrypted %d files under %s", n, d)
    return 0


# ------------------------------------------------------------------ downloads / replication
def cmd_hf_download(args) -> int:
    from ome_amd.storage.backends import fetch

    cfg = _cfg(args)
    repo = _opt(args, cfg, "repo", "HF_MODEL_ID")
    rev = _opt(args, cfg, "revision", "HF_REVISION", "main")
    dest = _opt(args, cfg, "local-path", "LOCAL_PATH")
    res = fetch(f"hf://{repo}@{rev}", dest, token=os.environ.get("HF_TOKEN") or os.environ.get("HUGGINGFACE_API_KEY"))
    log.info("downloaded %s@%s -> %s (%d files, sha %s)", repo, rev, res.path, res.files, res.sha)
    return 0


def _upload(src: Path, target: str) -> str:
    """Write a local tree to a target URI (object store / PVC / local) with an MD5 manifest."""
    from ome_amd.storage.backends import object_store_path, write_manifest
    from ome_amd.storage.uri import parse

    u = parse(target) if "://" in target else None
    if u is not None and u.type in ("S3", "OCI", "GCS", "AZURE"):
        from ome_amd.storage import objstore

        remote = objstore.client_for(u.parts, u.type)
        if remote is not None:   # real endpoint: parallel multipart upload
            client, bucket, prefix = remote
            objstore.upload_tree(client, bucket, prefix, src)
            return target
    if u is None or u.type == "LOCAL":
        dst = Path(u.parts["path"] if u else target)
    elif u.type == "PVC":
        root = Path(os.environ.get("OME_PVC_ROOT", "/var/lib/ome/pvc"))
        dst = root / (u.parts["namespace"] or "default") / u.parts["pvc"] / u.parts["subpath"]
    else:
        dst = object_store_path(target)
    dst.mkdir(parents=True, exist_ok=True)
    for p in sorted(src.rglob("*")):
        if p.is_file():
            out = dst / p.relative_to(src)
            out.parent.mkdir(parents=True, exist_ok=True)
            shutil.copy2(p, out)
    write_manifest(dst)
    return str(dst)


def cmd_replica(args) -> int:
    """Replicate a model between storages (HF/OCI/PVC/local -> OCI/PVC/local), verified by MD5
    manifest on the way in (object-store sources) and written with one on the way out
    (``internal/ome-agent/replica``)."""
    from ome_amd.storage.backends import fetch

    cfg = _cfg(args)
    src = _opt(args, cfg, "source", "SOURCE_STORAGE_URI")
    dst = _opt(args, cfg, "target", "TARGET_STORAGE_URI")
    with tempfile.TemporaryDirectory(prefix="ome-replica-") as tmp:
        res = fetch(src, tmp)
        out = _upload(Path(res.path), dst)
    log.info("replicated %s -> %s (%s)", src, dst, out)
    return 0


def cmd_fine_tuned_adapter(args) -> int:
    """Init container: fetch the adapter named by FINE_TUNED_WEIGHT_NAME into the download dir.
    The (Cluster)FineTunedWeight's storage URI is read from the manager API."""
    from ome_amd.storage.backends import fetch

    cfg = _cfg(args)
    name = _opt(args, cfg, "name", "FINE_TUNED_WEIGHT_NAME")
    dest = Path(_opt(args, cfg, "local-path", "FT_LOCAL_PATH", "/mnt/finetuned/download"))
    uri = _opt(args, cfg, "storage-uri", "FT_STORAGE_URI")
    if not uri:
        ftw = _api_get(f"/apis/ome.io/v1beta1/finetunedweights/{name}") or {}
        uri = ((ftw.get("spec") or {}).get("storage") or {}).get("storageUri")
    if not uri:
        log.error("no storage URI for fine-tuned weight %s", name)
        return 1
    res = fetch(uri, str(dest / name))
    _maybe_unzip(Path(res.path))
    log.info("fine-tuned weight %s -> %s", name, res.path)
    return 0


def _maybe_unzip(d: Path) -> None:
    for z in list(d.glob("*.zip")):
        with zipfile.ZipFile(z) as zf:
            for m in zf.namelist():  # no path traversal out of the adapter dir
                if m.startswith("/") or ".." in Path(m).parts:
                    raise SystemExit(f"unsafe path in {z}: {m}")
            zf.extractall(d)
        z.unlink()


def sync_adapters(spec_file: Path, adapters_dir: Path, engine_url: str | None = None) -> tuple[list, list]:
    """serving-agent core: make ``adapters_dir`` match the desired list in ``spec_file``
    (JSON ``[{"name", "storageUri"}]``); download+unzip new ones, delete removed ones, and tell
    the engine (``/load_lora_adapter`` / ``/unload_lora_adapter``).  Returns (added, removed)."""
    from ome_amd.storage.backends import fetch

    want = {a["name"]: a for a in json.loads(spec_file.read_text() or "[]")} if spec_file.exists() else {}
    adapters_dir.mkdir(parents=True, exist_ok=True)
    have = {p.name for p in adapters_dir.iterdir() if p.is_dir()}
    added, removed = [], []
    for name in sorted(set(want) - have):
        try:
            res = fetch(want[name]["storageUri"], str(adapters_dir / name))
            _maybe_unzip(Path(res.path))
            added.append(name)
            _engine(engine_url, "/load_lora_adapter", {"lora_name": name, "lora_path": str(adapters_dir / name)})
        except Exception as e:  # noqa: BLE001 — retried on the next change / poll
            log.warning("adapter %s download failed: %s", name, e)
            shutil.rmtree(adapters_dir / name, ignore_errors=True)
    for name in sorted(have - set(want)):
        shutil.rmtree(adapters_dir / name, ignore_errors=True)
        removed.append(name)
        _engine(engine_url, "/unload_lora_adapter", {"lora_name": name})
    return added, removed


def _engine(url, path, body):
    if not url:
        return
    try:
        req = urllib.request.Request(url.rstrip("/") + path, data=json.dumps(body).encode(),
                                     headers={"Content-Type": "application/json"})
        urllib.request.urlopen(req, timeout=30).read()
    except Exception as e:  # noqa: BLE001
        log.info("engine %s%s: %s", url, path, e)


def cmd_serving_agent(args) -> int:
    cfg = _cfg(args)
    spec = Path(_opt(args, cfg, "spec-file", "FT_SPEC_FILE", "/mnt/ft-config/adapters.json"))
    out = Path(_opt(args, cfg, "local-path", "FT_LOCAL_PATH", "/mnt/finetuned"))
    engine = _opt(args, cfg, "engine-url", "ENGINE_URL", "http://127.0.0.1:8080")
    interval = float(_opt(args, cfg, "poll-interval", None, 5.0))
    last = None
    while True:  # fsnotify stand-in: poll the (ConfigMap-mounted) spec file's mtime
        m = spec.stat().st_mtime if spec.exists() else None
        if m != last:
            last = m
            a, r = sync_adapters(spec, out, engine)
            if a or r:
                log.info("adapters added %s removed %s", a, r)
        if args.once:
            return 0
        time.sleep(interval)


def cmd_model_metadata(args) -> int:
    """One-shot job: parse the model directory and patch unset (Cluster)BaseModel spec fields
    through the manager API (``internal/ome-agent/model-metadata``)."""
    from ome_amd.modelagent.modelconfig import load_model_config, model_metadata

    cfg = _cfg(args)
    path = _opt(args, cfg, "model-path", "MODEL_PATH")
    name = _opt(args, cfg, "model-name", "MODEL_NAME")
    ns = _opt(args, cfg, "namespace", "MODEL_NAMESPACE")
    md = model_metadata(load_model_config(path))
    patch = {"spec": {k: md[k] for k in ("modelType", "modelArchitecture", "modelParameterSize", "maxTokens",
                                         "modelCapabilities", "modelFormat", "modelFramework", "quantization")
                      if md.get(k) not in (None, "", [])}}
    print(json.dumps(patch))
    api = os.environ.get("OME_API_SERVER")
    if api and name:
        url = (f"{api.rstrip('/')}/apis/ome.io/v1beta1/namespaces/{ns}/basemodels/{name}" if ns else
               f"{api.rstrip('/')}/apis/ome.io/v1beta1/clusterbasemodels/{name}")
        req = urllib.request.Request(url, data=json.dumps(patch).encode(), method="PATCH",
                                     headers={"Content-Type": "application/merge-patch+json"})
        with urllib.request.urlopen(req, timeout=30) as r:
            log.info("patched %s: %d", url, r.status)
    return 0


COMMANDS = {"enigma": cmd_enigma, "encrypt": cmd_encrypt, "hf-download": cmd_hf_download, "replica": cmd_replica,
            "fine-tuned-adapter": cmd_fine_tuned_adapter, "serving-agent": cmd_serving_agent,
            "model-metadata": cmd_model_metadata}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("ome-agent")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name in COMMANDS:
        p = sub.add_parser(name)
        p.add_argument("--config", default=os.environ.get("OME_AGENT_CONFIG", "/ome-agent.yaml"))
        p.add_argument("--local-path", default=None)
        p.add_argument("--temp-path", default=None)
        p.add_argument("--secret-name", default=None)
        p.add_argument("--key-name", default=None)
        p.add_argument("--disable-model-decryption", default=None)
        p.add_argument("--repo", default=None)
        p.add_argument("--revision", default=None)
        p.add_argument("--source", default=None)
        p.add_argument("--target", default=None)
        p.add_argument("--name", default=None)
        p.add_argument("--storage-uri", default=None)
        p.add_argument("--spec-file", default=None)
        p.add_argument("--engine-url", default=None)
        p.add_argument("--model-path", default=None)
        p.add_argument("--model-name", default=None)
        p.add_argument("--namespace", default=None)
        p.add_argument("--once", action="store_true")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s ome-agent %(levelname)s %(message)s")
    return COMMANDS[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())
