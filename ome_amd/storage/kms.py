"""Key management for encrypted model weights (reference ``internal/ome-agent/enigma/enigma.go``
:123-146, 193-209 and ``pkg/vault``): the per-model data encryption key (DEK) is stored wrapped
by a master encryption key (MEK) that never leaves the key service.

Interfaces:

* :class:`KeyProvider` -- ``master_key_id(metadata)`` (enigma.go:193 ``getMasterKeyID``: the
  first key matching the key metadata), ``decrypt(ciphertext_b64, key_id) -> bytes`` (the
  unwrapped DEK), ``encrypt(plaintext, key_id) -> ciphertext_b64`` (for sealing a model).
* :class:`SecretStore` -- ``get(name, vault_id) -> str`` (enigma.go:203
  ``GetSecretBundleContentByNameAndVaultId``: the wrapped DEK kept as a vault secret).

Implementations: :class:`OciKms` + :class:`OciSecrets` (OCI KMS crypto / management and Vault
secret-retrieval REST APIs, requests signed by any :mod:`.auth` OCI principal: user, instance,
resource or OKE workload identity); :class:`VaultTransit` + :class:`VaultKV` (HashiCorp Vault
transit engine and KV v2 over its HTTP API, ``X-Vault-Token``); :class:`LocalKeyProvider` (an
MEK held in a Kubernetes Secret / file, AES-256-GCM key wrap in libomeio).
"""
from __future__ import annotations

import base64
import json
import os
import urllib.error
import urllib.parse
import urllib.request


class KmsError(RuntimeError):
    pass


def _call(method: str, url: str, headers: dict, body: bytes | None = None, signer=None, timeout: float = 30.0) -> dict:
    h = dict(headers)
    if body is not None:
        h.setdefault("content-type", "application/json")
    if signer is not None:
        h = signer.sign(method, url, h, body or b"")
    req = urllib.request.Request(url, data=body, method=method, headers=h)
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            raw = r.read()
    except urllib.error.HTTPError as e:
        raise KmsError(f"{method} {url}: HTTP {e.code} {e.read()[:200]!r}") from e
    except OSError as e:
        raise KmsError(f"{method} {url}: {e}") from e
    return json.loads(raw) if raw else {}


class KeyProvider:
    def master_key_id(self, metadata: dict | None = None) -> str:
        raise NotImplementedError

    def decrypt(self, ciphertext_b64: str, key_id: str) -> bytes:
        raise NotImplementedError

    def encrypt(self, plaintext: bytes, key_id: str) -> str:
        raise NotImplementedError


class SecretStore:
    def get(self, name: str, vault_id: str | None = None) -> str:
        raise NotImplementedError


# ------------------------------------------------------------------ OCI KMS / Vault
class OciKms(KeyProvider):
    """OCI KMS (``/20180608``): keys are listed on the vault's management endpoint, encrypt /
    decrypt go to its crypto endpoint (AES-256-GCM master keys)."""

    def __init__(self, signer, management_endpoint: str, crypto_endpoint: str, compartment_id: str = ""):
        self.signer = signer
        self.mgmt, self.crypto = management_endpoint.rstrip("/"), crypto_endpoint.rstrip("/")
        self.compartment = compartment_id

    def master_key_id(self, metadata: dict | None = None) -> str:
        md = dict(metadata or {})
        q = {"compartmentId": md.pop("compartmentId", self.compartment)}
        for k in ("protectionMode", "algorithm", "length", "curveId"):
            if k in md:
                q[k] = md.pop(k)
        keys = _call("GET", f"{self.mgmt}/20180608/keys?{urllib.parse.urlencode(q)}", {}, signer=self.signer)
        items = keys if isinstance(keys, list) else keys.get("items", [])
        name = md.get("displayName")
        items = [k for k in items if k.get("lifecycleState", "ENABLED") == "ENABLED" and
                 (name is None or k.get("displayName") == name)]
        if not items:
            raise KmsError(f"no enabled KMS key matches {metadata}")
        return items[0]["id"]

    def decrypt(self, ciphertext_b64: str, key_id: str) -> bytes:
        d = _call("POST", f"{self.crypto}/20180608/decrypt", {}, json.dumps(
            {"ciphertext": ciphertext_b64, "keyId": key_id, "encryptionAlgorithm": "AES_256_GCM"}).encode(),
            signer=self.signer)
        return base64.b64decode(d["plaintext"])

    def encrypt(self, plaintext: bytes, key_id: str) -> str:
        d = _call("POST", f"{self.crypto}/20180608/encrypt", {}, json.dumps(
            {"plaintext": base64.b64encode(plaintext).decode(), "keyId": key_id,
             "encryptionAlgorithm": "AES_256_GCM"}).encode(), signer=self.signer)
        return d["ciphertext"]


class OciSecrets(SecretStore):
    """OCI Vault secret retrieval (``/20190301/secretbundles/actions/getByName``)."""

    def __init__(self, signer, endpoint: str):
        self.signer, self.endpoint = signer, endpoint.rstrip("/")

    def get(self, name: str, vault_id: str | None = None) -> str:
        q = urllib.parse.urlencode({"secretName": name, "vaultId": vault_id or ""})
        d = _call("GET", f"{self.endpoint}/20190301/secretbundles/actions/getByName?{q}", {}, signer=self.signer)
        content = (d.get("secretBundleContent") or {}).get("content")
        if content is None:
            raise KmsError(f"secret {name} has no content")
        return base64.b64decode(content).decode().strip()


# ------------------------------------------------------------------ HashiCorp Vault
class VaultTransit(KeyProvider):
    """Vault transit engine: ``POST /v1/<mount>/decrypt/<key>`` with ``vault:v1:`` ciphertexts."""

    def __init__(self, addr: str | None = None, token: str | None = None, mount: str = "transit",
                 key_name: str | None = None, namespace: str | None = None):
        self.addr = (addr or os.environ.get("VAULT_ADDR", "http://127.0.0.1:8200")).rstrip("/")
        self.token = token or os.environ.get("VAULT_TOKEN", "")
        self.mount, self.key_name, self.namespace = mount, key_name, namespace or os.environ.get("VAULT_NAMESPACE")

    def _h(self) -> dict:
        h = {"X-Vault-Token": self.token}
        if self.namespace:
            h["X-Vault-Namespace"] = self.namespace
        return h

    def master_key_id(self, metadata: dict | None = None) -> str:
        name = (metadata or {}).get("name") or self.key_name
        if not name:
            raise KmsError("vault transit: no key name")
        _call("GET", f"{self.addr}/v1/{self.mount}/keys/{urllib.parse.quote(name)}", self._h())   # exists?
        return name

    def decrypt(self, ciphertext_b64: str, key_id: str) -> bytes:
        ct = ciphertext_b64 if ciphertext_b64.startswith("vault:") else base64.b64decode(ciphertext_b64).decode()
        d = _call("POST", f"{self.addr}/v1/{self.mount}/decrypt/{urllib.parse.quote(key_id)}", self._h(),
                  json.dumps({"ciphertext": ct}).encode())
        return base64.b64decode(d["data"]["plaintext"])

    def encrypt(self, plaintext: bytes, key_id: str) -> str:
        d = _call("POST", f"{self.addr}/v1/{self.mount}/encrypt/{urllib.parse.quote(key_id)}", self._h(),
                  json.dumps({"plaintext": base64.b64encode(plaintext).decode()}).encode())
        return d["data"]["ciphertext"]


class VaultKV(SecretStore):
    """Vault KV v2: ``GET /v1/<mount>/data/<name>``; the value under ``field`` (default "value")."""

    def __init__(self, addr: str | None = None, token: str | None = None, mount: str = "secret",
                 field: str = "value"):
        self.t = VaultTransit(addr, token)
        self.mount, self.field = mount, field

    def get(self, name: str, vault_id: str | None = None) -> str:
        d = _call("GET", f"{self.t.addr}/v1/{self.mount}/data/{name}", self.t._h())
        data = (d.get("data") or {}).get("data") or {}
        if self.field not in data:
            raise KmsError(f"vault secret {name} has no field {self.field!r}")
        return str(data[self.field]).strip()


# ------------------------------------------------------------------ local MEK
class LocalKeyProvider(KeyProvider):
    """An AES-256 MEK held locally (Kubernetes Secret / file): AES-GCM key wrap (libomeio)."""

    def __init__(self, mek: bytes):
        if len(mek) != 32:
            raise KmsError("master key must be 32 bytes (AES-256)")
        self.mek = mek

    def master_key_id(self, metadata: dict | None = None) -> str:
        return "local"

    def decrypt(self, ciphertext_b64: str, key_id: str) -> bytes:
        from ome_amd.io import native

        return native.aes_gcm_decrypt(base64.b64decode(ciphertext_b64), self.mek)

    def encrypt(self, plaintext: bytes, key_id: str) -> str:
        from ome_amd.io import native

        return base64.b64encode(native.aes_gcm_encrypt(plaintext, self.mek, os.urandom(12))).decode()


def from_config(cfg: dict) -> tuple[KeyProvider | None, SecretStore | None]:
    """Key provider + secret store from an enigma config / env (None, None: use the local MEK).

    ``kms_provider``: "oci" (``kms_management_endpoint``, ``kms_crypto_endpoint``,
    ``secret_endpoint``, ``auth_type`` + principal fields as :mod:`.auth`) or "vault"
    (``vault_addr``, ``vault_token``, ``transit_mount``, ``kv_mount``)."""
    kind = (cfg.get("kms_provider") or os.environ.get("OME_KMS_PROVIDER") or "").lower()
    if not kind:
        return None, None
    if kind == "oci":
        from ome_amd.storage import auth

        signer = auth.DEFAULT_FACTORY.create({"provider": auth.OCI,
                                              "auth_type": cfg.get("auth_type") or "OCIInstancePrincipal",
                                              "region": cfg.get("region", ""), "extra": cfg.get("auth") or {}})
        kms = OciKms(signer, cfg["kms_management_endpoint"], cfg["kms_crypto_endpoint"], cfg.get("compartment_id", ""))
        sec = OciSecrets(signer, cfg["secret_endpoint"]) if cfg.get("secret_endpoint") else None
        return kms, sec
    if kind == "vault":
        kms = VaultTransit(cfg.get("vault_addr"), cfg.get("vault_token"), cfg.get("transit_mount", "transit"),
                           cfg.get("key_name"))
        sec = VaultKV(cfg.get("vault_addr"), cfg.get("vault_token"), cfg.get("kv_mount", "secret"),
                      cfg.get("secret_field", "value"))
        return kms, sec
    raise KmsError(f"unknown kms_provider {kind!r}")
