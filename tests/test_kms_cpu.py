"""Key services for encrypted models (reference enigma.go:123-146, 193-209, pkg/vault,
pkg/principals, pkg/imds) against local fakes:

* OCI KMS + Vault secret retrieval, every request's OCI signature verified by the fake: the
  ome-agent ``enigma`` model-init unwraps the DEK through KMS and decrypts the model;
* HashiCorp Vault transit + KV v2 (X-Vault-Token);
* the OCI instance principal: IMDS identity certificate -> X.509 federation (signed with the
  leaf key, key id ``<tenancy>/fed-x509-sha256/<fingerprint>``) -> session token; the KMS fake
  then verifies requests signed by the SESSION key under ``ST$<token>``."""
import base64
import json
import os
import subprocess
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from pathlib import Path

import pytest

from ome_amd.io import native
from ome_amd.storage import auth as A
from ome_amd.storage import kms

pytestmark = pytest.mark.skipif(not native.available(), reason="libomeio not built")


def _key(tmp: Path, name="k.pem") -> Path:
    p = tmp / name
    subprocess.run(["openssl", "genrsa", "-out", str(p), "2048"], check=True, capture_output=True)
    return p


def _pub_pem(priv: Path) -> str:
    return subprocess.run(["openssl", "rsa", "-in", str(priv), "-pubout"], check=True, capture_output=True,
                          text=True).stdout


def _verify_oci(handler, body: bytes, pub_for_keyid) -> str | None:
    """Rebuild the OCI signing string and verify it; returns the keyId or None."""
    auth = handler.headers.get("authorization", "")
    if not auth.startswith("Signature "):
        return None
    f = dict(kv.split("=", 1) for kv in auth[len("Signature "):].split(","))
    f = {k: v.strip('"') for k, v in f.items()}
    lines = []
    for n in f["headers"].split():
        if n == "(request-target)":
            lines.append(f"(request-target): {handler.command.lower()} {handler.path}")
        else:
            lines.append(f"{n}: {handler.headers.get(n)}")
    pem = pub_for_keyid(f["keyId"])
    if pem is None:
        return None
    if not native.rsa_verify_sha256(pem.encode(), "\n".join(lines).encode(), base64.b64decode(f["signature"])):
        return None
    return f["keyId"]


class FakeOci:
    """KMS management + crypto, Vault secrets, IMDS and the auth federation service in one server."""

    def __init__(self, tmp: Path):
        self.mek = os.urandom(32)
        self.user_key = _key(tmp, "user.pem")
        self.user_pub = _pub_pem(self.user_key)
        self.secrets: dict = {}
        self.session_pubs: dict = {}   # token -> session public key PEM
        self.calls = []
        # instance identity: leaf cert with the tenancy in its subject
        self.leaf_key = _key(tmp, "leaf.pem")
        cert = tmp / "leaf.crt"
        subprocess.run(["openssl", "req", "-new", "-x509", "-key", str(self.leaf_key), "-out", str(cert), "-days", "2",
                        "-subj", "/CN=ocid1.instance.oc1..inst/OU=opc-tenant:ocid1.tenancy.oc1..tenant"],
                       check=True, capture_output=True)
        self.leaf_cert = cert.read_text()
        self.leaf_pub = _pub_pem(self.leaf_key)
        fake = self

        def keyid_pub(kid: str):
            if kid == "ocid1.tenancy.oc1..t/ocid1.user.oc1..u/aa:bb":
                return fake.user_pub
            if kid.startswith("ST$"):
                return fake.session_pubs.get(kid[3:])
            if kid.startswith("ocid1.tenancy.oc1..tenant/fed-x509-sha256/"):
                if kid.split("/", 2)[2] == native.x509_info(fake.leaf_cert)["sha256"]:
                    return fake.leaf_pub
            return None

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, obj=None, raw=None):
                body = raw if raw is not None else json.dumps(obj or {}).encode()
                self.send_response(code)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _route(self, body=b""):
                u = urllib.parse.urlsplit(self.path)
                q = dict(urllib.parse.parse_qsl(u.query))
                fake.calls.append((self.command, u.path))
                if u.path.startswith("/opc/v2/"):
                    if self.headers.get("Authorization") != "Bearer Oracle":
                        return self._send(401)
                    p = u.path[len("/opc/v2"):]
                    if p == "/instance/":
                        return self._send(200, {"canonicalRegionName": "us-ashburn-1",
                                                "regionInfo": {"realmDomainComponent": "oraclecloud.com"}})
                    data = {"/identity/cert.pem": fake.leaf_cert, "/identity/key.pem": fake.leaf_key.read_text(),
                            "/identity/intermediate.pem": fake.leaf_cert}.get(p)
                    return self._send(200, raw=data.encode()) if data else self._send(404)
                kid = _verify_oci(self, body, keyid_pub)
                if kid is None:
                    return self._send(401, {"code": "NotAuthenticated"})
                if u.path == "/v1/x509" and self.command == "POST":
                    d = json.loads(body)
                    assert d["purpose"] == "DEFAULT" and d["fingerprintAlgorithm"] == "SHA256"
                    tok_payload = base64.urlsafe_b64encode(json.dumps({"exp": 4102444800}).encode()).decode().rstrip("=")
                    tok = f"hdr.{tok_payload}.sig{len(fake.session_pubs)}"
                    b64 = d["publicKey"]
                    fake.session_pubs[tok] = ("-----BEGIN PUBLIC KEY-----\n" +
                                              "\n".join(b64[i:i + 64] for i in range(0, len(b64), 64)) +
                                              "\n-----END PUBLIC KEY-----\n")
                    return self._send(200, {"token": tok})
                if u.path == "/20180608/keys":
                    assert q.get("compartmentId") == "ocid1.compartment.oc1..c"
                    return self._send(200, [{"id": "ocid1.key.oc1..old", "displayName": "model-mek",
                                             "lifecycleState": "DISABLED"},
                                            {"id": "ocid1.key.oc1..k1", "displayName": "model-mek",
                                             "lifecycleState": "ENABLED"}])
                if u.path == "/20180608/decrypt":
                    d = json.loads(body)
                    assert d["keyId"] == "ocid1.key.oc1..k1" and d["encryptionAlgorithm"] == "AES_256_GCM"
                    pt = native.aes_gcm_decrypt(base64.b64decode(d["ciphertext"]), fake.mek)
                    return self._send(200, {"plaintext": base64.b64encode(pt).decode()})
                if u.path == "/20180608/encrypt":
                    d = json.loads(body)
                    ct = native.aes_gcm_encrypt(base64.b64decode(d["plaintext"]), fake.mek, os.urandom(12))
                    return self._send(200, {"ciphertext": base64.b64encode(ct).decode()})
                if u.path == "/20190301/secretbundles/actions/getByName":
                    v = fake.secrets.get((q["secretName"], q["vaultId"]))
                    if v is None:
                        return self._send(404)
                    return self._send(200, {"secretBundleContent": {"contentType": "BASE64",
                                                                    "content": base64.b64encode(v.encode()).decode()}})
                return self._send(404)

            def do_GET(self):
                self._route()

            def do_POST(self):
                self._route(self.rfile.read(int(self.headers.get("Content-Length") or 0)))

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def close(self):
        self.srv.shutdown()


@pytest.fixture
def oci(tmp_path):
    f = FakeOci(tmp_path)
    yield f
    f.close()


def _user_signer(oci):
    return A.OciUserPrincipal("ocid1.tenancy.oc1..t", "ocid1.user.oc1..u", "aa:bb", oci.user_key.read_text())


def test_oci_kms_roundtrip_and_key_selection(oci):
    k = kms.OciKms(_user_signer(oci), oci.url, oci.url, "ocid1.compartment.oc1..c")
    kid = k.master_key_id({"displayName": "model-mek"})
    assert kid == "ocid1.key.oc1..k1"                     # disabled key skipped
    dek = os.urandom(32)
    assert k.decrypt(k.encrypt(dek, kid), kid) == dek
    bad = kms.OciKms(A.OciUserPrincipal("ocid1.tenancy.oc1..t", "ocid1.user.oc1..u", "aa:bb",
                                        _key(Path(oci.user_key).parent, "other.pem").read_text()),
                     oci.url, oci.url, "ocid1.compartment.oc1..c")
    with pytest.raises(kms.KmsError):                      # signature with the wrong key: rejected
        bad.master_key_id({})


def test_enigma_decrypts_model_through_kms_and_vault_secret(oci, tmp_path):
    from ome_amd.agent.__main__ import main as agent_main

    model = tmp_path / "model"
    model.mkdir()
    files = {"model.safetensors": os.urandom(5000), "config.json": b'{"model_type": "llama"}'}
    dek = os.urandom(32)
    for name, data in files.items():
        (model / name).write_bytes(data)
        if name.endswith(".safetensors"):   # metadata files (config.json, ...) stay plaintext
            native.aes_gcm_encrypt_file(model / name, model / name, dek, os.urandom(12))
    (model / ".ome-encrypted").write_text(json.dumps({"files": 2}))
    k = kms.OciKms(_user_signer(oci), oci.url, oci.url, "ocid1.compartment.oc1..c")
    oci.secrets[("model-dek", "ocid1.vault.oc1..v")] = k.encrypt(dek, "ocid1.key.oc1..k1")
    cfg = {"kms_provider": "oci", "kms_management_endpoint": oci.url, "kms_crypto_endpoint": oci.url,
           "secret_endpoint": oci.url, "compartment_id": "ocid1.compartment.oc1..c", "vault_id": "ocid1.vault.oc1..v",
           "auth_type": "OCIUserPrincipal",
           "auth": {"tenancy": "ocid1.tenancy.oc1..t", "user": "ocid1.user.oc1..u", "fingerprint": "aa:bb",
                    "key_pem": oci.user_key.read_text()},
           "key_metadata": {"displayName": "model-mek"}, "secret_name": "model-dek", "local_path": str(model)}
    (tmp_path / "agent.yaml").write_text(json.dumps(cfg))
    from ome_amd.agent import __main__ as agent_mod

    marker = agent_mod.MARKER
    if marker != ".ome-encrypted":
        (model / ".ome-encrypted").rename(model / marker)
    rc = agent_main(["enigma", "--config", str(tmp_path / "agent.yaml"), "--local-path", str(model),
                     "--secret-name", "model-dek"])
    assert rc == 0
    for name, data in files.items():
        assert (model / name).read_bytes() == data
    assert ("POST", "/20180608/decrypt") in oci.calls and ("GET", "/20190301/secretbundles/actions/getByName") in oci.calls


def test_instance_principal_federates_and_signs_with_session_key(oci):
    from ome_amd.storage.imds import Imds, tenancy_from_subject

    imds = Imds(oci.url + "/opc/v2", "")
    assert imds.region() == "us-ashburn-1"
    assert imds.tenancy_id() == "ocid1.tenancy.oc1..tenant"
    assert tenancy_from_subject("CN=x,OU=opc-tenant:ocid1.tenancy.oc1..z") == "ocid1.tenancy.oc1..z"
    ip = A.DEFAULT_FACTORY.create({"provider": A.OCI, "auth_type": "OCIInstancePrincipal",
                                   "extra": {"imds_endpoint": oci.url + "/opc/v2", "imds_fallback_endpoint": "",
                                             "auth_endpoint_override": oci.url}})
    assert isinstance(ip, A.OciInstancePrincipal)
    k = kms.OciKms(ip, oci.url, oci.url, "ocid1.compartment.oc1..c")
    assert k.master_key_id({}) == "ocid1.key.oc1..k1"       # request signed by the session key (ST$token)
    assert ip.key_id().startswith("ST$hdr.") and len(oci.session_pubs) == 1
    k.master_key_id({})
    assert len(oci.session_pubs) == 1                        # token cached until exp


class FakeVault:
    def __init__(self):
        self.key = os.urandom(32)
        self.kv = {}
        fake = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, obj):
                b = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def do_GET(self):
                if self.headers.get("X-Vault-Token") != "s.tok":
                    return self._send(403, {"errors": ["permission denied"]})
                if self.path == "/v1/transit/keys/mek":
                    return self._send(200, {"data": {"name": "mek"}})
                if self.path.startswith("/v1/secret/data/"):
                    name = self.path[len("/v1/secret/data/"):]
                    return self._send(200, {"data": {"data": {"value": fake.kv[name]}}})
                self._send(404, {})

            def do_POST(self):
                if self.headers.get("X-Vault-Token") != "s.tok":
                    return self._send(403, {"errors": ["permission denied"]})
                d = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
                if self.path == "/v1/transit/encrypt/mek":
                    ct = native.aes_gcm_encrypt(base64.b64decode(d["plaintext"]), fake.key, os.urandom(12))
                    return self._send(200, {"data": {"ciphertext": "vault:v1:" + base64.b64encode(ct).decode()}})
                if self.path == "/v1/transit/decrypt/mek":
                    ct = base64.b64decode(d["ciphertext"][len("vault:v1:"):])
                    pt = native.aes_gcm_decrypt(ct, fake.key)
                    return self._send(200, {"data": {"plaintext": base64.b64encode(pt).decode()}})
                self._send(404, {})

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()


def test_vault_transit_and_kv():
    v = FakeVault()
    try:
        prov, sec = kms.from_config({"kms_provider": "vault", "vault_addr": v.url, "vault_token": "s.tok",
                                     "key_name": "mek"})
        kid = prov.master_key_id({})
        dek = os.urandom(32)
        wrapped = prov.encrypt(dek, kid)
        assert wrapped.startswith("vault:v1:")
        v.kv["model-dek"] = wrapped
        assert prov.decrypt(sec.get("model-dek"), kid) == dek
        with pytest.raises(kms.KmsError):
            kms.VaultTransit(v.url, "wrong", key_name="mek").master_key_id({})
    finally:
        v.srv.shutdown()
