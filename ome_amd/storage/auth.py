"""Cloud credentials for the object-store clients (``pkg/auth``, ``pkg/principals``, ``pkg/imds``).

Same contract as the reference's ``auth.Credentials`` (``pkg/auth/interfaces.go:62-81``): every
credential knows its provider and auth type, can produce a bearer token where the provider uses
one, signs an HTTP request, refreshes itself and reports expiry.  A :class:`Factory` builds them
from ``{"provider", "auth_type", "extra", "fallback"}`` configs with a bounded fallback chain
(``pkg/auth/factory.go``: depth <= 10).

Signing schemes, written against the providers' published specifications with the standard
library only (no cloud SDK in this image):

* AWS Signature Version 4 (HMAC-SHA256 key derivation, canonical request / string to sign);
* OCI HTTP signatures (draft-cavage, ``rsa-sha256`` over ``date (request-target) host`` plus
  ``content-length content-type x-content-sha256`` for bodies) for user principals (API key) and
  resource / workload-identity principals (``ST$<token>`` key ids);
* Azure Storage Shared Key (HMAC-SHA256 over the canonicalised request) and SAS tokens;
* bearer tokens from the GCP metadata server, the Azure IMDS identity endpoint, AWS IMDSv2
  instance profiles and STS web identity.

RSA PKCS#1 v1.5 signatures are computed with Python integers from a PEM key (PKCS#1 or
unencrypted PKCS#8), parsed by a minimal DER reader.
"""
from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import hmac
import json
import os
import threading
import time
import urllib.parse
import urllib.request
from dataclasses import dataclass, field
from email.utils import formatdate

AWS, GCP, AZURE, OCI, GITHUB = "aws", "gcp", "azure", "oci", "github"


class AuthError(RuntimeError):
    pass


def _http(method: str, url: str, headers: dict | None = None, data: bytes | None = None, timeout: float = 5.0):
    req = urllib.request.Request(url, data=data, method=method, headers=headers or {})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.status, dict(r.headers), r.read()


# ------------------------------------------------------------------ base
class Credentials:
    provider = ""
    auth_type = ""

    def token(self) -> str | None:
        """Bearer token where the provider uses one (None: request signing instead)."""
        return None

    def sign(self, method: str, url: str, headers: dict, body: bytes = b"") -> dict:
        """Return ``headers`` plus the authentication headers for this request."""
        tok = self.token()
        out = dict(headers)
        if tok:
            out["Authorization"] = f"Bearer {tok}"
        return out

    def refresh(self) -> None:
        pass

    def expired(self) -> bool:
        return False


class _Expiring(Credentials):
    """Token credential with an expiry, refreshed (thread-safely) a minute ahead of time."""

    skew = 60.0

    def __init__(self):
        self._tok: str | None = None
        self._exp = 0.0
        self._lock = threading.Lock()

    def _fetch(self) -> tuple[str, float]:  # (token, absolute expiry epoch seconds)
        raise NotImplementedError

    def expired(self) -> bool:
        return self._tok is None or time.time() > self._exp - self.skew

    def refresh(self) -> None:
        with self._lock:
            self._tok, self._exp = self._fetch()

    def token(self) -> str | None:
        if self.expired():
            self.refresh()
        return self._tok


# ------------------------------------------------------------------ AWS SigV4
def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def sigv4_headers(method: str, url: str, headers: dict, body_sha256: str, access_key: str, secret_key: str,
                  region: str, service: str, amz_date: str | None = None, session_token: str | None = None) -> dict:
    """AWS Signature Version 4: returns ``headers`` + ``x-amz-date`` (+ token) + ``Authorization``.
    ``body_sha256`` is the hex SHA-256 of the payload (or ``UNSIGNED-PAYLOAD``)."""
    u = urllib.parse.urlsplit(url)
    amz_date = amz_date or _dt.datetime.now(_dt.timezone.utc).strftime("%Y%m%dT%H%M%SZ")
    day = amz_date[:8]
    h = {k: v for k, v in headers.items()}
    h["x-amz-date"] = amz_date
    if session_token:
        h["x-amz-security-token"] = session_token
    host = u.netloc
    canon_h = {"host": host}
    for k, v in h.items():
        canon_h[k.lower()] = " ".join(str(v).strip().split())
    signed = sorted(canon_h)
    path = urllib.parse.quote(urllib.parse.unquote(u.path or "/"), safe="/-_.~")
    q = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    cq = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}" for k, v in sorted(q))
    creq = "\n".join([method, path, cq, "".join(f"{k}:{canon_h[k]}\n" for k in signed), ";".join(signed),
                      body_sha256])
    scope = f"{day}/{region}/{service}/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(creq.encode()).hexdigest()])
    k = _hmac(_hmac(_hmac(_hmac(("AWS4" + secret_key).encode(), day), region), service), "aws4_request")
    sig = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
    h["Authorization"] = (f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, SignedHeaders={';'.join(signed)}, "
                          f"Signature={sig}")
    return h


class AwsKeys(Credentials):
    """Static / environment access keys (``AWSAccessKey``)."""
    provider, auth_type = AWS, "AWSAccessKey"

    def __init__(self, access_key: str, secret_key: str, session_token: str | None = None, region: str = "us-east-1",
                 service: str = "s3", expiry: float | None = None):
        self.access_key, self.secret_key, self.session_token = access_key, secret_key, session_token
        self.region, self.service, self.expiry = region, service, expiry

    def keys(self) -> tuple[str, str, str | None]:
        return self.access_key, self.secret_key, self.session_token

    def expired(self) -> bool:
        return self.expiry is not None and time.time() > self.expiry - 60

    def sign(self, method, url, headers, body=b""):
        ak, sk, tok = self.keys()
        h = dict(headers)
        sha = h.get("x-amz-content-sha256") or hashlib.sha256(body or b"").hexdigest()
        h["x-amz-content-sha256"] = sha
        return sigv4_headers(method, url, h, sha, ak, sk, self.region, self.service, session_token=tok)


class _AwsRefreshing(AwsKeys):
    def __init__(self, region: str = "us-east-1", service: str = "s3"):
        super().__init__("", "", None, region, service)
        self._lock = threading.Lock()
        self.expiry = 0.0

    def _fetch(self) -> tuple[str, str, str | None, float]:
        raise NotImplementedError

    def refresh(self) -> None:
        with self._lock:
            self.access_key, self.secret_key, self.session_token, self.expiry = self._fetch()

    def keys(self):
        if self.expired() or not self.access_key:
            self.refresh()
        return self.access_key, self.secret_key, self.session_token


def _iso_epoch(s: str) -> float:
    return _dt.datetime.fromisoformat(s.replace("Z", "+00:00")).timestamp()


class AwsInstanceProfile(_AwsRefreshing):
    """EC2 instance-profile role keys over IMDSv2 (session token PUT, then the role document)."""
    auth_type = "AWSInstanceProfile"

    def __init__(self, endpoint: str | None = None, **kw):
        super().__init__(**kw)
        self.endpoint = (endpoint or os.environ.get("AWS_EC2_METADATA_SERVICE_ENDPOINT", "http://169.254.169.254")
                         ).rstrip("/")

    def _fetch(self):
        try:
            _, _, tok = _http("PUT", self.endpoint + "/latest/api/token",
                              {"X-aws-ec2-metadata-token-ttl-seconds": "21600"})
            hdr = {"X-aws-ec2-metadata-token": tok.decode()}
            _, _, role = _http("GET", self.endpoint + "/latest/meta-data/iam/security-credentials/", hdr)
            role = role.decode().strip().splitlines()[0]
            _, _, doc = _http("GET", self.endpoint + "/latest/meta-data/iam/security-credentials/" + role, hdr)
        except OSError as e:
            raise AuthError(f"IMDS unavailable at {self.endpoint}: {e}") from e
        d = json.loads(doc)
        return d["AccessKeyId"], d["SecretAccessKey"], d.get("Token"), _iso_epoch(d["Expiration"])


class AwsWebIdentity(_AwsRefreshing):
    """IRSA-style ``AssumeRoleWithWebIdentity`` (token file + role ARN) against STS."""
    auth_type = "AWSWebIdentity"

    def __init__(self, role_arn: str | None = None, token_file: str | None = None, sts_endpoint: str | None = None,
                 session_name: str = "ome-agent", **kw):
        super().__init__(**kw)
        self.role_arn = role_arn or os.environ.get("AWS_ROLE_ARN", "")
        self.token_file = token_file or os.environ.get("AWS_WEB_IDENTITY_TOKEN_FILE", "")
        self.sts = (sts_endpoint or os.environ.get("AWS_STS_ENDPOINT", "https://sts.amazonaws.com")).rstrip("/")
        self.session_name = session_name
        if not self.role_arn or not self.token_file:
            raise AuthError("web identity needs AWS_ROLE_ARN and AWS_WEB_IDENTITY_TOKEN_FILE")

    def _fetch(self):
        import xml.etree.ElementTree as ET

        tok = open(self.token_file).read().strip()
        q = urllib.parse.urlencode({"Action": "AssumeRoleWithWebIdentity", "Version": "2011-06-15",
                                    "RoleArn": self.role_arn, "RoleSessionName": self.session_name,
                                    "WebIdentityToken": tok})
        try:
            _, _, body = _http("GET", f"{self.sts}/?{q}")
        except OSError as e:
            raise AuthError(f"STS AssumeRoleWithWebIdentity failed: {e}") from e
        root = ET.fromstring(body)

        def find(tag):
            for el in root.iter():
                if el.tag.rsplit("}", 1)[-1] == tag:
                    return el.text
            raise AuthError(f"STS response without {tag}")

        return find("AccessKeyId"), find("SecretAccessKey"), find("SessionToken"), _iso_epoch(find("Expiration"))


# ------------------------------------------------------------------ GCP
class GcpToken(Credentials):
    provider, auth_type = GCP, "GCPAccessToken"

    def __init__(self, token: str):
        self._t = token

    def token(self):
        return self._t


class GcpMetadata(_Expiring):
    """Workload identity / default service account token from the GCE metadata server."""
    provider, auth_type = GCP, "GCPWorkloadIdentity"

    def __init__(self, endpoint: str | None = None, account: str = "default"):
        super().__init__()
        host = endpoint or os.environ.get("GCE_METADATA_HOST", "metadata.google.internal")
        self.endpoint = host if host.startswith("http") else "http://" + host
        self.account = account

    def _fetch(self):
        try:
            _, _, body = _http("GET", f"{self.endpoint}/computeMetadata/v1/instance/service-accounts/{self.account}/token",
                               {"Metadata-Flavor": "Google"})
        except OSError as e:
            raise AuthError(f"GCP metadata server unavailable: {e}") from e
        d = json.loads(body)
        return d["access_token"], time.time() + float(d.get("expires_in", 3600))


# ------------------------------------------------------------------ Azure
class AzureSharedKey(Credentials):
    """Storage account key: ``SharedKey <account>:<HMAC-SHA256(canonicalised request)>``."""
    provider, auth_type = AZURE, "AzureAccountKey"

    def __init__(self, account: str, key_b64: str, version: str = "2021-08-06"):
        self.account, self.key, self.version = account, base64.b64decode(key_b64), version

    def sign(self, method, url, headers, body=b""):
        h = {k.lower(): str(v) for k, v in headers.items()}
        h.setdefault("x-ms-date", formatdate(usegmt=True))
        h.setdefault("x-ms-version", self.version)
        u = urllib.parse.urlsplit(url)
        clen = h.get("content-length", "")
        if clen == "0":
            clen = ""
        std = [method, h.get("content-encoding", ""), h.get("content-language", ""), clen, h.get("content-md5", ""),
               h.get("content-type", ""), "", h.get("if-modified-since", ""), h.get("if-match", ""),
               h.get("if-none-match", ""), h.get("if-unmodified-since", ""), h.get("range", "")]
        ms = "".join(f"{k}:{' '.join(h[k].split())}\n" for k in sorted(h) if k.startswith("x-ms-"))
        res = f"/{self.account}{urllib.parse.unquote(u.path or '/')}"
        params: dict[str, list[str]] = {}
        for k, v in urllib.parse.parse_qsl(u.query, keep_blank_values=True):
            params.setdefault(k.lower(), []).append(v)
        for k in sorted(params):
            res += f"\n{k}:{','.join(sorted(params[k]))}"
        sts = "\n".join(std) + "\n" + ms + res
        sig = base64.b64encode(hmac.new(self.key, sts.encode(), hashlib.sha256).digest()).decode()
        out = {**headers, "x-ms-date": h["x-ms-date"], "x-ms-version": h["x-ms-version"]}
        out["Authorization"] = f"SharedKey {self.account}:{sig}"
        return out


class AzureSas(Credentials):
    """Shared access signature: appended to the URL by the client (:meth:`apply_url`)."""
    provider, auth_type = AZURE, "AzureSAS"

    def __init__(self, sas: str):
        self.sas = sas.lstrip("?")

    def apply_url(self, url: str) -> str:
        return url + ("&" if "?" in url else "?") + self.sas


class AzureManagedIdentity(_Expiring):
    provider, auth_type = AZURE, "AzureManagedIdentity"

    def __init__(self, endpoint: str | None = None, resource: str = "https://storage.azure.com/",
                 client_id: str | None = None):
        super().__init__()
        self.endpoint = (endpoint or os.environ.get("AZURE_IMDS_ENDPOINT", "http://169.254.169.254")).rstrip("/")
        self.resource, self.client_id = resource, client_id

    def _fetch(self):
        q = {"api-version": "2018-02-01", "resource": self.resource}
        if self.client_id:
            q["client_id"] = self.client_id
        try:
            _, _, body = _http("GET", f"{self.endpoint}/metadata/identity/oauth2/token?{urllib.parse.urlencode(q)}",
                               {"Metadata": "true"})
        except OSError as e:
            raise AuthError(f"Azure IMDS unavailable: {e}") from e
        d = json.loads(body)
        return d["access_token"], float(d.get("expires_on") or time.time() + 3600)

    def sign(self, method, url, headers, body=b""):
        out = super().sign(method, url, headers, body)
        out.setdefault("x-ms-version", "2021-08-06")
        return out


# ------------------------------------------------------------------ RSA (PKCS#1 v1.5, SHA-256)
def _der(buf: bytes, i: int) -> tuple[int, int, int]:
    """(tag, content start, content end) of the DER element at ``i``."""
    tag = buf[i]
    n = buf[i + 1]
    j = i + 2
    if n & 0x80:
        k = n & 0x7F
        n = int.from_bytes(buf[j:j + k], "big")
        j += k
    return tag, j, j + n


def _der_children(buf: bytes, start: int, end: int) -> list[tuple[int, int, int]]:
    out = []
    i = start
    while i < end:
        t, s, e = _der(buf, i)
        out.append((t, s, e))
        i = e
    return out


@dataclass
class RsaKey:
    """An RSA private key.  Signing and verification go through OpenSSL in libomeio (blinded CRT
    private operation, strict PKCS#1 v1.5 DigestInfo check); the parsed (n, e) remain available."""
    n: int
    e: int
    d: int
    pem: bytes = b""

    @property
    def size(self) -> int:
        return (self.n.bit_length() + 7) // 8

    @classmethod
    def from_pem(cls, pem: str | bytes) -> "RsaKey":
        text = pem.decode() if isinstance(pem, bytes) else pem
        if "ENCRYPTED" in text:
            raise AuthError("encrypted private keys are not supported (decrypt the key into the Secret)")
        body = "".join(l for l in text.strip().splitlines() if not l.startswith("-----"))
        der = base64.b64decode(body)
        t, s, e = _der(der, 0)
        kids = _der_children(der, s, e)
        if len(kids) == 3 and kids[1][0] == 0x30:     # PKCS#8: version, algorithm, OCTET STRING(PKCS#1)
            inner = der[kids[2][1]:kids[2][2]]
            t, s, e = _der(inner, 0)
            der, kids = inner, _der_children(inner, s, e)
        ints = [int.from_bytes(der[s:e], "big") for t, s, e in kids if t == 0x02]
        if len(ints) < 4:
            raise AuthError("not an RSA private key")
        return cls(n=ints[1], e=ints[2], d=ints[3], pem=text.encode())

    def sign_sha256(self, msg: bytes) -> bytes:
        from ome_amd.io import native

        try:
            return native.rsa_sign_sha256(self.pem, msg)
        except native.OmeIOError as e:
            raise AuthError(f"RSA signing failed: {e}") from e

    def verify_sha256(self, msg: bytes, sig: bytes) -> bool:
        """Strict PKCS#1 v1.5 verification (the whole encoded message, not a prefix/suffix match)."""
        from ome_amd.io import native

        if len(sig) != self.size:
            return False
        return native.rsa_verify_sha256(self.pem, msg, sig)


# ------------------------------------------------------------------ OCI
class OciSigner(Credentials):
    """OCI request signing (``Signature version="1",keyId=...,algorithm="rsa-sha256"``)."""
    provider = OCI

    def __init__(self, key: RsaKey, key_id: str):
        self.key, self._key_id = key, key_id

    def key_id(self) -> str:
        return self._key_id

    def sign(self, method, url, headers, body=b""):
        u = urllib.parse.urlsplit(url)
        h = {k.lower(): str(v) for k, v in headers.items()}
        h.setdefault("date", formatdate(usegmt=True))
        h["host"] = u.netloc
        target = f"{method.lower()} {u.path or '/'}" + (f"?{u.query}" if u.query else "")
        names = ["date", "(request-target)", "host"]
        if method.upper() in ("PUT", "POST", "PATCH") and "x-content-sha256" not in h and \
                h.get("content-type") != "application/octet-stream":
            h["x-content-sha256"] = base64.b64encode(hashlib.sha256(body or b"").digest()).decode()
            h["content-length"] = str(len(body or b""))
            h.setdefault("content-type", "application/json")
            names += ["content-length", "content-type", "x-content-sha256"]
        lines = [f"(request-target): {target}" if n == "(request-target)" else f"{n}: {h[n]}" for n in names]
        sig = base64.b64encode(self.key.sign_sha256("\n".join(lines).encode())).decode()
        out = {k: v for k, v in headers.items()}
        for n in names:
            if n != "(request-target)":
                out[n] = h[n]
        out["authorization"] = (f'Signature version="1",keyId="{self.key_id()}",algorithm="rsa-sha256",'
                                f'headers="{" ".join(names)}",signature="{sig}"')
        return out


class OciUserPrincipal(OciSigner):
    """API-key user principal: ``<tenancy>/<user>/<fingerprint>`` key id (``~/.oci/config``)."""
    auth_type = "OCIUserPrincipal"

    def __init__(self, tenancy: str, user: str, fingerprint: str, key_pem: str | bytes):
        super().__init__(RsaKey.from_pem(key_pem), f"{tenancy}/{user}/{fingerprint}")

    @classmethod
    def from_config(cls, path: str | None = None, profile: str = "DEFAULT") -> "OciUserPrincipal":
        import configparser

        path = os.path.expanduser(path or os.environ.get("OCI_CONFIG_FILE", "~/.oci/config"))
        cp = configparser.ConfigParser()
        if not cp.read(path) or profile not in cp:
            raise AuthError(f"OCI config {path} has no [{profile}] profile")
        sec = cp[profile]
        return cls(sec["tenancy"], sec["user"], sec["fingerprint"],
                   open(os.path.expanduser(sec["key_file"])).read())


class OciResourcePrincipal(OciSigner):
    """Resource principal v2.2: session token (RPST) + its private key from the environment;
    key id ``ST$<token>``."""
    auth_type = "OCIResourcePrincipal"

    def __init__(self, rpst: str | None = None, key_pem: str | None = None):
        rpst = rpst or os.environ.get("OCI_RESOURCE_PRINCIPAL_RPST", "")
        key_pem = key_pem or os.environ.get("OCI_RESOURCE_PRINCIPAL_PRIVATE_PEM", "")
        if rpst and os.path.isfile(rpst):
            rpst = open(rpst).read().strip()
        if key_pem and os.path.isfile(key_pem):
            key_pem = open(key_pem).read()
        if not rpst or not key_pem:
            raise AuthError("resource principal needs OCI_RESOURCE_PRINCIPAL_RPST and _PRIVATE_PEM")
        super().__init__(RsaKey.from_pem(key_pem), "ST$" + rpst)


class OciOkeWorkloadIdentity(OciSigner):
    """OKE workload identity: the pod's service-account token is exchanged at the cluster's
    proxymux endpoint for a resource-principal session token bound to a key we hold."""
    auth_type = "OCIOkeWorkloadIdentity"

    def __init__(self, key_pem: str | bytes, endpoint: str | None = None, sa_token_file: str | None = None):
        super().__init__(RsaKey.from_pem(key_pem), "")
        host = os.environ.get("KUBERNETES_SERVICE_HOST", "127.0.0.1")
        self.endpoint = (endpoint or os.environ.get("OCI_KUBERNETES_PROXYMUX_ENDPOINT",
                                                    f"https://{host}:12250")).rstrip("/")
        self.sa_token_file = sa_token_file or "/var/run/secrets/kubernetes.io/serviceaccount/token"
        self._token, self._exp = "", 0.0
        self._lock = threading.Lock()

    def _public_pem(self) -> str:
        # SubjectPublicKeyInfo of (n, e)
        def der_int(x):
            b = x.to_bytes((x.bit_length() + 8) // 8, "big")
            return b"\x02" + _der_len(len(b)) + b

        rsa_pub = der_int(self.key.n) + der_int(self.key.e)
        seq = b"\x30" + _der_len(len(rsa_pub)) + rsa_pub
        bit = b"\x03" + _der_len(len(seq) + 1) + b"\x00" + seq
        alg = bytes.fromhex("300d06092a864886f70d0101010500")
        spki = b"\x30" + _der_len(len(alg) + len(bit)) + alg + bit
        b64 = base64.b64encode(spki).decode()
        return "-----BEGIN PUBLIC KEY-----\n" + "\n".join(b64[i:i + 64] for i in range(0, len(b64), 64)) + \
            "\n-----END PUBLIC KEY-----\n"

    def key_id(self) -> str:
        with self._lock:
            if not self._token or time.time() > self._exp - 60:
                sa = open(self.sa_token_file).read().strip()
                body = json.dumps({"podKey": base64.b64encode(self._public_pem().encode()).decode()}).encode()
                try:
                    _, _, resp = _http("POST", self.endpoint + "/resourcePrincipalSessionTokens",
                                       {"Authorization": f"Bearer {sa}", "Content-Type": "application/json"}, body)
                except OSError as e:
                    raise AuthError(f"workload identity token exchange failed: {e}") from e
                d = json.loads(resp)
                tok = d.get("token", "")
                if tok.startswith("ST$"):
                    tok = tok[3:]
                self._token, self._exp = tok, time.time() + float(d.get("expires_in", 3600))
            return "ST$" + self._token


class OciInstancePrincipal(OciSigner):
    """Instance principal (reference ``pkg/principals/instance_principal.go`` -> the OCI SDK
    flow): the instance's identity certificate and key from IMDS (:mod:`.imds`) sign an X.509
    federation request to ``https://auth.<region>.<realm domain>/v1/x509`` (key id
    ``<tenancy>/fed-x509-sha256/<cert SHA-256 fingerprint>``) that binds a fresh session key
    pair (generated by OpenSSL in libomeio); requests are then signed with the session key and
    key id ``ST$<token>``, refreshed before the token's ``exp``."""
    auth_type = "OCIInstancePrincipal"

    def __init__(self, imds=None, region: str | None = None, auth_endpoint: str | None = None):
        from ome_amd.io import native
        from ome_amd.storage.imds import Imds

        self.imds = imds or Imds()
        priv, self._session_pub = native.rsa_keygen(2048)
        super().__init__(RsaKey.from_pem(priv), "")
        self.region = region or os.environ.get("OCI_REGION") or ""
        self.auth_endpoint = auth_endpoint or os.environ.get("OCI_SDK_AUTH_CLIENT_REGION_URL") or ""
        self._token, self._exp = "", 0.0
        self._lock = threading.Lock()

    def _endpoint(self) -> str:
        if self.auth_endpoint:
            return self.auth_endpoint.rstrip("/")
        region = self.region or self.imds.region()
        return f"https://auth.{region}.{self.imds.realm_domain()}"

    def _federate(self) -> tuple[str, float]:
        from ome_amd.io import native
        from ome_amd.storage.imds import pem_body

        cert, key, inter = (self.imds.leaf_certificate(), self.imds.leaf_private_key(),
                            self.imds.intermediate_certificate())
        info = native.x509_info(cert)
        tenancy = self.imds.tenancy_id(cert)
        body = json.dumps({"certificate": pem_body(cert), "publicKey": pem_body(self._session_pub),
                           "intermediateCertificates": [pem_body(inter)], "purpose": "DEFAULT",
                           "fingerprintAlgorithm": "SHA256"}).encode()
        fed = OciSigner(RsaKey.from_pem(key), f"{tenancy}/fed-x509-sha256/{info['sha256']}")
        url = self._endpoint() + "/v1/x509"
        h = fed.sign("POST", url, {"content-type": "application/json"}, body)
        try:
            _, _, resp = _http("POST", url, h, body, timeout=30.0)
        except OSError as e:
            raise AuthError(f"instance principal federation at {url} failed: {e}") from e
        tok = json.loads(resp).get("token", "")
        if not tok:
            raise AuthError("instance principal federation returned no token")
        return tok, _jwt_exp(tok)

    def key_id(self) -> str:
        with self._lock:
            if not self._token or time.time() > self._exp - 60:
                self._token, self._exp = self._federate()
            return "ST$" + self._token


def _jwt_exp(token: str, default_s: float = 1200.0) -> float:
    """``exp`` claim of a JWT (no signature check: the token is opaque to us, the service checks it)."""
    try:
        payload = token.split(".")[1]
        d = json.loads(base64.urlsafe_b64decode(payload + "=" * (-len(payload) % 4)))
        return float(d["exp"])
    except (IndexError, ValueError, KeyError, TypeError):
        return time.time() + default_s


def _der_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


# ------------------------------------------------------------------ GitHub
class GithubToken(Credentials):
    provider, auth_type = GITHUB, "GitHubToken"

    def __init__(self, token: str):
        self._t = token

    def token(self):
        return self._t


# ------------------------------------------------------------------ factory
@dataclass
class AuthConfig:
    provider: str
    auth_type: str
    region: str = ""
    extra: dict = field(default_factory=dict)
    fallback: "AuthConfig | None" = None

    @classmethod
    def from_dict(cls, d: dict) -> "AuthConfig":
        fb = d.get("fallback")
        return cls(d["provider"], d.get("auth_type") or d.get("authType", ""), d.get("region", ""),
                   dict(d.get("extra") or {}), cls.from_dict(fb) if fb else None)


MAX_FALLBACK_DEPTH = 10


class Factory:
    """``pkg/auth/factory.go``: build credentials from a config; on failure walk the fallback
    chain (bounded: a cyclic A -> B -> A config stops at depth 10)."""

    def __init__(self):
        self.makers: dict[tuple[str, str], callable] = {}
        self._register_defaults()

    def register(self, provider: str, auth_type: str, maker) -> None:
        self.makers[(provider, auth_type)] = maker

    def supported_providers(self) -> list[str]:
        return sorted({p for p, _ in self.makers})

    def supported_auth_types(self, provider: str) -> list[str]:
        return sorted(t for p, t in self.makers if p == provider)

    def create(self, cfg: AuthConfig | dict, _depth: int = 0) -> Credentials:
        if isinstance(cfg, dict):
            cfg = AuthConfig.from_dict(cfg)
        if _depth > MAX_FALLBACK_DEPTH:
            raise AuthError("auth fallback chain deeper than 10 (cycle?)")
        maker = self.makers.get((cfg.provider, cfg.auth_type))
        try:
            if maker is None:
                raise AuthError(f"unsupported auth {cfg.provider}/{cfg.auth_type}")
            return maker(cfg)
        except (AuthError, OSError, KeyError, ValueError) as e:
            if cfg.fallback is not None:
                return self.create(cfg.fallback, _depth + 1)
            raise AuthError(str(e)) from e

    def _register_defaults(self) -> None:
        env = os.environ.get
        x = lambda c, k, d=None: c.extra.get(k, d)  # noqa: E731
        region = lambda c: c.region or env("AWS_REGION") or env("AWS_DEFAULT_REGION") or "us-east-1"  # noqa: E731

        def aws_keys(c):
            ak = x(c, "access_key_id") or env("AWS_ACCESS_KEY_ID")
            sk = x(c, "secret_access_key") or env("AWS_SECRET_ACCESS_KEY")
            if not ak or not sk:
                raise AuthError("no AWS access keys")
            return AwsKeys(ak, sk, x(c, "session_token") or env("AWS_SESSION_TOKEN"), region(c))

        def aws_default(c):
            for mk in (aws_keys, lambda c: AwsWebIdentity(region=region(c)),
                       lambda c: AwsInstanceProfile(x(c, "imds_endpoint"), region=region(c))):
                try:
                    cred = mk(c)
                    if isinstance(cred, _AwsRefreshing):
                        cred.refresh()
                    return cred
                except (AuthError, OSError):
                    continue
            raise AuthError("no AWS credentials in env, web identity or instance profile")

        self.register(AWS, "AWSAccessKey", aws_keys)
        self.register(AWS, "AWSInstanceProfile", lambda c: AwsInstanceProfile(x(c, "imds_endpoint"), region=region(c)))
        self.register(AWS, "AWSWebIdentity", lambda c: AwsWebIdentity(x(c, "role_arn"), x(c, "token_file"),
                                                                      x(c, "sts_endpoint"), region=region(c)))
        self.register(AWS, "AWSDefault", aws_default)

        def gcp_token(c):
            t = x(c, "access_token") or env("GOOGLE_OAUTH_ACCESS_TOKEN")
            if not t:
                raise AuthError("no GCP access token")
            return GcpToken(t)

        self.register(GCP, "GCPAccessToken", gcp_token)
        self.register(GCP, "GCPWorkloadIdentity", lambda c: GcpMetadata(x(c, "metadata_host")))
        self.register(GCP, "GCPDefault", lambda c: gcp_token(c) if (x(c, "access_token") or
                                                                   env("GOOGLE_OAUTH_ACCESS_TOKEN"))
                      else GcpMetadata(x(c, "metadata_host")))

        def az_key(c):
            acct = x(c, "account_name") or env("AZURE_STORAGE_ACCOUNT")
            key = x(c, "account_key") or env("AZURE_STORAGE_KEY")
            if not acct or not key:
                raise AuthError("no Azure account key")
            return AzureSharedKey(acct, key)

        def az_sas(c):
            sas = x(c, "sas_token") or env("AZURE_STORAGE_SAS_TOKEN")
            if not sas:
                raise AuthError("no Azure SAS token")
            return AzureSas(sas)

        self.register(AZURE, "AzureAccountKey", az_key)
        self.register(AZURE, "AzureSAS", az_sas)
        self.register(AZURE, "AzureManagedIdentity", lambda c: AzureManagedIdentity(x(c, "imds_endpoint"),
                                                                                    client_id=x(c, "client_id")))

        def oci_user(c):
            if x(c, "key_pem") or x(c, "key_file"):
                pem = x(c, "key_pem") or open(os.path.expanduser(x(c, "key_file"))).read()
                return OciUserPrincipal(x(c, "tenancy"), x(c, "user"), x(c, "fingerprint"), pem)
            return OciUserPrincipal.from_config(x(c, "config_file"), x(c, "profile", "DEFAULT"))

        self.register(OCI, "OCIUserPrincipal", oci_user)
        self.register(OCI, "OCIResourcePrincipal", lambda c: OciResourcePrincipal(x(c, "rpst"), x(c, "key_pem")))
        def oci_instance(c):
            from ome_amd.storage.imds import Imds

            imds = Imds(x(c, "imds_endpoint") or "http://169.254.169.254/opc/v2",
                        x(c, "imds_fallback_endpoint") or "http://169.254.169.254/opc/v1")
            return OciInstancePrincipal(imds, x(c, "region"), x(c, "auth_endpoint_override") or x(c, "auth_endpoint"))

        self.register(OCI, "OCIInstancePrincipal", oci_instance)
        self.register(OCI, "InstancePrincipal", oci_instance)
        self.register(OCI, "OCIOkeWorkloadIdentity", lambda c: OciOkeWorkloadIdentity(
            x(c, "key_pem") or open(x(c, "key_file")).read(), x(c, "endpoint"), x(c, "sa_token_file")))

        def gh(c):
            t = x(c, "token") or env("GITHUB_TOKEN")
            if not t:
                raise AuthError("no GitHub token")
            return GithubToken(t)

        self.register(GITHUB, "GitHubToken", gh)
        self.register(GITHUB, "GitHubPersonalAccessToken", gh)


DEFAULT_FACTORY = Factory()
