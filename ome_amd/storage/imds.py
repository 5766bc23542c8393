"""OCI Instance Metadata Service client (reference ``pkg/imds``): v2 endpoint with the
``Authorization: Bearer Oracle`` header, v1 fallback; instance facts (realm, region, compartment,
shape), the instance's identity leaf certificate / key / intermediate, and the tenancy OCID from
the leaf certificate's ``opc-tenant:`` subject attribute (``imds_client.go``)."""
from __future__ import annotations

import json
import urllib.error
import urllib.request

V2 = "http://169.254.169.254/opc/v2"
V1 = "http://169.254.169.254/opc/v1"
TENANT_PREFIX = "opc-tenant:"


class ImdsError(RuntimeError):
    pass


class Imds:
    def __init__(self, base: str = V2, fallback: str = V1, timeout: float = 10.0):
        self.base, self.fallback, self.timeout = base.rstrip("/"), fallback.rstrip("/"), timeout

    def _get(self, suffix: str) -> bytes:
        last = None
        for base, hdr in ((self.base, {"Authorization": "Bearer Oracle"}), (self.fallback, {})):
            if not base:
                continue
            try:
                req = urllib.request.Request(base + suffix, headers=hdr)
                with urllib.request.urlopen(req, timeout=self.timeout) as r:
                    return r.read()
            except (urllib.error.URLError, OSError) as e:
                last = e
        raise ImdsError(f"IMDS {suffix}: {last}")

    def instance(self) -> dict:
        return json.loads(self._get("/instance/"))

    def region(self) -> str:
        d = self.instance()
        return d.get("canonicalRegionName") or (d.get("regionInfo") or {}).get("regionIdentifier") or d.get("region", "")

    def realm_domain(self) -> str:
        return (self.instance().get("regionInfo") or {}).get("realmDomainComponent") or "oraclecloud.com"

    def leaf_certificate(self) -> str:
        return self._get("/identity/cert.pem").decode()

    def leaf_private_key(self) -> str:
        return self._get("/identity/key.pem").decode()

    def intermediate_certificate(self) -> str:
        return self._get("/identity/intermediate.pem").decode()

    def tenancy_id(self, cert_pem: str | None = None) -> str:
        from ome_amd.io import native

        subj = native.x509_info(cert_pem or self.leaf_certificate())["subject"]
        return tenancy_from_subject(subj)


def tenancy_from_subject(subject: str) -> str:
    """``OU=opc-tenant:ocid1.tenancy...`` (or any attribute with that prefix) of an RFC 2253 line."""
    for part in subject.replace("+", ",").split(","):
        _, _, v = part.strip().partition("=")
        if v.startswith(TENANT_PREFIX):
            return v[len(TENANT_PREFIX):]
    raise ImdsError(f"no {TENANT_PREFIX} attribute in the instance certificate subject {subject!r}")


def pem_body(pem: str) -> str:
    """Base64 body of a PEM block (no armour lines, no newlines): the federation request format."""
    return "".join(l.strip() for l in pem.strip().splitlines() if not l.startswith("-----"))
