"""Small private CAs and the certificates they sign (``openssl`` CLI).

Two users:

* the in-cluster admission webhook: the API server calls it over TLS and verifies it
  against the ``caBundle`` of the MutatingWebhookConfiguration, so the add-ons carry a
  private CA and a serving certificate for ``<service>.<namespace>.svc``
  (:func:`serving_cert`).  The Terraform add-on module makes the same pair with the
  ``tls`` provider (``tls_self_signed_cert`` + ``tls_locally_signed_cert``);
* the node agents: one CA per cluster manager signs each node agent's serving
  certificate for the node's address (``node/security.py``).

``cryptography`` is not a dependency; ``openssl`` is on every operator machine the SSH
path already needs.  Keys are EC P-256.
"""

import ipaddress
import os
import subprocess
import tempfile
from dataclasses import dataclass
from typing import List, Sequence

from ..errors import TKError


@dataclass
class ServingCert:
    ca_pem: str
    cert_pem: str
    key_pem: str


@dataclass
class CA:
    cert_pem: str
    key_pem: str


_EC = ["-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes"]


def _openssl(args: List[str], cwd: str) -> None:
    proc = subprocess.run(["openssl", *args], cwd=cwd, capture_output=True, text=True, check=False)
    if proc.returncode != 0:
        raise TKError(f"openssl {args[0]} failed: {proc.stderr.strip()[-400:]}")


def _read(d: str, name: str) -> str:
    with open(os.path.join(d, name), "r", encoding="utf-8") as fh:
        return fh.read()


def make_ca(common_name: str, days: int = 3650) -> CA:
    with tempfile.TemporaryDirectory(prefix="tk-tls-") as d:
        _openssl(["req", "-x509", *_EC, "-keyout", "ca.key", "-out", "ca.crt", "-days", str(days),
                  "-subj", f"/CN={common_name}", "-addext", "basicConstraints=critical,CA:TRUE",
                  "-addext", "keyUsage=critical,keyCertSign,cRLSign"], d)
        return CA(_read(d, "ca.crt"), _read(d, "ca.key"))


def san_entries(names: Sequence[str]) -> List[str]:
    """``IP:`` for addresses, ``DNS:`` for everything else."""
    out = []
    for n in names:
        try:
            ipaddress.ip_address(n)
            out.append(f"IP:{n}")
        except ValueError:
            out.append(f"DNS:{n}")
    return out


def issue(ca: CA, common_name: str, names: Sequence[str], days: int = 825, server: bool = True) -> ServingCert:
    """A key and a certificate for ``names`` (subjectAltName), signed by ``ca``."""
    with tempfile.TemporaryDirectory(prefix="tk-tls-") as d:
        with open(os.path.join(d, "ca.crt"), "w", encoding="utf-8") as fh:
            fh.write(ca.cert_pem)
        with open(os.path.join(d, "ca.key"), "w", encoding="utf-8") as fh:
            fh.write(ca.key_pem)
        os.chmod(os.path.join(d, "ca.key"), 0o600)
        _openssl(["req", "-new", *_EC, "-keyout", "tls.key", "-out", "tls.csr", "-subj", f"/CN={common_name}"], d)
        usage = "serverAuth" if server else "clientAuth"
        with open(os.path.join(d, "ext.cnf"), "w", encoding="utf-8") as fh:
            fh.write("basicConstraints=CA:FALSE\nkeyUsage=critical,digitalSignature,keyEncipherment\n"
                     f"extendedKeyUsage={usage}\nsubjectAltName=" + ",".join(san_entries(names)) + "\n")
        _openssl(["x509", "-req", "-in", "tls.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial",
                  "-out", "tls.crt", "-days", str(days), "-extfile", "ext.cnf"], d)
        return ServingCert(ca.cert_pem, _read(d, "tls.crt"), _read(d, "tls.key"))


def serving_cert(service: str, namespace: str, days: int = 3650) -> ServingCert:
    """A fresh CA and a serving certificate for ``service.namespace.svc`` (EC P-256)."""
    dns = [service, f"{service}.{namespace}", f"{service}.{namespace}.svc",
           f"{service}.{namespace}.svc.cluster.local"]
    ca = make_ca(f"{service}-ca", days)
    return issue(ca, dns[2], dns, days)


__all__ = ["CA", "ServingCert", "make_ca", "issue", "san_entries", "serving_cert"]
