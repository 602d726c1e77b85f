"""Serving certificate for the in-cluster admission webhook (``openssl`` CLI).

The API server calls the webhook over TLS and verifies it against the
``caBundle`` of the MutatingWebhookConfiguration, so the add-ons carry a small
private CA and a serving certificate for ``<service>.<namespace>.svc``.  The
Terraform add-on module makes the same pair with the ``tls`` provider
(``tls_self_signed_cert`` + ``tls_locally_signed_cert``); the DirectExecutor uses
this module (``cryptography`` is not a dependency; ``openssl`` is on every operator
machine the SSH path already needs).
"""

import os
import subprocess
import tempfile
from dataclasses import dataclass
from typing import List

from ..errors import TKError


@dataclass
class ServingCert:
    ca_pem: str
    cert_pem: str
    key_pem: str


def _openssl(args: List[str], cwd: str) -> None:
    proc = subprocess.run(["openssl", *args], cwd=cwd, capture_output=True, text=True, check=False)
    if proc.returncode != 0:
        raise TKError(f"openssl {args[0]} failed: {proc.stderr.strip()[-400:]}")


def serving_cert(service: str, namespace: str, days: int = 3650) -> ServingCert:
    """A fresh CA and a serving certificate for ``service.namespace.svc`` (EC P-256)."""
    dns = [service, f"{service}.{namespace}", f"{service}.{namespace}.svc",
           f"{service}.{namespace}.svc.cluster.local"]
    with tempfile.TemporaryDirectory(prefix="tk-tls-") as d:
        ec = ["-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes"]
        _openssl(["req", "-x509", *ec, "-keyout", "ca.key", "-out", "ca.crt", "-days", str(days),
                  "-subj", f"/CN={service}-ca", "-addext", "basicConstraints=critical,CA:TRUE",
                  "-addext", "keyUsage=critical,keyCertSign,cRLSign"], d)
        _openssl(["req", "-new", *ec, "-keyout", "tls.key", "-out", "tls.csr",
                  "-subj", f"/CN={dns[2]}"], d)
        with open(os.path.join(d, "ext.cnf"), "w", encoding="utf-8") as fh:
            fh.write("basicConstraints=CA:FALSE\nkeyUsage=critical,digitalSignature,keyEncipherment\n"
                     "extendedKeyUsage=serverAuth\nsubjectAltName=" + ",".join(f"DNS:{n}" for n in dns) + "\n")
        _openssl(["x509", "-req", "-in", "tls.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial",
                  "-out", "tls.crt", "-days", str(days), "-extfile", "ext.cnf"], d)

        def read(name: str) -> str:
            with open(os.path.join(d, name), "r", encoding="utf-8") as fh:
                return fh.read()

        return ServingCert(read("ca.crt"), read("tls.crt"), read("tls.key"))


__all__ = ["ServingCert", "serving_cert"]
