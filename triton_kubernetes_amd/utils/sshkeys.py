"""SSH private-key handling without third-party crypto libraries.

Covers what the reference gets from ``golang.org/x/crypto/ssh`` and
``triton-go/authentication``:

* parse PEM PKCS#1 (``RSA PRIVATE KEY``), PKCS#8 (``PRIVATE KEY``), SEC1
  (``EC PRIVATE KEY``) and OpenSSH (``OPENSSH PRIVATE KEY``, unencrypted) keys;
* the SSH wire-format public key blob and its colon-hex **MD5** fingerprint
  (``util/ssh_utils.go:13-42``: the Triton/Manta ``key_id``);
* RSA PKCS#1 v1.5 signatures (SHA-1/256/512) in pure Python, used for the
  Triton/Manta HTTP-signature scheme and GCP RS256 JWTs.  Non-RSA keys are
  signed through the ``openssl`` CLI when it can read the key.

Encrypted keys are decrypted through ``openssl`` when a passphrase is supplied.
"""

import base64
import hashlib
import os
import re
import struct
import subprocess
import tempfile
from dataclasses import dataclass
from typing import List, Optional, Tuple

from ..errors import TKError

_PEM_RE = re.compile(r"-----BEGIN ([A-Z0-9 ]+)-----\s*(.*?)\s*-----END \1-----", re.S)

OID_RSA = "1.2.840.113549.1.1.1"
OID_EC = "1.2.840.10045.2.1"
_CURVES = {
    "1.2.840.10045.3.1.7": ("nistp256", 32),
    "1.3.132.0.34": ("nistp384", 48),
    "1.3.132.0.35": ("nistp521", 66),
}
_DIGEST_INFO = {
    "sha1": bytes.fromhex("3021300906052b0e03021a05000414"),
    "sha256": bytes.fromhex("3031300d060960864801650304020105000420"),
    "sha512": bytes.fromhex("3051300d060960864801650304020305000440"),
}


class KeyParseError(TKError):
    pass


# --- DER -------------------------------------------------------------------------
def _der_read(data: bytes, pos: int) -> Tuple[int, bytes, int]:
    tag = data[pos]
    pos += 1
    length = data[pos]
    pos += 1
    if length & 0x80:
        n = length & 0x7F
        length = int.from_bytes(data[pos:pos + n], "big")
        pos += n
    return tag, data[pos:pos + length], pos + length


def _der_seq(data: bytes) -> List[Tuple[int, bytes]]:
    out = []
    pos = 0
    while pos < len(data):
        tag, val, pos = _der_read(data, pos)
        out.append((tag, val))
    return out


def _der_oid(val: bytes) -> str:
    first = val[0]
    parts = [first // 40, first % 40]
    acc = 0
    for b in val[1:]:
        acc = (acc << 7) | (b & 0x7F)
        if not b & 0x80:
            parts.append(acc)
            acc = 0
    return ".".join(str(p) for p in parts)


def _int(val: bytes) -> int:
    return int.from_bytes(val, "big", signed=False)


# --- SSH wire format --------------------------------------------------------------
def _ssh_string(b: bytes) -> bytes:
    return struct.pack(">I", len(b)) + b


def _ssh_mpint(n: int) -> bytes:
    if n == 0:
        return _ssh_string(b"")
    raw = n.to_bytes((n.bit_length() + 7) // 8, "big")
    if raw[0] & 0x80:
        raw = b"\x00" + raw
    return _ssh_string(raw)


class _Reader:
    def __init__(self, data: bytes):
        self.data, self.pos = data, 0

    def u32(self) -> int:
        (v,) = struct.unpack(">I", self.data[self.pos:self.pos + 4])
        self.pos += 4
        return v

    def string(self) -> bytes:
        n = self.u32()
        v = self.data[self.pos:self.pos + n]
        self.pos += n
        return v

    def mpint(self) -> int:
        return _int(self.string())


@dataclass
class PrivateKey:
    kind: str  # "rsa" | "ecdsa" | "ed25519"
    public_blob: bytes
    n: int = 0
    e: int = 0
    d: int = 0
    curve: str = ""
    path: Optional[str] = None
    pem: Optional[str] = None  # original PEM text (for openssl fallbacks)

    @property
    def ssh_type(self) -> str:
        return _Reader(self.public_blob).string().decode()

    def fingerprint_md5(self) -> str:
        return ":".join(f"{b:02x}" for b in hashlib.md5(self.public_blob).digest())

    # --- signing -----------------------------------------------------------------
    def sign(self, data: bytes, hash_name: str = "sha256") -> bytes:
        if self.kind == "rsa":
            return rsa_pkcs1v15_sign(self.n, self.d, data, hash_name)
        return _openssl_sign(self, data, hash_name)

    def http_signature_algorithm(self, hash_name: str = "sha256") -> str:
        prefix = {"rsa": "rsa", "ecdsa": "ecdsa", "ed25519": "ed25519"}[self.kind]
        return f"{prefix}-{hash_name}"


def rsa_pkcs1v15_sign(n: int, d: int, data: bytes, hash_name: str = "sha256") -> bytes:
    digest = hashlib.new(hash_name, data).digest()
    t = _DIGEST_INFO[hash_name] + digest
    k = (n.bit_length() + 7) // 8
    if k < len(t) + 11:
        raise TKError("RSA key too short for the requested digest")
    em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
    s = pow(int.from_bytes(em, "big"), d, n)
    return s.to_bytes(k, "big")


def rsa_pkcs1v15_verify(n: int, e: int, data: bytes, sig: bytes, hash_name: str = "sha256") -> bool:
    k = (n.bit_length() + 7) // 8
    m = pow(int.from_bytes(sig, "big"), e, n).to_bytes(k, "big")
    t = _DIGEST_INFO[hash_name] + hashlib.new(hash_name, data).digest()
    return m == b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t


def _openssl_sign(key: PrivateKey, data: bytes, hash_name: str) -> bytes:
    if key.pem is None or "OPENSSH" in key.pem:
        raise TKError(f"signing with {key.kind} keys in OpenSSH format is not supported; use an RSA key")
    with tempfile.NamedTemporaryFile("w", delete=False) as fh:
        fh.write(key.pem)
        kpath = fh.name
    try:
        args = ["openssl", "pkeyutl", "-sign", "-inkey", kpath, "-rawin"]
        if key.kind != "ed25519":
            args = ["openssl", "dgst", f"-{hash_name}", "-sign", kpath]
        proc = subprocess.run(args, input=data, capture_output=True, check=False)
        if proc.returncode != 0:
            raise TKError(f"openssl signing failed: {proc.stderr.decode(errors='replace').strip()}")
        return proc.stdout
    finally:
        os.unlink(kpath)


# --- parsing -----------------------------------------------------------------------
def _rsa_from_pkcs1(der: bytes) -> PrivateKey:
    (tag, body), = [_der_read(der, 0)[:2]]
    fields = _der_seq(body)
    n, e, d = _int(fields[1][1]), _int(fields[2][1]), _int(fields[3][1])
    blob = _ssh_string(b"ssh-rsa") + _ssh_mpint(e) + _ssh_mpint(n)
    return PrivateKey("rsa", blob, n=n, e=e, d=d)


def _ec_from_sec1(der: bytes, curve_oid: Optional[str] = None) -> PrivateKey:
    _, body, _ = _der_read(der, 0)
    fields = _der_seq(body)
    pub = None
    for tag, val in fields[2:]:
        if tag == 0xA0 and curve_oid is None:
            curve_oid = _der_oid(_der_read(val, 0)[1])
        elif tag == 0xA1:
            bit = _der_read(val, 0)[1]
            pub = bit[1:]
    if curve_oid not in _CURVES or pub is None:
        raise KeyParseError("unsupported EC key")
    curve = _CURVES[curve_oid][0]
    blob = _ssh_string(f"ecdsa-sha2-{curve}".encode()) + _ssh_string(curve.encode()) + _ssh_string(pub)
    return PrivateKey("ecdsa", blob, curve=curve)


def _from_pkcs8(der: bytes) -> PrivateKey:
    _, body, _ = _der_read(der, 0)
    fields = _der_seq(body)
    alg = _der_seq(fields[1][1])
    oid = _der_oid(alg[0][1])
    inner = fields[2][1]
    if oid == OID_RSA:
        return _rsa_from_pkcs1(inner)
    if oid == OID_EC:
        return _ec_from_sec1(inner, _der_oid(alg[1][1]))
    if oid == "1.3.101.112":  # Ed25519: public key not present in PKCS#8 v1
        raise KeyParseError("Ed25519 PKCS#8 keys are not supported; use an OpenSSH-format key")
    raise KeyParseError(f"unsupported key algorithm {oid}")


def _from_openssh(raw: bytes) -> PrivateKey:
    magic = b"openssh-key-v1\x00"
    if not raw.startswith(magic):
        raise KeyParseError("invalid openssh private key")
    r = _Reader(raw[len(magic):])
    cipher, kdf, _kdfopts = r.string(), r.string(), r.string()
    nkeys = r.u32()
    if nkeys != 1:
        raise KeyParseError("multi-key openssh files are not supported")
    public_blob = r.string()
    if cipher != b"none" or kdf != b"none":
        raise KeyParseError("ssh: this private key is passphrase protected")
    priv = _Reader(r.string())
    if priv.u32() != priv.u32():
        raise KeyParseError("corrupt openssh private key")
    ktype = priv.string().decode()
    if ktype == "ssh-rsa":
        n, e, d = priv.mpint(), priv.mpint(), priv.mpint()
        return PrivateKey("rsa", public_blob, n=n, e=e, d=d)
    if ktype == "ssh-ed25519":
        return PrivateKey("ed25519", public_blob)
    if ktype.startswith("ecdsa-sha2-"):
        return PrivateKey("ecdsa", public_blob, curve=ktype[len("ecdsa-sha2-"):])
    raise KeyParseError(f"unsupported openssh key type {ktype}")


def parse_private_key(text: str, passphrase: Optional[str] = None) -> PrivateKey:
    m = _PEM_RE.search(text)
    if not m:
        raise KeyParseError("ssh: no key found")
    label, body = m.group(1), m.group(2)
    headers, _, b64 = body.rpartition("\n\n") if "Proc-Type" in body else ("", "", body)
    if "ENCRYPTED" in label or "ENCRYPTED" in headers:
        if passphrase is None:
            raise KeyParseError("ssh: this private key is passphrase protected")
        return parse_private_key(_openssl_decrypt(text, passphrase))
    try:
        der = base64.b64decode("".join(b64.split()))
        if label == "RSA PRIVATE KEY":
            key = _rsa_from_pkcs1(der)
        elif label == "PRIVATE KEY":
            key = _from_pkcs8(der)
        elif label == "EC PRIVATE KEY":
            key = _ec_from_sec1(der)
        else:
            key = None
    except (IndexError, KeyError, TypeError, ValueError, struct.error) as exc:
        # a truncated or damaged file (a copy cut short, an edited line): the reference's
        # ssh.ParsePrivateKey errors the same way, without a stack
        raise KeyParseError(f"ssh: the {label} is damaged or truncated ({type(exc).__name__})") from None
    if key is not None:
        pass
    elif label == "OPENSSH PRIVATE KEY":
        try:
            key = _from_openssh(der)
        except KeyParseError as exc:
            if "passphrase" not in str(exc) or passphrase is None:
                raise
            return parse_private_key(_openssh_decrypt(text, passphrase))
        except (IndexError, KeyError, TypeError, ValueError, struct.error) as exc:
            raise KeyParseError(f"ssh: the {label} is damaged or truncated ({type(exc).__name__})") from None
    else:
        raise KeyParseError(f"ssh: unsupported key type \"{label}\"")
    key.pem = text
    return key


def _openssl_decrypt(text: str, passphrase: str) -> str:
    """Decrypt an encrypted PEM key (passphrase passed through the environment)."""
    env = dict(os.environ, TK_KEY_PASS=passphrase)
    proc = subprocess.run(["openssl", "pkey", "-passin", "env:TK_KEY_PASS", "-traditional"],
                          input=text.encode(), capture_output=True, check=False, env=env)
    if proc.returncode != 0:
        raise KeyParseError("x509: decryption password incorrect")
    return proc.stdout.decode()


def _openssh_decrypt(text: str, passphrase: str) -> str:
    """Decrypt an encrypted OpenSSH-format key on a private temp copy via ssh-keygen.

    The passphrase goes to ssh-keygen's stdin, never its argv (which every local user can
    read in ``ps``): without a controlling terminal (a new session) ssh-keygen reads the
    old passphrase from stdin."""
    with tempfile.TemporaryDirectory(prefix="tk-key-") as d:
        path = os.path.join(d, "key")
        with open(os.open(path, os.O_WRONLY | os.O_CREAT, 0o600), "w") as fh:
            fh.write(text)
        proc = subprocess.run(["ssh-keygen", "-q", "-p", "-N", "", "-f", path], input=(passphrase + "\n").encode(),
                              capture_output=True, check=False, start_new_session=True)
        if proc.returncode != 0:
            raise KeyParseError("ssh: incorrect passphrase")
        with open(path, "r", encoding="utf-8") as fh:
            return fh.read()


def load_private_key(path: str, passphrase: Optional[str] = None) -> PrivateKey:
    try:
        with open(path, "r", encoding="utf-8") as fh:
            text = fh.read()
    except FileNotFoundError as exc:
        raise TKError(f"Unable to read private key: open {path}: no such file or directory") from exc
    except OSError as exc:
        raise TKError(f"Unable to read private key: open {path}: {exc.strerror.lower()}") from exc
    key = parse_private_key(text, passphrase)
    key.path = path
    return key


def public_key_fingerprint(path: str, passphrase_cb=None) -> str:
    """Colon-hex MD5 fingerprint of the key's public half (``util/ssh_utils.go:13``).

    ``passphrase_cb`` is consulted only for encrypted keys; in non-interactive
    mode callers pass ``None`` and get an error instead of a hanging prompt
    (fixes SURVEY.md §7.5 Q14).
    """
    try:
        key = load_private_key(path)
    except KeyParseError as first:
        if passphrase_cb is None:
            raise TKError(f"Unable to parse private key: {first}") from first
        try:
            key = load_private_key(path, passphrase_cb())
        except KeyParseError as exc:
            raise TKError(f"Unable to parse private key: {exc}") from exc
    return key.fingerprint_md5()
