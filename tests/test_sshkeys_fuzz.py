"""A damaged private key file (a copy cut short, a changed byte, stray bytes) is refused
with a ``KeyParseError``, never another exception: the parsers walk DER and OpenSSH
structures whose lengths come from the file itself.  Property test over mutations of real
``ssh-keygen`` keys of every supported format."""

import base64
import subprocess

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.utils import sshkeys

FORMATS = [("rsa", ["-b", "2048", "-m", "PEM"]), ("rsa", ["-b", "2048"]), ("rsa", ["-b", "2048", "-m", "PKCS8"]),
           ("ecdsa", ["-m", "PEM"]), ("ecdsa", []), ("ecdsa", ["-m", "PKCS8"]), ("ed25519", [])]


@pytest.fixture(scope="module")
def keys(tmp_path_factory):
    d = tmp_path_factory.mktemp("keys")
    out = []
    for i, (kind, extra) in enumerate(FORMATS):
        path = d / f"k{i}"
        subprocess.run(["ssh-keygen", "-q", "-t", kind, *extra, "-N", "", "-f", str(path)], check=True)
        out.append(path.read_text())
    return out


@st.composite
def mutations(draw):
    kind = draw(st.sampled_from(["flip", "cut", "insert"]))
    return kind, draw(st.integers(0, 10 ** 6)), draw(st.binary(min_size=1, max_size=8))


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.integers(0, len(FORMATS) - 1), st.lists(mutations(), min_size=1, max_size=3))
def test_damaged_keys_are_refused_cleanly(keys, which, muts):
    lines = keys[which].splitlines()
    raw = bytearray(base64.b64decode("".join(lines[1:-1])))
    for kind, pos, data in muts:
        i = pos % max(1, len(raw))
        if kind == "flip" and raw:
            raw[i] ^= data[0] or 1
        elif kind == "cut":
            raw = raw[:i]
        else:
            raw[i:i] = data
    b64 = base64.b64encode(bytes(raw)).decode()
    text = lines[0] + "\n" + "\n".join(b64[j:j + 64] for j in range(0, len(b64), 64)) + "\n" + lines[-1] + "\n"
    try:
        sshkeys.parse_private_key(text).fingerprint_md5()
    except sshkeys.KeyParseError:
        pass


def test_intact_keys_still_parse(keys):
    for text in keys:
        assert sshkeys.parse_private_key(text).fingerprint_md5().count(":") == 15
