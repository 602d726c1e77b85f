"""Backends (local / Manta / memory) and the stdlib cloud clients."""

import base64
import datetime
import json
import os
import threading
import time

import pytest

from triton_kubernetes_amd.backend import LocalBackend, MemoryBackend
from triton_kubernetes_amd.backend.manta import MantaBackend
from triton_kubernetes_amd.cloud.aws import sigv4_headers
from triton_kubernetes_amd.cloud.fake_manta import FakeManta
from triton_kubernetes_amd.cloud.gcp import make_jwt
from triton_kubernetes_amd.cloud.triton import HTTPSignatureSigner, MantaClient
from triton_kubernetes_amd.errors import BackendError, TKError
from triton_kubernetes_amd.state import State
from triton_kubernetes_amd.utils.sshkeys import load_private_key, rsa_pkcs1v15_verify

from helpers import make_ssh_key


def test_local_backend_layout(tmp_path):
    be = LocalBackend(str(tmp_path / "root"))
    assert be.states() == []
    st = be.state("mgr")
    assert st.doc == {}
    st.set_manager({"name": "mgr"})
    be.persist_state(st)
    assert be.states() == ["mgr"]
    assert os.path.isfile(tmp_path / "root" / "mgr" / "main.tf.json")
    assert be.state_terraform_config("mgr") == ("terraform.backend.local",
                                                {"path": str(tmp_path / "root" / "mgr" / "terraform.tfstate")})
    be.write_tfstate("mgr", b"{}")
    assert be.read_tfstate("mgr") == b"{}"
    be.delete_state("mgr")
    assert be.states() == []
    with pytest.raises(BackendError):
        be.state("../etc")


def test_local_backend_default_root_is_home(tk_home):
    be = LocalBackend()
    assert be.root == str(tk_home / ".triton-kubernetes")


def test_local_backend_lock_serialises_writers(tmp_path):
    be = LocalBackend(str(tmp_path))
    order = []

    def writer(i):
        with be.lock("mgr"):
            st = be.state("mgr")
            n = len(st.modules())
            st.set_module(f"m{i}", {"i": i})
            order.append(n)
            be.persist_state(st)

    ts = [threading.Thread(target=writer, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(be.state("mgr").modules()) == 8  # no lost update
    assert "mgr" in be.states() and not any(s.startswith(".") for s in be.states())


def test_memory_backend_records_calls():
    be = MemoryBackend(states={"a": b'{"module":{}}'}, state_names=["a", "b"])
    assert be.states() == ["a", "b"]
    be.persist_state(State("c"))
    assert "c" in be.states() and ("PersistState", ("c",)) in be.calls


@pytest.fixture
def manta(tmp_path):
    key_path = make_ssh_key(tmp_path / "id_rsa")
    key = load_private_key(key_path)
    fake = FakeManta("acct").start()
    fake.add_key(key)
    yield fake, key_path, key
    fake.stop()


def test_manta_backend_roundtrip_with_signatures(manta):
    fake, key_path, key = manta
    be = MantaBackend("acct", key_path, key.fingerprint_md5(), "https://triton", fake.url)
    assert be.states() == []
    st = be.state("mgr")
    st.set_manager({"name": "mgr"})
    be.persist_state(st)
    assert be.states() == ["mgr"]
    assert json.loads(be.state("mgr").bytes())["module"]["cluster-manager"]["name"] == "mgr"
    path, cfg = be.state_terraform_config("mgr")
    assert path == "terraform.backend.manta"
    assert cfg == {"account": "acct", "key_material": key_path, "key_id": key.fingerprint_md5(),
                   "path": "/triton-kubernetes/mgr"}
    with be.lock("mgr"):
        assert "/acct/stor/triton-kubernetes/mgr/.lock" in fake.objects
    assert "/acct/stor/triton-kubernetes/mgr/.lock" not in fake.objects
    be.write_tfstate("mgr", b'{"version":4}')
    be.delete_state("mgr")
    assert be.states() == [] and fake.rejected == 0


def test_manta_pagination_beyond_100(manta):
    fake, key_path, key = manta
    client = MantaClient(fake.url, HTTPSignatureSigner("acct", key))
    client.put_directory("/stor/triton-kubernetes")
    for i in range(130):
        client.put_directory(f"/stor/triton-kubernetes/m{i:03d}")
    entries = client.list_directory("/stor/triton-kubernetes", limit=50)
    assert len(entries) == 130  # the reference stops at 100


def test_manta_rejects_bad_signature(manta, tmp_path):
    fake, _, _ = manta
    other = load_private_key(make_ssh_key(tmp_path / "other"))
    client = MantaClient(fake.url, HTTPSignatureSigner("acct", other))
    with pytest.raises(TKError) as exc:
        client.put_directory("/stor/x")
    assert "403" in str(exc.value) and fake.rejected == 1


def test_http_signature_header(tmp_path):
    key = load_private_key(make_ssh_key(tmp_path / "k"))
    signer = HTTPSignatureSigner("acct", key)
    hdrs = {}
    signer("GET", "https://x/acct/machines", hdrs, b"")
    auth = hdrs["Authorization"]
    assert auth.startswith(f'Signature keyId="/acct/keys/{key.fingerprint_md5()}",algorithm="rsa-sha256"')
    sig = base64.b64decode(auth.split('signature="')[1].rstrip('"'))
    assert rsa_pkcs1v15_verify(key.n, key.e, f"date: {hdrs['Date']}".encode(), sig)


def test_sigv4_get_vanilla_vector():
    """AWS SigV4 test suite 'get-vanilla'."""
    now = datetime.datetime(2015, 8, 30, 12, 36, 0)
    hdrs = sigv4_headers("GET", "https://example.amazonaws.com/", b"", "AKIDEXAMPLE",
                         "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY", "us-east-1", "service", now=now)
    assert hdrs["Authorization"] == (
        "AWS4-HMAC-SHA256 Credential=AKIDEXAMPLE/20150830/us-east-1/service/aws4_request, "
        "SignedHeaders=host;x-amz-date, "
        "Signature=5fa00fa31553b73ebf1942676e86291e8372ff2a2260956d9b8aae1d763fbf31")


def test_gcp_jwt_rs256(tmp_path):
    key_path = make_ssh_key(tmp_path / "sa")
    key = load_private_key(key_path)
    creds = {"client_email": "sa@p.iam.gserviceaccount.com", "private_key": open(key_path).read(),
             "private_key_id": "abc"}
    jwt = make_jwt(creds, "scope", now=1000)
    head, claims, sig = jwt.split(".")
    pad = lambda s: s + "=" * (-len(s) % 4)  # noqa: E731
    assert json.loads(base64.urlsafe_b64decode(pad(head))) == {"alg": "RS256", "typ": "JWT", "kid": "abc"}
    c = json.loads(base64.urlsafe_b64decode(pad(claims)))
    assert c["iss"] == creds["client_email"] and c["exp"] == 4600
    assert rsa_pkcs1v15_verify(key.n, key.e, f"{head}.{claims}".encode(), base64.urlsafe_b64decode(pad(sig)))


def test_fingerprint_matches_ssh_keygen(tmp_path):
    import subprocess

    for kind in ("rsa", "ed25519", "ecdsa"):
        path = make_ssh_key(tmp_path / f"k_{kind}", kind)
        want = subprocess.run(["ssh-keygen", "-l", "-E", "md5", "-f", path], capture_output=True,
                              text=True).stdout.split()[1]
        assert want == "MD5:" + load_private_key(path).fingerprint_md5()


def test_encrypted_key_needs_passphrase(tmp_path):
    import subprocess

    from triton_kubernetes_amd.utils.sshkeys import public_key_fingerprint

    path = str(tmp_path / "enc")
    subprocess.run(["ssh-keygen", "-q", "-t", "rsa", "-b", "2048", "-m", "PEM", "-N", "hunter22", "-f", path],
                   check=True)
    with pytest.raises(TKError) as exc:
        public_key_fingerprint(path)  # non-interactive: no hanging prompt (Q14)
    assert str(exc.value).startswith("Unable to parse private key:")
    assert public_key_fingerprint(path, lambda: "hunter22") == load_private_key(path, "hunter22").fingerprint_md5()


def test_openssh_key_passphrase_never_on_argv(tmp_path, monkeypatch):
    """the passphrase of an encrypted OpenSSH key reaches ssh-keygen on
    stdin; ``ps`` (every local user) sees only the argv."""
    import subprocess

    from triton_kubernetes_amd.utils import sshkeys

    path = str(tmp_path / "enc-ed25519")
    subprocess.run(["ssh-keygen", "-q", "-t", "ed25519", "-N", "c0rrect horse", "-f", path], check=True)
    seen = []
    real = subprocess.run

    def spy(argv, *a, **kw):
        seen.append((list(argv), kw.get("input")))
        return real(argv, *a, **kw)

    monkeypatch.setattr(sshkeys.subprocess, "run", spy)
    key = load_private_key(path, "c0rrect horse")
    want = real(["ssh-keygen", "-l", "-E", "md5", "-f", path + ".pub"], capture_output=True, text=True).stdout.split()[1]
    assert "MD5:" + key.fingerprint_md5() == want
    keygen = [argv for argv, _ in seen if argv[0] == "ssh-keygen"]
    assert keygen and not any("c0rrect horse" in " ".join(argv) for argv, _ in seen)
    assert any(inp and b"c0rrect horse" in inp for _, inp in seen)
    with pytest.raises(sshkeys.KeyParseError, match="incorrect passphrase"):
        load_private_key(path, "wrong")


def test_manta_create_then_destroy_manager_removes_every_object(manta, tmp_path):
    """BASELINE config #4 teardown: status.json, backups and the lock are deleted before the
    directory (reference backend/manta/backend.go:160-194); Manta refuses a non-empty one."""
    from triton_kubernetes_amd import workflows as wf
    from triton_kubernetes_amd.rancher.fake import FakeRancher
    from helpers import make_ctx

    fake, key_path, key = manta
    be = MantaBackend("acct", key_path, key.fingerprint_md5(), "https://triton", fake.url)
    pw = "tk-admin-pw-0123"
    with FakeRancher.for_manager("mgr", pw) as rancher:
        wf.new_manager(make_ctx({"backend_provider": "manta", "executor": "direct",
                                 "manager_cloud_provider": "baremetal", "name": "mgr",
                                 "rancher_admin_password": pw, "rancher_bootstrap_password": rancher.bootstrap_password, "host": "rancher+" + rancher.url,
                                 "ssh_user": "u", "bastion_host": "", "key_path": "k"}), be)
    be.write_blob("mgr", "backups.json", b'["b1"]')
    be.write_blob("mgr", "backup-b1.json", b"{}")
    names = {p.rsplit("/", 1)[1] for p in fake.objects if "/triton-kubernetes/mgr/" in p}
    assert {"main.tf.json", "terraform.tfstate", "status.json", "backups.json", "backup-b1.json"} <= names
    wf.delete_manager(make_ctx({"cluster_manager": "mgr", "executor": "direct"}), be)
    assert be.states() == []
    assert not any("/triton-kubernetes/mgr" in p for p in list(fake.objects) + list(fake.dirs))
    be.delete_state("mgr")  # idempotent on a missing manager


def test_manta_conditional_put_semantics(manta):
    fake, key_path, key = manta
    client = MantaClient(fake.url, HTTPSignatureSigner("acct", key))
    client.put_directory("/stor/x")
    e1 = client.put_object("/stor/x/o", b"1", if_none_match="*")
    assert e1 and client.put_object("/stor/x/o", b"2", if_none_match="*") is None  # exists
    assert client.put_object("/stor/x/o", b"3", if_match="stale") is None
    e2 = client.put_object("/stor/x/o", b"4", if_match=e1)
    assert e2 and e2 != e1 and client.get_object_etag("/stor/x/o") == (b"4", e2)
    assert client.delete("/stor/x/o", if_match=e1) is False  # stale etag: not deleted
    assert client.delete("/stor/x/o", if_match=e2) is True and client.get_object("/stor/x/o") is None
    with pytest.raises(TKError, match="DirectoryNotEmpty"):
        client.put_object("/stor/x/p", b"")
        client.delete("/stor/x")


def test_manta_lock_is_mutually_exclusive_under_contention(manta):
    import threading

    fake, key_path, key = manta
    be = MantaBackend("acct", key_path, key.fingerprint_md5(), "https://triton", fake.url)
    holders, max_holders, order = [0], [0], []
    mu = threading.Lock()
    start = threading.Barrier(6)

    def worker(i):
        start.wait()
        with be.lock("mgr", timeout=60, poll=0.01):
            with mu:
                holders[0] += 1
                max_holders[0] = max(max_holders[0], holders[0])
                order.append(i)
            time.sleep(0.02)
            with mu:
                holders[0] -= 1

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert max_holders[0] == 1 and sorted(order) == list(range(6))
    assert "/acct/stor/triton-kubernetes/mgr/.lock" not in fake.objects


def test_manta_expired_lock_taken_over_by_exactly_one(manta):
    import threading

    fake, key_path, key = manta
    be = MantaBackend("acct", key_path, key.fingerprint_md5(), "https://triton", fake.url)
    be.client.put_directory("/stor/triton-kubernetes/mgr")
    be.client.put_object("/stor/triton-kubernetes/mgr/.lock", json.dumps({"token": "dead", "expires": 0}).encode())
    winners, losers = [], []
    start = threading.Barrier(4)
    release = threading.Event()

    def worker(i):
        start.wait()
        try:
            with be.lock("mgr", timeout=1.0, poll=0.01):
                winners.append(i)
                release.wait(30)
        except Exception:  # noqa: BLE001 - the losers time out while the winner holds it
            losers.append(i)

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    for t in threads:
        t.start()
    # the winner holds the lock until every other thread has given up (on a loaded machine a
    # loser's last attempt can still be in flight well after its timeout)
    deadline = time.monotonic() + 30
    while len(losers) < 3 and time.monotonic() < deadline:
        time.sleep(0.02)
    release.set()
    for t in threads:
        t.join()
    assert len(winners) == 1 and len(losers) == 3


@pytest.mark.parametrize("held", [b"[1, 2]", b"not json", b'{"expires": "soon"}', b'"x"'])
def test_manta_unreadable_lock_object_is_stale(manta, held):
    """A lock object this CLI did not write (corrupt, another format) is taken over, not a
    traceback."""
    fake, key_path, key = manta
    be = MantaBackend("acct", key_path, key.fingerprint_md5(), "https://triton", fake.url)
    be.client.put_directory("/stor/triton-kubernetes/mgr")
    be.client.put_object("/stor/triton-kubernetes/mgr/.lock", held)
    with be.lock("mgr", timeout=5.0, poll=0.01):
        pass


def test_a_reply_that_is_not_json_is_an_error_with_its_first_bytes():
    from triton_kubernetes_amd.cloud.http import Response
    from triton_kubernetes_amd.errors import TKError

    with pytest.raises(TKError, match="expected a JSON response \\(HTTP 200\\), got: b'<html>"):
        Response(200, {}, b"<html>proxy error</html>", 0.0).json()
    assert Response(204, {}, b"", 0.0).json() is None
