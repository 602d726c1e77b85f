"""An adopted Rancher server gets no function of the admin password.

``host: rancher+https://...`` adopts a server someone else started.  Its first-login password
is ``rancher_bootstrap_password`` (kept in the state backend, never in ``main.tf.json``), or
the server is already bootstrapped and takes the admin password.  The derivation earlier
versions of this framework used (sha256 of ``tk-bootstrap:<name>:<admin password>``, an
offline brute-force oracle for the admin password) is sent only behind
``rancher_legacy_bootstrap: true``.  The fake Rancher records every request body, so the
tests check what actually reached the server.
"""

import pytest

from triton_kubernetes_amd import versions
from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.rancher import bootstrap_secret
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.workflows import new_manager

from helpers import make_ctx

PW = "adopted-admin-pw-0123"


def _create(fake, backend, **extra):
    new_manager(make_ctx(dict({"executor": "direct"}, manager_cloud_provider="baremetal", name="mgr",
                              rancher_admin_password=PW, host="rancher+" + fake.url, ssh_user="u",
                              bastion_host="", key_path="k", **extra)), backend)


def _sent(fake, secret):
    return [b for b in fake.request_bodies if secret.encode() in b]


def test_legacy_server_without_opt_in_is_refused_and_never_sees_the_derivation(tmp_path):
    derived = versions.bootstrap_password("mgr", PW)
    with FakeRancher.for_manager("mgr", PW) as fake:  # started by round <= 4 of this framework
        backend = LocalBackend(str(tmp_path / "state"))
        with pytest.raises(TKError, match="rancher_bootstrap_password"):
            _create(fake, backend)
        assert _sent(fake, derived) == []
        assert _sent(fake, PW)  # the admin password was tried: an already-bootstrapped server


def test_legacy_derivation_only_behind_the_opt_in(tmp_path):
    derived = versions.bootstrap_password("mgr", PW)
    with FakeRancher.for_manager("mgr", PW) as fake:
        backend = LocalBackend(str(tmp_path / "state"))
        _create(fake, backend, rancher_legacy_bootstrap=True)
        assert _sent(fake, derived)  # the opted-in login (and the password change)
        assert backend.state("mgr").module("cluster-manager")["host"] == "rancher+" + fake.url


def test_given_bootstrap_password_is_used_and_kept_out_of_the_state_document(tmp_path):
    with FakeRancher(bootstrap_password="their-b00tstrap-secret") as fake:
        backend = LocalBackend(str(tmp_path / "state"))
        _create(fake, backend, rancher_bootstrap_password="their-b00tstrap-secret")
        assert _sent(fake, versions.bootstrap_password("mgr", PW)) == []
        holding = [str(f.relative_to(tmp_path)) for f in (tmp_path / "state").rglob("*")
                   if f.is_file() and b"their-b00tstrap-secret" in f.read_bytes()]
        assert holding and all(h.endswith(bootstrap_secret.BLOB) for h in holding), holding  # not main.tf.json
        assert bootstrap_secret.load(backend, "mgr") == "their-b00tstrap-secret"
        assert not bootstrap_secret.legacy_allowed(backend, "mgr")


def test_an_already_bootstrapped_server_takes_the_admin_password(tmp_path):
    """A server whose admin password is already the one given (bootstrapped by hand, or by
    another manager document): no bootstrap password needed, and nothing derived sent."""
    with FakeRancher(bootstrap_password=PW) as fake:
        backend = LocalBackend(str(tmp_path / "state"))
        _create(fake, backend)
        assert _sent(fake, versions.bootstrap_password("mgr", PW)) == []
        assert backend.state("mgr").module("cluster-manager")
