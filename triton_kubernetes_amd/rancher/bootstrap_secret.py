"""The Rancher server's first-login password, random and kept in the state backend.

Rancher >= 2.6 has no admin/admin: a server starts with ``CATTLE_BOOTSTRAP_PASSWORD`` and
the first login uses it, after which :meth:`~.client.RancherClient.bootstrap` changes the
admin password (reference: admin/admin, ``terraform/modules/files/setup_rancher.sh.tpl:13-38``).

Round 4 derived that password as an unsalted sha256 of the admin password and handed it
to ``docker run -e`` on the command line: visible in ``ps``, kept by ``docker inspect`` for
the container's life, and an offline brute-force oracle for the admin password.  Now:

* it is random (``secrets.token_urlsafe``: 192 bits) and no function of anything, generated
  once per cluster manager and kept in the manager's state backend (blob
  ``rancher-bootstrap.json``, written 0600 by the local backend), so a re-run of the install
  or of the bootstrap finds it;
* the server gets it through ``docker run --env-file`` from a 0600 file that is removed as
  soon as the container has started -- never on a command line;
* the Terraform manager modules take it as ``rancher_bootstrap_password``, rendered by the
  executor from the same blob (a sensitive root variable).

An adopted server (``host: rancher+https://...``) was started by someone else.  Its
first-login password is given as ``rancher_bootstrap_password`` (kept in this same blob,
never in ``main.tf.json``), or the server is already bootstrapped and takes the admin
password.  Nothing derived from the admin password goes to it unless the operator says the
server is one an earlier version of this framework started (``rancher_legacy_bootstrap:
true``, :func:`legacy_password`): that derivation is an offline brute-force oracle for the
admin password, and an adopted server is not ours to hand it to.
"""

import json
import secrets
from typing import Any, Optional

BLOB = "rancher-bootstrap.json"


def load(backend: Any, manager: str) -> Optional[str]:
    try:
        raw = backend.read_blob(manager, BLOB)
    except NotImplementedError:
        return None
    if not raw:
        return None
    return str(json.loads(raw).get("password", "")) or None


def ensure(backend: Any, manager: str) -> str:
    """The manager's bootstrap password, created (and stored) on first use."""
    pw = load(backend, manager)
    if pw:
        return pw
    pw = secrets.token_urlsafe(24)
    try:
        backend.write_blob(manager, BLOB, json.dumps({"password": pw}).encode())
    except NotImplementedError:
        pass
    return pw


def save_adopted(backend: Any, manager: str, password: str = "", legacy: bool = False) -> None:
    """An adopted server's first-login password (``rancher_bootstrap_password``; may be
    empty: an already-bootstrapped server) and whether the legacy derivation may be tried."""
    try:
        backend.write_blob(manager, BLOB, json.dumps({"password": password, "adopted": True,
                                                      "legacy": bool(legacy)}).encode())
    except NotImplementedError:
        pass


def legacy_allowed(backend: Any, manager: str) -> bool:
    """The operator opted in to :func:`legacy_password` for this adopted server."""
    try:
        raw = backend.read_blob(manager, BLOB)
    except NotImplementedError:
        return False
    return bool(raw) and bool(json.loads(raw).get("legacy"))


def legacy_password(manager_name: str, admin_password: str) -> str:
    """What servers started by round <= 4 of this framework (and the test fake's
    ``for_manager``) hold: a login attempt against an adopted server, never sent to a host."""
    from ..versions import bootstrap_password

    return bootstrap_password(manager_name, admin_password)


__all__ = ["BLOB", "ensure", "legacy_allowed", "legacy_password", "load", "save_adopted"]
