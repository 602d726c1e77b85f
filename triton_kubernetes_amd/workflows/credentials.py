"""``credentials node``: a node agent's TLS certificate, token and image allow-list.

The cluster manager's agent PKI (``node/security.py``) signs a certificate for the
node's address and derives the node's own token; the allow-list is the manager's agent
image (``rancher_agent_image`` of the manager document, else the pinned default) unless
``agent_images`` names others (digest pins: ``repo@sha256:...``).  The files go to
``credentials_dir`` (default ``./agent-credentials-<address>``), to be installed as the
node's ``/etc/triton-kubernetes/agent/`` (the ``tk-node-agent`` unit reads them with
``--credentials``).

Settings: ``cluster_manager``, ``agent_address`` (IP or DNS name the CLI reaches the
agent at), ``agent_images`` (list, optional), ``credentials_dir`` (optional).
"""

import os

from ..backend.base import Backend
from ..config.context import Context, not_blank
from ..errors import ConfigError
from ..node.security import load_pki
from ..state.document import MANAGER_KEY
from .. import versions
from .select import select_manager


def node_credentials(ctx: Context, backend: Backend) -> str:
    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    manager = select_manager(ctx, managers)
    address = ctx.resolve("agent_address", "Node agent address (IP or DNS name)",
                          validate=not_blank("agent_address cannot be blank"))
    images = ctx.settings.get("agent_images") if ctx.is_set("agent_images") else None
    if images is None:
        mgr = backend.state(manager).modules().get(MANAGER_KEY) or {}
        images = [mgr.get("rancher_agent_image") or versions.AGENT_IMAGE]
    if isinstance(images, str):
        images = [i.strip() for i in images.split(",") if i.strip()]
    if not images:
        raise ConfigError("agent_images must name at least one image")
    out = ctx.get_string("credentials_dir") if ctx.is_set("credentials_dir") else f"agent-credentials-{address}"
    creds = load_pki(backend, manager).issue(address, list(images))
    files = creds.write(os.path.abspath(os.path.expanduser(out)))
    ctx.echo(f"Agent credentials for {creds.address} (manager '{manager}') written to {os.path.dirname(files[0])}:")
    for f in files:
        ctx.echo(f"  {os.path.basename(f)}")
    ctx.echo("Install them as /etc/triton-kubernetes/agent/ on the node (mode 0600, root).")
    return os.path.dirname(files[0])


__all__ = ["node_credentials"]
