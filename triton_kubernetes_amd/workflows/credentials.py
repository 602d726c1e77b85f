"""``credentials node``: a node agent's TLS certificate, token and image allow-list.

The cluster manager's agent PKI (``node/security.py``) signs a certificate for the
node's address and derives the node's own token; the allow-list is the manager's agent
image (``rancher_agent_image`` of the manager document, else the pinned default) unless
``agent_images`` names others (digest pins: ``repo@sha256:...``); the servers an RKE2
node may take its ``system-agent-install.sh`` from are the manager's ``rancher_url``
(from its Terraform state) unless ``agent_servers`` names them.  The files go to
``credentials_dir`` (default ``./agent-credentials-<address>``), to be installed as the
node's ``/etc/triton-kubernetes/agent/`` (the ``tk-node-agent`` unit reads them with
``--credentials``).

The node is enrolled for one Kubernetes distribution (``agent_distribution``, default
the pinned default, RKE2): a plan naming the other one is refused, so a token holder
cannot switch an RKE2 node to the RKE1 path (a privileged ``rancher-agent`` container).

Settings: ``cluster_manager``, ``agent_address`` (IP or DNS name the CLI reaches the
agent at), ``agent_images`` (list, optional), ``agent_servers`` (list, optional),
``agent_distribution`` (rke2 | rke1, optional), ``credentials_dir`` (optional).
"""

import os

from ..backend.base import Backend
from ..config.context import Context, not_blank
from ..errors import ConfigError
from ..node.security import load_pki, server_origin
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
    servers = ctx.settings.get("agent_servers") if ctx.is_set("agent_servers") else None
    if servers is None:
        from ..executor.base import outputs_from_tfstate

        try:
            url = outputs_from_tfstate(backend.read_tfstate(manager), MANAGER_KEY).get("rancher_url", "")
        except (NotImplementedError, ValueError):  # no state yet
            url = ""
        servers = [url] if url else []
    if isinstance(servers, str):
        servers = [u.strip() for u in servers.split(",") if u.strip()]
    bad = [u for u in servers if not server_origin(u)]
    if bad:
        raise ConfigError(f"agent_servers: {bad[0]!r} is not an http(s) URL")
    dist = (ctx.get_string("agent_distribution") if ctx.is_set("agent_distribution")
            else versions.DEFAULT_DISTRIBUTION).lower()
    if dist not in versions.DISTRIBUTIONS:
        raise ConfigError(f"agent_distribution must be one of {', '.join(versions.DISTRIBUTIONS)}, not {dist!r}")
    out = ctx.get_string("credentials_dir") if ctx.is_set("credentials_dir") else f"agent-credentials-{address}"
    creds = load_pki(backend, manager).issue(address, list(images), servers=list(servers), distributions=[dist])
    files = creds.write(os.path.abspath(os.path.expanduser(out)))
    ctx.echo(f"Agent credentials for {creds.address} (manager '{manager}') written to {os.path.dirname(files[0])}:")
    for f in files:
        ctx.echo(f"  {os.path.basename(f)}")
    if not servers:
        ctx.echo("note: no Rancher server in the allow-list (the manager has no rancher_url yet; set "
                 "agent_servers): this node cannot join RKE2 clusters.")
    ctx.echo("Install them as /etc/triton-kubernetes/agent/ on the node (mode 0600, root).")
    return os.path.dirname(files[0])


__all__ = ["node_credentials"]
