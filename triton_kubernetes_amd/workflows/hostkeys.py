"""``forget host-key``: drop a machine's pinned SSH host key (``parallel/hostkeys.py``).

A reinstalled machine presents a new host key, which every SSH path refuses (that is the
point of pinning).  Once the operator has checked the new key out of band, this removes
the old entry from the cluster manager's ``known_hosts`` blob; the next contact pins the
new key.
"""

from ..backend.base import Backend
from ..config.context import Context, not_blank
from ..errors import ConfigError
from ..parallel.hostkeys import HostKeys
from .create import NO_MANAGERS
from .select import select_manager


def forget_host_key(ctx: Context, backend: Backend) -> int:
    managers = backend.states()
    if not managers:
        raise ConfigError(NO_MANAGERS)
    manager = select_manager(ctx, managers)
    host = ctx.resolve("host", "Host whose pinned SSH key to forget", validate=not_blank("host cannot be blank"))
    with HostKeys(backend, manager) as keys:
        n = keys.forget(host)
    ctx.echo(f"Forgot {n} pinned SSH host key(s) of {host} for cluster manager \"{manager}\"."
             if n else f"No SSH host key of {host} is pinned for cluster manager \"{manager}\".")
    return n


__all__ = ["forget_host_key"]
