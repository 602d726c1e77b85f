"""Executor selection from settings.

==========================  ================================================================
``executor``                ``terraform`` | ``direct`` | ``auto`` (default)
``terraform_binary``        path/name of the Terraform CLI (default ``terraform``)
``terraform_parallelism``   ``-parallelism=N`` for apply/destroy (default: Terraform's 10)
``direct_parallelism``      max modules in flight in the DirectExecutor (default 64)
``agent_token``             development only: one shared token for every ``agent+`` host
                            (default: per-node tokens and TLS from the manager's agent
                            PKI, ``node/security.py``)
``rancher_bootstrap``       ``operator`` (default) | ``remote``
``node_cleanup``            take destroyed bare-metal hosts out of their cluster (uninstall the
                            agent and RKE2/RKE1, node/cleanup.py; default true); a host
                            module's own ``node_cleanup`` can turn it off for that host
``host_retries``            re-run a failed host bootstrap this many times (default 0)
``rancher_ca_file``         PEM CA bundle of the Rancher server: pinned for the manager (an
                            adopted server, a custom CA, a deliberate re-pin after a CA
                            rotation); default: read on the manager host at create manager
                            (rancher/trust.py)
``host_retry_backoff``      first retry delay in seconds, doubling per attempt (default 2)
==========================  ================================================================

``auto`` picks Terraform when the binary is on ``PATH``; otherwise the
DirectExecutor when it implements every module of the document.
"""

from typing import Optional

from ..config.context import Context
from ..errors import ConfigError
from ..state import State
from .base import Executor
from .shell import which


def build_executor(ctx: Context, state: Optional[State] = None) -> Executor:
    s = ctx.settings
    kind = (s.get_string("executor") or "auto").lower()
    tf_bin = s.get_string("terraform_binary") or "terraform"
    if kind == "auto":
        if which(tf_bin):
            kind = "terraform"
        else:
            from .direct import DirectExecutor

            kind = "direct" if state is not None and DirectExecutor.supports(state) else "terraform"
    if kind == "terraform":
        from .terraform import TerraformExecutor

        par = s.get_int("terraform_parallelism") if s.is_set("terraform_parallelism") else None
        return TerraformExecutor(binary=tf_bin, parallelism=par, ca_file=s.get_string("rancher_ca_file") or "")
    if kind == "direct":
        from ..parallel.transport import SSHTransport, TransportRouter
        from .direct import DirectExecutor

        from ..readiness.waiter import agent_transport_for

        transport = ctx.extras.get("transport") or TransportRouter(
            ssh=SSHTransport(), agent=agent_transport_for(ctx, state.name if state is not None else ""))
        par = s.get_int("direct_parallelism") if s.is_set("direct_parallelism") else 64
        return DirectExecutor(transport=transport, parallelism=par,
                              rancher_bootstrap=s.get_string("rancher_bootstrap") or "operator",
                              node_cleanup=s.get_bool("node_cleanup") if s.is_set("node_cleanup") else True,
                              host_retries=s.get_int("host_retries") if s.is_set("host_retries") else 0,
                              retry_backoff=s.get_float("host_retry_backoff", 2.0),
                              rancher_factory=ctx.extras.get("rancher_factory"),
                              ca_file=s.get_string("rancher_ca_file") or "")
    raise ConfigError(f"executor must be one of terraform, direct, auto. Found '{kind}'.")
