"""``triton-kubernetes`` command line (reference ``cmd/*.go``).

    triton-kubernetes [--config FILE] [--non-interactive] create  manager|cluster|node
    triton-kubernetes [--config FILE] [--non-interactive] destroy manager|cluster|node
    triton-kubernetes [--config FILE] [--non-interactive] get     manager|cluster
    triton-kubernetes version

Additions: ``get nodes`` (the cluster's nodes with their MI355X GPU state),
``wait cluster`` (the readiness waiter on an existing cluster),
``credentials node`` (a node agent's TLS certificate, token and image allow-list),
``health cluster`` (GPU RAS health of the MI355X nodes; optional taint fencing),
``backup cluster`` / ``restore cluster`` (namespace backup to the state backend
or S3 — advertised by the reference README, never implemented there),
``gpu …`` (the native MI355X probes), ``agent`` (the node agent) and
``image`` (machine-image templates -> Packer JSON, the reference's
``packer/packer-config``).

Exit codes follow the reference: argument errors exit 255 (``os.Exit(-1)``),
workflow errors print the message and exit 1.  The dead ``-t/--toggle`` scaffold
flag (``cmd/root.go:44``) is not reproduced.
"""

import argparse
import os
import sys
from typing import List, Optional, Sequence, TextIO

from .. import __version__
from ..errors import Canceled, TKError

# Injected at build time (the reference's -ldflags -X cmd.cliVersion).
CLI_VERSION = ""
try:  # pragma: no cover - generated file
    from .._build_info import CLI_VERSION as _BUILD_VERSION  # type: ignore

    CLI_VERSION = _BUILD_VERSION
except ImportError:
    pass

VALID = {
    "create": ["manager", "cluster", "node"],
    "destroy": ["manager", "cluster", "node"],
    "get": ["manager", "cluster", "nodes", "scrape-config", "alert-rules"],
    "wait": ["cluster"],
    "backup": ["cluster"],
    "restore": ["cluster"],
    "userdata": ["node"],
    "migrate": ["manager"],
    "credentials": ["node"],
    "health": ["cluster"],
    "drain": ["node"],
    "upgrade": ["cluster"],
    "cordon": ["node"],
    "uncordon": ["node"],
    "forget": ["host-key"],
}
# the reference's error text has the "destory" typo (cmd/destroy.go:22,31)
_ARG_NAME = {"create": "create", "destroy": "destory", "get": "get", "wait": "wait", "backup": "backup",
             "restore": "restore", "userdata": "userdata", "migrate": "migrate", "credentials": "credentials", "health": "health",
             "drain": "drain", "cordon": "cordon", "uncordon": "uncordon", "upgrade": "upgrade",
             "forget": "forget"}


class ArgError(Exception):
    pass


def version_text(cli_version: Optional[str] = None) -> str:
    v = CLI_VERSION if cli_version is None else cli_version
    prefix = ""
    if not v:
        prefix = "no version set for this build... "
        v = "local"
    return f"{prefix}triton-kubernetes v{__version__} ({v})\n"


def _check_args(cmd: str, args: List[str]) -> str:
    if len(args) != 1:
        raise ArgError(f'"triton-kubernetes {_ARG_NAME[cmd]}" requires one argument')
    if args[0] not in VALID[cmd]:
        raise ArgError(f'invalid argument "{args[0]}" for "triton-kubernetes {_ARG_NAME[cmd]}"')
    return args[0]


def build_parser() -> argparse.ArgumentParser:
    common = argparse.ArgumentParser(add_help=False)
    common.add_argument("--config", default=argparse.SUPPRESS,
                        help="config file (default is $HOME/.triton-kubernetes.yaml)")
    common.add_argument("--non-interactive", action="store_true", default=argparse.SUPPRESS,
                        help="Prevent interactive prompts")
    root = argparse.ArgumentParser(
        prog="triton-kubernetes", parents=[common],
        description="A tool to deploy Kubernetes to multiple cloud providers and to bare-metal 8xMI355X nodes.")
    sub = root.add_subparsers(dest="command")
    for cmd, help_ in (("create", "Create cluster managers, kubernetes clusters or individual kubernetes cluster "
                                  "nodes."),
                       ("destroy", "Destroy cluster managers, kubernetes clusters or individual kubernetes "
                                   "cluster nodes."),
                       ("get", "Display resource information"),
                       ("wait", "Wait until a cluster is kubectl-ready (and GPU-ready) and report timings"),
                       ("backup", "Back up a cluster's namespaces to the state backend (local/manta) or S3"),
                       ("restore", "Restore a cluster's namespaces from a backup"),
                       ("userdata", "Print cloud-init user-data that bootstraps a node (PXE/MAAS delivery)"),
                       ("migrate", "Point a cluster manager's document (e.g. one written by the reference's "
                                   "Terraform 0.11 modules) at this framework's modules"),
                       ("credentials", "Issue a node agent's TLS certificate, token and image allow-list "
                                       "(signed by the cluster manager's agent CA)"),
                       ("health", "Re-read the GPU health (ECC, retired pages) of a cluster's MI355X nodes and, "
                                  "with health_taint, fence unhealthy ones"),
                       ("drain", "Cordon a node and evict its pods (disruption budgets honoured)"),
                       ("upgrade", "Upgrade a cluster's Kubernetes release (one minor at a time) and wait for it"),
                       ("cordon", "Mark a node unschedulable"),
                       ("uncordon", "Mark a node schedulable again"),
                       ("forget", "Forget a reinstalled machine's pinned SSH host key (host setting)")):
        p = sub.add_parser(cmd, parents=[common], help=help_)
        p.add_argument("args", nargs="*")
    sub.add_parser("version", parents=[common], help="Print the version number of triton-kubernetes")
    g = sub.add_parser("gpu", help="MI355X node probes (burnin, topology, labels, health, metrics, rccl-local, rccl-slim, links, "
                                      "hbm, mfma, gemm)")
    g.add_argument("gpu_args", nargs=argparse.REMAINDER)
    a = sub.add_parser("agent", help="Run the node agent (tk-node-agent)")
    a.add_argument("agent_args", nargs=argparse.REMAINDER)
    i = sub.add_parser("image", help="Render a machine-image template to Packer JSON (packer-config)")
    i.add_argument("image_args", nargs=argparse.REMAINDER)
    return root


def make_context(ns: argparse.Namespace, out: TextIO, env=None):
    from ..config import Context, Settings

    settings = Settings.discover(getattr(ns, "config", None), env=env)
    if getattr(ns, "non_interactive", False):
        settings.set_flag("non-interactive", True)
    ctx = Context(settings=settings, out=out)
    if settings.non_interactive:
        ctx.echo("Running in non interactive mode")
    if settings.config_file_used:
        ctx.echo(f"Using config file: {settings.config_file_used}")
    return ctx


def run(argv: Sequence[str], out: Optional[TextIO] = None, ctx=None) -> int:
    out = out or sys.stdout
    parser = build_parser()
    ns = parser.parse_args(list(argv))
    if ns.command is None:
        parser.print_help(out)
        return 0
    if ns.command == "version":
        out.write(version_text())
        return 0
    if ns.command == "gpu":
        from ..ops.cli import main as gpu_main

        return gpu_main(ns.gpu_args)
    if ns.command == "agent":
        from ..node.agent import main as agent_main

        return agent_main(ns.agent_args)
    if ns.command == "image":
        from ..images.packer import main as image_main

        return image_main(ns.image_args)
    try:
        what = _check_args(ns.command, ns.args)
    except ArgError as exc:
        out.write(f"{exc}\n")
        return 255
    try:
        if ctx is None:
            ctx = make_context(ns, out)
        from ..backend import prompt_for_backend

        backend = prompt_for_backend(ctx)
        return dispatch(ctx, backend, ns.command, what)
    except Canceled:
        return 0
    except TKError as exc:
        out.write(f"{exc}\n")
        return 1
    except KeyboardInterrupt:
        out.write("^C\n")
        return 1


def dispatch(ctx, backend, command: str, what: str) -> int:
    from .. import workflows as wf

    ctx.echo(f"{command} {what} called")
    if command == "create":
        {"manager": wf.new_manager, "cluster": wf.new_cluster, "node": wf.new_node}[what](ctx, backend)
    elif command == "destroy":
        {"manager": wf.delete_manager, "cluster": wf.delete_cluster, "node": wf.delete_node}[what](ctx, backend)
    elif command == "get":
        if what == "nodes":
            from ..workflows.get import get_nodes

            get_nodes(ctx, backend)
        elif what == "scrape-config":
            from ..workflows.scrape import scrape_config

            scrape_config(ctx, backend)
        elif what == "alert-rules":
            from ..workflows.scrape import alert_rules

            alert_rules(ctx, backend)
        else:
            {"manager": wf.get_manager, "cluster": wf.get_cluster}[what](ctx, backend)
    elif command == "backup":
        from ..workflows.backup import backup_cluster

        backup_cluster(ctx, backend)
    elif command == "restore":
        from ..workflows.backup import restore_cluster

        restore_cluster(ctx, backend)
    elif command == "userdata":
        from ..workflows.userdata import node_userdata

        node_userdata(ctx, backend)
    elif command == "migrate":
        from ..workflows.migrate import migrate_manager

        migrate_manager(ctx, backend)
    elif command == "credentials":
        from ..workflows.credentials import node_credentials

        node_credentials(ctx, backend)
    elif command == "health":
        from ..workflows.health import cluster_health

        cluster_health(ctx, backend)
    elif command == "upgrade":
        from ..workflows.upgrade import upgrade_cluster

        upgrade_cluster(ctx, backend)
    elif command == "drain":
        from ..workflows.drain import drain_command

        drain_command(ctx, backend)
    elif command in ("cordon", "uncordon"):
        from ..workflows.drain import cordon_command

        cordon_command(ctx, backend, command == "cordon")
    elif command == "forget":
        from ..workflows.hostkeys import forget_host_key

        forget_host_key(ctx, backend)
    elif command == "wait":
        from ..readiness.waiter import wait_after_create
        from ..workflows.select import select_cluster, select_manager

        managers = backend.states()
        if not managers:
            raise TKError("No cluster managers.")
        state = backend.state(select_manager(ctx, managers))
        _, key = select_cluster(ctx, state.clusters(), "Cluster to wait for")
        wait_after_create(ctx, backend, state, key)
    return 0


def main(argv: Optional[Sequence[str]] = None) -> int:
    code = run(sys.argv[1:] if argv is None else argv)
    trace = os.environ.get("TK_TRACE")
    if trace:
        from ..utils.trace import TRACER

        TRACER.dump_chrome(trace)
    return code


if __name__ == "__main__":
    sys.exit(main())
