"""Shared config builders for the provider "model families".

Base module configs (field order = the reference's Go struct order, so the
JSON documents match):

* manager — ``create/manager.go:16-27`` + ``getBaseManagerTerraformConfig`` (l.156-300)
* cluster — ``create/cluster.go:24-43`` + ``getBaseClusterTerraformConfig`` (l.292-516)
* node    — ``create/node.go:19-41``    + ``getBaseNodeTerraformConfig`` (l.197-347)

Every builder returns a plain ``dict``; ``omitempty`` fields are dropped when
empty exactly as Go's encoder would.
"""

import ipaddress
import re
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

from ..config.context import Context, not_blank
from ..errors import ConfigError
from ..state import MANAGER_KEY, State
from ..terraform.catalog import module_source, packaged_source
from ..versions import (DISTRIBUTIONS, PASSWORD_MIN_LENGTH, RKE2_CNIS, distribution_of, normalize_k8s_version,
                        releases, resolve_distribution)

# The reference defaults to its own GitHub repo (create/cluster.go:20-21), which is
# where its modules live.  This CLI's modules ship inside the package, so the default
# is the symbolic tk:: source of that tree (resolved to a directory only when an
# executor runs the document; a zipapp extracts it to a cache first);
# SOURCE_URL / SOURCE_REF still select a git or registry copy.
DEFAULT_SOURCE_URL = ""  # "" = the packaged module tree (catalog.packaged_source())
DEFAULT_SOURCE_REF = "master"

DNS1123_RE = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$")
DNS1123_MESSAGE = ("A DNS-1123 subdomain must consist of lower case alphanumeric characters, '-' or '.', "
                   "and must start and end with an alphanumeric character")

# interactive choices: display name -> value (create/cluster.go:349-356 offers the
# releases of its pinned Rancher; these are the pinned Rancher v2.10.3's, versions.py).
# The reference offered calico / flannel (RKE1); RKE2 ships canal (its default), calico,
# cilium and flannel.
NETWORK_PROVIDERS = {"rke2": list(RKE2_CNIS), "rke1": ["calico", "flannel", "canal", "weave"]}
DISTRIBUTION_CHOICES = ["RKE2 (rancher-system-agent, containerd)",
                        "RKE1 (end-of-life; Docker + rancher-agent, reference-era clusters)"]
HOST_LABELS = ["worker", "etcd", "control"]
_ATOI_RE = re.compile(r"^[+-]?[0-9]+$")


def omit_empty(cfg: Dict, keys: Sequence[str]) -> Dict:
    for k in keys:
        if k in cfg and cfg[k] in ("", None, [], {}):
            del cfg[k]
    return cfg


def source_for(ctx: Context, module_path: str) -> str:
    """The persisted ``source`` of a module block.

    * default: the location-free ``tk::<module_path>?ref=v<version>`` of the modules this
      CLI ships (``terraform/catalog.py``), resolved to this install's directory only in
      the document an executor runs — so a shared (Manta) document applies from any
      operator's machine, as the reference's GitHub sources do;
    * ``source_url`` set: ``<url>//<module_path>?ref=<source_ref>`` (``create/manager.go:160-171``),
      or ``<dir>/<module_path>`` when the URL is a local directory (a deliberate,
      machine-local choice)."""
    url = ctx.get_string("source_url") if ctx.is_set("source_url") else DEFAULT_SOURCE_URL
    if not url:
        return packaged_source(module_path)
    ref = ctx.get_string("source_ref") if ctx.is_set("source_ref") else DEFAULT_SOURCE_REF
    return module_source(url, module_path, ref)


# --- validators -------------------------------------------------------------------
def parse_cidr(value: str) -> ipaddress.IPv4Network:
    try:
        return ipaddress.ip_network(value, strict=False)  # type: ignore[return-value]
    except ValueError as exc:
        raise ConfigError(f"invalid CIDR address: {value}") from exc


def validate_vpc_cidr(value: str) -> Optional[str]:
    try:
        net = parse_cidr(value)
    except ConfigError as exc:
        return str(exc)
    if net.prefixlen < 16:
        return f"Prefix length must be 16 or greater. Found {net.prefixlen}."
    return None


def subnet_validator(vpc_cidr: str):
    vpc = parse_cidr(vpc_cidr)

    def _check(value: str) -> Optional[str]:
        try:
            iface = ipaddress.ip_interface(value)
        except ValueError:
            return f"invalid CIDR address: {value}"
        if iface.ip not in vpc or iface.network.prefixlen < vpc.prefixlen:
            return f"Subnet CIDR '{value}' is not within bounds of VPC CIDR '{vpc_cidr}'."
        return None

    return _check


def positive_int(value: str) -> Optional[str]:
    try:
        n = int(value)
    except ValueError:
        return "Invalid number"
    if n <= 0:
        return "Number must be greater than 0"
    return None


# --- base manager -------------------------------------------------------------------
def _registry_creds(ctx: Context, cfg: Dict, prefix_key: str, user_key: str, pass_key: str,
                    user_label: str, pass_label: str, out_user: str, out_pass: str) -> None:
    if cfg.get(prefix_key):
        cfg[out_user] = ctx.resolve(user_key, user_label)
        cfg[out_pass] = ctx.resolve(pass_key, pass_label, mask=True)


def base_manager_config(ctx: Context, module_path: str, name: str) -> Dict:
    cfg: Dict = {
        "source": source_for(ctx, module_path),
        "name": name,
        "rancher_admin_password": "",
        "rancher_server_image": "",
        "rancher_agent_image": "",
        "rancher_registry": "",
        "rancher_registry_username": "",
        "rancher_registry_password": "",
    }
    cfg["rancher_registry"] = ctx.resolve("private_registry", "Private Registry", required=False,
                                          none_sentinel="None")
    _registry_creds(ctx, cfg, "rancher_registry", "private_registry_username", "private_registry_password",
                    "Private Registry Username", "Private Registry Password",
                    "rancher_registry_username", "rancher_registry_password")
    cfg["rancher_server_image"] = ctx.resolve("rancher_server_image", "Rancher Server Image", required=False,
                                              none_sentinel="Default")
    cfg["rancher_agent_image"] = ctx.resolve("rancher_agent_image", "Rancher Agent Image", required=False,
                                             none_sentinel="Default")
    cfg["rancher_admin_password"] = ctx.resolve(
        "rancher_admin_password", "Set UI Admin Password", mask=True,
        validate=not_blank("password cannot be blank"),
        missing_message="UI Admin Password must be specified")
    if not cfg["rancher_admin_password"]:
        raise ConfigError("Invalid UI Admin password")
    if len(cfg["rancher_admin_password"]) < PASSWORD_MIN_LENGTH:
        # Rancher >= 2.6 rejects the password change with a shorter one (password-min-length)
        raise ConfigError(f"UI Admin password must be at least {PASSWORD_MIN_LENGTH} characters")
    return omit_empty(cfg, ["rancher_admin_password", "rancher_server_image", "rancher_agent_image",
                            "rancher_registry", "rancher_registry_username", "rancher_registry_password"])


# --- base cluster -------------------------------------------------------------------
def base_cluster_config(ctx: Context, module_path: str) -> Dict:
    cfg: Dict = {
        "source": source_for(ctx, module_path),
        "name": "",
        "rancher_api_url": f"${{module.{MANAGER_KEY}.rancher_url}}",
        "rancher_access_key": f"${{module.{MANAGER_KEY}.rancher_access_key}}",
        "rancher_secret_key": f"${{module.{MANAGER_KEY}.rancher_secret_key}}",
        "k8s_distribution": "",
        "k8s_version": "",
        "k8s_network_provider": "",
        "rancher_registry": "",
        "rancher_registry_username": "",
        "rancher_registry_password": "",
        "k8s_registry": "",
        "k8s_registry_username": "",
        "k8s_registry_password": "",
    }
    name = ctx.resolve("name", "Cluster Name",
                       validate=lambda v: None if DNS1123_RE.fullmatch(v) else DNS1123_MESSAGE)
    if not name or not DNS1123_RE.fullmatch(name):
        raise ConfigError("Invalid Cluster Name")
    cfg["name"] = name
    dist = cluster_distribution(ctx)
    cfg["k8s_distribution"] = dist
    pinned = releases(dist)
    cfg["k8s_version"] = ctx.resolve_choice("k8s_version", "Kubernetes Version",
                                            [d for d, _ in pinned], values=[v for _, v in pinned])
    try:
        cfg["k8s_version"] = normalize_k8s_version(cfg["k8s_version"], dist)
    except ValueError as exc:
        raise ConfigError(str(exc)) from None
    cnis = NETWORK_PROVIDERS[dist]
    cfg["k8s_network_provider"] = ctx.resolve_choice("k8s_network_provider", "Kubernetes Network Provider", cnis)
    if cfg["k8s_network_provider"] not in cnis:
        raise ConfigError(f"k8s_network_provider '{cfg['k8s_network_provider']}' is not a {dist.upper()} network "
                          f"provider; choose one of: {', '.join(cnis)}")
    cfg["rancher_registry"] = ctx.resolve("private_registry", "Private Registry", required=False,
                                          none_sentinel="None")
    _registry_creds(ctx, cfg, "rancher_registry", "private_registry_username", "private_registry_password",
                    "Private Registry Username", "Private Registry Password",
                    "rancher_registry_username", "rancher_registry_password")
    cfg["k8s_registry"] = ctx.resolve("k8s_registry", "k8s Registry", required=False, none_sentinel="None")
    _registry_creds(ctx, cfg, "k8s_registry", "k8s_registry_username", "k8s_registry_password",
                    "k8s Registry Username", "k8s Registry Password",
                    "k8s_registry_username", "k8s_registry_password")
    return omit_empty(cfg, ["k8s_version", "k8s_network_provider", "rancher_registry",
                            "rancher_registry_username", "rancher_registry_password", "k8s_registry",
                            "k8s_registry_username", "k8s_registry_password"])


def cluster_distribution(ctx: Context) -> str:
    """``k8s_distribution`` of a new cluster: the setting, else the one its
    ``k8s_version`` names (``...+rke2rN`` / ``...-rancherN-N``), else a prompt
    (interactive) or RKE2 (silent)."""
    explicit = ctx.get_string("k8s_distribution") if ctx.is_set("k8s_distribution") else ""
    version = ctx.get_string("k8s_version") if ctx.is_set("k8s_version") else ""
    if not explicit and not distribution_of(version) and not ctx.non_interactive:
        explicit = ctx.resolve_choice("k8s_distribution", "Kubernetes Distribution", DISTRIBUTION_CHOICES,
                                      values=list(DISTRIBUTIONS))
    try:
        return resolve_distribution(version, explicit)
    except ValueError as exc:
        raise ConfigError(str(exc)) from None


def node_distribution(state: State, cluster: str) -> str:
    """The distribution a cluster's nodes join with, read from its module block: its
    ``k8s_distribution``, else the one its ``k8s_version`` names, else the module
    default (``migrate manager`` writes ``rke1`` into reference-era blocks)."""
    block = state.module(cluster) or {}
    explicit = str(block.get("k8s_distribution") or "")
    return explicit or distribution_of(str(block.get("k8s_version") or "")) or resolve_distribution()


# --- base node -------------------------------------------------------------------------
@dataclass
class NodeBase:
    cfg: Dict
    count: int

    @property
    def hostname(self) -> str:
        return self.cfg["hostname"]


def base_node_config(ctx: Context, module_path: str, cluster: str, state: State) -> NodeBase:
    cfg: Dict = {
        "source": source_for(ctx, module_path),
        "hostname": "",
        "rancher_api_url": f"${{module.{MANAGER_KEY}.rancher_url}}",
        "rancher_cluster_registration_token": f"${{module.{cluster}.rancher_cluster_registration_token}}",
        "rancher_cluster_ca_checksum": f"${{module.{cluster}.rancher_cluster_ca_checksum}}",
        "rancher_host_labels": {},
        # copied *by value* from the manager / cluster modules (create/node.go:198-209)
        "rancher_agent_image": state.get(f"module.{MANAGER_KEY}.rancher_agent_image"),
        "rancher_registry": state.get(f"module.{cluster}.rancher_registry"),
        "rancher_registry_username": state.get(f"module.{cluster}.rancher_registry_username"),
        "rancher_registry_password": state.get(f"module.{cluster}.rancher_registry_password"),
        "k8s_distribution": node_distribution(state, cluster),
    }
    cfg["source"] = source_for(ctx, module_path)

    # Host label.  Deliberate fix: non-interactive mode
    # errors instead of prompting.
    label = ctx.resolve_choice("rancher_host_label", "Which type of node?", HOST_LABELS)
    if label not in HOST_LABELS:
        raise ConfigError(f"Invalid rancher_host_label '{label}', must be 'worker', 'etcd' or 'control'")
    cfg["rancher_host_labels"] = {label: "true"}

    # Node count: free text for workers (default 3), 1/3/5/7 otherwise.
    if ctx.is_set("node_count"):
        count_input = ctx.get_string("node_count")
    elif ctx.non_interactive:
        raise ConfigError("node_count must be specified")
    elif label == "worker":
        count_input = ctx.prompter.prompt("Number of nodes to create", default="3", validate=positive_int)
    else:
        _, count_input = ctx.prompter.select("Number of nodes to create", ["1", "3", "5", "7"])
    try:
        count = int(str(count_input).strip())
    except ValueError as exc:
        raise ConfigError(f"node_count must be a valid number. Found '{count_input}'.") from exc
    if count <= 0:
        raise ConfigError(f"node_count must be greater than 0. Found '{count}'.")

    cfg["hostname"] = ctx.resolve("hostname", "Hostname prefix",
                                  validate=not_blank("hostname prefix cannot be blank"))
    if not cfg["hostname"]:
        raise ConfigError("Invalid Hostname")
    omit_empty(cfg, ["rancher_agent_image", "rancher_registry", "rancher_registry_username",
                     "rancher_registry_password"])
    return NodeBase(cfg, count)


def _go_atoi(text: str) -> Optional[int]:
    """Go's ``strconv.Atoi`` on a 64-bit build: an optional sign and decimal digits, nothing
    else (not even a trailing newline), within int64; None where Atoi returns an error."""
    if not _ATOI_RE.fullmatch(text):
        return None
    num = int(text)
    return num if -(1 << 63) <= num < (1 << 63) else None


def new_hostnames(existing: Sequence[str], prefix: str, count: int) -> List[str]:
    """``<prefix>-<n>`` numbered after the highest existing suffix (``create/node.go:350-380``)."""
    if count < 1:
        return []
    start = 1
    target = prefix + "-"
    for name in existing:
        if not name.startswith(target):
            continue
        num = _go_atoi(name[len(target):])
        if num is None:
            continue
        if num >= start:
            start = num + 1
    return [f"{prefix}-{start + i}" for i in range(count)]


def add_nodes(state: State, cluster: str, base: NodeBase, extra: Dict,
              per_node: Optional[Sequence[Dict]] = None) -> List[str]:
    """Add ``base.count`` node modules (``cfgCopy`` loop of every node_*.go)."""
    existing = list(state.nodes(cluster).keys())
    hostnames = new_hostnames(existing, base.hostname, base.count)
    for i, hostname in enumerate(hostnames):
        cfg = dict(base.cfg)
        cfg.update(extra)
        if per_node is not None:
            cfg.update(per_node[i])
        cfg["hostname"] = hostname
        state.add_node(cluster, hostname, cfg)
    return hostnames


def nodes_added_message(hostnames: Sequence[str]) -> str:
    """``printNodesAddedMessage`` (``create/cluster.go:518-525``)."""
    if len(hostnames) == 1:
        return f"1 node added: {', '.join(hostnames)}"
    return f"{len(hostnames)} nodes added: {', '.join(hostnames)}"
