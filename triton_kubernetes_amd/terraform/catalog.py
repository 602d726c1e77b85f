"""Catalog of the Terraform module library (``terraform/modules/*``).

The 17 reference modules keep their names, input
variables and outputs — the module name is part of the ``main.tf.json``
``source`` contract.  Two MI355X modules are added:

* ``bare-metal-mi355x-rancher-k8s-host`` — bare-metal 8xMI355X worker: ROCm /
  amdgpu preflight, ``/dev/kfd`` + ``/dev/dri`` passthrough, native topology
  labeller (N1) feeding agent ``--label`` flags, RCCL environment file;
* ``rancher-k8s-mi355x-addons`` — cluster add-on step run once the cluster is
  active: ROCm k8s device plugin + node labeller DaemonSets, xGMI affinity
  example, RCCL readiness Job (N2).

Executors use the catalog to know which outputs a module exposes (root outputs
for Terraform >= 0.12, whose ``terraform output -module`` no longer exists).
"""

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from ..errors import ExecutorError

MODULES_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "modules")

# tk_* outputs are the CLI's own bookkeeping (pinned SSH host keys), not shown by `get`
MANAGER_OUTPUTS = ("rancher_url", "rancher_access_key", "rancher_secret_key", "tk_ssh_known_hosts", "tk_rancher_ca_certs")
CLUSTER_OUTPUTS = ("rancher_cluster_id", "rancher_cluster_registration_token", "rancher_cluster_ca_checksum")


@dataclass(frozen=True)
class ModuleInfo:
    name: str
    kind: str  # manager | cluster | host | addon
    provider: str  # triton | aws | gcp | azure | baremetal | vsphere
    outputs: Tuple[str, ...] = ()
    mi355x: bool = False
    # which provider-network outputs a host module consumes from its cluster
    consumes: Tuple[str, ...] = field(default_factory=tuple)

    @property
    def path(self) -> str:
        return f"terraform/modules/{self.name}"

    @property
    def local_dir(self) -> str:
        return os.path.join(MODULES_DIR, self.name)


_MODULES: List[ModuleInfo] = [
    # managers (T1-T5)
    ModuleInfo("triton-rancher", "manager", "triton", MANAGER_OUTPUTS),
    ModuleInfo("aws-rancher", "manager", "aws", MANAGER_OUTPUTS),
    ModuleInfo("gcp-rancher", "manager", "gcp", MANAGER_OUTPUTS),
    ModuleInfo("azure-rancher", "manager", "azure", MANAGER_OUTPUTS),
    ModuleInfo("bare-metal-rancher", "manager", "baremetal", MANAGER_OUTPUTS),
    # clusters (T6-T11)
    ModuleInfo("triton-rancher-k8s", "cluster", "triton", CLUSTER_OUTPUTS),
    ModuleInfo("aws-rancher-k8s", "cluster", "aws",
               CLUSTER_OUTPUTS + ("aws_subnet_id", "aws_security_group_id", "aws_key_name")),
    ModuleInfo("gcp-rancher-k8s", "cluster", "gcp",
               CLUSTER_OUTPUTS + ("gcp_compute_network_name", "gcp_compute_firewall_host_tag")),
    ModuleInfo("azure-rancher-k8s", "cluster", "azure",
               CLUSTER_OUTPUTS + ("azure_resource_group_name", "azure_network_security_group_id", "azure_subnet_id")),
    ModuleInfo("bare-metal-rancher-k8s", "cluster", "baremetal", CLUSTER_OUTPUTS),
    ModuleInfo("vsphere-rancher-k8s", "cluster", "vsphere",
               CLUSTER_OUTPUTS + ("vsphere_datacenter_name", "vsphere_datastore_name", "vsphere_resource_pool_name",
                                  "vsphere_network_name")),
    # hosts (T12-T17)
    ModuleInfo("triton-rancher-k8s-host", "host", "triton"),
    ModuleInfo("aws-rancher-k8s-host", "host", "aws",
               consumes=("aws_subnet_id", "aws_security_group_id", "aws_key_name")),
    ModuleInfo("gcp-rancher-k8s-host", "host", "gcp",
               consumes=("gcp_compute_network_name", "gcp_compute_firewall_host_tag")),
    ModuleInfo("azure-rancher-k8s-host", "host", "azure",
               consumes=("azure_resource_group_name", "azure_network_security_group_id", "azure_subnet_id")),
    ModuleInfo("bare-metal-rancher-k8s-host", "host", "baremetal"),
    ModuleInfo("vsphere-rancher-k8s-host", "host", "vsphere",
               consumes=("vsphere_datacenter_name", "vsphere_datastore_name", "vsphere_resource_pool_name",
                         "vsphere_network_name")),
    # MI355X additions
    ModuleInfo("bare-metal-mi355x-rancher-k8s-host", "host", "baremetal", ("gpu_node_labels", "tk_ssh_known_hosts"),
               mi355x=True),
    ModuleInfo("rancher-k8s-mi355x-addons", "addon", "baremetal", ("addons_applied",), mi355x=True),
]

CATALOG: Dict[str, ModuleInfo] = {m.name: m for m in _MODULES}
REFERENCE_MODULES = [m.name for m in _MODULES if not m.mi355x]


# The package directory: ``<PACKAGE_ROOT>/terraform/modules/<name>`` is this project's
# module tree.  Documents name it location-free (``tk::`` sources, below) and executors
# resolve those to it, so documents run the modules that ship with this CLI instead of
# the reference's Terraform 0.11 ones.
PACKAGE_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def is_local_source(source_url: str) -> bool:
    """A filesystem location (Terraform copies absolute paths into its module cache)."""
    return source_url.startswith(("/", "./", "../", "~"))


def packaged_root() -> str:
    """A real directory holding ``terraform/modules``: the package itself, or — when
    running from a zipapp, whose files are not on disk — a per-version extraction under
    ``~/.cache/triton-kubernetes``."""
    if os.path.isdir(MODULES_DIR):
        return PACKAGE_ROOT
    import zipfile

    from .. import __version__

    archive = PACKAGE_ROOT
    while archive and not os.path.isfile(archive):
        archive = os.path.dirname(archive)
    if not archive or not zipfile.is_zipfile(archive):
        raise FileNotFoundError(f"terraform modules not found at {MODULES_DIR}")
    inner = os.path.relpath(MODULES_DIR, archive).replace(os.sep, "/") + "/"
    cache = os.path.join(os.path.expanduser("~"), ".cache", "triton-kubernetes", f"modules-{__version__}")
    root = os.path.join(cache, "pkg")
    if not os.path.isdir(os.path.join(root, "terraform", "modules")):
        tmp = f"{cache}.tmp-{os.getpid()}"
        with zipfile.ZipFile(archive) as zf:
            for member in zf.namelist():
                if member.startswith(inner) and not member.endswith("/"):
                    rel = member[len(inner):]
                    dest = os.path.join(tmp, "pkg", "terraform", "modules", *rel.split("/"))
                    os.makedirs(os.path.dirname(dest), exist_ok=True)
                    with zf.open(member) as src, open(dest, "wb") as out:
                        out.write(src.read())
        os.makedirs(os.path.dirname(cache), exist_ok=True)
        try:
            os.rename(tmp, cache)
        except OSError:  # another process extracted it first
            import shutil

            shutil.rmtree(tmp, ignore_errors=True)
    return root


def module_source(source_url: str, module_path: str, source_ref: str) -> str:
    """``<url>//<path>?ref=<ref>`` for a remote (git/registry) prefix
    (``create/manager.go:160-171``); ``<dir>/<path>`` for a local directory, which
    Terraform reads directly (no ``//`` subdir or ``?ref=`` on filesystem sources)."""
    if is_local_source(source_url):
        return os.path.join(os.path.abspath(os.path.expanduser(source_url)), module_path)
    return f"{source_url}//{module_path}?ref={source_ref}"


# --- location-free sources of the packaged modules ------------------------------------
#
# The reference persists ``github.com/joyent/triton-kubernetes//terraform/modules/<m>?ref=``
# (create/manager.go:160-171): any operator, on any machine, can apply the document.  This
# CLI's modules ship inside the package, whose directory differs between machines, venvs
# and versions, so the persisted document names them symbolically:
#
#     tk::terraform/modules/<module>?ref=v<package version>
#
# and only the document an executor runs (executor/terraform.py:render, the direct
# executor's plan) sees the directory of *this* install.  A document pinned to another
# version of the modules is refused until ``migrate manager`` re-pins it: silently
# applying different module code to running infrastructure is what the pin prevents.
PACKAGED_SCHEME = "tk::"


def packaged_ref() -> str:
    from .. import __version__

    return f"v{__version__}"


def packaged_source(module_path: str) -> str:
    """The persisted source of a packaged module (``module_path`` = ``terraform/modules/<m>``)."""
    return f"{PACKAGED_SCHEME}{module_path}?ref={packaged_ref()}"


def is_packaged_source(source: str) -> bool:
    return source.startswith(PACKAGED_SCHEME)


def _packaged_parts(source: str) -> Tuple[str, str]:
    """``(module name, ref)`` of a ``tk::`` source."""
    body = source[len(PACKAGED_SCHEME):]
    path, _, query = body.partition("?")
    ref = ""
    for part in query.split("&"):
        if part.startswith("ref="):
            ref = part[len("ref="):]
    return path.rstrip("/").rsplit("/", 1)[-1], ref


class ModuleRefMismatch(ExecutorError):
    """A ``tk::`` source pinned to modules of another CLI version."""


def resolve_source(source: str, key: str = "") -> str:
    """The source Terraform is given: a ``tk::`` source becomes this install's module
    directory; every other source is returned unchanged.

    Raises :class:`ModuleRefMismatch` for a ``tk::`` source pinned to another version and
    :class:`ExecutorError` for a module this package does not ship."""
    if not is_packaged_source(source):
        return source
    name, ref = _packaged_parts(source)
    where = f"module.{key}" if key else source
    if name not in CATALOG:
        raise ExecutorError(f"{where}: {source!r} names no module of this CLI")
    want = packaged_ref()
    if ref != want:
        raise ModuleRefMismatch(
            f"{where} is pinned to the triton-kubernetes modules {ref or '(no ref)'}, but this CLI ships {want}. "
            "Run `triton-kubernetes migrate manager` to re-pin the document to the installed modules, "
            f"or use triton-kubernetes {ref.lstrip('v') or 'of that version'} to operate on it.")
    return os.path.join(packaged_root(), "terraform", "modules", name)


def check_sources(modules: Dict[str, Dict]) -> None:
    """Refuse a document this install cannot run, before anything is built on it: a
    ``tk::`` source of another version or of an unknown module, or an absolute path into
    another install's module tree that does not exist here (documents written before the
    ``tk::`` form)."""
    for key, mod in modules.items():
        if not isinstance(mod, dict):  # Terraform refuses such a document too
            raise ExecutorError(f"module.{key} in main.tf.json is not a module block (an object): {mod!r:.60}")
        source = str(mod.get("source", ""))
        if is_packaged_source(source):
            resolve_source(source, key)
        elif packaged_module_of_path(source) is not None and not os.path.isdir(source.split("?", 1)[0]):
            raise ExecutorError(
                f"module.{key} points at {source}, a module directory of another triton-kubernetes install that "
                "does not exist on this machine. Run `triton-kubernetes migrate manager` to rewrite the document's "
                "module sources to the location-free tk:: form.")


_DECLARED: Dict[Tuple[str, float], frozenset] = {}


def declared_variables(mod_dir: str) -> frozenset:
    """Names of the ``variable`` blocks a module directory declares (top level of its .tf
    files), cached per directory and modification time."""
    try:
        stamp = max(os.path.getmtime(os.path.join(mod_dir, f)) for f in os.listdir(mod_dir) if f.endswith(".tf"))
    except (OSError, ValueError):
        return frozenset()
    key = (mod_dir, stamp)
    if key not in _DECLARED:
        import re

        names = set()
        for fn in os.listdir(mod_dir):
            if fn.endswith(".tf"):
                with open(os.path.join(mod_dir, fn), encoding="utf-8") as fh:
                    names.update(re.findall(r'^variable\s+"([^"]+)"', fh.read(), re.M))
        _DECLARED[key] = frozenset(names)
    return _DECLARED[key]


def local_module_dir(source: str) -> Optional[str]:
    """The directory a local ``source`` points at (None for remote sources); a ``tk::``
    source resolves to this install's module directory (see :func:`resolve_source`)."""
    if is_packaged_source(source):
        return resolve_source(source)
    path = source.split("?", 1)[0]
    return path if is_local_source(path) else None


def packaged_module_of_path(source: str) -> Optional[ModuleInfo]:
    """The catalog module an *absolute path* source names when that path is some
    install's packaged tree (``.../terraform/modules/<m>``): what ``migrate manager``
    rewrites to a ``tk::`` source."""
    path = source.split("?", 1)[0].rstrip("/")
    if not path.startswith("/"):
        return None
    parent, name = os.path.split(path)
    if os.path.basename(parent) != "modules" or os.path.basename(os.path.dirname(parent)) != "terraform":
        return None
    return CATALOG.get(name)


def module_from_source(source: str) -> Optional[ModuleInfo]:
    """Identify the catalog module a ``source`` string points at."""
    path = source.split("?", 1)[0]
    name = path.rstrip("/").rsplit("/", 1)[-1]
    return CATALOG.get(name)


def outputs_for_source(source: str) -> Tuple[str, ...]:
    info = module_from_source(source)
    return info.outputs if info else ()


_SENSITIVE: Optional[Dict[str, Dict[str, bool]]] = None


def sensitive_outputs(module_name: str) -> Tuple[str, ...]:
    """Outputs of a catalog module declared ``sensitive = true`` (from the generator's
    module definitions, the single source of truth for the rendered ``outputs.tf``)."""
    global _SENSITIVE
    if _SENSITIVE is None:
        from .generate import output_sensitivity  # lazy: generate imports this module

        _SENSITIVE = output_sensitivity()
    return tuple(n for n, s in _SENSITIVE.get(module_name, {}).items() if s)
