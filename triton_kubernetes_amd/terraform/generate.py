"""Generator of the Terraform module library (``terraform/modules/*``).

The 19 modules are data here and written out as plain HCL files (committed;
``tests/test_terraform_modules.py`` checks that they are in sync with this
generator and internally consistent).  Run ``python -m
triton_kubernetes_amd.terraform.generate`` after editing.

Design (rewritten for Terraform >= 1.x and a current Rancher):

* managers (T1-T5): VM (or the bare-metal host) -> docker via user-data or
  remote-exec -> Rancher server -> API bootstrap on the host -> API key read
  back with a ``data "external"`` SSH program (replaces ``matti/outputs/shell``);
* clusters (T6-T11): ``data "external"`` find-or-create of the RKE cluster
  (S4) + the provider network the hosts join;
* hosts (T12-T17): the agent bootstrap (S5) as user-data / remote-exec, the
  reference's ``control`` -> ``controlplane`` role mapping, optional data disks
  (the GCP disk is now attached, Q15; vSphere CPU/memory are variables, Q15);
* ``bare-metal-mi355x-rancher-k8s-host`` and ``rancher-k8s-mi355x-addons``.

Every module pins ``required_version >= 1.4`` (``terraform_data`` is a 1.4 resource)
and its providers'
sources (``joyent/triton``, ``hashicorp/aws|google|azurerm|vsphere|external``).
"""

import json
import os
import shutil
import sys
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

from .. import sizing, versions
from ..parallel import rccl_env
from ..node.cleanup import cleanup_script
from ..node.tools import PREBUILT_DIR, SOURCES_DIR
from . import scripts
from .catalog import MODULES_DIR

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ops", "csrc")

DOCKER_URL = versions.DOCKER_INSTALL_URL
SERVER_IMAGE = versions.SERVER_IMAGE
AGENT_IMAGE = versions.AGENT_IMAGE

PROVIDERS = {
    "triton": ('triton = {\n      source  = "joyent/triton"\n      version = ">= 0.8"\n    }',
               'provider "triton" {\n  account      = var.triton_account\n  key_material = file(pathexpand(var.triton_key_path))\n  key_id       = var.triton_key_id\n  url          = var.triton_url\n}'),
    "aws": ('aws = {\n      source  = "hashicorp/aws"\n      version = ">= 4.0"\n    }',
            'provider "aws" {\n  access_key = var.aws_access_key\n  secret_key = var.aws_secret_key\n  region     = var.aws_region\n}'),
    "gcp": ('google = {\n      source  = "hashicorp/google"\n      version = ">= 4.0"\n    }',
            'provider "google" {\n  credentials = file(pathexpand(var.gcp_path_to_credentials))\n  project     = var.gcp_project_id\n  region      = var.gcp_compute_region\n}'),
    "azure": ('azurerm = {\n      source  = "hashicorp/azurerm"\n      version = ">= 3.0"\n    }',
              'provider "azurerm" {\n  features {}\n  subscription_id = var.azure_subscription_id\n  client_id       = var.azure_client_id\n  client_secret   = var.azure_client_secret\n  tenant_id       = var.azure_tenant_id\n  environment     = var.azure_environment\n}'),
    "vsphere": ('vsphere = {\n      source  = "hashicorp/vsphere"\n      version = ">= 2.0"\n    }',
                'provider "vsphere" {\n  user                 = var.vsphere_user\n  password             = var.vsphere_password\n  vsphere_server       = var.vsphere_server\n  allow_unverified_ssl = true\n}'),
    "external": ('external = {\n      source  = "hashicorp/external"\n      version = ">= 2.0"\n    }', ""),
    "tls": ('tls = {\n      source  = "hashicorp/tls"\n      version = ">= 4.0"\n    }', ""),
}


@dataclass
class Var:
    name: str
    default: Any = None  # None -> required
    description: str = ""
    type: Optional[str] = None
    sensitive: bool = False

    def hcl(self) -> str:
        """Terraform >= 1.3 declaration: explicit type, description, default, validation."""
        vtype = self.type or _infer_type(self.default)
        desc = self.description or VAR_DOCS.get(self.name) or _doc_from_name(self.name)
        lines = [f'variable "{self.name}" {{', f"  description = {json.dumps(desc)}", f"  type        = {vtype}"]
        if self.default is not None:
            lines.append(f"  default     = {hcl_value(self.default)}")
        if self.sensitive:
            lines.append("  sensitive   = true")
        rule = VAR_VALIDATIONS.get(self.name)
        if rule is not None:
            cond, msg = rule
            lines += ["", "  validation {", f"    condition     = {cond}",
                      f"    error_message = {json.dumps(msg)}", "  }"]
        lines.append("}")
        return "\n".join(lines)


def _infer_type(default: Any) -> str:
    if isinstance(default, bool):
        return "bool"
    if isinstance(default, (list, tuple)):
        return "list(string)"
    if isinstance(default, dict):
        return "map(string)"
    if isinstance(default, (int, float)) and not isinstance(default, bool):
        return "number"
    return "string"


def _doc_from_name(name: str) -> str:
    words = name.replace("_", " ")
    for prefix, cloud in (("aws ", "AWS"), ("gcp ", "GCP"), ("azure ", "Azure"), ("triton ", "Triton"),
                          ("vsphere ", "vSphere"), ("ebs ", "EBS"), ("k8s ", "Kubernetes")):
        if words.startswith(prefix):
            words = cloud + " " + words[len(prefix):]
    return words[0].upper() + words[1:] + "."


# Descriptions for variables shared by many modules (the rest are derived from the name).
VAR_DOCS = {
    "rancher_api_url": "Base URL of the Rancher server (the cluster manager's rancher_url output).",
    "rancher_access_key": "Rancher API access key (cluster manager output).",
    "rancher_secret_key": "Rancher API secret key (cluster manager output).",
    "rancher_cluster_registration_token": "Registration token of the cluster the node joins.",
    "rancher_cluster_ca_checksum": "SHA-256 of the Rancher CA bundle, pinned by the agent.",
    "rancher_server_image": "Rancher server container image.",
    "rancher_agent_image": "Rancher agent container image.",
    "rancher_registry": "Private registry serving the Rancher images (empty: Docker Hub).",
    "rancher_registry_username": "User for rancher_registry.",
    "rancher_registry_password": "Password for rancher_registry.",
    "k8s_version": "RKE Kubernetes version.",
    "k8s_network_provider": "CNI plugin of the cluster.",
    "k8s_registry": "Private registry for the Kubernetes system images (empty: default).",
    "k8s_registry_username": "User for k8s_registry.",
    "k8s_registry_password": "Password for k8s_registry.",
    "hostname": "Host name given to the node.",
    "docker_engine_install_url": "Script that installs the container runtime when it is missing.",
    "host": "Address of the machine reached over SSH.",
    "ssh_user": "SSH login user.",
    "key_path": "Private key used for SSH.",
    "bastion_host": "Optional SSH jump host (empty: direct).",
    "gpu_count": "GPUs the MI355X node must expose.",
    "gpu_burnin": "Burn-in level run on every GPU before the node joins.",
    "rccl_env": "Extra RCCL/HSA environment written to /etc/rccl/rccl.env.",
    "docker_install_sha256": "SHA-256 the downloaded runtime install script must match (empty: not checked).",
    "tk_known_hosts": ("known_hosts lines of the cluster manager's pinned SSH host keys (set by the executor "
                       "through the root variable of the same name, parallel/hostkeys.py)."),
    "host_key": "Pinned SSH host key of host (\"<type> <base64>\", set by the executor; empty: not pinned yet).",
    "bastion_host_key": "Pinned SSH host key of bastion_host (set by the executor; empty: not pinned yet).",
    "tk_operation": ("Which CLI operation runs this configuration (set by the executor through the root "
                     "variable of the same name): apply runs the create-side data sources in full; destroy and read "
                     "make them find-only and tolerant of hosts that are gone."),
    "rancher_bootstrap_password": ("First-login password of the Rancher server (CATTLE_BOOTSTRAP_PASSWORD); "
                                   "empty: derived from name and rancher_admin_password."),
}
# values spliced into single-quoted shell words and JSON bodies by the bootstrap scripts
# (HCL string "['\"\\\\]" is the RE2 class ['"\\]: single quote, double quote, backslash)
_SHELL_SAFE = (r'length(regexall("[' + "'" + r'\"\\\\]", var.{0})) == 0', "{0} must not contain quotes or backslashes.")
_NON_NEG = "^[0-9]+([.][0-9]+)?$"
# values the host scripts put inside single quotes or on a command line (the node agent checks
# the same fields with node/agent_steps.py's patterns): no quote, space or shell syntax
_URL = "^https?://[][A-Za-z0-9._:-]+(/[A-Za-z0-9._/-]*)?$"
_SHELL_WORDS = {
    "rancher_api_url": (_URL, "an http(s) URL"),
    "rancher_cluster_registration_token": ("^[A-Za-z0-9._:-]{1,512}$", "a Rancher registration token"),
    "rancher_cluster_ca_checksum": ("^[A-Za-z0-9]{0,128}$", "a hex checksum (or empty)"),
    "rancher_agent_image": ("^[A-Za-z0-9][A-Za-z0-9._/:@-]{0,254}$", "a container image reference"),
    "rancher_registry": ("^([A-Za-z0-9][A-Za-z0-9._/:@-]{0,254})?$", "a registry host (or empty)"),
    "docker_engine_install_url": ("^(https?://[][A-Za-z0-9._:-]+(/[A-Za-z0-9._/~%+=-]*)?)?$",
                                  "an http(s) URL (or empty)"),
    "docker_install_sha256": ("^[A-Fa-f0-9]{0,64}$", "a sha256 hex digest (or empty)"),
    "hostname": ("^[A-Za-z0-9]([-A-Za-z0-9.]{0,251}[A-Za-z0-9])?$", "a DNS host name"),
}
VAR_VALIDATIONS = {
    **{name: (f'length(regexall("{pat}", var.{name})) > 0', f"{name} must be {what}.")
       for name, (pat, what) in _SHELL_WORDS.items()},
    "rancher_registry_username": (_SHELL_SAFE[0].format("rancher_registry_username"),
                                  _SHELL_SAFE[1].format("rancher_registry_username")),
    "rancher_registry_password": (_SHELL_SAFE[0].format("rancher_registry_password"),
                                  _SHELL_SAFE[1].format("rancher_registry_password")),
    # numbers the host script passes to the node tools' argv
    "rccl_min_busbw": (f'length(regexall("{_NON_NEG}", var.rccl_min_busbw)) > 0',
                       "rccl_min_busbw must be a non-negative number (GB/s)."),
    "gpu_link_min_gbps": (f'length(regexall("{_NON_NEG}", var.gpu_link_min_gbps)) > 0',
                          "gpu_link_min_gbps must be a non-negative number (GB/s)."),
    "gpu_link_min_frac": ('length(regexall("^(0([.][0-9]+)?|1([.]0+)?|[.][0-9]+)$", var.gpu_link_min_frac)) > 0',
                          "gpu_link_min_frac must be a number between 0 and 1."),
    # the node's RCCL environment file is loaded as root (parallel/rccl_env.py:env_problems)
    "rccl_env": ('alltrue([for k, v in var.rccl_env : length(regexall("' + rccl_env.ENV_KEY_RE + '", k)) > 0 && '
                 'length(regexall("' + rccl_env.ENV_KEY_DENY_RE + '", k)) == 0 && '
                 f'length(v) <= {rccl_env.ENV_VALUE_MAX} && '
                 'alltrue([for item in split(",", v) : length(regexall("' + rccl_env.ENV_ITEM_RE + '", item)) > 0])])',
                 "rccl_env takes NCCL_*, RCCL_* and HSA_* settings whose values are comma lists of letters, digits and "
                 "_ . : = ^ + - (an address range's /N allowed); settings that name a library, plugin, file, path or "
                 "directory are not accepted."),
    "rancher_admin_password": (f'length(var.rancher_admin_password) >= {versions.PASSWORD_MIN_LENGTH} && '
                               + _SHELL_SAFE[0].format("rancher_admin_password"),
                               f"rancher_admin_password must be at least {versions.PASSWORD_MIN_LENGTH} characters "
                               "(Rancher >= 2.6) without quotes or backslashes."),
    "rancher_bootstrap_password": (_SHELL_SAFE[0].format("rancher_bootstrap_password"),
                                   _SHELL_SAFE[1].format("rancher_bootstrap_password")),
    # (which distribution the release belongs to is checked against k8s_distribution in a
    # precondition: a validation block may only read its own variable before Terraform 1.9)
    "k8s_version": ('(contains([' + ", ".join(f'"{m}"' for m in versions.RKE2_MINORS) + '], '
                    'join(".", slice(split(".", var.k8s_version), 0, 2))) && '
                    'length(regexall("[+]rke2r[0-9]+$", var.k8s_version)) > 0) || '
                    '(contains([' + ", ".join(f'"{m}"' for m in versions.K8S_MINORS) + '], '
                    'join(".", slice(split(".", var.k8s_version), 0, 2))) && '
                    'length(regexall("-rancher[0-9]+-[0-9]+$", var.k8s_version)) > 0)',
                    f"k8s_version must be an RKE2 ({', '.join(v for _, v in versions.RKE2_VERSIONS)}) or RKE1 "
                    f"({', '.join(v for _, v in versions.K8S_VERSIONS)}) release of Rancher "
                    f"{versions.RANCHER_VERSION}."),
    "tk_operation": ('contains(["apply", "destroy", "read"], var.tk_operation)',
                     "tk_operation must be apply, destroy or read."),
    "k8s_distribution": ('contains(["rke2", "rke1"], var.k8s_distribution)', "k8s_distribution must be rke2 or rke1."),
    "k8s_network_provider": ('contains(["canal", "calico", "cilium", "flannel", "weave"], var.k8s_network_provider)',
                             "k8s_network_provider must be one of canal, calico, cilium, flannel (RKE2) or weave "
                             "(RKE1)."),
    "gpu_burnin": ('contains(["quick", "full", "off"], var.gpu_burnin)', "gpu_burnin must be quick, full or off."),
    "rccl_slim": ('contains(["on", "off"], var.rccl_slim)', "rccl_slim must be on or off."),
    "gpu_compute_partition": ('contains(["spx", "dpx", "qpx", "cpx"], var.gpu_compute_partition)',
                              "gpu_compute_partition must be one of spx, dpx, qpx, cpx."),
    "gpu_memory_partition": ('contains(["nps1", "nps2"], var.gpu_memory_partition)',
                             "gpu_memory_partition must be nps1 or nps2."),
    # GPU policies (node/health.py, node/hosttune.py, node/metrics.py)
    "gpu_health": ('contains(["fail", "taint", "off"], var.gpu_health)', "gpu_health must be fail, taint or off."),
    "gpu_host_tuning": ('contains(["warn", "enforce", "off"], var.gpu_host_tuning)',
                        "gpu_host_tuning must be warn, enforce or off."),
    "gpu_max_uncorrectable_ecc": ('length(regexall("^[0-9]+$", var.gpu_max_uncorrectable_ecc)) > 0',
                                  "gpu_max_uncorrectable_ecc must be a non-negative integer."),
    "gpu_max_retired_pages": ('var.gpu_max_retired_pages == "auto" || '
                              'length(regexall("^[0-9]+$", var.gpu_max_retired_pages)) > 0',
                              "gpu_max_retired_pages must be a non-negative integer or auto."),
    "gpu_metrics_textfile": ('var.gpu_metrics_textfile == "" || '
                             '(length(regexall("^/[A-Za-z0-9._/-]+$", var.gpu_metrics_textfile)) > 0 && '
                             'length(regexall("/[.][.](/|$)", var.gpu_metrics_textfile)) == 0)',
                             "gpu_metrics_textfile must be empty or an absolute directory path."),
    "rancher_host_labels": ('length(var.rancher_host_labels) == 1 && contains(["worker", "etcd", "control"], '
                            'keys(var.rancher_host_labels)[0])',
                            "rancher_host_labels must hold exactly one of worker, etcd or control."),
}


@dataclass
class Module:
    name: str
    providers: Sequence[str]
    variables: List[Var]
    main: str
    outputs: List[Tuple[str, str, bool]]  # name, expression, sensitive
    files: Dict[str, str] = field(default_factory=dict)  # filename -> content
    copies: Dict[str, str] = field(default_factory=dict)  # filename -> source path to copy


def hcl_value(v: Any, indent: int = 0) -> str:
    pad = "  " * indent
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return json.dumps(v)
    if isinstance(v, str):
        return json.dumps(v).replace("${", "$${").replace("%{", "%%{")
    if isinstance(v, list):
        if not v:
            return "[]"
        inner = ",\n".join(f"{pad}  {hcl_value(x, indent + 1)}" for x in v)
        return "[\n" + inner + f"\n{pad}]"
    if isinstance(v, dict):
        if not v:
            return "{}"
        inner = "\n".join(f"{pad}  {json.dumps(k)} = {hcl_value(x, indent + 1)}" for k, x in v.items())
        return "{\n" + inner + f"\n{pad}}}"
    raise TypeError(type(v))


# --- variable sets ---------------------------------------------------------------------------
def _rancher_image_vars(server: bool = True) -> List[Var]:
    out = [Var("docker_engine_install_url", DOCKER_URL, "The URL to the shell script to install the docker engine."),
           Var("docker_install_sha256", "")]
    if server:
        out.append(Var("rancher_server_image", SERVER_IMAGE, "The Rancher Server image to use."))
    out.append(Var("rancher_agent_image", AGENT_IMAGE, "The Rancher Agent image to use."))
    out += [Var("rancher_registry", "", "The docker registry to use for rancher server and agent images"),
            Var("rancher_registry_username", "", "The username to login as."),
            Var("rancher_registry_password", "", "The password to use.", sensitive=True)]
    return out


MANAGER_BASE = [Var("name", None, "Human readable name used as prefix to generated names."),
                Var("rancher_admin_password", None, "The Rancher admin password", sensitive=True),
                Var("rancher_bootstrap_password", "", sensitive=True), Var("tk_operation", "apply"),
                Var("tk_known_hosts", "")]
# SSH host keys pinned by the CLI (parallel/hostkeys.py), rendered by the executor
PINNED_KEY_VARS = [Var("host_key", ""), Var("bastion_host_key", "")]
CLUSTER_BASE = [
    Var("name", None, "Human readable name used as prefix to generated names."), Var("tk_operation", "apply"),
    Var("rancher_api_url", None), Var("rancher_access_key", None), Var("rancher_secret_key", None, sensitive=True),
    Var("k8s_distribution", versions.DEFAULT_DISTRIBUTION,
        "rke2 (provisioning.cattle.io/v1 custom cluster, nodes join with rancher-system-agent) or rke1 "
        "(v3 cluster + rancher-agent; reference-era documents)"),
    Var("k8s_version", versions.DEFAULT_K8S_VERSION), Var("k8s_network_provider", "canal"),
    Var("tk_rancher_ca", "", "PEM CA bundle the Rancher server is verified against (the manager's pinned CA, "
        "rendered by the CLI; empty: a publicly trusted certificate)"),
    Var("rancher_registry", ""), Var("rancher_registry_username", ""), Var("rancher_registry_password", "", sensitive=True),
    Var("k8s_registry", ""), Var("k8s_registry_username", ""), Var("k8s_registry_password", "", sensitive=True),
]
HOST_BASE = [
    Var("hostname", None), Var("rancher_api_url", None),
    Var("k8s_distribution", versions.DEFAULT_DISTRIBUTION,
        "the cluster's distribution: rke2 joins with the server's system-agent installer, rke1 with docker run "
        "rancher/rancher-agent"),
    Var("rancher_cluster_registration_token", None, sensitive=True), Var("rancher_cluster_ca_checksum", None),
    Var("rancher_host_labels", None, "A single-key map: {worker|etcd|control = \"true\"}", "map(string)"),
] + _rancher_image_vars(server=False)

TRITON_CREDS = [Var("triton_account", None), Var("triton_key_path", None), Var("triton_key_id", None),
                Var("triton_url", "https://us-east-1.api.joyent.com")]
AWS_CREDS = [Var("aws_access_key", None), Var("aws_secret_key", None, sensitive=True), Var("aws_region", None)]
GCP_CREDS = [Var("gcp_path_to_credentials", None), Var("gcp_compute_region", None), Var("gcp_project_id", None)]
AZURE_CREDS = [Var("azure_subscription_id", ""), Var("azure_client_id", ""), Var("azure_client_secret", "", sensitive=True),
               Var("azure_tenant_id", ""), Var("azure_environment", "public"), Var("azure_location", "westus2")]
AZURE_IMAGE = [Var("azure_image_publisher", "Canonical"), Var("azure_image_offer", "0001-com-ubuntu-server-jammy"),
               Var("azure_image_sku", "22_04-lts-gen2"), Var("azure_image_version", "latest")]
VSPHERE_CREDS = [Var("vsphere_user", None), Var("vsphere_password", None, sensitive=True), Var("vsphere_server", None)]
VSPHERE_NAMES = [Var("vsphere_datacenter_name", None), Var("vsphere_datastore_name", None),
                 Var("vsphere_resource_pool_name", None), Var("vsphere_network_name", None)]

# RKE1 + RKE2 node ports (9345: the RKE2 supervisor, 2381: etcd metrics)
RKE_PORTS = [(22, 22), (80, 80), (443, 443), (2376, 2376), (2379, 2381), (6443, 6443), (8472, 8472),
             (9099, 9099), (9345, 9345), (10250, 10252), (10254, 10256), (30000, 32767)]

ROLE_LOCAL = """locals {
  rancher_node_role_raw = keys(var.rancher_host_labels)[0]
  rancher_node_role     = local.rancher_node_role_raw == "control" ? "controlplane" : local.rancher_node_role_raw
}"""

MANAGER_OUTPUTS = [
    ("rancher_url", '"https://${local.rancher_master_ip}"', False),
    ("rancher_access_key", "data.external.rancher_api_key.result.access_key", False),
    ("rancher_secret_key", "data.external.rancher_api_key.result.secret_key", True),
    # the host keys the key read pinned (parallel/hostkeys.py; not shown by `get manager`)
    ("tk_ssh_known_hosts", "data.external.rancher_api_key.result.known_hosts", False),
    # the server's CA bundle as read on the manager host (rancher/trust.py pins it)
    ("tk_rancher_ca_certs", "data.external.rancher_api_key.result.ca_certs", False),
]
CLUSTER_OUTPUTS = [
    ("rancher_cluster_id", 'data.external.cluster.result["cluster_id"]', False),
    ("rancher_cluster_registration_token", 'data.external.cluster.result["registration_token"]', True),
    ("rancher_cluster_ca_checksum", 'data.external.cluster.result["ca_checksum"]', False),
]
OUTPUT_DOCS = {
    "rancher_url": "URL of the Rancher server.",
    "rancher_access_key": "API access key created for triton-kubernetes.",
    "rancher_secret_key": "API secret key created for triton-kubernetes.",
    "rancher_cluster_id": "Rancher id of the cluster (found by name or created).",
    "tk_ssh_known_hosts": "known_hosts lines of the hosts this module's SSH reads contacted (pinned by the CLI).",
    "tk_rancher_ca_certs": "The Rancher server's CA bundle as its host serves it (pinned by the CLI; empty: public CA).",
    "rancher_cluster_registration_token": "Token nodes present when they register.",
    "rancher_cluster_ca_checksum": "Checksum of the Rancher CA bundle that agents pin.",
}


def _manager_tail(connection: str, install_docker_remote: bool) -> str:
    """Rancher server install + bootstrap + API key read-back (shared by T1-T5)."""
    docker = ""
    after = ""
    if install_docker_remote:
        docker = f'''
resource "terraform_data" "install_docker" {{
  triggers_replace = [local.rancher_master_id]
{connection}
  provisioner "remote-exec" {{
    inline = [templatefile("${{path.module}}/files/install_docker.sh.tftpl", {{
      docker_engine_install_url = var.docker_engine_install_url
      docker_install_sha256     = var.docker_install_sha256
      rancher_server_image      = var.rancher_server_image
      rancher_registry          = var.rancher_registry
      rancher_registry_username = var.rancher_registry_username
      rancher_registry_password = var.rancher_registry_password
    }})]
  }}
}}
'''
        after = "\n  depends_on       = [terraform_data.install_docker]"
    return docker + f'''
locals {{
  # Rancher >= 2.6 first login (CATTLE_BOOTSTRAP_PASSWORD): random, kept in the state
  # backend by the CLI and rendered here (rancher/bootstrap_secret.py) -- no function of
  # the admin password
  bootstrap_password = var.rancher_bootstrap_password
}}

resource "terraform_data" "install_rancher_master" {{
  triggers_replace = [local.rancher_master_id]{after}
{connection}
  provisioner "remote-exec" {{
    inline = [templatefile("${{path.module}}/files/install_rancher_server.sh.tftpl", {{
      rancher_server_image = var.rancher_server_image
      bootstrap_password   = local.bootstrap_password
    }})]
  }}
}}

resource "terraform_data" "setup_rancher_k8s" {{
  triggers_replace = [local.rancher_master_id]
  depends_on       = [terraform_data.install_rancher_master]
{connection}
  provisioner "remote-exec" {{
    inline = [templatefile("${{path.module}}/files/setup_rancher.sh.tftpl", {{
      rancher_host           = "https://127.0.0.1"
      host_registration_url  = "https://${{local.rancher_master_ip}}"
      bootstrap_password     = local.bootstrap_password
    }})]
  }}
}}

# The API key and the CA bundle setup_rancher saved are read back over SSH, which then also
# carries the admin password (on the host's curl stdin, never a command line or a file).
data "external" "rancher_api_key" {{
  depends_on = [terraform_data.setup_rancher_k8s]
  program    = ["bash", "${{path.module}}/files/read_api_key.sh"]
  query = {{
    host               = local.rancher_master_ip
    ssh_user           = local.ssh_user
    key_path           = local.key_path
    bastion_host       = local.bastion_host
    operation          = var.tk_operation
    known_hosts        = var.tk_known_hosts
    admin_password     = var.rancher_admin_password
    bootstrap_password = local.bootstrap_password
  }}
}}
'''


# the MI355X host module's prebuilt node tools (node/tools.py), staged by the CLI
PREBUILT_VAR = "tk_prebuilt_tools"
PREBUILT_README = """The CLI uploads its prebuilt gfx950 node tools from a staging directory it passes as
tk_prebuilt_tools; this placeholder is uploaded when none is passed.  The node then builds the
tools from the shipped sources (files/src) with hipcc.  See triton_kubernetes_amd/node/tools.py.
"""
NODE_CLEANUP_VAR = Var("node_cleanup", True,
                       "on destroy, take the host out of its cluster: uninstall rancher-system-agent and RKE2 (or "
                       "the RKE1 containers) and remove their state, keeping the node tools and the container "
                       "runtime (bare metal outlives its cluster; node/cleanup.py)", "bool")


def _node_cleanup(install: str) -> str:
    """The bare-metal host's destroy-time teardown.  Destroy-time provisioners may reference
    only ``self`` (and ``path``): the connection is kept in ``input``, refreshed by every
    apply (``input`` changes update in place; only a new host replaces it, which tears
    down the old host).  ``on_failure = continue``: a dead host must not pin the state.

    The resource always exists: ``node_cleanup`` travels in ``input`` and the script skips
    the teardown when it is false (``TK_NODE_CLEANUP``).  A ``count = var.node_cleanup ? 1
    : 0`` would make turning the flag off on a host in service destroy instance [0] -- and
    so run the very teardown the flag is meant to prevent.  ``agent_image``
    (``TK_AGENT_IMAGE``): the RKE1 agent image the join ran, whose containers the teardown
    removes with any registry and tag.  Remote-exec joins ``inline`` into one script: the
    shebang goes first."""
    return f'''
resource "terraform_data" "node_cleanup" {{
  depends_on       = [terraform_data.{install}]
  triggers_replace = [var.host]
  input = {{
    host             = var.host
    user             = var.ssh_user
    key_path         = var.key_path
    host_key         = var.host_key
    bastion_host     = var.bastion_host
    bastion_host_key = var.bastion_host_key
    node_cleanup     = var.node_cleanup
    agent_image      = var.rancher_agent_image
  }}
  provisioner "remote-exec" {{
    when       = destroy
    on_failure = continue
    connection {{
      type             = "ssh"
      user             = self.input.user
      host             = self.input.host
      private_key      = file(pathexpand(self.input.key_path))
      host_key         = self.input.host_key == "" ? null : self.input.host_key
      bastion_host     = self.input.bastion_host == "" ? null : self.input.bastion_host
      bastion_host_key = self.input.bastion_host_key == "" ? null : self.input.bastion_host_key
    }}
    inline = [
      "#!/bin/bash",
      "export TK_NODE_CLEANUP='${{self.input.node_cleanup}}' TK_AGENT_IMAGE='${{self.input.agent_image}}'",
      file("${{path.module}}/files/cleanup_host.sh"),
    ]
  }}
}}
'''


def _connection(host: str = "local.rancher_master_ip", user: str = "local.ssh_user", key: str = "local.key_path",
                bastion: Optional[str] = "local.bastion_host", pinned: bool = False) -> str:
    """A provisioner ``connection``; ``pinned``: check the host's (and bastion's) key against
    the keys the CLI pinned (``host_key`` / ``bastion_host_key``, rendered by the executor
    from the manager's ``known_hosts``; empty = not pinned yet)."""
    lines = ["  connection {", '    type        = "ssh"', f"    user        = {user}", f"    host        = {host}",
             f"    private_key = file(pathexpand({key}))"]
    if pinned:
        lines.append('    host_key    = var.host_key == "" ? null : var.host_key')
    if bastion:
        lines.append(f"    bastion_host = {bastion} == \"\" ? null : {bastion}")
        if pinned:
            lines.append('    bastion_host_key = var.bastion_host_key == "" ? null : var.bastion_host_key')
    lines.append("  }")
    return "\n".join(lines)


def _docker_userdata(server: bool) -> str:
    image = "var.rancher_server_image" if server else '""'
    return f'''templatefile("${{path.module}}/files/install_docker.sh.tftpl", {{
    docker_engine_install_url = var.docker_engine_install_url
    docker_install_sha256     = var.docker_install_sha256
    rancher_server_image      = {image}
    rancher_registry          = var.rancher_registry
    rancher_registry_username = var.rancher_registry_username
    rancher_registry_password = var.rancher_registry_password
  }})'''


def _agent_userdata(disk_device: str = '""', disk_mount: str = '""', extra: str = '""') -> str:
    return f'''templatefile("${{path.module}}/files/install_rancher_agent.sh.tftpl", {{
    hostname                           = var.hostname
    docker_engine_install_url          = var.docker_engine_install_url
    docker_install_sha256              = var.docker_install_sha256
    rancher_api_url                    = var.rancher_api_url
    rancher_cluster_registration_token = var.rancher_cluster_registration_token
    rancher_cluster_ca_checksum        = var.rancher_cluster_ca_checksum
    rancher_node_role                  = local.rancher_node_role
    k8s_distribution                   = var.k8s_distribution
    rancher_agent_image                = var.rancher_agent_image
    rancher_registry                   = var.rancher_registry
    rancher_registry_username          = var.rancher_registry_username
    rancher_registry_password          = var.rancher_registry_password
    disk_device                        = {disk_device}
    disk_mount_path                    = {disk_mount}
    extra_agent_args                   = {extra}
  }})'''


RKE1_CNIS = ("calico", "flannel", "canal", "weave")


def _cluster_data() -> str:
    """S4 as a data source: find-or-create the cluster by name (RKE2 or RKE1), then its
    registration token and CA checksum (files/ensure_cluster.sh, run on the operator machine)."""
    rke2_cnis = "[" + ", ".join(f'"{c}"' for c in versions.RKE2_CNIS) + "]"
    rke1_cnis = "[" + ", ".join(f'"{c}"' for c in RKE1_CNIS) + "]"
    rke2_cni_list, rke1_cni_list = ", ".join(versions.RKE2_CNIS), ", ".join(RKE1_CNIS)
    return f'''locals {{
  # everything ensure_cluster.sh needs, passed as its JSON query
  cluster_request = merge(
    {{
      name         = var.name
      version      = var.k8s_version
      network      = var.k8s_network_provider
      distribution = var.k8s_distribution
      operation    = var.tk_operation
    }},
    {{
      api_url    = var.rancher_api_url
      access_key = var.rancher_access_key
      secret_key = var.rancher_secret_key
      ca_pem     = var.tk_rancher_ca
    }},
    {{
      registry          = var.k8s_registry
      registry_username = var.k8s_registry_username
      registry_password = var.k8s_registry_password
    }},
  )
}}

data "external" "cluster" {{
  program = ["bash", "${{path.module}}/files/ensure_cluster.sh"]
  query   = local.cluster_request
  lifecycle {{
    precondition {{
      condition     = (var.k8s_distribution == "rke2") == (length(regexall("[+]rke2r[0-9]+$", var.k8s_version)) > 0)
      error_message = "k8s_version must be a release of k8s_distribution (RKE2: vX.Y.Z+rke2rN, RKE1: vX.Y.Z-rancherN-N)."
    }}
    precondition {{
      condition     = contains(var.k8s_distribution == "rke2" ? {rke2_cnis} : {rke1_cnis}, var.k8s_network_provider)
      error_message = "k8s_network_provider is not a CNI of k8s_distribution (RKE2: {rke2_cni_list}; RKE1: {rke1_cni_list})."
    }}
  }}
}}
'''


MANAGER_FILES = {"install_docker.sh.tftpl": scripts.INSTALL_DOCKER,
                 "install_rancher_server.sh.tftpl": scripts.INSTALL_RANCHER_SERVER,
                 "setup_rancher.sh.tftpl": scripts.SETUP_RANCHER, "read_api_key.sh": scripts.READ_API_KEY}
CLUSTER_FILES = {"ensure_cluster.sh": scripts.RANCHER_CLUSTER}
HOST_FILES = {"install_rancher_agent.sh.tftpl": scripts.INSTALL_RANCHER_AGENT}


def _sg_rules(self_only: bool) -> str:
    out = []
    for lo, hi in RKE_PORTS:
        src = "self = true" if self_only else 'cidr_blocks = ["0.0.0.0/0"]'
        out.append(f"""  ingress {{
    from_port = {lo}
    to_port   = {hi}
    protocol  = "tcp"
    {src}
  }}""")
    out.append("""  ingress {
    from_port = 8472
    to_port   = 8472
    protocol  = "udp"
    self      = true
  }
  egress {
    from_port   = 0
    to_port     = 0
    protocol    = "-1"
    cidr_blocks = ["0.0.0.0/0"]
  }""")
    return "\n".join(out)


# --- module definitions ---------------------------------------------------------------------------------
def modules() -> List[Module]:
    mods: List[Module] = []

    # T1 triton-rancher
    mods.append(Module("triton-rancher", ["triton", "external"],
                       MANAGER_BASE + _rancher_image_vars() + TRITON_CREDS + [
                           Var("triton_network_names", ["Joyent-SDC-Public"], type="list(string)"),
                           Var("triton_image_name", "ubuntu-certified-22.04"), Var("triton_image_version", None),
                           Var("triton_ssh_user", "ubuntu"),
                           Var("master_triton_machine_package", sizing.default_size("triton", "manager")[1])],
                       f'''data "triton_network" "networks" {{
  count = length(var.triton_network_names)
  name  = var.triton_network_names[count.index]
}}

data "triton_image" "image" {{
  name        = var.triton_image_name
  version     = var.triton_image_version
  most_recent = true
}}

resource "triton_machine" "rancher_master" {{
  package     = var.master_triton_machine_package
  image       = data.triton_image.image.id
  name        = var.name
  user_script = {_docker_userdata(True)}
  networks    = data.triton_network.networks[*].id
  cns {{
    services = [var.name]
  }}
  affinity = ["role!=~gcm"]
  tags = {{
    role = "gcm"
  }}
}}

locals {{
  rancher_master_id = triton_machine.rancher_master.id
  rancher_master_ip = triton_machine.rancher_master.primaryip
  ssh_user          = var.triton_ssh_user
  key_path          = var.triton_key_path
  bastion_host      = ""
}}
''' + _manager_tail(_connection(), False), MANAGER_OUTPUTS, dict(MANAGER_FILES)))

    # T2 aws-rancher
    mods.append(Module("aws-rancher", ["aws", "external"],
                       MANAGER_BASE + _rancher_image_vars() + AWS_CREDS + [
                           Var("aws_vpc_cidr", "10.0.0.0/16"), Var("aws_subnet_cidr", "10.0.2.0/24"),
                           Var("aws_ami_id", None), Var("aws_instance_type", sizing.default_size("aws", "manager")[1]), Var("aws_key_name", None),
                           Var("aws_public_key_path", "~/.ssh/id_rsa.pub"), Var("aws_private_key_path", "~/.ssh/id_rsa"),
                           Var("aws_ssh_user", "ubuntu")],
                       f'''resource "aws_vpc" "default" {{
  cidr_block           = var.aws_vpc_cidr
  enable_dns_hostnames = true
  tags = {{ Name = var.name }}
}}

resource "aws_internet_gateway" "default" {{
  vpc_id = aws_vpc.default.id
}}

resource "aws_subnet" "public" {{
  vpc_id                  = aws_vpc.default.id
  cidr_block              = var.aws_subnet_cidr
  map_public_ip_on_launch = true
  depends_on              = [aws_internet_gateway.default]
  tags = {{ Name = "${{var.name}}-public" }}
}}

resource "aws_route_table" "public" {{
  vpc_id = aws_vpc.default.id
  route {{
    cidr_block = "0.0.0.0/0"
    gateway_id = aws_internet_gateway.default.id
  }}
}}

resource "aws_route_table_association" "public" {{
  subnet_id      = aws_subnet.public.id
  route_table_id = aws_route_table.public.id
}}

resource "aws_key_pair" "deployer" {{
  count      = var.aws_public_key_path != "" ? 1 : 0
  key_name   = var.aws_key_name
  public_key = file(pathexpand(var.aws_public_key_path))
}}

resource "aws_security_group" "rancher" {{
  name        = var.name
  description = "Rancher server ${{var.name}}"
  vpc_id      = aws_vpc.default.id
  dynamic "ingress" {{
    for_each = [22, 80, 443]
    content {{
      from_port   = ingress.value
      to_port     = ingress.value
      protocol    = "tcp"
      cidr_blocks = ["0.0.0.0/0"]
    }}
  }}
  egress {{
    from_port   = 0
    to_port     = 0
    protocol    = "-1"
    cidr_blocks = ["0.0.0.0/0"]
  }}
}}

resource "aws_instance" "host" {{
  ami                    = var.aws_ami_id
  instance_type          = var.aws_instance_type
  subnet_id              = aws_subnet.public.id
  vpc_security_group_ids = [aws_security_group.rancher.id]
  key_name               = var.aws_key_name
  depends_on             = [aws_key_pair.deployer]
  user_data              = {_docker_userdata(True)}
  tags = {{ Name = var.name }}
}}

locals {{
  rancher_master_id = aws_instance.host.id
  rancher_master_ip = aws_instance.host.public_ip
  ssh_user          = var.aws_ssh_user
  key_path          = var.aws_private_key_path
  bastion_host      = ""
}}
''' + _manager_tail(_connection(), False), MANAGER_OUTPUTS, dict(MANAGER_FILES)))

    # T3 gcp-rancher
    mods.append(Module("gcp-rancher", ["gcp", "external"],
                       MANAGER_BASE + _rancher_image_vars() + GCP_CREDS + [
                           Var("gcp_machine_type", sizing.default_size("gcp", "manager")[1]), Var("gcp_instance_zone", None),
                           Var("gcp_image", "ubuntu-os-cloud/ubuntu-2204-lts"), Var("gcp_ssh_user", "ubuntu"),
                           Var("gcp_public_key_path", "~/.ssh/id_rsa.pub"), Var("gcp_private_key_path", "~/.ssh/id_rsa")],
                       f'''resource "google_compute_network" "default" {{
  name                    = var.name
  auto_create_subnetworks = true
}}

resource "google_compute_firewall" "default" {{
  name    = var.name
  network = google_compute_network.default.name
  allow {{
    protocol = "tcp"
    ports    = ["22", "80", "443"]
  }}
  source_ranges = ["0.0.0.0/0"]
  target_tags   = ["${{var.name}}-rancher"]
}}

resource "google_compute_instance" "host" {{
  name         = var.name
  machine_type = var.gcp_machine_type
  zone         = var.gcp_instance_zone
  tags         = ["${{var.name}}-rancher"]
  boot_disk {{
    initialize_params {{
      image = var.gcp_image
      size  = 100
    }}
  }}
  network_interface {{
    network = google_compute_network.default.name
    access_config {{}}
  }}
  metadata = {{
    ssh-keys = "${{var.gcp_ssh_user}}:${{file(pathexpand(var.gcp_public_key_path))}}"
  }}
  metadata_startup_script = {_docker_userdata(True)}
}}

locals {{
  rancher_master_id = google_compute_instance.host.id
  rancher_master_ip = google_compute_instance.host.network_interface[0].access_config[0].nat_ip
  ssh_user          = var.gcp_ssh_user
  key_path          = var.gcp_private_key_path
  bastion_host      = ""
}}
''' + _manager_tail(_connection(), False), MANAGER_OUTPUTS, dict(MANAGER_FILES)))

    # T4 azure-rancher (NSG uses destination ports — the reference's source_port_ranges bug Q6 is fixed)
    mods.append(Module("azure-rancher", ["azure", "external"],
                       MANAGER_BASE + _rancher_image_vars() + AZURE_CREDS + AZURE_IMAGE + [
                           Var("azure_virtual_network_name", "rancher-network"),
                           Var("azure_virtual_network_address_space", "10.0.0.0/16"),
                           Var("azure_subnet_name", "rancher-subnet"), Var("azure_subnet_address_prefix", "10.0.2.0/24"),
                           Var("azurerm_network_security_group_name", "rancher-firewall"),
                           Var("azure_resource_group_name", ""), Var("azure_size", sizing.default_size("azure", "manager")[1]),
                           Var("azure_ssh_user", "ubuntu"), Var("azure_public_key_path", "~/.ssh/id_rsa.pub"),
                           Var("azure_private_key_path", "~/.ssh/id_rsa")],
                       f'''locals {{
  resource_group = var.azure_resource_group_name != "" ? var.azure_resource_group_name : "${{var.name}}-rancher"
}}

resource "azurerm_resource_group" "resource_group" {{
  name     = local.resource_group
  location = var.azure_location
}}

resource "azurerm_virtual_network" "vnet" {{
  name                = var.azure_virtual_network_name
  address_space       = [var.azure_virtual_network_address_space]
  location            = var.azure_location
  resource_group_name = azurerm_resource_group.resource_group.name
}}

resource "azurerm_subnet" "subnet" {{
  name                 = var.azure_subnet_name
  resource_group_name  = azurerm_resource_group.resource_group.name
  virtual_network_name = azurerm_virtual_network.vnet.name
  address_prefixes     = [var.azure_subnet_address_prefix]
}}

resource "azurerm_network_security_group" "rancher" {{
  name                = var.azurerm_network_security_group_name
  location            = var.azure_location
  resource_group_name = azurerm_resource_group.resource_group.name
  security_rule {{
    name                       = "rancher"
    priority                   = 1000
    direction                  = "Inbound"
    access                     = "Allow"
    protocol                   = "Tcp"
    source_port_range          = "*"
    destination_port_ranges    = ["22", "80", "443"]
    source_address_prefix      = "*"
    destination_address_prefix = "*"
  }}
}}

resource "azurerm_public_ip" "ip" {{
  name                = "${{var.name}}-ip"
  location            = var.azure_location
  resource_group_name = azurerm_resource_group.resource_group.name
  allocation_method   = "Static"
  sku                 = "Standard"
}}

resource "azurerm_network_interface" "nic" {{
  name                = "${{var.name}}-nic"
  location            = var.azure_location
  resource_group_name = azurerm_resource_group.resource_group.name
  ip_configuration {{
    name                          = "primary"
    subnet_id                     = azurerm_subnet.subnet.id
    private_ip_address_allocation = "Dynamic"
    public_ip_address_id          = azurerm_public_ip.ip.id
  }}
}}

resource "azurerm_network_interface_security_group_association" "nic" {{
  network_interface_id      = azurerm_network_interface.nic.id
  network_security_group_id = azurerm_network_security_group.rancher.id
}}

resource "azurerm_linux_virtual_machine" "host" {{
  name                  = var.name
  location              = var.azure_location
  resource_group_name   = azurerm_resource_group.resource_group.name
  size                  = var.azure_size
  admin_username        = var.azure_ssh_user
  network_interface_ids = [azurerm_network_interface.nic.id]
  custom_data           = base64encode({_docker_userdata(True)})
  admin_ssh_key {{
    username   = var.azure_ssh_user
    public_key = file(pathexpand(var.azure_public_key_path))
  }}
  os_disk {{
    caching              = "ReadWrite"
    storage_account_type = "Premium_LRS"
  }}
  source_image_reference {{
    publisher = var.azure_image_publisher
    offer     = var.azure_image_offer
    sku       = var.azure_image_sku
    version   = var.azure_image_version
  }}
}}

locals {{
  rancher_master_id = azurerm_linux_virtual_machine.host.id
  rancher_master_ip = azurerm_public_ip.ip.ip_address
  ssh_user          = var.azure_ssh_user
  key_path          = var.azure_private_key_path
  bastion_host      = ""
}}
''' + _manager_tail(_connection(), False), MANAGER_OUTPUTS, dict(MANAGER_FILES)))

    # T5 bare-metal-rancher (the bastion is honoured, fixing Q11)
    mods.append(Module("bare-metal-rancher", ["external"],
                       MANAGER_BASE + _rancher_image_vars() + [
                           Var("ssh_user", "ubuntu"), Var("host", None), Var("bastion_host", ""),
                           Var("key_path", "~/.ssh/id_rsa")] + PINNED_KEY_VARS,
                       '''locals {
  rancher_master_id = var.host
  rancher_master_ip = var.host
  ssh_user          = var.ssh_user
  key_path          = var.key_path
  bastion_host      = var.bastion_host
}
''' + _manager_tail(_connection(pinned=True), True), MANAGER_OUTPUTS, dict(MANAGER_FILES)))

    # T6 triton-rancher-k8s
    mods.append(Module("triton-rancher-k8s", ["external"], CLUSTER_BASE + TRITON_CREDS, _cluster_data(),
                       CLUSTER_OUTPUTS, dict(CLUSTER_FILES)))

    # T7 aws-rancher-k8s
    mods.append(Module("aws-rancher-k8s", ["aws", "external"], CLUSTER_BASE + AWS_CREDS + [
        Var("aws_vpc_cidr", "10.0.0.0/16"), Var("aws_subnet_cidr", "10.0.2.0/24"),
        Var("aws_public_key_path", "~/.ssh/id_rsa.pub"), Var("aws_key_name", None),
        # declared by the reference's module too (never read there): a configuration that
        # sets it on the cluster stays valid; every host module takes its own AMI
        Var("aws_ami_id", "", "Accepted for compatibility; the hosts' AMI is set per node.")],
        _cluster_data() + f'''
resource "aws_vpc" "default" {{
  cidr_block           = var.aws_vpc_cidr
  enable_dns_hostnames = true
  tags = {{ Name = var.name }}
}}

resource "aws_internet_gateway" "default" {{
  vpc_id = aws_vpc.default.id
}}

resource "aws_subnet" "public" {{
  vpc_id                  = aws_vpc.default.id
  cidr_block              = var.aws_subnet_cidr
  map_public_ip_on_launch = true
  depends_on              = [aws_internet_gateway.default]
  tags = {{ Name = "${{var.name}}-public" }}
}}

resource "aws_route_table" "public" {{
  vpc_id = aws_vpc.default.id
  route {{
    cidr_block = "0.0.0.0/0"
    gateway_id = aws_internet_gateway.default.id
  }}
}}

resource "aws_route_table_association" "public" {{
  subnet_id      = aws_subnet.public.id
  route_table_id = aws_route_table.public.id
}}

resource "aws_key_pair" "deployer" {{
  count      = var.aws_public_key_path != "" ? 1 : 0
  key_name   = var.aws_key_name
  public_key = file(pathexpand(var.aws_public_key_path))
}}

# RKE node ports (rancher.com/docs: port requirements)
resource "aws_security_group" "rke_ports" {{
  name        = var.name
  description = "Security group for rancher hosts in ${{var.name}} cluster"
  vpc_id      = aws_vpc.default.id
{_sg_rules(True)}
}}
''', CLUSTER_OUTPUTS + [("aws_subnet_id", "aws_subnet.public.id", False),
                          ("aws_security_group_id", "aws_security_group.rke_ports.id", False),
                          ("aws_key_name", "var.aws_key_name", False)], dict(CLUSTER_FILES)))

    # T8 gcp-rancher-k8s
    ports = ", ".join(f'"{lo}-{hi}"' if lo != hi else f'"{lo}"' for lo, hi in RKE_PORTS)
    mods.append(Module("gcp-rancher-k8s", ["gcp", "external"], CLUSTER_BASE + GCP_CREDS, _cluster_data() + f'''
resource "google_compute_network" "default" {{
  name                    = var.name
  auto_create_subnetworks = true
}}

resource "google_compute_firewall" "rke_ports" {{
  name    = var.name
  network = google_compute_network.default.name
  allow {{
    protocol = "tcp"
    ports    = [{ports}]
  }}
  allow {{
    protocol = "udp"
    ports    = ["8472"]
  }}
  source_tags = ["${{var.name}}-nodes"]
  target_tags = ["${{var.name}}-nodes"]
}}

resource "google_compute_firewall" "ssh" {{
  name          = "${{var.name}}-ssh"
  network       = google_compute_network.default.name
  source_ranges = ["0.0.0.0/0"]
  target_tags   = ["${{var.name}}-nodes"]
  allow {{
    protocol = "tcp"
    ports    = ["22", "80", "443", "6443"]
  }}
}}
''', CLUSTER_OUTPUTS + [("gcp_compute_network_name", "google_compute_network.default.name", False),
                          ("gcp_compute_firewall_host_tag", '"${var.name}-nodes"', False)], dict(CLUSTER_FILES)))

    # T9 azure-rancher-k8s
    mods.append(Module("azure-rancher-k8s", ["azure", "external"], CLUSTER_BASE + AZURE_CREDS + AZURE_IMAGE + [
        Var("azure_virtual_network_name", "k8s-network"), Var("azure_virtual_network_address_space", "10.0.0.0/16"),
        Var("azure_subnet_name", "k8s-subnet"), Var("azure_subnet_address_prefix", "10.0.2.0/24"),
        Var("azurerm_network_security_group_name", "k8s-firewall")], _cluster_data() + '''
resource "azurerm_resource_group" "resource_group" {
  name     = "${var.name}-k8s"
  location = var.azure_location
}

resource "azurerm_virtual_network" "vnet" {
  name                = var.azure_virtual_network_name
  address_space       = [var.azure_virtual_network_address_space]
  location            = var.azure_location
  resource_group_name = azurerm_resource_group.resource_group.name
}

resource "azurerm_subnet" "subnet" {
  name                 = var.azure_subnet_name
  resource_group_name  = azurerm_resource_group.resource_group.name
  virtual_network_name = azurerm_virtual_network.vnet.name
  address_prefixes     = [var.azure_subnet_address_prefix]
}

resource "azurerm_network_security_group" "rke_ports" {
  name                = var.azurerm_network_security_group_name
  location            = var.azure_location
  resource_group_name = azurerm_resource_group.resource_group.name
  security_rule {
    name                       = "rke-internal"
    priority                   = 1000
    direction                  = "Inbound"
    access                     = "Allow"
    protocol                   = "*"
    source_port_range          = "*"
    destination_port_ranges    = ["2376", "2379-2380", "6443", "8472", "9099", "10250-10252", "10254-10256", "30000-32767"]
    source_address_prefix      = "VirtualNetwork"
    destination_address_prefix = "*"
  }
  security_rule {
    name                       = "ssh-http"
    priority                   = 1010
    direction                  = "Inbound"
    access                     = "Allow"
    protocol                   = "Tcp"
    source_port_range          = "*"
    destination_port_ranges    = ["22", "80", "443"]
    source_address_prefix      = "*"
    destination_address_prefix = "*"
  }
}
''', CLUSTER_OUTPUTS + [("azure_resource_group_name", "azurerm_resource_group.resource_group.name", False),
                          ("azure_network_security_group_id", "azurerm_network_security_group.rke_ports.id", False),
                          ("azure_subnet_id", "azurerm_subnet.subnet.id", False)], dict(CLUSTER_FILES)))

    # T10 bare-metal-rancher-k8s
    mods.append(Module("bare-metal-rancher-k8s", ["external"], CLUSTER_BASE, _cluster_data(), CLUSTER_OUTPUTS,
                       dict(CLUSTER_FILES)))

    # T11 vsphere-rancher-k8s (data sources validate the names)
    mods.append(Module("vsphere-rancher-k8s", ["vsphere", "external"], CLUSTER_BASE + VSPHERE_CREDS + VSPHERE_NAMES,
                       _cluster_data() + '''
data "vsphere_datacenter" "dc" {
  name = var.vsphere_datacenter_name
}

data "vsphere_datastore" "datastore" {
  name          = var.vsphere_datastore_name
  datacenter_id = data.vsphere_datacenter.dc.id
}

data "vsphere_resource_pool" "pool" {
  name          = var.vsphere_resource_pool_name
  datacenter_id = data.vsphere_datacenter.dc.id
}

data "vsphere_network" "network" {
  name          = var.vsphere_network_name
  datacenter_id = data.vsphere_datacenter.dc.id
}
''', CLUSTER_OUTPUTS + [("vsphere_datacenter_name", "data.vsphere_datacenter.dc.name", False),
                          ("vsphere_datastore_name", "data.vsphere_datastore.datastore.name", False),
                          ("vsphere_resource_pool_name", "data.vsphere_resource_pool.pool.name", False),
                          ("vsphere_network_name", "data.vsphere_network.network.name", False)], dict(CLUSTER_FILES)))

    # T12 triton-rancher-k8s-host
    mods.append(Module("triton-rancher-k8s-host", ["triton"], HOST_BASE + TRITON_CREDS + [
        Var("triton_network_names", ["Joyent-SDC-Public"], type="list(string)"),
        Var("triton_image_name", "ubuntu-certified-22.04"), Var("triton_image_version", None),
        Var("triton_ssh_user", "ubuntu"), Var("triton_machine_package", sizing.default_size("triton", "host")[1])],
        ROLE_LOCAL + f'''

data "triton_network" "networks" {{
  count = length(var.triton_network_names)
  name  = var.triton_network_names[count.index]
}}

data "triton_image" "image" {{
  name        = var.triton_image_name
  version     = var.triton_image_version
  most_recent = true
}}

resource "triton_machine" "host" {{
  package     = var.triton_machine_package
  image       = data.triton_image.image.id
  name        = var.hostname
  user_script = {_agent_userdata()}
  networks    = data.triton_network.networks[*].id
  cns {{
    services = ["${{local.rancher_node_role}}.${{var.hostname}}"]
  }}
  affinity = ["role!=~${{local.rancher_node_role}}"]
  tags = {{
    role = local.rancher_node_role
  }}
}}
''', [], dict(HOST_FILES)))

    # T13 aws-rancher-k8s-host
    mods.append(Module("aws-rancher-k8s-host", ["aws"], HOST_BASE + AWS_CREDS + [
        Var("aws_ami_id", None), Var("aws_instance_type", sizing.default_size("aws", "host")[1]), Var("aws_subnet_id", None),
        Var("aws_security_group_id", None), Var("aws_key_name", None), Var("ebs_volume_device_name", ""),
        Var("ebs_volume_mount_path", ""), Var("ebs_volume_type", "gp3"), Var("ebs_volume_iops", ""),
        Var("ebs_volume_size", "")],
        ROLE_LOCAL + f'''

locals {{
  # /dev/sdX is exposed as /dev/xvdX (Xen) or as an NVMe namespace (Nitro)
  ebs_candidates = var.ebs_volume_device_name == "" ? "" : join(" ", [
    var.ebs_volume_device_name,
    replace(var.ebs_volume_device_name, "/dev/sd", "/dev/xvd"),
    "/dev/nvme1n1",
  ])
}}

resource "aws_instance" "host" {{
  ami                    = var.aws_ami_id
  instance_type          = var.aws_instance_type
  subnet_id              = var.aws_subnet_id
  vpc_security_group_ids = [var.aws_security_group_id]
  key_name               = var.aws_key_name
  user_data              = {_agent_userdata("local.ebs_candidates", "var.ebs_volume_mount_path")}
  tags = {{ Name = var.hostname }}
}}

resource "aws_ebs_volume" "volume" {{
  count             = var.ebs_volume_device_name != "" ? 1 : 0
  availability_zone = aws_instance.host.availability_zone
  type              = var.ebs_volume_type
  size              = var.ebs_volume_size == "" ? 100 : tonumber(var.ebs_volume_size)
  iops              = var.ebs_volume_iops == "" ? null : tonumber(var.ebs_volume_iops)
}}

resource "aws_volume_attachment" "volume" {{
  count        = var.ebs_volume_device_name != "" ? 1 : 0
  device_name  = var.ebs_volume_device_name
  volume_id    = aws_ebs_volume.volume[0].id
  instance_id  = aws_instance.host.id
  force_detach = true
}}
''', [], dict(HOST_FILES)))

    # T14 gcp-rancher-k8s-host (the data disk is attached: Q15 fixed)
    mods.append(Module("gcp-rancher-k8s-host", ["gcp"], HOST_BASE + GCP_CREDS + [
        Var("gcp_machine_type", sizing.default_size("gcp", "host")[1]), Var("gcp_instance_zone", None),
        Var("gcp_image", "ubuntu-os-cloud/ubuntu-2204-lts"), Var("gcp_compute_network_name", None),
        Var("gcp_compute_firewall_host_tag", None), Var("gcp_disk_type", ""), Var("gcp_disk_size", ""),
        Var("gcp_disk_mount_path", "")],
        ROLE_LOCAL + f'''

resource "google_compute_disk" "data" {{
  count = var.gcp_disk_type != "" ? 1 : 0
  name  = "${{var.hostname}}-data"
  type  = var.gcp_disk_type
  zone  = var.gcp_instance_zone
  size  = tonumber(var.gcp_disk_size)
}}

resource "google_compute_instance" "host" {{
  name         = var.hostname
  machine_type = var.gcp_machine_type
  zone         = var.gcp_instance_zone
  tags         = [var.gcp_compute_firewall_host_tag]
  boot_disk {{
    initialize_params {{
      image = var.gcp_image
      size  = 100
    }}
  }}
  dynamic "attached_disk" {{
    for_each = google_compute_disk.data
    content {{
      source      = attached_disk.value.self_link
      device_name = "data"
    }}
  }}
  network_interface {{
    network = var.gcp_compute_network_name
    access_config {{}}
  }}
  metadata_startup_script = {_agent_userdata('var.gcp_disk_type != "" ? "/dev/disk/by-id/google-data" : ""', "var.gcp_disk_mount_path")}
}}
''', [], dict(HOST_FILES)))

    # T15 azure-rancher-k8s-host
    mods.append(Module("azure-rancher-k8s-host", ["azure"], HOST_BASE + AZURE_CREDS + AZURE_IMAGE + [
        Var("azure_resource_group_name", None), Var("azure_network_security_group_id", None),
        Var("azure_subnet_id", None), Var("azure_size", sizing.default_size("azure", "host")[1]), Var("azure_ssh_user", "ubuntu"),
        Var("azure_public_key_path", "~/.ssh/id_rsa.pub"), Var("azure_disk_mount_path", ""),
        Var("azure_disk_size", "")],
        ROLE_LOCAL + f'''

resource "azurerm_public_ip" "ip" {{
  name                = "${{var.hostname}}-ip"
  location            = var.azure_location
  resource_group_name = var.azure_resource_group_name
  allocation_method   = "Static"
  sku                 = "Standard"
}}

resource "azurerm_network_interface" "nic" {{
  name                = "${{var.hostname}}-nic"
  location            = var.azure_location
  resource_group_name = var.azure_resource_group_name
  ip_configuration {{
    name                          = "primary"
    subnet_id                     = var.azure_subnet_id
    private_ip_address_allocation = "Dynamic"
    public_ip_address_id          = azurerm_public_ip.ip.id
  }}
}}

resource "azurerm_network_interface_security_group_association" "nic" {{
  network_interface_id      = azurerm_network_interface.nic.id
  network_security_group_id = var.azure_network_security_group_id
}}

resource "azurerm_linux_virtual_machine" "host" {{
  name                  = var.hostname
  location              = var.azure_location
  resource_group_name   = var.azure_resource_group_name
  size                  = var.azure_size
  admin_username        = var.azure_ssh_user
  network_interface_ids = [azurerm_network_interface.nic.id]
  custom_data           = base64encode({_agent_userdata('var.azure_disk_mount_path != "" ? "/dev/disk/azure/scsi1/lun0" : ""', "var.azure_disk_mount_path")})
  admin_ssh_key {{
    username   = var.azure_ssh_user
    public_key = file(pathexpand(var.azure_public_key_path))
  }}
  os_disk {{
    caching              = "ReadWrite"
    storage_account_type = "Premium_LRS"
  }}
  source_image_reference {{
    publisher = var.azure_image_publisher
    offer     = var.azure_image_offer
    sku       = var.azure_image_sku
    version   = var.azure_image_version
  }}
}}

resource "azurerm_managed_disk" "data" {{
  count                = var.azure_disk_mount_path != "" ? 1 : 0
  name                 = "${{var.hostname}}-data"
  location             = var.azure_location
  resource_group_name  = var.azure_resource_group_name
  storage_account_type = "Premium_LRS"
  create_option        = "Empty"
  disk_size_gb         = tonumber(var.azure_disk_size)
}}

resource "azurerm_virtual_machine_data_disk_attachment" "data" {{
  count              = var.azure_disk_mount_path != "" ? 1 : 0
  managed_disk_id    = azurerm_managed_disk.data[0].id
  virtual_machine_id = azurerm_linux_virtual_machine.host.id
  lun                = 0
  caching            = "ReadWrite"
}}
''', [], dict(HOST_FILES)))

    # T16 bare-metal-rancher-k8s-host
    mods.append(Module("bare-metal-rancher-k8s-host", [], HOST_BASE + [
        Var("ssh_user", "ubuntu"), Var("host", None), Var("bastion_host", ""), Var("key_path", "~/.ssh/id_rsa")]
        + PINNED_KEY_VARS + [NODE_CLEANUP_VAR],
        ROLE_LOCAL + f'''

resource "terraform_data" "install_rancher_agent" {{
  triggers_replace = [var.host]
{_connection("var.host", "var.ssh_user", "var.key_path", "var.bastion_host", pinned=True)}
  provisioner "remote-exec" {{
    inline = [{_agent_userdata()}]
  }}
}}
''' + _node_cleanup("install_rancher_agent"), [], dict(HOST_FILES, **{"cleanup_host.sh": cleanup_script()})))

    # T17 vsphere-rancher-k8s-host (CPU / memory are variables: Q15 fixed)
    mods.append(Module("vsphere-rancher-k8s-host", ["vsphere"], HOST_BASE + VSPHERE_CREDS + VSPHERE_NAMES + [
        Var("vsphere_template_name", None), Var("ssh_user", "ubuntu"), Var("key_path", "~/.ssh/id_rsa"),
        Var("vsphere_num_cpus", sizing.VSPHERE_DEFAULT_CPUS),
        Var("vsphere_memory_mb", sizing.default_size("vsphere", "host")[1])],
        ROLE_LOCAL + f'''

data "vsphere_datacenter" "dc" {{
  name = var.vsphere_datacenter_name
}}

data "vsphere_datastore" "datastore" {{
  name          = var.vsphere_datastore_name
  datacenter_id = data.vsphere_datacenter.dc.id
}}

data "vsphere_resource_pool" "pool" {{
  name          = var.vsphere_resource_pool_name
  datacenter_id = data.vsphere_datacenter.dc.id
}}

data "vsphere_network" "network" {{
  name          = var.vsphere_network_name
  datacenter_id = data.vsphere_datacenter.dc.id
}}

data "vsphere_virtual_machine" "template" {{
  name          = var.vsphere_template_name
  datacenter_id = data.vsphere_datacenter.dc.id
}}

resource "vsphere_virtual_machine" "vm" {{
  name             = var.hostname
  resource_pool_id = data.vsphere_resource_pool.pool.id
  datastore_id     = data.vsphere_datastore.datastore.id
  num_cpus         = tonumber(var.vsphere_num_cpus)
  memory           = tonumber(var.vsphere_memory_mb)
  guest_id         = data.vsphere_virtual_machine.template.guest_id
  network_interface {{
    network_id = data.vsphere_network.network.id
  }}
  disk {{
    label = "disk0"
    size  = data.vsphere_virtual_machine.template.disks[0].size
  }}
  clone {{
    template_uuid = data.vsphere_virtual_machine.template.id
  }}
}}

resource "terraform_data" "install_rancher_agent" {{
  triggers_replace = [vsphere_virtual_machine.vm.id]
{_connection("vsphere_virtual_machine.vm.default_ip_address", "var.ssh_user", "var.key_path", None)}
  provisioner "remote-exec" {{
    inline = [{_agent_userdata()}]
  }}
}}
''', [], dict(HOST_FILES)))

    # MI355X bare-metal host
    mods.append(Module("bare-metal-mi355x-rancher-k8s-host", ["external"], HOST_BASE + [
        Var("ssh_user", "ubuntu"), Var("host", None), Var("bastion_host", ""), Var("key_path", "~/.ssh/id_rsa"),
        Var("tk_operation", "apply"), Var("tk_known_hosts", ""), *PINNED_KEY_VARS, NODE_CLEANUP_VAR,
        Var("gpu_product", "MI355X"), Var("gpu_count", 8, "GPUs the node must expose"),
        Var("gpu_burnin", "full", "quick | full | off"),
        Var("rccl_env", {}, "RCCL / HSA environment for GPU pods", "map(string)"),
        Var("rccl_min_busbw", "0", "node-level all-reduce bus bandwidth gate (GB/s)"),
        Var("gpu_link_min_frac", "0.5",
            "fail the node when a GPU pair's peer copy bandwidth is below this fraction of the node median"),
        Var("gpu_compute_partition", "spx",
            "compute partition mode every GPU of the node must run in (spx | dpx | qpx | cpx); "
            "amd.com/gpu = gpu_count x partitions per GPU"),
        Var("gpu_memory_partition", "nps1", "memory partition mode every GPU of the node must run in (nps1 | nps2)"),
        Var("gpu_link_min_gbps", "38",
            "fail the node when a GPU pair's kernel-driven peer read is below this many GB/s (absolute floor: "
            "half of one xGMI link's ~76.8 GB/s one way)"),
        Var("gpu_host_tuning", "warn",
            "host settings check (NUMA auto-balancing off, IOMMU passthrough): warn = labels and warnings; "
            "enforce = fail the node; off = not checked"),
        Var("gpu_health", "fail",
            "GPU health policy (RAS counters): fail = an unhealthy GPU fails the node; taint = the node joins "
            "tainted amd.com/gpu-health=unhealthy:NoSchedule (no GPU pods); off = not checked"),
        Var("gpu_max_uncorrectable_ecc", "0", "uncorrectable ECC errors a GPU may have logged"),
        Var("gpu_metrics_textfile", "",
            "node_exporter textfile collector directory: write the GPU health metrics there (tk_gpu.prom) "
            "and refresh them every minute from a systemd timer (empty: off)"),
        Var("gpu_max_retired_pages", "auto",
            "retired VRAM pages a GPU may have (auto: the amdgpu driver's default threshold, one page per "
            "100 MiB of VRAM)"),
        Var("rccl_slim", "off",
            "on: build a single-target (gfx950) copy of the node's librccl for faster cold communicator init, "
            "verify it with a one-rank all-reduce, and run rccl-ready on it while it matches the installed "
            "librccl (a modified vendor binary: off by default)"),
        Var(PREBUILT_VAR, "",
            "directory of prebuilt gfx950 node tools, each with its <tool>.sha256 source stamp, that the CLI "
            "stages (node/tools.py); empty: none uploaded, the node builds the tools with hipcc")],
        ROLE_LOCAL + f'''

locals {{
  rccl_env_file = join("\\n", [for k in sort(keys(var.rccl_env)) : "${{k}}=\\"${{var.rccl_env[k]}}\\""])
  prebuilt_tools = var.{PREBUILT_VAR} != "" ? var.{PREBUILT_VAR} : "${{path.module}}/files/prebuilt"
}}

resource "terraform_data" "install_mi355x_node" {{
  triggers_replace = [var.host]
{_connection("var.host", "var.ssh_user", "var.key_path", "var.bastion_host", pinned=True)}
  provisioner "remote-exec" {{
    inline = ["sudo mkdir -p {SOURCES_DIR} {PREBUILT_DIR} && sudo chown $(id -un) {SOURCES_DIR} {PREBUILT_DIR} && rm -rf {PREBUILT_DIR}/*"]
  }}
  provisioner "file" {{
    source      = "${{path.module}}/files/src/"
    destination = "{SOURCES_DIR}"
  }}
  provisioner "file" {{
    source      = "${{local.prebuilt_tools}}/"
    destination = "{PREBUILT_DIR}"
  }}
  provisioner "remote-exec" {{
    inline = [templatefile("${{path.module}}/files/install_mi355x_node.sh.tftpl", {{
      hostname                           = var.hostname
      docker_engine_install_url          = var.docker_engine_install_url
      docker_install_sha256              = var.docker_install_sha256
      rancher_api_url                    = var.rancher_api_url
      rancher_cluster_registration_token = var.rancher_cluster_registration_token
      rancher_cluster_ca_checksum        = var.rancher_cluster_ca_checksum
      rancher_node_role                  = local.rancher_node_role
      k8s_distribution                   = var.k8s_distribution
      rancher_agent_image                = var.rancher_agent_image
      rancher_registry                   = var.rancher_registry
      rancher_registry_username          = var.rancher_registry_username
      rancher_registry_password          = var.rancher_registry_password
      gpu_count                          = tonumber(var.gpu_count)
      gpu_burnin                         = var.gpu_burnin
      rccl_env_file                      = local.rccl_env_file
      rccl_min_busbw                     = var.rccl_min_busbw
      gpu_link_min_frac                  = var.gpu_link_min_frac
      gpu_link_min_gbps                  = var.gpu_link_min_gbps
      gpu_compute_partition              = var.gpu_compute_partition
      gpu_memory_partition               = var.gpu_memory_partition
      gpu_partitions                     = lookup({{ spx = 1, dpx = 2, qpx = 4, cpx = 8 }}, var.gpu_compute_partition, 1)
      rccl_slim                          = var.rccl_slim
      gpu_health                         = var.gpu_health
      gpu_host_tuning                    = var.gpu_host_tuning
      gpu_max_uncorrectable_ecc          = var.gpu_max_uncorrectable_ecc
      gpu_max_retired_pages              = var.gpu_max_retired_pages
      gpu_metrics_textfile               = var.gpu_metrics_textfile
    }})]
  }}
}}
''' + _node_cleanup("install_mi355x_node") + f'''
data "external" "gpu_labels" {{
  depends_on = [terraform_data.install_mi355x_node]
  program    = ["bash", "${{path.module}}/files/read_gpu_labels.sh"]
  query = {{
    host         = var.host
    ssh_user     = var.ssh_user
    key_path     = var.key_path
    bastion_host = var.bastion_host
    operation    = var.tk_operation
    known_hosts  = var.tk_known_hosts
  }}
}}
''', [("gpu_node_labels", "data.external.gpu_labels.result.labels", False),
          ("tk_ssh_known_hosts", "data.external.gpu_labels.result.known_hosts", False)],
        {"install_mi355x_node.sh.tftpl": scripts.INSTALL_MI355X_NODE, "read_gpu_labels.sh": scripts.READ_REMOTE_LABELS,
         "cleanup_host.sh": cleanup_script(), "prebuilt/README": PREBUILT_README},
        {"src/tk_topo.cpp": os.path.join(CSRC, "tk_topo.cpp"),
         "src/tk_gpu_probe.hip": os.path.join(CSRC, "tk_gpu_probe.hip"),
         "src/tk_link_verdict.h": os.path.join(CSRC, "tk_link_verdict.h"),
         "src/tk_gemm_screen.hip": os.path.join(CSRC, "tk_gemm_screen.hip"),
         "src/tk_rccl_probe.hip": os.path.join(CSRC, "tk_rccl_probe.hip"),
         "src/tk_rccl_verify.h": os.path.join(CSRC, "tk_rccl_verify.h"),
         "src/tk_rccl_group.h": os.path.join(CSRC, "tk_rccl_group.h"),
         "src/tk_elf_scan.h": os.path.join(CSRC, "tk_elf_scan.h")}))

    # MI355X cluster add-ons: one template per object from k8s/addons.py (the DirectExecutor
    # renders these same files), filtered by group, then applied through Rancher's k8s proxy
    from ..k8s import addons as addon_defs

    templates = addon_defs.addon_templates()
    files = {"apply_addons.sh": scripts.APPLY_ADDONS}
    for obj in templates:
        files[f"manifests/{obj.file}.tftpl"] = addon_defs.template_text(obj)
    group_of = "\n".join(f'    {json.dumps(o.file)} = {json.dumps(o.group)}' for o in templates)
    tvars = "\n".join(f"      {v} = local.values.{v}" for v in addon_defs.TEMPLATE_VARS)
    mods.append(Module("rancher-k8s-mi355x-addons", ["external", "tls"], [
        Var("name", None), Var("rancher_api_url", None), Var("rancher_access_key", None),
        Var("rancher_secret_key", None, sensitive=True), Var("rancher_cluster_id", None),
        Var("tk_rancher_ca", "", "PEM CA bundle the Rancher server is verified against (the manager's pinned CA, "
            "rendered by the CLI; empty: a publicly trusted certificate)"),
        Var("device_plugin_image", versions.DEVICE_PLUGIN_IMAGE),
        Var("node_labeller_image", "",
            f"ROCm node labeller image, opt-in (e.g. {versions.NODE_LABELLER_IMAGE}); it writes only keys the "
            "bootstrap labeller does not. Empty: no labeller DaemonSet or its RBAC."),
        Var("rccl_probe_image", versions.RCCL_PROBE_IMAGE,
            "Image of the node-level rccl-ready Job (runs the node's installed tools)."),
        Var("webhook_image", versions.WEBHOOK_IMAGE, "Python image running the RCCL-env injector webhook."),
        Var("rccl_gate", "true", "Apply the rccl-ready Job (true/false)."),
        Var("rccl_env_injector", "true",
            "Inject the rccl-env values into every pod requesting amd.com/gpu (mutating webhook; true/false).")],
        '''locals {
  manifest_dir = "${path.root}/.tk-addons-${var.name}"
  # group of every manifest file (k8s/addons.py) and whether the group is on
  group_of = {
''' + group_of + '''
  }
  enabled = {
    base  = true
    label = var.node_labeller_image != ""
    env   = var.rccl_env_injector == "true"
    gate  = var.rccl_gate == "true"
  }
  values = {
    device_plugin_image = var.device_plugin_image
    node_labeller_image = var.node_labeller_image
    rccl_probe_image    = var.rccl_probe_image
    webhook_image       = var.webhook_image
    injector_ca_b64     = base64encode(tls_self_signed_cert.injector_ca.cert_pem)
    injector_cert_b64   = base64encode(tls_locally_signed_cert.injector.cert_pem)
    injector_key_b64    = base64encode(tls_private_key.injector.private_key_pem)
  }
  manifests = {
    for f in fileset("${path.module}/files/manifests", "*.tftpl") :
    trimsuffix(f, ".tftpl") => templatefile("${path.module}/files/manifests/${f}", {
''' + tvars + '''
    }) if local.enabled[lookup(local.group_of, trimsuffix(f, ".tftpl"), "base")]
  }
}

# serving certificate of the RCCL-env injector (the API server verifies it against caBundle)
resource "tls_private_key" "injector_ca" {
  algorithm   = "ECDSA"
  ecdsa_curve = "P256"
}

resource "tls_self_signed_cert" "injector_ca" {
  private_key_pem       = tls_private_key.injector_ca.private_key_pem
  is_ca_certificate     = true
  validity_period_hours = 87600
  allowed_uses          = ["cert_signing", "crl_signing"]
  subject {
    common_name = "rccl-env-injector-ca"
  }
}

resource "tls_private_key" "injector" {
  algorithm   = "ECDSA"
  ecdsa_curve = "P256"
}

resource "tls_cert_request" "injector" {
  private_key_pem = tls_private_key.injector.private_key_pem
  dns_names = ["rccl-env-injector", "rccl-env-injector.kube-system", "rccl-env-injector.kube-system.svc",
  "rccl-env-injector.kube-system.svc.cluster.local"]
  subject {
    common_name = "rccl-env-injector.kube-system.svc"
  }
}

resource "tls_locally_signed_cert" "injector" {
  cert_request_pem      = tls_cert_request.injector.cert_request_pem
  ca_private_key_pem    = tls_private_key.injector_ca.private_key_pem
  ca_cert_pem           = tls_self_signed_cert.injector_ca.cert_pem
  validity_period_hours = 87600
  allowed_uses          = ["digital_signature", "key_encipherment", "server_auth"]
}

resource "terraform_data" "apply_addons" {
  triggers_replace = [var.rancher_cluster_id, sha256(jsonencode(local.manifests))]
  input            = length(local.manifests)
  provisioner "local-exec" {
    command = <<-EOT
      rm -rf "${local.manifest_dir}" && mkdir -p "${local.manifest_dir}"
      %{for name, body in local.manifests~}
      printf '%s' '${replace(body, "'", "'\\\\''")}' > "${local.manifest_dir}/${name}"
      %{endfor~}
      MANIFEST_DIR="${local.manifest_dir}" bash "${path.module}/files/apply_addons.sh"
    EOT
    environment = {
      RANCHER_URL        = var.rancher_api_url
      RANCHER_ACCESS_KEY = var.rancher_access_key
      RANCHER_SECRET_KEY = var.rancher_secret_key
      RANCHER_CA         = var.tk_rancher_ca
      CLUSTER_ID         = var.rancher_cluster_id
    }
  }
}
''', [("addons_applied", "tostring(terraform_data.apply_addons.output)", False)], files))
    return mods


# ``terraform_data`` (every remote-exec / local-exec step of the modules) is new in 1.4
REQUIRED_VERSION = ">= 1.4"
MIN_TERRAFORM = (1, 4, 0)


def output_sensitivity() -> Dict[str, Dict[str, bool]]:
    """``{module: {output: sensitive}}`` straight from the module definitions — the one
    source the catalog and the executor's root-output rendering read (Terraform >= 0.15
    rejects a root output over a sensitive module output unless it is marked too)."""
    return {m.name: {name: bool(sens) for name, _, sens in m.outputs} for m in modules()}


def render_versions(mod: Module) -> str:
    req = [PROVIDERS[p][0] for p in mod.providers]
    body = "\n    ".join(req)
    block = f"  required_providers {{\n    {body}\n  }}\n" if req else ""
    return f"terraform {{\n  required_version = \"{REQUIRED_VERSION}\"\n{block}}}\n"


def render_main(mod: Module) -> str:
    provider_blocks = [PROVIDERS[p][1] for p in mod.providers if PROVIDERS[p][1]]
    head = "# Generated by triton_kubernetes_amd.terraform.generate — edit the generator, not this file.\n\n"
    return head + "\n\n".join(provider_blocks + [mod.main.strip()]) + "\n"


def render_variables(mod: Module) -> str:
    return "\n\n".join(v.hcl() for v in mod.variables) + "\n"


def render_outputs(mod: Module) -> str:
    out = []
    for name, expr, sensitive in mod.outputs:
        lines = [f'output "{name}" {{', f"  description = {json.dumps(OUTPUT_DOCS.get(name, _doc_from_name(name)))}",
                 f"  value       = {expr}"]
        if sensitive:
            lines.append("  sensitive   = true")
        lines.append("}")
        out.append("\n".join(lines))
    return ("\n\n".join(out) + "\n") if out else "# This module has no outputs.\n"


def rendered_files(mod: Module) -> Dict[str, str]:
    files = {
        "versions.tf": render_versions(mod),
        "main.tf": render_main(mod),
        "variables.tf": render_variables(mod),
        "outputs.tf": render_outputs(mod),
    }
    for name, content in mod.files.items():
        files[f"files/{name}"] = content
    for name, src in mod.copies.items():
        with open(src, "r", encoding="utf-8") as fh:
            files[f"files/{name}"] = fh.read()
    return files


def write_all(root: str = MODULES_DIR) -> List[str]:
    written = []
    if os.path.isdir(root):
        shutil.rmtree(root)
    for mod in modules():
        copies = {f"files/{name}": src for name, src in mod.copies.items()}
        for rel, content in rendered_files(mod).items():
            path = os.path.join(root, mod.name, rel)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            if rel in copies:
                # shipped sources stay single-copy: a relative symlink into the package
                # (git keeps it; module sources fetched from git resolve it)
                os.symlink(os.path.relpath(copies[rel], os.path.dirname(path)), path)
                written.append(path)
                continue
            with open(path, "w", encoding="utf-8") as fh:
                fh.write(content)
            if path.endswith(".sh"):
                os.chmod(path, 0o755)
            written.append(path)
    return written


if __name__ == "__main__":
    paths = write_all()
    print(f"wrote {len(paths)} files under {MODULES_DIR}")
    sys.exit(0)
