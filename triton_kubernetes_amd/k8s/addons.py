"""MI355X cluster add-ons: ONE definition, rendered by both delivery paths.

The ``rancher-k8s-mi355x-addons`` Terraform module ships one ``templatefile``
per object (``files/manifests/NN-<name>.json.tftpl``, written by
``terraform/generate.py`` from :func:`addon_templates`) and the DirectExecutor
renders *those same files* (:func:`rendered_addons`), so the two paths apply the
same objects by construction (``tests/test_addons.py`` pins it).

Objects, in apply order:

=====  ====================  ===================================================
group  objects               what
=====  ====================  ===================================================
base   DaemonSet             ROCm device plugin (advertises ``amd.com/gpu``)
base   ConfigMap             ``rccl-env``: cluster RCCL/HSA environment
label  SA/ClusterRole/Bind.  RBAC the node labeller needs to patch node labels
label  DaemonSet             ROCm node labeller, opt-in (``node_labeller_image``):
                             simd count, driver version, partitioning support
env    Secret/ConfigMap/     the RCCL-env injector: a mutating admission webhook
       Deployment/Service/   (``k8s/webhook.py``) that gives every pod requesting
       MutatingWebhookConf.  ``amd.com/gpu`` the ``rccl-env`` values and the node's
                             ``/etc/rccl`` (north star: "RCCL env injected")
gate   Job                   node-level ``rccl-ready`` on an MI355X node
=====  ====================  ===================================================

Template variables (all plain strings; certificate material is base64 so it can sit
inside JSON strings): :data:`TEMPLATE_VARS`.
"""

import base64
import json
import os
import re
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

from .. import versions
from ..parallel.rccl_env import default_rccl_env
from . import webhook
from .manifests import (GPU_SELECTOR, LABELLER_NAME, NAMESPACE, device_plugin_daemonset, gpu_job_manifest,
                        labeller_daemonset, rccl_configmap)

MODULE = "rancher-k8s-mi355x-addons"
INJECTOR = "rccl-env-injector"
TEMPLATE_VARS = ("device_plugin_image", "node_labeller_image", "rccl_probe_image", "webhook_image",
                 "injector_ca_b64", "injector_cert_b64", "injector_key_b64")
# group -> module variable that enables it ("" = always on)
GROUPS = {"base": "", "label": "node_labeller_image", "env": "rccl_env_injector", "gate": "rccl_gate"}


@dataclass
class AddonObject:
    file: str  # "10-device-plugin.json" (the module's files/manifests/<file>.tftpl)
    group: str
    path: str  # API collection path the object is POSTed to
    obj: Dict[str, Any]


def _v(name: str) -> str:
    return "${" + name + "}"


def _labeller_rbac() -> List[Tuple[str, str, Dict[str, Any]]]:
    sa = {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": LABELLER_NAME, "namespace": NAMESPACE}}
    role = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole", "metadata": {"name": LABELLER_NAME},
            "rules": [{"apiGroups": [""], "resources": ["nodes"], "verbs": ["get", "list", "watch", "patch", "update"]}]}
    bind = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
            "metadata": {"name": LABELLER_NAME},
            "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": LABELLER_NAME},
            "subjects": [{"kind": "ServiceAccount", "name": LABELLER_NAME, "namespace": NAMESPACE}]}
    return [("21-labeller-sa.json", f"/api/v1/namespaces/{NAMESPACE}/serviceaccounts", sa),
            ("22-labeller-clusterrole.json", "/apis/rbac.authorization.k8s.io/v1/clusterroles", role),
            ("23-labeller-clusterrolebinding.json", "/apis/rbac.authorization.k8s.io/v1/clusterrolebindings", bind)]


def webhook_source() -> str:
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "webhook.py"), "r", encoding="utf-8") as fh:
        return fh.read()


def _injector() -> List[Tuple[str, str, Dict[str, Any]]]:
    labels = {"app": INJECTOR}
    secret = {"apiVersion": "v1", "kind": "Secret", "type": "kubernetes.io/tls",
              "metadata": {"name": f"{INJECTOR}-tls", "namespace": NAMESPACE},
              "data": {"tls.crt": _v("injector_cert_b64"), "tls.key": _v("injector_key_b64")}}
    src = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": f"{INJECTOR}-src", "namespace": NAMESPACE},
           "data": {"webhook.py": webhook_source()}}
    deploy = {
        "apiVersion": "apps/v1", "kind": "Deployment",
        "metadata": {"name": INJECTOR, "namespace": NAMESPACE, "labels": dict(labels)},
        "spec": {
            "replicas": 2, "selector": {"matchLabels": dict(labels)},
            "template": {
                "metadata": {"labels": dict(labels)},
                "spec": {
                    "priorityClassName": "system-cluster-critical",
                    "tolerations": [{"key": "CriticalAddonsOnly", "operator": "Exists"},
                                    {"key": "node-role.kubernetes.io/controlplane", "operator": "Exists"}],
                    "containers": [{
                        "name": "injector", "image": _v("webhook_image"),
                        "command": ["python3", "/app/webhook.py", "--port", "8443", "--cert", "/tls/tls.crt",
                                    "--key", "/tls/tls.key", "--env-dir", "/etc/rccl-env"],
                        "ports": [{"containerPort": 8443, "name": "https"}],
                        "readinessProbe": {"httpGet": {"path": "/healthz", "port": 8443, "scheme": "HTTPS"}},
                        "securityContext": {"runAsNonRoot": True, "runAsUser": 65534,
                                            "allowPrivilegeEscalation": False, "readOnlyRootFilesystem": True,
                                            "capabilities": {"drop": ["ALL"]}},
                        "resources": {"requests": {"cpu": "10m", "memory": "32Mi"},
                                      "limits": {"memory": "128Mi"}},
                        "volumeMounts": [{"name": "tls", "mountPath": "/tls", "readOnly": True},
                                         {"name": "src", "mountPath": "/app", "readOnly": True},
                                         {"name": "env", "mountPath": "/etc/rccl-env", "readOnly": True}],
                    }],
                    "volumes": [{"name": "tls", "secret": {"secretName": f"{INJECTOR}-tls"}},
                                {"name": "src", "configMap": {"name": f"{INJECTOR}-src"}},
                                {"name": "env", "configMap": {"name": "rccl-env"}}],
                },
            },
        },
    }
    svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": INJECTOR, "namespace": NAMESPACE},
           "spec": {"selector": dict(labels), "ports": [{"port": 443, "targetPort": 8443, "name": "https"}]}}
    never_own = {"key": "kubernetes.io/metadata.name", "operator": "NotIn", "values": [NAMESPACE]}
    opted_in = {"key": webhook.NODE_ENV_OPT_IN, "operator": "In", "values": ["true"]}
    not_opted_in = dict(opted_in, operator="NotIn")
    privileged = {"key": webhook.PSA_LABEL, "operator": "In", "values": ["privileged"]}
    not_privileged = dict(privileged, operator="NotIn")

    def entry(name: str, path: str, *select: Dict[str, Any]) -> Dict[str, Any]:
        return {
            "name": name,
            "clientConfig": {"service": {"name": INJECTOR, "namespace": NAMESPACE, "path": path, "port": 443},
                             "caBundle": _v("injector_ca_b64")},
            "rules": [{"operations": ["CREATE"], "apiGroups": [""], "apiVersions": ["v1"], "resources": ["pods"],
                       "scope": "Namespaced"}],
            # never the injector's own namespace (its pods must start without it)
            "namespaceSelector": {"matchExpressions": [dict(never_own)] + [dict(e) for e in select]},
            "failurePolicy": "Ignore", "sideEffects": "None", "admissionReviewVersions": ["v1"],
            "timeoutSeconds": 5, "reinvocationPolicy": "IfNeeded",
        }

    # Pod Security Admission runs after mutation, its baseline/restricted levels forbid
    # hostPath, and a cluster-wide default level applies to namespaces without a label: the
    # node's /etc/rccl mount goes only to namespaces that opt in (the rccl-node-env label, or
    # an explicit privileged enforce label); every other namespace gets the env without it.
    # (matchExpressions are ANDed: one entry per alternative, disjoint by construction.)
    hook = {
        "apiVersion": "admissionregistration.k8s.io/v1", "kind": "MutatingWebhookConfiguration",
        "metadata": {"name": INJECTOR},
        "webhooks": [entry("rccl-env-node.amd.com", "/mutate", opted_in),
                     entry("rccl-env-privileged.amd.com", "/mutate", privileged, not_opted_in),
                     entry("rccl-env.amd.com", "/mutate?node-env=omit", not_privileged, not_opted_in)],
    }
    return [("40-injector-tls.json", f"/api/v1/namespaces/{NAMESPACE}/secrets", secret),
            ("41-injector-src.json", f"/api/v1/namespaces/{NAMESPACE}/configmaps", src),
            ("42-injector-deployment.json", f"/apis/apps/v1/namespaces/{NAMESPACE}/deployments", deploy),
            ("43-injector-service.json", f"/api/v1/namespaces/{NAMESPACE}/services", svc),
            ("44-injector-webhook.json", "/apis/admissionregistration.k8s.io/v1/mutatingwebhookconfigurations", hook)]


def rccl_ready_job() -> Dict[str, Any]:
    """Node-level ``rccl-ready`` (all GPUs of one node) with the node's installed tools."""
    job = gpu_job_manifest("rccl-ready", _v("rccl_probe_image"), ["/opt/triton-kubernetes/bin/rccl-ready"],
                           namespace="default", host_paths={"/opt/triton-kubernetes": "/opt/triton-kubernetes",
                                                            "/opt/rocm": "/opt/rocm"})
    job["spec"]["template"]["spec"]["containers"][0]["env"] = [{"name": "LD_LIBRARY_PATH", "value": "/opt/rocm/lib"}]
    return job


def addon_templates() -> List[AddonObject]:
    """Every add-on object with ``${var}`` placeholders, in apply order."""
    out = [AddonObject("10-device-plugin.json", "base", f"/apis/apps/v1/namespaces/{NAMESPACE}/daemonsets",
                       device_plugin_daemonset(_v("device_plugin_image"))),
           AddonObject("20-rccl-env.json", "base", f"/api/v1/namespaces/{NAMESPACE}/configmaps",
                       rccl_configmap(default_rccl_env()))]
    out += [AddonObject(f, "label", p, o) for f, p, o in _labeller_rbac()]
    out.append(AddonObject("30-node-labeller.json", "label", f"/apis/apps/v1/namespaces/{NAMESPACE}/daemonsets",
                           labeller_daemonset(_v("node_labeller_image"))))
    out += [AddonObject(f, "env", p, o) for f, p, o in _injector()]
    out.append(AddonObject("50-rccl-ready-job.json", "gate", "/apis/batch/v1/namespaces/default/jobs",
                           rccl_ready_job()))
    return out


# --- templatefile subset ---------------------------------------------------------------------------------
_VAR_RE = re.compile(r"\$\{([A-Za-z_][A-Za-z0-9_]*)\}")


def escape_literal(text: str) -> str:
    """Literal text -> templatefile source (``${`` / ``%{`` become ``$${`` / ``%%{``)."""
    return text.replace("${", "$${").replace("%{", "%%{")


def template_text(obj: AddonObject) -> str:
    """The ``.tftpl`` file body: {"path", "object"} JSON; placeholders stay live, literal
    ``${``/``%{`` elsewhere are escaped."""
    text = json.dumps({"path": obj.path, "object": obj.obj}, indent=2)
    # escape everything, then re-enable exactly the module's variables
    text = escape_literal(text)
    for name in TEMPLATE_VARS:
        text = text.replace("$${" + name + "}", "${" + name + "}")
    return text


def render_template(text: str, values: Dict[str, str]) -> str:
    """Terraform ``templatefile`` for these files: ``${name}`` interpolation and the two
    escapes.  Unknown names raise (as Terraform does)."""
    def sub(m: "re.Match[str]") -> str:
        name = m.group(1)
        if name not in values:
            raise KeyError(f"template variable {name!r} not set")
        return str(values[name])

    parts = re.split(r"(\$\$\{|%%\{)", text)
    out = []
    for p in parts:
        if p == "$${":
            out.append("${")
        elif p == "%%{":
            out.append("%{")
        else:
            out.append(_VAR_RE.sub(sub, p))
    return "".join(out)


def module_files_dir() -> str:
    from ..terraform.catalog import MODULES_DIR

    return os.path.join(MODULES_DIR, MODULE, "files", "manifests")


def enabled(group: str, cfg: Dict[str, Any]) -> bool:
    var = GROUPS[group]
    if not var:
        return True
    v = cfg.get(var)
    if var.endswith("_image"):
        return bool(v)
    return str(v if v is not None else "true").lower() == "true"


def addon_values(cfg: Dict[str, Any], cert: Optional[Any] = None) -> Dict[str, str]:
    """Template values from the add-on module's inputs (module defaults for unset ones)."""
    def b64(s: str) -> str:
        return base64.b64encode(s.encode()).decode()

    return {
        "device_plugin_image": cfg.get("device_plugin_image") or versions.DEVICE_PLUGIN_IMAGE,
        "node_labeller_image": cfg.get("node_labeller_image") or "",
        "rccl_probe_image": cfg.get("rccl_probe_image") or versions.RCCL_PROBE_IMAGE,
        "webhook_image": cfg.get("webhook_image") or versions.WEBHOOK_IMAGE,
        "injector_ca_b64": b64(cert.ca_pem) if cert else "",
        "injector_cert_b64": b64(cert.cert_pem) if cert else "",
        "injector_key_b64": b64(cert.key_pem) if cert else "",
    }


def module_cfg_defaults(cfg: Dict[str, Any]) -> Dict[str, Any]:
    """The module's variable defaults applied to a document entry (what Terraform sees)."""
    out = {"node_labeller_image": "", "rccl_env_injector": "true", "rccl_gate": "true"}
    out.update({k: v for k, v in cfg.items() if v is not None})
    return out


def rendered_addons(cfg: Dict[str, Any], cert: Optional[Any] = None,
                    files_dir: Optional[str] = None) -> List[Tuple[str, Dict[str, Any]]]:
    """``(collection path, object)`` in apply order: the module's own ``.tftpl`` files,
    filtered by group and rendered -- exactly what the Terraform module applies."""
    cfg = module_cfg_defaults(cfg)
    groups = {o.file: o.group for o in addon_templates()}
    d = files_dir or module_files_dir()
    values = addon_values(cfg, cert)
    out = []
    for fname in sorted(os.listdir(d)):
        if not fname.endswith(".json.tftpl"):
            continue
        name = fname[: -len(".tftpl")]
        if not enabled(groups.get(name, "base"), cfg):
            continue
        with open(os.path.join(d, fname), "r", encoding="utf-8") as fh:
            doc = json.loads(render_template(fh.read(), values))
        out.append((doc["path"], doc["object"]))
    return out


__all__ = ["AddonObject", "addon_templates", "template_text", "render_template", "rendered_addons", "addon_values",
           "enabled", "GROUPS", "TEMPLATE_VARS", "INJECTOR", "MODULE", "webhook_source", "module_cfg_defaults",
           "GPU_SELECTOR"]
