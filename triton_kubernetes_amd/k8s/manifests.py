"""Kubernetes manifests for MI355X clusters + applying them through Rancher.

* ROCm device plugin DaemonSet (advertises ``amd.com/gpu``), scheduled on nodes
  labelled ``amd.com/gpu.present=true`` by the bootstrap labeller;
* ROCm node-labeller DaemonSet (opt-in, ``node_labeller_image``): only the keys the
  bootstrap labeller does not write (:data:`ROCM_LABELLER_ARGS`);
* ``rccl-env`` ConfigMap carrying the RCCL/HSA environment for GPU pods (the
  injector webhook, ``webhook.py``, puts it into every pod requesting ``amd.com/gpu``);
* :func:`gpu_job_manifest` — an example/utility Job that requests all 8 GPUs
  of one xGMI hive (node affinity on ``amd.com/xgmi.fully-connected`` and the
  GPU count) and, for multi-node jobs, pod affinity on ``amd.com/xgmi.hive-id``
  so ranks land inside one hive; the RCCL readiness Job (N2) is built with it.
"""

from typing import Any, Dict, List, Optional, Tuple

from ..errors import TKError
from ..parallel.rccl_env import default_rccl_env

NAMESPACE = "kube-system"
DEVICE_PLUGIN_NAME = "amdgpu-device-plugin"
LABELLER_NAME = "amdgpu-node-labeller"
GPU_SELECTOR = {"amd.com/gpu.present": "true"}
# The ROCm labeller's keys that ``amdgpu-topo-labeller`` does not write.  Its product-name,
# family, device-id, cu-count and vram keys are ours too, in other value formats (its
# product name is the marketing string, ours "MI355X"); both writing one key would flip
# the label on every reconcile, and the bootstrap labeller's values are the ones node
# selectors and the readiness waiter use.
ROCM_LABELLER_ARGS = ("-simd-count", "-driver-version", "-compute-partitioning-supported",
                      "-memory-partitioning-supported")


def device_plugin_daemonset(image: str) -> Dict[str, Any]:
    return {
        "apiVersion": "apps/v1", "kind": "DaemonSet",
        "metadata": {"name": DEVICE_PLUGIN_NAME, "namespace": NAMESPACE},
        "spec": {
            "selector": {"matchLabels": {"name": DEVICE_PLUGIN_NAME}},
            "template": {
                "metadata": {"labels": {"name": DEVICE_PLUGIN_NAME}},
                "spec": {
                    "nodeSelector": dict(GPU_SELECTOR),
                    "priorityClassName": "system-node-critical",
                    "tolerations": [{"key": "CriticalAddonsOnly", "operator": "Exists"},
                                    {"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}],
                    "containers": [{
                        "name": "device-plugin", "image": image,
                        "securityContext": {"allowPrivilegeEscalation": False,
                                            "capabilities": {"drop": ["ALL"]}},
                        "volumeMounts": [{"name": "dp", "mountPath": "/var/lib/kubelet/device-plugins"},
                                         {"name": "sys", "mountPath": "/sys"}],
                    }],
                    "volumes": [{"name": "dp", "hostPath": {"path": "/var/lib/kubelet/device-plugins"}},
                                {"name": "sys", "hostPath": {"path": "/sys"}}],
                },
            },
        },
    }


def labeller_daemonset(image: str) -> Dict[str, Any]:
    return {
        "apiVersion": "apps/v1", "kind": "DaemonSet",
        "metadata": {"name": LABELLER_NAME, "namespace": NAMESPACE},
        "spec": {
            "selector": {"matchLabels": {"name": LABELLER_NAME}},
            "template": {
                "metadata": {"labels": {"name": LABELLER_NAME}},
                "spec": {
                    "nodeSelector": dict(GPU_SELECTOR),
                    "serviceAccountName": LABELLER_NAME,
                    "containers": [{
                        "name": "labeller", "image": image,
                        "args": list(ROCM_LABELLER_ARGS),
                        "env": [{"name": "DS_NODE_NAME", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}}],
                        "securityContext": {"privileged": True},
                        "volumeMounts": [{"name": "sys", "mountPath": "/sys"}, {"name": "dev", "mountPath": "/dev"}],
                    }],
                    "volumes": [{"name": "sys", "hostPath": {"path": "/sys"}},
                                {"name": "dev", "hostPath": {"path": "/dev"}}],
                },
            },
        },
    }


def rccl_configmap(env: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
    return {"apiVersion": "v1", "kind": "ConfigMap",
            "metadata": {"name": "rccl-env", "namespace": NAMESPACE},
            "data": dict(env or default_rccl_env())}


# sources the node's /etc/rccl/rccl.env (if any) over the ConfigMap env, then execs the command
NODE_ENV_WRAPPER = 'set -a; [ -r /etc/rccl/rccl.env ] && . /etc/rccl/rccl.env; set +a; exec "$0" "$@"'


def gpu_job_manifest(name: str, image: str, command: List[str], gpus_per_pod: int = 8, pods: int = 1,
                     namespace: str = "default", hive_affinity: bool = True,
                     host_paths: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
    """A Job whose pods each take ``gpus_per_pod`` GPUs of one fully connected xGMI hive.
    ``host_paths`` maps node directories to container mount points (read-only)."""
    node_terms = [{"matchExpressions": [
        {"key": "amd.com/gpu.present", "operator": "In", "values": ["true"]},
        {"key": "amd.com/gpu.count", "operator": "In", "values": [str(gpus_per_pod)]},
    ]}]
    if gpus_per_pod > 1:
        node_terms[0]["matchExpressions"].append(
            {"key": "amd.com/xgmi.fully-connected", "operator": "In", "values": ["true"]})
    affinity: Dict[str, Any] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": node_terms}}}
    if hive_affinity and pods > 1:
        affinity["podAffinity"] = {"preferredDuringSchedulingIgnoredDuringExecution": [{
            "weight": 100,
            "podAffinityTerm": {"labelSelector": {"matchLabels": {"job-name": name}},
                                "topologyKey": "amd.com/xgmi.hive-id"}}]}
    mounts = [{"name": "rccl-env", "mountPath": "/etc/rccl", "readOnly": True}]
    volumes = [{"name": "rccl-env", "hostPath": {"path": "/etc/rccl", "type": "DirectoryOrCreate"}}]
    for i, (host, target) in enumerate(sorted((host_paths or {}).items())):
        mounts.append({"name": f"host-{i}", "mountPath": target, "readOnly": True})
        volumes.append({"name": f"host-{i}", "hostPath": {"path": host, "type": "Directory"}})
    return {
        "apiVersion": "batch/v1", "kind": "Job",
        "metadata": {"name": name, "namespace": namespace},
        "spec": {
            "parallelism": pods, "completions": pods, "backoffLimit": 0,
            "template": {
                "metadata": {"labels": {"job-name": name}},
                "spec": {
                    "restartPolicy": "Never",
                    "affinity": affinity,
                    "containers": [{
                        "name": "main", "image": image,
                        # cluster defaults come from the ConfigMap; the node's own file (its
                        # discovered RDMA ports, per-node overrides) is sourced on top
                        "command": ["/bin/sh", "-c", NODE_ENV_WRAPPER, command[0]] + list(command[1:]),
                        "envFrom": [{"configMapRef": {"name": "rccl-env"}}],
                        "resources": {"limits": {"amd.com/gpu": str(gpus_per_pod)}},
                        "securityContext": {"capabilities": {"add": ["SYS_PTRACE"]}},
                        "volumeMounts": mounts,
                    }],
                    "volumes": volumes,
                    "hostIPC": True,
                },
            },
        },
    }


def addon_manifests(cfg: Dict[str, Any], cert: Any = None) -> List[Tuple[str, Dict[str, Any]]]:
    """``(api collection path, object)`` pairs of the MI355X add-on module, rendered from the
    module's own template files (``k8s/addons.py``; the single source both paths share).
    Without ``cert`` the injector's certificate fields are empty (dry runs, tests)."""
    from .addons import rendered_addons

    return rendered_addons(cfg, cert)


def apply_manifests(client, cluster_id: str, manifests: List[Tuple[str, Dict[str, Any]]]) -> List[str]:
    """Create each object (PUT on 409 AlreadyExists) through Rancher's k8s proxy."""
    applied = []
    for path, obj in manifests:
        name = obj["metadata"]["name"]
        try:
            client.k8s(cluster_id, "POST", path, obj, ok=(200, 201, 202))
        except TKError as exc:
            if getattr(exc, "status", None) == 409:
                client.k8s(cluster_id, "PUT", f"{path}/{name}", obj, ok=(200, 201))
            else:
                raise
        applied.append(f"{obj['kind']}/{name}")
    return applied
