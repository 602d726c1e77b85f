"""Namespace backup / restore (``backup cluster``, ``restore cluster``).

The reference README advertises "backup/restore a kubernetes namespace from any of
your clusters to manta/S3" (``README.md:16``), but the CLI never implemented it
(SURVEY.md §7.5 Q12).  This implements it.

* **Backup** reads the namespaces' objects through Rancher's Kubernetes proxy. The
  objects are namespaces, configmaps, secrets, services, service accounts, PVCs,
  deployments, statefulsets, daemonsets, jobs, cronjobs and ingresses.
  Server-populated fields are stripped: uid, resourceVersion, timestamps,
  managedFields, status, allocated cluster IPs (a headless service keeps
  ``clusterIP: None``), a Job's generated selector and controller-uid labels (an API
  server refuses to create a Job that carries them). Objects owned by a controller
  are skipped, because the controller re-creates them. The result is written as one
  JSON archive either to the manager's state backend (local or Manta, the index of
  archives updated under the backend's lock) or to S3 (server-side encrypted: the
  archive holds the namespaces' Secrets).
* **Restore** creates the namespaces, then the objects, in dependency order. An
  object that already exists is replaced (PUT on 409), so a restore can be re-run.

Settings: ``cluster_manager``, ``cluster_name``, ``backup_namespaces`` (list; default:
every non-system namespace), ``backup_target`` (``state`` | ``s3``), ``backup_name``
(restore; default: the newest).  The S3 target needs ``s3_bucket``, ``aws_access_key``,
``aws_secret_key`` and ``aws_region``, plus ``s3_endpoint`` for S3-compatible stores.
"""

import copy
import json
import time
from typing import Any, Dict, List, Optional, Tuple

from ..backend.base import Backend
from ..config.context import Context
from ..errors import ConfigError, TKError
from ..executor.base import outputs_from_tfstate
from ..rancher.client import RancherClient
from ..state import MANAGER_KEY
from .select import select_cluster, select_manager

SYSTEM_NAMESPACES = {"kube-system", "kube-public", "kube-node-lease", "cattle-system", "cattle-prometheus",
                     "cattle-global-data", "cattle-fleet-system", "cattle-impersonation-system", "ingress-nginx",
                     "local", "fleet-system", "security-scan"}
# (collection path template, kind), restore order
RESOURCES: List[Tuple[str, str]] = [
    ("/api/v1/namespaces/{ns}/serviceaccounts", "ServiceAccount"),
    ("/api/v1/namespaces/{ns}/configmaps", "ConfigMap"),
    ("/api/v1/namespaces/{ns}/secrets", "Secret"),
    ("/api/v1/namespaces/{ns}/persistentvolumeclaims", "PersistentVolumeClaim"),
    ("/api/v1/namespaces/{ns}/services", "Service"),
    ("/apis/apps/v1/namespaces/{ns}/deployments", "Deployment"),
    ("/apis/apps/v1/namespaces/{ns}/statefulsets", "StatefulSet"),
    ("/apis/apps/v1/namespaces/{ns}/daemonsets", "DaemonSet"),
    ("/apis/batch/v1/namespaces/{ns}/jobs", "Job"),
    ("/apis/batch/v1/namespaces/{ns}/cronjobs", "CronJob"),
    ("/apis/networking.k8s.io/v1/namespaces/{ns}/ingresses", "Ingress"),
]
ARCHIVE_VERSION = 1
_JOB_GENERATED_LABELS = ("controller-uid", "batch.kubernetes.io/controller-uid", "job-name",
                         "batch.kubernetes.io/job-name")
_META_DROP = ("uid", "resourceVersion", "creationTimestamp", "managedFields", "selfLink", "generation",
              "deletionTimestamp", "deletionGracePeriodSeconds")


def sanitize(obj: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    """A restorable copy of ``obj``, or None when it should not be backed up."""
    meta = obj.get("metadata") or {}
    if meta.get("ownerReferences"):
        return None  # re-created by its controller
    kind = obj.get("kind", "")
    if kind == "Secret" and obj.get("type") == "kubernetes.io/service-account-token":
        return None
    if kind == "ServiceAccount" and meta.get("name") == "default":
        return None
    if kind == "ConfigMap" and meta.get("name") == "kube-root-ca.crt":
        return None
    out = copy.deepcopy(obj)
    out.pop("status", None)
    m = out.setdefault("metadata", {})
    for k in _META_DROP:
        m.pop(k, None)
    ann = m.get("annotations") or {}
    ann.pop("kubectl.kubernetes.io/last-applied-configuration", None)
    if kind == "Service":
        spec = out.get("spec") or {}
        if str(spec.get("clusterIP", "")) != "None":  # headless services stay headless
            for k in ("clusterIP", "clusterIPs"):
                spec.pop(k, None)
    if kind == "Job":
        # the API server generates selector + controller-uid labels and rejects a Job
        # that brings its own (unless manualSelector): drop them, as velero does
        spec = out.get("spec") or {}
        if not spec.get("manualSelector"):
            spec.pop("selector", None)
            labels = ((spec.get("template") or {}).get("metadata") or {}).get("labels") or {}
            for k in _JOB_GENERATED_LABELS:
                labels.pop(k, None)
    if kind == "PersistentVolumeClaim":
        (out.get("spec") or {}).pop("volumeName", None)
    return out


# --- targets -------------------------------------------------------------------------------
class StateTarget:
    """Archives next to the manager's state (``backup-<cluster>-<stamp>.json``)."""

    def __init__(self, backend: Backend, manager: str):
        self.backend, self.manager = backend, manager

    def put(self, name: str, data: bytes) -> str:
        self.backend.write_blob(self.manager, name, data)
        return f"{self.backend.kind}:{self.manager}/{name}"

    def get(self, name: str) -> bytes:
        data = self.backend.read_blob(self.manager, name)
        if data is None:
            raise TKError(f"Backup '{name}' does not exist.")
        return data

    def list(self, prefix: str) -> List[str]:
        index = self.backend.read_blob(self.manager, "backups.json")
        names = json.loads(index) if index else []
        return [n for n in names if n.startswith(prefix)]

    def record(self, name: str) -> None:
        with self.backend.lock(self.manager):  # concurrent backups must not drop each other's entry
            index = self.backend.read_blob(self.manager, "backups.json")
            names = json.loads(index) if index else []
            if name not in names:
                names.append(name)
            self.backend.write_blob(self.manager, "backups.json", json.dumps(names).encode())


class S3Target:
    def __init__(self, client, bucket: str, prefix: str):
        self.client, self.bucket, self.prefix = client, bucket, prefix.rstrip("/")

    def _key(self, name: str) -> str:
        return f"{self.prefix}/{name}" if self.prefix else name

    def put(self, name: str, data: bytes) -> str:
        self.client.put_object(self.bucket, self._key(name), data)
        return f"s3://{self.bucket}/{self._key(name)}"

    def get(self, name: str) -> bytes:
        return self.client.get_object(self.bucket, self._key(name))

    def list(self, prefix: str) -> List[str]:
        keys = self.client.list_keys(self.bucket, self._key(prefix))
        strip = len(self.prefix) + 1 if self.prefix else 0
        return [k[strip:] for k in keys]

    def record(self, name: str) -> None:
        pass


def _target(ctx: Context, backend: Backend, manager: str):
    s = ctx.settings
    kind = (s.get_string("backup_target") or "state").lower()
    if kind == "state":
        return StateTarget(backend, manager)
    if kind == "s3":
        bucket = ctx.resolve("s3_bucket", "S3 Bucket")
        factory = ctx.extras.get("s3_factory")
        if factory is not None:
            client = factory()
        else:
            from ..cloud.aws import S3Client

            client = S3Client(ctx.resolve("aws_access_key", "AWS Access Key"),
                              ctx.resolve("aws_secret_key", "AWS Secret Key"),
                              s.get_string("aws_region") or "us-east-1", s.get_string("s3_endpoint") or None)
        return S3Target(client, bucket, f"triton-kubernetes/{manager}")
    raise ConfigError(f"Unsupported backup_target '{kind}', must be 'state' or 's3'")


# --- cluster access -----------------------------------------------------------------------------
def _cluster_client(ctx: Context, backend: Backend) -> Tuple[str, str, str, RancherClient]:
    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    manager = select_manager(ctx, managers)
    state = backend.state(manager)
    clusters = state.clusters()
    if not clusters:
        raise ConfigError("No clusters.")
    name, key = select_cluster(ctx, clusters, "Cluster")
    raw = backend.read_tfstate(manager)
    mgr = outputs_from_tfstate(raw, MANAGER_KEY)
    cl = outputs_from_tfstate(raw, key)
    if not mgr.get("rancher_url") or not cl.get("rancher_cluster_id"):
        raise TKError(f"Cluster '{name}' has no Rancher outputs yet (was it applied?)")
    from ..rancher import trust

    factory = ctx.extras.get("rancher_factory") or (  # verified against the pinned CA (rancher/trust.py)
        lambda url, ak="", sk="": trust.client(backend, manager, url, ak, sk))
    client = factory(mgr["rancher_url"], mgr.get("rancher_access_key", ""), mgr.get("rancher_secret_key", ""))
    return manager, name, cl["rancher_cluster_id"], client


def _items(client: RancherClient, cid: str, path: str) -> List[Dict[str, Any]]:
    try:
        return (client.k8s(cid, "GET", path) or {}).get("items", []) or []
    except TKError as exc:
        if getattr(exc, "status", None) == 404:  # API group not served by this cluster
            return []
        raise


def backup_cluster(ctx: Context, backend: Backend) -> str:
    manager, name, cid, client = _cluster_client(ctx, backend)
    wanted = ctx.settings.get_string_slice("backup_namespaces")
    all_ns = [(o.get("metadata") or {}).get("name", "") for o in _items(client, cid, "/api/v1/namespaces")]
    if wanted:
        missing = sorted(set(wanted) - set(all_ns))
        if missing:
            raise ConfigError(f"Namespace '{missing[0]}' does not exist in cluster '{name}'.")
        namespaces = list(wanted)
    else:
        namespaces = sorted(n for n in all_ns if n and n not in SYSTEM_NAMESPACES and n != "default")
    objects: List[Dict[str, Any]] = []
    ns_objs = {(o.get("metadata") or {}).get("name"): o for o in _items(client, cid, "/api/v1/namespaces")}
    for ns in namespaces:
        ns_obj = sanitize(ns_objs.get(ns) or {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
        objects.append({"path": "/api/v1/namespaces", "object": ns_obj})
        for tmpl, kind in RESOURCES:
            path = tmpl.format(ns=ns)
            for item in _items(client, cid, path):
                item.setdefault("kind", kind)
                clean = sanitize(item)
                if clean is not None:
                    objects.append({"path": path, "object": clean})
    stamp = time.strftime("%Y%m%dT%H%M%SZ", time.gmtime())
    archive = {"version": ARCHIVE_VERSION, "manager": manager, "cluster": name, "cluster_id": cid,
               "created": stamp, "namespaces": namespaces, "objects": objects}
    fname = f"backup-{name}-{stamp}.json"
    target = _target(ctx, backend, manager)
    where = target.put(fname, json.dumps(archive, indent=1, sort_keys=True).encode())
    target.record(fname)
    ctx.echo(f"Backed up {len(objects)} objects from {len(namespaces)} namespaces of cluster '{name}' to {where}")
    return fname


def restore_cluster(ctx: Context, backend: Backend) -> int:
    manager, name, cid, client = _cluster_client(ctx, backend)
    target = _target(ctx, backend, manager)
    backup = ctx.settings.get_string("backup_name")
    if not backup:
        found = sorted(target.list(f"backup-{name}-"))
        if not found:
            raise ConfigError(f"No backups of cluster '{name}'.")
        backup = found[-1]
    archive = json.loads(target.get(backup))
    if archive.get("version") != ARCHIVE_VERSION:
        raise TKError(f"Unsupported backup version {archive.get('version')!r}")
    only = set(ctx.settings.get_string_slice("backup_namespaces"))
    from ..k8s.manifests import apply_manifests

    todo = [(e["path"], e["object"]) for e in archive.get("objects", [])
            if not only or (e["object"].get("metadata") or {}).get("namespace", e["object"]["metadata"]["name"])
            in only]
    applied = apply_manifests(client, cid, todo)
    ctx.echo(f"Restored {len(applied)} objects from {backup} into cluster '{name}'")
    return len(applied)


__all__ = ["backup_cluster", "restore_cluster", "sanitize", "RESOURCES", "SYSTEM_NAMESPACES"]
