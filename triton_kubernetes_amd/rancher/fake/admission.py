"""Admission of the fake Rancher's downstream API servers: what a Pod create goes through.

In the order a real kube-apiserver runs them:

1. **mutating admission webhooks** -- every applied ``MutatingWebhookConfiguration`` whose
   rules match a Pod CREATE and whose ``namespaceSelector`` matches the namespace's labels
   (``matchLabels`` and every ``matchExpressions`` entry ANDed) is called over HTTPS.  The
   certificate is verified against the entry's ``caBundle`` for
   ``<service>.<namespace>.svc`` (``FakeRancher.service_endpoints`` maps the service to where
   a test's webhook really listens) and the returned JSONPatch is applied.  An unreachable
   or failing webhook rejects the create under ``failurePolicy: Fail`` (the default) and is
   skipped under ``Ignore``; ``allowed: false`` rejects it;
2. **Pod Security Admission** -- after mutation, the namespace's
   ``pod-security.kubernetes.io/enforce`` label (else the cluster default,
   ``FakeRancher.default_pod_security``) decides: ``baseline`` refuses host namespaces,
   privileged containers, capabilities beyond the default set, hostPath volumes and host
   ports; ``restricted`` also requires ``runAsNonRoot``, ``allowPrivilegeEscalation: false``,
   dropping ``ALL`` capabilities, a RuntimeDefault/Localhost seccomp profile and only the
   restricted volume types.

Refusals, as the API server words them: webhook failure/denial -> 400 ``BadRequest``; a
Pod Security violation -> 403 ``Forbidden`` ``violates PodSecurity "<level>:latest"``.
Negative tests: ``tests/test_fake_rancher_contract.py`` (``test_admission_*``).
"""

import base64
import http.client
import json
import socket
import ssl
import urllib.parse
import uuid
from typing import Any, Dict, List, Optional, Tuple

PSA_ENFORCE = "pod-security.kubernetes.io/enforce"
PSA_LEVELS = ("privileged", "baseline", "restricted")
_BASELINE_CAPS = {"AUDIT_WRITE", "CHOWN", "DAC_OVERRIDE", "FOWNER", "FSETID", "KILL", "MKNOD", "NET_BIND_SERVICE",
                  "SETFCAP", "SETGID", "SETPCAP", "SETUID", "SYS_CHROOT"}
_RESTRICTED_VOLUMES = {"configMap", "csi", "downwardAPI", "emptyDir", "ephemeral", "persistentVolumeClaim",
                       "projected", "secret"}
WEBHOOK_CONFIGS = "/apis/admissionregistration.k8s.io/v1/mutatingwebhookconfigurations"


class Rejected(Exception):
    """A mutating webhook refused the object (or failed under ``failurePolicy: Fail``)."""


def pod_security_violations(pod: Dict[str, Any], level: str) -> List[str]:
    """Pod Security Standards checks (the subset a GPU workload meets) for ``level``:
    ``privileged`` allows everything, ``baseline`` and ``restricted`` as documented."""
    if level not in ("baseline", "restricted"):
        return []
    spec = pod.get("spec") or {}
    containers = list(spec.get("initContainers") or []) + list(spec.get("containers") or [])
    out: List[str] = []
    for f in ("hostNetwork", "hostPID", "hostIPC"):
        if spec.get(f):
            out.append(f"host namespaces ({f}=true)")
    host_path = [v.get("name") for v in spec.get("volumes") or [] if "hostPath" in v]
    if host_path:
        out.append("hostPath volumes (" + ", ".join(f'volume "{n}"' for n in host_path) + ")")
    for c in containers:
        sc = c.get("securityContext") or {}
        if sc.get("privileged"):
            out.append(f'privileged (container "{c.get("name")}")')
        added = set(((sc.get("capabilities") or {}).get("add")) or [])
        if added - _BASELINE_CAPS:
            out.append(f'non-default capabilities (container "{c.get("name")}")')
        if any(p.get("hostPort") for p in c.get("ports") or []):
            out.append(f'hostPort (container "{c.get("name")}")')
    if level == "restricted":
        psc = spec.get("securityContext") or {}
        bad_vol = [v.get("name") for v in spec.get("volumes") or []
                   if not (set(v) - {"name"}) & _RESTRICTED_VOLUMES]
        if bad_vol:
            out.append("restricted volume types (" + ", ".join(f'volume "{n}"' for n in bad_vol) + ")")
        for c in containers:
            sc = c.get("securityContext") or {}
            name = c.get("name")
            if sc.get("allowPrivilegeEscalation") is not False:
                out.append(f'allowPrivilegeEscalation != false (container "{name}")')
            if "ALL" not in (((sc.get("capabilities") or {}).get("drop")) or []):
                out.append(f'unrestricted capabilities (container "{name}" must drop ALL)')
            if not (sc.get("runAsNonRoot", psc.get("runAsNonRoot"))):
                out.append(f'runAsNonRoot != true (container "{name}")')
            prof = (sc.get("seccompProfile") or psc.get("seccompProfile") or {}).get("type")
            if prof not in ("RuntimeDefault", "Localhost"):
                out.append(f'seccompProfile (container "{name}" must be RuntimeDefault or Localhost)')
    return out


def namespace_selected(selector: Dict[str, Any], labels: Dict[str, str]) -> bool:
    """A webhook's ``namespaceSelector`` against the namespace's labels (all terms ANDed)."""
    for k, v in (selector.get("matchLabels") or {}).items():
        if labels.get(k) != v:
            return False
    for e in selector.get("matchExpressions") or []:
        have = labels.get(e.get("key"))
        op, vals = e.get("operator"), e.get("values") or []
        if (op == "In" and have not in vals) or (op == "NotIn" and have in vals) \
                or (op == "Exists" and have is None) or (op == "DoesNotExist" and have is not None):
            return False
    return True


def rule_matches_pod_create(rule: Dict[str, Any]) -> bool:
    def has(key: str, want: str) -> bool:
        vals = rule.get(key) or []
        return "*" in vals or want in vals

    return has("operations", "CREATE") and has("apiGroups", "") and has("apiVersions", "v1") \
        and has("resources", "pods")


def call_webhook(endpoints: Dict[str, str], hook: Dict[str, Any], review: Dict[str, Any]) -> Dict[str, Any]:
    """POST the AdmissionReview to the webhook's service over verified TLS."""
    cc = hook.get("clientConfig") or {}
    svc = cc.get("service") or {}
    base = endpoints.get(f"{svc.get('name')}.{svc.get('namespace')}")
    if base is None:
        raise ConnectionError(f"service {svc.get('name')}.{svc.get('namespace')} has no endpoints")
    u = urllib.parse.urlsplit(base)
    ctx = ssl.create_default_context(cadata=base64.b64decode(cc.get("caBundle", "")).decode())
    raw = socket.create_connection((u.hostname, u.port), timeout=float(hook.get("timeoutSeconds", 10)))
    conn = http.client.HTTPConnection(u.hostname, u.port)
    conn.sock = ctx.wrap_socket(raw, server_hostname=f"{svc['name']}.{svc['namespace']}.svc")
    try:
        data = json.dumps(review).encode()
        conn.request("POST", svc.get("path", "/"), body=data, headers={"Content-Type": "application/json"})
        resp = conn.getresponse()
        out = resp.read()
        if resp.status != 200:
            raise ConnectionError(f"webhook HTTP {resp.status}")
        return json.loads(out)
    finally:
        conn.close()


def mutate_pod(fake, cid: str, namespace: str, pod: Dict[str, Any]) -> Dict[str, Any]:
    """Run the matching mutating webhooks over ``pod`` (raises :class:`Rejected`)."""
    from ...k8s.webhook import apply_patch

    st = fake.state
    prefix = f"{cid}|{WEBHOOK_CONFIGS}|"
    with st.mu:
        configs = [st.objects[k] for k in st.cluster_objects.get(cid, ()) if k.startswith(prefix)]
    labels = fake.namespace_labels(cid, namespace)
    for cfg in configs:
        for hook in cfg.get("webhooks") or []:
            if not any(rule_matches_pod_create(r) for r in hook.get("rules") or []):
                continue
            if not namespace_selected(hook.get("namespaceSelector") or {}, labels):
                continue
            review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                      "request": {"uid": str(uuid.uuid4()), "kind": {"group": "", "version": "v1", "kind": "Pod"},
                                  "operation": "CREATE", "namespace": namespace, "object": pod}}
            try:
                resp = call_webhook(fake.service_endpoints, hook, review).get("response") or {}
            except (OSError, ValueError, ssl.SSLError) as exc:
                if hook.get("failurePolicy", "Fail") == "Fail":
                    raise Rejected(f"failed calling webhook {hook.get('name')}: {exc}") from exc
                continue
            if not resp.get("allowed", False):
                raise Rejected(f"admission webhook {hook.get('name')} denied the request")
            if resp.get("patch"):
                pod = apply_patch(pod, json.loads(base64.b64decode(resp["patch"])))
    return pod


def admit_pod(fake, cid: str, namespace: str, pod: Dict[str, Any]) -> Tuple[Optional[Dict[str, Any]],
                                                                           Optional[Tuple[int, Any]]]:
    """``(admitted pod, None)`` or ``(None, (status, Status object))``: mutation, then Pod
    Security on the mutated object, as the API server orders them."""
    try:
        pod = mutate_pod(fake, cid, namespace, pod)
    except Rejected as exc:
        return None, (400, {"kind": "Status", "reason": "BadRequest", "code": 400, "message": str(exc)})
    level = fake.namespace_labels(cid, namespace).get(PSA_ENFORCE, fake.default_pod_security)
    problems = pod_security_violations(pod, level)
    if problems:
        name = (pod.get("metadata") or {}).get("name", "")
        return None, (403, {"kind": "Status", "reason": "Forbidden", "code": 403,
                            "message": f'pods "{name}" is forbidden: violates PodSecurity "{level}:latest": '
                                       + "; ".join(problems)})
    return pod, None


__all__ = ["PSA_ENFORCE", "PSA_LEVELS", "Rejected", "admit_pod", "mutate_pod", "namespace_selected",
           "pod_security_violations", "rule_matches_pod_create"]
