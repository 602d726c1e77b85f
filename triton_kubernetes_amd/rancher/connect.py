"""The agent side of Rancher's node registration (``POST /v3/connect/register``).

A Rancher agent opens its tunnel with two headers: ``X-API-Tunnel-Token`` (the cluster's
registration token) and ``X-API-Tunnel-Params`` (base64 JSON describing the node).  The
simulated node agents (``node/agent_steps.py``, sim mode) register through it, and the
fake server (``rancher/fake/v3.py``) decodes the same document, so both sides share this
encoder.
"""

import base64
import json
from typing import Any, Dict, List, Optional


def tunnel_params(hostname: str, roles: Dict[str, bool], labels: Dict[str, str],
                  capacity: Dict[str, Any], taints: Optional[List[Dict[str, str]]] = None) -> str:
    """The ``X-API-Tunnel-Params`` header a node agent sends (base64 JSON).  ``capacity``
    carries the node's GPU devices (``amd.com/gpu``: what a device plugin on it would
    enumerate), not what the kubelet advertises."""
    node = {"requestedHostname": hostname, "etcd": roles.get("etcd", False),
            "controlPlane": roles.get("controlplane", False), "worker": roles.get("worker", False),
            "labels": labels, "capacity": capacity, "taints": list(taints or [])}
    return base64.b64encode(json.dumps({"node": node}).encode()).decode()


__all__ = ["tunnel_params"]
