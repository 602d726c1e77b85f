"""In-process fake Rancher 2.x server (the Rancher API fake SURVEY.md §4 calls for).

Split by API so each contract can be reviewed and tested on its own:

* :mod:`.v3` -- Norman ``/v3``: bootstrap (login, tokens, password change, settings),
  RKE1 custom clusters, registration tokens, nodes, agent registration;
* :mod:`.provisioning` -- Steve ``/v1``: RKE2 custom clusters
  (``provisioning.cattle.io/v1``), management-cluster Secrets, the node installer;
* :mod:`.k8s` -- ``/k8s/clusters/<id>``: each downstream cluster's API server (nodes,
  pods, evictions, an object store) and the kubelets' device-plugin model;
* :mod:`.admission` -- mutating admission webhooks and Pod Security Admission;
* :mod:`.server` -- shared state, HTTP, routing and the RKE/upgrade simulation.

Every module lists what the server refuses (with the status a real server answers);
``tests/test_fake_rancher_contract.py`` holds a negative test for each refusal.
"""

from .admission import PSA_ENFORCE, pod_security_violations
from .k8s import DEVICE_PLUGIN_REPOS, DEVICE_PLUGIN_SOCKET_DIR, INITIAL_NAMESPACES
from .provisioning import SYSTEM_AGENT_INSTALL_SCRIPT
from .server import FAKE_CACERTS, FakeRancher, State
from .v3 import tunnel_params

__all__ = ["FakeRancher", "State", "FAKE_CACERTS", "SYSTEM_AGENT_INSTALL_SCRIPT", "PSA_ENFORCE",
           "pod_security_violations", "tunnel_params", "DEVICE_PLUGIN_REPOS", "DEVICE_PLUGIN_SOCKET_DIR",
           "INITIAL_NAMESPACES"]
