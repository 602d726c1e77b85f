"""triton_kubernetes_amd — multi-cloud Kubernetes provisioning with a first-class
bare-metal 8xMI355X path.

Capability parity target: ``nimajalali/triton-kubernetes`` v0.8.2 (a Go CLI over
Terraform).  Layer map of this package::

    cli/        L7  argparse CLI: create|destroy|get {manager,cluster,node}, version
    config/     L6  layered config (overrides > flags > ENV > YAML) + prompt interface
    models/     L4/L5 provider "model families" (triton/aws/gcp/azure/baremetal/
                    vsphere/mi355x) and the create/destroy/get workflows
    state/      L3  the main.tf.json document (module-key schema)
    backend/    L2  local FS / Manta / in-memory state backends
    executor/   L1  Terraform executor (version-aware) + native DirectExecutor
    rancher/        Rancher v3 REST client and an in-process fake server
    cloud/          REST clients for cloud listings (Triton, AWS SigV4, GCP, Azure)
    parallel/       bounded parallel fan-out, SSH / agent transports, RCCL env
    node/           node bootstrap plan (shell renderer + in-process runner), node agent
    readiness/      create -> kubectl-ready waiter with per-phase timing
    k8s/            device-plugin / labeller / xGMI-affinity manifests, k8s client
    ops/            native MI355X probes: HIP burn-in kernels, amd_smi topology
                    labeller, RCCL all-reduce readiness probe (C++/HIP, gfx950)
    terraform/      Terraform >=1.x module library (17 reference modules + MI355X)
    utils/          timing/tracing, JSON encoding, misc helpers
"""

__version__ = "0.8.2"
CLI_NAME = "triton-kubernetes"
