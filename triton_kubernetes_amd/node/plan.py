"""Node bootstrap plans: one definition, two renderers.

A :class:`BootstrapPlan` is the ordered list of steps a host runs to join a
cluster (the reference's ``install_rancher_agent.sh.tpl``, S5, plus the MI355X
steps).  It renders to

* a POSIX shell script (:meth:`BootstrapPlan.render_shell`) delivered over SSH
  or as cloud-init user-data — each step a function with timing markers
  ``::tk-step <name> <status> <ms>`` that the executor parses; and
* a structured document (:meth:`BootstrapPlan.to_json`) that a
  :class:`~.agent.NodeAgent` executes step by step in-process, running the GPU
  steps through the native MI355X probes.

Step catalogue (``action`` ids):

==================  ==============================================================
``firewall``        stop/disable firewalld (S5)
``runtime``         RKE1: install Docker if absent, overlay2 (S1/S5/S6); RKE2 brings
                    its own containerd (no step)
``hostname``        ``hostnamectl set-hostname`` (S5)
``registry_login``  RKE1: ``docker login`` when registry credentials are given (S5);
                    RKE2 nodes get registries from the cluster's ``rkeConfig``
``gpu_preflight``   MI355X: amdgpu loaded, ``/dev/kfd`` + ``/dev/dri`` present, N GPUs, the
                    partition modes, host tuning (NUMA balancing, IOMMU mode: ``node/hosttune.py``)
``gpu_labels``      MI355X: N1 topology labeller -> node labels file
``gpu_burnin``      MI355X: HBM / MFMA / memtest probes per GPU
``gpu_health``      MI355X: RAS verdict (uncorrectable ECC, retired VRAM pages) under the
                    cluster's ``gpu_health`` policy: fail the node, or join it tainted
                    ``amd.com/gpu-health=unhealthy:NoSchedule`` (``node/health.py``)
``rccl_env``        MI355X: write ``/etc/rccl/rccl.env``
``rccl_local``      MI355X: node-level RCCL all-reduce sweep over the local GPUs (N2)
``agent``           join: RKE2 -> the server's ``system-agent-install.sh`` (installs
                    ``rancher-system-agent``) with ``--server/--token/--ca-checksum/
                    --node-name/--<role>``; RKE1 -> ``docker run rancher/rancher-agent``
                    with ``--server/--token/--ca-checksum/--<role>``; both with
                    ``--label`` flags (GPU labels on MI355X nodes) and ``--taints``
                    (an unhealthy GPU node under the ``taint`` policy)
==================  ==============================================================
"""

import shlex
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional

from ..parallel.rccl_env import render_env_file
from ..terraform.scripts import RCCL_SLIM_ENABLE_FN, RCCL_SLIM_FN, RCCL_SLIM_ROOT

from ..versions import AGENT_IMAGE as DEFAULT_AGENT_IMAGE
from ..versions import DEFAULT_DISTRIBUTION, SYSTEM_AGENT_INSTALL_PATH
from ..versions import DOCKER_INSTALL_URL as DEFAULT_DOCKER_INSTALL_URL
from .cleanup import join_guard_shell, join_record_shell
from .labels import DEFAULT_MIN_LINK_GBPS
from .manager import docker_install_lines

LABEL_FILE = "/etc/triton-kubernetes/gpu-labels"
BURNIN_LABEL_FILE = "/etc/triton-kubernetes/gpu-burnin-labels"
TOPOLOGY_FILE = "/etc/triton-kubernetes/gpu-topology.json"
HEALTH_FILE = "/etc/triton-kubernetes/gpu-health.json"
TAINT_FILE = "/etc/triton-kubernetes/gpu-taints"  # key=value:Effect lines the join passes as --taints
RCCL_ENV_FILE = "/etc/rccl/rccl.env"
TOOLS_DIR = "/opt/triton-kubernetes/bin"

ROLE_FLAG = {"worker": "worker", "etcd": "etcd", "control": "controlplane", "controlplane": "controlplane"}


@dataclass
class Step:
    name: str
    action: str
    shell: str
    params: Dict[str, Any] = field(default_factory=dict)
    gpu: bool = False


@dataclass
class BootstrapPlan:
    hostname: str
    role: str  # worker | etcd | controlplane
    rancher_url: str
    token: str
    ca_checksum: str
    steps: List[Step] = field(default_factory=list)
    gpu: Optional[Dict[str, Any]] = None
    distribution: str = DEFAULT_DISTRIBUTION  # rke2 | rke1: how the agent step joins

    def step_names(self) -> List[str]:
        return [s.name for s in self.steps]

    def to_json(self) -> Dict[str, Any]:
        return asdict(self)

    @classmethod
    def from_json(cls, doc: Dict[str, Any]) -> "BootstrapPlan":
        steps = [Step(**s) for s in doc.get("steps", [])]
        d = {k: v for k, v in doc.items() if k != "steps"}
        return cls(steps=steps, **d)

    def render_shell(self) -> str:
        out = [
            "#!/bin/bash",
            f"# triton-kubernetes node bootstrap: {self.hostname} ({self.role})",
            "set -euo pipefail",
            "_tk_now() { date +%s%3N; }",
            # each step body runs in a subshell with errexit in force: a failing command
            # anywhere in the body fails the step (a function called as an `if` condition
            # would run with errexit ignored), and an `exit` in a body ends only its step
            "_tk_step() { local _tk_name=$1; shift; local _tk_t0 _tk_rc; _tk_t0=$(_tk_now);",
            "  echo \"::tk-step $_tk_name start 0\";",
            "  set +e; ( set -e; \"$@\" ); _tk_rc=$?; set -e",
            "  if [ $_tk_rc -eq 0 ]; then echo \"::tk-step $_tk_name ok $(( $(_tk_now) - _tk_t0 ))\";",
            "  else echo \"::tk-step $_tk_name failed $(( $(_tk_now) - _tk_t0 ))\" >&2; exit $_tk_rc; fi; }",
        ]
        for s in self.steps:
            body = s.shell.strip("\n")
            out.append(f"step_{s.name}() {{")
            # bodies are emitted verbatim: indenting them would break heredoc terminators
            out.extend(body.splitlines())
            out.append("}")
        # one compound command: bash parses all of it before running a step, and
        # the steps' stdin is /dev/null, so a step that reads stdin cannot eat the
        # rest of a script delivered through `bash -s`
        out.append("{")
        for s in self.steps:
            out.append(f"_tk_step {s.name} step_{s.name}")
        out.append("echo '::tk-done'")
        out.append("} </dev/null")
        return "\n".join(out) + "\n"


def render_cloud_init(plan: "BootstrapPlan", rccl_env: Optional[Dict[str, str]] = None) -> str:
    """``#cloud-config`` user-data that runs the plan at first boot.

    For hosts provisioned by PXE/MAAS/cloud images instead of SSH: the RCCL
    environment and the bootstrap script are written by cloud-init's
    ``write_files`` (so the RCCL env exists before anything GPU-related starts),
    then ``runcmd`` executes the script with its step markers logged to
    ``/var/log/triton-kubernetes-bootstrap.log``."""
    import yaml

    files = []
    if rccl_env is not None:
        files.append({"path": RCCL_ENV_FILE, "permissions": "0644", "owner": "root:root",
                      "content": render_env_file(rccl_env)})
    files.append({"path": "/opt/triton-kubernetes/bootstrap.sh", "permissions": "0755", "owner": "root:root",
                  "content": plan.render_shell()})
    doc = {
        "hostname": plan.hostname,
        "preserve_hostname": False,
        "write_files": files,
        "runcmd": [["bash", "-c", "/opt/triton-kubernetes/bootstrap.sh "
                                  ">> /var/log/triton-kubernetes-bootstrap.log 2>&1"]],
    }
    return "#cloud-config\n" + yaml.safe_dump(doc, sort_keys=False, default_flow_style=False, width=1 << 30)


def _q(v: Any) -> str:
    return shlex.quote(str(v))


def host_role(cfg: Dict[str, Any]) -> str:
    labels = cfg.get("rancher_host_labels") or {}
    for k in ("control", "etcd", "worker"):
        if str(labels.get(k, "")).lower() == "true":
            return ROLE_FLAG[k]
    raise ValueError(f"node {cfg.get('hostname')!r} has no rancher_host_labels role")


def build_host_plan(cfg: Dict[str, Any], rancher_url: str, token: str, ca_checksum: str,
                    mi355x: bool = False, sequential: bool = False) -> BootstrapPlan:
    """Plan for a ``*-rancher-k8s-host`` module config with resolved interpolations.

    ``sequential``: the plan runs as one shell script (SSH, cloud-init), each step after the
    previous.  The burn-in then goes after the node's RCCL check: the driver clears the
    ~300 GB per GPU it releases for seconds afterwards, and a communicator started meanwhile
    waits behind that (profiles/round5/README.md).  A node agent runs the default order:
    it overlaps the burn-in with the gate's communicator start and holds the release."""
    role = host_role(cfg)
    hostname = cfg.get("hostname", "")
    dist = str(cfg.get("k8s_distribution") or DEFAULT_DISTRIBUTION)
    if dist not in ("rke2", "rke1"):
        raise ValueError(f"k8s_distribution must be rke2 or rke1, not {dist!r}")
    rke1 = dist == "rke1"
    plan = BootstrapPlan(hostname, role, rancher_url, token, ca_checksum, distribution=dist)
    install_url = cfg.get("docker_engine_install_url") or DEFAULT_DOCKER_INSTALL_URL
    image = cfg.get("rancher_agent_image") or DEFAULT_AGENT_IMAGE
    reg, reg_user, reg_pass = (cfg.get("rancher_registry", ""), cfg.get("rancher_registry_username", ""),
                               cfg.get("rancher_registry_password", ""))
    plan.steps.append(Step("firewall", "firewall", """
if command -v firewalld >/dev/null 2>&1; then
  sudo systemctl stop firewalld.service || true
  sudo systemctl disable firewalld.service || true
fi"""))
    if rke1:
        plan.steps.append(Step("runtime", "runtime", f"""
{docker_install_lines(install_url, cfg.get("docker_install_sha256", "")).rstrip()}
if [ ! -f /etc/docker/daemon.json ] || ! grep -q overlay2 /etc/docker/daemon.json; then
  echo '{{"storage-driver": "overlay2"}}' | sudo tee /etc/docker/daemon.json >/dev/null
  sudo systemctl restart docker || sudo service docker restart
fi""", {"install_url": install_url}))
    plan.steps.append(Step("hostname", "hostname", f"sudo hostnamectl set-hostname {_q(hostname)}",
                           {"hostname": hostname}))
    if reg_user and rke1:
        plan.steps.append(Step("registry_login", "registry_login",
                               f"echo {_q(reg_pass)} | sudo docker login -u {_q(reg_user)} --password-stdin {_q(reg)}",
                               {"registry": reg, "username": reg_user, "password": reg_pass}))
    label_args = ""
    if mi355x:
        from .partition import modes_of, partitions_per_gpu

        physical = int(cfg.get("gpu_count", 8) or 8)
        cpart, mpart = modes_of(cfg)
        ngpu = physical * partitions_per_gpu(cpart)  # logical GPUs: amd.com/gpu units, RCCL ranks
        burnin = cfg.get("gpu_burnin", "full")
        env = dict(cfg.get("rccl_env") or {})
        from .hosttune import policy_of as tuning_policy
        from .hosttune import shell_check as host_tuning_check

        tuning = tuning_policy(cfg)
        plan.gpu = {"product": cfg.get("gpu_product", "MI355X"), "count": ngpu, "burnin": burnin,
                    "physical": physical, "compute_partition": cpart, "memory_partition": mpart}
        plan.steps.append(Step("gpu_preflight", "gpu_preflight", f"""
lsmod | grep '^amdgpu' >/dev/null || {{ echo 'amdgpu kernel module not loaded' >&2; exit 1; }}
test -c /dev/kfd || {{ echo '/dev/kfd missing' >&2; exit 1; }}
test -d /dev/dri || {{ echo '/dev/dri missing' >&2; exit 1; }}
local found f m
found=$(ls /dev/dri/renderD* 2>/dev/null | wc -l || true)  # pipefail: ls fails when there are none
[ "$found" -ge {ngpu} ] || {{ echo "expected {ngpu} GPUs ({physical} x {cpart}), found $found render nodes" >&2; exit 1; }}
for f in /sys/class/drm/renderD*/device/current_compute_partition /sys/class/drm/renderD*/device/current_memory_partition; do
  [ -r "$f" ] || continue
  m=$(tr 'A-Z' 'a-z' < "$f")
  case $f in
    *compute*) [ "$m" = {cpart} ] || {{ echo "compute partition is $m, the cluster expects {cpart}" >&2; exit 1; }} ;;
    *) [ "$m" = {mpart} ] || {{ echo "memory partition is $m, the cluster expects {mpart}" >&2; exit 1; }} ;;
  esac
done
sudo usermod -aG video,render "$(id -un)" || true
sudo rm -f {BURNIN_LABEL_FILE} {TAINT_FILE}
{host_tuning_check(tuning, BURNIN_LABEL_FILE)}""", {"count": ngpu, "compute_partition": cpart, "memory_partition": mpart,
                                               "host_tuning": tuning}, gpu=True))
        if physical > 1 and cpart == "spx":  # links are a whole GPU's (a partition has no own)
            # per-link xGMI health: kernel-driven peer read of every GPU pair against the
            # node's median (relative) and an absolute floor (a uniformly slow fabric).  Before
            # the burn-in: the peer reads then run on idle GPUs, never beside the driver's
            # clearing of the ~300 GB per GPU a full burn-in releases
            frac = float(cfg.get("gpu_link_min_frac", 0.5) or 0.5)
            floor = float(cfg.get("gpu_link_min_gbps", DEFAULT_MIN_LINK_GBPS) or 0.0)
            plan.steps.append(Step("gpu_links", "gpu_links", f"""
{TOOLS_DIR}/gpu-burnin --p2p --min-link-frac {frac} --min-link-gbps {floor} --labels /tmp/tk-link-labels | sudo tee /etc/triton-kubernetes/gpu-links.json
cat /tmp/tk-link-labels | sudo tee -a {BURNIN_LABEL_FILE} >/dev/null""", {"min_frac": frac, "min_gbps": floor,
                                                                       "method": "kernel-read"}, gpu=True))
        # burn-in before labels: the agent discovers the topology concurrently
        # with the burn-in kernels and only joins it at the labels step
        if burnin != "off":
            plan.steps.append(Step("gpu_burnin", "gpu_burnin", f"""
sudo mkdir -p /etc/triton-kubernetes
{TOOLS_DIR}/gpu-burnin --all --level {_q(burnin)} --compute-partition {cpart} --memory-partition {mpart} --labels /tmp/tk-burnin-labels | sudo tee /etc/triton-kubernetes/gpu-burnin.json
sudo tee -a {BURNIN_LABEL_FILE} < /tmp/tk-burnin-labels >/dev/null""",
                                   {"level": burnin, "compute_partition": cpart, "memory_partition": mpart},
                                   gpu=True))
        plan.steps.append(Step("gpu_labels", "gpu_labels", f"""
sudo mkdir -p "$(dirname {LABEL_FILE})"
{TOOLS_DIR}/amdgpu-topo-labeller | sudo tee {TOPOLOGY_FILE} >/dev/null
{TOOLS_DIR}/amdgpu-topo-labeller --labels | sudo tee {LABEL_FILE} >/dev/null""", gpu=True))
        from .health import limits_of, policy_of, taint_flag

        policy = policy_of(cfg)
        if policy != "off":
            # RAS verdict per physical GPU (node/health.py): exit 3 = a GPU is unhealthy
            max_ue, max_bad = limits_of(cfg)
            bad_arg = "auto" if max_bad < 0 else str(max_bad)
            args = f"--health --max-uncorrectable {max_ue} --max-bad-pages {bad_arg}"
            on_bad = (f"echo {_q(taint_flag())} | sudo tee {TAINT_FILE} >/dev/null" if policy == "taint" else
                      "echo 'unhealthy GPUs (gpu_health = fail):' >&2; cat /tmp/tk-gpu-health.json >&2; exit 1")
            plan.steps.append(Step("gpu_health", "gpu_health", f"""
local rc=0
{TOOLS_DIR}/amdgpu-topo-labeller {args} > /tmp/tk-gpu-health.json || rc=$?
sudo install -m 0644 /tmp/tk-gpu-health.json {HEALTH_FILE}
{{ {TOOLS_DIR}/amdgpu-topo-labeller {args} --labels || true; }} | sudo tee -a {BURNIN_LABEL_FILE} >/dev/null
case $rc in
  0) ;;
  3) {on_bad} ;;
  *) echo "GPU health check failed (exit $rc)" >&2; exit 1 ;;
esac""", {"policy": policy, "max_uncorrectable": max_ue, "max_bad_pages": max_bad}, gpu=True))
        from .metrics import textfile_dir_of, textfile_script

        mdir = textfile_dir_of(cfg)
        if mdir:
            # opt-in: GPU health as Prometheus text for node_exporter, refreshed every minute
            m_ue, m_bad = limits_of(cfg)
            plan.steps.append(Step("gpu_metrics", "gpu_metrics",
                                   textfile_script(TOOLS_DIR, mdir, str(m_ue), "auto" if m_bad < 0 else str(m_bad)),
                                   {"dir": mdir, "max_uncorrectable": m_ue, "max_bad_pages": m_bad}, gpu=True))
        # discovered inter-node settings (active RDMA ports) first; the configured
        # values follow, so an explicit rccl_env key wins when the file is sourced
        plan.steps.append(Step("rccl_env", "rccl_env", f"""
sudo mkdir -p "$(dirname {RCCL_ENV_FILE})"
{{ {TOOLS_DIR}/amdgpu-topo-labeller --rccl-env || true; cat <<'TK_RCCL_EOF'
{render_env_file(env).rstrip()}
TK_RCCL_EOF
}} | sudo tee {RCCL_ENV_FILE} >/dev/null""", {"env": env}, gpu=True))
        slim = str(cfg.get("rccl_slim", "off") or "off").lower() == "on"
        if slim:
            # OPT-IN single-target RCCL (terraform/scripts.py): built, verified by a one-rank
            # all-reduce that must map it, then used through rccl-ready-slim; never fatal
            plan.steps.append(Step("rccl_slim", "rccl_slim", f"""
{RCCL_SLIM_FN}
{RCCL_SLIM_ENABLE_FN}
sudo bash -c "$(declare -f tk_rccl_slim tk_rccl_slim_enable); tk_rccl_slim_enable {RCCL_SLIM_ROOT} ${{ROCM_PATH:-/opt/rocm}} {TOOLS_DIR}" >/dev/null \\
  || echo 'rccl slim: not enabled, the node tools load the installed RCCL' >&2""", {"root": RCCL_SLIM_ROOT}, gpu=True))
        if ngpu > 1:
            tool = f"{TOOLS_DIR}/rccl-ready"
            if slim:
                tool = f"$([ -x {TOOLS_DIR}/rccl-ready-slim ] && echo {TOOLS_DIR}/rccl-ready-slim || echo {tool})"
            plan.steps.append(Step("rccl_local", "rccl_local",
                                   f"{tool} --ngpus {ngpu} --min-busbw "
                                   f"{float(cfg.get('rccl_min_busbw', 0) or 0)}",
                                   {"count": ngpu, "min_busbw": float(cfg.get("rccl_min_busbw", 0) or 0)},
                                   gpu=True))
        label_args = (f' $(cat {LABEL_FILE} $([ -r {BURNIN_LABEL_FILE} ] && echo {BURNIN_LABEL_FILE}) '
                      f'| sed "s/^/--label /" | tr "\\n" " ")'
                      f'$([ -r {TAINT_FILE} ] && sed "s/^/ --taints /" {TAINT_FILE} | tr -d "\\n")')
    # a host still joined to another cluster is refused before anything is installed, and a
    # successful join is recorded (node/cleanup.py): reused bare metal is cleaned on destroy
    guard = join_guard_shell(rancher_url, token)
    record = join_record_shell(rancher_url, token, dist, hostname, image if rke1 else "")
    if rke1:
        plan.steps.append(Step("agent", "agent", (
            guard +
            f"sudo docker run -d --privileged --restart=unless-stopped --net=host "
            f"-v /etc/kubernetes:/etc/kubernetes -v /var/run:/var/run {_q(image)} "
            f"--server {_q(rancher_url)} --token {_q(token)} --ca-checksum {_q(ca_checksum)} --{role}{label_args}\n"
            + record),
            {"image": image, "role": role, "distribution": "rke1"}))
    else:
        # the registration command Rancher shows for a custom RKE2 cluster: the server's
        # installer sets up rancher-system-agent, which then installs RKE2 for the role
        # installer over TLS verified against the server's CA, which must first match the
        # cluster's CA checksum (an empty CA: a publicly trusted certificate)
        base = rancher_url.rstrip("/")
        plan.steps.append(Step("agent", "agent", (
            guard +
            "_tk_installer=$(mktemp); _tk_ca=$(mktemp)\n"
            "trap 'rm -f \"$_tk_installer\" \"$_tk_ca\"' EXIT\n"
            f"curl -fsSLk -o \"$_tk_ca\" {_q(base + '/cacerts')}\n"
            "if [ -s \"$_tk_ca\" ]; then\n"
            f"  [ \"$(sha256sum < \"$_tk_ca\" | cut -d' ' -f1)\" = {_q(ca_checksum)} ] || "
            "{ echo 'the Rancher CA does not match the cluster CA checksum' >&2; exit 1; }\n"
            f"  curl -fsSL --cacert \"$_tk_ca\" -o \"$_tk_installer\" {_q(base + SYSTEM_AGENT_INSTALL_PATH)}\n"
            "else\n"
            f"  curl -fsSL -o \"$_tk_installer\" {_q(base + SYSTEM_AGENT_INSTALL_PATH)}\n"
            "fi\n"
            f"sudo sh \"$_tk_installer\" --server {_q(rancher_url)} --label cattle.io/os=linux "
            f"--token {_q(token)} --ca-checksum {_q(ca_checksum)} --node-name {_q(hostname)} --{role}{label_args}\n"
            + record),
            {"server": rancher_url, "role": role, "distribution": "rke2"}))
    names = plan.step_names()
    if sequential and "gpu_burnin" in names and "rccl_local" in names:
        burn = plan.steps.pop(names.index("gpu_burnin"))
        plan.steps.insert(plan.step_names().index("rccl_local") + 1, burn)
    return plan


def parse_step_markers(output: str) -> Dict[str, Dict[str, Any]]:
    """``::tk-step`` markers of a shell run -> ``{step: {status, ms}}``."""
    steps: Dict[str, Dict[str, Any]] = {}
    for line in output.splitlines():
        if line.startswith("::tk-step "):
            parts = line.split()
            if len(parts) >= 4:
                steps[parts[1]] = {"status": parts[2], "ms": int(parts[3]) if parts[3].isdigit() else 0}
    return steps
