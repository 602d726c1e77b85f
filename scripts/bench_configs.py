#!/usr/bin/env python3
"""Wall-clock of BASELINE.json configs #1–#4 on CPU, through the real CLI code path.

Config #5 (MI355X bare-metal with the device plugin and xGMI labels) is `bench.py`, run
on the GPU. These four are pure orchestration: no GPU, no cloud. Every external service
is the in-process fake the tests use:

1. `get manager` against a memory backend holding a local-layout state (mocked backend,
   no Terraform).
2. `create manager`, non-interactive, local backend, bare-metal provider, 1 node. The
   DirectExecutor adopts a running (fake) Rancher server and bootstraps it (S3).
3. `create cluster`, bare-metal, 3 nodes (1 etcd/control + 2 workers), local backend.
   DirectExecutor; the three hosts are sim-mode node agents.
4. `create cluster`, Triton provider, 8 nodes, Manta state backend. The Triton CloudAPI
   listings and Manta are fakes with HTTP-signature checks. The apply goes through the
   TerraformExecutor with a fake `terraform` 1.5.7 on PATH, which enforces what a real
   1.5 does (no `manta` backend, sensitive root outputs, the modules' `required_version`)
   and keeps a tfstate; the executor carries that tfstate to and from FakeManta under
   the Manta lock. After the timed creates: `get manager`, then `destroy manager`.

Each config runs `--runs` times after one warm-up run. The script prints one JSON line
per config with the median and min wall-clock in ms.
"""

import argparse
import io
import json
import os
import shutil
import statistics
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))

from triton_kubernetes_amd.backend import LocalBackend, MemoryBackend  # noqa: E402
from triton_kubernetes_amd.config import Context, Settings  # noqa: E402
from triton_kubernetes_amd.node.agent import NodeAgent  # noqa: E402
from triton_kubernetes_amd.rancher.fake import FakeRancher  # noqa: E402
from triton_kubernetes_amd import workflows as wf  # noqa: E402

TOKEN = "bench-configs-token"


def ctx_of(values, cloud=None):
    return Context(settings=Settings(dict(values, **{"non-interactive": True}), env={}), out=io.StringIO(),
                   cloud=cloud)


def timed(fn, runs):
    fn(-1)  # warm-up
    out = []
    for i in range(runs):
        t0 = time.perf_counter()
        fn(i)
        out.append((time.perf_counter() - t0) * 1e3)
    return {"median_ms": round(statistics.median(out), 3), "min_ms": round(min(out), 3), "runs": runs}


def config1(runs):
    st = LocalBackend(tempfile.mkdtemp()).state("mgr")
    st.set_manager({"source": "github.com/joyent/triton-kubernetes//terraform/modules/bare-metal-rancher?ref=master",
                    "name": "mgr"})
    tf = json.dumps({"version": 4, "module_outputs": {"cluster-manager": {
        "rancher_url": "https://10.0.0.1", "rancher_access_key": "token-x", "rancher_secret_key": "s"}},
        "module_state": {}}).encode()
    backend = MemoryBackend(states={"mgr": st.bytes()})
    backend.write_blob("mgr", "terraform.tfstate", tf)

    def run(_):
        wf.get_manager(ctx_of({"cluster_manager": "mgr", "executor": "direct"}), backend)
    return timed(run, runs)


def config2_3(runs):
    fake = FakeRancher.for_manager("mgr", "tk-admin-pw-0123").start()
    agents = [NodeAgent(name=f"n{i}", mode="sim", token=TOKEN, root=tempfile.mkdtemp()) for i in range(3)]
    urls = ["agent+" + a.serve() for a in agents]
    root = tempfile.mkdtemp()
    base = {"backend_provider": "local", "executor": "direct", "agent_token": TOKEN}

    # a fresh Rancher per run: the bootstrap changes the initial admin password
    fresh = [FakeRancher.for_manager("mgr", "tk-admin-pw-0123").start() for _ in range(runs + 1)]

    def mgr(i):
        backend = LocalBackend(os.path.join(root, f"m{i}"))
        wf.new_manager(ctx_of(dict(base, manager_cloud_provider="baremetal", name="mgr",
                                   rancher_admin_password="tk-admin-pw-0123", rancher_bootstrap_password=fresh[i + 1].bootstrap_password, host="rancher+" + fresh[i + 1].url, ssh_user="u",
                                   bastion_host="", key_path="k")), backend)

    r2 = timed(mgr, runs)
    for f in fresh:
        f.stop()
    backend = LocalBackend(os.path.join(root, "c"))
    wf.new_manager(ctx_of(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password="tk-admin-pw-0123",
                               rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="u", bastion_host="", key_path="k")), backend)

    def cluster(i):
        nodes = [{"rancher_host_label": "etcd", "node_count": 1, "hostname": f"c{i}-e", "ssh_user": "u",
                  "bastion_host": "", "key_path": "k", "hosts": [urls[0]]},
                 {"rancher_host_label": "worker", "node_count": 2, "hostname": f"c{i}-w", "ssh_user": "u",
                  "bastion_host": "", "key_path": "k", "hosts": urls[1:]}]
        wf.new_cluster(ctx_of(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal",
                                   name=f"three-{i + 1}", k8s_version="v1.28.10-rancher1-1",
                                   k8s_network_provider="flannel", nodes=nodes)), backend)

    r3 = timed(cluster, runs)
    for a in agents:
        a.stop()
    fake.stop()
    return r2, r3


def config4(runs):
    from helpers import FAKE_TF, make_ssh_key
    from triton_kubernetes_amd.backend.manta import MantaBackend
    from triton_kubernetes_amd.cloud.fake import FakeCloud
    from triton_kubernetes_amd.cloud.fake_manta import FakeManta
    from triton_kubernetes_amd.utils.sshkeys import load_private_key

    work = tempfile.mkdtemp()
    key_path = make_ssh_key(os.path.join(work, "id_rsa"))
    key = load_private_key(key_path)
    manta = FakeManta("acct").start()
    manta.add_key(key)
    bindir = os.path.join(work, "bin")
    os.makedirs(bindir)
    exe = os.path.join(bindir, "terraform")
    with open(exe, "w") as fh:
        fh.write(f"#!/bin/sh\nexec {sys.executable} {FAKE_TF} \"$@\"\n")
    os.chmod(exe, 0o755)
    os.environ["PATH"] = bindir + os.pathsep + os.environ["PATH"]
    os.environ["FAKE_TF_LOG"] = os.path.join(work, "tf.log")
    os.environ["FAKE_TF_VERSION"] = "1.5.7"
    cloud = FakeCloud()
    triton = {"triton_account": "acct", "triton_key_path": key_path, "triton_url": "https://tr.example",
              "triton_network_names": ["Joyent-SDC-Public"], "triton_image_name": "ubuntu-certified-16.04",
              "triton_image_version": "20180222", "triton_ssh_user": "ubuntu"}
    backend = MantaBackend("acct", key_path, key.fingerprint_md5(), "https://tr.example", manta.url)
    wf.new_manager(ctx_of(dict(triton, backend_provider="manta", executor="terraform", manager_cloud_provider="triton",
                               name="tmgr", rancher_admin_password="tk-admin-pw-0123",
                               master_triton_machine_package="k4-highcpu-kvm-7.75G"), cloud=cloud), backend)

    def cluster(i):
        nodes = [{"rancher_host_label": lbl, "node_count": n, "hostname": f"t{i}-{lbl}",
                  "triton_machine_package": "k4-highcpu-kvm-7.75G", **{k: triton[k] for k in (
                      "triton_network_names", "triton_image_name", "triton_image_version", "triton_ssh_user")}}
                 for lbl, n in (("etcd", 1), ("control", 1), ("worker", 6))]
        wf.new_cluster(ctx_of(dict(triton, backend_provider="manta", executor="terraform", cluster_manager="tmgr",
                                   cluster_cloud_provider="triton", name=f"eight-{i + 1}",
                                   k8s_version="v1.28.10-rancher1-1", k8s_network_provider="flannel", nodes=nodes),
                              cloud=cloud), backend)

    r4 = timed(cluster, runs)
    # the tfstate round-tripped through Manta: one lineage, one serial per apply
    st = json.loads(backend.read_tfstate("tmgr"))
    assert st["serial"] == runs + 2 and len(st["resources"]) == 1 + 9 * (runs + 1), st["serial"]
    out = io.StringIO()
    ctx = ctx_of({"cluster_manager": "tmgr", "executor": "terraform"})
    ctx.out = out
    wf.get_manager(ctx, backend)
    assert "rancher_url = fake-cluster-manager__rancher_url" in out.getvalue()
    wf.delete_manager(ctx_of({"cluster_manager": "tmgr", "executor": "terraform"}), backend)
    assert backend.states() == [] and not any("/triton-kubernetes/tmgr" in p for p in manta.objects)
    assert manta.rejected == 0
    manta.stop()
    shutil.rmtree(work, ignore_errors=True)
    return r4


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--runs", type=int, default=5)
    args = ap.parse_args()
    rows = [("1 get manager (mocked backend)", config1(args.runs))]
    r2, r3 = config2_3(args.runs)
    rows += [("2 create manager baremetal (direct)", r2), ("3 create cluster baremetal 3-node (direct)", r3),
             ("4 create cluster triton 8-node + manta (terraform executor, fake terraform)", config4(args.runs))]
    for name, r in rows:
        print(json.dumps({"config": name, **r}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
