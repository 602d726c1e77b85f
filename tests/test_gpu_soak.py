"""A node agent is a long-lived daemon: one process takes cluster after cluster, each with a
burn-in, a link check and an RCCL gate communicator on its GPUs.  Soak on the MI355X: the
same resident agents take ``ROUNDS`` create -> ready -> destroy cycles.  After two warm-up
cycles, whatever this process holds must not grow with the cycles: open file descriptors,
threads, resident memory, and the GPU's device memory once the teardowns have drained.
"""

import os
import tempfile
import time

import pytest

pytestmark = pytest.mark.gpu

ROUNDS = int(os.environ.get("TK_SOAK_ROUNDS", "16"))
WARM = 4


def _held() -> dict:
    """What this process holds, after a garbage collection (closed connections whose
    objects are unreachable but not yet collected would otherwise count)."""
    import gc

    from triton_kubernetes_amd.ops import probe

    gc.collect()
    import ctypes

    class _MallInfo2(ctypes.Structure):
        _fields_ = [(n, ctypes.c_size_t) for n in ("arena", "ordblks", "smblks", "hblks", "hblkhd", "usmblks",
                                                   "fsmblks", "uordblks", "fordblks", "keepcost")]

    libc = ctypes.CDLL(None)
    libc.mallinfo2.restype = _MallInfo2
    libc.malloc_trim(0)  # freed heap back to the system: RSS then counts what is held
    mi = libc.mallinfo2()
    with open("/proc/self/statm", encoding="ascii") as fh:
        rss_pages = int(fh.read().split()[1])
    return {"fds": len(os.listdir("/proc/self/fd")), "threads": len(os.listdir("/proc/self/task")),
            "rss_mib": rss_pages * os.sysconf("SC_PAGE_SIZE") / 2 ** 20,
            "malloc_in_use_mib": round((mi.uordblks + mi.hblkhd) / 2 ** 20, 2),
            "gpu_used_mib": (probe.device_info(0).total_mem_gib - probe.device_info(0).free_mem_gib) * 1024}


def _drained(timeout_s: float = 30.0) -> None:
    """Asynchronous communicator teardowns and burn-in releases finished."""
    from triton_kubernetes_amd.ops import probe, rccl

    rccl.drain()
    probe.wait_frees()
    deadline = time.monotonic() + timeout_s
    while time.monotonic() < deadline and (rccl.inits_running() or rccl.preloads_running()):
        time.sleep(0.05)


def test_resident_agent_takes_cluster_after_cluster_without_growing(tmp_path):
    from triton_kubernetes_amd.backend import LocalBackend
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.parallel.transport import AgentTransport
    from triton_kubernetes_amd.rancher.fake import FakeRancher
    from triton_kubernetes_amd.workflows import delete_cluster, new_cluster, new_manager

    from helpers import make_ctx

    token = "gpu-soak-token-1234"
    fake = FakeRancher.for_manager("mgr", "tk-admin-pw-0123").start()
    cp = NodeAgent(name="cp", mode="sim", token=token, root=tempfile.mkdtemp())
    w = NodeAgent(name="w0", mode="sim", devices=[0], token=token, root=tempfile.mkdtemp())
    cp_url, w_url = cp.serve(), w.serve()
    backend = LocalBackend(str(tmp_path / "state"))
    base = {"executor": "direct", "agent_token": token}
    seen = []
    trace_mem = os.environ.get("TK_SOAK_TRACEMALLOC") == "1"  # diagnostic: where Python memory grows
    if trace_mem:
        import tracemalloc

        tracemalloc.start(8)
    snap = None
    try:
        new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr",
                                  rancher_admin_password="tk-admin-pw-0123",
                                  rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url,
                                  ssh_user="u", bastion_host="", key_path="k")), backend)
        for i in range(ROUNDS):
            name = f"soak-{i}"
            ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name=name,
                                k8s_version="v1.31", k8s_network_provider="canal", gpu_addons=True, wait=True,
                                rccl_gate=os.environ.get("TK_SOAK_GATE", "1") == "1", nodes=[
                                    {"rancher_host_label": "control", "node_count": 1, "hostname": f"{name}-cp",
                                     "ssh_user": "u", "bastion_host": "", "key_path": "k", "hosts": ["agent+" + cp_url]},
                                    {"rancher_host_label": "etcd", "node_count": 1, "hostname": f"{name}-etcd",
                                     "ssh_user": "u", "bastion_host": "", "key_path": "k", "hosts": ["agent+" + cp_url]},
                                    {"rancher_host_label": "worker", "node_count": 1, "hostname": f"{name}-gpu",
                                     "ssh_user": "u", "bastion_host": "", "key_path": "k", "hosts": ["agent+" + w_url],
                                     "gpu": "mi355x", "gpu_count": 1, "gpu_burnin": "quick"},
                                ]))
            ctx.extras["agent_transport"] = AgentTransport(token=token)
            new_cluster(ctx, backend)
            rep = ctx.extras["last_readiness"]
            if os.environ.get("TK_SOAK_GATE", "1") == "1":
                assert rep.rccl and rep.rccl["ok"] is True, rep.rccl
            dctx = make_ctx(dict(base, cluster_manager="mgr", cluster_name=name))
            dctx.extras["agent_transport"] = AgentTransport(token=token)
            delete_cluster(dctx, backend)
            _drained()
            seen.append(_held())
            print(i, seen[-1], flush=True)
            if trace_mem and i == WARM - 1:
                snap = tracemalloc.take_snapshot()
        if snap is not None:
            for st in tracemalloc.take_snapshot().compare_to(snap, "filename")[:12]:
                print("grew:", st, flush=True)
        import collections
        import threading

        print(collections.Counter(t.name.rstrip("0123456789-_") for t in threading.enumerate()), flush=True)
        first, last = seen[WARM - 1], seen[-1]
        assert last["fds"] <= first["fds"] + 4, seen
        assert last["threads"] <= first["threads"] + 4, seen
        assert last["rss_mib"] <= first["rss_mib"] + 96, seen
        assert last["gpu_used_mib"] <= first["gpu_used_mib"] + 512, seen
        assert len(w.history) <= w.HISTORY_KEEP
    finally:
        w.stop()
        cp.stop()
        fake.stop()
