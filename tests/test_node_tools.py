"""Prebuilt MI355X node tools on Terraform-delivered hosts (node/tools.py).

The install script's ``tk_node_tools`` runs here against a sandbox: stub ``sudo``, a
``hipcc``/``g++`` that count their calls, the module's shipped sources and a staged
prebuilt directory."""

import hashlib
import json
import os
import shutil
import subprocess

import pytest

from triton_kubernetes_amd.node import tools
from triton_kubernetes_amd.ops.build import CSRC
from triton_kubernetes_amd.terraform import catalog

MODULE = os.path.join(catalog.MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host")


def _stub(path, body):
    path.write_text("#!/bin/bash\n" + body)
    path.chmod(0o755)


@pytest.fixture
def node(tmp_path):
    """(run, calls, dirs): run(tools_dir, srcs, prebuilt, rocm) -> CompletedProcess."""
    bin_dir = tmp_path / "stubs"
    bin_dir.mkdir()
    calls = tmp_path / "compiler-calls"
    calls.write_text("")
    _stub(bin_dir / "sudo", 'exec "$@"\n')
    rocm = tmp_path / "rocm"
    (rocm / "bin").mkdir(parents=True)
    compiler = f'echo "$(basename "$0") $*" >> {calls}\nwhile [ "$1" != -o ]; do shift; done\n' \
               'printf "#!/bin/sh\\necho built\\n" > "$2"; chmod 755 "$2"\n'
    _stub(rocm / "bin" / "hipcc", compiler)
    _stub(bin_dir / "g++", compiler)
    srcs = tmp_path / "src"
    shutil.copytree(os.path.join(MODULE, "files", "src"), srcs)  # what the module ships (symlinks followed)

    def run(tools_dir, src_dir=srcs, prebuilt=tmp_path / "prebuilt", rocm_dir=rocm, path_extra=""):
        script = "set -euo pipefail\n" + tools.NODE_TOOLS_FN + f"\ntk_node_tools {tools_dir} {src_dir} {prebuilt} {rocm_dir}\n"
        env = dict(os.environ, PATH=f"{path_extra}{bin_dir}:{os.environ['PATH']}")
        return subprocess.run(["bash", "-c", script], capture_output=True, text=True, env=env, timeout=60)

    def compiles():
        return [ln for ln in calls.read_text().splitlines() if ln]

    return run, compiles, tmp_path


def _staged(tmp_path):
    fake_bins = tmp_path / "in-tree"
    fake_bins.mkdir(exist_ok=True)

    def binary(name):
        p = fake_bins / name
        p.write_text(f"#!/bin/sh\necho prebuilt {name}\n")
        return str(p)

    return tools.stage(str(tmp_path / "prebuilt"), binary=binary)


def test_stamp_is_the_one_the_node_computes_from_the_shipped_sources(node):
    run, compiles, tmp = node
    _staged(tmp)
    for name in tools.TOOL_SOURCES:
        stamp, binary_sum = (tmp / "prebuilt" / f"{name}.sha256").read_text().split()
        assert stamp == tools.node_stamp(name)
        assert binary_sum == hashlib.sha256((tmp / "prebuilt" / name).read_bytes()).hexdigest()
        # the module ships exactly the sources the stamp covers
        assert tools.node_stamp(name, str(tmp / "src")) == tools.node_stamp(name, CSRC)
    res = run(tmp / "bin")
    assert res.returncode == 0, res.stderr
    assert compiles() == []
    for name in tools.TOOL_SOURCES:
        assert f"{name}: prebuilt binary installed" in res.stdout
        out = subprocess.run([str(tmp / "bin" / name)], capture_output=True, text=True).stdout
        assert out == f"prebuilt {name}\n"


def test_second_node_and_reapply_compile_nothing(node):
    run, compiles, tmp = node
    _staged(tmp)
    assert run(tmp / "node1").returncode == 0
    assert run(tmp / "node2").returncode == 0
    again = run(tmp / "node1")
    assert again.returncode == 0 and compiles() == []
    assert all(f"{n}: installed copy is current" in again.stdout for n in tools.TOOL_SOURCES)
    assert "node tools:" in again.stdout  # the step's time, for the e2e to read


def test_node_without_hipcc_installs_the_prebuilt_tools(node, tmp_path):
    run, compiles, tmp = node
    _staged(tmp)
    res = run(tmp / "bin", rocm_dir=tmp_path / "no-rocm")
    assert res.returncode == 0, res.stderr
    assert sorted(os.listdir(tmp / "bin")) == sorted([".stamps", *tools.TOOL_SOURCES])


def test_only_the_tool_whose_sources_changed_is_built(node):
    run, compiles, tmp = node
    _staged(tmp)
    with open(tmp / "src" / "tk_gemm_screen.hip", "a") as fh:
        fh.write("\n// changed on the way to the node\n")
    res = run(tmp / "bin")
    assert res.returncode == 0, res.stderr
    assert len(compiles()) == 1 and compiles()[0].startswith("hipcc ") and "-DTK_PROBE_MAIN" in compiles()[0]
    assert "gpu-burnin: no matching prebuilt binary; building with" in res.stdout
    # the node's own build is stamped too: the next apply keeps it
    assert run(tmp / "bin").returncode == 0 and len(compiles()) == 1


def test_a_binary_damaged_on_the_way_is_rebuilt(node):
    run, compiles, tmp = node
    _staged(tmp)
    with open(tmp / "prebuilt" / "gpu-burnin", "a") as fh:
        fh.write("# truncated or altered in transit\n")
    res = run(tmp / "bin")
    assert res.returncode == 0, res.stderr
    assert len(compiles()) == 1 and "-DTK_PROBE_MAIN" in compiles()[0]
    assert res.stdout.count("prebuilt binary installed") == 2


def test_stale_prebuilt_and_no_compiler_fails_naming_the_tool(node, tmp_path):
    run, compiles, tmp = node
    _staged(tmp)
    with open(tmp / "src" / "tk_rccl_probe.hip", "a") as fh:
        fh.write("\n")
    res = run(tmp / "bin", rocm_dir=tmp_path / "no-rocm")
    assert res.returncode != 0
    assert "rccl-ready: no prebuilt binary for the shipped sources was uploaded" in res.stderr
    assert compiles() == []


def test_prebuilt_binary_with_unresolved_libraries_is_rebuilt(node):
    run, compiles, tmp = node
    _staged(tmp)
    ldd = tmp / "ldd-stub"
    ldd.mkdir()
    _stub(ldd / "ldd", 'case "$1" in *rccl-ready) echo "librccl.so.1 => not found" ;; *) echo "libc.so.6 => /lib/libc.so.6" ;; esac\n')
    res = run(tmp / "bin", path_extra=f"{ldd}:")
    assert res.returncode == 0, res.stderr
    assert [c.split()[0] for c in compiles()] == ["hipcc"] and "-DTK_RCCL_MAIN" in compiles()[0]


def test_nothing_staged_means_the_node_builds_everything_in_parallel(node):
    run, compiles, tmp = node
    (tmp / "prebuilt").mkdir()
    res = run(tmp / "bin")
    assert res.returncode == 0, res.stderr
    assert sorted(c.split()[0] for c in compiles()) == ["g++", "hipcc", "hipcc"]


def test_stage_skips_tools_this_machine_cannot_build(tmp_path):
    from triton_kubernetes_amd.ops.native import NativeUnavailable

    def binary(name):
        raise NativeUnavailable("no hipcc")

    logged = []
    got = tools.stage(str(tmp_path / "p"), binary=binary, log=logged.append)
    assert all(v.startswith("not staged") for v in got.values()) and len(logged) == 3
    assert os.listdir(tmp_path / "p") == []


def test_module_uploads_the_staged_dir_and_the_script_installs_from_it():
    main = open(os.path.join(MODULE, "main.tf")).read()
    assert 'prebuilt_tools = var.tk_prebuilt_tools != "" ? var.tk_prebuilt_tools : "${path.module}/files/prebuilt"' in main
    assert 'source      = "${local.prebuilt_tools}/"' in main and f'destination = "{tools.PREBUILT_DIR}"' in main
    script = open(os.path.join(MODULE, "files", "install_mi355x_node.sh.tftpl")).read()
    assert tools.NODE_TOOLS_FN in script and f"tk_node_tools $T $S {tools.PREBUILT_DIR} $ROCM" in script
    assert "prebuilt binary was uploaded" not in script.split("tk_libs_resolve")[0]  # the header no longer claims it
    assert os.path.exists(os.path.join(MODULE, "files", "prebuilt", "README"))


def test_terraform_apply_stages_the_tools_for_mi355x_hosts(tmp_path, monkeypatch):
    from triton_kubernetes_amd.executor.terraform import PREBUILT_VAR, TerraformExecutor, _takes, render
    from triton_kubernetes_amd.backend.local import LocalBackend
    from triton_kubernetes_amd.models import baremetal
    from triton_kubernetes_amd import versions
    from helpers import make_ctx

    be = LocalBackend(str(tmp_path / "state"))
    st = be.state("mgr")
    baremetal.new_manager(make_ctx({"manager_cloud_provider": "baremetal", "name": "mgr",
                                    "rancher_admin_password": "Pw-123456789", "host": "10.0.0.10", "ssh_user": "u",
                                    "bastion_host": "", "key_path": "k"}), st, "mgr")
    assert not _takes(st, PREBUILT_VAR)
    name = baremetal.new_cluster(make_ctx({"name": "dev", "k8s_version": versions.DEFAULT_K8S_VERSION,
                                           "k8s_network_provider": "canal"}), None, st)
    st.add_node(st.clusters()[name], "gpu", {"source": catalog.module_source(catalog.PACKAGE_ROOT,
                                                              "terraform/modules/bare-metal-mi355x-rancher-k8s-host", "x"),
                              "hostname": "gpu", "host": "10.0.0.21", "gpu_count": "8"})
    assert _takes(st, PREBUILT_VAR)
    doc = json.loads(render(st, (1, 5, 7), be, prebuilt_tools="/tmp/x/tk-prebuilt-tools").body)
    gpu = [m for m in doc["module"].values() if m["source"].endswith("bare-metal-mi355x-rancher-k8s-host")]
    assert gpu and all(m[PREBUILT_VAR] == f"${{var.{PREBUILT_VAR}}}" for m in gpu)
    assert doc["variable"][PREBUILT_VAR]["default"] == "/tmp/x/tk-prebuilt-tools"

    staged = {}

    def fake_stage(dest, binary=None, log=None):
        os.makedirs(dest)
        staged["dest"] = dest
        return {"gpu-burnin": "prebuilt"}

    monkeypatch.setattr(tools, "stage", fake_stage)
    ex = TerraformExecutor(version=(1, 5, 7))
    monkeypatch.setattr(ex, "_run", lambda wd, *args: None)
    with ex.workdir(st, be, stage=True) as wd:
        body = json.load(open(os.path.join(wd, "main.tf.json")))
        assert staged["dest"] == os.path.join(wd, "tk-prebuilt-tools") and os.path.isdir(staged["dest"])
        assert body["variable"][PREBUILT_VAR]["default"] == staged["dest"]
    staged.clear()
    with ex.workdir(st, be) as wd:  # destroy / output: nothing staged
        assert not staged


def test_machine_image_builds_with_the_same_stamped_function(node, tmp_path):
    from triton_kubernetes_amd.images import packer

    script = open(os.path.join(packer.FILES_DIR, "build-node-tools.sh")).read()
    assert script == tools.image_build_script()  # python -m triton_kubernetes_amd.node.tools rewrites it
    run, compiles, tmp = node
    bindir = tmp / "stubs"
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}", TK_SRC=str(tmp / "src"), TK_BIN=str(tmp / "img"),
               ROCM_PATH=str(tmp / "rocm"))
    # the image's last line runs the labeller: the stub compiler's output prints "built"
    proc = subprocess.run(["bash", "-c", script], capture_output=True, text=True, env=env, timeout=60)
    assert proc.returncode == 0, proc.stderr
    assert len(compiles()) == 3
    # a Terraform apply on a node made from that image: every tool is current, nothing compiled
    _staged(tmp)
    again = run(tmp / "img")
    assert again.returncode == 0 and len(compiles()) == 3
    assert again.stdout.count("installed copy is current") == 3


def test_direct_executor_uploads_only_tools_the_host_lacks(tmp_path, monkeypatch):
    from triton_kubernetes_amd.executor.direct import DirectExecutor
    from triton_kubernetes_amd.node.plan import TOOLS_DIR
    from triton_kubernetes_amd.ops import native
    from triton_kubernetes_amd.parallel.transport import HostRef, RecordingTransport

    host_stamps = {}

    class Host(RecordingTransport):
        def run_script(self, host, script, timeout=3600):
            super().run_script(host, script, timeout)
            if ".stamps/*.sha256" in script:
                return "".join(f"{n} {s}\n" for n, s in host_stamps.items())
            if "sudo tee" in script:
                name = script.split(".stamps/")[1].split(".sha256")[0]
                host_stamps[name] = script.split("echo ")[1].split(" |")[0]
            return ""

    monkeypatch.setattr(native, "executable", lambda name: f"/lib/{name}")
    t = Host()
    ex = DirectExecutor(transport=t)
    ref = HostRef("10.0.0.30", "u", "k", "")
    assert sorted(ex._upload_tools(ref)) == sorted(tools.TOOL_SOURCES)
    assert sorted(t.files) == sorted(f"{TOOLS_DIR}/{n}" for n in tools.TOOL_SOURCES)
    assert host_stamps == {n: tools.node_stamp(n) for n in tools.TOOL_SOURCES}
    assert ex._upload_tools(ref) == []  # re-apply: nothing sent
    host_stamps["gpu-burnin"] = "0" * 64  # built from other sources
    assert ex._upload_tools(ref) == ["gpu-burnin"]
