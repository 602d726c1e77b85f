"""Machine-image templates (reference packer/) and the bundled host scripts."""

import json
import os
import subprocess

import pytest

from triton_kubernetes_amd.images import packer

BUNDLED = sorted(f[:-5] for f in os.listdir(packer.TEMPLATES_DIR) if f.endswith(".yaml"))


def test_bundled_templates_present():
    assert BUNDLED == ["mi355x-node", "rancher-agent", "rancher-host", "rancher-server"]


@pytest.mark.parametrize("name", BUNDLED)
def test_bundled_templates_render(name):
    doc = json.loads(packer.render_template(packer.resolve(name)))
    assert isinstance(doc["variables"], dict) and doc["variables"]["files_dir"] == packer.FILES_DIR
    assert doc["builders"] and all(isinstance(b, dict) and "type" in b for b in doc["builders"])
    assert all(isinstance(p, dict) and "type" in p for p in doc["provisioners"])  # flattened
    for p in doc["provisioners"]:
        if "script" in p:
            path = p["script"].replace("{{user `files_dir`}}", packer.FILES_DIR)
            assert os.path.isfile(path), path


def test_include_flatten_and_variables(tmp_path):
    (tmp_path / "sub").mkdir()
    (tmp_path / "sub" / "vars.yaml").write_text("a: 1\nb: 2\n")
    (tmp_path / "sub" / "steps.yaml").write_text("- type: shell\n  inline: [one]\n- type: shell\n  inline: [two]\n")
    (tmp_path / "t.yaml").write_text(
        "variables:\n- !include sub/vars.yaml\n- b: 3\nbuilders:\n- type: null\n"
        "provisioners:\n- !include sub/steps.yaml\n- type: file\n  source: x\n")
    doc = packer.load_template(str(tmp_path / "t.yaml"))
    assert doc["variables"] == {"a": 1, "b": 3}
    assert [p.get("inline", ["file"])[0] for p in doc["provisioners"]] == ["one", "two", "file"]
    out = packer.render_template(str(tmp_path / "t.yaml"), {"a": "9"})
    assert json.loads(out)["variables"]["a"] == "9"


def test_include_cycle_and_missing(tmp_path):
    (tmp_path / "a.yaml").write_text("x: !include b.yaml\n")
    (tmp_path / "b.yaml").write_text("y: !include a.yaml\n")
    with pytest.raises(packer.TemplateError, match="include cycle"):
        packer.load_template(str(tmp_path / "a.yaml"))
    with pytest.raises(packer.TemplateError, match="Template not found"):
        packer.load_template(str(tmp_path / "nope.yaml"))


def test_unsafe_tags_rejected(tmp_path):
    import yaml

    (tmp_path / "evil.yaml").write_text("x: !!python/object/apply:os.system ['echo pwned']\n")
    with pytest.raises(yaml.YAMLError):
        packer.load_template(str(tmp_path / "evil.yaml"))


def test_cli_exit_codes(tmp_path, capsys):
    assert packer.main([]) == 1
    assert packer.main([str(tmp_path / "missing.yaml")]) == 2
    assert packer.main(["rancher-host", "docker_version=25.0"]) == 0
    assert json.loads(capsys.readouterr().out)["variables"]["docker_version"] == "25.0"


@pytest.mark.parametrize("script", ["install-docker.sh", "build-node-tools.sh"])
def test_host_scripts_valid_bash(script):
    path = os.path.join(packer.FILES_DIR, script)
    assert os.access(path, os.X_OK)
    assert subprocess.run(["bash", "-n", path], capture_output=True).returncode == 0


def test_install_docker_dry_run_ubuntu(tmp_path):
    """Dry run against a fake /etc/os-release: prints the apt plan, touches nothing."""
    src = open(os.path.join(packer.FILES_DIR, "install-docker.sh")).read()
    osrel = tmp_path / "os-release"
    osrel.write_text('ID=ubuntu\nVERSION_CODENAME=jammy\n')
    script = src.replace("/etc/os-release", str(osrel))
    bindir = tmp_path / "bin"
    bindir.mkdir()
    for tool in ("dpkg", "apt-cache"):
        p = bindir / tool
        p.write_text("#!/bin/sh\necho amd64\n")
        p.chmod(0o755)
    env = {"PATH": f"{bindir}:/usr/bin:/bin", "DOCKER_VERSION": "24.0"}
    proc = subprocess.run(["bash", "-s", "--", "--dry-run", "--mirror", "Aliyun"], input=script, env=env,
                          capture_output=True, text=True)
    assert proc.returncode == 0, proc.stderr
    assert "mirrors.aliyun.com/docker-ce/linux/ubuntu jammy stable" in proc.stdout
    assert "docker-ce=24.0" in proc.stdout
    bad = subprocess.run(["bash", "-s", "--", "--mirror", "Nowhere"], input=script, env=env, capture_output=True,
                         text=True)
    assert bad.returncode == 64
