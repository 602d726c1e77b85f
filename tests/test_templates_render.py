"""Every templatefile() template of the 19 modules, rendered the way Terraform renders it
(``terraform/hcl.py:templatefile``: interpolation, %{if}/%{for}, ``~`` strip markers) with
both empty and filled-in values, then checked: shell templates with ``bash -n``, JSON
manifests with a JSON parser (and against the DirectExecutor's renderer)."""

import json
import os
import subprocess

import pytest

from triton_kubernetes_amd.k8s import addons
from triton_kubernetes_amd.terraform import hcl
from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

TEMPLATES = sorted(os.path.join(root, f) for root, _, files in os.walk(MODULES_DIR) for f in files
                   if f.endswith(".tftpl"))


def _values(names, filled):
    out = {}
    for n in names:
        if "count" in n:
            out[n] = 8 if filled else 1
        elif n == "gpu_burnin":
            out[n] = "full" if filled else "off"
        elif n == "rancher_node_role":
            out[n] = "worker"
        elif n.endswith("_b64"):
            out[n] = "Zm9v" if filled else ""
        elif n == "rccl_min_busbw":
            out[n] = 150 if filled else 0
        elif n == "gpu_partitions":
            out[n] = 8 if filled else 1
        elif n == "gpu_compute_partition":
            out[n] = "cpx" if filled else "spx"
        elif n == "gpu_memory_partition":
            out[n] = "nps2" if filled else "nps1"
        else:
            out[n] = f"v-{n}" if filled else ""
    return out


def test_templates_found():
    assert len(TEMPLATES) >= 22


@pytest.mark.parametrize("path", TEMPLATES, ids=lambda p: os.path.relpath(p, MODULES_DIR))
@pytest.mark.parametrize("filled", [False, True])
def test_template_renders_to_valid_output(path, filled):
    src = open(path, encoding="utf-8").read()
    names = hcl.template_names(hcl.parse_template(src, path))
    text = hcl.templatefile(src, _values(names, filled), path)
    assert "${" not in text.replace("$${", "") or path.endswith(".sh.tftpl")  # shell may use ${VAR}
    if path.endswith(".sh.tftpl"):
        proc = subprocess.run(["bash", "-n"], input=text, capture_output=True, text=True)
        assert proc.returncode == 0, f"{path}: {proc.stderr}\n{text}"
    elif path.endswith(".json.tftpl"):
        doc = json.loads(text)
        assert doc["object"]["metadata"]["name"]
        # the DirectExecutor's renderer gives byte-identical output
        assert addons.render_template(src, _values(names, filled)) == text


def test_strip_markers_and_conditionals():
    src = "a\n%{ if x != \"\" ~}\nX=${x}\n%{ endif ~}\nb\n%{ for k, v in m ~}\n${k}=${v}\n%{ endfor ~}\nend"
    assert hcl.templatefile(src, {"x": "1", "m": {"p": 1, "q": "z"}}) == "a\nX=1\nb\np=1\nq=z\nend"
    assert hcl.templatefile(src, {"x": "", "m": {}}) == "a\nb\nend"
    assert hcl.templatefile("${a > 1 && b == \"y\" ? \"hi\" : \"lo\"}", {"a": 2, "b": "y"}) == "hi"
    with pytest.raises(hcl.TemplateError, match="undefined variable"):
        hcl.templatefile("${nope}", {})
