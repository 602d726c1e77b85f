"""Drop-in parity of the Terraform wire contract: every variable a reference module declares
is declared by the module of the same name here, so a ``main.tf.json`` written for the
reference's modules (its CLI's ``module.<name>`` blocks, ``/root/reference/create/*.go``)
never meets an "Unsupported argument"; and every output it declares exists here, so the
interpolations other modules' blocks make (``${module.<manager>.rancher_url}``, §3.6 of
SURVEY.md) resolve.  Reads the reference's ``variables.tf`` files; skipped
where the reference tree is not present."""

import glob
import os
import re

import pytest

from triton_kubernetes_amd.terraform import catalog

REF = "/root/reference/terraform/modules"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")


def _declared(module_dir: str, kind: str = "variable") -> set:
    names = set()
    for path in glob.glob(os.path.join(module_dir, "*.tf")):
        with open(path, encoding="utf-8") as fh:
            names |= set(re.findall(kind + r'\s+"([^"]+)"', fh.read()))
    return names


def _reference_modules():
    return sorted(m for m in os.listdir(REF) if _declared(os.path.join(REF, m))) if os.path.isdir(REF) else []


def test_every_reference_module_exists_here():
    mods = _reference_modules()
    assert len(mods) == len(catalog.REFERENCE_MODULES) == 17
    for m in mods:
        assert os.path.isdir(os.path.join(catalog.MODULES_DIR, m)), m


@pytest.mark.parametrize("module", _reference_modules())
def test_every_reference_variable_is_accepted(module):
    theirs = _declared(os.path.join(REF, module))
    ours = _declared(os.path.join(catalog.MODULES_DIR, module))
    assert theirs <= ours, f"{module}: not declared here: {sorted(theirs - ours)}"


@pytest.mark.parametrize("module", _reference_modules())
def test_every_reference_output_exists(module):
    theirs = _declared(os.path.join(REF, module), "output")
    ours = _declared(os.path.join(catalog.MODULES_DIR, module), "output")
    assert theirs <= ours, f"{module}: outputs missing here: {sorted(theirs - ours)}"
