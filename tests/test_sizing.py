"""Cloud defaults coherent with the pinned stack (``sizing.py``).

For every provider the size the CLI emits by default equals the module variable's
default, and that size meets the Rancher v2.8 server minimum (managers) or the node
minimum (hosts); a size known to be too small is refused with the reason.  The AWS AMI
picker lists the Ubuntu LTS the Docker 24.0 installer supports (reference
``create/manager_aws.go:426-436`` filtered xenial for its Docker 17.03).
"""

import os

import pytest

from triton_kubernetes_amd import sizing
from triton_kubernetes_amd.cloud import aws as aws_cloud
from triton_kubernetes_amd.errors import ConfigError
from triton_kubernetes_amd.models import aws
from triton_kubernetes_amd.terraform import hcl
from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

from helpers import make_ctx

MODULE = {("aws", "manager"): "aws-rancher", ("aws", "host"): "aws-rancher-k8s-host",
          ("gcp", "manager"): "gcp-rancher", ("gcp", "host"): "gcp-rancher-k8s-host",
          ("azure", "manager"): "azure-rancher", ("azure", "host"): "azure-rancher-k8s-host",
          ("triton", "manager"): "triton-rancher", ("triton", "host"): "triton-rancher-k8s-host",
          ("vsphere", "host"): "vsphere-rancher-k8s-host"}


def _module_default(module: str, var: str):
    body = hcl.check_module(os.path.join(MODULES_DIR, module)).files["variables.tf"]
    blk = next(b for b in body.blocks if b.type == "variable" and b.labels == [var])
    return blk.body.attr("default").expr.value


@pytest.mark.parametrize("provider,kind", sorted(sizing.DEFAULT_SIZES))
def test_module_default_is_the_cli_default_and_meets_the_minimum(provider, kind):
    var, value = sizing.default_size(provider, kind)
    assert _module_default(MODULE[(provider, kind)], var) == value
    mem = sizing.memory_gib(provider, value)
    floor = sizing.SERVER_MIN_GIB if kind == "manager" else sizing.NODE_MIN_GIB
    assert mem is not None and mem >= floor, (provider, kind, value, mem)
    sizing.check_size(provider, kind, value)  # does not raise


def test_aws_cli_prompt_default_is_the_module_default():
    """The AWS instance-type prompt's default (the reference pre-filled t2.micro) is the
    module's default for that kind; non-interactive runs must name it (reference error)."""
    for kind, module in (("manager", "aws-rancher"), ("host", "aws-rancher-k8s-host")):
        ctx = make_ctx({}, answers=[""], non_interactive=False)
        assert aws._instance_type(ctx, kind) == _module_default(module, "aws_instance_type") == \
            sizing.default_size("aws", kind)[1]
    with pytest.raises(ConfigError, match="aws_instance_type must be specified"):
        aws._instance_type(make_ctx({}), "manager")
    with pytest.raises(ConfigError, match="t2.micro' has 1 GiB"):
        aws._instance_type(make_ctx({"aws_instance_type": "t2.micro"}), "manager")


@pytest.mark.parametrize("provider,kind,value", [
    ("aws", "manager", "t2.micro"), ("aws", "host", "t3.small"), ("gcp", "manager", "n1-standard-1"),
    ("azure", "manager", "Standard_A0"), ("triton", "manager", "k4-highcpu-kvm-3.75G"),
    ("triton", "host", "k4-highcpu-kvm-1.75G"), ("vsphere", "host", "2048")])
def test_undersized_choices_are_refused(provider, kind, value):
    with pytest.raises(ConfigError, match="needs at least 4 GiB"):
        sizing.check_size(provider, kind, value)


def test_listing_memory_decides_for_unknown_sizes():
    sizing.check_size("triton", "manager", "custom-pkg", memory=8.0)
    with pytest.raises(ConfigError, match="custom-pkg"):
        sizing.check_size("triton", "manager", "custom-pkg", memory=2.0)
    sizing.check_size("aws", "manager", "x9.unknown")  # unknown and unlisted: not held against it


def test_aws_ami_filter_is_the_supported_ubuntu_lts():
    assert aws_cloud.UBUNTU_AMI_FILTER == "*hvm-ssd/ubuntu-jammy-22.04-amd64-server*"
    assert "xenial" not in aws_cloud.UBUNTU_AMI_FILTER
    assert _module_default("gcp-rancher", "gcp_image").endswith("ubuntu-2204-lts")
    assert _module_default("triton-rancher", "triton_image_name") == sizing.TRITON_IMAGE_PREFIX
