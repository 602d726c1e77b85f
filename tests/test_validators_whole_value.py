"""Every Python validator matches the whole value: Python's ``$`` also matches before a
final newline, so ``pattern.match`` let ``"name\\n"`` through where the reference's Go (RE2)
regexes and Kubernetes refuse it.  The validators now use ``fullmatch``; Terraform-side
patterns go through ``hcl.re2_pattern``, which already turned ``$`` into ``\\Z``."""

import pytest

from triton_kubernetes_amd import versions
from triton_kubernetes_amd.models import aws, common
from triton_kubernetes_amd.node import agent_steps, metrics


@pytest.mark.parametrize("good,bad", [("gpu-cluster", "gpu-cluster\n"), ("a.b", "a.b\n")])
def test_cluster_names(good, bad):
    assert common.DNS1123_RE.fullmatch(good) and not common.DNS1123_RE.fullmatch(bad)


@pytest.mark.parametrize("pattern,good", [
    (agent_steps._HOSTNAME_RE, "mi355x-gpu-1"), (agent_steps._IMAGE_RE, "rancher/rancher-agent:v2.10.3"),
    (agent_steps._TOKEN_RE, "abc123"), (agent_steps._URL_RE, "https://10.0.0.1"),
    (agent_steps._TAINT_RE, "amd.com/gpu-unhealthy=true:NoSchedule")])
def test_agent_step_values(pattern, good):
    assert agent_steps._check(pattern, good, "x") == good
    with pytest.raises(ValueError):
        agent_steps._check(pattern, good + "\n", "x")


def test_versions_and_paths():
    assert versions.k8s_minor("v1.31.6+rke2r1") is not None
    assert versions.k8s_minor("v1.31.6+rke2r1\n") is None
    assert aws.EBS_DEVICE_RE.fullmatch("/dev/sdf") and not aws.EBS_DEVICE_RE.fullmatch("/dev/sdf\n")
    assert metrics.textfile_dir_of({"gpu_metrics_textfile": "/var/lib/node_exporter/"}) == "/var/lib/node_exporter"
