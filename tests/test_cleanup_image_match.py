"""The RKE1 teardown picks containers by image repository in three places that must agree:
``node/cleanup.py:image_repository`` / ``repo_matches`` (the agent path), and in the
teardown script the bash ``_tk_repo`` (the recorded and Terraform-given agent images) and the
awk filter over ``docker ps -a`` (the SSH and Terraform paths).  Property test over generated
image references: any registry (with port), path depth, tag and digest."""

import re
import subprocess

from hypothesis import given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.node import cleanup

SCRIPT = cleanup.cleanup_script()
AWK = re.search(r"awk -v repos=\"\$repos\" '(.*?)' \|\| true", SCRIPT, re.S).group(1)
TK_REPO = re.search(r"^\s*(_tk_repo\(\) \{.*?\})\s*$", SCRIPT, re.M).group(1)

_comp = st.from_regex(r"[a-z0-9]([a-z0-9_.-]{0,6}[a-z0-9])?", fullmatch=True)
_registry = st.sampled_from(["", "docker.io/", "quay.io/", "reg.example.com:5000/", "localhost:5000/",
                             "10.0.0.7:443/"])
_path = st.one_of(
    st.sampled_from(["rancher/rancher-agent", "rancher/rke-tools", "rancher/hyperkube", "rancher-agent",
                     "myrancher/rancher-agent", "rancher/rancher-agent-extra", "mirror/rancher/rancher-agent"]),
    st.lists(_comp, min_size=1, max_size=3).map("/".join))
_tag = st.one_of(st.just(""), st.from_regex(r":[A-Za-z0-9_][A-Za-z0-9_.-]{0,11}", fullmatch=True))
_digest = st.one_of(st.just(""), st.from_regex(r"@sha256:[0-9a-f]{64}", fullmatch=True))
IMAGES = st.builds(lambda r, p, t, d: r + p + t + d, _registry, _path, _tag, _digest)
REPOS = st.lists(st.one_of(st.sampled_from(list(cleanup.RKE1_REPOS) + ["custom/agent", "reg.example.com:5000/x/agent"]),
                           st.builds(lambda r, p: r + p, _registry, _path)), min_size=1, max_size=5)


def _awk_ids(images, repos):
    lines = "".join(f"id{i} {img}\n" for i, img in enumerate(images))
    out = subprocess.run(["awk", "-v", "repos=" + " ".join(repos), AWK], input=lines, capture_output=True,
                         text=True, check=True).stdout
    return {int(x[2:]) for x in out.split()}


@settings(max_examples=150, deadline=None)
@given(st.lists(IMAGES, min_size=1, max_size=12), REPOS)
def test_awk_filter_agrees_with_repo_matches(images, repos):
    want = {i for i, img in enumerate(images) if cleanup.repo_matches(img, repos)}
    assert _awk_ids(images, repos) == want


@settings(max_examples=150, deadline=None)
@given(st.lists(IMAGES, min_size=1, max_size=12))
def test_bash_tk_repo_agrees_with_image_repository(images):
    prog = TK_REPO + '\nfor a in "$@"; do _tk_repo "$a"; done\n'
    out = subprocess.run(["bash", "-c", prog, "tk"] + images, capture_output=True, text=True, check=True).stdout
    assert out.splitlines() == [cleanup.image_repository(i) for i in images]


def test_no_match_across_a_path_boundary():
    repos = ["rancher/rancher-agent"]
    for img, hit in (("rancher/rancher-agent:v2.10.3", True), ("reg:5000/rancher/rancher-agent@sha256:" + "a" * 64, True),
                     ("myrancher/rancher-agent:v1", False), ("rancher/rancher-agent-extra:v1", False),
                     ("reg:5000/rancher-agent:v1", False)):
        assert cleanup.repo_matches(img, repos) is hit, img
        assert (_awk_ids([img], repos) == {0}) is hit, img
