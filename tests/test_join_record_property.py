"""The join record is written by a shell line on SSH / Terraform nodes
(``node/cleanup.py:join_record_shell``) and by the agent in Python, and read by the next
join's guard and by the teardown (both with ``sed``) and by the agent (JSON).  Property
test over generated servers, hostnames and agent images -- shell metacharacters, quotes and
non-ASCII in the server URL included: the record bash writes is the JSON the Python side
writes, and the guard's and the teardown's ``sed`` read back its cluster and agent image."""

import json
import re
import subprocess

from hypothesis import given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.node import cleanup

SERVERS = st.builds(lambda host, path: f"https://{host}{path}", st.from_regex(r"[a-z0-9.-]{1,20}(:[0-9]{2,5})?",
                                                                                fullmatch=True),
                    st.text(alphabet=st.characters(blacklist_categories=("Cs", "Cc")), max_size=16))
HOSTS = st.from_regex(r"[a-z0-9]([a-z0-9-]{0,20}[a-z0-9])?", fullmatch=True)
IMAGES = st.one_of(st.just(""), st.from_regex(r"([a-z0-9.-]+(:[0-9]+)?/)?[a-z0-9]+(/[a-z0-9_.-]+)?:[A-Za-z0-9_.-]{1,10}",
                                              fullmatch=True))

GUARD_SED = re.search(r"_tk_prev=\$\(sed -n '(.*?)'", cleanup.join_guard_shell("https://x", "t")).group(1)
IMAGE_SED = re.search(r"rec_img=\$\(sed -n '(.*?)'", cleanup.cleanup_script()).group(1)


@settings(max_examples=150, deadline=None)
@given(SERVERS, st.text(min_size=1, max_size=12), st.sampled_from(["rke1", "rke2"]), HOSTS, IMAGES)
def test_shell_record_is_the_python_record_and_reads_back(tmp_path_factory, server, token, dist, host, image):
    root = tmp_path_factory.mktemp("host")
    line = cleanup.join_record_shell(server, token, dist, host, image)
    prog = "sudo() { \"$@\"; }\n" + line + \
        f"f=\"$TK_HOST_ROOT{cleanup.JOIN_RECORD}\"\nsed -n '{GUARD_SED}' \"$f\"\nsed -n '{IMAGE_SED}' \"$f\"\n"
    out = subprocess.run(["bash", "-c", prog], env={"TK_HOST_ROOT": str(root), "PATH": "/usr/bin:/bin"},
                         capture_output=True, text=True, check=True).stdout.splitlines()
    want = cleanup.join_record(server, token, dist, host, image)
    with open(f"{root}{cleanup.JOIN_RECORD}", encoding="utf-8") as fh:
        assert json.load(fh) == want
    assert out[0] == want["cluster"]
    assert out[1:] == ([image] if image else [])
