"""The node's RCCL environment file (``/etc/rccl/rccl.env``) has three readers: the node
agent (``parallel/rccl_env.py:parse_env_file``), its systemd unit (``EnvironmentFile=``) and
the SSH / Terraform bootstrap scripts, which source it with bash.  Property test: every
environment ``env_problems`` accepts renders to a file that the Python reader and bash both
read back as exactly that environment; and what it refuses never reaches a file."""

import re
import subprocess

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.parallel import rccl_env

KEYS = st.builds(lambda p, rest: f"{p}_{rest}", st.sampled_from(["NCCL", "RCCL", "HSA"]),
                 st.from_regex(r"[A-Z0-9][A-Z0-9_]{0,20}", fullmatch=True)).filter(
    lambda k: not re.search(rccl_env.ENV_KEY_DENY_RE, k))
ITEM = st.from_regex(r"[A-Za-z0-9_.:=^+-]{0,12}(/[0-9]{1,3})?", fullmatch=True)
VALUES = st.lists(ITEM, min_size=1, max_size=4).map(",".join).filter(lambda v: len(v) <= rccl_env.ENV_VALUE_MAX)
ENVS = st.dictionaries(KEYS, VALUES, max_size=8)


@settings(max_examples=200, deadline=None)
@given(ENVS)
def test_accepted_env_round_trips_through_python_and_bash(env):
    assert rccl_env.env_problems(env) == []
    text = rccl_env.render_env_file(env)
    assert rccl_env.parse_env_file(text) == env
    if env:
        prog = "set -a\n. /dev/stdin\nset +a\n" + "".join(f'printf "%s\\0" "${{{k}}}"\n' for k in sorted(env))
        out = subprocess.run(["bash", "-c", prog], input=text, capture_output=True, text=True, check=True).stdout
        assert out.split("\0")[:-1] == [env[k] for k in sorted(env)]


@settings(max_examples=100, deadline=None)
@given(st.dictionaries(st.text(min_size=1, max_size=12), st.text(max_size=12), min_size=1, max_size=3))
def test_refused_env_never_renders(env):
    if rccl_env.env_problems(env):
        with pytest.raises(ValueError):
            rccl_env.render_env_file(env)
    else:
        assert rccl_env.parse_env_file(rccl_env.render_env_file(env)) == {str(k): str(v) for k, v in env.items()}
