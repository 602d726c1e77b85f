"""Terminal prompter (promptui replacement) driven through in-memory streams, plus the full
interactive `create manager` flow over it — the reference could not test interactive paths."""

import io

import pytest

from triton_kubernetes_amd.config import Context, Settings
from triton_kubernetes_amd.config.prompt import NoPrompter, TerminalPrompter
from triton_kubernetes_amd.errors import PromptAborted, TKError


def _tp(text):
    out = io.StringIO()
    return TerminalPrompter(io.StringIO(text), out), out


def test_select_by_number_name_and_invalid():
    p, out = _tp("9\nflannel\n")
    assert p.select("Network", ["calico", "flannel"]) == (1, "flannel")
    assert "invalid choice" in out.getvalue()
    p, out = _tp("1\n")
    assert p.select("Network", ["calico", "flannel"]) == (0, "calico")
    assert "✔ Network: calico" in out.getvalue()


def test_searchable_select_filters():
    p, out = _tp("east\n2\n")
    idx, val = p.select("Region", ["us-west-1", "us-east-1", "eu-west-1", "us-east-2"], searchable=True)
    assert (idx, val) == (3, "us-east-2")
    assert "text to filter" in out.getvalue()


def test_prompt_default_and_validation():
    p, out = _tp("\n")
    assert p.prompt("SSH User", default="ubuntu") == "ubuntu"
    p, out = _tp("Bad_Name\ngood-name\n")
    v = (lambda s: None if "_" not in s else "Invalid Cluster Name")
    assert p.prompt("Cluster Name", validate=v) == "good-name"
    assert "✗ Invalid Cluster Name" in out.getvalue()


def test_select_with_add_and_eof():
    p, _ = _tp("3\nmy-new-key\n")
    assert p.select_with_add("Key Pair", ["a", "b"], "Upload new key") == (-1, "my-new-key")
    p, _ = _tp("")
    with pytest.raises(PromptAborted):
        p.prompt("anything")


def test_confirm_and_no_prompter():
    p, _ = _tp("2\n")
    assert p.confirm("Proceed") is False
    with pytest.raises(TKError, match="interactive prompt 'x' reached in non-interactive mode"):
        NoPrompter().prompt("x")


def test_interactive_create_manager_over_terminal(tk_home):
    """Whole bare-metal `create manager` dialogue answered over a terminal stream."""
    from triton_kubernetes_amd.backend import MemoryBackend
    from triton_kubernetes_amd.workflows import new_manager

    key = tk_home / "id_rsa"
    key.write_text("not-read-for-baremetal")
    answers = "\n".join([
        "lab",          # Cluster Manager Name
        "",             # Private Registry [None]
        "",             # Rancher Server Image [Default]
        "",             # Rancher Agent Image [Default]
        "s3cret-passw0rd",  # UI admin password
        "10.0.0.9",     # host
        "",             # ssh user [ubuntu]
        "",             # Bastion Host [None]
        str(key),       # key path
        "1",            # Proceed? -> Yes
    ]) + "\n"
    out = io.StringIO()
    ctx = Context(settings=Settings({"manager_cloud_provider": "baremetal", "executor": "terraform"}, env={}),
                  prompter=TerminalPrompter(io.StringIO(answers), out), out=out)
    applied = []

    class Exec:
        name = "recording"

        def apply(self, state, backend):
            applied.append(state.manager())

    ctx.executor_factory = lambda ctx, state=None: Exec()
    be = MemoryBackend()
    try:
        new_manager(ctx, be)
    except TKError as exc:  # surface the dialogue on failure
        raise AssertionError(out.getvalue()) from exc
    m = be.state("lab").manager()
    assert m["host"] == "10.0.0.9" and m["ssh_user"] == "ubuntu" and m["rancher_admin_password"] == "s3cret-passw0rd"
