"""``migrate manager``: a document written against the reference's Terraform 0.11 modules
(``github.com/joyent/triton-kubernetes//terraform/modules/<name>?ref=master``) is pointed
at this framework's modules, checked, backed up and persisted."""

import json

import pytest

from triton_kubernetes_amd.backend import MemoryBackend
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.state import State
from triton_kubernetes_amd.terraform import hcl
from triton_kubernetes_amd.terraform.catalog import local_module_dir, module_from_source
from triton_kubernetes_amd.workflows.migrate import BACKUP_BLOB, migrate_manager, plan_migration

from helpers import make_ctx

REF = "github.com/joyent/triton-kubernetes//terraform/modules/{}?ref=master"


def reference_doc():
    """The shape the reference's ``create manager/cluster/node`` (bare metal) writes."""
    return {
        "terraform": {"backend": {"local": {"path": "terraform.tfstate"}}},
        "module": {
            "cluster-manager": {"source": REF.format("bare-metal-rancher"), "name": "mgr", "host": "10.0.0.10",
                                "ssh_user": "ubuntu", "key_path": "~/.ssh/id_rsa",
                                "rancher_admin_password": "s3cret"},
            "cluster_baremetal_prod": {"source": REF.format("bare-metal-rancher-k8s"), "name": "prod",
                                       "rancher_api_url": "${module.cluster-manager.rancher_url}",
                                       "rancher_access_key": "${module.cluster-manager.rancher_access_key}",
                                       "rancher_secret_key": "${module.cluster-manager.rancher_secret_key}",
                                       "k8s_version": "v1.11.3-rancher1-1"},
            "node_baremetal_prod_w-1": {
                "source": REF.format("bare-metal-rancher-k8s-host"), "hostname": "w-1", "host": "10.0.0.11",
                "rancher_api_url": "${module.cluster-manager.rancher_url}",
                "rancher_cluster_registration_token": "${module.cluster_baremetal_prod.rancher_cluster_registration_token}",
                "rancher_cluster_ca_checksum": "${module.cluster_baremetal_prod.rancher_cluster_ca_checksum}",
                "rancher_host_labels": {"worker": "true"}},
        },
    }


def _backend(doc):
    be = MemoryBackend()
    be.persist_state(State("mgr", json.dumps(doc).encode()))
    return be


def test_plan_rewrites_every_reference_source_to_the_packaged_modules():
    ctx = make_ctx({"cluster_manager": "mgr"})
    blocks, errors, warnings = plan_migration(ctx, reference_doc())
    assert not errors, errors
    assert sorted(blocks) == ["cluster-manager", "cluster_baremetal_prod", "node_baremetal_prod_w-1"]
    for key, block in blocks.items():
        info = module_from_source(block["source"])
        assert local_module_dir(block["source"]) == info.local_dir  # the packaged tree, on disk
        problems = hcl.check_inputs(info.local_dir, block)
        assert all(not p.startswith(("unsupported", "missing")) for p in problems)
    # failing validations of the new modules are reported, not fatal: the reference's
    # 0.11 modules accepted a 6-character Rancher password and a v1.11 release
    assert any("rancher_admin_password" in w and "12 characters" in w for w in warnings)
    assert any("k8s_version" in w for w in warnings), warnings
    assert not any(": plan: " in w for w in warnings), warnings  # every new module evaluates cleanly
    # arguments other than the source are carried over unchanged
    assert blocks["node_baremetal_prod_w-1"]["rancher_host_labels"] == {"worker": "true"}
    # an already-migrated document has nothing left to do
    doc2 = reference_doc()
    for k, b in blocks.items():
        doc2["module"][k] = b
    assert plan_migration(ctx, doc2)[0] == {}


def test_unknown_arguments_refuse_unless_dropped():
    doc = reference_doc()
    doc["module"]["cluster_baremetal_prod"]["aws_ami_id"] = "ami-1"  # not a variable of the new module
    ctx = make_ctx({"cluster_manager": "mgr"})
    _, errors, _ = plan_migration(ctx, doc)
    assert any("aws_ami_id" in e and "migrate_drop_unknown" in e for e in errors)
    blocks, errors, warnings = plan_migration(ctx, doc, drop_unknown=True)
    assert not errors and "aws_ami_id" not in blocks["cluster_baremetal_prod"]
    assert any("dropped 'aws_ami_id'" in w for w in warnings)


def test_missing_required_and_unknown_module_are_errors():
    doc = reference_doc()
    del doc["module"]["node_baremetal_prod_w-1"]["host"]
    doc["module"]["extra"] = {"source": REF.format("no-such-module")}
    _, errors, _ = plan_migration(make_ctx({"cluster_manager": "mgr"}), doc)
    assert any("missing required argument 'host'" in e for e in errors)
    assert any("unknown module source" in e for e in errors)


def test_migrate_manager_backs_up_and_persists():
    be = _backend(reference_doc())
    ctx = make_ctx({"cluster_manager": "mgr"})
    migrate_manager(ctx, be)
    after = be.state("mgr").doc
    assert all(not m["source"].startswith("github.com/joyent") for m in after["module"].values())
    assert after["terraform"] == reference_doc()["terraform"]
    backup = json.loads(be.read_blob("mgr", BACKUP_BLOB))
    assert backup["module"]["cluster-manager"]["source"] == REF.format("bare-metal-rancher")
    out = ctx.out.getvalue()
    assert "migrated" in out and "github.com/joyent" in out
    # running again is a no-op
    ctx2 = make_ctx({"cluster_manager": "mgr"})
    migrate_manager(ctx2, be)
    assert "already uses" in ctx2.out.getvalue()


def test_migrate_refusal_leaves_the_document_alone():
    doc = reference_doc()
    doc["module"]["cluster-manager"]["bogus"] = 1
    be = _backend(doc)
    with pytest.raises(TKError, match="migration refused"):
        migrate_manager(make_ctx({"cluster_manager": "mgr"}), be)
    assert be.state("mgr").doc == doc and be.read_blob("mgr", BACKUP_BLOB) is None


def test_migrate_refuses_a_document_changed_during_confirmation():
    from triton_kubernetes_amd.state import State

    be = _backend(reference_doc())
    ctx = make_ctx({"cluster_manager": "mgr"})
    real_confirm = ctx.confirm

    def confirm(*a, **kw):  # another CLI persists while this one asks
        changed = reference_doc()
        changed["module"]["cluster-manager"]["name"] = "renamed"
        be.persist_state(State("mgr", json.dumps(changed).encode()))
        return real_confirm(*a, **kw)

    ctx.confirm = confirm
    with pytest.raises(TKError, match="changed while the migration was being confirmed"):
        migrate_manager(ctx, be)
    assert be.state("mgr").doc["module"]["cluster-manager"]["name"] == "renamed"
    assert be.read_blob("mgr", BACKUP_BLOB) is None


def test_cli_migrate_manager_on_the_local_backend(tk_home):
    """``triton-kubernetes migrate manager`` end to end on ~/.triton-kubernetes/<manager>/."""
    import io

    from triton_kubernetes_amd.backend.local import LocalBackend
    from triton_kubernetes_amd.cli.main import run

    be = LocalBackend()
    be.persist_state(State("mgr", json.dumps(reference_doc()).encode()))
    cfg = tk_home / "m.yaml"
    cfg.write_text("backend_provider: local\ncluster_manager: mgr\n")
    out = io.StringIO()
    assert run(["--non-interactive", "--config", str(cfg), "migrate", "manager"], out=out) == 0, out.getvalue()
    doc = LocalBackend().state("mgr").doc
    assert not any(m["source"].startswith("github.com/joyent") for m in doc["module"].values())
    assert LocalBackend().read_blob("mgr", BACKUP_BLOB) is not None
    out = io.StringIO()
    assert run(["migrate", "cluster"], out=out) == 255
    assert out.getvalue() == 'invalid argument "cluster" for "triton-kubernetes migrate"\n'
