"""Provider plugins (L4): non-interactive configs, validations, interactive flows.

Every provider's manager / cluster / node builder is driven through the real
``Context.resolve`` contract with a :class:`FakeCloud` for the cloud listings.
"""

import json
import os

import pytest

from triton_kubernetes_amd import __version__
from triton_kubernetes_amd.cloud.fake import FakeCloud
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.models import aws, azure, baremetal, gcp, triton, vsphere
from triton_kubernetes_amd.state import State
from triton_kubernetes_amd.terraform import catalog

from helpers import assert_blocks_match_modules, make_ctx, make_ssh_key

BASE_MGR = {"rancher_admin_password": "tk-admin-pw-0123"}
BASE_CLUSTER = {"name": "dev", "k8s_version": "v1.28.10-rancher1-1", "k8s_network_provider": "flannel"}
NODE_BASE = {"rancher_host_label": "worker", "node_count": 2, "hostname": "dev-w"}


@pytest.fixture
def key(tmp_path):
    return make_ssh_key(tmp_path / "id_rsa")


@pytest.fixture
def gcp_creds(tmp_path, key):
    path = tmp_path / "creds.json"
    path.write_text(json.dumps({"project_id": "my-project", "client_email": "sa@x.iam", "private_key":
                                open(key).read(), "token_uri": "https://oauth2.example/token"}))
    return str(path)


def _err(fn, *args):
    with pytest.raises(TKError) as exc:
        fn(*args)
    return str(exc.value)


# --- bare metal -------------------------------------------------------------------------------
def test_baremetal_manager_document():
    st = State("mgr")
    baremetal.new_manager(make_ctx(dict(BASE_MGR, host="10.0.0.10", ssh_user="ubuntu", bastion_host="",
                                        key_path="~/.ssh/id_rsa")), st, "mgr")
    m = st.manager()
    # default: this package's own module tree, named location-free (resolved only when run)
    assert m["source"] == "tk::terraform/modules/bare-metal-rancher?ref=v" + __version__
    assert os.path.isfile(os.path.join(catalog.local_module_dir(m["source"]), "main.tf"))
    assert list(m) == ["source", "name", "rancher_admin_password", "host", "ssh_user", "key_path"]
    assert m["key_path"] == "~/.ssh/id_rsa"  # not expanded (reference quirk Q11 kept)
    assert_blocks_match_modules(st)


def test_baremetal_manager_required_keys():
    st = State("mgr")
    assert _err(baremetal.new_manager, make_ctx(BASE_MGR), st, "m") == "host must be specified"
    assert _err(baremetal.new_manager, make_ctx(dict(BASE_MGR, host="h")), st, "m") == "ssh_user must be specified"
    assert _err(baremetal.new_manager, make_ctx(dict(BASE_MGR, host="h", ssh_user="u")), st, "m") == \
        "bastion_host must be specified"
    assert _err(baremetal.new_manager, make_ctx({"host": "h"}), st, "m") == "UI Admin Password must be specified"


def test_baremetal_source_override_env():
    st = State("mgr")
    ctx = make_ctx(dict(BASE_MGR, host="h", ssh_user="u", bastion_host="", key_path="k"),
                   env={"SOURCE_URL": "github.com/me/fork", "SOURCE_REF": "dev"})
    baremetal.new_manager(ctx, st, "m")
    assert st.manager()["source"] == "github.com/me/fork//terraform/modules/bare-metal-rancher?ref=dev"


def test_baremetal_cluster_and_nodes():
    st = State("mgr")
    name = baremetal.new_cluster(make_ctx(BASE_CLUSTER), None, st)
    key = st.clusters()[name]
    assert key == "cluster_baremetal_dev"
    cfg = st.module(key)
    assert cfg["rancher_api_url"] == "${module.cluster-manager.rancher_url}"
    hosts = baremetal.new_node(make_ctx(dict(NODE_BASE, ssh_user="u", bastion_host="b", key_path="k",
                                             hosts=["10.0.0.1", "10.0.0.2"])), "mgr", key, None, st)
    assert hosts == ["dev-w-1", "dev-w-2"]
    n = st.module("node_baremetal_dev_dev-w-2")
    assert n["host"] == "10.0.0.2" and n["rancher_host_labels"] == {"worker": "true"}
    assert n["rancher_cluster_registration_token"] == "${module.cluster_baremetal_dev.rancher_cluster_registration_token}"
    # same prefix again in the same session: numbering continues (Q1 fixed)
    more = baremetal.new_node(make_ctx(dict(NODE_BASE, node_count=1, ssh_user="u", bastion_host="", key_path="k",
                                            hosts=["10.0.0.3"])), "mgr", key, None, st)
    assert more == ["dev-w-3"]
    assert_blocks_match_modules(st)


def test_baremetal_node_errors():
    st = State("mgr")
    key = st.add_cluster("baremetal", "dev", {"name": "dev"})
    ctx = make_ctx(dict(NODE_BASE, ssh_user="u", bastion_host="", key_path="k", hosts=["only-one"]))
    assert _err(baremetal.new_node, ctx, "m", key, None, st) == "not enough hosts"
    ctx = make_ctx(dict(NODE_BASE, ssh_user="u", bastion_host="", key_path="k"))
    assert _err(baremetal.new_node, ctx, "m", key, None, st) == "hosts must be specified"
    ctx = make_ctx(dict(NODE_BASE, rancher_host_label="gpu"))
    assert _err(baremetal.new_node, ctx, "m", key, None, st) == \
        "Invalid rancher_host_label 'gpu', must be 'worker', 'etcd' or 'control'"
    ctx = make_ctx(dict(NODE_BASE, node_count="x"))
    assert _err(baremetal.new_node, ctx, "m", key, None, st) == "node_count must be a valid number. Found 'x'."
    ctx = make_ctx(dict(NODE_BASE, node_count=0))
    assert _err(baremetal.new_node, ctx, "m", key, None, st) == "node_count must be greater than 0. Found '0'."
    # Q3 fix: non-interactive errors instead of prompting
    assert _err(baremetal.new_node, make_ctx({}), "m", key, None, st) == "rancher_host_label must be specified"
    assert _err(baremetal.new_node, make_ctx({"rancher_host_label": "etcd", "node_count": 1}), "m", key, None,
                st) == "hostname must be specified"


def test_mi355x_node_and_addons():
    st = State("mgr")
    name = baremetal.new_cluster(make_ctx(dict(BASE_CLUSTER, gpu_addons=True)), None, st)
    assert st.module("addons_baremetal_dev")["rancher_cluster_id"] == "${module.cluster_baremetal_dev.rancher_cluster_id}"
    key = st.clusters()[name]
    baremetal.new_node(make_ctx(dict(NODE_BASE, ssh_user="u", bastion_host="", key_path="k", gpu="mi355x",
                                     hosts=["a", "b"], rccl_env={"NCCL_SOCKET_IFNAME": "eth0"})), "m", key, None, st)
    n = st.module("node_baremetal_dev_dev-w-1")
    assert n["source"].startswith("tk::terraform/modules/bare-metal-mi355x-rancher-k8s-host?ref=")
    assert n["gpu_count"] == "8" and n["gpu_burnin"] == "full" and n["gpu_product"] == "MI355X"
    assert n["rccl_env"]["NCCL_SOCKET_IFNAME"] == "eth0" and n["rccl_env"]["HSA_FORCE_FINE_GRAIN_PCIE"] == "1"
    assert_blocks_match_modules(st)
    baremetal.new_node(make_ctx(dict(NODE_BASE, node_count=1, ssh_user="u", bastion_host="", key_path="k",
                                     gpu="mi355x", hosts=["c"], rccl_min_busbw="150")), "m", key, None, st)
    assert st.module("node_baremetal_dev_dev-w-3")["rccl_min_busbw"] == "150"
    assert_blocks_match_modules(st)
    baremetal.new_node(make_ctx(dict(NODE_BASE, node_count=1, ssh_user="u", bastion_host="", key_path="k",
                                     gpu="mi355x", hosts=["e"], gpu_link_min_frac="0.7")), "m", key, None, st)
    assert st.module("node_baremetal_dev_dev-w-4")["gpu_link_min_frac"] == "0.7"
    assert_blocks_match_modules(st)
    frac = make_ctx(dict(NODE_BASE, node_count=1, ssh_user="u", bastion_host="", key_path="k", gpu="mi355x",
                         hosts=["f"], gpu_link_min_frac="2"))
    assert _err(baremetal.new_node, frac, "m", key, None, st) == \
        "gpu_link_min_frac must be a number between 0 and 1. Found '2'."
    neg = make_ctx(dict(NODE_BASE, node_count=1, ssh_user="u", bastion_host="", key_path="k", gpu="mi355x",
                        hosts=["d"], rccl_min_busbw="-1"))
    assert _err(baremetal.new_node, neg, "m", key, None, st) == "rccl_min_busbw must be a non-negative number. Found '-1'."
    bad = make_ctx(dict(NODE_BASE, ssh_user="u", bastion_host="", key_path="k", gpu="h100", hosts=["a", "b"]))
    assert "Invalid gpu 'h100'" in _err(baremetal.new_node, bad, "m", key, None, st)


def test_interactive_baremetal_manager_prompts():
    st = State("mgr")
    answers = ["None", "Default", "Default", "tk-admin-pw-0123", "10.0.0.9", "", "None", "~/.ssh/id_rsa"]
    ctx = make_ctx({}, answers=answers, non_interactive=False)
    os.makedirs(os.path.expanduser("~/.ssh"), exist_ok=True)
    keyfile = os.path.expanduser("~/.ssh/id_rsa")
    created = not os.path.exists(keyfile)
    if created:
        open(keyfile, "w").close()
    try:
        baremetal.new_manager(ctx, st, "m")
    finally:
        if created:
            os.unlink(keyfile)
    m = st.manager()
    assert m["host"] == "10.0.0.9" and m["ssh_user"] == "ubuntu" and "bastion_host" not in m
    assert [q[1] for q in ctx.prompter.asked][:4] == ["Private Registry", "Rancher Server Image", "Rancher Agent Image",
                                                      "Set UI Admin Password"]


def test_registry_credentials_required_with_registry():
    st = State("mgr")
    ctx = make_ctx(dict(BASE_MGR, private_registry="reg.example", host="h"))
    assert _err(baremetal.new_manager, ctx, st, "m") == "private_registry_username must be specified"
    ctx = make_ctx(dict(BASE_CLUSTER, k8s_registry="reg", k8s_registry_username="u"))
    assert _err(baremetal.new_cluster, ctx, None, st) == "k8s_registry_password must be specified"


def test_cluster_name_validation():
    st = State("mgr")
    assert _err(baremetal.new_cluster, make_ctx(dict(BASE_CLUSTER, name="Bad_Name")), None, st) == \
        "Invalid Cluster Name"
    assert _err(baremetal.new_cluster, make_ctx({"name": "ok"}), None, st) == "k8s_version must be specified"


# --- triton -----------------------------------------------------------------------------------------
def _triton_vals(key):
    return {"triton_account": "acct", "triton_key_path": key, "triton_url": "https://tr.example",
            "triton_network_names": ["Joyent-SDC-Public"], "triton_image_name": "ubuntu-certified-16.04",
            "triton_image_version": "20180222", "triton_ssh_user": "ubuntu"}


def test_triton_manager_cluster_node(key):
    cloud = FakeCloud()
    st = State("mgr")
    triton.new_manager(make_ctx(dict(BASE_MGR, master_triton_machine_package="k4-highcpu-kvm-7.75G",
                                     **_triton_vals(key)), cloud=cloud), st, "mgr")
    m = st.manager()
    from triton_kubernetes_amd.utils.sshkeys import load_private_key

    assert m["triton_key_id"] == load_private_key(key).fingerprint_md5()
    assert m["triton_network_names"] == ["Joyent-SDC-Public"]
    name = triton.new_cluster(make_ctx(dict(BASE_CLUSTER, **_triton_vals(key)), cloud=cloud), None, st)
    ckey = st.clusters()[name]
    hosts = triton.new_node(make_ctx(dict(NODE_BASE, triton_machine_package="k4-highcpu-kvm-7.75G",
                                          **_triton_vals(key)), cloud=cloud), "mgr", ckey, None, st)
    n = st.module(f"node_triton_dev_{hosts[0]}")
    assert n["triton_account"] == "acct"  # copied by value from the cluster
    assert n["triton_machine_package"] == "k4-highcpu-kvm-7.75G"
    assert_blocks_match_modules(st)


def test_triton_validation_errors(key):
    cloud = FakeCloud()
    st = State("mgr")
    vals = dict(BASE_MGR, master_triton_machine_package="k4-highcpu-kvm-7.75G", **_triton_vals(key))
    vals["triton_network_names"] = ["nope"]
    assert _err(triton.new_manager, make_ctx(vals, cloud=cloud), st, "m") == \
        "Invalid Triton Network 'nope', must be one of the following: Joyent-SDC-Public, Joyent-SDC-Private, My-Fabric"
    vals = dict(BASE_MGR, master_triton_machine_package="huge", **_triton_vals(key))
    assert _err(triton.new_manager, make_ctx(vals, cloud=cloud), st, "m") == \
        "Invalid Master Triton Machine Package 'huge'"
    vals = dict(BASE_MGR, master_triton_machine_package="k4-highcpu-kvm-7.75G", **_triton_vals(key))
    vals["triton_image_version"] = "1999"
    assert _err(triton.new_manager, make_ctx(vals, cloud=cloud), st, "m") == \
        "Invalid Triton Image Name and Version 'ubuntu-certified-16.04@1999'"
    vals.pop("triton_image_version")
    assert _err(triton.new_manager, make_ctx(vals, cloud=cloud), st, "m") == \
        "Both triton_image_name and triton_image_version must be specified"


def test_triton_offline_mode_skips_listing(key):
    st = State("mgr")
    vals = dict(BASE_MGR, master_triton_machine_package="anything", cloud_validation=False, **_triton_vals(key))
    vals["triton_network_names"] = "net-a net-b"
    triton.new_manager(make_ctx(vals), st, "m")
    assert st.manager()["triton_network_names"] == ["net-a", "net-b"]


# --- aws ------------------------------------------------------------------------------------------------
AWS = {"aws_access_key": "AK", "aws_secret_key": "SK", "aws_region": "us-west-2", "aws_key_name": "k",
       "aws_vpc_cidr": "10.0.0.0/16", "aws_subnet_cidr": "10.0.2.0/24"}


def test_aws_manager_cluster_node(tmp_path):
    cloud = FakeCloud()
    st = State("mgr")
    aws.new_manager(make_ctx(dict(BASE_MGR, aws_private_key_path="~/.ssh/id_rsa", aws_ssh_user="ubuntu",
                                  aws_ami_id="ami-1", aws_instance_type="t3.medium", **AWS), cloud=cloud), st, "mgr")
    assert list(st.manager())[-11:] == ["aws_access_key", "aws_secret_key", "aws_region", "aws_vpc_cidr",
                                        "aws_subnet_cidr", "aws_public_key_path", "aws_private_key_path",
                                        "aws_key_name", "aws_ssh_user", "aws_ami_id", "aws_instance_type"]
    name = aws.new_cluster(make_ctx(dict(BASE_CLUSTER, **AWS), cloud=cloud), None, st)
    ckey = st.clusters()[name]
    hosts = aws.new_node(make_ctx(dict(NODE_BASE, aws_ami_id="ami-1", aws_instance_type="m5.large",
                                       ebs_volume_device_name="/dev/sdf", ebs_volume_mount_path="/data",
                                       ebs_volume_type="gp2"), cloud=cloud), "mgr", ckey, None, st)
    n = st.module(f"node_aws_dev_{hosts[0]}")
    assert n["aws_subnet_id"] == "${module.cluster_aws_dev.aws_subnet_id}"
    assert n["ebs_volume_size"] == "100" and "ebs_volume_iops" not in n
    # Q2 fix: no device name in non-interactive mode -> no volume, no prompt
    hosts = aws.new_node(make_ctx(dict(NODE_BASE, aws_ami_id="a", aws_instance_type="t"), cloud=cloud), "mgr",
                         ckey, None, st)
    assert "ebs_volume_device_name" not in st.module(f"node_aws_dev_{hosts[0]}")
    assert_blocks_match_modules(st)


def test_aws_validation_errors():
    cloud = FakeCloud()
    st = State("mgr")
    vals = dict(BASE_MGR, **AWS)
    vals["aws_region"] = "mars-1"
    assert _err(aws.new_manager, make_ctx(vals, cloud=cloud), st, "m") == "Selected AWS Region 'mars-1' does not exist."
    key = st.add_cluster("aws", "dev", {"name": "dev", "aws_region": "us-west-2"})
    bad = make_ctx(dict(NODE_BASE, aws_ami_id="a", aws_instance_type="t", ebs_volume_device_name="/dev/sdf",
                        ebs_volume_type="fast"), cloud=cloud)
    assert _err(aws.new_node, bad, "m", key, None, st) == "ebs_volume_type must be a valid volume type. Found 'fast'."
    from triton_kubernetes_amd.models.common import subnet_validator, validate_vpc_cidr

    assert validate_vpc_cidr("10.0.0.0/8") == "Prefix length must be 16 or greater. Found 8."
    assert subnet_validator("10.0.0.0/16")("192.168.0.0/24") == \
        "Subnet CIDR '192.168.0.0/24' is not within bounds of VPC CIDR '10.0.0.0/16'."
    assert subnet_validator("10.0.0.0/16")("10.0.3.0/24") is None


def test_aws_interactive_key_upload(tmp_path):
    cloud = FakeCloud()
    st = State("mgr")
    pub = tmp_path / "id.pub"
    pub.write_text("ssh-rsa AAAA")
    answers = ["", "", ("add", "new-key"), str(pub)]  # registry None, k8s registry None, key, path
    ctx = make_ctx(dict(BASE_CLUSTER, aws_access_key="A", aws_secret_key="S", aws_region="us-west-2",
                        aws_vpc_cidr="10.0.0.0/16", aws_subnet_cidr="10.0.2.0/24"), answers=answers,
                   non_interactive=False, cloud=cloud)
    aws.new_cluster(ctx, None, st)
    c = st.module("cluster_aws_dev")
    assert c["aws_key_name"] == "new-key" and c["aws_public_key_path"] == str(pub)


# --- gcp ----------------------------------------------------------------------------------------------------
def test_gcp_manager_cluster_node(gcp_creds, key, tmp_path):
    cloud = FakeCloud()
    st = State("mgr")
    pub = tmp_path / "k.pub"
    pub.write_text("ssh-rsa AAAA")
    gcp.new_manager(make_ctx(dict(BASE_MGR, gcp_path_to_credentials=gcp_creds, gcp_compute_region="us-central1",
                                  gcp_instance_zone="us-central1-a", gcp_machine_type="n1-standard-2",
                                  gcp_image="ubuntu-1604-xenial-v20180222", gcp_public_key_path=str(pub),
                                  gcp_private_key_path=key, gcp_ssh_user="ubuntu"), cloud=cloud), st, "mgr")
    assert st.manager()["gcp_project_id"] == "my-project"
    name = gcp.new_cluster(make_ctx(dict(BASE_CLUSTER, gcp_path_to_credentials=gcp_creds,
                                         gcp_compute_region="us-central1"), cloud=cloud), None, st)
    ckey = st.clusters()[name]
    hosts = gcp.new_node(make_ctx(dict(NODE_BASE, gcp_instance_zone="us-central1-b", gcp_machine_type="n1-standard-2",
                                       gcp_image="ubuntu-1804-bionic-v20180808"), cloud=cloud), "m", ckey, None, st)
    n = st.module(f"node_gcp_dev_{hosts[0]}")
    assert n["gcp_compute_network_name"] == "${module.cluster_gcp_dev.gcp_compute_network_name}"
    assert n["gcp_disk_type"] == ""
    assert_blocks_match_modules(st)
    bad = make_ctx(dict(NODE_BASE, gcp_instance_zone="us-east1-b", gcp_machine_type="x", gcp_image="y"), cloud=cloud)
    assert _err(gcp.new_node, bad, "m", ckey, None, st) == "Selected GCP Instance Zone 'us-east1-b' does not exist."


# --- azure ---------------------------------------------------------------------------------------------------
AZ = {"azure_subscription_id": "s", "azure_client_id": "c", "azure_client_secret": "x", "azure_tenant_id": "t",
      "azure_environment": "public", "azure_location": "westus2"}


def test_azure_manager_cluster_node(tmp_path, key):
    cloud = FakeCloud()
    st = State("mgr")
    pub = tmp_path / "k.pub"
    pub.write_text("ssh-rsa AAAA")
    azure.new_manager(make_ctx(dict(BASE_MGR, azure_size="Standard_D4s_v5", azure_ssh_user="ubuntu",
                                    azure_public_key_path=str(pub), azure_private_key_path=key, **AZ), cloud=cloud),
                      st, "mgr")
    assert st.manager()["azure_resource_group_name"] == ""
    name = azure.new_cluster(make_ctx(dict(BASE_CLUSTER, **AZ), cloud=cloud), None, st)
    ckey = st.clusters()[name]
    hosts = azure.new_node(make_ctx(dict(NODE_BASE, azure_size="Standard_D2_v2", azure_ssh_user="u",
                                         azure_public_key_path=str(pub), azure_disk_mount_path="/data",
                                         azure_disk_size="100"), cloud=cloud), "m", ckey, None, st)
    n = st.module(f"node_azure_dev_{hosts[0]}")
    assert n["azure_subnet_id"] == "${module.cluster_azure_dev.azure_subnet_id}" and n["azure_disk_size"] == "100"
    assert_blocks_match_modules(st)
    bad = make_ctx(dict(NODE_BASE, azure_size="Standard_D4s_v5", azure_ssh_user="u", azure_public_key_path=str(pub),
                        azure_disk_mount_path="/data"), cloud=cloud)
    assert _err(azure.new_node, bad, "m", ckey, None, st) == \
        "If azure_disk_mount_path is set, then azure_disk_size must also be set."
    vals = dict(BASE_CLUSTER, **AZ)
    vals["azure_environment"] = "moon"
    assert _err(azure.new_cluster, make_ctx(vals, cloud=cloud), None, st) == (
        "Invalid azure_environment 'moon', must be one of the following: 'public', 'government', 'german', or 'china'")
    vals = dict(BASE_CLUSTER, **AZ)
    vals["azure_location"] = "mars"
    assert _err(azure.new_cluster, make_ctx(vals, cloud=cloud), None, st) == \
        "Invalid azure_location 'mars', must be one of the following: westus2, eastus"


# --- vsphere --------------------------------------------------------------------------------------------------
def test_vsphere_cluster_and_node(key):
    st = State("mgr")
    vals = dict(BASE_CLUSTER, vsphere_user="u", vsphere_password="p", vsphere_server="vc",
                vsphere_datacenter_name="dc", vsphere_datastore_name="ds", vsphere_resource_pool_name="rp",
                vsphere_network_name="net")
    name = vsphere.new_cluster(make_ctx(vals), None, st)
    ckey = st.clusters()[name]
    hosts = vsphere.new_node(make_ctx(dict(NODE_BASE, vsphere_template_name="ubuntu", ssh_user="ubuntu",
                                           key_path=key, vsphere_num_cpus=16)), "m", ckey, None, st)
    n = st.module(f"node_vsphere_dev_{hosts[0]}")
    assert n["vsphere_datastore_name"] == "${module.cluster_vsphere_dev.vsphere_datastore_name}"
    assert n["vsphere_num_cpus"] == "16" and n["vsphere_user"] == "u"
    assert_blocks_match_modules(st)
    vals.pop("vsphere_user")
    assert _err(vsphere.new_cluster, make_ctx(vals), None, st) == "vsphere_user must be specified."
