"""AWS provider: manager (C19), cluster (C25), node (C32).

Reference: ``create/manager_aws.go:23-515``, ``create/cluster_aws.go:23-364``,
``create/node_aws.go:23-354``.  EC2 listings: regions (validated against a
us-west-1 client), key pairs (select-or-upload), Ubuntu AMIs newest first.
Deliberate fix: a non-interactive node without
``ebs_volume_device_name`` gets no volume instead of a "Create a volume" prompt.
"""

import re
from typing import Dict, List

from ..config.context import Context, expand_home, file_exists, not_blank
from .. import sizing
from ..errors import ConfigError
from ..state import State
from .cloudctx import cloud, validation_enabled
from .common import (add_nodes, base_cluster_config, base_manager_config, base_node_config, omit_empty,
                     positive_int, subnet_validator, validate_vpc_cidr)

MANAGER_MODULE = "terraform/modules/aws-rancher"
CLUSTER_MODULE = "terraform/modules/aws-rancher-k8s"
NODE_MODULE = "terraform/modules/aws-rancher-k8s-host"

# (key, display name, default size GiB) — node_aws.go:28-38
EBS_VOLUME_TYPES = [
    ("standard", "Magnetic", "100"),
    ("gp2", "General Purpose SSD", "100"),
    ("io1", "Provisioned IOPS SSD", "100"),
    ("st1", "Throughput Optimised HDD", "500"),
    ("sc1", "Cold HDD", "500"),
]
EBS_DEVICE_RE = re.compile(r"^/dev/sd[f-p]$")


def _creds(ctx: Context) -> Dict[str, str]:
    return {
        "aws_access_key": ctx.resolve("aws_access_key", "AWS Access Key", validate=not_blank("Invalid access key")),
        "aws_secret_key": ctx.resolve("aws_secret_key", "AWS Secret Key", mask=True,
                                      validate=not_blank("Invalid secret key")),
    }


def _region(ctx: Context, creds: Dict[str, str]) -> str:
    regions = None
    if validation_enabled(ctx):
        regions = cloud(ctx).aws(creds["aws_access_key"], creds["aws_secret_key"], "us-west-1").regions()
    if ctx.is_set("aws_region"):
        region = ctx.get_string("aws_region")
        if regions is not None and region not in regions:
            raise ConfigError(f"Selected AWS Region '{region}' does not exist.")
        return region
    if ctx.non_interactive:
        raise ConfigError("aws_region must be specified")
    if not regions:
        return ctx.prompter.prompt("AWS Region", default="us-west-1")
    _, region = ctx.prompter.select("AWS Region", regions)
    return region


def _key_pair(ctx: Context, ec2) -> Dict[str, str]:
    out = {"aws_key_name": "", "aws_public_key_path": ""}
    if ctx.is_set("aws_key_name"):
        out["aws_key_name"] = ctx.get_string("aws_key_name")
        if ctx.is_set("aws_public_key_path"):
            out["aws_public_key_path"] = expand_home(ctx.get_string("aws_public_key_path"))
        return out
    if ctx.non_interactive:
        raise ConfigError("aws_key_name must be specified")
    pairs = ec2.key_pairs() if ec2 is not None else []
    create = False
    if not pairs:
        create = True
        out["aws_key_name"] = ctx.prompter.prompt("Name for new aws public key",
                                                  default="triton-kubernetes_public_key")
    else:
        idx, value = ctx.prompter.select_with_add("AWS Key to use", pairs, "Upload new key")
        create = idx == -1
        out["aws_key_name"] = value
    if create:
        path = ctx.prompter.prompt("AWS Public Key Path", default="~/.ssh/id_rsa.pub", validate=file_exists())
        out["aws_public_key_path"] = expand_home(path)
    return out


def _network(ctx: Context) -> Dict[str, str]:
    vpc = ctx.resolve("aws_vpc_cidr", "AWS VPC CIDR", default="10.0.0.0/16", validate=validate_vpc_cidr)
    if ctx.is_set("aws_subnet_cidr"):
        subnet = ctx.get_string("aws_subnet_cidr")
    elif ctx.non_interactive:
        raise ConfigError("aws_subnet_cidr must be specified")
    else:
        subnet = ctx.prompter.prompt("AWS Subnet CIDR", default="10.0.2.0/24", validate=subnet_validator(vpc))
    return {"aws_vpc_cidr": vpc, "aws_subnet_cidr": subnet}


def _ami(ctx: Context, ec2) -> str:
    if ctx.is_set("aws_ami_id"):
        return ctx.get_string("aws_ami_id")
    if ctx.non_interactive:
        raise ConfigError("aws_ami_id must be specified")
    amis = ec2.images() if ec2 is not None else []
    if not amis:
        return ctx.prompter.prompt("AWS AMI ID")
    idx, _ = ctx.prompter.select("AWS AMI to use", [a.name for a in amis], searchable=True)
    return amis[idx].id


def _instance_type(ctx: Context, kind: str) -> str:
    """Default from ``sizing.py`` (the module variable's default too): t3.medium for the
    Rancher server, t3.large for nodes; a type known to be too small is refused."""
    value = ctx.resolve("aws_instance_type", "AWS Instance Type", default=sizing.default_size("aws", kind)[1],
                        validate=not_blank("Invalid Instance Type"))
    sizing.check_size("aws", kind, value)
    return value


def _ec2(ctx: Context, creds: Dict[str, str], region: str):
    if not validation_enabled(ctx):
        return None
    return cloud(ctx).aws(creds["aws_access_key"], creds["aws_secret_key"], region)


def new_manager(ctx: Context, state: State, name: str) -> None:
    cfg = base_manager_config(ctx, MANAGER_MODULE, name)
    creds = _creds(ctx)
    region = _region(ctx, creds)
    ec2 = _ec2(ctx, creds, region)
    key = _key_pair(ctx, ec2)
    private = ctx.resolve("aws_private_key_path", "AWS Private Key Path", default="~/.ssh/id_rsa",
                          validate=file_exists())
    ssh_user = ctx.resolve("aws_ssh_user", "AWS SSH User", default="ubuntu")
    net = _network(ctx)
    cfg.update(creds)
    cfg.update({
        "aws_region": region,
        "aws_vpc_cidr": net["aws_vpc_cidr"],
        "aws_subnet_cidr": net["aws_subnet_cidr"],
        "aws_public_key_path": key["aws_public_key_path"],
        "aws_private_key_path": expand_home(private),
        "aws_key_name": key["aws_key_name"],
        "aws_ssh_user": ssh_user,
        "aws_ami_id": _ami(ctx, ec2),
        "aws_instance_type": _instance_type(ctx, "manager"),
    })
    state.set_manager(cfg)


def new_cluster(ctx: Context, backend, state: State) -> str:
    cfg = base_cluster_config(ctx, CLUSTER_MODULE)
    creds = _creds(ctx)
    region = _region(ctx, creds)
    key = _key_pair(ctx, _ec2(ctx, creds, region))
    net = _network(ctx)
    cfg.update(creds)
    cfg.update({
        "aws_region": region,
        "aws_vpc_cidr": net["aws_vpc_cidr"],
        "aws_subnet_cidr": net["aws_subnet_cidr"],
        "aws_public_key_path": key["aws_public_key_path"],
        "aws_key_name": key["aws_key_name"],
    })
    state.add_cluster("aws", cfg["name"], cfg)
    return cfg["name"]


def _ebs(ctx: Context) -> Dict[str, str]:
    s = ctx.settings
    out = {"ebs_volume_device_name": "", "ebs_volume_mount_path": "", "ebs_volume_type": "",
           "ebs_volume_size": ""}
    if ctx.non_interactive:
        if not s.is_set("ebs_volume_device_name"):
            return out  # Q2 fix: no prompt, no volume
        out["ebs_volume_device_name"] = s.get_string("ebs_volume_device_name")
        out["ebs_volume_mount_path"] = s.get_string("ebs_volume_mount_path")
        out["ebs_volume_type"] = s.get_string("ebs_volume_type")
        if not any(k == out["ebs_volume_type"] for k, _, _ in EBS_VOLUME_TYPES):
            raise ConfigError(f"ebs_volume_type must be a valid volume type. Found '{out['ebs_volume_type']}'.")
        out["ebs_volume_size"] = s.get_string("ebs_volume_size") if s.is_set("ebs_volume_size") else next(
            d for k, _, d in EBS_VOLUME_TYPES if k == out["ebs_volume_type"])
        return out
    if not ctx.prompter.confirm("Create a volume for this node", "Volume Created"):
        return out
    out["ebs_volume_device_name"] = s.get_string("ebs_volume_device_name") if s.is_set(
        "ebs_volume_device_name") else ctx.prompter.prompt(
        "EBS Volume Device Name", default="/dev/sdf",
        validate=lambda v: None if EBS_DEVICE_RE.fullmatch(v) else
        "Device name must follow the format: /dev/sd[f-p] (e.g. /dev/sdf, /dev/sdp")
    out["ebs_volume_mount_path"] = s.get_string("ebs_volume_mount_path") if s.is_set(
        "ebs_volume_mount_path") else ctx.prompter.prompt("EBS Volume Mount Path")
    if s.is_set("ebs_volume_type"):
        out["ebs_volume_type"] = s.get_string("ebs_volume_type")
    else:
        idx, _ = ctx.prompter.select("EBS Volume Type", [n for _, n, _ in EBS_VOLUME_TYPES])
        out["ebs_volume_type"] = EBS_VOLUME_TYPES[idx][0]
    default = next((d for k, _, d in EBS_VOLUME_TYPES if k == out["ebs_volume_type"]), "")
    out["ebs_volume_size"] = s.get_string("ebs_volume_size") if s.is_set("ebs_volume_size") else \
        ctx.prompter.prompt("EBS Volume Size in GiB", default=default, validate=positive_int)
    return out


def new_node(ctx: Context, manager: str, cluster: str, backend, state: State) -> List[str]:
    base = base_node_config(ctx, NODE_MODULE, cluster, state)
    creds = {k: state.get(f"module.{cluster}.{k}") for k in ("aws_access_key", "aws_secret_key", "aws_region")}
    ec2 = _ec2(ctx, creds, creds["aws_region"] or "us-west-1")
    extra: Dict = dict(creds)
    extra.update({
        "aws_subnet_id": f"${{module.{cluster}.aws_subnet_id}}",
        "aws_security_group_id": f"${{module.{cluster}.aws_security_group_id}}",
        "aws_key_name": f"${{module.{cluster}.aws_key_name}}",
        "aws_ami_id": _ami(ctx, ec2),
        "aws_instance_type": _instance_type(ctx, "host"),
    })
    ebs = _ebs(ctx)
    extra.update({"ebs_volume_device_name": ebs["ebs_volume_device_name"],
                  "ebs_volume_mount_path": ebs["ebs_volume_mount_path"],
                  "ebs_volume_type": ebs["ebs_volume_type"],
                  "ebs_volume_iops": "",
                  "ebs_volume_size": ebs["ebs_volume_size"]})
    omit_empty(extra, ["ebs_volume_device_name", "ebs_volume_mount_path", "ebs_volume_type", "ebs_volume_iops",
                       "ebs_volume_size"])
    return add_nodes(state, cluster, base, extra)
