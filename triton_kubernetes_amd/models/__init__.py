"""Provider "model families" (reference L4, ``create/*_{provider}.go``).

``MANAGER_PROVIDERS`` / ``CLUSTER_PROVIDERS`` / ``NODE_PROVIDERS`` are the
dispatch tables of ``create/manager.go:108-122``, ``create/cluster.go:125-141``
and ``create/node.go:179-194``.  Support matrix: vSphere has no
manager.
"""

from . import aws, azure, baremetal, gcp, triton, vsphere

MANAGER_PROVIDERS = {
    "triton": triton.new_manager,
    "aws": aws.new_manager,
    "gcp": gcp.new_manager,
    "azure": azure.new_manager,
    "baremetal": baremetal.new_manager,
}
CLUSTER_PROVIDERS = {
    "triton": triton.new_cluster,
    "aws": aws.new_cluster,
    "gcp": gcp.new_cluster,
    "azure": azure.new_cluster,
    "baremetal": baremetal.new_cluster,
    "vsphere": vsphere.new_cluster,
}
NODE_PROVIDERS = {
    "triton": triton.new_node,
    "aws": aws.new_node,
    "gcp": gcp.new_node,
    "azure": azure.new_node,
    "baremetal": baremetal.new_node,
    "vsphere": vsphere.new_node,
}

MANAGER_CHOICES = ["Triton", "AWS", "GCP", "Azure", "BareMetal"]
CLUSTER_CHOICES = ["Triton", "AWS", "GCP", "Azure", "BareMetal", "vSphere"]

# Keys copied from each `nodes:` YAML entry (create/cluster.go:177-208).  The
# reference copies only a subset; we copy these *and* any
# other key present in the entry.
NODE_ENTRY_KEYS = {
    "common": ["rancher_host_label", "node_count", "hostname"],
    "aws": ["aws_ami_id", "aws_instance_type", "ebs_volume_device_name", "ebs_volume_mount_path",
            "ebs_volume_type", "ebs_volume_size"],
    "triton": ["triton_network_names", "triton_image_name", "triton_image_version", "triton_ssh_user",
               "triton_machine_package"],
    "gcp": ["gcp_instance_zone", "gcp_machine_type", "gcp_image", "gcp_disk_type", "gcp_disk_size",
            "gcp_disk_mount_path"],
    "azure": ["azure_size", "azure_ssh_user", "azure_public_key_path", "azure_disk_mount_path", "azure_disk_size"],
    "baremetal": ["ssh_user", "key_path", "bastion_host", "hosts", "gpu", "gpu_count", "gpu_burnin", "rccl_env",
                  "rccl_min_busbw", "node_cleanup"],
    "vsphere": ["vsphere_template_name", "ssh_user", "key_path", "vsphere_num_cpus", "vsphere_memory_mb"],
}
