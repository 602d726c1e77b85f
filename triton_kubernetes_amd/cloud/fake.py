"""Canned cloud listings (the cloud-API fake the reference never had)."""

from dataclasses import dataclass, field
from typing import Dict, List

from .aws import AMI
from .gcp import GCPImage
from .triton import Image, Network, Package


@dataclass
class FakeTriton:
    networks_: List[Network] = field(default_factory=lambda: [
        Network("n1", "Joyent-SDC-Public", True), Network("n2", "Joyent-SDC-Private"), Network("n3", "My-Fabric")])
    images_: List[Image] = field(default_factory=lambda: [
        Image("i1", "ubuntu-certified-16.04", "20180222", "2018-02-22T00:00:00Z"),
        Image("i2", "ubuntu-certified-18.04", "20180808", "2018-08-08T00:00:00Z"),
        Image("i3", "ubuntu-certified-22.04", "20240301", "2024-03-01T00:00:00Z"),
    ])
    packages_: List[Package] = field(default_factory=lambda: [
        Package("p2", "k4-highcpu-kvm-7.75G", 7936), Package("p1", "k4-highcpu-kvm-1.75G", 1792)])
    calls: List[str] = field(default_factory=list)

    def networks(self):
        self.calls.append("networks")
        return list(self.networks_)

    def images(self):
        self.calls.append("images")
        return sorted(self.images_, key=lambda i: i.published_at, reverse=True)

    def packages(self):
        self.calls.append("packages")
        return sorted(self.packages_, key=lambda p: p.memory)


@dataclass
class FakeEC2:
    regions_: List[str] = field(default_factory=lambda: ["us-east-1", "us-west-1", "us-west-2", "eu-west-1"])
    key_pairs_: List[str] = field(default_factory=lambda: ["existing-key"])
    amis_: List[AMI] = field(default_factory=lambda: [
        AMI("ami-0001", "ubuntu/images/hvm-ssd/ubuntu-jammy-22.04-amd64-server-20240101", "2024-01-01"),
        AMI("ami-0002", "ubuntu/images/hvm-ssd/ubuntu-jammy-22.04-amd64-server-20240301", "2024-03-01"),
    ])

    def regions(self):
        return list(self.regions_)

    def key_pairs(self):
        return list(self.key_pairs_)

    def images(self, name_filter: str = ""):
        return sorted(self.amis_, key=lambda a: a.creation_date, reverse=True)

    def for_region(self, region: str):
        return self


@dataclass
class FakeGCP:
    project: str = "my-project"
    regions_: List[str] = field(default_factory=lambda: ["us-central1", "us-east1"])
    zones_: Dict[str, List[str]] = field(default_factory=lambda: {
        "us-central1": ["us-central1-a", "us-central1-b"], "us-east1": ["us-east1-b"]})
    machine_types_: List[str] = field(default_factory=lambda: ["n1-standard-1", "n1-standard-2", "n1-standard-4"])
    images_: List[GCPImage] = field(default_factory=lambda: [
        GCPImage("ubuntu-1604-xenial-v20180222", "", "2018-02-22"),
        GCPImage("ubuntu-1804-bionic-v20180808", "", "2018-08-08"),
        GCPImage("ubuntu-2204-jammy-v20240301", "", "2024-03-01")])

    def regions(self):
        return list(self.regions_)

    def zones(self, region):
        return list(self.zones_.get(region, []))

    def machine_types(self, zone):
        return list(self.machine_types_)

    def images(self, image_project: str = "ubuntu-os-cloud"):
        return sorted(self.images_, key=lambda i: i.creation_timestamp, reverse=True)


@dataclass
class FakeAzure:
    locations_: List[str] = field(default_factory=lambda: ["westus2", "eastus"])
    sizes_: List[str] = field(default_factory=lambda: ["Standard_A0", "Standard_D2_v2", "Standard_D4s_v5"])

    def locations(self):
        return list(self.locations_)

    def vm_sizes(self, location):
        return list(self.sizes_)


@dataclass
class FakeCloud:
    triton_: FakeTriton = field(default_factory=FakeTriton)
    ec2_: FakeEC2 = field(default_factory=FakeEC2)
    gcp_: FakeGCP = field(default_factory=FakeGCP)
    azure_: FakeAzure = field(default_factory=FakeAzure)

    def triton(self, account, key_path, key_id, url):
        return self.triton_

    def aws(self, access_key, secret_key, region="us-west-1"):
        return self.ec2_

    def gcp(self, credentials_path):
        return self.gcp_

    def azure(self, subscription_id, client_id, client_secret, tenant_id, environment):
        return self.azure_
