"""Cloud listing facade used by provider plugins for validation and prompts.

:class:`CloudClients` builds the real REST clients; :class:`FakeCloud`
(``cloud.fake``) serves canned listings for tests and offline use.  Setting
``cloud_validation: false`` makes providers skip every listing call (values are
then taken as given), which is how the bench and CI run without network.
"""


class CloudClients:
    def triton(self, account: str, key_path: str, key_id: str, url: str):
        from .triton import HTTPSignatureSigner, TritonCloudAPI

        return TritonCloudAPI(url, HTTPSignatureSigner.from_path(account, key_path, key_id or None))

    def aws(self, access_key: str, secret_key: str, region: str = "us-west-1"):
        from .aws import EC2Client

        return EC2Client(access_key, secret_key, region)

    def gcp(self, credentials_path: str):
        from .gcp import ComputeClient

        return ComputeClient(credentials_path)

    def azure(self, subscription_id: str, client_id: str, client_secret: str, tenant_id: str, environment: str):
        from .azure import ARMClient

        return ARMClient(subscription_id, client_id, client_secret, tenant_id, environment)
