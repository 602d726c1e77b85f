"""Azure Resource Manager listing client (AAD client-credentials, stdlib only).

Replaces the ADAL + azure-sdk-for-go calls of the reference
(``create/manager_azure.go:185-290``): service-principal token,
``subscriptions.ListLocations`` and ``VirtualMachineSizes.List(location)``.
"""

import time
import urllib.parse
from typing import Dict, List, Optional

from ..errors import ConfigError
from .http import HTTPClient

ENVIRONMENTS: Dict[str, Dict[str, str]] = {
    "public": {"login": "https://login.microsoftonline.com", "arm": "https://management.azure.com"},
    "government": {"login": "https://login.microsoftonline.us", "arm": "https://management.usgovcloudapi.net"},
    "german": {"login": "https://login.microsoftonline.de", "arm": "https://management.microsoftazure.de"},
    "china": {"login": "https://login.chinacloudapi.cn", "arm": "https://management.chinacloudapi.cn"},
}


def environment_endpoints(name: str) -> Dict[str, str]:
    if name not in ENVIRONMENTS:
        raise ConfigError(
            f"Invalid azure_environment '{name}', must be one of the following: "
            "'public', 'government', 'german', or 'china'")
    return ENVIRONMENTS[name]


class ARMClient:
    def __init__(self, subscription_id: str, client_id: str, client_secret: str, tenant_id: str,
                 environment: str = "public", http: Optional[HTTPClient] = None,
                 endpoints: Optional[Dict[str, str]] = None):
        self.subscription_id = subscription_id
        self.client_id, self.client_secret, self.tenant_id = client_id, client_secret, tenant_id
        self.endpoints = endpoints or environment_endpoints(environment)
        self.http = http or HTTPClient()
        self._token: Optional[str] = None
        self._exp = 0.0

    def token(self) -> str:
        if self._token and time.time() < self._exp - 60:
            return self._token
        body = urllib.parse.urlencode({
            "grant_type": "client_credentials",
            "client_id": self.client_id,
            "client_secret": self.client_secret,
            "resource": self.endpoints["arm"].rstrip("/") + "/",
        }).encode()
        resp = self.http.request("POST", f"{self.endpoints['login']}/{self.tenant_id}/oauth2/token", data=body,
                                 headers={"Content-Type": "application/x-www-form-urlencoded"})
        data = resp.json()
        self._token = data["access_token"]
        self._exp = time.time() + float(data.get("expires_in", 3600))
        return self._token

    def _get(self, path: str, api_version: str) -> Dict:
        return self.http.get_json(f"{self.endpoints['arm']}{path}", params={"api-version": api_version},
                                  headers={"Authorization": f"Bearer {self.token()}"})

    def locations(self) -> List[str]:
        data = self._get(f"/subscriptions/{self.subscription_id}/locations", "2016-06-01")
        return [loc["name"] for loc in data.get("value", [])]

    def vm_sizes(self, location: str) -> List[str]:
        data = self._get(
            f"/subscriptions/{self.subscription_id}/providers/Microsoft.Compute/locations/{location}/vmSizes",
            "2017-12-01")
        return [s["name"] for s in data.get("value", [])]
