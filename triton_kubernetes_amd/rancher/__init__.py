"""rancher package."""
