"""k8s package."""
