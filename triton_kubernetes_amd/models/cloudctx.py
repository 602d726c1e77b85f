"""Access to cloud listing clients from a workflow context."""

from typing import Any

from ..config.context import Context


def cloud(ctx: Context) -> Any:
    if ctx.cloud is None:
        from ..cloud import CloudClients

        ctx.cloud = CloudClients()
    return ctx.cloud


def validation_enabled(ctx: Context) -> bool:
    """``cloud_validation: false`` skips every listing call (offline mode)."""
    if ctx.settings.is_set("cloud_validation"):
        return ctx.settings.get_bool("cloud_validation")
    return True
