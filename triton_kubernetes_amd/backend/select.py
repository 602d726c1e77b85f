"""Backend selection (reference ``util/backend_prompt.go:18-168``)."""

from ..config.context import Context, expand_home, file_exists, not_blank
from ..errors import ConfigError, TKError
from ..utils.sshkeys import public_key_fingerprint


def resolve_triton_key_id(ctx: Context, key_path: str) -> str:
    """``triton_key_id`` or the MD5 fingerprint of ``key_path`` (``backend_prompt.go:115-124``)."""
    if ctx.is_set("triton_key_id"):
        return ctx.get_string("triton_key_id")
    cb = None
    if not ctx.non_interactive:
        cb = lambda: ctx.prompter.prompt("Private Key Password", mask=True)  # noqa: E731
    return public_key_fingerprint(key_path, cb)


def prompt_for_backend(ctx: Context):
    """Build the state backend named by ``backend_provider`` (local | manta)."""
    provider = ctx.resolve_choice(
        "backend_provider", "Backend to persist data", ["Local", "Manta"],
        missing_message="backend_provider must be provided", transform=str.lower,
    )
    provider = provider.lower() if provider in ("Local", "Manta") else provider
    if provider == "local":
        from .local import LocalBackend

        return LocalBackend(ctx.settings.get_string("state_root") or None)
    if provider == "manta":
        account = ctx.resolve("triton_account", "Triton Account Name", validate=not_blank("Invalid Triton Account"))
        raw_key_path = ctx.resolve("triton_key_path", "Triton Key Path", default="~/.ssh/id_rsa",
                                   validate=file_exists())
        key_path = expand_home(raw_key_path)
        key_id = resolve_triton_key_id(ctx, key_path)
        triton_url = ctx.resolve("triton_url", "Triton URL", default="https://us-east-1.api.joyent.com")
        manta_url = ctx.resolve("manta_url", "Manta URL", default="https://us-east.manta.joyent.com")
        factory = ctx.extras.get("manta_backend_factory")
        if factory is not None:
            return factory(account, key_path, key_id, triton_url, manta_url)
        from .manta import MantaBackend

        try:
            return MantaBackend(account, key_path, key_id, triton_url, manta_url)
        except TKError:
            raise
        except OSError as exc:
            raise ConfigError(str(exc)) from exc
    raise ConfigError(f"Unsupported backend provider '{provider}'")
