"""Error types.

The reference surfaces every failure as a Go ``error`` whose *text* is the
contract (its tests assert exact strings).  We keep that: every
user-facing failure is a :class:`TKError` whose ``str()`` is the exact message.
"""


class TKError(Exception):
    """A user-facing error; ``str(err)`` is the exact message printed by the CLI."""

    def __init__(self, message: str):
        super().__init__(message)
        self.message = message

    def __str__(self) -> str:  # pragma: no cover - trivial
        return self.message


class ConfigError(TKError):
    """Missing/invalid configuration value (e.g. ``"<key> must be specified"``)."""


class StateError(TKError):
    """Malformed state document or key."""


class BackendError(TKError):
    """State backend failure."""


class ExecutorError(TKError):
    """Terraform / direct executor failure."""


class PromptAborted(TKError):
    """The user aborted an interactive prompt (Ctrl-C / EOF)."""


class Canceled(Exception):
    """User declined a confirmation prompt; the workflow returns cleanly."""
