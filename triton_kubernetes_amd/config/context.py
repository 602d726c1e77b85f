"""Run context threaded through every workflow + the field resolution contract.

Every provider field in the reference follows one pattern (~80 times,
SURVEY.md §2.3)::

    if viper.IsSet(k)       -> take the value (then validate)
    elif non-interactive    -> error "<k> must be specified"   (or a default)
    else                    -> prompt (select / free text / searchable)

:meth:`Context.resolve` and friends implement it once.  Workflows and provider
specs only declare *what* to ask.
"""

import os
import sys
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, TextIO

from ..errors import ConfigError
from .prompt import NoPrompter, Prompter, TerminalPrompter, Validator
from .settings import Settings


def expand_home(path: str) -> str:
    """``homedir.Expand``: only a leading ``~`` is expanded."""
    if path.startswith("~"):
        return os.path.expanduser(path)
    return path


@dataclass
class Context:
    settings: Settings = field(default_factory=Settings)
    prompter: Optional[Prompter] = None
    out: TextIO = field(default_factory=lambda: sys.stdout)
    # Factories injected by the CLI (or by tests): executor + cloud clients.
    executor_factory: Optional[Callable[["Context"], Any]] = None
    cloud: Optional[Any] = None
    extras: Dict[str, Any] = field(default_factory=dict)

    def __post_init__(self):
        if self.prompter is None:
            self.prompter = NoPrompter() if self.settings.non_interactive else TerminalPrompter(stdout=self.out)

    # --- helpers -----------------------------------------------------------------------
    @property
    def non_interactive(self) -> bool:
        return self.settings.non_interactive

    def echo(self, text: str = "") -> None:
        self.out.write(text + "\n")
        self.out.flush()

    def is_set(self, key: str) -> bool:
        return self.settings.is_set(key)

    def get_string(self, key: str) -> str:
        return self.settings.get_string(key)

    # --- the resolution contract --------------------------------------------------------
    def resolve(
        self,
        key: str,
        label: str,
        *,
        required: bool = True,
        default: Optional[str] = None,
        validate: Validator = None,
        mask: bool = False,
        none_sentinel: Optional[str] = None,
        missing_message: Optional[str] = None,
        non_interactive_default: Optional[str] = None,
    ) -> str:
        """Free-text field.

        * ``required`` — non-interactive mode without the key raises
          ``missing_message`` (default ``"<key> must be specified"``); otherwise
          ``non_interactive_default`` (or ``""``) is used silently.
        * ``none_sentinel`` — the interactive default meaning "leave empty"
          (reference uses ``"None"`` / ``"Default"``).
        """
        if self.is_set(key):
            return self.get_string(key)
        if self.non_interactive:
            if required:
                raise ConfigError(missing_message or f"{key} must be specified")
            return non_interactive_default or ""
        prompt_default = default if default is not None else none_sentinel
        value = self.prompter.prompt(label, default=prompt_default, validate=validate, mask=mask)
        if none_sentinel is not None and value == none_sentinel:
            return ""
        return value

    def resolve_choice(
        self,
        key: str,
        label: str,
        items: Sequence[str],
        *,
        values: Optional[Sequence[str]] = None,
        required: bool = True,
        missing_message: Optional[str] = None,
        searchable: bool = False,
        transform: Optional[Callable[[str], str]] = None,
    ) -> str:
        """Select field: display ``items``; return ``values[i]`` (or the item)."""
        if self.is_set(key):
            return self.get_string(key)
        if self.non_interactive:
            if required:
                raise ConfigError(missing_message or f"{key} must be specified")
            return ""
        idx, item = self.prompter.select(label, list(items), searchable=searchable)
        value = values[idx] if values is not None else item
        return transform(value) if transform else value

    def resolve_list(
        self,
        key: str,
        label: str,
        items: Sequence[str],
        *,
        more_label: str = "Attach another",
        missing_message: Optional[str] = None,
    ) -> List[str]:
        """Multi-select loop (triton network picker, ``create/manager_triton.go:201-261``)."""
        if self.is_set(key):
            return self.settings.get_string_slice(key)
        if self.non_interactive:
            raise ConfigError(missing_message or f"{key} must be specified")
        chosen: List[str] = []
        remaining = list(items)
        while remaining:
            _, value = self.prompter.select(label, remaining, searchable=True)
            chosen.append(value)
            remaining.remove(value)
            if not remaining or not self.prompter.yes_no(more_label):
                break
        return chosen

    def confirm(self, label: str, selected: str) -> bool:
        """``util.PromptForConfirmation`` (no-op ``True`` in non-interactive mode)."""
        if self.non_interactive:
            return True
        return self.prompter.confirm(label, selected)


def not_blank(message: str) -> Validator:
    return lambda value: message if value == "" else None


def file_exists() -> Validator:
    def _check(value: str) -> Optional[str]:
        if not os.path.exists(expand_home(value)):
            return "File not found"
        return None

    return _check
