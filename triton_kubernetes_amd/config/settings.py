"""Layered configuration (the reference's viper usage).

Precedence, highest first (viper ``find``):

1. explicit overrides (:meth:`Settings.set`) — used by the ``nodes:`` loop;
2. command-line flags (``--non-interactive``);
3. environment variables named as the UPPER-CASED key (``AutomaticEnv``), e.g.
   ``TRITON_ACCOUNT``, ``SOURCE_URL``, ``SOURCE_REF``;
4. the YAML/JSON config file (``--config`` or ``$HOME/.triton-kubernetes.yaml``).

Unlike the reference, settings are an explicit object threaded through the
workflows instead of a process-global, so tests cannot leak state into each
other (SURVEY.md §4 "hygiene issues").
"""

import json
import os
from typing import Any, Dict, Iterable, List, Mapping, Optional

import yaml

from ..errors import ConfigError

_MISSING = object()
_MISSING_TOKEN = object()

CONFIG_BASENAME = ".triton-kubernetes"
CONFIG_EXTS = ("yaml", "yml", "json")


def _env_name(key: str) -> str:
    # viper maps "non-interactive" -> "NON-INTERACTIVE"; keep both that and the
    # shell-friendly underscore form.
    return key.upper()


class Settings:
    def __init__(
        self,
        file_values: Optional[Mapping[str, Any]] = None,
        env: Optional[Mapping[str, str]] = None,
        flags: Optional[Mapping[str, Any]] = None,
        automatic_env: bool = True,
    ):
        self._file: Dict[str, Any] = {k.lower(): v for k, v in dict(file_values or {}).items()}
        self._env = dict(os.environ if env is None else env)
        self._flags: Dict[str, Any] = dict(flags or {})
        self._overrides: Dict[str, Any] = {}
        self.automatic_env = automatic_env
        self.config_file_used: Optional[str] = None

    # --- construction --------------------------------------------------------------
    @classmethod
    def from_file(cls, path: str, **kw) -> "Settings":
        values = load_config_file(path)
        s = cls(values, **kw)
        s.config_file_used = path
        return s

    @classmethod
    def discover(cls, explicit_path: Optional[str] = None, home: Optional[str] = None, **kw) -> "Settings":
        """``initConfig`` (``cmd/root.go:48-66``): explicit file, else ``$HOME/.triton-kubernetes.*``."""
        if explicit_path:
            return cls.from_file(explicit_path, **kw)
        home = home or os.path.expanduser("~")
        for ext in CONFIG_EXTS:
            candidate = os.path.join(home, f"{CONFIG_BASENAME}.{ext}")
            if os.path.isfile(candidate):
                return cls.from_file(candidate, **kw)
        return cls(None, **kw)

    # --- layers --------------------------------------------------------------------------
    def set(self, key: str, value: Any) -> None:
        """Override a key (``viper.Set``).

        As in viper 1.0, overriding with ``None`` *shadows* lower layers: the key
        then reads as unset even if the config file or environment has it.
        """
        self._overrides[key.lower()] = _MISSING if value is None else value

    def unset(self, key: str) -> None:
        self._overrides.pop(key.lower(), None)

    def push_overrides(self, values: Mapping[str, Any]) -> Dict[str, Any]:
        """Apply several overrides; return a token for :meth:`pop_overrides`."""
        saved = {}
        for key, value in values.items():
            k = key.lower()
            saved[k] = self._overrides.get(k, _MISSING_TOKEN)
            self.set(k, value)
        return saved

    def pop_overrides(self, saved: Mapping[str, Any]) -> None:
        for k, old in saved.items():
            if old is _MISSING_TOKEN:
                self._overrides.pop(k, None)
            else:
                self._overrides[k] = old

    def set_flag(self, key: str, value: Any) -> None:
        self._flags[key.lower()] = value

    def _find(self, key: str) -> Any:
        key = key.lower()
        if key in self._overrides:
            return self._overrides[key]
        if key in self._flags and self._flags[key] is not None:
            return self._flags[key]
        if self.automatic_env:
            for name in (_env_name(key), _env_name(key).replace("-", "_")):
                if name in self._env:
                    return self._env[name]
        if key in self._file:
            return self._file[key]
        return _MISSING

    # --- typed getters ---------------------------------------------------------------------
    def is_set(self, key: str) -> bool:
        value = self._find(key)
        return value is not _MISSING and value is not None

    def get(self, key: str, default: Any = None) -> Any:
        value = self._find(key)
        if value is _MISSING or value is None:
            return default
        return value

    def get_string(self, key: str) -> str:
        value = self.get(key)
        if value is None:
            return ""
        if isinstance(value, bool):
            return "true" if value else "false"
        if isinstance(value, (list, tuple)):
            return " ".join(str(v) for v in value)
        return str(value)

    def get_bool(self, key: str) -> bool:
        value = self.get(key)
        if isinstance(value, bool):
            return value
        if value is None:
            return False
        if isinstance(value, (int, float)):
            return value != 0
        return str(value).strip().lower() in ("1", "t", "true", "yes", "y", "on")

    def get_int(self, key: str) -> int:
        value = self.get(key)
        try:
            return int(str(value).strip())
        except (TypeError, ValueError) as exc:
            raise ConfigError(f"{key} must be a valid number. Found '{value}'.") from exc

    def get_float(self, key: str, default: float) -> float:
        """A number of the settings (seconds, MiB); ``default`` when unset or empty, and a
        :class:`ConfigError` naming the key for anything that is not a number."""
        value = self.get(key)
        if value is None or (isinstance(value, str) and not value.strip()):
            return float(default)
        if isinstance(value, bool):
            raise ConfigError(f"{key} must be a number. Found '{value}'.")
        try:
            return float(str(value).strip())
        except ValueError:
            raise ConfigError(f"{key} must be a number. Found '{value}'.") from None

    def get_int_or(self, key: str, default: int) -> int:
        """:meth:`get_int` with a default for an unset or empty key."""
        value = self.get(key)
        if value is None or (isinstance(value, str) and not value.strip()):
            return int(default)
        return self.get_int(key)

    def get_string_slice(self, key: str) -> List[str]:
        """``viper.GetStringSlice``: lists as-is; strings split on whitespace/commas."""
        value = self.get(key)
        if value is None:
            return []
        if isinstance(value, (list, tuple)):
            return [str(v) for v in value]
        text = str(value).strip()
        if text.startswith("[") and text.endswith("]"):
            try:
                parsed = json.loads(text)
                if isinstance(parsed, list):
                    return [str(v) for v in parsed]
            except ValueError:
                pass
        return [p for p in text.replace(",", " ").split() if p]

    @property
    def non_interactive(self) -> bool:
        return self.get_bool("non-interactive")

    def keys(self) -> Iterable[str]:
        seen = set(self._file) | set(self._flags) | {k for k, v in self._overrides.items() if v is not _MISSING}
        return sorted(seen)

    def snapshot(self) -> Dict[str, Any]:
        return {k: self.get(k) for k in self.keys()}


def load_config_file(path: str) -> Dict[str, Any]:
    """The silent-install file's settings.  A file that cannot be read or parsed is a
    :class:`ConfigError` naming the file and the parser's reason (the reference's viper
    ignored such a file and went on without it, to fail later on a missing key)."""
    try:
        with open(path, "r", encoding="utf-8") as fh:
            text = fh.read()
    except (OSError, UnicodeDecodeError) as exc:
        raise ConfigError(f"config file '{path}': {getattr(exc, 'strerror', None) or exc}") from None
    try:
        if path.endswith(".json"):
            data = json.loads(text or "{}")
        else:
            data = yaml.safe_load(text) or {}
    except (ValueError, yaml.YAMLError) as exc:
        raise ConfigError(f"config file '{path}' is not valid {'JSON' if path.endswith('.json') else 'YAML'}: "
                          f"{' '.join(str(exc).split())}") from None
    if not isinstance(data, dict):
        raise ConfigError(f"config file '{path}' must contain a mapping at the top level")
    return data
