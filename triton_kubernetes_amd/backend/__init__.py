from .base import CONFIG_FILE, TFSTATE_FILE, Backend  # noqa: F401
from .local import LocalBackend  # noqa: F401
from .memory import MemoryBackend  # noqa: F401
from .select import prompt_for_backend  # noqa: F401
