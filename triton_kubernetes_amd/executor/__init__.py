from .base import Executor, outputs_from_tfstate  # noqa: F401
from .factory import build_executor  # noqa: F401
