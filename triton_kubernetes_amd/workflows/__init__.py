"""L5 workflow commands: create / destroy / get (reference ``create/``, ``destroy/``, ``get/``)."""

from .create import new_cluster, new_manager, new_node  # noqa: F401
from .destroy import delete_cluster, delete_manager, delete_node  # noqa: F401
from .get import get_cluster, get_manager  # noqa: F401
