from .document import (  # noqa: F401
    MANAGER_KEY,
    State,
    cluster_key,
    cluster_key_parts,
    node_key,
)
