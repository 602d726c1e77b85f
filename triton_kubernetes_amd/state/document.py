"""The ``main.tf.json`` state document (reference ``state/state.go:1-160``).

The document *is* the Terraform root configuration.  The key naming is the
schema:

* manager  -> ``module.cluster-manager``
* cluster  -> ``module.cluster_{provider}_{name}``
* node     -> ``module.node_{provider}_{cluster}_{hostname}``
* backend  -> ``terraform.backend.{local|manta}``

Design differences from the reference (deliberate):

* values are stored as plain JSON dicts, never opaque structs, so
  :meth:`State.clusters` / :meth:`State.nodes` see modules added in the same
  session (the reference needs a re-parse workaround, ``create/cluster.go:146-152``,
  and produces colliding hostnames when the same prefix is used twice);
* module keys are addressed directly (not through dotted paths) so hostnames
  containing ``.`` cannot corrupt the document.

Dotted-path :meth:`get` / :meth:`set` / :meth:`delete` keep gabs semantics for
callers that use them (``state_test.go``).
"""

import copy
from typing import Any, Dict, List, Optional, Tuple

from ..errors import StateError
from ..utils.jsonenc import dumps_go, loads

MANAGER_KEY = "cluster-manager"


def cluster_key(provider: str, name: str) -> str:
    return f"cluster_{provider}_{name}"


def cluster_key_parts(key: str) -> Tuple[str, str]:
    """Split ``cluster_{provider}_{name}`` (``state/state.go:149-159``).

    Like the reference, ``name`` is the third ``_``-separated field, so cluster
    names must not contain ``_`` (DNS-1123 names cannot).
    """
    parts = key.split("_")
    if len(parts) < 3:
        raise StateError(
            "Could not get cluster key parts, cluster does not follow format "
            f"`cluster_{{provider}}_{{clusterName}}` '{key}'"
        )
    return parts[1], parts[2]


def node_key(cluster: str, hostname: str) -> str:
    provider, name = cluster_key_parts(cluster)
    return f"node_{provider}_{name}_{hostname}"


def _to_json_obj(obj: Any) -> Any:
    """Normalise an arbitrary config object to plain JSON data."""
    if hasattr(obj, "to_json") and callable(obj.to_json):
        return obj.to_json()
    return copy.deepcopy(obj)


class State:
    """Mutable view over one manager's ``main.tf.json``."""

    def __init__(self, name: str, raw: Any = b"{}"):
        self.name = name
        if isinstance(raw, (bytes, bytearray, str)):
            try:
                doc = loads(raw) if raw else {}
            except ValueError as exc:
                raise StateError(f"invalid state document for '{name}': {exc}") from exc
        else:
            doc = copy.deepcopy(raw)
        if not isinstance(doc, dict):
            raise StateError(f"invalid state document for '{name}': top level must be an object")
        self._doc: Dict[str, Any] = doc
        self._base: Optional[Dict[str, Any]] = None  # mark_base(): the document as read

    # --- generic dotted-path access (gabs Path/SetP/DeleteP semantics) -------
    @property
    def doc(self) -> Dict[str, Any]:
        return self._doc

    def lookup(self, path: str) -> Any:
        node: Any = self._doc
        for part in path.split("."):
            if not isinstance(node, dict) or part not in node:
                return None
            node = node[part]
        return node

    def get(self, path: str) -> str:
        """String value at ``path`` or ``""`` (``state/state.go:27-34``)."""
        value = self.lookup(path)
        return value if isinstance(value, str) else ""

    def set(self, path: str, obj: Any) -> None:
        self._set_parts(path.split("."), obj)

    def _set_parts(self, parts: List[str], obj: Any) -> None:
        node = self._doc
        for part in parts[:-1]:
            child = node.get(part)
            if not isinstance(child, dict):
                child = {}
                node[part] = child
            node = child
        node[parts[-1]] = _to_json_obj(obj)

    def delete(self, path: str) -> None:
        parts = path.split(".")
        node: Any = self._doc
        for part in parts[:-1]:
            if not isinstance(node, dict) or part not in node:
                raise StateError(f"Path not found: '{path}'")
            node = node[part]
        if not isinstance(node, dict) or parts[-1] not in node:
            raise StateError(f"Path not found: '{path}'")
        del node[parts[-1]]

    # --- schema-aware helpers --------------------------------------------------
    def modules(self) -> Dict[str, Any]:
        mods = self._doc.get("module")
        return mods if isinstance(mods, dict) else {}

    def module(self, key: str) -> Optional[Dict[str, Any]]:
        mod = self.modules().get(key)
        return mod if isinstance(mod, dict) else None

    def _modules_for_write(self) -> Dict[str, Any]:
        mods = self._doc.get("module")
        if not isinstance(mods, dict):
            mods = {}
            self._doc["module"] = mods
        return mods

    def set_module(self, key: str, obj: Any) -> None:
        self._modules_for_write()[key] = _to_json_obj(obj)

    def delete_module(self, key: str) -> None:
        mods = self.modules()
        if key not in mods:
            raise StateError(f"Path not found: 'module.{key}'")
        del mods[key]

    def set_manager(self, obj: Any) -> None:
        self.set_module(MANAGER_KEY, obj)

    def manager(self) -> Optional[Dict[str, Any]]:
        return self.module(MANAGER_KEY)

    def set_terraform_backend_config(self, path: str, obj: Any) -> None:
        # The backend block is *replaced* (a doc has exactly one backend).
        self.set(path, obj)

    def add_cluster(self, provider: str, name: str, obj: Any) -> str:
        key = cluster_key(provider, name)
        self.set_module(key, obj)
        return key

    def add_node(self, cluster: str, hostname: str, obj: Any) -> str:
        key = node_key(cluster, hostname)
        self.set_module(key, obj)
        return key

    def clusters(self) -> Dict[str, str]:
        """Map cluster ``name`` -> module key (``state/state.go:94-113``)."""
        result: Dict[str, str] = {}
        for key, child in self.modules().items():
            if key.startswith("cluster_") and isinstance(child, dict):
                name = child.get("name")
                if isinstance(name, str):
                    result[name] = key
        return result

    def nodes(self, cluster: str) -> Dict[str, str]:
        """Map ``hostname`` -> node key for one cluster (``state/state.go:117-147``)."""
        provider, name = cluster_key_parts(cluster)
        prefix = f"node_{provider}_{name}_"
        result: Dict[str, str] = {}
        for key, child in self.modules().items():
            if key.startswith(prefix) and isinstance(child, dict):
                hostname = child.get("hostname")
                if isinstance(hostname, str):
                    result[hostname] = key
        return result

    def backend_block(self) -> Tuple[Optional[str], Dict[str, Any]]:
        backends = self.lookup("terraform.backend")
        if isinstance(backends, dict) and backends:
            kind = next(iter(backends))
            cfg = backends[kind]
            return kind, cfg if isinstance(cfg, dict) else {}
        return None, {}

    # --- concurrent writers ---------------------------------------------------------
    def mark_base(self) -> "State":
        """Remember the document as read from the backend: :meth:`rebase` later replays
        only what this run changed on top of what is persisted then."""
        self._base = copy.deepcopy(self._doc)
        return self

    def rebase(self, current: "State") -> List[str]:
        """Three-way merge onto ``current`` (the persisted document, read under the backend
        lock): every module (and top-level key) this run added, changed or deleted since
        :meth:`mark_base` is applied to ``current``; everything else is ``current``'s, so
        another CLI's clusters and nodes persisted meanwhile are kept.  Raises
        :class:`StateError` when both changed the same module differently.  Returns the
        keys another writer changed (empty: nobody did).  No-op without a base."""
        if self._base is None:
            return []
        base = self._base
        if current.doc == base:
            return []
        conflicts: List[str] = []

        def merge(b: Dict[str, Any], m: Dict[str, Any], c: Dict[str, Any], skip: str = "") -> Dict[str, Any]:
            out = {k: v for k, v in c.items() if k != skip}
            for k in (set(b) | set(m)) - {skip}:
                bv, mv = b.get(k), m.get(k)
                if bv == mv:
                    continue  # not ours
                cv = c.get(k)
                if cv != bv and cv != mv:
                    conflicts.append(f"module.{k}" if not skip else k)
                    continue
                if mv is None:
                    out.pop(k, None)
                else:
                    out[k] = copy.deepcopy(mv)
            return out

        others = sorted(k for k in set(base.get("module") or {}) | set(current.modules())
                        if (base.get("module") or {}).get(k) != current.modules().get(k))
        modules = merge(base.get("module") or {}, self.modules(), current.modules())
        doc = merge(base, self._doc, current.doc, skip="module")
        if conflicts:
            raise StateError(f"'{self.name}' was changed by another triton-kubernetes run "
                             f"({', '.join(sorted(conflicts))}); re-run the command")
        if modules or "module" in self._doc or "module" in current.doc:
            doc["module"] = modules
        self._doc.clear()
        self._doc.update(doc)
        self._base = copy.deepcopy(self._doc)
        return others

    # --- serialisation -----------------------------------------------------------
    def bytes(self) -> bytes:
        """Tab-indented Go-compatible JSON (``state/state.go:88-90``)."""
        return dumps_go(self._doc)

    def copy(self) -> "State":
        return State(self.name, copy.deepcopy(self._doc))

    def __repr__(self) -> str:  # pragma: no cover
        return f"State(name={self.name!r}, modules={list(self.modules())})"
