"""The DirectExecutor's ``terraform.tfstate``: load and save in time independent of the
number of modules that did not change.

Every ``create cluster`` re-applies the manager's whole document (reference
``create/cluster.go:277-287``), so the tfstate holds every module of every cluster the
manager owns, and the executor saves it after each finished module (the resume point,
SURVEY.md §5.4).  Re-encoding the whole document with ``json.dumps(indent=2)`` on each save
made a create cost grow by ≈1.8 ms per cluster already on the manager (40 clusters: 18 ms
-> 89 ms per create in ``bench.py --sim-gpu``).  Here:

* the per-module entries (``module_outputs[key]``, ``module_state[key]``) are immutable
  once stored — the executor replaces an entry, never edits it — so each entry's text is
  encoded once and reused by identity;
* the root ``outputs`` (``<key>__<output>``, read by Terraform-style consumers) are derived
  from ``module_outputs`` at encode time, from the same per-entry cache;
* a load whose bytes equal the last save reuses that document instead of parsing again.

The bytes are identical to ``json.dumps(doc, indent=2, sort_keys=True)`` of the document
with its derived ``outputs`` (``tests/test_direct_executor.py`` checks it).
"""

import json
import threading
from typing import Any, Dict, List, Optional, Tuple

SECTIONS = ("module_outputs", "module_state")


def _nested(obj: Any, depth: int) -> str:
    """``obj`` as ``json.dumps(indent=2, sort_keys=True)`` writes it ``depth`` levels deep."""
    text = json.dumps(obj, indent=2, sort_keys=True)
    return text.replace("\n", "\n" + "  " * depth) if depth else text


def _line(key: str, text: str, depth: int) -> str:
    """One ``"key": value`` member of an object ``depth`` levels deep."""
    return "  " * (depth + 1) + json.dumps(key) + ": " + text


def _object(lines: List[str], depth: int) -> str:
    """A JSON object from member lines already sorted by key."""
    if not lines:
        return "{}"
    return "{\n" + ",\n".join(lines) + "\n" + "  " * depth + "}"


def derived_outputs(module_outputs: Dict[str, Dict[str, Any]]) -> Dict[str, Dict[str, Any]]:
    """The root outputs Terraform >= 0.12 consumers read (``executor/base.py:outputs_from_tfstate``)."""
    return {f"{key}__{k}": {"type": "string", "value": v}
            for key, outs in module_outputs.items() for k, v in outs.items()}


def copy_doc(doc: Dict[str, Any]) -> Dict[str, Any]:
    """A copy the caller may add to / pop from; entries are shared (they are immutable)."""
    out = dict(doc)
    for s in SECTIONS:
        if isinstance(out.get(s), dict):
            out[s] = dict(out[s])
    return out


class TfstateCodec:
    """Process-wide per-manager cache of the last saved tfstate and its encoded entries."""

    def __init__(self) -> None:
        self._mu = threading.Lock()
        self._last: Dict[str, Tuple[bytes, Dict[str, Any]]] = {}
        # manager -> (section, key) -> (entry object, its member line one level deep)
        self._frags: Dict[str, Dict[Tuple[str, str], Tuple[Any, str]]] = {}
        # manager -> module key -> (module_outputs entry, [(root output key, member line)])
        self._outs: Dict[str, Dict[str, Tuple[Any, List[Tuple[str, str]]]]] = {}

    def load(self, name: str, raw: Optional[bytes]) -> Optional[Dict[str, Any]]:
        """The document stored as ``raw``; None when ``raw`` is not a DirectExecutor tfstate."""
        if not raw:
            return None
        with self._mu:
            last = self._last.get(name)
            if last is not None and last[0] == raw:
                return copy_doc(last[1])
        try:
            doc = json.loads(raw)
        except ValueError:
            return None
        if not isinstance(doc, dict) or not isinstance(doc.get("module_state"), dict):
            return None
        doc.setdefault("module_outputs", {})
        doc.pop("outputs", None)  # derived again on every save
        return doc

    def dumps(self, name: str, doc: Dict[str, Any]) -> bytes:
        """Encode ``doc`` (its ``outputs`` derived from ``module_outputs``) and remember it."""
        with self._mu:
            frags = self._frags.get(name, {})
            outs_cache = self._outs.get(name, {})
            new_frags: Dict[Tuple[str, str], Tuple[Any, str]] = {}
            new_outs: Dict[str, Tuple[Any, List[Tuple[str, str]]]] = {}
            mods = doc.get("module_outputs")
            cacheable = isinstance(mods, dict) and all(isinstance(v, dict) for v in mods.values()) and all(
                isinstance(doc.get(s), dict) and all(isinstance(k, str) for k in doc[s]) for s in SECTIONS)
            if not cacheable:  # not our shape: plain encoding, derived outputs included
                full = dict(doc)
                if isinstance(mods, dict) and all(isinstance(v, dict) for v in mods.values()):
                    full["outputs"] = derived_outputs(mods)
                self._last.pop(name, None)
                return json.dumps(full, indent=2, sort_keys=True).encode()
            top: List[str] = []
            keys = set(doc) | {"outputs"}  # the document's own "outputs", if any, is replaced
            for k in sorted(keys):
                if k in SECTIONS:
                    lines = []
                    for key in sorted(doc[k]):
                        entry = doc[k][key]
                        hit = frags.get((k, key))
                        line = hit[1] if hit is not None and hit[0] is entry else _line(key, _nested(entry, 2), 1)
                        new_frags[(k, key)] = (entry, line)
                        lines.append(line)
                    top.append(_line(k, _object(lines, 1), 0))
                elif k == "outputs":
                    pairs: List[Tuple[str, str]] = []
                    for key, entry in mods.items():
                        hit = outs_cache.get(key)
                        if hit is not None and hit[0] is entry:
                            lst = hit[1]
                        else:
                            lst = [(f"{key}__{o}", _line(f"{key}__{o}", _nested({"type": "string", "value": v}, 2), 1))
                                   for o, v in entry.items()]
                        new_outs[key] = (entry, lst)
                        pairs.extend(lst)
                    pairs.sort(key=lambda p: p[0])
                    top.append(_line(k, _object([p[1] for p in pairs], 1), 0))
                else:
                    top.append(_line(k, _nested(doc[k], 1), 0))
            raw = _object(top, 0).encode()
            self._frags[name] = new_frags
            self._outs[name] = new_outs
            snapshot = copy_doc(doc)
            snapshot.pop("outputs", None)
            self._last[name] = (raw, snapshot)
            return raw

    def forget(self, name: str) -> None:
        with self._mu:
            self._last.pop(name, None)
            self._frags.pop(name, None)
            self._outs.pop(name, None)


CODEC = TfstateCodec()

__all__ = ["CODEC", "TfstateCodec", "copy_doc", "derived_outputs"]
