"""JSON encoding compatible with the reference's ``main.tf.json`` output.

The reference writes the document with gabs ``BytesIndent("", "\\t")`` which is
Go ``encoding/json`` ``MarshalIndent`` (``state/state.go:88-90``): tab
indentation, ``": "`` separators, raw UTF-8, and HTML-safe escaping of ``<``,
``>`` and ``&`` (plus U+2028/U+2029).  :func:`dumps_go` reproduces that byte
format so documents written by either tool diff cleanly.
"""

import json
import threading
from typing import Any, Dict, Tuple

_GO_ESCAPES = {
    "<": "\\u003c",
    ">": "\\u003e",
    "&": "\\u0026",
    "\u2028": "\\u2028",
    "\u2029": "\\u2029",
}


def _go_escape(text: str) -> str:
    # The escaped characters can only occur inside JSON strings, so a plain
    # textual replacement over the encoded document is exact.
    for raw, esc in _GO_ESCAPES.items():
        if raw in text:
            text = text.replace(raw, esc)
    return text


def _dumps_indent(obj: Any, indent: str) -> str:
    return json.dumps(obj, indent=indent, ensure_ascii=False, separators=(",", ": "))


# (indent, depth, compact encoding) -> Go-escaped indented text nested `depth` levels deep
_MEMO: Dict[Tuple[str, int, str], str] = {}
_MEMO_MAX = 16384
_MEMO_MU = threading.Lock()
# objects expanded by hand down to this depth; their values below are memoised whole
_EXPAND_DEPTH = 2


def _encode(obj: Any, indent: str, depth: int) -> str:
    if depth < _EXPAND_DEPTH and isinstance(obj, dict) and obj and all(isinstance(k, str) for k in obj):
        pad = indent * (depth + 1)
        body = ",\n".join(
            pad + _go_escape(json.dumps(k, ensure_ascii=False)) + ": " + _encode(v, indent, depth + 1)
            for k, v in obj.items())
        return "{\n" + body + "\n" + indent * depth + "}"
    if not isinstance(obj, (dict, list)):
        return _go_escape(_dumps_indent(obj, indent))
    key = (indent, depth, json.dumps(obj, ensure_ascii=False, separators=(",", ":")))
    hit = _MEMO.get(key)
    if hit is None:
        text = _go_escape(_dumps_indent(obj, indent))
        hit = text.replace("\n", "\n" + indent * depth) if depth else text
        with _MEMO_MU:
            if len(_MEMO) >= _MEMO_MAX:
                _MEMO.clear()
            _MEMO[key] = hit
    return hit


def dumps_go(obj: Any, indent: str = "\t") -> bytes:
    """Encode like Go's ``json.MarshalIndent(obj, "", indent)``.

    The state document is re-written on every create and holds every module of every
    cluster of the manager, so the objects two levels down (one module's configuration)
    are encoded once and memoised by their compact encoding (C encoder, ~20x cheaper
    than the indented pure-Python one); the bytes equal a plain ``json.dumps`` of the
    whole document (``tests/test_state.py``).  JSON strings cannot hold a raw newline,
    so re-indenting a memoised value by replacing ``\\n`` is exact.
    """
    if indent:
        return _encode(obj, indent, 0).encode("utf-8")
    return _go_escape(json.dumps(obj, ensure_ascii=False, separators=(",", ":"))).encode("utf-8")


def dumps_go_plain(obj: Any, indent: str = "\t") -> bytes:
    """Reference implementation of :func:`dumps_go` without the memo (tests)."""
    if indent:
        return _go_escape(_dumps_indent(obj, indent)).encode("utf-8")
    return _go_escape(json.dumps(obj, ensure_ascii=False, separators=(",", ":"))).encode("utf-8")


def loads(raw: Any) -> Any:
    if isinstance(raw, (bytes, bytearray)):
        raw = raw.decode("utf-8")
    return json.loads(raw)
