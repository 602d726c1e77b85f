"""JSON encoding compatible with the reference's ``main.tf.json`` output.

The reference writes the document with gabs ``BytesIndent("", "\\t")`` which is
Go ``encoding/json`` ``MarshalIndent`` (``state/state.go:88-90``): tab
indentation, ``": "`` separators, raw UTF-8, and HTML-safe escaping of ``<``,
``>`` and ``&`` (plus U+2028/U+2029).  :func:`dumps_go` reproduces that byte
format so documents written by either tool diff cleanly.
"""

import json
from typing import Any

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


def dumps_go(obj: Any, indent: str = "\t") -> bytes:
    """Encode like Go's ``json.MarshalIndent(obj, "", indent)``."""
    if indent:
        text = json.dumps(obj, indent=indent, ensure_ascii=False, separators=(",", ": "))
    else:
        text = json.dumps(obj, ensure_ascii=False, separators=(",", ":"))
    return _go_escape(text).encode("utf-8")


def loads(raw: Any) -> Any:
    if isinstance(raw, (bytes, bytearray)):
        raw = raw.decode("utf-8")
    return json.loads(raw)
