"""Terraform version constraints (``required_version``) and version-dependent rules.

Terraform refuses to ``init`` a configuration whose root or any module declares a
``required_version`` the running binary does not satisfy ("Unsupported Terraform Core
version").  The executor checks the same thing up front, so a too-old Terraform fails
with a message naming the module and the fix, not halfway into a run.

Constraint grammar (Terraform's): comma-separated ``<op> <version>`` terms, ``op`` one of
``= != > >= < <= ~>`` (none means ``=``); ``~> 1.4`` is ``>= 1.4, < 2.0`` and
``~> 1.4.2`` is ``>= 1.4.2, < 1.5.0``.
"""

import os
import re
from typing import Dict, List, Optional, Tuple

Version = Tuple[int, int, int]

_TERM = re.compile(r"^\s*(=|!=|>=|<=|>|<|~>)?\s*v?(\d+)(?:\.(\d+))?(?:\.(\d+))?(?:-[0-9A-Za-z.]+)?\s*$")
_REQ = re.compile(r'required_version\s*=\s*"([^"]*)"')

# Backend types Terraform dropped (v1.3.0 removed the deprecated artifactory, etcd, etcdv3,
# manta and swift backends: `init` reports "Unsupported backend type").
REMOVED_BACKENDS: Dict[str, Version] = {
    "artifactory": (1, 3, 0), "etcd": (1, 3, 0), "etcdv3": (1, 3, 0), "manta": (1, 3, 0), "swift": (1, 3, 0),
}
# From 0.15 a root output whose value is sensitive must say ``sensitive = true``.
SENSITIVE_ROOT_OUTPUTS_FROM: Version = (0, 15, 0)


def backend_removed(kind: str, version: Version) -> bool:
    cut = REMOVED_BACKENDS.get(kind)
    return cut is not None and tuple(version) >= cut


def _term(text: str) -> Tuple[str, Version, int]:
    m = _TERM.match(text)
    if not m:
        raise ValueError(f"invalid version constraint {text!r}")
    op = m.group(1) or "="
    parts = [m.group(2), m.group(3), m.group(4)]
    given = sum(p is not None for p in parts)
    v = tuple(int(p) if p is not None else 0 for p in parts)
    return op, v, given  # type: ignore[return-value]


def satisfies(version: Version, constraint: str) -> bool:
    """True when ``version`` meets every term of ``constraint``."""
    version = tuple(version)  # type: ignore[assignment]
    for raw in constraint.split(","):
        if not raw.strip():
            continue
        op, v, given = _term(raw)
        if op == "=" and version != v:
            return False
        if op == "!=" and version == v:
            return False
        if op == ">" and not version > v:
            return False
        if op == ">=" and not version >= v:
            return False
        if op == "<" and not version < v:
            return False
        if op == "<=" and not version <= v:
            return False
        if op == "~>":
            if version < v:
                return False
            if given <= 2:  # ~> 1.4  -> < 2.0.0
                upper = (v[0] + 1, 0, 0)
            else:  # ~> 1.4.2 -> < 1.5.0
                upper = (v[0], v[1] + 1, 0)
            if version >= upper:
                return False
    return True


def required_versions(module_dir: str) -> List[str]:
    """Every ``required_version`` string declared in the ``*.tf`` files of a module."""
    out: List[str] = []
    try:
        names = sorted(os.listdir(module_dir))
    except OSError:
        return out
    for fn in names:
        if fn.endswith(".tf"):
            with open(os.path.join(module_dir, fn), "r", encoding="utf-8") as fh:
                out += _REQ.findall(fh.read())
    return out


def unsupported_by(version: Version, module_dir: str) -> Optional[str]:
    """The first ``required_version`` of the module that ``version`` fails, or None."""
    for req in required_versions(module_dir):
        if not satisfies(version, req):
            return req
    return None


def fmt(version: Version) -> str:
    return ".".join(str(x) for x in version)
