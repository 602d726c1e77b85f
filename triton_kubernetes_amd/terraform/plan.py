"""Static plan of one module call: every expression of a module evaluated the way
``terraform plan`` evaluates it, with apply-time values unknown.

No ``terraform`` binary is available where this framework is built and tested, and the
modules under ``terraform/modules`` are only ever applied by a user's Terraform.  The
syntax checker (``hcl.check_module``) proves they parse and that every reference names
something declared; this module goes one step further and *evaluates* them for a
concrete module block (the inputs a provider plugin wrote into ``main.tf.json``):

* input conversion to the declared variable types (``"8"`` -> number, ``"true"`` -> bool),
  ``${module...}`` interpolations are unknown (known after apply);
* ``locals`` (dependency order, cycles reported), provider, resource, data and output
  blocks, nested and ``dynamic`` blocks (with their iterator), ``connection`` and
  provisioner blocks (``self`` unknown);
* ``count`` / ``for_each`` must be known at plan time (Terraform's "Invalid count
  argument"), and a counted resource must be indexed before its attributes are read
  ("Missing resource instance key");
* functions run for real on known arguments (``file`` reads the file, ``templatefile``
  renders the template with ``hcl.templatefile``, ``tonumber`` / ``substr`` / ``lookup`` /
  indexing fail the way Terraform's do) and yield unknown on unknown arguments;
* conditionals report errors of the selected branch only (both when the condition is
  unknown), as HCL does.

The reference has no counterpart: its modules were Terraform 0.11 files exercised only by
hand.  ``tests/helpers.py:assert_blocks_match_modules`` runs this over every
module block the provider tests render.
"""

import base64
import contextvars
import fnmatch
import hashlib
import json
import os
import re
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from . import hcl
from .hcl import Block, Body, Node


class PlanError(ValueError):
    pass


class _Unknown:
    """A value known only after apply."""

    _inst = None

    def __new__(cls):
        if cls._inst is None:
            cls._inst = super().__new__(cls)
        return cls._inst

    def __repr__(self) -> str:
        return "(known after apply)"


UNKNOWN = _Unknown()


class _Instance:
    """One resource / data instance: every attribute is known after apply."""

    def __init__(self, addr: str):
        self.addr = addr


class _InstanceList(list):
    """A resource with ``count``: a list of instances that must be indexed."""

    def __init__(self, addr: str, items):
        super().__init__(items)
        self.addr = addr


class _InstanceMap(dict):
    """A resource with ``for_each``: instances by key."""

    def __init__(self, addr: str, items):
        super().__init__(items)
        self.addr = addr


def _is_unknown(v: Any) -> bool:
    if v is UNKNOWN:
        return True
    if isinstance(v, list):
        return any(_is_unknown(x) for x in v)
    if isinstance(v, dict):
        return any(_is_unknown(x) for x in v.values())
    return False


def _tf_str(v: Any) -> str:
    if v is None:
        raise PlanError("a null value cannot be used in a string")
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, (int, float, str)):
        return str(v)
    raise PlanError(f"cannot use a {_kind(v)} where a string is required")


def _num(v: Any) -> float:
    if isinstance(v, bool) or v is None:
        raise PlanError(f"a {_kind(v)} is not a number")
    if isinstance(v, (int, float)):
        return v
    if isinstance(v, str):
        try:
            return int(v) if re.fullmatch(r"[+-]?[0-9]+", v.strip()) else float(v)
        except ValueError as exc:
            raise PlanError(f"{v!r} is not a number") from exc
    raise PlanError(f"a {_kind(v)} is not a number")


def _bool(v: Any) -> bool:
    if isinstance(v, bool):
        return v
    if isinstance(v, str) and v in ("true", "false"):
        return v == "true"
    raise PlanError(f"a {_kind(v)} ({v!r}) is not a bool")


def _kind(v: Any) -> str:
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, (int, float)):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, (_InstanceList,)):
        return f"list of {v.addr} instances"
    if isinstance(v, list):
        return "list"
    if isinstance(v, dict):
        return "object"
    if isinstance(v, _Instance):
        return "resource instance"
    return type(v).__name__


# --- functions ----------------------------------------------------------------------------------
# Files outside the module directory (SSH keys and the like) belong to the machine that
# runs terraform; plan_module(check_files=False) treats a missing one as unknown.
@dataclass
class _Run:
    """The plan in progress (per thread / context): what file() may treat as unknown, and
    the fully known templatefile() renderings collected for the report."""
    check_files: bool = True
    module_dir: str = ""
    rendered: List[Tuple[str, str]] = field(default_factory=list)


_RUN: contextvars.ContextVar = contextvars.ContextVar("tk_plan_run", default=_Run())


def _f_file(path):
    p = os.path.expanduser(_tf_str(path))
    if not os.path.isfile(p):
        run = _RUN.get()
        inside = bool(run.module_dir) and os.path.abspath(p).startswith(run.module_dir + os.sep)
        if not inside and not run.check_files:
            return UNKNOWN
        raise PlanError(f"file({p!r}): no such file")
    with open(p, encoding="utf-8") as fh:
        return fh.read()


def _f_fileset(base, pattern):
    base, pattern = _tf_str(base), _tf_str(pattern)
    out = []
    for root, _dirs, files in os.walk(base):
        for f in files:
            rel = os.path.relpath(os.path.join(root, f), base).replace(os.sep, "/")
            if fnmatch.fnmatchcase(rel, pattern.replace("**/", "*")) or fnmatch.fnmatchcase(rel, pattern):
                out.append(rel)
    return sorted(out)


def _f_templatefile(path, variables):
    if not isinstance(variables, dict):
        raise PlanError(f"templatefile() vars must be an object, not a {_kind(variables)}")
    src = _f_file(path)
    if _is_unknown(variables):
        hcl.parse_template(src, os.path.basename(path))  # parses; names were checked statically
        return UNKNOWN
    try:
        text = hcl.templatefile(src, variables, os.path.basename(path))
    except (hcl.TemplateError, KeyError, TypeError, IndexError) as exc:
        raise PlanError(f"templatefile({os.path.basename(path)!r}): {exc}") from exc
    _RUN.get().rendered.append((os.path.basename(path), text))
    return text


def _f_lookup(m, key, *default):
    if not isinstance(m, dict):
        raise PlanError(f"lookup() needs a map, not a {_kind(m)}")
    k = _tf_str(key)
    if k in m:
        return m[k]
    if default:
        return default[0]
    raise PlanError(f"lookup(): key {k!r} not in the map and no default")


def _f_merge(*maps):
    out: Dict[str, Any] = {}
    for m in maps:
        if m is None:
            continue
        if not isinstance(m, dict):
            raise PlanError(f"merge() arguments must be maps or objects, not a {_kind(m)}")
        out.update(m)
    return out


def _f_substr(s, offset, length):
    s, o, n = _tf_str(s), int(_num(offset)), int(_num(length))
    if o < 0:
        o += len(s)
    if o < 0 or o > len(s):
        raise PlanError(f"substr(): offset {o} out of range for a {len(s)}-character string")
    return s[o:] if n < 0 else s[o:o + n]


def _f_length(v):
    if isinstance(v, (list, dict, str)):
        return len(v)
    raise PlanError(f"length() of a {_kind(v)}")


def _f_join(sep, items):
    if not isinstance(items, list):
        raise PlanError(f"join() needs a list, not a {_kind(items)}")
    return _tf_str(sep).join(_tf_str(x) for x in items)


def _f_element(lst, idx):
    if not isinstance(lst, list) or not lst:
        raise PlanError("element() needs a non-empty list")
    return lst[int(_num(idx)) % len(lst)]


def _f_slice(lst, a, b):
    if not isinstance(lst, list):
        raise PlanError(f"slice() needs a list, not a {_kind(lst)}")
    a, b = int(_num(a)), int(_num(b))
    if not 0 <= a <= b <= len(lst):
        raise PlanError(f"slice(): [{a}:{b}] out of range for {len(lst)} elements")
    return lst[a:b]


def _f_replace(s, sub, rep):
    s, sub, rep = _tf_str(s), _tf_str(sub), _tf_str(rep)
    if len(sub) > 1 and sub.startswith("/") and sub.endswith("/"):
        return re.sub(sub[1:-1], re.sub(r"\$(\d+)", r"\\\1", rep), s)
    return s.replace(sub, rep)


def re2(pattern: str) -> str:
    """A Terraform (RE2) pattern for Python's ``re``: RE2's ``$`` matches only at the end of
    the text (without the ``m`` flag), Python's also before a final newline."""
    return re.sub(r"(?<!\\)\$", r"\\Z", pattern)


def _f_alltrue(items):
    return all(_tf_bool(x) for x in items)


def _f_anytrue(items):
    return any(_tf_bool(x) for x in items)


def _tf_bool(v):
    if isinstance(v, bool):
        return v
    if v in ("true", "false"):
        return v == "true"
    raise PlanError(f"a bool is required, got {v!r}")


def _f_regexall(pattern, s):
    rx = re.compile(re2(_tf_str(pattern)))
    out = []
    for m in rx.finditer(_tf_str(s)):
        if rx.groups == 0:
            out.append(m.group(0))
        elif rx.groupindex:
            out.append({k: m.group(k) for k in rx.groupindex})
        else:
            out.append(list(m.groups()))
    return out


def _f_tostring(v):
    if v is None:
        return None
    return _tf_str(v)


def _f_tonumber(v):
    if v is None:
        return None
    return _num(v)


def _f_keys(m):
    if not isinstance(m, dict):
        raise PlanError(f"keys() needs a map, not a {_kind(m)}")
    return sorted(m)


def _f_values(m):
    if not isinstance(m, dict):
        raise PlanError(f"values() needs a map, not a {_kind(m)}")
    return [m[k] for k in sorted(m)]


def _f_contains(lst, v):
    if not isinstance(lst, list):
        raise PlanError(f"contains() needs a list or set, not a {_kind(lst)}")
    return v in lst


def _f_sort(lst):
    if not isinstance(lst, list):
        raise PlanError(f"sort() needs a list, not a {_kind(lst)}")
    return sorted(_tf_str(x) for x in lst)


def _f_jsonencode(v):
    def conv(x):
        if isinstance(x, _Instance):
            raise PlanError("jsonencode() of a resource instance")
        return x

    return json.dumps(conv(v), separators=(",", ":"), sort_keys=True)


# name -> (callable, min args, max args or None)
FUNCTIONS: Dict[str, Tuple[Callable[..., Any], int, Optional[int]]] = {
    "alltrue": (_f_alltrue, 1, 1),
    "anytrue": (_f_anytrue, 1, 1),
    "base64encode": (lambda s: base64.b64encode(_tf_str(s).encode()).decode(), 1, 1),
    "concat": (lambda *ls: [x for lst in ls for x in lst], 0, None),
    "contains": (_f_contains, 2, 2),
    "element": (_f_element, 2, 2),
    "file": (_f_file, 1, 1),
    "fileset": (_f_fileset, 2, 2),
    "join": (_f_join, 2, 2),
    "jsonencode": (_f_jsonencode, 1, 1),
    "keys": (_f_keys, 1, 1),
    "length": (_f_length, 1, 1),
    "lookup": (_f_lookup, 2, 3),
    "lower": (lambda s: _tf_str(s).lower(), 1, 1),
    "merge": (_f_merge, 0, None),
    "pathexpand": (lambda p: os.path.expanduser(_tf_str(p)), 1, 1),
    "regexall": (_f_regexall, 2, 2),
    "replace": (_f_replace, 3, 3),
    "sha256": (lambda s: hashlib.sha256(_tf_str(s).encode()).hexdigest(), 1, 1),
    "slice": (_f_slice, 3, 3),
    "sort": (_f_sort, 1, 1),
    "split": (lambda sep, s: _tf_str(s).split(_tf_str(sep)), 2, 2),
    "substr": (_f_substr, 3, 3),
    "templatefile": (_f_templatefile, 2, 2),
    "tonumber": (_f_tonumber, 1, 1),
    "tostring": (_f_tostring, 1, 1),
    "trimspace": (lambda s: _tf_str(s).strip(), 1, 1),
    "trimsuffix": (lambda s, suf: _tf_str(s)[:-len(_tf_str(suf))] if _tf_str(suf) and _tf_str(s).endswith(
        _tf_str(suf)) else _tf_str(s), 2, 2),
    "upper": (lambda s: _tf_str(s).upper(), 1, 1),
    "values": (_f_values, 1, 1),
}


# --- the evaluator ------------------------------------------------------------------------------
class _Scope:
    """Name resolution for one evaluation: roots (var, local, path, resource types, ...)."""

    def __init__(self, plan: "_ModulePlan", extra: Optional[Dict[str, Any]] = None):
        self.plan = plan
        self.extra = dict(extra or {})

    def with_(this, **kw) -> "_Scope":  # noqa: N805 - "self" is a binding name callers pass
        s = _Scope(this.plan, this.extra)
        s.extra.update(kw)
        return s

    def root(self, name: str) -> Any:
        if name in self.extra:
            return self.extra[name]
        return self.plan.root(name)


def _traverse(base: Any, step: Node, scope: _Scope, where: str) -> Any:
    if step.kind == "splat":
        if base is UNKNOWN:
            return UNKNOWN
        if isinstance(base, list):
            return base
        return [] if base is None else [base]
    if step.kind == "attr":
        if base is UNKNOWN or isinstance(base, _Instance):
            return UNKNOWN
        if isinstance(base, _InstanceList):
            raise PlanError(f"{base.addr} has count: an instance key is required to read .{step.value} "
                            f"(e.g. {base.addr}[0].{step.value})")
        if isinstance(base, _InstanceMap):
            raise PlanError(f"{base.addr} has for_each: an instance key is required to read .{step.value}")
        if isinstance(base, dict):
            if step.value not in base:
                raise PlanError(f"{where}has no attribute {step.value!r}")
            return base[step.value]
        if isinstance(base, list) and step.value.isdigit():
            return _index(base, int(step.value), where)
        raise PlanError(f"cannot read .{step.value} of a {_kind(base)}")
    if step.kind == "index":
        key = evaluate(step.children[0], scope)
        if base is UNKNOWN or key is UNKNOWN or isinstance(base, _Instance):
            return UNKNOWN
        if isinstance(base, list):
            return _index(base, int(_num(key)), where)
        if isinstance(base, dict):
            k = _tf_str(key)
            if k not in base:
                raise PlanError(f"{where}has no element {k!r}")
            return base[k]
        raise PlanError(f"cannot index a {_kind(base)}")
    raise PlanError(f"unsupported traversal {step.kind}")


def _index(lst: list, i: int, where: str) -> Any:
    if not 0 <= i < len(lst):
        raise PlanError(f"{where}index {i} out of range for {len(lst)} elements")
    return lst[i]


def _arith(op: str, a: Any, b: Any) -> Any:
    x, y = _num(a), _num(b)
    if op == "+":
        return x + y
    if op == "-":
        return x - y
    if op == "*":
        return x * y
    if op in ("/", "%") and y == 0:
        raise PlanError("division by zero")
    if op == "/":
        return x / y
    if op == "%":
        return x % y
    return {"<": x < y, ">": x > y, "<=": x <= y, ">=": x >= y}[op]


def evaluate(node: Node, scope: _Scope) -> Any:
    k = node.kind
    if k == "lit":
        return node.value
    if k == "paren":
        return evaluate(node.children[0], scope)
    if k == "trav":
        if node.value is None:
            base, steps, name = evaluate(node.children[0], scope), node.children[1:], "value "
        else:
            base, steps, name = scope.root(node.value), node.children, node.value
        for i, st in enumerate(steps):
            where = f"{name} " if isinstance(name, str) else ""
            if st.kind == "splat":
                # a splat maps the remaining steps over the elements: x[*].id
                base = _traverse(base, st, scope, where)
                if base is UNKNOWN:
                    return UNKNOWN
                rest = steps[i + 1:]
                out = []
                for el in base:
                    for r in rest:
                        el = _traverse(el, r, scope, where)
                    out.append(el)
                return out
            base = _traverse(base, st, scope, where)
            if st.kind == "attr":
                name = f"{name}.{st.value}" if isinstance(name, str) and name != "value " else name
        return base
    if k == "tmpl":
        return _render(node.children, scope)
    if k == "unary":
        v = evaluate(node.children[0], scope)
        if v is UNKNOWN:
            return UNKNOWN
        return (not _bool(v)) if node.value == "!" else -_num(v)
    if k == "op":
        op = node.value
        a = evaluate(node.children[0], scope)
        b = evaluate(node.children[1], scope)
        if op in ("&&", "||"):
            if a is not UNKNOWN:
                _bool(a)
            if b is not UNKNOWN:
                _bool(b)
            if a is UNKNOWN or b is UNKNOWN:
                return UNKNOWN
            return (_bool(a) and _bool(b)) if op == "&&" else (_bool(a) or _bool(b))
        if op in ("==", "!="):
            if _is_unknown(a) or _is_unknown(b):
                return UNKNOWN
            return (a == b) if op == "==" else (a != b)
        if a is not UNKNOWN and not isinstance(a, _Instance):
            _num(a)
        if b is not UNKNOWN and not isinstance(b, _Instance):
            _num(b)
        if a is UNKNOWN or b is UNKNOWN:
            return UNKNOWN
        return _arith(op, a, b)
    if k == "cond":
        c = evaluate(node.children[0], scope)
        if c is UNKNOWN:
            evaluate(node.children[1], scope)
            evaluate(node.children[2], scope)
            return UNKNOWN
        return evaluate(node.children[1] if _bool(c) else node.children[2], scope)
    if k == "tuple":
        return [evaluate(c, scope) for c in node.children]
    if k == "object":
        out: Dict[str, Any] = {}
        for item in node.children:
            key = item.children[0]
            if key.kind == "trav" and not key.children:
                kv = key.value
            else:
                kv = evaluate(key, scope)
                if kv is UNKNOWN:
                    return UNKNOWN
                kv = _tf_str(kv)
            out[kv] = evaluate(item.children[1], scope)
        return out
    if k == "for":
        return _for(node, scope)
    if k == "call":
        return _call(node, scope)
    raise PlanError(f"unsupported expression {k}")


def _for(node: Node, scope: _Scope) -> Any:
    names, is_obj = node.value["names"], node.value["object"]
    coll = evaluate(node.children[0], scope)
    if coll is UNKNOWN:
        return UNKNOWN
    if isinstance(coll, dict):
        items = sorted(coll.items())
    elif isinstance(coll, list):
        items = list(enumerate(coll))
    else:
        raise PlanError(f"a for expression needs a collection, not a {_kind(coll)}")
    out_list: List[Any] = []
    out_obj: Dict[str, Any] = {}
    nchild = 3 if is_obj else 2
    cond = node.children[nchild] if len(node.children) > nchild else None
    for key, val in items:
        bind = {names[0]: val} if len(names) == 1 else {names[0]: key, names[1]: val}
        inner = scope.with_(**bind)
        if cond is not None:
            c = evaluate(cond, inner)
            if c is UNKNOWN:
                return UNKNOWN
            if not _bool(c):
                continue
        if is_obj:
            kv = evaluate(node.children[1], inner)
            vv = evaluate(node.children[2], inner)
            if kv is UNKNOWN:
                return UNKNOWN
            kv = _tf_str(kv)
            if node.value.get("group"):
                out_obj.setdefault(kv, []).append(vv)
            else:
                if kv in out_obj:
                    raise PlanError(f"duplicate key {kv!r} in a for expression (use ... to group)")
                out_obj[kv] = vv
        else:
            out_list.append(evaluate(node.children[1], inner))
    return out_obj if is_obj else out_list


def _call(node: Node, scope: _Scope) -> Any:
    name = node.value
    if name in ("try", "can"):
        # lazy: the first argument that evaluates without error (can: whether the first does)
        for arg in node.children:
            try:
                v = evaluate(arg, scope)
                return True if name == "can" else v
            except PlanError:
                if name == "can":
                    return False
        if name == "can":
            return False
        raise PlanError("try(): no argument evaluated without errors")
    args = [evaluate(c, scope) for c in node.children]
    spec = FUNCTIONS.get(name)
    if spec is None:
        if name not in hcl.TERRAFORM_FUNCTIONS:
            raise PlanError(f"call to unknown function {name}()")
        return UNKNOWN  # a real function this evaluator does not model
    fn, lo, hi = spec
    if len(args) < lo or (hi is not None and len(args) > hi):
        want = f"{lo}" if lo == hi else f"{lo}..{hi if hi is not None else 'n'}"
        raise PlanError(f"{name}() takes {want} arguments, got {len(args)}")
    if name == "templatefile":
        if args[0] is UNKNOWN:
            return UNKNOWN
        return fn(*args)
    if any(_is_unknown(a) for a in args):
        return UNKNOWN
    try:
        return fn(*args)
    except PlanError:
        raise
    except (TypeError, ValueError, KeyError, IndexError, re.error) as exc:
        raise PlanError(f"{name}(): {exc}") from exc


def _render(parts: List[Node], scope: _Scope) -> Any:
    parts = hcl._apply_strip(parts)
    out: List[str] = []
    unknown = False

    def run(i: int, end_kinds: Tuple[str, ...], emit: bool) -> int:
        nonlocal unknown
        while i < len(parts):
            p = parts[i]
            if p.kind in end_kinds:
                return i
            if p.kind == "lit":
                if emit:
                    out.append(p.value)
                i += 1
            elif p.kind == "interp":
                v = evaluate(p.children[0], scope)
                if emit:
                    if _is_unknown(v):
                        unknown = True
                    else:
                        out.append(_tf_str(v))
                i += 1
            elif p.kind == "if":
                c = evaluate(p.children[0], scope)
                if c is UNKNOWN:
                    unknown = True
                    c = False
                cond = _bool(c)
                j = run(i + 1, ("else", "endif"), emit and cond)
                if parts[j].kind == "else":
                    j = run(j + 1, ("endif",), emit and not cond)
                i = j + 1
            elif p.kind == "tfor":
                coll = evaluate(p.children[0], scope)
                end = hcl._matching_endfor(parts, i)
                if coll is UNKNOWN:
                    unknown = True
                elif emit:
                    items = sorted(coll.items()) if isinstance(coll, dict) else list(enumerate(coll))
                    names = p.value
                    for key, val in items:
                        bind = {names[0]: val} if len(names) == 1 else {names[0]: key, names[1]: val}
                        saved = scope.extra
                        scope.extra = dict(saved, **bind)
                        try:
                            run(i + 1, ("endfor",), True)
                        finally:
                            scope.extra = saved
                i = end + 1
            else:
                raise PlanError(f"unexpected template part {p.kind}")
        return i

    run(0, (), True)
    return UNKNOWN if unknown else "".join(out)


# --- module-level plan --------------------------------------------------------------------------
@dataclass
class PlanReport:
    module: str
    errors: List[str] = field(default_factory=list)
    locals: Dict[str, Any] = field(default_factory=dict)
    outputs: Dict[str, Any] = field(default_factory=dict)
    instances: Dict[str, int] = field(default_factory=dict)  # resource/data address -> instance count
    # template file name -> texts of the templatefile() calls whose inputs are all known
    rendered: Dict[str, List[str]] = field(default_factory=dict)

    @property
    def ok(self) -> bool:
        return not self.errors


def _convert(vtype: Optional[Node], value: Any, name: str) -> Any:
    """An input value converted to the variable's declared type (Terraform's rules)."""
    if isinstance(value, str) and "${" in value:
        return UNKNOWN
    if value is None or vtype is None:
        return value
    if vtype.kind == "trav" and not vtype.children:
        t = vtype.value
        if t == "string":
            if isinstance(value, (dict, list)):
                raise PlanError(f"var.{name}: a {_kind(value)} is not a string")
            return _tf_str(value)
        if t == "number":
            return _num(value)
        if t == "bool":
            return _bool(value)
        return value  # any
    if vtype.kind == "call" and vtype.children:
        inner = vtype.children[0]
        if vtype.value in ("list", "set"):
            if not isinstance(value, list):
                raise PlanError(f"var.{name}: a {_kind(value)} is not a {vtype.value}")
            return [_convert(inner, v, name) for v in value]
        if vtype.value == "map":
            if not isinstance(value, dict):
                raise PlanError(f"var.{name}: a {_kind(value)} is not a map")
            return {k: _convert(inner, v, name) for k, v in value.items()}
    return value


class _ModulePlan:
    def __init__(self, module_dir: str, inputs: Dict[str, Any]):
        self.dir = os.path.abspath(module_dir)
        self.name = os.path.basename(self.dir.rstrip("/"))
        self.report = PlanReport(self.name)
        rep = hcl.check_module(self.dir)
        self.report.errors += rep.errors
        self.files: Dict[str, Body] = rep.files
        self.sources: Dict[str, str] = {}
        for fn in self.files:
            with open(os.path.join(self.dir, fn), encoding="utf-8") as fh:
                self.sources[fn] = fh.read()
        self.blocks: List[Tuple[str, Block]] = [(fn, b) for fn, body in self.files.items() for b in body.blocks]
        self.local_nodes: Dict[str, Tuple[str, Node]] = {}
        for fn, b in self.blocks:
            if b.type == "locals":
                for a in b.body.attributes:
                    self.local_nodes[a.name] = (fn, a.expr)
        self.local_values: Dict[str, Any] = {}
        self.local_busy: List[str] = []
        self.resources: Dict[Tuple[str, str, str], Tuple[str, Block]] = {}
        for fn, b in self.blocks:
            if b.type in ("resource", "data") and len(b.labels) == 2:
                self.resources[(b.type, b.labels[0], b.labels[1])] = (fn, b)
        self.resource_values: Dict[Tuple[str, str, str], Any] = {}
        self.vars = self._inputs(inputs)
        self.scope = _Scope(self)
        self._validate()

    def _validate(self) -> None:
        """The variables' ``validation`` blocks, as Terraform checks them before planning
        ("Invalid value for variable"); a condition over an unknown value is skipped."""
        for fn, b in self.blocks:
            if b.type != "variable" or not b.labels or _is_unknown(self.vars.get(b.labels[0])):
                continue
            for vb in b.body.blocks:
                cond = vb.body.attr("condition") if vb.type == "validation" else None
                if cond is None:
                    continue
                try:
                    ok = evaluate(cond.expr, self.scope)
                    if _is_unknown(ok) or ok is not False:
                        continue
                    msg_attr = vb.body.attr("error_message")
                    msg = evaluate(msg_attr.expr, self.scope) if msg_attr is not None else "validation failed"
                except PlanError as exc:
                    msg = f"validation condition: {exc}"
                self.report.errors.append(f"{self.where(fn, vb.pos)}: Invalid value for variable "
                                          f"{b.labels[0]!r}: {msg}")

    def where(self, fn: str, pos: int) -> str:
        return f"{self.name}/{fn}:{self.sources[fn].count(chr(10), 0, pos) + 1}"

    def _inputs(self, inputs: Dict[str, Any]) -> Dict[str, Any]:
        out: Dict[str, Any] = {}
        for fn, b in self.blocks:
            if b.type != "variable" or not b.labels:
                continue
            name = b.labels[0]
            tattr, dattr = b.body.attr("type"), b.body.attr("default")
            try:
                if name in inputs:
                    raw = inputs[name]
                elif dattr is not None:
                    raw = evaluate(dattr.expr, _Scope(self, {}))
                else:
                    self.report.errors.append(f"{self.where(fn, b.pos)}: variable {name!r} is required")
                    out[name] = UNKNOWN
                    continue
                out[name] = _convert(tattr.expr if tattr else None, raw, name)
            except PlanError as exc:
                self.report.errors.append(f"{self.where(fn, b.pos)}: {exc}")
                out[name] = UNKNOWN
        return out

    # roots -------------------------------------------------------------------------------------
    def root(self, name: str) -> Any:
        if name == "var":
            return self.vars
        if name == "local":
            return _LocalView(self)
        if name == "path":
            return {"module": self.dir, "root": os.getcwd(), "cwd": os.getcwd()}
        if name == "terraform":
            return {"workspace": "default"}
        if name == "data":
            return {t: {n: self.resource_value(("data", t, n)) for (m, tt, n) in self.resources if m == "data"
                        and tt == t} for (m, t, _) in self.resources if m == "data"}
        if name == "module":
            return _AnyView()
        if name in ("self", "count", "each"):
            raise PlanError(f"{name} is not available here")
        types = {t for (m, t, _) in self.resources if m == "resource"}
        if name in types:
            return {n: self.resource_value(("resource", name, n)) for (m, t, n) in self.resources
                    if m == "resource" and t == name}
        raise PlanError(f"unknown reference {name!r}")

    def local(self, name: str) -> Any:
        if name in self.local_values:
            return self.local_values[name]
        if name not in self.local_nodes:
            raise PlanError(f"local.{name} is not defined")
        if name in self.local_busy:
            raise PlanError("cycle among locals: " + " -> ".join(self.local_busy + [name]))
        self.local_busy.append(name)
        try:
            fn, expr = self.local_nodes[name]
            value = evaluate(expr, self.scope)
        finally:
            self.local_busy.pop()
        self.local_values[name] = value
        return value

    def resource_value(self, key: Tuple[str, str, str]) -> Any:
        if key in self.resource_values:
            return self.resource_values[key]
        fn, b = self.resources[key]
        addr = ".".join(key[1:]) if key[0] == "resource" else "data." + ".".join(key[1:])
        count, each = b.body.attr("count"), b.body.attr("for_each")
        if count is not None:
            n = evaluate(count.expr, self.scope)
            if _is_unknown(n):
                raise PlanError(f"{addr}: the count value depends on values known only after apply")
            n = int(_num(n))
            if n < 0:
                raise PlanError(f"{addr}: count must not be negative")
            value: Any = _InstanceList(addr, [_Instance(f"{addr}[{i}]") for i in range(n)])
        elif each is not None:
            coll = evaluate(each.expr, self.scope)
            if _is_unknown(coll) and not isinstance(coll, (list, dict)):
                raise PlanError(f"{addr}: the for_each value depends on values known only after apply")
            keys = sorted(coll) if isinstance(coll, dict) else [_tf_str(x) for x in coll]
            value = _InstanceMap(addr, {k: _Instance(f"{addr}[{k!r}]") for k in keys})
        else:
            value = _Instance(addr)
        self.resource_values[key] = value
        return value

    # blocks ------------------------------------------------------------------------------------
    def eval_body(self, fn: str, body: Body, scope: _Scope, skip: Tuple[str, ...] = ()) -> None:
        for a in body.attributes:
            if a.name in skip:
                continue
            try:
                evaluate(a.expr, scope)
            except PlanError as exc:
                self.report.errors.append(f"{self.where(fn, a.pos)}: {a.name}: {exc}")
        for nb in body.blocks:
            if nb.type == "lifecycle":
                self.eval_conditions(fn, nb, scope)
                continue
            if nb.type == "dynamic" and nb.labels:
                self.eval_dynamic(fn, nb, scope)
                continue
            inner = scope.with_(self=_Instance("self")) if nb.type in ("connection", "provisioner") else scope
            if nb.type == "provisioner":
                self.check_provisioner_meta(fn, nb)
                self.eval_body(fn, nb.body, inner, skip=("when", "on_failure"))
            else:
                self.eval_body(fn, nb.body, inner)
            if nb.type == "provisioner" and nb.labels == ["file"]:
                self.check_upload(fn, nb, inner)

    # keyword meta-arguments of a provisioner, and what a destroy-time one may reference
    PROVISIONER_KEYWORDS = {"when": ("create", "destroy"), "on_failure": ("continue", "fail")}
    DESTROY_REFS = ("self", "count", "each", "path", "terraform")

    def check_provisioner_meta(self, fn: str, blk: Block) -> None:
        """``when`` / ``on_failure`` take keywords, not expressions; a destroy-time
        provisioner (and its connection) may reference only ``self``, ``count.index``,
        ``each.key``, ``path`` and ``terraform`` -- Terraform refuses anything else
        ("Invalid reference from destroy provisioner")."""
        destroy = False
        for name, allowed in self.PROVISIONER_KEYWORDS.items():
            a = blk.body.attr(name)
            if a is None:
                continue
            word = a.expr.value if a.expr.kind == "trav" and isinstance(a.expr.value, str) else None
            if word not in allowed:
                self.report.errors.append(f"{self.where(fn, a.pos)}: {name}: must be one of {', '.join(allowed)}")
            destroy = destroy or (name == "when" and word == "destroy")
        if not destroy:
            return
        body = Body(attributes=[a for a in blk.body.attributes if a.name not in self.PROVISIONER_KEYWORDS],
                    blocks=blk.body.blocks)
        for root, _, pos in hcl.references(body):
            if root not in self.DESTROY_REFS:
                self.report.errors.append(
                    f"{self.where(fn, pos)}: invalid reference from destroy provisioner: {root} (a destroy-time "
                    f"provisioner may reference only self, count.index, each.key, path and terraform)")

    def eval_conditions(self, fn: str, lifecycle: Block, scope: _Scope) -> None:
        """``precondition`` blocks: a known false condition is the plan error Terraform
        reports ("Resource precondition failed") with the block's ``error_message``."""
        for cb in lifecycle.body.blocks:
            if cb.type != "precondition":
                continue
            cond = cb.body.attr("condition")
            if cond is None:
                continue
            try:
                ok = evaluate(cond.expr, scope)
            except PlanError as exc:
                self.report.errors.append(f"{self.where(fn, cond.pos)}: precondition: {exc}")
                continue
            if ok is UNKNOWN or _bool(ok):
                continue
            msg_attr = cb.body.attr("error_message")
            try:
                msg = _tf_str(evaluate(msg_attr.expr, scope)) if msg_attr is not None else "condition false"
            except PlanError:
                msg = "condition false"
            self.report.errors.append(f"{self.where(fn, cb.pos)}: precondition failed: {msg}")

    def check_upload(self, fn: str, blk: Block, scope: _Scope) -> None:
        """A ``file`` provisioner's ``source`` must exist where terraform runs."""
        src = blk.body.attr("source")
        if src is None:
            if blk.body.attr("content") is None:
                self.report.errors.append(f"{self.where(fn, blk.pos)}: file provisioner needs source or content")
            return
        try:
            path = evaluate(src.expr, scope)
        except PlanError:
            return  # reported by eval_body
        if path is UNKNOWN:
            return
        p = os.path.expanduser(_tf_str(path))
        if not os.path.exists(p) and (_RUN.get().check_files or p.startswith(self.dir + os.sep)):
            self.report.errors.append(f"{self.where(fn, src.pos)}: file provisioner source {p!r} does not exist")

    def eval_dynamic(self, fn: str, blk: Block, scope: _Scope) -> None:
        it_attr = blk.body.attr("iterator")
        it = it_attr.expr.value if it_attr is not None else blk.labels[0]
        fe = blk.body.attr("for_each")
        content = next((b for b in blk.body.blocks if b.type == "content"), None)
        if fe is None or content is None:
            self.report.errors.append(f"{self.where(fn, blk.pos)}: dynamic {blk.labels[0]!r} needs for_each "
                                      "and a content block")
            return
        try:
            coll = evaluate(fe.expr, scope)
        except PlanError as exc:
            self.report.errors.append(f"{self.where(fn, fe.pos)}: for_each: {exc}")
            return
        if coll is UNKNOWN:
            items: List[Tuple[Any, Any]] = [(UNKNOWN, UNKNOWN)]
        elif isinstance(coll, dict):
            items = sorted(coll.items())
        elif isinstance(coll, list):
            items = list(enumerate(coll))
        else:
            self.report.errors.append(f"{self.where(fn, fe.pos)}: dynamic for_each needs a collection, "
                                      f"not a {_kind(coll)}")
            return
        for key, val in items:
            self.eval_body(fn, content.body, scope.with_(**{it: {"key": key, "value": val}}))

    def run(self) -> PlanReport:
        for name in sorted(self.local_nodes):
            fn, expr = self.local_nodes[name]
            try:
                self.report.locals[name] = self.local(name)
            except PlanError as exc:
                self.report.errors.append(f"{self.where(fn, expr.pos)}: local.{name}: {exc}")
        for fn, b in self.blocks:
            if b.type == "provider":
                self.eval_body(fn, b.body, self.scope)
            elif b.type in ("resource", "data") and len(b.labels) == 2:
                key = (b.type, b.labels[0], b.labels[1])
                addr = ".".join(b.labels) if b.type == "resource" else "data." + ".".join(b.labels)
                try:
                    value = self.resource_value(key)
                except PlanError as exc:
                    self.report.errors.append(f"{self.where(fn, b.pos)}: {exc}")
                    continue
                if isinstance(value, _InstanceList):
                    self.report.instances[addr] = len(value)
                    scopes = [self.scope.with_(count={"index": i}) for i in range(len(value))]
                elif isinstance(value, _InstanceMap):
                    self.report.instances[addr] = len(value)
                    scopes = [self.scope.with_(each={"key": k, "value": k}) for k in value]
                else:
                    self.report.instances[addr] = 1
                    scopes = [self.scope]
                for sc in scopes:
                    self.eval_body(fn, b.body, sc, skip=("count", "for_each", "depends_on"))
            elif b.type == "output" and b.labels:
                va = b.body.attr("value")
                if va is None:
                    self.report.errors.append(f"{self.where(fn, b.pos)}: output {b.labels[0]!r} has no value")
                    continue
                try:
                    self.report.outputs[b.labels[0]] = evaluate(va.expr, self.scope)
                except PlanError as exc:
                    self.report.errors.append(f"{self.where(fn, va.pos)}: output {b.labels[0]}: {exc}")
        return self.report


class _LocalView(dict):
    """``local.<name>``: evaluated on first read."""

    def __init__(self, plan: _ModulePlan):
        super().__init__()
        self._plan = plan

    def __contains__(self, key) -> bool:  # type: ignore[override]
        return key in self._plan.local_nodes

    def __getitem__(self, key):
        return self._plan.local(key)


class _AnyView(dict):
    """``module.<name>``: outputs of child modules, known after apply."""

    def __contains__(self, key) -> bool:  # type: ignore[override]
        return True

    def __getitem__(self, key):
        return UNKNOWN


def plan_module(module_dir: str, inputs: Dict[str, Any], check_files: bool = True) -> PlanReport:
    """Evaluate every expression of the module at ``module_dir`` for one module block
    (``inputs``: the block's arguments, ``source`` ignored).  ``check_files`` False: a
    ``file()`` outside the module that does not exist here (a user's SSH key path) is
    unknown rather than an error; the module's own files are always checked."""
    given = {k: v for k, v in inputs.items() if k != "source"}
    run = _Run(check_files, os.path.abspath(module_dir))
    token = _RUN.set(run)
    try:
        report = _ModulePlan(module_dir, given).run()
    finally:
        _RUN.reset(token)
    for name, text in run.rendered:
        report.rendered.setdefault(name, []).append(text)
    return report


__all__ = ["PlanError", "PlanReport", "UNKNOWN", "plan_module", "evaluate", "FUNCTIONS"]


def plan_root(doc: Dict[str, Any], version: Tuple[int, int, int]) -> List[str]:
    """Checks on the *root* document (``main.tf.json`` as the executor renders it) that
    depend on the Terraform version running it — the failures a real Terraform reports
    before touching any resource:

    * the backend type must exist in that version (``manta`` and four others were
      removed in 1.3: "Unsupported backend type");
    * every local module's ``required_version`` must accept the version;
    * from 0.15, a root output whose value is a module output declared ``sensitive``
      must be marked ``sensitive = true`` ("Output refers to sensitive values").

    Module outputs' sensitivity is read from the module's own ``outputs.tf`` with the HCL
    parser, not from the generator, so this check and the executor's rendering (which
    reads the generator) are independent."""
    from . import constraints
    from .catalog import local_module_dir

    errors: List[str] = []
    backend = (doc.get("terraform") or {}).get("backend") or {}
    for kind in backend:
        if constraints.backend_removed(kind, version):
            errors.append(f"terraform.backend.{kind}: there is no backend type named {kind!r} in Terraform "
                          f"{constraints.fmt(version)} (removed in "
                          f"{constraints.fmt(constraints.REMOVED_BACKENDS[kind])})")
    modules = doc.get("module") or {}
    sensitive: Dict[str, Dict[str, bool]] = {}
    for key, mod in modules.items():
        local = local_module_dir(str(mod.get("source", "")))
        if local is None:
            continue
        bad = constraints.unsupported_by(version, local)
        if bad is not None:
            errors.append(f"module.{key}: required_version {bad!r} is not met by Terraform {constraints.fmt(version)}")
        outs: Dict[str, bool] = {}
        for body in hcl.check_module(local).files.values():
            for b in body.blocks:
                if b.type == "output" and b.labels:
                    attr = b.body.attr("sensitive")
                    outs[b.labels[0]] = attr is not None and evaluate(attr.expr, _Scope.__new__(_Scope)) is True
        sensitive[key] = outs
    if tuple(version) >= constraints.SENSITIVE_ROOT_OUTPUTS_FROM:
        for name, out in (doc.get("output") or {}).items():
            m = re.fullmatch(r"\$\{module\.([^.}]+)\.([^.}]+)\}", str((out or {}).get("value", "")))
            if m and sensitive.get(m.group(1), {}).get(m.group(2)) and (out or {}).get("sensitive") is not True:
                errors.append(f"output.{name}: refers to the sensitive output module.{m.group(1)}.{m.group(2)} "
                              "and must be marked sensitive = true")
    return errors


__all__.append("plan_root")
