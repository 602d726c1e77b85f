"""The hand-written HCL parser and evaluator (``terraform/hcl.py``) against generated
expressions: operator precedence and associativity (HCL's, which is not Python's: ``==``
binds looser than ``<``, comparisons do not chain), unary operators and conditionals.  Each
tree is rendered with only the parentheses HCL's precedence needs, parsed, evaluated, and
compared with a direct evaluation of the tree."""

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.terraform import hcl

PREC = {"||": 1, "&&": 2, "==": 3, "!=": 3, "<": 4, ">": 4, "<=": 4, ">=": 4, "+": 5, "-": 5, "*": 6}
UNARY, ATOM = 7, 8

def _trees(depth):
    """(numeric, boolean) expression strategies, ``depth`` operators deep at most."""
    if depth == 0:
        return st.integers(0, 99).map(lambda v: ("num", v)), st.booleans().map(lambda b: ("bool", b))
    n, b = _trees(depth - 1)
    num = st.one_of(n, n.map(lambda x: ("neg", x)),
                    st.tuples(st.sampled_from(["+", "-", "*"]), n, n).map(lambda t: ("bin",) + t),
                    st.tuples(b, n, n).map(lambda t: ("cond",) + t))
    boo = st.one_of(b, b.map(lambda x: ("not", x)),
                    st.tuples(st.sampled_from(["<", ">", "<=", ">=", "==", "!="]), n, n).map(lambda t: ("bin",) + t),
                    st.tuples(st.sampled_from(["&&", "||", "==", "!="]), b, b).map(lambda t: ("bin",) + t),
                    st.tuples(b, b, b).map(lambda t: ("cond",) + t))
    return num, boo


nums, bools = _trees(4)


def prec(t):
    fixed = {"num": ATOM, "bool": ATOM, "neg": UNARY, "not": UNARY, "cond": 0}
    return fixed[t[0]] if t[0] in fixed else PREC[t[1]]


def render(t):
    k = t[0]
    if k == "num":
        return str(t[1])
    if k == "bool":
        return "true" if t[1] else "false"
    if k in ("neg", "not"):
        inner = render(t[1])
        return ("-" if k == "neg" else "!") + (inner if prec(t[1]) >= UNARY else f"({inner})")
    if k == "cond":
        return " ? ".join([f"({render(t[1])})" if prec(t[1]) == 0 else render(t[1]),
                           f"({render(t[2])})" if prec(t[2]) == 0 else render(t[2])]) + \
            " : " + (f"({render(t[3])})" if prec(t[3]) == 0 else render(t[3]))
    op, left, right = t[1], t[2], t[3]
    p = PREC[op]
    ls = render(left) if prec(left) >= p and prec(left) != 0 else f"({render(left)})"
    rs = render(right) if prec(right) > p else f"({render(right)})"  # left-associative
    return f"{ls} {op} {rs}"


def value(t):
    k = t[0]
    if k in ("num", "bool"):
        return t[1]
    if k == "neg":
        return -value(t[1])
    if k == "not":
        return not value(t[1])
    if k == "cond":
        return value(t[2]) if value(t[1]) else value(t[3])
    op, a, b = t[1], value(t[2]), value(t[3])
    return {"+": lambda: a + b, "-": lambda: a - b, "*": lambda: a * b, "<": lambda: a < b, ">": lambda: a > b,
            "<=": lambda: a <= b, ">=": lambda: a >= b, "==": lambda: a == b, "!=": lambda: a != b,
            "&&": lambda: a and b, "||": lambda: a or b}[op]()


def hcl_value(text):
    return hcl.eval_expr(hcl.parse(f"x = {text}\n").attr("x").expr, {})


@settings(max_examples=300, deadline=None)
@given(st.one_of(nums, bools))
def test_generated_expressions_evaluate_as_their_trees(tree):
    text = render(tree)
    got, want = hcl_value(text), value(tree)
    assert got == want and isinstance(got, bool) == isinstance(want, bool), (text, got, want)


def test_hcl_precedence_is_not_pythons():
    assert hcl_value("1 < 2 == true") is True  # (1 < 2) == true; Python would chain
    assert hcl_value("2 - 3 - 4") == -5 and hcl_value("2 * 3 + 4 * 5") == 26
    assert hcl_value("true || false && false") is True
    assert hcl_value("!true == false") is True
    assert hcl_value("1 == 1 ? 2 + 3 : 4") == 5


import glob  # noqa: E402
import os  # noqa: E402

_MODULES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "triton_kubernetes_amd",
                        "terraform", "modules")
_SOURCES = sorted(glob.glob(os.path.join(_MODULES, "*", "*.tf")))
_TEMPLATES = sorted(glob.glob(os.path.join(_MODULES, "*", "files", "*.tftpl")))
_ALPHABET = '{}[]()"\'$%~<>=!?:,.\\\n\t #/*-+abcxuU0123'


@settings(max_examples=300, deadline=None)
@given(st.booleans(), st.integers(0, 10 ** 6), st.lists(st.tuples(st.sampled_from(["set", "insert", "delete"]),
                                                                  st.integers(0, 10 ** 6), st.sampled_from(_ALPHABET)),
                                                        min_size=1, max_size=6))
def test_damaged_sources_raise_only_syntax_errors(template, pick, edits):
    """Mutations of the shipped module sources and templates: the parser answers with its own
    syntax error (file:line:col), never an IndexError, ValueError or OverflowError."""
    files = _TEMPLATES if template else _SOURCES
    with open(files[pick % len(files)], encoding="utf-8") as fh:
        s = list(fh.read())
    for op, pos, ch in edits:
        i = pos % (len(s) + 1)
        if op == "set" and s:
            s[min(i, len(s) - 1)] = ch
        elif op == "insert":
            s.insert(i, ch)
        else:
            del s[i:i + 1 + pos % 20]
    try:
        (hcl.parse_template if template else hcl.parse)("".join(s))
    except (hcl.HCLSyntaxError, hcl.TemplateError):
        pass


def test_unicode_escapes():
    assert hcl_value('"a\\u00e9b\\U0001F600"') == "aéb\U0001F600"
    for bad in ('"\\urerm"', '"\\u12"', '"\\UFFFFFFFF"', '"\\U00110000"'):
        with pytest.raises(hcl.HCLSyntaxError):
            hcl_value(bad)
