"""HCL2 native-syntax parser and a static checker for this project's Terraform modules.

There is no ``terraform`` binary in CI, so the generated modules need a parser of
their own to be checked at all.  This is a scannerless recursive-descent parser of
the HCL2 native syntax Terraform ≥0.12 reads:

* bodies of attributes (``name = expr``) and blocks (``type "label" ident { … }``);
* expressions: literals, template strings with ``${…}`` interpolations and
  ``%{if}/%{else}/%{endif}`` / ``%{for}/%{endfor}`` directives (strip markers ``~``),
  heredocs (``<<EOT`` / ``<<-EOT``), tuples, objects, function calls (``f(a, b...)``),
  traversals (``a.b[0].c``, ``.*``, ``[*]``), unary/binary operators with HCL's
  precedence, conditionals and ``for`` expressions in both brackets;
* newlines terminate attributes in bodies and separate object items, and are
  insignificant inside ``()`` and ``[]``, as in the HCL spec.

:func:`check_module` then does what ``terraform validate`` would catch first for
these modules: every ``var.X`` declared, every ``local.X`` defined, every
``data.T.N`` / ``T.N`` resource reference defined, and every
``templatefile(path, {…})`` call passing exactly the names its template uses
(Terraform fails on a missing one at apply time).  :func:`parse_template` checks
``.tftpl`` files on their own (balanced directives, valid interpolation syntax).

The reference ships Terraform 0.11 modules and has no checker; this is new
("no terraform in the dev sandbox").
"""

import os
import re
import threading
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Set, Tuple


class HCLSyntaxError(ValueError):
    def __init__(self, msg: str, src: str, pos: int, name: str = "<hcl>"):
        line = src.count("\n", 0, pos) + 1
        col = pos - (src.rfind("\n", 0, pos) + 1) + 1
        super().__init__(f"{name}:{line}:{col}: {msg}")
        self.line, self.col = line, col


# --- AST ---------------------------------------------------------------------------------------
@dataclass
class Node:
    kind: str  # lit | tmpl | trav | call | tuple | object | op | unary | cond | for | paren
    value: Any = None
    children: List["Node"] = field(default_factory=list)
    pos: int = 0
    # template parts only: whitespace strip markers ``~`` on the (left, right) of ``${``/``%{``
    strip: Tuple[bool, bool] = (False, False)


@dataclass
class Attribute:
    name: str
    expr: Node
    pos: int


@dataclass
class Block:
    type: str
    labels: List[str]
    body: "Body"
    pos: int


@dataclass
class Body:
    attributes: List[Attribute] = field(default_factory=list)
    blocks: List[Block] = field(default_factory=list)

    def attr(self, name: str) -> Optional[Attribute]:
        return next((a for a in self.attributes if a.name == name), None)

    def blocks_of(self, kind: str) -> List[Block]:
        return [b for b in self.blocks if b.type == kind]


_IDENT_RE = re.compile(r"[A-Za-z_][A-Za-z0-9_-]*")
_NUM_RE = re.compile(r"[0-9]+(\.[0-9]+)?([eE][+-]?[0-9]+)?")
_BINARY = [("||",), ("&&",), ("==", "!="), ("<=", ">=", "<", ">"), ("+", "-"), ("*", "/", "%")]
_KEYWORD_LITS = {"true": True, "false": False, "null": None}


class _Parser:
    def __init__(self, src: str, name: str):
        self._rstrip = False
        self.s = src
        self.n = len(src)
        self.i = 0
        self.name = name

    # --- low level -------------------------------------------------------------------------------
    def err(self, msg: str, pos: Optional[int] = None) -> HCLSyntaxError:
        return HCLSyntaxError(msg, self.s, self.i if pos is None else pos, self.name)

    def skip(self, newlines: bool) -> None:
        """Skip blanks and comments (and newlines when ``newlines``)."""
        s, n = self.s, self.n
        while self.i < n:
            c = s[self.i]
            if c in " \t\r":
                self.i += 1
            elif c == "\n" and newlines:
                self.i += 1
            elif c == "#" or s.startswith("//", self.i):
                j = s.find("\n", self.i)
                self.i = n if j < 0 else j
            elif s.startswith("/*", self.i):
                j = s.find("*/", self.i + 2)
                if j < 0:
                    raise self.err("unterminated /* comment")
                self.i = j + 2
            else:
                break

    def peek(self, tok: str) -> bool:
        return self.s.startswith(tok, self.i)

    def eat(self, tok: str, newlines: bool) -> bool:
        self.skip(newlines)
        if self.s.startswith(tok, self.i):
            self.i += len(tok)
            return True
        return False

    def expect(self, tok: str, newlines: bool, what: str = "") -> None:
        if not self.eat(tok, newlines):
            found = self.s[self.i:self.i + 12].split("\n")[0] or "end of input"
            raise self.err(f"expected {tok!r}{' ' + what if what else ''}, found {found!r}")

    def ident(self, newlines: bool) -> Optional[str]:
        self.skip(newlines)
        m = _IDENT_RE.match(self.s, self.i)
        if not m:
            return None
        self.i = m.end()
        return m.group(0)

    # --- bodies ------------------------------------------------------------------------------------
    def body(self, closing: Optional[str]) -> Body:
        out = Body()
        while True:
            self.skip(True)
            if self.i >= self.n:
                if closing:
                    raise self.err(f"expected {closing!r} before end of input")
                return out
            if closing and self.peek(closing):
                self.i += 1
                return out
            start = self.i
            name = self.ident(False)
            if name is None:
                raise self.err("expected an attribute name or block type")
            self.skip(False)
            if self.peek("=") and not self.peek("=="):
                self.i += 1
                expr = self.expr(False)
                out.attributes.append(Attribute(name, expr, start))
                self.end_of_line()
                continue
            labels: List[str] = []
            while True:
                self.skip(False)
                if self.peek('"'):
                    lab = self.string()
                    if lab.kind != "lit":
                        raise self.err("block labels must be literal strings", lab.pos)
                    labels.append(lab.value)
                    continue
                lab_ident = self.ident(False)
                if lab_ident is not None:
                    labels.append(lab_ident)
                    continue
                break
            self.expect("{", False, f"to open block {name!r}")
            blk = self.body("}")
            out.blocks.append(Block(name, labels, blk, start))
            self.end_of_line()

    def end_of_line(self) -> None:
        self.skip(False)
        if self.i >= self.n or self.s[self.i] in "\n}":
            if self.i < self.n and self.s[self.i] == "\n":
                self.i += 1
            return
        raise self.err(f"unexpected {self.s[self.i:self.i + 12].split(chr(10))[0]!r} after a definition")

    # --- expressions ------------------------------------------------------------------------------
    def expr(self, nl: bool) -> Node:
        cond = self.binary(0, nl)
        self.skip(nl)
        if self.peek("?"):
            self.i += 1
            a = self.expr(nl)
            self.expect(":", nl, "in conditional")
            b = self.expr(nl)
            return Node("cond", None, [cond, a, b], cond.pos)
        return cond

    def binary(self, level: int, nl: bool) -> Node:
        if level == len(_BINARY):
            return self.unary(nl)
        left = self.binary(level + 1, nl)
        while True:
            self.skip(nl)
            op = next((o for o in _BINARY[level] if self.peek(o)), None)
            # "=>" / "==" are not "=", "<" is not "<<" (heredoc) or "<=" handled above
            if op is None or (op in ("<", ">") and self.peek(op + "=")) or (op == "/" and self.peek("//")) \
                    or (op == "*" and self.peek("*/")):
                return left
            self.i += len(op)
            right = self.binary(level + 1, nl)
            left = Node("op", op, [left, right], left.pos)

    def unary(self, nl: bool) -> Node:
        self.skip(nl)
        if self.peek("!") and not self.peek("!="):
            pos = self.i
            self.i += 1
            return Node("unary", "!", [self.unary(nl)], pos)
        if self.peek("-"):
            pos = self.i
            self.i += 1
            return Node("unary", "-", [self.unary(nl)], pos)
        return self.postfix(self.primary(nl), nl)

    def postfix(self, node: Node, nl: bool) -> Node:
        while True:
            # traversal operators bind tightly: no newline may precede them
            if self.peek(".*"):
                self.i += 2
                node = Node("trav", node.value if node.kind == "trav" else None, node.children + [Node("splat")]
                            if node.kind == "trav" else [node, Node("splat")], node.pos)
                continue
            if self.peek(".") and not self.peek("..."):
                self.i += 1
                m = _NUM_RE.match(self.s, self.i)
                name = None
                if m:
                    self.i = m.end()
                    name = m.group(0)
                else:
                    name = self.ident(False)
                if name is None:
                    raise self.err("expected an attribute name after '.'")
                node = self._extend(node, Node("attr", name, pos=self.i))
                continue
            if self.peek("["):
                self.i += 1
                self.skip(True)
                if self.peek("*"):
                    self.i += 1
                    self.expect("]", True, "after '[*'")
                    node = self._extend(node, Node("splat"))
                    continue
                key = self.expr(True)
                self.expect("]", True, "to close an index")
                node = self._extend(node, Node("index", None, [key]))
                continue
            return node

    @staticmethod
    def _extend(node: Node, step: Node) -> Node:
        if node.kind == "trav":
            return Node("trav", node.value, node.children + [step], node.pos)
        return Node("trav", None, [node, step], node.pos)  # traversal of an expression result

    def primary(self, nl: bool) -> Node:
        self.skip(nl)
        pos = self.i
        if self.i >= self.n:
            raise self.err("expected an expression before end of input")
        c = self.s[self.i]
        if c == '"':
            return self.string()
        if self.peek("<<"):
            return self.heredoc()
        if c.isdigit():
            m = _NUM_RE.match(self.s, self.i)
            self.i = m.end()
            return Node("lit", float(m.group(0)) if ("." in m.group(0) or "e" in m.group(0).lower())
                        else int(m.group(0)), pos=pos)
        if c == "(":
            self.i += 1
            inner = self.expr(True)
            self.expect(")", True, "to close '('")
            return Node("paren", None, [inner], pos)
        if c == "[":
            self.i += 1
            return self.tuple_or_for(pos)
        if c == "{":
            self.i += 1
            return self.object_or_for(pos)
        name = self.ident(False)
        if name is None:
            raise self.err(f"unexpected {self.s[self.i:self.i + 12].split(chr(10))[0]!r} in expression")
        if name in _KEYWORD_LITS:
            return Node("lit", _KEYWORD_LITS[name], pos=pos)
        if self.peek("("):  # function call (no space allowed before '(' in practice; tolerate it)
            self.i += 1
            args: List[Node] = []
            expand = False
            while True:
                self.skip(True)
                if self.peek(")"):
                    self.i += 1
                    break
                args.append(self.expr(True))
                self.skip(True)
                if self.peek("..."):
                    self.i += 3
                    expand = True
                    self.expect(")", True, "after '...' argument expansion")
                    break
                if self.eat(",", True):
                    continue
                self.expect(")", True, f"to close the call to {name}()")
                break
            return Node("call", name, args, pos)
        return Node("trav", name, [], pos)

    def tuple_or_for(self, pos: int) -> Node:
        self.skip(True)
        if self._for_keyword():
            names, coll = self.for_intro()
            value = self.expr(True)
            cond = self._for_if()
            self.expect("]", True, "to close the for expression")
            return Node("for", {"names": names, "object": False},
                        [coll, value] + ([cond] if cond else []), pos)
        items: List[Node] = []
        while True:
            self.skip(True)
            if self.peek("]"):
                self.i += 1
                return Node("tuple", None, items, pos)
            items.append(self.expr(True))
            self.skip(True)
            if self.eat(",", True):
                continue
            self.expect("]", True, "to close the tuple")
            return Node("tuple", None, items, pos)

    def object_or_for(self, pos: int) -> Node:
        self.skip(True)
        if self._for_keyword():
            names, coll = self.for_intro()
            key = self.expr(True)
            self.expect("=>", True, "in object for expression")
            value = self.expr(True)
            self.skip(True)
            group = self.eat("...", True)
            cond = self._for_if()
            self.expect("}", True, "to close the for expression")
            return Node("for", {"names": names, "object": True, "group": group},
                        [coll, key, value] + ([cond] if cond else []), pos)
        items: List[Node] = []
        while True:
            self.skip(True)
            if self.peek("}"):
                self.i += 1
                return Node("object", None, items, pos)
            kpos = self.i
            key = self.expr(False)
            self.skip(False)
            if self.peek("=") and not self.peek("==") and not self.peek("=>"):
                self.i += 1
            elif self.peek(":"):
                self.i += 1
            else:
                raise self.err("expected '=' or ':' after an object key")
            value = self.expr(False)
            items.append(Node("item", None, [key, value], kpos))
            self.skip(False)
            if self.peek(","):
                self.i += 1
            elif self.peek("\n"):
                self.i += 1
            elif not self.peek("}"):
                raise self.err("expected ',', a newline or '}' after an object item")

    def _for_keyword(self) -> bool:
        m = _IDENT_RE.match(self.s, self.i)
        return bool(m and m.group(0) == "for" and self.s[m.end():m.end() + 1] in (" ", "\t", "\n"))

    def for_intro(self) -> Tuple[List[str], Node]:
        self.i += 3
        names = [self.ident(True)]
        if names[0] is None:
            raise self.err("expected a variable name after 'for'")
        if self.eat(",", True):
            second = self.ident(True)
            if second is None:
                raise self.err("expected a second variable name after ','")
            names.append(second)
        if self.ident(True) != "in":
            raise self.err("expected 'in' in for expression")
        coll = self.expr(True)
        self.expect(":", True, "after the for collection")
        return names, coll

    def _for_if(self) -> Optional[Node]:
        self.skip(True)
        m = _IDENT_RE.match(self.s, self.i)
        if m and m.group(0) == "if":
            self.i = m.end()
            return self.expr(True)
        return None

    # --- templates ----------------------------------------------------------------------------------
    def string(self) -> Node:
        pos = self.i
        self.i += 1  # opening quote
        parts = self.template_parts(end='"', quoted=True)
        return self._template_node(parts, pos)

    def heredoc(self) -> Node:
        pos = self.i
        m = re.compile(r"<<(-?)([A-Za-z_][A-Za-z0-9_-]*)[ \t]*\n").match(self.s, self.i)
        if not m:
            raise self.err("malformed heredoc introducer")
        marker = m.group(2)
        end = re.compile(r"^[ \t]*" + re.escape(marker) + r"[ \t]*$", re.M).search(self.s, m.end())
        if not end:
            raise self.err(f"heredoc {marker!r} is never closed", pos)
        sub = _Parser(self.s[:end.start()], self.name)
        sub.i = m.end()
        parts = sub.template_parts(end=None, quoted=False)
        self.i = end.end()
        return self._template_node(parts, pos)

    @staticmethod
    def _template_node(parts: List[Node], pos: int) -> Node:
        if all(p.kind == "lit" for p in parts):
            return Node("lit", "".join(p.value for p in parts), pos=pos)
        return Node("tmpl", None, parts, pos)

    def template_parts(self, end: Optional[str], quoted: bool) -> List[Node]:
        """Literal text, ``${expr}`` and ``%{directive}`` up to ``end`` (None: end of input).
        Directives are checked for nesting here (if/else/endif, for/endfor)."""
        parts: List[Node] = []
        buf: List[str] = []
        stack: List[Tuple[str, int]] = []
        s = self.s
        while True:
            if self.i >= self.n:
                if end is not None:
                    raise self.err("unterminated string")
                break
            c = s[self.i]
            if end is not None and c == end:
                self.i += 1
                break
            if quoted and c == "\n":
                raise self.err("newline in a quoted string (use a heredoc)")
            if quoted and c == "\\":
                esc = s[self.i + 1:self.i + 2]
                if esc in ('"', "\\", "n", "r", "t"):
                    buf.append({"n": "\n", "r": "\r", "t": "\t"}.get(esc, esc))
                    self.i += 2
                    continue
                if esc in ("u", "U"):
                    width = 4 if esc == "u" else 8
                    digits = s[self.i + 2:self.i + 2 + width]
                    if len(digits) != width or any(ch not in "0123456789abcdefABCDEF" for ch in digits):
                        raise self.err(f"invalid escape \\{esc}{digits}: {width} hex digits expected")
                    try:
                        buf.append(chr(int(digits, 16)))
                    except (ValueError, OverflowError):  # past U+10FFFF
                        raise self.err(f"invalid escape \\{esc}{digits}: not a Unicode code point") from None
                    self.i += 2 + width
                    continue
                raise self.err(f"invalid escape \\{esc}")
            if s.startswith("$${", self.i) or s.startswith("%%{", self.i):
                buf.append(s[self.i + 1:self.i + 3])
                self.i += 3
                continue
            if s.startswith("${", self.i) or s.startswith("%{", self.i):
                if buf:
                    parts.append(Node("lit", "".join(buf)))
                    buf = []
                directive = s[self.i] == "%"
                start = self.i
                self.i += 2
                lstrip = self.peek("~")
                if lstrip:
                    self.i += 1
                if directive:
                    node = self._directive(stack, start)
                else:
                    e = self.expr(True)
                    self.skip(True)
                    self._rstrip = self.peek("~")
                    if self._rstrip:
                        self.i += 1
                    self.expect("}", True, "to close '${'")
                    node = Node("interp", None, [e], start)
                node.strip = (lstrip, self._rstrip)
                parts.append(node)
                continue
            buf.append(c)
            self.i += 1
        if stack:
            raise self.err(f"%{{{stack[-1][0]}}} is never closed", stack[-1][1])
        if buf:
            parts.append(Node("lit", "".join(buf)))
        return parts

    def _directive(self, stack: List[Tuple[str, int]], start: int) -> Node:
        word = self.ident(True)
        node: Node
        if word == "if":
            node = Node("if", None, [self.expr(True)], start)
            stack.append(("if", start))
        elif word == "else":
            if not stack or stack[-1][0] != "if":
                raise self.err("%{else} without %{if}", start)
            node = Node("else", pos=start)
        elif word == "endif":
            if not stack or stack[-1][0] != "if":
                raise self.err("%{endif} without %{if}", start)
            stack.pop()
            node = Node("endif", pos=start)
        elif word == "for":
            names = [self.ident(True)]
            if self.eat(",", True):
                names.append(self.ident(True))
            if None in names or self.ident(True) != "in":
                raise self.err("malformed %{for}", start)
            node = Node("tfor", names, [self.expr(True)], start)
            stack.append(("for", start))
        elif word == "endfor":
            if not stack or stack[-1][0] != "for":
                raise self.err("%{endfor} without %{for}", start)
            stack.pop()
            node = Node("endfor", pos=start)
        else:
            raise self.err(f"unknown template directive %{{{word}}}", start)
        self.skip(True)
        self._rstrip = self.peek("~")
        if self._rstrip:
            self.i += 1
        self.expect("}", True, "to close the directive")
        return node


def parse(src: str, name: str = "<hcl>") -> Body:
    """Parse a ``.tf`` file (HCL2 native syntax); raises :class:`HCLSyntaxError`."""
    p = _Parser(src, name)
    return p.body(None)


def parse_template(src: str, name: str = "<template>") -> List[Node]:
    """Parse a ``templatefile`` template; raises :class:`HCLSyntaxError`."""
    p = _Parser(src, name)
    return p.template_parts(end=None, quoted=False)


# --- analysis -----------------------------------------------------------------------------------------
def walk(node: Any):
    """Every Node under ``node`` (itself included), depth first."""
    if isinstance(node, Node):
        yield node
        for ch in node.children:
            yield from walk(ch)
    elif isinstance(node, Body):
        for a in node.attributes:
            yield from walk(a.expr)
        for b in node.blocks:
            yield from walk(b.body)
    elif isinstance(node, list):
        for x in node:
            yield from walk(x)


def references(node: Any, bound: Optional[Set[str]] = None) -> List[Tuple[str, List[str], int]]:
    """Traversals ``(root, [attr names...], pos)`` under ``node`` whose root is not bound
    by an enclosing ``for`` (expression or template directive)."""
    bound = set(bound or ())
    out: List[Tuple[str, List[str], int]] = []

    def visit(n: Any, b: Set[str]) -> None:
        if isinstance(n, Body):
            for a in n.attributes:
                visit(a.expr, b)
            for blk in n.blocks:
                if blk.type == "variable":  # `type = list(string)` is a type constraint, not references
                    for a in blk.body.attributes:
                        if a.name != "type":
                            visit(a.expr, b)
                    visit(Body(blocks=blk.body.blocks), b)
                elif blk.type == "provisioner":  # `when = destroy`, `on_failure = continue`: keywords
                    visit(Body(attributes=[a for a in blk.body.attributes if a.name not in ("when", "on_failure")],
                               blocks=blk.body.blocks), b)
                elif blk.type == "dynamic" and blk.labels:  # binds its label (or iterator) in content
                    it = blk.body.attr("iterator")
                    name = it.expr.value if it is not None and it.expr.kind == "trav" else blk.labels[0]
                    visit(blk.body, b | {name})
                else:
                    visit(blk.body, b)
            return
        if isinstance(n, list):
            inner = set(b)
            for x in n:  # template part lists: %{for} binds until %{endfor}
                if isinstance(x, Node) and x.kind == "tfor":
                    visit(x.children[0], inner)
                    inner = inner | set(x.value)
                else:
                    visit(x, inner)
            return
        if not isinstance(n, Node):
            return
        if n.kind == "trav" and n.value is not None:
            if n.value not in b:
                out.append((n.value, [c.value for c in n.children if c.kind == "attr"], n.pos))
            for c in n.children:
                if c.kind == "index":
                    visit(c.children[0], b)
            return
        if n.kind == "for":
            visit(n.children[0], b)
            inner = b | set(n.value["names"])
            for c in n.children[1:]:
                visit(c, inner)
            return
        if n.kind == "tmpl":
            visit(n.children, b)
            return
        if n.kind == "item":  # object item: a bare-identifier key is a name, not a reference
            key = n.children[0]
            if not (key.kind == "trav" and key.value is not None and not key.children):
                visit(key, b)
            visit(n.children[1], b)
            return
        for c in n.children:
            visit(c, b)

    visit(node, bound)
    return out


def template_names(parts: List[Node]) -> Set[str]:
    """Root names a template reads (its ``templatefile`` vars)."""
    return {root for root, _, _ in references(parts)}


def object_keys(node: Node) -> Optional[Set[str]]:
    """Literal keys of an object constructor (None if it is not one)."""
    if node.kind != "object":
        return None
    keys = set()
    for item in node.children:
        k = item.children[0]
        if k.kind == "trav" and not k.children:
            keys.add(k.value)
        elif k.kind == "lit" and isinstance(k.value, str):
            keys.add(k.value)
        else:
            return None
    return keys


_BUILTIN_ROOTS = {"path", "count", "each", "self", "terraform"}

# Terraform >= 1.3's built-in functions.  ``list()``/``map()`` are not here: they were
# removed in 0.15, so a module still calling them would not plan (type constraints such
# as ``map(string)`` are not calls and are skipped by :func:`_value_calls`).
TERRAFORM_FUNCTIONS = frozenset("""
abs ceil floor log max min parseint pow signum
chomp endswith format formatlist indent join lower regex regexall replace split startswith
strcontains strrev substr title trim trimprefix trimsuffix trimspace upper
alltrue anytrue chunklist coalesce coalescelist compact concat contains distinct element flatten
index keys length lookup matchkeys merge one range reverse setintersection setproduct setsubtract
setunion slice sort sum transpose values zipmap
base64decode base64encode base64gzip csvdecode jsondecode jsonencode textdecodebase64
textencodebase64 urlencode yamldecode yamlencode
abspath dirname pathexpand basename file fileexists fileset filebase64 templatefile
formatdate plantimestamp timeadd timecmp timestamp
base64sha256 base64sha512 bcrypt filebase64sha256 filebase64sha512 filemd5 filesha1 filesha256
filesha512 md5 rsadecrypt sha1 sha256 sha512 uuid uuidv5
cidrhost cidrnetmask cidrsubnet cidrsubnets
can issensitive nonsensitive sensitive tobool tolist tomap tonumber toset tostring try type
""".split())
# resource/data types served by Terraform itself, not by a required provider
_BUILTIN_RESOURCE_TYPES = {"terraform_data", "terraform_remote_state"}


def _value_calls(body: Body, block_type: str = ""):
    """Function-call nodes in value positions (a variable's ``type`` is a constraint)."""
    for a in body.attributes:
        if block_type == "variable" and a.name == "type":
            continue
        for n in walk(a.expr):
            if n.kind == "call":
                yield n
    for b in body.blocks:
        yield from _value_calls(b.body, b.type)


def _provider_of(rtype: str) -> str:
    return rtype.split("_", 1)[0]


@dataclass
class ModuleReport:
    name: str
    files: Dict[str, Body]
    errors: List[str]
    variables: Set[str]
    required: Set[str]
    outputs: Set[str]


def check_module(module_dir: str) -> ModuleReport:
    """Parse every ``.tf`` of a module and cross-check references and templatefile calls."""
    name = os.path.basename(module_dir.rstrip("/"))
    files: Dict[str, Body] = {}
    errors: List[str] = []
    for fn in sorted(os.listdir(module_dir)):
        if fn.endswith(".tf"):
            path = os.path.join(module_dir, fn)
            with open(path, encoding="utf-8") as fh:
                src = fh.read()
            try:
                files[fn] = parse(src, f"{name}/{fn}")
            except HCLSyntaxError as exc:
                errors.append(str(exc))
    variables: Set[str] = set()
    required: Set[str] = set()
    locals_: Set[str] = set()
    resources: Set[Tuple[str, str]] = set()
    datas: Set[Tuple[str, str]] = set()
    modules: Set[str] = set()
    outputs: Set[str] = set()
    for fn, body in files.items():
        for b in body.blocks:
            if b.type == "variable" and b.labels:
                variables.add(b.labels[0])
                if b.body.attr("default") is None:
                    required.add(b.labels[0])
            elif b.type == "locals":
                locals_ |= {a.name for a in b.body.attributes}
            elif b.type == "resource" and len(b.labels) == 2:
                resources.add((b.labels[0], b.labels[1]))
            elif b.type == "data" and len(b.labels) == 2:
                datas.add((b.labels[0], b.labels[1]))
            elif b.type == "module" and b.labels:
                modules.add(b.labels[0])
            elif b.type == "output" and b.labels:
                outputs.add(b.labels[0])
    resource_types = {t for t, _ in resources}
    providers: Set[str] = set()
    for body in files.values():
        for tb in body.blocks_of("terraform"):
            for rp in tb.body.blocks_of("required_providers"):
                providers |= {a.name for a in rp.body.attributes}
    for rtype in sorted(resource_types | {t for t, _ in datas}):
        if rtype not in _BUILTIN_RESOURCE_TYPES and _provider_of(rtype) not in providers:
            errors.append(f"{name}: {rtype} needs provider {_provider_of(rtype)!r}, "
                          f"which required_providers does not declare")
    for fn, body in files.items():
        for call in _value_calls(body):
            if call.value not in TERRAFORM_FUNCTIONS:
                errors.append(f"{name}/{fn}: call to unknown function {call.value}()")
        for root, attrs, pos in references(body):
            where = f"{name}/{fn}"
            if root == "var":
                if attrs and attrs[0] not in variables:
                    errors.append(f"{where}: reference to undeclared variable var.{attrs[0]}")
            elif root == "local":
                if attrs and attrs[0] not in locals_:
                    errors.append(f"{where}: reference to undefined local.{attrs[0]}")
            elif root == "data":
                if len(attrs) >= 2 and (attrs[0], attrs[1]) not in datas:
                    errors.append(f"{where}: reference to undefined data.{attrs[0]}.{attrs[1]}")
            elif root == "module":
                if attrs and attrs[0] not in modules:
                    errors.append(f"{where}: reference to undefined module.{attrs[0]}")
            elif root in resource_types:
                if attrs and (root, attrs[0]) not in resources:
                    errors.append(f"{where}: reference to undefined resource {root}.{attrs[0]}")
            elif root not in _BUILTIN_ROOTS:
                errors.append(f"{where}: unknown reference {'.'.join([root] + attrs[:1])}")
        for node in walk(body):
            if node.kind == "call" and node.value == "templatefile":
                errors += _check_templatefile(module_dir, f"{name}/{fn}", node)
    return ModuleReport(name, files, errors, variables, required, outputs)


def _check_templatefile(module_dir: str, where: str, call: Node) -> List[str]:
    if len(call.children) != 2:
        return [f"{where}: templatefile() takes 2 arguments"]
    path_node, vars_node = call.children
    rel = _module_relative_path(path_node)
    if rel is None:
        return []  # computed path (e.g. for-expression over fileset): checked by the caller's test
    tpl_path = os.path.join(module_dir, rel)
    if not os.path.isfile(tpl_path):
        return [f"{where}: templatefile() of missing file {rel}"]
    with open(tpl_path, encoding="utf-8") as fh:
        try:
            names = template_names(parse_template(fh.read(), rel))
        except HCLSyntaxError as exc:
            return [str(exc)]
    keys = object_keys(vars_node)
    if keys is None:
        return [f"{where}: templatefile({rel}) vars must be an object constructor"]
    errs = []
    if names - keys:
        errs.append(f"{where}: templatefile({rel}) does not pass {sorted(names - keys)}")
    if keys - names:
        errs.append(f"{where}: templatefile({rel}) passes unused {sorted(keys - names)}")
    return errs


def _module_relative_path(node: Node) -> Optional[str]:
    """``"${path.module}/files/x.tftpl"`` -> ``files/x.tftpl``."""
    if node.kind != "tmpl" or len(node.children) != 2:
        return None
    head, tail = node.children
    if head.kind != "interp" or tail.kind != "lit":
        return None
    ref = head.children[0]
    if ref.kind == "trav" and ref.value == "path" and [c.value for c in ref.children] == ["module"]:
        return tail.value.lstrip("/")
    return None


# --- template evaluation (templatefile) ---------------------------------------------------------------
class TemplateError(ValueError):
    pass


def _apply_strip(parts: List[Node]) -> List[Node]:
    """Terraform's ``~`` markers: remove the whitespace (newlines included) of the literal
    next to the marked side."""
    out = [Node(p.kind, p.value, p.children, p.pos, p.strip) for p in parts]
    for i, p in enumerate(out):
        if p.kind == "lit":
            continue
        left, right = p.strip
        if left and i > 0 and out[i - 1].kind == "lit":
            out[i - 1].value = out[i - 1].value.rstrip(" \t\r\n")
        if right and i + 1 < len(out) and out[i + 1].kind == "lit":
            out[i + 1].value = out[i + 1].value.lstrip(" \t\r\n")
    return out


_FUNCS = {
    "length": lambda v: len(v),
    "upper": lambda v: str(v).upper(),
    "lower": lambda v: str(v).lower(),
    "trimspace": lambda v: str(v).strip(),
    "join": lambda sep, items: str(sep).join(str(x) for x in items),
    "replace": lambda v, a, b: str(v).replace(str(a), str(b)),
    "tostring": lambda v: _to_str(v),
    "jsonencode": lambda v: __import__("json").dumps(v, separators=(",", ":")),
    "base64encode": lambda v: __import__("base64").b64encode(str(v).encode()).decode(),
    "keys": lambda m: sorted(m),
    "values": lambda m: [m[k] for k in sorted(m)],
    "element": lambda lst, i: lst[int(i) % len(lst)],
    "contains": lambda lst, v: v in lst,
    "split": lambda sep, v: str(v).split(str(sep)),
    "slice": lambda lst, a, b: list(lst)[int(a):int(b)],
    "regexall": lambda pat, v: __import__("re").findall(re2_pattern(str(pat)), str(v)),
    "alltrue": lambda items: all(x is True or x == "true" for x in items),
    "anytrue": lambda items: any(x is True or x == "true" for x in items),
}


def re2_pattern(pat: str) -> str:
    """An RE2 pattern (Terraform's ``regex``/``regexall``) for Python's ``re``: RE2's ``$``
    matches only at the end of the text, Python's also before a final newline, so a bare
    ``$`` becomes ``\\Z``.  Escaped pairs (``\\$``, ``\\\\``) and character classes
    (``[$]``, ``[^]$]``) are copied as they are: there ``$`` is a literal."""
    out: List[str] = []
    i, n = 0, len(pat)
    while i < n:
        c = pat[i]
        if c == "\\" and i + 1 < n:
            out.append(pat[i:i + 2])
            i += 2
            continue
        if c == "[":
            j = i + 1
            if j < n and pat[j] == "^":
                j += 1
            if j < n and pat[j] == "]":  # a leading ']' is a member, not the end
                j += 1
            while j < n and pat[j] != "]":
                j += 2 if pat[j] == "\\" else 1
            out.append(pat[i:j + 1])
            i = j + 1
            continue
        out.append("\\Z" if c == "$" else c)
        i += 1
    return "".join(out)


def _to_str(v: Any) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, (dict, list)):
        raise TemplateError(f"cannot interpolate a {type(v).__name__} into a string")
    return str(v)


def _num(v: Any) -> float:
    if isinstance(v, bool):
        raise TemplateError("a bool is not a number")
    try:
        return float(v)
    except (TypeError, ValueError) as exc:
        raise TemplateError(f"{v!r} is not a number") from exc


def eval_expr(node: Node, env: Dict[str, Any]) -> Any:
    """Evaluate the HCL expression subset templates use: literals, variables (with attribute
    and index traversal), operators, conditionals, tuples/objects, string templates and a few
    functions.  Unknown variables or functions raise :class:`TemplateError`, as Terraform does."""
    k = node.kind
    if k == "lit":
        return node.value
    if k == "paren":
        return eval_expr(node.children[0], env)
    if k == "trav":
        if node.value is None:
            base = eval_expr(node.children[0], env)
            steps = node.children[1:]
        else:
            if node.value not in env:
                raise TemplateError(f"undefined variable {node.value!r}")
            base = env[node.value]
            steps = node.children
        for st in steps:
            if st.kind == "attr":
                base = base[st.value]
            elif st.kind == "index":
                key = eval_expr(st.children[0], env)
                base = base[int(key)] if isinstance(base, list) else base[key]
            else:
                raise TemplateError(f"unsupported traversal {st.kind}")
        return base
    if k == "tmpl":
        return render_parts(node.children, env)
    if k == "unary":
        v = eval_expr(node.children[0], env)
        return (not v) if node.value == "!" else -_num(v)
    if k == "op":
        op = node.value
        if op == "&&":
            return bool(eval_expr(node.children[0], env)) and bool(eval_expr(node.children[1], env))
        if op == "||":
            return bool(eval_expr(node.children[0], env)) or bool(eval_expr(node.children[1], env))
        a, b = eval_expr(node.children[0], env), eval_expr(node.children[1], env)
        if op == "==":
            return a == b
        if op == "!=":
            return a != b
        ops = {"<": lambda x, y: x < y, ">": lambda x, y: x > y, "<=": lambda x, y: x <= y, ">=": lambda x, y: x >= y,
               "+": lambda x, y: x + y, "-": lambda x, y: x - y, "*": lambda x, y: x * y, "/": lambda x, y: x / y,
               "%": lambda x, y: x % y}
        if op not in ops:
            raise TemplateError(f"unsupported operator {op}")
        r = ops[op](_num(a), _num(b))
        return r
    if k == "cond":
        return eval_expr(node.children[1] if eval_expr(node.children[0], env) else node.children[2], env)
    if k == "tuple":
        return [eval_expr(c, env) for c in node.children]
    if k == "object":
        out = {}
        for item in node.children:
            key = item.children[0]
            kv = key.value if key.kind == "trav" and not key.children else eval_expr(key, env)
            out[kv] = eval_expr(item.children[1], env)
        return out
    if k == "call":
        fn = _FUNCS.get(node.value)
        if fn is None:
            raise TemplateError(f"function {node.value}() is not supported by this evaluator")
        return fn(*[eval_expr(c, env) for c in node.children])
    if k == "for":
        # [for k, v in coll : value if cond] / {for k, v in coll : key => value if cond}; a
        # map is walked in key order, as Terraform does
        names = node.value["names"]
        if node.value.get("group"):
            raise TemplateError("grouping for-expressions (key => value...) are not supported by this evaluator")
        coll = eval_expr(node.children[0], env)
        pairs = sorted(coll.items()) if isinstance(coll, dict) else list(enumerate(coll))
        obj = node.value["object"]
        body = node.children[1:3] if obj else node.children[1:2]
        cond = node.children[len(body) + 1] if len(node.children) > len(body) + 1 else None
        out_list, out_obj = [], {}
        for key, val in pairs:
            scope = dict(env, **({names[0]: key, names[1]: val} if len(names) == 2 else {names[0]: val}))
            if cond is not None and not eval_expr(cond, scope):
                continue
            if obj:
                out_obj[_to_str(eval_expr(body[0], scope))] = eval_expr(body[1], scope)
            else:
                out_list.append(eval_expr(body[0], scope))
        return out_obj if obj else out_list
    raise TemplateError(f"unsupported expression {k}")


def render_parts(parts: List[Node], env: Dict[str, Any]) -> str:
    parts = _apply_strip(parts)
    out: List[str] = []

    def run(i: int, end_kinds: Tuple[str, ...], emit: bool) -> int:
        while i < len(parts):
            p = parts[i]
            if p.kind in end_kinds:
                return i
            if p.kind == "lit":
                if emit:
                    out.append(p.value)
                i += 1
            elif p.kind == "interp":
                if emit:
                    out.append(_to_str(eval_expr(p.children[0], env)))
                i += 1
            elif p.kind == "if":
                cond = bool(eval_expr(p.children[0], env)) if emit else False
                j = run(i + 1, ("else", "endif"), emit and cond)
                if parts[j].kind == "else":
                    j = run(j + 1, ("endif",), emit and not cond)
                i = j + 1
            elif p.kind == "tfor":
                coll = eval_expr(p.children[0], env) if emit else []
                names = p.value
                body_end = _matching_endfor(parts, i)
                items = list(coll.items()) if isinstance(coll, dict) else list(enumerate(coll))
                if isinstance(coll, dict):
                    items = sorted(items)
                for key, val in items if emit else []:
                    saved = dict(env)
                    if len(names) == 2:
                        env[names[0]], env[names[1]] = key, val
                    else:
                        env[names[0]] = val
                    run(i + 1, ("endfor",), True)
                    env.clear()
                    env.update(saved)
                i = body_end + 1
            else:
                raise TemplateError(f"unexpected {p.kind}")
        return i

    run(0, (), True)
    return "".join(out)


def _matching_endfor(parts: List[Node], i: int) -> int:
    depth = 0
    for j in range(i, len(parts)):
        if parts[j].kind == "tfor":
            depth += 1
        elif parts[j].kind == "endfor":
            depth -= 1
            if depth == 0:
                return j
    raise TemplateError("%{for} without %{endfor}")


def templatefile(src: str, variables: Dict[str, Any], name: str = "<template>") -> str:
    """Terraform's ``templatefile(path, vars)`` over template source ``src``."""
    return render_parts(parse_template(src, name), dict(variables))


def _var_type_ok(vtype: str, value: Any) -> bool:
    """Terraform's conversion rules for the primitive / collection types the modules use."""
    if isinstance(value, str) and "${" in value:
        return True  # an interpolation: known only at apply time
    if vtype == "string":
        return isinstance(value, (str, int, float, bool))
    if vtype == "number":
        try:
            float(value)
            return not isinstance(value, bool)
        except (TypeError, ValueError):
            return False
    if vtype == "bool":
        return isinstance(value, bool) or str(value).lower() in ("true", "false")
    if vtype.startswith("list("):
        return isinstance(value, list)
    if vtype.startswith("map("):
        return isinstance(value, dict)
    return True


_REPORTS: Dict[str, Tuple[Tuple[Tuple[str, int], ...], "ModuleReport"]] = {}
_REPORTS_MU = threading.Lock()
_REPORT_LOCKS: Dict[str, threading.Lock] = {}


def module_report(module_dir: str) -> "ModuleReport":
    """:func:`check_module`, cached while the module's ``.tf`` files are unchanged (the
    DirectExecutor checks every module call it applies; a parse per call would be waste)."""
    stamp = tuple(sorted((fn, os.stat(os.path.join(module_dir, fn)).st_mtime_ns)
                         for fn in os.listdir(module_dir) if fn.endswith(".tf")))
    with _REPORTS_MU:
        hit = _REPORTS.get(module_dir)
        mu = _REPORT_LOCKS.setdefault(module_dir, threading.Lock())
    if hit is not None and hit[0] == stamp:
        return hit[1]
    # one parse per module: the host modules of a cluster start together, and each parse
    # is ~40 ms of interpreter time (128 concurrent misses serialised ~5 s on the GIL)
    with mu:
        with _REPORTS_MU:
            hit = _REPORTS.get(module_dir)
        if hit is not None and hit[0] == stamp:
            return hit[1]
        rep = check_module(module_dir)
        with _REPORTS_MU:
            _REPORTS[module_dir] = (stamp, rep)
    return rep


def check_inputs(module_dir: str, inputs: Dict[str, Any], cached: bool = False) -> List[str]:
    """What ``terraform plan`` would reject about one module call: unknown inputs, missing
    required variables, values of the wrong type, and failing ``validation`` conditions
    (evaluated with this module's evaluator).  Inputs that are interpolations
    (``${module...}``) are only known at apply time and skip the value checks.  ``cached``:
    reuse the module's parse while its files are unchanged (:func:`module_report`)."""
    rep = module_report(module_dir) if cached else check_module(module_dir)
    errors = list(rep.errors)
    given = {k: v for k, v in inputs.items() if k != "source"}
    errors += [f"unsupported argument {k!r}" for k in sorted(set(given) - rep.variables)]
    errors += [f"missing required argument {k!r}" for k in sorted(rep.required - set(given))]
    decls: Dict[str, Block] = {}
    for body in rep.files.values():
        for b in body.blocks:
            if b.type == "variable" and b.labels:
                decls[b.labels[0]] = b
    values: Dict[str, Any] = {}
    for name, blk in decls.items():
        if name in given:
            values[name] = given[name]
        elif blk.body.attr("default") is not None:
            try:
                values[name] = eval_expr(blk.body.attr("default").expr, {})
            except TemplateError:
                values[name] = None
    for name, blk in sorted(decls.items()):
        if name not in given:
            continue
        v = given[name]
        tattr = blk.body.attr("type")
        if tattr is not None:
            tname = tattr.expr.value if tattr.expr.kind == "trav" and not tattr.expr.children else \
                (f"{tattr.expr.value}(string)" if tattr.expr.kind == "call" else "")
            if tname and not _var_type_ok(tname, v):
                errors.append(f"{name}: {v!r} is not a {tname}")
        if isinstance(v, str) and "${" in v:
            continue
        for vb in blk.body.blocks:
            if vb.type != "validation":
                continue
            cond = vb.body.attr("condition")
            msg = vb.body.attr("error_message")
            try:
                ok = bool(eval_expr(cond.expr, {"var": values}))
            except (TemplateError, KeyError, IndexError, TypeError) as exc:
                errors.append(f"{name}: validation not evaluable: {exc}")
                continue
            if not ok:
                errors.append(f"{name}: {eval_expr(msg.expr, {}) if msg is not None else 'invalid value'}")
    return errors
