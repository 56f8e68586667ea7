"""HCL2 native-syntax parser -> small AST.

Covers what Terraform configurations use: blocks with labels, attributes,
literals, templates + heredocs (interpolations and %{if}/%{for} directives),
tuples, objects, function calls (incl. ``...`` expansion), index/attribute
traversal, attribute and full splats, for-expressions, conditionals, unary
and binary operators with HCL precedence.

The AST is deliberately tiny; :func:`walk_refs` yields every variable
traversal (root name + static attribute/index path) with the names bound by
enclosing for-expressions, which is all the static checker needs.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path

from .lexer import HCLSyntaxError, TemplatePart, Token, tokenize


# ----------------------------------------------------------------------- AST
class Expr:
    line: int = 0


@dataclass
class Literal(Expr):
    value: object
    line: int = 0


@dataclass
class Template(Expr):
    parts: list  # str | Expr | Directive
    line: int = 0

    def literal(self) -> str | None:
        """The string value if the template has no interpolation."""
        if all(isinstance(p, str) for p in self.parts):
            return "".join(self.parts)
        return None


@dataclass
class Directive(Expr):
    kind: str            # if / else / endif / for / endfor
    expr: Expr | None
    names: tuple = ()
    line: int = 0


@dataclass
class Traversal(Expr):
    root: str
    ops: list            # ("attr", name) | ("index", Expr) | ("splat", None)
    line: int = 0

    def path(self) -> list[str]:
        """Static attribute/index path after the root (stops at dynamic parts)."""
        out = []
        for kind, v in self.ops:
            if kind == "attr":
                out.append(v)
            elif kind == "index" and isinstance(v, Literal):
                out.append(str(v.value))
            elif kind == "index" and isinstance(v, Template) and v.literal() is not None:
                out.append(v.literal())
            else:
                break
        return out


@dataclass
class Postfix(Expr):
    """Attribute / index / splat applied to a non-variable expression."""

    base: Expr
    ops: list
    line: int = 0


@dataclass
class Call(Expr):
    name: str
    args: list
    expand: bool = False
    line: int = 0


@dataclass
class TupleExpr(Expr):
    items: list
    line: int = 0


@dataclass
class ObjectExpr(Expr):
    items: list          # list[(key Expr, value Expr)]
    line: int = 0

    def get(self, key: str):
        for k, v in self.items:
            if key_name(k) == key:
                return v
        return None


@dataclass
class ForExpr(Expr):
    key_var: str | None
    val_var: str
    coll: Expr
    key_expr: Expr | None   # object form only
    val_expr: Expr
    cond: Expr | None
    grouping: bool
    is_object: bool
    line: int = 0


@dataclass
class Conditional(Expr):
    cond: Expr
    true: Expr
    false: Expr
    line: int = 0


@dataclass
class BinOp(Expr):
    op: str
    left: Expr
    right: Expr
    line: int = 0


@dataclass
class UnOp(Expr):
    op: str
    operand: Expr
    line: int = 0


@dataclass
class Attribute:
    name: str
    expr: Expr
    line: int


@dataclass
class Block:
    type: str
    labels: list
    body: "Body"
    line: int


@dataclass
class Body:
    attributes: dict = field(default_factory=dict)   # name -> Attribute
    blocks: list = field(default_factory=list)        # Block

    def blocks_of(self, typ: str) -> list[Block]:
        return [b for b in self.blocks if b.type == typ]

    def attr(self, name: str) -> Expr | None:
        a = self.attributes.get(name)
        return a.expr if a else None


def key_name(k: Expr) -> str | None:
    """Object-constructor key as a string when it is static."""
    if isinstance(k, Traversal) and not k.ops:
        return k.root
    if isinstance(k, Template):
        return k.literal()
    if isinstance(k, Literal):
        return str(k.value)
    return None


# -------------------------------------------------------------------- parser
_BINARY_PREC = [
    ("||",),
    ("&&",),
    ("==", "!="),
    ("<", ">", "<=", ">="),
    ("+", "-"),
    ("*", "/", "%"),
]


class Parser:
    def __init__(self, toks: list[Token], filename: str = ""):
        self.t = toks
        self.p = 0
        self.filename = filename
        self.nl_stack: list[bool] = [False]   # True: newlines are insignificant

    # -- token helpers
    def err(self, msg: str, tok: Token | None = None) -> HCLSyntaxError:
        tok = tok or self.peek()
        return HCLSyntaxError(msg, tok.line, tok.col, self.filename)

    def peek(self, k: int = 0) -> Token:
        j = self.p
        skip_nl = self.nl_stack[-1]
        seen = 0
        while True:
            tok = self.t[j]
            if skip_nl and tok.kind == "NEWLINE":
                j += 1
                continue
            if seen == k:
                return tok
            seen += 1
            j += 1

    def next(self) -> Token:
        skip_nl = self.nl_stack[-1]
        while skip_nl and self.t[self.p].kind == "NEWLINE":
            self.p += 1
        tok = self.t[self.p]
        self.p += 1
        return tok

    def at(self, kind: str, value=None) -> bool:
        tok = self.peek()
        return tok.kind == kind and (value is None or tok.value == value)

    def at_punct(self, *vals: str) -> bool:
        tok = self.peek()
        return tok.kind == "PUNCT" and tok.value in vals

    def expect_punct(self, val: str) -> Token:
        tok = self.next()
        if tok.kind != "PUNCT" or tok.value != val:
            raise self.err(f"expected {val!r}, got {tok.value!r}", tok)
        return tok

    def skip_newlines(self) -> None:
        while self.t[self.p].kind == "NEWLINE":
            self.p += 1

    # -- structure
    def parse_file(self) -> Body:
        body = self.parse_body(top=True)
        if not self.at("EOF"):
            raise self.err("unexpected token at top level")
        return body

    def parse_body(self, top: bool = False) -> Body:
        body = Body()
        self.nl_stack.append(False)
        try:
            while True:
                self.skip_newlines()
                tok = self.peek()
                if tok.kind == "EOF" or (not top and tok.kind == "PUNCT" and tok.value == "}"):
                    break
                if tok.kind != "IDENT":
                    raise self.err(f"expected attribute or block, got {tok.value!r}")
                name_tok = self.next()
                nxt = self.peek()
                if nxt.kind == "PUNCT" and nxt.value == "=":
                    self.next()
                    expr = self.parse_expr()
                    if name_tok.value in body.attributes:
                        raise self.err(f"duplicate attribute {name_tok.value!r}", name_tok)
                    body.attributes[name_tok.value] = Attribute(name_tok.value, expr, name_tok.line)
                    self.end_of_item()
                else:
                    labels = []
                    while True:
                        lt = self.peek()
                        if lt.kind == "TEMPLATE":
                            self.next()
                            lit = "".join(p.text for p in lt.value if not p.is_expr and not p.is_directive)
                            labels.append(lit)
                        elif lt.kind == "IDENT":
                            self.next()
                            labels.append(lt.value)
                        else:
                            break
                    self.expect_punct("{")
                    self.nl_stack.append(False)
                    # single-line block: `name { attr = 1 }` is allowed when the body is empty or one item
                    inner = self.parse_body()
                    self.nl_stack.pop()
                    self.expect_punct("}")
                    body.blocks.append(Block(name_tok.value, labels, inner, name_tok.line))
                    self.end_of_item()
        finally:
            self.nl_stack.pop()
        return body

    def end_of_item(self) -> None:
        tok = self.t[self.p]
        if tok.kind in ("NEWLINE", "EOF"):
            return
        if tok.kind == "PUNCT" and tok.value == "}":
            return
        raise self.err(f"expected newline after item, got {tok.value!r}", tok)

    # -- expressions
    def parse_expr(self) -> Expr:
        cond = self.parse_binary(0)
        if self.at_punct("?"):
            self.next()
            self.nl_stack.append(True)
            t = self.parse_expr()
            self.expect_punct(":")
            f = self.parse_expr()
            self.nl_stack.pop()
            return Conditional(cond, t, f, line=getattr(cond, "line", 0))
        return cond

    def parse_binary(self, level: int) -> Expr:
        if level == len(_BINARY_PREC):
            return self.parse_unary()
        left = self.parse_binary(level + 1)
        while self.at_punct(*_BINARY_PREC[level]):
            op = self.next().value
            right = self.parse_binary(level + 1)
            left = BinOp(op, left, right, line=getattr(left, "line", 0))
        return left

    def parse_unary(self) -> Expr:
        if self.at_punct("!", "-"):
            tok = self.next()
            return UnOp(tok.value, self.parse_unary(), line=tok.line)
        return self.parse_postfix(self.parse_primary())

    def parse_postfix(self, base: Expr) -> Expr:
        ops: list = []
        while True:
            if self.at_punct(".") and not self._dot_is_number():
                self.next()
                tok = self.next()
                if tok.kind == "PUNCT" and tok.value == "*":
                    ops.append(("splat", None))
                elif tok.kind == "IDENT":
                    ops.append(("attr", tok.value))
                elif tok.kind == "NUMBER":
                    ops.append(("index", Literal(tok.value, tok.line)))
                else:
                    raise self.err("bad attribute access", tok)
            elif self.at_punct("[") and self.t[self.p].kind != "NEWLINE":
                self.next()
                self.nl_stack.append(True)
                if self.at_punct("*"):
                    self.next()
                    ops.append(("splat", None))
                else:
                    ops.append(("index", self.parse_expr()))
                self.expect_punct("]")
                self.nl_stack.pop()
            else:
                break
        if not ops:
            return base
        if isinstance(base, Traversal):
            base.ops.extend(ops)
            return base
        return Postfix(base, ops, line=getattr(base, "line", 0))

    def _dot_is_number(self) -> bool:
        return False

    def parse_primary(self) -> Expr:
        tok = self.peek()
        if tok.kind == "NUMBER":
            self.next()
            return Literal(tok.value, tok.line)
        if tok.kind == "TEMPLATE":
            self.next()
            return self.build_template(tok.value, tok.line)
        if tok.kind == "IDENT":
            self.next()
            if tok.value in ("true", "false"):
                return Literal(tok.value == "true", tok.line)
            if tok.value == "null":
                return Literal(None, tok.line)
            if self.at_punct("(") and self.t[self.p].kind == "PUNCT":
                return self.parse_call(tok)
            if self.at_punct(":") and self.peek(1).kind == "PUNCT" and self.peek(1).value == ":":
                # provider-namespaced function  provider::ns::fn(...)
                raise self.err("provider functions are not supported", tok)
            return Traversal(tok.value, [], line=tok.line)
        if tok.kind == "PUNCT":
            if tok.value == "(":
                self.next()
                self.nl_stack.append(True)
                e = self.parse_expr()
                self.expect_punct(")")
                self.nl_stack.pop()
                return e
            if tok.value == "[":
                return self.parse_tuple()
            if tok.value == "{":
                return self.parse_object()
        raise self.err(f"unexpected token {tok.value!r} in expression", tok)

    def parse_call(self, name_tok: Token) -> Expr:
        self.expect_punct("(")
        self.nl_stack.append(True)
        args, expand = [], False
        while not self.at_punct(")"):
            args.append(self.parse_expr())
            if self.at_punct("..."):
                self.next()
                expand = True
            if self.at_punct(","):
                self.next()
            elif not self.at_punct(")"):
                raise self.err("expected ',' or ')' in call")
        self.expect_punct(")")
        self.nl_stack.pop()
        return Call(name_tok.value, args, expand, line=name_tok.line)

    def parse_tuple(self) -> Expr:
        start = self.expect_punct("[")
        self.nl_stack.append(True)
        if self.at("IDENT", "for"):
            e = self.parse_for(start, is_object=False)
            self.expect_punct("]")
            self.nl_stack.pop()
            return e
        items = []
        while not self.at_punct("]"):
            items.append(self.parse_expr())
            if self.at_punct(","):
                self.next()
            elif not self.at_punct("]"):
                raise self.err("expected ',' or ']' in tuple")
        self.expect_punct("]")
        self.nl_stack.pop()
        return TupleExpr(items, line=start.line)

    def parse_object(self) -> Expr:
        start = self.expect_punct("{")
        self.nl_stack.append(True)
        if self.at("IDENT", "for"):
            e = self.parse_for(start, is_object=True)
            self.expect_punct("}")
            self.nl_stack.pop()
            return e
        items = []
        while not self.at_punct("}"):
            k = self.parse_expr()
            if not self.at_punct("=", ":"):
                raise self.err("expected '=' or ':' in object")
            self.next()
            v = self.parse_expr()
            items.append((k, v))
            if self.at_punct(","):
                self.next()
        self.expect_punct("}")
        self.nl_stack.pop()
        return ObjectExpr(items, line=start.line)

    def parse_for(self, start: Token, is_object: bool) -> Expr:
        self.next()  # 'for'
        a = self.next()
        if a.kind != "IDENT":
            raise self.err("expected identifier after for", a)
        key_var, val_var = None, a.value
        if self.at_punct(","):
            self.next()
            b = self.next()
            key_var, val_var = a.value, b.value
        if not self.at("IDENT", "in"):
            raise self.err("expected 'in'")
        self.next()
        coll = self.parse_expr()
        self.expect_punct(":")
        key_expr = None
        if is_object:
            key_expr = self.parse_expr()
            self.expect_punct("=>")
        val_expr = self.parse_expr()
        grouping = False
        if self.at_punct("..."):
            self.next()
            grouping = True
        cond = None
        if self.at("IDENT", "if"):
            self.next()
            cond = self.parse_expr()
        return ForExpr(key_var, val_var, coll, key_expr, val_expr, cond, grouping, is_object,
                       line=start.line)

    # -- templates
    def build_template(self, parts: list[TemplatePart], line: int) -> Template:
        out: list = []
        for part in parts:
            if not part.is_expr and not part.is_directive:
                out.append(part.text)
                continue
            if part.is_expr:
                out.append(parse_expression(part.text, self.filename, part.line or line))
                continue
            words = part.text.split(None, 1)
            kind = words[0] if words else ""
            rest = words[1] if len(words) > 1 else ""
            if kind == "if":
                out.append(Directive("if", parse_expression(rest, self.filename, line), line=line))
            elif kind in ("else", "endif", "endfor"):
                out.append(Directive(kind, None, line=line))
            elif kind == "for":
                head, _, coll = rest.partition(" in ")
                names = tuple(n.strip() for n in head.split(","))
                out.append(Directive("for", parse_expression(coll, self.filename, line), names, line=line))
            else:
                raise HCLSyntaxError(f"unknown template directive {kind!r}", line, 0, self.filename)
        return Template(out, line=line)


def parse_expression(src: str, filename: str = "", line: int = 0) -> Expr:
    toks = tokenize(src, filename)
    for t in toks:
        t.line += max(0, line - 1)
    p = Parser(toks, filename)
    p.nl_stack = [True]
    e = p.parse_expr()
    if not p.at("EOF"):
        raise p.err("trailing tokens in expression")
    return e


def parse(src: str, filename: str = "") -> Body:
    return Parser(tokenize(src, filename), filename).parse_file()


def parse_file(path: str | Path) -> Body:
    path = Path(path)
    return parse(path.read_text(), str(path))


# -------------------------------------------------------------- traversal walk
def children(e) -> list:
    if isinstance(e, Template):
        return [p for p in e.parts if isinstance(p, Expr)]
    if isinstance(e, Directive):
        return [e.expr] if e.expr is not None else []
    if isinstance(e, Traversal):
        return [v for k, v in e.ops if k == "index"]
    if isinstance(e, Postfix):
        return [e.base] + [v for k, v in e.ops if k == "index"]
    if isinstance(e, Call):
        return list(e.args)
    if isinstance(e, TupleExpr):
        return list(e.items)
    if isinstance(e, ObjectExpr):
        return [x for kv in e.items for x in kv]
    if isinstance(e, Conditional):
        return [e.cond, e.true, e.false]
    if isinstance(e, BinOp):
        return [e.left, e.right]
    if isinstance(e, UnOp):
        return [e.operand]
    return []


def walk_refs(e, bound: frozenset = frozenset()):
    """Yield (Traversal, bound_names) for every variable reference in ``e``.

    Names introduced by for-expressions and %{for} directives are passed in
    ``bound`` so callers can ignore them. Object keys that are bare
    identifiers are literal keys in HCL, not references.
    """
    if e is None:
        return
    if isinstance(e, Traversal):
        yield e, bound
        for k, v in e.ops:
            if k == "index":
                yield from walk_refs(v, bound)
        return
    if isinstance(e, ForExpr):
        yield from walk_refs(e.coll, bound)
        inner = bound | {n for n in (e.key_var, e.val_var) if n}
        yield from walk_refs(e.key_expr, inner)
        yield from walk_refs(e.val_expr, inner)
        yield from walk_refs(e.cond, inner)
        return
    if isinstance(e, ObjectExpr):
        for k, v in e.items:
            if not (isinstance(k, Traversal) and not k.ops):
                yield from walk_refs(k, bound)
            yield from walk_refs(v, bound)
        return
    if isinstance(e, Template):
        scope = bound
        for p in e.parts:
            if isinstance(p, Directive) and p.kind == "for":
                yield from walk_refs(p.expr, scope)
                scope = scope | set(p.names)
            elif isinstance(p, Directive) and p.kind == "endfor":
                scope = bound
            elif isinstance(p, Expr):
                yield from walk_refs(p, scope)
        return
    for c in children(e):
        yield from walk_refs(c, bound)


def iter_calls(e):
    """Yield every function Call node in ``e``."""
    if e is None:
        return
    if isinstance(e, Call):
        yield e
    if isinstance(e, ForExpr):
        for c in (e.coll, e.key_expr, e.val_expr, e.cond):
            yield from iter_calls(c)
        return
    for c in children(e):
        yield from iter_calls(c)


def iter_strings(e):
    """Yield every literal string fragment in ``e`` (for lint rules)."""
    if e is None:
        return
    if isinstance(e, Template):
        for p in e.parts:
            if isinstance(p, str):
                yield p
            else:
                yield from iter_strings(p)
        return
    if isinstance(e, ForExpr):
        for c in (e.coll, e.key_expr, e.val_expr, e.cond):
            yield from iter_strings(c)
        return
    for c in children(e):
        yield from iter_strings(c)


def evaluate_static(e):
    """Best-effort constant folding of literal expressions (defaults, tfvars)."""
    if isinstance(e, Literal):
        return e.value
    if isinstance(e, Template):
        lit = e.literal()
        if lit is None:
            raise ValueError("non-static template")
        return lit
    if isinstance(e, TupleExpr):
        return [evaluate_static(x) for x in e.items]
    if isinstance(e, ObjectExpr):
        out = {}
        for k, v in e.items:
            name = key_name(k)
            if name is None:
                raise ValueError("non-static object key")
            out[name] = evaluate_static(v)
        return out
    if isinstance(e, UnOp) and e.op == "-":
        return -evaluate_static(e.operand)
    raise ValueError(f"non-static expression {type(e).__name__}")
