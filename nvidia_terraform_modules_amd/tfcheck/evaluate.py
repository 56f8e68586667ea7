"""A Terraform expression evaluator with plan-time unknowns.

Enough of Terraform's language for an offline ``plan`` (tfcheck/plan.py):
variables (tfvars + defaults, type-converted), locals, ``path.*``,
``terraform.workspace``, ``count.index`` / ``each.*``, operators,
conditionals, ``for`` expressions, splats, and the common function library.
Anything that only exists after apply - resource and data-source attributes,
registry-module outputs - evaluates to :data:`UNKNOWN`, which propagates the
way Terraform's unknown values do (an unknown condition is not an error; an
unknown ``count`` is, exactly as in ``terraform plan``).
"""
from __future__ import annotations

import base64
import hashlib
import ipaddress
import json
import math
import re

from .hcl import (BinOp, Call, Conditional, Directive, ForExpr, Literal, ObjectExpr, Postfix,
                  Template, Traversal, TupleExpr, UnOp, key_name)


class _Unknown:
    _inst = None

    def __new__(cls):
        if cls._inst is None:
            cls._inst = super().__new__(cls)
        return cls._inst

    def __repr__(self):
        return "(known after apply)"


UNKNOWN = _Unknown()


class EvalError(Exception):
    pass


def is_unknown(v) -> bool:
    if v is UNKNOWN:
        return True
    if isinstance(v, (list, tuple)):
        return any(is_unknown(x) for x in v)
    if isinstance(v, dict):
        return any(is_unknown(x) for x in v.values())
    return False


# ------------------------------------------------------------------ functions
def _tostring(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if v is None:
        return None
    if isinstance(v, (list, dict)):
        raise EvalError("cannot convert collection to string")
    return str(v)


def _tonumber(v):
    if v is None:
        return None
    if isinstance(v, bool):
        raise EvalError("cannot convert bool to number")
    if isinstance(v, (int, float)):
        return v
    try:
        f = float(v)
    except (TypeError, ValueError):
        raise EvalError(f"cannot convert {v!r} to number")
    return int(f) if f.is_integer() else f


def _tobool(v):
    if v is None or isinstance(v, bool):
        return v
    if v in ("true", "false"):
        return v == "true"
    raise EvalError(f"cannot convert {v!r} to bool")


def _length(v):
    if isinstance(v, (str, list, dict)):
        return len(v)
    raise EvalError("length() needs a string or collection")


def _merge(*maps):
    out = {}
    for m in maps:
        if m is None:
            continue
        if not isinstance(m, dict):
            raise EvalError("merge() arguments must be maps/objects")
        out.update(m)
    return out


def _flatten(v):
    out = []
    for x in v:
        if isinstance(x, list):
            out.extend(_flatten(x))
        else:
            out.append(x)
    return out


def _cidrsubnet(prefix, newbits, netnum):
    net = ipaddress.ip_network(prefix, strict=False)
    new = net.prefixlen + int(newbits)
    subnets = net.subnets(new_prefix=new)
    for i, s in enumerate(subnets):
        if i == int(netnum):
            return str(s)
    raise EvalError("cidrsubnet: netnum out of range")


def _format(fmt, *args):
    # %s %d %v %q %%; enough for module naming patterns
    out, i, ai = "", 0, 0
    while i < len(fmt):
        c = fmt[i]
        if c == "%" and i + 1 < len(fmt):
            t = fmt[i + 1]
            if t == "%":
                out += "%"
            elif t in "sdvq":
                a = args[ai]
                ai += 1
                out += json.dumps(a) if t == "q" else (_tostring(a) if t != "d" else str(int(a)))
            else:
                raise EvalError(f"format verb %{t} unsupported")
            i += 2
        else:
            out += c
            i += 1
    return out


def _regex(pattern, s):
    m = re.search(pattern, s)
    if not m:
        raise EvalError("regex: no match")
    if m.groupdict():
        return m.groupdict()
    if m.groups():
        return list(m.groups())
    return m.group(0)


def _lookup(m, k, *default):
    if k in m:
        return m[k]
    if default:
        return default[0]
    raise EvalError(f"lookup: key {k!r} not found")


def _element(lst, i):
    return lst[int(i) % len(lst)]


def _one(v):
    if not v:
        return None
    if len(v) == 1:
        return v[0] if isinstance(v, list) else list(v.values())[0]
    raise EvalError("one(): more than one element")


FUNCS = {
    "tostring": _tostring, "tonumber": _tonumber, "tobool": _tobool,
    "tolist": lambda v: list(v), "toset": lambda v: sorted(set(v), key=str) if v else [],
    "tomap": lambda v: dict(v),
    "length": _length, "merge": _merge, "concat": lambda *ls: [x for l in ls for x in l],
    "contains": lambda c, v: v in c, "keys": lambda m: sorted(m), "values": lambda m: [m[k] for k in sorted(m)],
    "lookup": _lookup, "element": _element, "flatten": _flatten, "distinct": lambda l: list(dict.fromkeys(l)),
    "compact": lambda l: [x for x in l if x not in (None, "")], "coalesce": lambda *a: next(x for x in a if x not in (None, "")),
    "coalescelist": lambda *a: next((x for x in a if x), []),
    "join": lambda sep, l: sep.join(_tostring(x) for x in l), "split": lambda sep, s: s.split(sep),
    "upper": str.upper, "lower": str.lower, "title": str.title, "trimspace": str.strip,
    "trimprefix": lambda s, p: s[len(p):] if s.startswith(p) else s,
    "trimsuffix": lambda s, p: s[: -len(p)] if p and s.endswith(p) else s,
    "replace": lambda s, a, b: (re.sub(a[1:-1], b, s) if len(a) > 1 and a.startswith("/") and a.endswith("/") else s.replace(a, b)),
    "substr": lambda s, o, n: s[int(o):] if int(n) < 0 else s[int(o): int(o) + int(n)],
    "startswith": lambda s, p: s.startswith(p), "endswith": lambda s, p: s.endswith(p),
    "format": _format, "regex": _regex, "regexall": lambda p, s: [m.group(0) for m in re.finditer(p, s)],
    "min": lambda *a: min(a), "max": lambda *a: max(a), "abs": abs, "ceil": math.ceil, "floor": math.floor,
    "sum": lambda l: sum(l), "range": lambda *a: list(range(*[int(x) for x in a])),
    "zipmap": lambda k, v: dict(zip(k, v)), "one": _one,
    "alltrue": lambda l: all(l), "anytrue": lambda l: any(l),
    "jsonencode": lambda v: json.dumps(v, separators=(",", ":")),
    "jsondecode": json.loads, "base64encode": lambda s: base64.b64encode(s.encode()).decode(),
    "base64decode": lambda s: base64.b64decode(s).decode(),
    "sha1": lambda s: hashlib.sha1(s.encode()).hexdigest(), "sha256": lambda s: hashlib.sha256(s.encode()).hexdigest(),
    "md5": lambda s: hashlib.md5(s.encode()).hexdigest(),
    "cidrsubnet": _cidrsubnet, "slice": lambda l, a, b: l[int(a):int(b)], "reverse": lambda l: list(reversed(l)),
    "sort": lambda l: sorted(l), "index": lambda l, v: l.index(v), "setunion": lambda *s: sorted(set().union(*s), key=str),
}
# functions whose result cannot be known offline (clock, files, templates, encoders
# with exact formatting we do not reproduce) -> UNKNOWN
UNKNOWN_FUNCS = {"timestamp", "uuid", "file", "filebase64", "templatefile", "fileexists",
                 "yamlencode", "yamldecode", "base64gzip", "filemd5", "filesha256", "bcrypt"}


# ------------------------------------------------------------------ evaluator
class Scope:
    """Name resolution for one module instance."""

    def __init__(self, variables: dict, locals_exprs: dict, module_path: str = ".",
                 extra: dict | None = None):
        self.variables = variables          # name -> value
        self.locals_exprs = locals_exprs    # name -> Expr
        self.local_values: dict = {}
        self._evaluating: set = set()
        self.module_path = module_path
        self.extra = extra or {}            # count / each bindings

    def child(self, **extra) -> "Scope":
        s = Scope(self.variables, self.locals_exprs, self.module_path, {**self.extra, **extra})
        s.local_values = self.local_values
        s._evaluating = self._evaluating
        return s


def _index(v, k):
    if v is UNKNOWN or k is UNKNOWN:
        return UNKNOWN
    if isinstance(v, list):
        return v[int(k)] if -len(v) <= int(k) < len(v) else _raise(f"index {k} out of range")
    if isinstance(v, dict):
        if k in v:
            return v[k]
        raise EvalError(f"key {k!r} not found")
    raise EvalError("cannot index a primitive")


def _raise(msg):
    raise EvalError(msg)


def _apply_ops(v, ops, ev, scope):
    for i, (kind, arg) in enumerate(ops):
        if v is UNKNOWN:
            return UNKNOWN
        if kind == "attr":
            if isinstance(v, dict):
                if arg not in v:
                    raise EvalError(f"attribute {arg!r} not found")
                v = v[arg]
            elif isinstance(v, list):  # legacy attribute splat after [*]
                v = [x[arg] if isinstance(x, dict) else UNKNOWN for x in v]
            else:
                raise EvalError(f"cannot read attribute {arg!r} of a primitive")
        elif kind == "index":
            v = _index(v, ev(arg, scope))
        elif kind in ("splat", "attr_splat"):
            rest = ops[i + 1:]
            items = v if isinstance(v, list) else ([] if v is None else [v])
            return [_apply_ops(x, rest, ev, scope) for x in items]
    return v


class Evaluator:
    def __init__(self, funcs: dict | None = None):
        self.funcs = dict(FUNCS)
        self.funcs.update(funcs or {})

    # ---- public
    def eval(self, e, scope: Scope):
        try:
            return self._eval(e, scope)
        except EvalError:
            raise
        except (TypeError, ValueError, KeyError, IndexError, ZeroDivisionError, StopIteration) as x:
            raise EvalError(str(x) or type(x).__name__)

    # ---- internals
    def _local(self, name: str, scope: Scope):
        if name in scope.local_values:
            return scope.local_values[name]
        if name not in scope.locals_exprs:
            raise EvalError(f"undefined local.{name}")
        if name in scope._evaluating:
            raise EvalError(f"cycle through local.{name}")
        scope._evaluating.add(name)
        try:
            v = self.eval(scope.locals_exprs[name], scope)
        finally:
            scope._evaluating.discard(name)
        scope.local_values[name] = v
        return v

    def _traversal(self, e: Traversal, scope: Scope):
        root, ops = e.root, e.ops
        if root == "var":
            name = ops[0][1]
            if name not in scope.variables:
                raise EvalError(f"undefined var.{name}")
            return _apply_ops(scope.variables[name], ops[1:], self._eval, scope)
        if root == "local":
            return _apply_ops(self._local(ops[0][1], scope), ops[1:], self._eval, scope)
        if root == "path":
            return scope.module_path if ops and ops[0][1] in ("module", "root", "cwd") else UNKNOWN
        if root == "terraform":
            return "default" if ops and ops[0][1] == "workspace" else UNKNOWN
        if root in ("count", "each"):
            if root not in scope.extra:
                raise EvalError(f"{root} used outside a resource with {root}")
            return _apply_ops(scope.extra[root], ops, self._eval, scope)
        if root in scope.extra:              # for-expression variables
            return _apply_ops(scope.extra[root], ops, self._eval, scope)
        # resources, data sources, modules, self: only known after apply
        return UNKNOWN

    def _eval(self, e, scope: Scope):
        if isinstance(e, Literal):
            return e.value
        if isinstance(e, Template):
            lit = e.literal()
            if lit is not None:
                return lit
            if len(e.parts) == 1 and not isinstance(e.parts[0], (str, Directive)):
                return self._eval(e.parts[0], scope)      # "${x}" keeps x's type
            out = ""
            for p in e.parts:
                if isinstance(p, str):
                    out += p
                elif isinstance(p, Directive):
                    return UNKNOWN                         # %{ } directives: not modelled
                else:
                    v = self._eval(p, scope)
                    if is_unknown(v):
                        return UNKNOWN
                    out += _tostring(v)
            return out
        if isinstance(e, Traversal):
            return self._traversal(e, scope)
        if isinstance(e, Postfix):
            return _apply_ops(self._eval(e.base, scope), e.ops, self._eval, scope)
        if isinstance(e, TupleExpr):
            return [self._eval(x, scope) for x in e.items]
        if isinstance(e, ObjectExpr):
            out = {}
            for k, v in e.items:
                name = key_name(k)
                if name is None:
                    kv = self._eval(k, scope)
                    if is_unknown(kv):
                        return UNKNOWN
                    name = _tostring(kv)
                out[name] = self._eval(v, scope)
            return out
        if isinstance(e, Conditional):
            c = self._eval(e.cond, scope)
            if c is UNKNOWN:
                return UNKNOWN
            return self._eval(e.true if c else e.false, scope)
        if isinstance(e, UnOp):
            v = self._eval(e.operand, scope)
            if v is UNKNOWN:
                return UNKNOWN
            return (not v) if e.op == "!" else -v
        if isinstance(e, BinOp):
            return self._binop(e, scope)
        if isinstance(e, Call):
            return self._call(e, scope)
        if isinstance(e, ForExpr):
            return self._for(e, scope)
        raise EvalError(f"cannot evaluate {type(e).__name__}")

    def _binop(self, e: BinOp, scope: Scope):
        op = e.op
        a = self._eval(e.left, scope)
        if op == "&&" and a is False:
            return False
        if op == "||" and a is True:
            return True
        b = self._eval(e.right, scope)
        if op in ("==", "!="):
            if is_unknown(a) or is_unknown(b):
                return UNKNOWN
            r = a == b
            return r if op == "==" else not r
        if a is UNKNOWN or b is UNKNOWN:
            return UNKNOWN
        if op == "&&":
            return bool(a) and bool(b)
        if op == "||":
            return bool(a) or bool(b)
        a, b = _tonumber(a), _tonumber(b)
        return {"+": lambda: a + b, "-": lambda: a - b, "*": lambda: a * b,
                "/": lambda: a / b, "%": lambda: a % b, "<": lambda: a < b, ">": lambda: a > b,
                "<=": lambda: a <= b, ">=": lambda: a >= b}[op]()

    def _call(self, e: Call, scope: Scope):
        name = e.name
        if name == "can":
            try:
                v = self._eval(e.args[0], scope)
                return UNKNOWN if v is UNKNOWN else True
            except EvalError:
                return False
        if name == "try":
            for a in e.args:
                try:
                    return self._eval(a, scope)
                except EvalError:
                    continue
            raise EvalError("try(): no argument succeeded")
        if name in UNKNOWN_FUNCS:
            return UNKNOWN
        if name not in self.funcs:
            return UNKNOWN                # provider / unmodelled function
        args = [self._eval(a, scope) for a in e.args]
        if e.expand and args:
            args = args[:-1] + list(args[-1])
        if any(is_unknown(a) for a in args):
            return UNKNOWN
        return self.funcs[name](*args)

    def _for(self, e: ForExpr, scope: Scope):
        coll = self._eval(e.coll, scope)
        if is_unknown(coll):
            return UNKNOWN
        pairs = list(coll.items()) if isinstance(coll, dict) else list(enumerate(coll))
        out_list, out_map = [], {}
        for k, v in pairs:
            binds = {e.val_var: v}
            if e.key_var:
                binds[e.key_var] = k
            s = scope.child(**binds)
            if e.cond is not None:
                c = self._eval(e.cond, s)
                if c is UNKNOWN:
                    return UNKNOWN
                if not c:
                    continue
            if e.is_object:
                kk = self._eval(e.key_expr, s)
                vv = self._eval(e.val_expr, s)
                if e.grouping:
                    out_map.setdefault(kk, []).append(vv)
                else:
                    out_map[kk] = vv
            else:
                out_list.append(self._eval(e.val_expr, s))
        return out_map if e.is_object else out_list


# ------------------------------------------------------------ type conversion
def convert(value, type_expr, ev: Evaluator | None = None):
    """Convert a tfvars / default value to a variable's declared type (the
    primitive conversions Terraform performs; collections recurse)."""
    if type_expr is None or value is None or value is UNKNOWN:
        return value
    if isinstance(type_expr, Traversal) and not type_expr.ops:
        t = type_expr.root
        if t == "string":
            return _tostring(value)
        if t == "number":
            return _tonumber(value)
        if t == "bool":
            return _tobool(value)
        return value                                   # any
    if isinstance(type_expr, Call):
        t = type_expr.name
        inner = type_expr.args[0] if type_expr.args else None
        if t in ("list", "set") and isinstance(value, list):
            return [convert(v, inner) for v in value]
        if t == "map" and isinstance(value, dict):
            return {k: convert(v, inner) for k, v in value.items()}
        if t == "object" and isinstance(value, dict) and isinstance(inner, ObjectExpr):
            out = dict(value)
            for k, te in inner.items:
                n = key_name(k)
                if n in out:
                    out[n] = convert(out[n], te)
            return out
        if t in ("list", "set", "map", "object", "tuple"):
            raise EvalError(f"value is not a {t}")
    return value
