"""Offline ``terraform fmt`` layout check (the reference's one mandated static
gate: ``/root/reference/CONTRIBUTING.md:12``).

There is no terraform binary here, so this re-implements the whitespace model
of HCL's canonical formatter over its own token stream:

* **lines and cells.** Every source line is split into a *lead* cell, an
  *assign* cell (from the first ``=`` at a position > 0, but only when the
  rest of the line has balanced brackets: ``tags = {`` keeps its ``=`` in the
  lead) and a trailing *comment* cell (a ``#`` / ``//`` comment after code).
* **indentation.** Two spaces per level. A line whose lead + assign cells open
  more brackets than they close indents the lines after it by ONE level
  (however many it opened) and remembers how many; closing brackets unwind
  those levels; the closing line itself is already dedented.
* **spacing.** One space between tokens, except: none after an open bracket
  or before a close bracket, before ``,`` / ``...`` / ``.``, after ``.``,
  between a function name and ``(``, before ``[`` of an index, inside string
  templates, and after a unary minus; ``{`` and ``}`` take spaces (``{}``
  does not).
* **alignment.** In a run of consecutive assign lines the ``=`` signs line up
  one column after the longest lead; in a run of consecutive lines with
  trailing comments the comments line up one column after the longest code.
  A blank line, a comment-only line or a line opening a multi-line value ends
  the run.

Heredoc bodies and ``%{ }`` directives are left as they are (never
flagged). ``formatted(text)`` returns the canonical text; ``fmt_diff``
returns the lines that differ (the tab / trailing-whitespace checks stay in
``analysis.fmt_findings``). The reference's own ``.tf`` files - which its
contribution rule says were ``terraform fmt``-ed - are the test corpus
(tests/test_tfcheck_fmt.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path

OPEN = {"OBRACE", "OBRACK", "OPAREN", "TINTERP", "TCONTROL"}
CLOSE = {"CBRACE", "CBRACK", "CPAREN", "TSEQEND"}
_P3 = {"...": "ELLIPSIS"}
_P2 = {"==": "EQOP", "!=": "NEQ", "<=": "LTE", ">=": "GTE", "&&": "AND", "||": "OR",
       "=>": "ARROW"}
_P1 = {"{": "OBRACE", "}": "CBRACE", "[": "OBRACK", "]": "CBRACK", "(": "OPAREN",
       ")": "CPAREN", "=": "EQUAL", ",": "COMMA", ".": "DOT", ":": "COLON", "?": "QUESTION",
       "+": "PLUS", "-": "MINUS", "*": "STAR", "/": "SLASH", "%": "PERCENT", "<": "LT",
       ">": "GT", "!": "BANG", "~": "TILDE"}
# a minus after one of these is a negation (no space after it)
_NEG_BEFORE = {None, "OPAREN", "OBRACE", "OBRACK", "EQUAL", "COLON", "COMMA", "QUESTION",
               "PLUS", "STAR", "SLASH", "PERCENT", "MINUS", "EQOP", "NEQ", "GT", "GTE", "LT",
               "LTE", "AND", "OR", "BANG", "ARROW", "TINTERP"}


@dataclass
class Tok:
    kind: str
    text: str
    spaces: int = 0        # spaces before it in the source
    verbatim: bool = False  # inside a %{ } directive: spacing not checked


@dataclass
class Line:
    lead: list[Tok] = field(default_factory=list)
    assign: list[Tok] = field(default_factory=list)
    comment: list[Tok] = field(default_factory=list)
    newline: bool = False


class FmtLexError(ValueError):
    pass


class _Lexer:
    def __init__(self, s: str):
        self.s, self.i, self.n = s, 0, len(s)
        self.out: list[Tok] = []

    def run(self) -> list[Tok]:
        self._code(stop_at_brace=False, verbatim=False)
        return self.out

    def _emit(self, kind: str, text: str, spaces: int, verbatim: bool = False) -> None:
        self.out.append(Tok(kind, text, spaces, verbatim))

    def _code(self, stop_at_brace: bool, verbatim: bool) -> None:
        """Tokens until EOF, or (inside ``${``/``%{``) the brace that closes it."""
        s = self.s
        depth = 0
        while self.i < self.n:
            sp = 0
            while self.i < self.n and s[self.i] in " \t\r":
                sp += 1
                self.i += 1
            if self.i >= self.n:
                break
            c = s[self.i]
            if c == "\n":
                self._emit("NEWLINE", "\n", 0)
                self.i += 1
            elif c == "#" or s.startswith("//", self.i):
                j = s.find("\n", self.i)
                j = self.n if j < 0 else j + 1
                self._emit("COMMENT", s[self.i:j], sp)
                self.i = j
            elif s.startswith("/*", self.i):
                j = s.find("*/", self.i + 2)
                if j < 0:
                    raise FmtLexError("unterminated /* comment")
                self._emit("BLOCKCOMMENT", s[self.i:j + 2], sp)
                self.i = j + 2
            elif c == '"':
                self._emit("OQUOTE", '"', sp, verbatim)
                self.i += 1
                self._template(verbatim)
            elif s.startswith("<<", self.i) and self._heredoc(sp):
                pass
            elif c.isalpha() or c == "_":
                j = self.i + 1
                while j < self.n and (s[j].isalnum() or s[j] in "_-"):
                    j += 1
                self._emit("IDENT", s[self.i:j], sp, verbatim)
                self.i = j
            elif c.isdigit():
                j = self.i + 1
                while j < self.n and (s[j].isalnum() or s[j] == "." and j + 1 < self.n
                                      and s[j + 1].isdigit()):
                    j += 1
                self._emit("NUMBER", s[self.i:j], sp, verbatim)
                self.i = j
            else:
                for table, k in ((_P3, 3), (_P2, 2), (_P1, 1)):
                    t = s[self.i:self.i + k]
                    if t in table:
                        kind = table[t]
                        if kind == "CBRACE" and stop_at_brace and depth == 0:
                            self._emit("TSEQEND", "}", sp, verbatim)
                            self.i += 1
                            return
                        if kind == "OBRACE":
                            depth += 1
                        elif kind == "CBRACE":
                            depth -= 1
                        self._emit(kind, t, sp, verbatim)
                        self.i += k
                        break
                else:
                    raise FmtLexError(f"unexpected character {c!r}")
        if stop_at_brace:
            raise FmtLexError("unterminated template interpolation")

    def _template(self, verbatim: bool) -> None:
        """Body of a quoted string up to and including its closing quote."""
        s = self.s
        lit = []
        while self.i < self.n:
            c = s[self.i]
            if c == "\\" and self.i + 1 < self.n:
                lit.append(s[self.i:self.i + 2])
                self.i += 2
            elif (s.startswith("$${", self.i) or s.startswith("%%{", self.i)):
                lit.append(s[self.i:self.i + 3])
                self.i += 3
            elif s.startswith("${", self.i) or s.startswith("%{", self.i):
                if lit:
                    self._emit("QLIT", "".join(lit), 0, verbatim)
                    lit = []
                directive = c == "%"
                self._emit("TCONTROL" if directive else "TINTERP", s[self.i:self.i + 2], 0,
                           verbatim)
                self.i += 2
                self._code(stop_at_brace=True, verbatim=verbatim or directive)
            elif c == '"':
                if lit:
                    self._emit("QLIT", "".join(lit), 0, verbatim)
                self._emit("CQUOTE", '"', 0, verbatim)
                self.i += 1
                return
            elif c == "\n":
                raise FmtLexError("newline in a quoted string")
            else:
                lit.append(c)
                self.i += 1
        raise FmtLexError("unterminated string")

    def _heredoc(self, sp: int) -> bool:
        """``<<EOT`` / ``<<-EOT`` through its closing marker, as ONE opaque token
        (the formatter never re-indents a heredoc body)."""
        s = self.s
        j = self.i + 2
        if j < self.n and s[j] == "-":
            j += 1
        k = j
        while k < self.n and (s[k].isalnum() or s[k] == "_"):
            k += 1
        if k == j or k >= self.n or s[k] != "\n":
            return False
        marker = s[j:k]
        pos = k + 1
        while pos < self.n:
            e = s.find("\n", pos)
            e = self.n if e < 0 else e
            if s[pos:e].strip() == marker:
                self._emit("HEREDOC", s[self.i:e], sp)
                self.i = e
                return True
            pos = e + 1
        raise FmtLexError(f"unterminated heredoc {marker}")


def _bracket(t: Tok) -> int:
    return 1 if t.kind in OPEN else -1 if t.kind in CLOSE else 0


def _lines(toks: list[Tok]) -> list[Line]:
    lines, cur = [], []
    for t in toks:
        cur.append(t)
        if t.kind in ("NEWLINE", "COMMENT"):
            lines.append(cur)
            cur = []
    if cur:
        lines.append(cur)
    out = []
    for raw in lines:
        ln = Line()
        if raw and raw[-1].kind == "NEWLINE":
            ln.newline = True
            raw = raw[:-1]
        if len(raw) > 1 and raw[-1].kind == "COMMENT":
            ln.comment = [raw[-1]]
            raw = raw[:-1]
        for i, t in enumerate(raw):
            if i > 0 and t.kind == "EQUAL":
                if sum(_bracket(x) for x in raw[i:]) == 0:
                    ln.assign = raw[i:]
                    raw = raw[:i]
                break
        ln.lead = raw
        out.append(ln)
    return out


def _space_after(subject: Tok, before: Tok | None, after: Tok) -> bool | None:
    """Spaces between ``subject`` and ``after`` (True = one, False = none, None =
    not checked)."""
    sk, ak = subject.kind, after.kind
    if subject.verbatim or after.verbatim:
        return None
    if sk == "IDENT" and ak == "OPAREN":
        # a call; "for ... if (cond)" reads the keyword as a function name too,
        # which the corpus does not pin: never flagged
        return None if subject.text == "if" else False
    if sk == "DOT" or ak == "DOT":
        return False
    if ak in ("COMMA", "ELLIPSIS"):
        return False
    if sk == "COMMA":
        return True
    if sk in ("QLIT", "OQUOTE", "HEREDOC") or ak in ("QLIT", "CQUOTE"):
        return False
    if sk == "IDENT" and subject.text == "in" and before is not None and before.kind == "IDENT":
        return True
    if ak == "OBRACK" and (sk in ("IDENT", "NUMBER") or _bracket(subject) < 0):
        return False
    if sk == "MINUS":
        return (before.kind if before is not None else None) not in _NEG_BEFORE
    if sk == "BANG":
        return None      # "!x": not pinned by the corpus; never flagged
    if sk == "TILDE" or ak == "TILDE":
        return None      # template strip markers ("${~ x ~}"): never flagged
    if sk == "OBRACE" or ak == "CBRACE":
        return not (sk == "OBRACE" and ak == "CBRACE")
    if sk in ("TINTERP", "TCONTROL") and ak == "OBRACE":
        return True
    if sk == "CBRACE" and ak == "TSEQEND":
        return True
    if sk == "TSEQEND" and ak in ("TINTERP", "TCONTROL"):
        return False
    if _bracket(subject) > 0:
        return False
    if _bracket(after) < 0:
        return False
    return True


def _cols(toks: list[Tok]) -> int:
    return sum(t.spaces + len(t.text) for t in toks)


def _layout(lines: list[Line]) -> None:
    """Rewrite every token's ``spaces`` to the canonical value, in place (a
    token whose spacing is not checked keeps its source spacing)."""
    indents: list[int] = []
    for ln in lines:
        first = (ln.lead or ln.assign or ln.comment or [None])[0]
        if first is None:
            continue
        net = 0
        for t in ln.lead + ln.assign:
            net += _bracket(t)
        if net > 0:
            first.spaces = 2 * len(indents)
            indents.append(net)
        elif net < 0:
            closed = -net
            while closed > 0 and indents:
                if closed > indents[-1]:
                    closed -= indents.pop()
                elif closed < indents[-1]:
                    indents[-1] -= closed
                    closed = 0
                else:
                    indents.pop()
                    closed = 0
            first.spaces = 2 * len(indents)
        else:
            first.spaces = 2 * len(indents)
        for cell in (ln.lead, ln.assign):
            for i, t in enumerate(cell):
                if cell is ln.assign and i == 0:
                    t.spaces = 1
                if i + 1 < len(cell):
                    v = _space_after(t, cell[i - 1] if i else None, cell[i + 1])
                    if v is not None:
                        cell[i + 1].spaces = 1 if v else 0
    # "=" alignment over runs of assign lines, then trailing-comment alignment
    for has, cols, head in ((lambda l: bool(l.assign), lambda l: _cols(l.lead),
                             lambda l: l.assign[0]),
                            (lambda l: bool(l.comment), lambda l: _cols(l.lead) + _cols(l.assign),
                             lambda l: l.comment[0])):
        run: list[Line] = []
        for ln in lines + [Line()]:
            if has(ln):
                run.append(ln)
                continue
            if run:
                width = max(cols(x) for x in run)
                for x in run:
                    head(x).spaces = 1 + width - cols(x)
                run = []


def _render(lines: list[Line]) -> str:
    out = []
    for ln in lines:
        out.append("".join(" " * t.spaces + t.text for t in ln.lead + ln.assign + ln.comment))
        if ln.newline:
            out.append("\n")
    return "".join(out)


def formatted(text: str) -> str:
    """``text`` laid out the way ``terraform fmt`` would (whitespace only)."""
    lines = _lines(_Lexer(text).run())
    _layout(lines)
    return _render(lines)


def fmt_diff(text: str) -> list[tuple[int, str, str]]:
    """(line number, source line, canonical line) for every line whose layout
    differs; trailing whitespace is ignored here (``analysis`` reports it)."""
    want = formatted(text).split("\n")
    have = text.split("\n")
    out = []
    for i, (h, w) in enumerate(zip(have, want), 1):
        if h.rstrip() != w.rstrip():
            out.append((i, h, w))
    return out


def hcl_files(root: Path) -> list[Path]:
    """Every .tf / .tfvars under ``root`` (no .terraform caches, no scratch)."""
    root = Path(root)
    files = sorted(root.rglob("*.tf")) + sorted(root.rglob("*.tfvars"))
    return [f for f in files if not ({".terraform", "gpurun_out", ".git"} & set(f.parts))]


def write_formatted(root: Path) -> list[Path]:
    """Rewrite the files under ``root`` whose layout is not canonical; returns them."""
    changed = []
    for f in hcl_files(root):
        text = f.read_text()
        new = formatted(text)   # heredoc bodies and comments stay byte for byte
        if new != text:
            f.write_text(new)
            changed.append(f)
    return changed
