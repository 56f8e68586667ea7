"""HCL2 native-syntax lexer (offline; no terraform binary in this environment).

Produces a flat token stream. Template strings ("...${x}..." and heredocs) are
tokenised into a single TEMPLATE token holding raw parts; the parser re-lexes
the interpolation bodies. Comments (#, //, /* */) are dropped but counted so
line numbers stay exact.
"""
from __future__ import annotations

from dataclasses import dataclass

PUNCT3 = ("...",)
PUNCT2 = ("==", "!=", "<=", ">=", "&&", "||", "=>", "${", "%{")
PUNCT1 = set("{}[]()=,.:?+-*/%<>!")


class HCLSyntaxError(ValueError):
    def __init__(self, msg: str, line: int, col: int = 0, filename: str = ""):
        super().__init__(f"{filename}:{line}:{col}: {msg}")
        self.line, self.col, self.filename = line, col, filename


@dataclass
class Token:
    kind: str     # IDENT NUMBER TEMPLATE HEREDOC PUNCT NEWLINE EOF
    value: object
    line: int
    col: int

    def __repr__(self) -> str:  # pragma: no cover - debugging aid
        return f"Token({self.kind},{self.value!r},{self.line})"


@dataclass
class TemplatePart:
    """A literal chunk (``is_expr`` False) or an interpolation/directive source."""

    text: str
    is_expr: bool = False
    is_directive: bool = False
    line: int = 0


def _is_ident_start(c: str) -> bool:
    return c.isalpha() or c == "_"


def _is_ident(c: str) -> bool:
    return c.isalnum() or c in "_-"


class Lexer:
    def __init__(self, src: str, filename: str = ""):
        self.s = src
        self.n = len(src)
        self.i = 0
        self.line = 1
        self.col = 1
        self.filename = filename
        self.toks: list[Token] = []

    def err(self, msg: str) -> HCLSyntaxError:
        return HCLSyntaxError(msg, self.line, self.col, self.filename)

    def _adv(self, k: int = 1) -> str:
        out = self.s[self.i:self.i + k]
        for ch in out:
            if ch == "\n":
                self.line += 1
                self.col = 1
            else:
                self.col += 1
        self.i += k
        return out

    def _peek(self, k: int = 0) -> str:
        j = self.i + k
        return self.s[j] if j < self.n else ""

    def tokens(self) -> list[Token]:
        while self.i < self.n:
            c = self._peek()
            if c in " \t\r":
                self._adv()
            elif c == "\n":
                self.toks.append(Token("NEWLINE", "\n", self.line, self.col))
                self._adv()
            elif c == "#" or (c == "/" and self._peek(1) == "/"):
                while self.i < self.n and self._peek() != "\n":
                    self._adv()
            elif c == "/" and self._peek(1) == "*":
                start = self.line
                self._adv(2)
                while self.i < self.n and not (self._peek() == "*" and self._peek(1) == "/"):
                    self._adv()
                if self.i >= self.n:
                    raise HCLSyntaxError("unterminated block comment", start, 0, self.filename)
                self._adv(2)
            elif c == '"':
                self._string()
            elif c == "<" and self._peek(1) == "<" and (self._peek(2).isalpha() or self._peek(2) == "-"):
                self._heredoc()
            elif c.isdigit():
                self._number()
            elif _is_ident_start(c):
                line, col = self.line, self.col
                j = self.i
                while j < self.n and _is_ident(self.s[j]):
                    j += 1
                word = self.s[self.i:j]
                self._adv(j - self.i)
                self.toks.append(Token("IDENT", word, line, col))
            else:
                line, col = self.line, self.col
                for p in PUNCT3 + PUNCT2:
                    if self.s.startswith(p, self.i):
                        self._adv(len(p))
                        self.toks.append(Token("PUNCT", p, line, col))
                        break
                else:
                    if c in PUNCT1:
                        self._adv()
                        self.toks.append(Token("PUNCT", c, line, col))
                    else:
                        raise self.err(f"unexpected character {c!r}")
        self.toks.append(Token("EOF", None, self.line, self.col))
        return self.toks

    def _number(self) -> None:
        line, col = self.line, self.col
        j = self.i
        while j < self.n and self.s[j].isdigit():
            j += 1
        if j < self.n and self.s[j] == "." and j + 1 < self.n and self.s[j + 1].isdigit():
            j += 1
            while j < self.n and self.s[j].isdigit():
                j += 1
        if j < self.n and self.s[j] in "eE":
            k = j + 1
            if k < self.n and self.s[k] in "+-":
                k += 1
            if k < self.n and self.s[k].isdigit():
                j = k
                while j < self.n and self.s[j].isdigit():
                    j += 1
        text = self.s[self.i:j]
        self._adv(j - self.i)
        val = float(text) if any(ch in text for ch in ".eE") else int(text)
        self.toks.append(Token("NUMBER", val, line, col))

    def _template_body(self, end_quote: bool, terminator: str | None = None) -> list[TemplatePart]:
        """Read template parts until a closing quote (quoted strings) or EOF of
        the heredoc body (terminator handled by caller)."""
        parts: list[TemplatePart] = []
        buf: list[str] = []
        while True:
            if self.i >= self.n:
                if end_quote:
                    raise self.err("unterminated string")
                break
            c = self._peek()
            if end_quote and c == '"':
                self._adv()
                break
            if end_quote and c == "\n":
                raise self.err("newline in quoted string")
            if end_quote and c == "\\":
                nxt = self._peek(1)
                esc = {"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\"}
                if nxt in esc:
                    buf.append(esc[nxt])
                    self._adv(2)
                    continue
                if nxt == "u":
                    code = self.s[self.i + 2:self.i + 6]
                    buf.append(chr(int(code, 16)))
                    self._adv(6)
                    continue
                if nxt == "U":
                    code = self.s[self.i + 2:self.i + 10]
                    buf.append(chr(int(code, 16)))
                    self._adv(10)
                    continue
                raise self.err(f"invalid escape \\{nxt}")
            if c in "$%" and self._peek(1) == c and self._peek(2) == "{":
                buf.append(c + "{")  # $${ / %%{ escapes
                self._adv(3)
                continue
            if c in "$%" and self._peek(1) == "{":
                if buf:
                    parts.append(TemplatePart("".join(buf)))
                    buf = []
                line = self.line
                self._adv(2)
                depth = 1
                start = self.i
                in_str = False
                while self.i < self.n:
                    ch = self._peek()
                    if in_str:
                        if ch == "\\":
                            self._adv(2)
                            continue
                        if ch == '"':
                            in_str = False
                    elif ch == '"':
                        in_str = True
                    elif ch == "{":
                        depth += 1
                    elif ch == "}":
                        depth -= 1
                        if depth == 0:
                            break
                    self._adv()
                if self.i >= self.n:
                    raise self.err("unterminated interpolation")
                body = self.s[start:self.i]
                self._adv()  # closing }
                body = body.strip()
                if body.startswith("~"):
                    body = body[1:]
                if body.endswith("~"):
                    body = body[:-1]
                parts.append(TemplatePart(body.strip(), is_expr=(c == "$"), is_directive=(c == "%"),
                                          line=line))
                continue
            buf.append(c)
            self._adv()
        if buf:
            parts.append(TemplatePart("".join(buf)))
        return parts

    def _string(self) -> None:
        line, col = self.line, self.col
        self._adv()
        parts = self._template_body(end_quote=True)
        self.toks.append(Token("TEMPLATE", parts, line, col))

    def _heredoc(self) -> None:
        line, col = self.line, self.col
        self._adv(2)
        indent = False
        if self._peek() == "-":
            indent = True
            self._adv()
        j = self.i
        while j < self.n and _is_ident(self.s[j]):
            j += 1
        marker = self.s[self.i:j]
        self._adv(j - self.i)
        while self._peek() in " \t\r":
            self._adv()
        if self._peek() != "\n":
            raise self.err("heredoc marker must be followed by a newline")
        self._adv()
        body_lines: list[str] = []
        while True:
            if self.i >= self.n:
                raise HCLSyntaxError(f"unterminated heredoc {marker}", line, col, self.filename)
            j = self.s.find("\n", self.i)
            if j < 0:
                j = self.n
            raw = self.s[self.i:j]
            if raw.strip() == marker:
                self._adv(j - self.i)
                break
            body_lines.append(raw)
            self._adv(j - self.i)
            if self.i < self.n:
                self._adv()  # newline
        if indent:
            ws = [len(ln) - len(ln.lstrip(" \t")) for ln in body_lines if ln.strip()]
            cut = min(ws) if ws else 0
            body_lines = [ln[cut:] for ln in body_lines]
        text = "\n".join(body_lines) + ("\n" if body_lines else "")
        sub = Lexer(text, self.filename)
        sub.line = line + 1
        parts = sub._template_body(end_quote=False)
        self.toks.append(Token("TEMPLATE", parts, line, col))


def tokenize(src: str, filename: str = "") -> list[Token]:
    return Lexer(src, filename).tokens()
