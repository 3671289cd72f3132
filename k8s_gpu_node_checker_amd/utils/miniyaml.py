"""Dependency-free parser for the YAML subset kubeconfig files use.

Importing PyYAML costs ~10 ms, about a third of this CLI's own start-up
(at 1-16 nodes the check is import-bound).  kubeconfigs written by
``kubectl``/cloud CLIs use block mappings, block sequences (``- key: v``),
plain / single- / double-quoted scalars, ``{}``/``[]`` and comments.  This
parser handles exactly that and raises :class:`Unsupported` on anything else
(anchors, tags, block scalars, flow collections with content, multi-document
streams), in which case the caller falls back to PyYAML -- results are never
silently different.
"""

from __future__ import annotations

TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, List, Optional, Tuple


class Unsupported(ValueError):
    pass


_BOOLS = {"true": True, "True": True, "TRUE": True, "false": False, "False": False, "FALSE": False}
_NULLS = {"", "~", "null", "Null", "NULL"}


def _strip_comment(s: str) -> str:
    """Remove a trailing `` # comment`` outside quotes."""
    if "#" not in s:
        return s.rstrip()
    q = None
    i = 0
    while i < len(s):
        c = s[i]
        if q:
            if c == "\\" and q == '"':
                i += 2
                continue
            if c == q:
                if q == "'" and i + 1 < len(s) and s[i + 1] == "'":
                    i += 2
                    continue
                q = None
        elif c in "'\"" and (i == 0 or s[i - 1] in " :-[{,"):
            q = c
        elif c == "#" and (i == 0 or s[i - 1] in " \t"):
            return s[:i].rstrip()
        i += 1
    return s.rstrip()


_ESC = {"n": "\n", "t": "\t", "r": "\r", "\\": "\\", '"': '"', "/": "/", "0": "\0", "b": "\b", "f": "\f", " ": " "}


def _scalar(tok: str) -> Any:
    t = tok.strip()
    if not t:
        return None
    c = t[0]
    if c == '"':
        if len(t) < 2 or t[-1] != '"':
            raise Unsupported("multi-line or unterminated double-quoted scalar")
        body = t[1:-1]
        out = []
        i = 0
        while i < len(body):
            ch = body[i]
            if ch == "\\":
                nx = body[i + 1:i + 2]
                if nx in _ESC:
                    out.append(_ESC[nx])
                    i += 2
                    continue
                width = {"x": 2, "u": 4, "U": 8}.get(nx)
                if width and len(body) >= i + 2 + width:
                    try:
                        out.append(chr(int(body[i + 2:i + 2 + width], 16)))
                    except ValueError:
                        raise Unsupported("escape")
                    i += 2 + width
                    continue
                raise Unsupported("escape")
            out.append(ch)
            i += 1
        return "".join(out)
    if c == "'":
        if len(t) < 2 or t[-1] != "'":
            raise Unsupported("multi-line or unterminated single-quoted scalar")
        return t[1:-1].replace("''", "'")
    if t == "{}":
        return {}
    if t == "[]":
        return []
    if c in "{[&*!|>%@`":
        raise Unsupported(f"construct {c!r}")
    if t in _NULLS:
        return None
    if t in _BOOLS:
        return _BOOLS[t]
    if t.lstrip("-+").isdigit() and not (len(t.lstrip("-+")) > 1 and t.lstrip("-+")[0] == "0"):
        return int(t)
    if t[0].isdigit() or t[0] in "-+.":
        try:
            float(t)
        except ValueError:
            return t
        raise Unsupported("float scalar")  # YAML float forms differ from Python's; let PyYAML decide
    return t


def _split_key(s: str) -> Optional[Tuple[str, str]]:
    """``key: value`` -> (key, value) with quoted keys supported; None if not a mapping entry."""
    if s[:1] in "'\"":
        q = s[0]
        end = 1
        while True:
            end = s.find(q, end)
            if end < 0:
                raise Unsupported("quoted key")
            if q == '"' and s[end - 1] == "\\":
                end += 1
                continue
            if q == "'" and s[end + 1:end + 2] == "'":
                end += 2
                continue
            break
        rest = s[end + 1:]
        if not rest.startswith(":") or (len(rest) > 1 and rest[1] != " "):
            return None
        return _scalar(s[:end + 1]), rest[1:]
    i = s.find(": ")
    if i < 0:
        if s.endswith(":"):
            return s[:-1], ""
        return None
    return s[:i], s[i + 2:]


class _Parser:
    def __init__(self, text: str):
        self.lines: List[Tuple[int, str]] = []
        for raw in text.splitlines():
            if "\t" in raw[: len(raw) - len(raw.lstrip())]:
                raise Unsupported("tab indentation")
            body = _strip_comment(raw)
            if not body.strip():
                continue
            if body.strip() in ("---", "..."):
                if self.lines:
                    raise Unsupported("multi-document stream")
                continue
            ind = len(body) - len(body.lstrip(" "))
            self.lines.append((ind, body.strip()))
        self.i = 0

    def parse(self) -> Any:
        if not self.lines:
            return None
        val = self.block(self.lines[0][0])
        if self.i != len(self.lines):
            raise Unsupported("trailing content")
        return val

    def block(self, ind: int) -> Any:
        first = self.lines[self.i][1]
        if first == "-" or first.startswith("- "):
            return self.seq(ind)
        if _split_key(first) is not None:
            return self.mapping(ind)
        if len(self.lines) == 1:
            self.i += 1
            return _scalar(first)
        raise Unsupported("multi-line plain scalar")

    def mapping(self, ind: int, first_inline: Optional[str] = None) -> dict:
        out: dict = {}
        pending = first_inline
        while True:
            if pending is not None:
                text, pending = pending, None
            else:
                if self.i >= len(self.lines):
                    break
                li, text = self.lines[self.i]
                if li < ind:
                    break
                if li > ind:
                    raise Unsupported("bad indentation")
                if text == "-" or text.startswith("- "):
                    break
                self.i += 1
            kv = _split_key(text)
            if kv is None:
                raise Unsupported(f"expected key: {text[:30]!r}")
            k, v = kv
            if v.strip():
                out[k] = _scalar(v)
            elif self.i < len(self.lines) and (self.lines[self.i][0] > ind or (
                    self.lines[self.i][0] == ind and (self.lines[self.i][1] == "-" or
                                                      self.lines[self.i][1].startswith("- ")))):
                out[k] = self.block(self.lines[self.i][0])
            else:
                out[k] = None
        return out

    def seq(self, ind: int) -> list:
        out: list = []
        while self.i < len(self.lines):
            li, text = self.lines[self.i]
            if li != ind or not (text == "-" or text.startswith("- ")):
                if li > ind:
                    raise Unsupported("bad indentation")
                break
            self.i += 1
            rest = text[1:].lstrip(" ")
            if not rest:
                if self.i < len(self.lines) and self.lines[self.i][0] > ind:
                    out.append(self.block(self.lines[self.i][0]))
                else:
                    out.append(None)
                continue
            if rest == "-" or rest.startswith("- "):
                raise Unsupported("nested inline sequence")
            if _split_key(rest) is not None:
                # "- key: v" opens a mapping whose keys sit at the column of "key"
                col = ind + (len(text) - len(rest))
                out.append(self.mapping(col, first_inline=rest))
            else:
                out.append(_scalar(rest))
        return out


def loads(text: str) -> Any:
    """Parse ``text``; raises :class:`Unsupported` for YAML outside the kubeconfig subset."""
    return _Parser(text).parse()
