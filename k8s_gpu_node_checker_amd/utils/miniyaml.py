"""Dependency-free parser for the YAML subset kubeconfig files use.

Importing PyYAML costs ~10 ms, about a third of this CLI's own start-up
(at 1-16 nodes the check is import-bound).  kubeconfigs written by
``kubectl``/cloud CLIs use block mappings, block sequences (``- key: v``),
plain / single- / double-quoted scalars, ``{}``/``[]`` and comments.  This
parser handles exactly that and raises :class:`Unsupported` on anything else
(anchors, tags, block scalars, flow collections with content, multi-document
streams), in which case the caller falls back to PyYAML -- results are never
silently different.

Plain scalars (values *and* keys) resolve with PyYAML's YAML 1.1 implicit
resolver (``yaml/resolver.py``, the loader ``kubernetes.config`` uses for the
reference, ``check-gpu-node.py:160-169``): the 18 bool spellings
``yes/no/on/off/true/false`` in three cases, the four null forms, decimal
ints.  Every other form PyYAML's resolver would turn into a non-string (octal,
hex, binary and sexagesimal ints, floats, ``.inf``/``.nan``, timestamps,
``<<``, ``=``) is refused, so PyYAML decides it.  A kubeconfig line
``insecure-skip-tls-verify: no`` is therefore ``False`` here exactly as there.
"""

from __future__ import annotations

TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, List, Optional, Tuple


class Unsupported(ValueError):
    pass


# PyYAML's tag:yaml.org,2002:bool resolver (YAML 1.1) and SafeConstructor.bool_values
_BOOLS = {w: v for v, words in ((True, ("yes", "true", "on")), (False, ("no", "false", "off")))
          for b in words for w in (b, b.capitalize(), b.upper())}
_NULLS = {"", "~", "null", "Null", "NULL"}
_DIGITS = "0123456789"
# printable ASCII, LF and CR; tabs are refused (PyYAML's tab rules differ by context and kubeconfigs have none)
_ASCII_OK = bytes([10, 13]) + bytes(range(0x20, 0x7F))


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
            if ch == '"':
                raise Unsupported("content after a double-quoted scalar")
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
        body = t[1:-1]
        if "'" in body.replace("''", ""):
            raise Unsupported("content after a single-quoted scalar")
        return body.replace("''", "'")
    if t == "{}":
        return {}
    if t == "[]":
        return []
    return _plain(t)


def _plain(t: str) -> Any:
    """Resolve a stripped, non-empty plain scalar the way PyYAML's SafeLoader does, or refuse."""
    c = t[0]
    if c in "{[]},#&*!|>'\"%@`" or (c in "-?:" and (len(t) == 1 or t[1] in " \t")):
        raise Unsupported(f"construct {c!r}")
    if t.endswith(":") or ": " in t or "\t" in t or " #" in t:
        raise Unsupported("indicator inside a plain scalar")
    if t in _NULLS:
        return None
    b = _BOOLS.get(t)
    if b is not None:
        return b
    # int / float / timestamp resolvers all start with [-+]?[0-9.]; merge is "<<", value is "="
    num = t[1:] if c in "-+" else t
    if num[:1] in _DIGITS or num[:1] == ".":
        if num.isdigit() and num.isascii() and (num == "0" or num[0] != "0"):
            return int(t)
        raise Unsupported("non-decimal number, float or timestamp scalar")
    if t in ("<<", "="):
        raise Unsupported("merge/value key")
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
        if not s.endswith(":"):
            return None
        i = len(s) - 1
    k = s[:i].rstrip(" ")
    if not k:
        raise Unsupported("empty key")
    return _plain(k), s[i + 2:]


class _Parser:
    def __init__(self, text: str):
        self.lines: List[Tuple[int, str]] = []
        try:
            bad = text.encode("ascii").translate(None, _ASCII_OK)
        except UnicodeEncodeError:
            bad = b"non-ASCII"  # rare in kubeconfigs: PyYAML's reader rules for it are not replicated here
        if bad:
            raise Unsupported("tab, control or non-ASCII character")
        for raw in text.split("\n"):
            if raw.endswith("\r"):
                raw = raw[:-1]
            if "\r" in raw:
                raise Unsupported("bare carriage return")
            if "\t" in raw[: len(raw) - len(raw.lstrip())]:
                raise Unsupported("tab indentation")
            body = _strip_comment(raw)
            if not body.strip():
                continue
            if body[:3] in ("---", "..."):
                if body != "---" or self.lines:
                    raise Unsupported("document marker with content, document end or multi-document stream")
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
