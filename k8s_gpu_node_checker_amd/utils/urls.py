"""URL splitting and path-segment quoting for the transport, without ``urllib.parse``.

``urllib.parse`` pulls in ``re``, ``ipaddress`` and ``warnings`` (~7 ms of a 1-node cold start on a
clean interpreter).  The URLs the checker builds or reads -- the apiserver ``server:`` of a kubeconfig,
a Slack webhook, a proxy -- are plain ``scheme://host[:port][/path][?query]``; anything else (user
info, percent-escapes in the authority, non-ASCII) is handed to ``urllib.parse`` so the result is
always the same as ``urlsplit``'s.
"""

from __future__ import annotations

TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only
    from typing import Optional, Tuple

_UNRESERVED = frozenset("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789_.-~")


class SplitURL:
    """The parts of ``urllib.parse.urlsplit`` the transport reads."""

    __slots__ = ("scheme", "netloc", "hostname", "port", "path", "query", "username", "password")

    def __init__(self, scheme: str, netloc: str, hostname: "Optional[str]", port: "Optional[int]", path: str,
                 query: str, username: "Optional[str]" = None, password: "Optional[str]" = None):
        self.scheme = scheme
        self.netloc = netloc
        self.hostname = hostname
        self.port = port
        self.path = path
        self.query = query
        #: user info, percent-decoded (a proxy's credentials); only URLs with '@' have any
        self.username = username
        self.password = password

    def astuple(self) -> "Tuple":
        return (self.scheme, self.netloc, self.hostname, self.port, self.path, self.query)


def _slow(url: str) -> SplitURL:
    from urllib.parse import unquote, urlsplit
    p = urlsplit(url)
    return SplitURL(p.scheme, p.netloc, p.hostname, p.port, p.path, p.query,
                    unquote(p.username) if p.username is not None else None,
                    unquote(p.password) if p.password is not None else None)


def split(url: str) -> SplitURL:
    """``urlsplit(url)`` -> scheme, hostname (lower case, IPv6 without brackets), port, path, query."""
    # ASCII and printable without space = no byte <= 32 and no DEL (127)
    if not url.isascii() or not url.isprintable() or " " in url or "@" in url or "%" in url or "#" in url or \
            "\\" in url:
        return _slow(url)
    scheme, sep, rest = url.partition("://")
    if not sep or not scheme.isalpha():
        return _slow(url)
    cut = len(rest)
    for ch in "/?":
        i = rest.find(ch)
        if i != -1:
            cut = min(cut, i)
    netloc, tail = rest[:cut], rest[cut:]
    path, _, query = tail.partition("?")
    if netloc.startswith("["):
        end = netloc.find("]")
        if end == -1:
            return _slow(url)
        host, after = netloc[1:end], netloc[end + 1:]
        if after and not after.startswith(":"):
            return _slow(url)
        port_s = after[1:] if after else ""
    else:
        if "]" in netloc or "[" in netloc:
            return _slow(url)  # a stray bracket: urlsplit's "Invalid IPv6 URL"
        host, _, port_s = netloc.partition(":")
        if ":" in port_s:
            return _slow(url)
    port = None
    if port_s:
        if not port_s.isdigit():
            return _slow(url)  # urlsplit raises for these; let it
        port = int(port_s)
        if port > 65535:
            return _slow(url)
    return SplitURL(scheme.lower(), netloc, host.lower() if host else None, port, path, query)


def quote(s: str) -> str:
    """``urllib.parse.quote(s, safe="")``: every byte outside ``A-Za-z0-9_.-~`` percent-encoded (UTF-8)."""
    if all(c in _UNRESERVED for c in s):
        return s  # node names, namespaces: DNS-1123, nothing to escape
    return "".join(chr(b) if chr(b) in _UNRESERVED else f"%{b:02X}" for b in s.encode("utf-8"))
