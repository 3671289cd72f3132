"""One webhook POST with the semantics of ``requests.post`` (the reference's Slack transport).

The reference posts with ``requests.post(url, json=payload, timeout=10, headers={"Content-Type": ...})``
(``check-gpu-node.py:73-78``), so its webhook inherits everything a default ``requests`` session does.
This module reproduces that on the raw-socket transport (:mod:`..utils.http`), without importing
``requests`` (138 ms) or ``urllib3``:

* **URL preparation** (``PreparedRequest.prepare_url`` over urllib3's ``parse_url``): leading blanks
  stripped; a non-http scheme has no adapter; an authority urllib3 cannot parse (a port above 65535,
  an unclosed IPv6 bracket) is ``Failed to parse: <url>``; no scheme / no host are requests' own
  messages; dot segments are removed and the path and query are re-quoted (``requote_uri``).
* **Credentials** (``trust_env``): a ``~/.netrc`` (or ``$NETRC``) entry for the host wins; otherwise
  the URL's ``user:password@`` (both parts present, percent-decoded) is sent as ``Authorization: Basic``.
* **Headers**, in requests' order: ``User-Agent``, ``Accept-Encoding: gzip, deflate``, ``Accept: */*``,
  ``Connection: keep-alive``, ``Content-Type``, ``Content-Length``, ``Authorization``.  Only the
  ``User-Agent`` value differs (this package names itself, not ``python-requests``).
* **Redirects** (``Session.resolve_redirects``): up to 30 followed, the 31st is ``Exceeded 30 redirects.``;
  301 (for a POST), 302 and 303 become a body-less GET (``Content-Type``/``Content-Length`` dropped),
  307/308 re-POST the same body; relative and scheme-relative ``Location`` values are resolved against
  the current URL and the fragment carried; ``Authorization`` is dropped when the host (or, off the
  default ports, the port or scheme) changes, then re-read from ``.netrc`` for the new URL; cookies a
  redirect sets are sent on later hops (``http.cookiejar``, requests' jar); the proxy and the CA bundle
  are re-chosen for every hop.
* **TLS**: ``REQUESTS_CA_BUNDLE`` / ``CURL_CA_BUNDLE`` (a file or a hashed directory) verify https; a path
  that does not exist is requests' ``Could not find a suitable TLS CA certificate bundle, invalid path``.
* **Response text** (``Response.text``): the ``charset`` of ``Content-Type``; ``text/*`` without one is
  ISO-8859-1 and ``application/json`` UTF-8; otherwise guessed (``charset_normalizer`` when importable).

Every failure is an exception whose ``str()`` is what the reference prints after
``슬랙 메시지 전송 실패: `` (``:98``, ``:103``, ``:108``); :class:`..utils.http.HTTPError` for the
network ones (requests' ``ConnectionError`` / ``Timeout``, which the reference retries on a reset),
:class:`RequestError` for the rest.
"""

from __future__ import annotations

import os
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563)
    from typing import Dict, List, Optional, Tuple

from ..utils.http import HTTPError, Response, env_proxy, request

MAX_REDIRECTS = 30  # requests.models.DEFAULT_REDIRECT_LIMIT
REDIRECT_STATI = (301, 302, 303, 307, 308)
DEFAULT_PORTS = {"http": 80, "https": 443}
ACCEPT_ENCODING = "gzip, deflate"


class RequestError(Exception):
    """A failure requests raises as a ``RequestException`` that is not a connection error (invalid URL,
    too many redirects), or as a plain exception (the CA bundle's ``OSError``): never retried."""


# -- URL preparation (urllib3.util.url.parse_url + requests' prepare_url) ------------------------------------------

_HEX = "[0-9A-Fa-f]{1,4}"
_IPV4 = r"(?:[0-9]{1,3}\.){3}[0-9]{1,3}"
_LS32 = f"(?:{_HEX}:{_HEX}|{_IPV4})"
_IPV6 = "(?:" + "|".join(v.format(h=_HEX, ls32=_LS32) for v in (
    "(?:{h}:){{6}}{ls32}", "::(?:{h}:){{5}}{ls32}", "(?:{h})?::(?:{h}:){{4}}{ls32}",
    "(?:(?:{h}:)?{h})?::(?:{h}:){{3}}{ls32}", "(?:(?:{h}:){{0,2}}{h})?::(?:{h}:){{2}}{ls32}",
    "(?:(?:{h}:){{0,3}}{h})?::{h}:{ls32}", "(?:(?:{h}:){{0,4}}{h})?::{ls32}", "(?:(?:{h}:){{0,5}}{h})?::{h}",
    "(?:(?:{h}:){{0,6}}{h})?::")) + ")"
_UNRESERVED = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789._\\-~"
_ZONE = "(?:%25|%)(?:[" + _UNRESERVED + "]|%[a-fA-F0-9]{2})+"
_HOST_PORT = ("^((?:[^\\[\\]%:/?#]|%[a-fA-F0-9]{2})*|" + _IPV4 + "|\\[" + _IPV6 + "(?:" + _ZONE + ")?\\])"
              "(?::0*?(|0|[1-9][0-9]{0,4}))?$")
_URI = (r"^(?:([a-zA-Z][a-zA-Z0-9+.-]*):)?(?://([^\\/?#]*))?([^?#]*)(?:\?([^#]*))?(?:#(.*))?$")

_UNRESERVED_CHARS = frozenset("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789._-~")
_USERINFO_CHARS = _UNRESERVED_CHARS | frozenset("!$&'()*+,;=:")
_PATH_CHARS = _USERINFO_CHARS | frozenset("@/")
_QUERY_CHARS = _PATH_CHARS | frozenset("?")


def _encode_invalid_chars(component: Optional[str], allowed: frozenset) -> Optional[str]:
    """urllib3's ``_encode_invalid_chars``: upper-case existing escapes, percent-encode the rest (UTF-8)."""
    if not component:
        return component
    import re
    component, n = re.subn(r"%[a-fA-F0-9]{2}", lambda m: m.group(0).upper(), component)
    raw = component.encode("utf-8", "surrogatepass")
    escaped = n == raw.count(b"%")
    out = bytearray()
    for b in raw:
        if (escaped and b == 0x25) or (b < 128 and chr(b) in allowed):
            out.append(b)
        else:
            out += b"%%%02X" % b
    return out.decode()


def _remove_dot_segments(path: str) -> str:
    segments = path.split("/")
    out: List[str] = []
    for seg in segments:
        if seg == ".":
            continue
        if seg != "..":
            out.append(seg)
        elif out:
            out.pop()
    if path.startswith("/") and (not out or out[0]):
        out.insert(0, "")
    if path.endswith(("/.", "/..")):
        out.append("")
    return "/".join(out)


def _unquote_unreserved(uri: str) -> str:
    parts = uri.split("%")
    for i in range(1, len(parts)):
        h = parts[i][0:2]
        if len(h) == 2 and h.isalnum():
            try:
                c = chr(int(h, 16))
            except ValueError:
                raise RequestError(f"Invalid percent-escape sequence: '{h}'")
            parts[i] = c + parts[i][2:] if c in _UNRESERVED_CHARS else f"%{parts[i]}"
        else:
            parts[i] = f"%{parts[i]}"
    return "".join(parts)


def requote_uri(uri: str) -> str:
    """``requests.utils.requote_uri``."""
    from urllib.parse import quote
    try:
        return quote(_unquote_unreserved(uri), safe="!#$%&'()*+,/:;=?@[]~")
    except RequestError:
        return quote(uri, safe="!#$&'()*+,/:;=?@[]~")


_SIMPLE_PATH = _UNRESERVED_CHARS | frozenset("!$&'()*+,;=:/")
_SIMPLE_HOST = frozenset("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789.-")


def _simple(url: str) -> Optional[str]:
    """The prepared form of a plain ``http(s)://host[:port]/path[?query]`` URL -- every webhook URL in
    practice -- without ``re`` or ``urllib.parse`` (~20 ms of a cold Slack send); None for anything else, which
    takes the full urllib3/requests path.  Plain means: no user info, escapes, fragment or dot segments,
    only characters neither urllib3 nor ``requote_uri`` rewrites, a letter-digit-dot-dash host not starting
    with a dot, and a port without leading zeros."""
    low = url[:8].lower()
    if low.startswith("http://"):
        scheme, rest = "http", url[7:]
    elif low.startswith("https://"):
        scheme, rest = "https", url[8:]
    else:
        return None
    cut = len(rest)
    for ch in "/?":
        i = rest.find(ch)
        if i != -1 and i < cut:
            cut = i
    netloc, tail = rest[:cut], rest[cut:]
    path, _, query = tail.partition("?")
    host, colon, port = netloc.partition(":")
    if not host or host[0] == "." or not all(c in _SIMPLE_HOST for c in host):
        return None
    if colon and not (port.isdigit() and port.isascii() and port[0] != "0" and int(port) <= 65535):
        return None
    if not all(c in _SIMPLE_PATH for c in path) or not all(c in _SIMPLE_PATH or c == "?" for c in query):
        return None
    if "/./" in path + "/" or "/../" in path + "/" or path in (".", ".."):
        return None
    return f"{scheme}://{host.lower()}{colon}{port}{path or '/'}{'?' + query if query else ''}"


def prepare_url(url: str) -> str:
    """``PreparedRequest.prepare_url``: the URL requests would send to, or :class:`RequestError` with its
    message.  A URL with a non-http scheme is returned as is (the caller reports the missing adapter)."""
    url = url.lstrip()
    fast = _simple(url)
    if fast is not None:
        return fast
    import re
    if ":" in url and not url.lower().startswith("http"):
        return url
    source = url
    work = url if re.search(r"^(?:[a-zA-Z][a-zA-Z0-9+-]*:|/)", url) else "//" + url
    try:
        m = re.match(_URI, work, re.DOTALL)
        scheme, authority, path, query, fragment = m.groups()  # type: ignore[union-attr]
        normalize = scheme is None or scheme.lower() in ("http", "https")
        scheme = scheme.lower() if scheme else scheme
        auth = host = port = None
        if authority:
            auth, _, host_port = authority.rpartition("@")
            auth = auth or None
            hm = re.match(_HOST_PORT, host_port, re.DOTALL)
            host, port = hm.groups()  # type: ignore[union-attr]
            if auth and normalize:
                auth = _encode_invalid_chars(auth, _USERINFO_CHARS)
            if port == "":
                port = None
        if port is not None and not 0 <= int(port) <= 65535:
            raise ValueError(port)
        if host and scheme in ("http", "https", None) and "%" not in host:
            host = host.lower()
        if normalize and path:
            path = _encode_invalid_chars(_remove_dot_segments(path), _PATH_CHARS)
        if normalize and query:
            query = _encode_invalid_chars(query, _QUERY_CHARS)
        if normalize and fragment:
            fragment = _encode_invalid_chars(fragment, _QUERY_CHARS)
    except (ValueError, AttributeError):
        raise RequestError(f"Failed to parse: {source}")
    if not scheme:
        raise RequestError(f"Invalid URL {url!r}: No scheme supplied. Perhaps you meant https://{url}?")
    if not host:
        raise RequestError(f"Invalid URL {url!r}: No host supplied")
    if not host.isascii():
        try:
            host = host.encode("idna").decode("ascii")
        except UnicodeError:
            raise RequestError("URL has an invalid label.")
    elif host.startswith(("*", ".")):
        raise RequestError("URL has an invalid label.")
    netloc = (auth + "@" if auth else "") + host + (f":{int(port)}" if port and int(port) else "")  # requests' `if port:`
    out = f"{scheme}://{netloc}{path or '/'}"
    if query:
        out += "?" + query
    if fragment:
        out += "#" + fragment
    return requote_uri(out)


# -- credentials --------------------------------------------------------------------------------------------------

def url_auth(url: str) -> Optional[Tuple[str, str]]:
    """``requests.utils.get_auth_from_url``: both user and password must be present (an empty one counts)."""
    if "@" not in url:
        return None
    from urllib.parse import unquote, urlparse
    p = urlparse(url)
    if p.username is None or p.password is None:
        return None
    auth = (unquote(p.username), unquote(p.password))
    return auth if any(auth) else None


def netrc_auth(url: str, environ: Optional[Dict[str, str]] = None) -> Optional[Tuple[str, str]]:
    """``requests.utils.get_netrc_auth``: ``$NETRC``, else ``~/.netrc`` then ``~/_netrc``; unreadable or
    malformed files are skipped silently."""
    env = os.environ if environ is None else environ
    path = env.get("NETRC")
    locations = (path,) if path is not None else ("~/.netrc", "~/_netrc")
    found = None
    for loc in locations:
        full = os.path.expanduser(loc)
        if os.path.exists(full):
            found = full
            break
    if found is None:
        return None
    from urllib.parse import urlparse
    host = urlparse(url).hostname
    try:
        from netrc import netrc
        entry = netrc(found).authenticators(host)
    except Exception:  # NetrcParseError, OSError (permissions): skipped, as requests does
        return None
    if entry and any(entry):
        return (entry[0] if entry[0] else entry[1], entry[2])
    return None


def basic_auth(user: str, password: str) -> str:
    """``requests.auth._basic_auth_str`` (latin-1: a character outside it fails as it does there)."""
    import base64
    return "Basic " + base64.b64encode(user.encode("latin1") + b":" + password.encode("latin1")).decode("ascii")


# -- TLS ----------------------------------------------------------------------------------------------------------

def env_ssl_context(environ: Optional[Dict[str, str]] = None):
    """``REQUESTS_CA_BUNDLE`` / ``CURL_CA_BUNDLE`` (a file or an OpenSSL hashed directory) as requests verifies
    https with; None keeps the default trust store.  A missing path is requests' ``OSError`` text."""
    env = os.environ if environ is None else environ
    bundle = env.get("REQUESTS_CA_BUNDLE") or env.get("CURL_CA_BUNDLE")
    if not bundle:
        return None
    if not os.path.exists(bundle):
        raise RequestError(f"Could not find a suitable TLS CA certificate bundle, invalid path: {bundle}")
    import ssl
    if os.path.isdir(bundle):
        return ssl.create_default_context(capath=bundle)
    return ssl.create_default_context(cafile=bundle)


# -- redirects ----------------------------------------------------------------------------------------------------

def should_strip_auth(old_url: str, new_url: str) -> bool:
    """``Session.should_strip_auth``."""
    from urllib.parse import urlparse
    o, n = urlparse(old_url), urlparse(new_url)
    if o.hostname != n.hostname:
        return True
    if o.scheme == "http" and o.port in (80, None) and n.scheme == "https" and n.port in (443, None):
        return False
    changed_port = o.port != n.port
    changed_scheme = o.scheme != n.scheme
    default = (DEFAULT_PORTS.get(o.scheme), None)
    if not changed_scheme and o.port in default and n.port in default:
        return False
    return changed_port or changed_scheme


def redirect_target(resp: Response) -> Optional[str]:
    loc = resp.header("Location")
    if loc is None or resp.status not in REDIRECT_STATI:
        return None
    return loc.encode("latin-1").decode("utf-8")  # requests' re-decoding of a UTF-8 Location


def next_url(current: str, location: str, fragment: str) -> Tuple[str, str]:
    """The absolute URL a ``Location`` points to from ``current`` (and the fragment carried on)."""
    from urllib.parse import urljoin, urlparse
    if location.startswith("//"):
        location = urlparse(current).scheme + ":" + location
    parsed = urlparse(location)
    if parsed.fragment == "" and fragment:
        parsed = parsed._replace(fragment=fragment)
    elif parsed.fragment:
        fragment = parsed.fragment
    location = parsed.geturl()
    if not parsed.netloc:
        return urljoin(current, requote_uri(location)), fragment
    return requote_uri(location), fragment


class _Cookies:
    """The cookies redirect responses set, kept and sent the way requests' ``RequestsCookieJar`` does (the
    stdlib ``http.cookiejar`` policy over urllib-shaped request/response stand-ins)."""

    def __init__(self) -> None:
        from http.cookiejar import CookieJar
        self.jar = CookieJar()

    def extract(self, url: str, resp: Response) -> None:
        import email.message
        import urllib.request
        msg = email.message.Message()
        for k, v in resp.headers:
            msg[k] = v

        class _R:
            def info(self):
                return msg
        self.jar.extract_cookies(_R(), urllib.request.Request(url))  # type: ignore[arg-type]

    def header(self, url: str) -> Optional[str]:
        import urllib.request
        r = urllib.request.Request(url)
        self.jar.add_cookie_header(r)
        return r.get_header("Cookie")


# -- the POST -----------------------------------------------------------------------------------------------------

def _target(url: str) -> str:
    """Where the transport connects: the prepared URL without user info (urllib3 never sends it)."""
    if "@" not in url:
        return url
    from urllib.parse import urlsplit, urlunsplit
    p = urlsplit(url)
    if "@" not in p.netloc:
        return url
    return urlunsplit((p.scheme, p.netloc.rpartition("@")[2], p.path, p.query, ""))


def post(url: str, body: bytes, content_type: str = "application/json", timeout: float = 10.0,
         user_agent: str = "k8s-gpu-node-checker-amd/0.1", environ: Optional[Dict[str, str]] = None,
         ssl_context=None) -> Response:
    """``requests.post(url, data=body, timeout=timeout, headers={"Content-Type": content_type})``: the final
    response after redirects.  Raises :class:`HTTPError` (connection errors / timeouts) or
    :class:`RequestError`."""
    env = os.environ if environ is None else environ
    prepared = prepare_url(url)
    if not prepared.lower().startswith(("http://", "https://")):
        raise RequestError(f"No connection adapters were found for {prepared!r}")
    headers: Dict[str, str] = {"User-Agent": user_agent, "Accept-Encoding": ACCEPT_ENCODING, "Accept": "*/*",
                               "Connection": "keep-alive", "Content-Type": content_type,
                               "Content-Length": str(len(body))}
    auth = netrc_auth(prepared, env) or url_auth(prepared)
    if auth:
        headers["Authorization"] = basic_auth(*auth)
    method: str = "POST"
    data: Optional[bytes] = body
    fragment = prepared.partition("#")[2]
    cookies: Optional[_Cookies] = None
    current = prepared
    redirects = 0
    while True:
        ctx = ssl_context
        if ctx is None and current.lower().startswith("https"):
            ctx = env_ssl_context(env)
        target = _target(current)
        resp = request(target, method, headers, data, timeout=timeout, ssl_context=ctx,
                       proxy_url=env_proxy(target, env))
        location = redirect_target(resp)
        if location is None:
            return resp
        redirects += 1
        if redirects > MAX_REDIRECTS:
            raise RequestError(f"Exceeded {MAX_REDIRECTS} redirects.")
        new, fragment = next_url(current, location, fragment)
        if resp.status == 303 and method != "HEAD":
            method = "GET"
        if resp.status == 302 and method != "HEAD":
            method = "GET"
        if resp.status == 301 and method == "POST":
            method = "GET"
        if resp.status not in (307, 308):
            for h in ("Content-Length", "Content-Type", "Transfer-Encoding"):
                headers.pop(h, None)
            data = None
        headers.pop("Cookie", None)
        if resp.header("Set-Cookie") is not None or cookies is not None:
            cookies = cookies or _Cookies()
            cookies.extract(_target(current), resp)
            c = cookies.header(_target(new))
            if c:
                headers["Cookie"] = c
        if "Authorization" in headers and should_strip_auth(current, new):
            del headers["Authorization"]
        again = netrc_auth(new, env)
        if again:
            headers["Authorization"] = basic_auth(*again)
        current = new


def response_text(resp: Response) -> str:
    """``requests.Response.text``."""
    if not resp.body:
        return ""
    enc = _encoding_from_headers(resp.header("Content-Type"))
    if enc is None:
        enc = _apparent_encoding(resp.body)
    try:
        return str(resp.body, enc, errors="replace")
    except (LookupError, TypeError):
        return str(resp.body, errors="replace")


def _encoding_from_headers(content_type: Optional[str]) -> Optional[str]:
    if not content_type:
        return None
    parts = content_type.split(";")
    ctype = parts[0].strip()
    params: Dict[str, str] = {}
    for p in parts[1:]:
        p = p.strip()
        if p:
            k, sep, v = p.partition("=")
            params[k.strip(" '\"").lower()] = v.strip(" '\"") if sep else True  # type: ignore[assignment]
    if "charset" in params and isinstance(params["charset"], str):
        return params["charset"].strip("'\"")
    if "text" in ctype:
        return "ISO-8859-1"
    if "application/json" in ctype:
        return "utf-8"
    return None


def _apparent_encoding(body: bytes) -> Optional[str]:
    try:
        import charset_normalizer
        return charset_normalizer.detect(body)["encoding"]
    except ImportError:
        try:
            body.decode("utf-8")
            return "utf-8"
        except UnicodeDecodeError:
            return "ISO-8859-1"
