"""Minimal HTTP/1.1 client on raw sockets (+ ``ssl``): the checker's only transport.

Why not ``requests``/``urllib3``/``aiohttp``: at 1-16 nodes the reference's
process wall clock is ~95 % interpreter + import cost (``import
requests`` 138 ms, ``aiohttp`` 310 ms).  This module imports only ``_socket``
(and ``ssl`` for https, ``zlib`` for gzip) and reads bodies with
``recv_into`` a pre-sized buffer, so a 5.9 MB NodeList is one allocation.

Features: keep-alive connection reuse, ``Content-Length`` / chunked /
close-delimited bodies, ``gzip`` content coding, connect/read timeouts, an
HTTP ``CONNECT`` proxy for https and absolute-form requests for http proxies.

Errors are :class:`HTTPError` with a ``kind`` (``refused``, ``reset``,
``aborted``, ``timeout``, ``connect_timeout``, ``dns``, ``tls``,
``protocol``) and a message shaped like the one ``requests`` prints for the
same failure, because the reference's Slack retry policy keys on that text
(``check-gpu-node.py:88``).
"""

from __future__ import annotations

import _socket  # the C module: socket.py's enum setup costs ~2 ms of a 1-node cold start
import errno
import os
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Dict, List, Optional, Tuple

from .urls import split as urlsplit

_DEFAULT_PORTS = {"http": 80, "https": 443}


class HTTPError(Exception):
    def __init__(self, kind: str, message: str, cause: Optional[BaseException] = None):
        super().__init__(message)
        self.kind = kind
        self.cause = cause

    @property
    def retryable_reset(self) -> bool:
        """Matches the reference's "Connection reset by peer" / "Connection aborted" test."""
        return self.kind in ("reset", "aborted")


class Response:
    __slots__ = ("status", "reason", "headers", "body")

    def __init__(self, status: int, reason: str, headers: List[Tuple[str, str]], body: bytes):
        self.status = status
        self.reason = reason
        self.headers = headers
        self.body = body

    def header(self, name: str, default: Optional[str] = None) -> Optional[str]:
        name = name.lower()
        for k, v in self.headers:
            if k.lower() == name:
                return v
        return default

    def header_dict(self) -> Dict[str, str]:
        return {k: v for k, v in self.headers}

    @property
    def text(self) -> str:
        return self.body.decode("utf-8", "replace")


class _Shown:
    """An object whose repr is the given text (an exception as urllib3 nests it inside a tuple's str)."""
    __slots__ = ("text",)

    def __init__(self, text: str):
        self.text = text

    def __repr__(self) -> str:
        return self.text


def nodelay(sock: Any) -> None:
    """``TCP_NODELAY`` on a connection one of our HTTP servers accepted (``setup()`` of the agent's and the watcher's
    handlers).  ``BaseHTTPRequestHandler`` writes a response's head and body separately; with Nagle on, the body
    waits for the client's ACK of the head, and a keep-alive client past its first exchanges (a Prometheus scraper)
    delays that ACK by up to 40 ms."""
    try:
        sock.setsockopt(_socket.IPPROTO_TCP, _socket.TCP_NODELAY, 1)
    except (OSError, AttributeError):  # not a TCP socket (a test's socketpair)
        pass


def _broken(inner: str) -> str:
    """urllib3's ``ProtocolError(f"Connection broken: {e!r}", e)`` as requests prints it (a body cut short or
    malformed after the head arrived: not a connection error, never retried by the reference)."""
    return str((f"Connection broken: {inner}", _Shown(inner)))


def _aborted(inner: str) -> HTTPError:
    """urllib3's ``ProtocolError('Connection aborted.', e)`` for a head http.client refused."""
    return HTTPError("aborted", f"('Connection aborted.', {inner})")


_MAXLINE = 65536   # http.client's limits on a status / header line (bytes, CRLF included) and on header lines
_MAXHEADERS = 100
_CRLF = b"\r\n"


def _pool_name(scheme: str, host: str, port: int) -> str:
    pool = "HTTPSConnectionPool" if scheme == "https" else "HTTPConnectionPool"
    return f"{pool}(host='{host}', port={port})"


def _connect(target: Tuple[Optional[str], int], timeout: float, plain: bool = True) -> "socket.socket":
    """``socket.create_connection`` without the ``getaddrinfo`` round for IPv4 literals.

    A plain-TCP connection to an IPv4 literal (a mock or in-cluster service IP over http) uses a bare
    ``_socket.socket``; names, IPv6 and anything TLS wraps (``ssl`` wants a ``socket.socket``) go
    through the ``socket`` module, imported then."""
    host, port = target
    if host and host.count(".") == 3 and host.replace(".", "").isdigit():
        if plain:
            sock = _socket.socket(_socket.AF_INET, _socket.SOCK_STREAM)
        else:
            import socket
            sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        try:
            sock.settimeout(timeout)
            sock.connect((host, port))
            return sock
        except BaseException:
            sock.close()
            raise
    import socket
    return socket.create_connection((host, port), timeout=timeout)


class Connection:
    """One persistent HTTP/1.1 connection to ``scheme://host:port``."""

    def __init__(self, url: str, timeout: float = 30.0, ssl_context=None, server_hostname: Optional[str] = None,
                 proxy_url: Optional[str] = None, tracer=None):
        #: ``utils.timing.Tracer`` (or None): :meth:`request` adds ``connect`` (TCP + TLS), ``first_byte`` (request
        #: sent to response head read) and ``body`` (the rest of the response read)
        self.tracer = tracer
        parts = urlsplit(url)
        self.scheme = parts.scheme or "http"
        self.host = parts.hostname or "localhost"
        self.port = parts.port or _DEFAULT_PORTS.get(self.scheme, 80)
        self.base_path = parts.path.rstrip("/")
        self.timeout = timeout
        self.ssl_context = ssl_context
        self.server_hostname = server_hostname or self.host
        self.proxy = urlsplit(proxy_url) if proxy_url else None
        self.sock: Optional["socket.socket"] = None
        self._buf = bytearray()
        host_hdr = self.host if ":" not in self.host else f"[{self.host}]"
        if self.port != _DEFAULT_PORTS.get(self.scheme):
            host_hdr += f":{self.port}"
        self.host_header = host_hdr

    # -- connection management ------------------------------------------------
    def _fail(self, kind: str, url: str, e: BaseException) -> HTTPError:
        pool = _pool_name(self.scheme, self.host, self.port)
        if kind in ("reset", "aborted"):
            msg = f"('Connection aborted.', {e!r})"
        elif kind == "timeout":
            msg = f"{pool}: Read timed out. (read timeout={self.timeout:g})"
        elif kind == "connect_timeout":
            msg = (f"{pool}: Max retries exceeded with url: {url} (Caused by ConnectTimeoutError("
                   f"'Connection to {self.host} timed out. (connect timeout={self.timeout:g})'))")
        elif kind in ("refused", "dns"):
            # urllib3 2.6's text (the reference's requests stack as installed): the connection renders as
            # HTTP[S]Connection(host=..., port=...); a failed lookup is a NameResolutionError
            conn = f"{'HTTPSConnection' if self.scheme == 'https' else 'HTTPConnection'}(host={self.host!r}, port={self.port!r})"
            if kind == "dns":
                inner = f"NameResolutionError({conn + ': ' + f'Failed to resolve {self.host!r} ({e})'!r})"
            else:
                inner = f"NewConnectionError({conn + ': Failed to establish a new connection: ' + str(e)!r})"
            msg = f"{pool}: Max retries exceeded with url: {url} (Caused by {inner})"
        elif kind == "tls":
            msg = f"{pool}: Max retries exceeded with url: {url} (Caused by SSLError({e!r}))"
        else:
            msg = f"{pool}: {e}"
        return HTTPError(kind, msg, e)

    def connect(self, url: str = "/") -> None:
        if self.sock is not None:
            return
        target = (self.proxy.hostname, self.proxy.port or 80) if self.proxy else (self.host, self.port)
        try:
            sock = _connect(target, self.timeout, plain=self.scheme != "https")
        except _socket.timeout as e:
            raise self._fail("connect_timeout", url, e) if not self.proxy else self._proxy_down("connect_timeout", url, e)
        except _socket.gaierror as e:
            raise self._fail("dns", url, e) if not self.proxy else self._proxy_down("dns", url, e)
        except ConnectionRefusedError as e:
            raise self._fail("refused", url, e) if not self.proxy else self._proxy_down("refused", url, e)
        except OSError as e:
            kind = "refused" if e.errno in (errno.ECONNREFUSED, errno.EHOSTUNREACH, errno.ENETUNREACH) else "aborted"
            raise self._fail(kind, url, e) if not self.proxy or kind == "aborted" else self._proxy_down(kind, url, e)
        sock.setsockopt(_socket.IPPROTO_TCP, _socket.TCP_NODELAY, 1)
        handshake = False
        try:
            if self.proxy and self.scheme == "https":
                self._tunnel(sock, url)
            if self.scheme == "https":
                ctx = self.ssl_context
                if ctx is None:
                    import ssl
                    ctx = ssl.create_default_context()
                handshake = True
                sock = ctx.wrap_socket(sock, server_hostname=self.server_hostname)
        except HTTPError:
            sock.close()
            raise
        except _socket.timeout as e:
            sock.close()
            # a peer that never answers the handshake (a plain-HTTP port, a black hole): urllib3 reports the
            # handshake's socket timeout as a read timeout
            raise self._fail("timeout" if handshake else "tls", url, e)
        except OSError as e:
            sock.close()
            raise self._fail("tls", url, e)
        self.sock = sock
        self._buf = bytearray()

    def _proxy_auth(self) -> str:
        """``Proxy-Authorization: Basic ...`` line for a proxy URL with credentials (requests does the same)."""
        if self.proxy is None or self.proxy.username is None:
            return ""
        import base64
        cred = f"{self.proxy.username}:{self.proxy.password or ''}".encode("latin-1")
        return f"Proxy-Authorization: Basic {base64.b64encode(cred).decode('ascii')}\r\n"

    def _proxy_error(self, url: str, inner: str) -> HTTPError:
        """urllib3's MaxRetryError(ProxyError('Unable to connect to proxy', e)) text, as requests prints it."""
        pool = _pool_name(self.scheme, self.host, self.port)
        return HTTPError("proxy", f"{pool}: Max retries exceeded with url: {url} (Caused by ProxyError('Unable to "
                                  f"connect to proxy', {inner}))")

    def _proxy_down(self, kind: str, url: str, e: BaseException) -> HTTPError:
        """The proxy itself unreachable, as urllib3 words it: ``ProxyError('Unable to connect to proxy', <the
        connection error naming the proxy>)``, under the target's pool for a tunnel (https) and under the proxy's
        own pool, with the absolute URL, for a forwarded http request."""
        assert self.proxy is not None
        phost, pport = self.proxy.hostname or "", self.proxy.port or 80
        conn = f"{'HTTPSConnection' if self.scheme == 'https' else 'HTTPConnection'}(host={phost!r}, port={pport!r})"
        if kind == "dns":
            inner = f"NameResolutionError({conn + ': ' + f'Failed to resolve {phost!r} ({e})'!r})"
        elif kind == "connect_timeout":
            inner = (f"ConnectTimeoutError({conn!r}, 'Connection to {phost} timed out. (connect timeout="
                     f"{self.timeout:g})')")
        else:
            inner = f"NewConnectionError({conn + ': Failed to establish a new connection: ' + str(e)!r})"
        if self.scheme == "https":
            return self._proxy_error(url, inner)
        pool = _pool_name("http", phost, pport)
        return HTTPError("proxy", f"{pool}: Max retries exceeded with url: http://{self.host_header}{self.base_path}"
                                  f"{url} (Caused by ProxyError('Unable to connect to proxy', {inner}))")

    def _tunnel(self, sock: "socket.socket", url: str = "/") -> None:
        req = (f"CONNECT {self.host}:{self.port} HTTP/1.1\r\nHost: {self.host}:{self.port}\r\n"
               f"{self._proxy_auth()}\r\n").encode("latin-1")
        sock.sendall(req)
        data = b""
        while b"\r\n\r\n" not in data:
            chunk = sock.recv(4096)
            if not chunk:
                raise self._proxy_error(url, "RemoteDisconnected('Remote end closed connection without response')")
            data += chunk
        first = data.split(b"\r\n", 1)[0]
        status = first.split(None, 2)
        code = int(status[1]) if len(status) >= 2 and status[1].isdigit() else 0
        if code != 200:
            # http.client's _tunnel: OSError("Tunnel connection failed: <code> <reason>")
            reason = status[2].decode("latin-1").strip() if len(status) > 2 else ""
            raise self._proxy_error(url, repr(OSError(f"Tunnel connection failed: {code} {reason}")))

    def close(self) -> None:
        if self.sock is not None:
            try:
                self.sock.close()
            except OSError:
                pass
            self.sock = None

    # -- request/response -----------------------------------------------------
    def _recv_more(self) -> bool:
        assert self.sock is not None
        chunk = self.sock.recv(262144)
        if not chunk:
            return False
        self._buf += chunk
        return True

    def _read_exact(self, n: int):
        buf = self._buf
        if len(buf) >= n:
            out = bytes(buf[:n])
            del buf[:n]
            return out
        out = bytearray(n)
        view = memoryview(out)
        have = len(buf)
        view[:have] = buf
        self._buf = bytearray()
        sock = self.sock
        assert sock is not None
        while have < n:
            got = sock.recv_into(view[have:], n - have)
            if not got:
                raise HTTPError("incomplete", _broken(f"IncompleteRead({have} bytes read, {n - have} more expected)"))
            have += got
        return out  # bytearray: json.loads and the native scanner take it without a copy

    def _read_line(self) -> bytes:
        while True:
            i = self._buf.find(b"\r\n")
            if i >= 0:
                line = bytes(self._buf[:i])
                del self._buf[:i + 2]
                return line
            if not self._recv_more():
                raise HTTPError("aborted", "('Connection aborted.', RemoteDisconnected("
                                           "'Remote end closed connection without response'))")

    def _encode(self, method: str, path: str, headers: Optional[Dict[str, str]], body: Optional[bytes]) -> bytes:
        req_target = self.base_path + path
        if self.proxy and self.scheme == "http":
            req_target = f"http://{self.host_header}{req_target}"
        lines = [f"{method} {req_target} HTTP/1.1", f"Host: {self.host_header}"]
        if self.proxy and self.scheme == "http" and self.proxy.username is not None:
            lines.append(self._proxy_auth().rstrip("\r\n"))
        given_length = False
        for k, v in (headers or {}).items():
            lines.append(f"{k}: {v}")
            given_length = given_length or k.lower() == "content-length"
        if body is not None and not given_length:
            lines.append(f"Content-Length: {len(body)}")
        raw = ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1")
        return raw + body if body else raw

    def send_only(self, method: str, path: str, headers: Optional[Dict[str, str]] = None,
                  body: Optional[bytes] = None) -> None:
        """Send a request now and read its response later with :meth:`read_pending` (pipelining)."""
        try:
            self.connect(path)
            assert self.sock is not None
            self.sock.sendall(self._encode(method, path, headers, body))
        except HTTPError:
            self.close()
            raise
        except OSError as e:
            self.close()
            raise self._fail("aborted", path, e)

    def read_pending(self, method: str = "GET", path: str = "/", peek=None) -> Response:
        try:
            return self._read_response(method, peek)
        except HTTPError:
            self.close()
            raise
        except _socket.timeout as e:
            self.close()
            raise self._fail("timeout", path, e)
        except OSError as e:
            self.close()
            raise self._fail("reset" if isinstance(e, ConnectionResetError) else "aborted", path, e)

    def request(self, method: str, path: str, headers: Optional[Dict[str, str]] = None,
                body: Optional[bytes] = None, peek=None) -> Response:
        """Send and read one request.  ``peek(prefix)`` is called once with the first bytes of the
        (decoded) body before the rest is read -- the kube client uses it to pipeline pagination."""
        url = path
        raw = self._encode(method, path, headers, body)
        reused = self.sock is not None
        try:
            tr = self.tracer
            if tr is not None:
                return self._traced(tr, method, url, raw, peek)
            self.connect(url)
            assert self.sock is not None
            self.sock.sendall(raw)
            return self._read_response(method, peek)
        except HTTPError as e:
            self.close()
            if reused and e.kind in ("aborted", "reset"):
                # stale keep-alive socket: one transparent reconnect (idempotent callers only)
                self.connect(url)
                assert self.sock is not None
                self.sock.sendall(raw)
                return self._read_response(method, peek)
            raise
        except _socket.timeout as e:
            self.close()
            raise self._fail("timeout", url, e)
        except ConnectionResetError as e:
            self.close()
            raise self._fail("reset", url, e)
        except (BrokenPipeError, ConnectionAbortedError) as e:
            self.close()
            raise self._fail("aborted", url, e)
        except OSError as e:
            self.close()
            if e.__class__.__name__.startswith("SSL"):
                raise self._fail("tls", url, e)
            raise self._fail("aborted", url, e)

    def _traced(self, tr, method: str, url: str, raw: bytes, peek) -> Response:
        """:meth:`request`'s send and read with its three spans recorded on ``tr``."""
        from time import perf_counter
        t0 = perf_counter()
        self.connect(url)
        t1 = perf_counter()
        assert self.sock is not None
        self.sock.sendall(raw)
        status, reason, headers, hmap = self._read_head()
        t2 = perf_counter()
        resp = self._finish_body(method, status, reason, headers, hmap, peek)
        t3 = perf_counter()
        tr.add("connect", t1 - t0)
        tr.add("first_byte", t2 - t1)
        tr.add("body", t3 - t2)
        return resp

    def _peek_prefix(self, want: int, gz: bool, peek) -> None:
        """Buffer up to ``want`` body bytes (Content-Length bodies) and hand them to ``peek``."""
        while len(self._buf) < want and self._recv_more():
            pass
        prefix = bytes(self._buf[:want])
        if gz:
            import zlib
            try:
                prefix = zlib.decompressobj(16 + zlib.MAX_WBITS).decompress(prefix, 65536)
            except zlib.error:
                return
        peek(prefix)

    def _read_head(self) -> Tuple[int, str, List[Tuple[str, str]], Dict[str, str]]:
        while True:
            # the whole header block at once (one find for its end, one split) rather than line by line
            buf = self._buf
            end = buf.find(b"\r\n\r\n")
            while end < 0:
                seen = len(buf)
                if not self._recv_more():
                    raise HTTPError("aborted", "('Connection aborted.', RemoteDisconnected("
                                               "'Remote end closed connection without response'))")
                buf = self._buf
                end = buf.find(b"\r\n\r\n", max(0, seen - 3))
            lines = bytes(buf[:end]).split(b"\r\n")
            del buf[:end + 4]
            status_line = lines[0]
            # http.client's checks, with its exceptions' text (urllib3 reports them as 'Connection aborted.')
            if len(status_line) + 2 > _MAXLINE:
                raise _aborted("LineTooLong('got more than 65536 bytes when reading status line')")
            parts = status_line.split(None, 2)
            status = 0
            if len(parts) >= 2 and parts[0].startswith(b"HTTP/"):
                try:
                    status = int(parts[1])
                except ValueError:
                    status = 0
            if not 100 <= status <= 999:
                shown = (status_line + _CRLF).decode("latin-1")
                raise _aborted(f"BadStatusLine({shown!r})")
            reason = parts[2].decode("latin-1") if len(parts) > 2 else ""
            if len(lines) > _MAXHEADERS:  # header lines + the blank one ending the head > 100 (lines[0]: status)
                raise _aborted(f"HTTPException('got more than {_MAXHEADERS} headers')")
            headers: List[Tuple[str, str]] = []
            hmap: Dict[str, str] = {}
            for line in lines[1:]:
                if len(line) + 2 > _MAXLINE:
                    raise _aborted("LineTooLong('got more than 65536 bytes when reading header line')")
                k, _, v = line.partition(b":")
                k, v = k.decode("latin-1").strip(), v.decode("latin-1").strip()
                headers.append((k, v))
                kl = k.lower()
                if kl == "content-length" and kl in hmap:
                    hmap[kl] += ", " + v  # urllib3's HTTPHeaderDict joins repeats; unmatching ones are refused
                else:
                    hmap[kl] = v
            if 100 <= status < 200 and status != 101:
                continue  # 100-continue / 103 early hints: read the real response
            return status, reason, headers, hmap

    def open_stream(self, method: str, path: str, headers: Optional[Dict[str, str]] = None,
                    read_timeout: Optional[float] = None) -> "Response | LineStream":
        """Send a request whose 2xx body is a stream of newline-delimited records (a kube watch).

        Returns a :class:`LineStream` for 2xx responses, else the complete :class:`Response`.
        ``read_timeout`` replaces the connection timeout for the stream's reads.
        """
        try:
            self.connect(path)
            assert self.sock is not None
            self.sock.sendall(self._encode(method, path, headers, None))
            status, reason, hdrs, hmap = self._read_head()
            if not 200 <= status < 300:
                return self._finish_body(method, status, reason, hdrs, hmap, None)
        except HTTPError:
            self.close()
            raise
        except _socket.timeout as e:
            self.close()
            raise self._fail("timeout", path, e)
        except OSError as e:
            self.close()
            raise self._fail("reset" if isinstance(e, ConnectionResetError) else "aborted", path, e)
        if read_timeout is not None:
            self.sock.settimeout(read_timeout)
        return LineStream(self, status, reason, hdrs, hmap, path)

    def _read_response(self, method: str, peek=None) -> Response:
        status, reason, headers, hmap = self._read_head()
        return self._finish_body(method, status, reason, headers, hmap, peek)

    def _finish_body(self, method: str, status: int, reason: str, headers: List[Tuple[str, str]],
                     hmap: Dict[str, str], peek) -> Response:
        try:
            return self._body_of(method, status, reason, headers, hmap, peek)
        except _socket.timeout:
            raise
        except OSError as e:
            # the head arrived, the body did not (a reset or abort mid-body): urllib3's ProtocolError("Connection
            # broken: ...") that requests raises as ChunkedEncodingError -- a RequestException, not a ConnectionError,
            # so the reference does not retry it (a server that processed the POST is not sent it twice)
            self.close()
            raise HTTPError("incomplete", _broken(repr(e)))

    def _body_of(self, method: str, status: int, reason: str, headers: List[Tuple[str, str]],
                 hmap: Dict[str, str], peek) -> Response:
        if method == "HEAD" or status in (204, 304):
            body = b""
        elif "chunked" in hmap.get("transfer-encoding", "").lower():
            body = self._read_chunked(peek if 200 <= status < 300 else None,
                                      hmap.get("content-encoding", "").lower() == "gzip")
        elif "content-length" in hmap and (n := _content_length(hmap["content-length"])) is not None:
            if peek is not None and 200 <= status < 300 and n > 0:
                self._peek_prefix(min(n, 4096), hmap.get("content-encoding", "").lower() == "gzip", peek)
            body = self._read_exact(n)
        else:
            chunks = [bytes(self._buf)]
            self._buf = bytearray()
            assert self.sock is not None
            while True:
                c = self.sock.recv(262144)
                if not c:
                    break
                chunks.append(c)
            body = b"".join(chunks)
            self.close()
        coding = hmap.get("content-encoding", "").lower()
        if coding and body:
            body = _decode_content(body, coding)
        if hmap.get("connection", "").lower() == "close":
            self.close()
        return Response(status, reason, headers, body)

    def _read_chunked(self, peek=None, gz: bool = False) -> bytes:
        out = []
        have = 0
        while True:
            try:
                size_line = self._read_line()
            except HTTPError as e:
                if e.kind == "aborted":  # urllib3: the body ended where a chunk size was due
                    raise HTTPError("incomplete", "Response ended prematurely")
                raise
            try:
                size = int(size_line.split(b";", 1)[0].strip() or b"0", 16)
            except ValueError:
                got = (size_line + b"\r\n").split(b";", 1)[0]
                raise HTTPError("incomplete", _broken(f"InvalidChunkLength(got length {got!r}, {have} bytes read)"))
            if size == 0:
                while self._read_line():  # trailers
                    pass
                if peek is not None and out:
                    peek(b"".join(out)[:4096] if not gz else b"")
                return b"".join(out)
            out.append(self._read_exact(size))
            have += size
            self._read_line()
            if peek is not None and have >= 4096:
                prefix = b"".join(out)[:65536]
                if gz:
                    import zlib
                    try:
                        prefix = zlib.decompressobj(16 + zlib.MAX_WBITS).decompress(prefix, 65536)
                    except zlib.error:
                        prefix = b""
                if prefix:
                    peek(prefix)
                peek = None


def _content_length(value: str) -> Optional[int]:
    """urllib3's reading of Content-Length: repeats must agree (else ``InvalidHeader``), a value that is not a
    non-negative integer means none (the body runs to the close)."""
    if "," not in value:
        try:
            n = int(value)
        except ValueError:
            return None
        return n if n >= 0 else None
    try:
        lengths = {int(v) for v in value.split(",")}
    except ValueError:
        return None
    if len(lengths) > 1:
        raise HTTPError("protocol", f"Content-Length contained multiple unmatching values ({value})")
    n = lengths.pop()
    return n if n >= 0 else None


def _decode_content(body: bytes, coding: str) -> bytes:
    """Undo ``Content-Encoding`` as urllib3 does: ``gzip`` (and ``x-gzip``), ``deflate`` (zlib-wrapped, or raw
    as some servers send it), several codings applied in order listed; an unknown coding is left alone."""
    import zlib
    for c in reversed([c.strip() for c in coding.split(",") if c.strip()]):
        try:
            if c in ("gzip", "x-gzip"):
                body = zlib.decompress(body, 16 + zlib.MAX_WBITS)
            elif c == "deflate":
                try:
                    body = zlib.decompress(body)
                except zlib.error:
                    body = zlib.decompress(body, -zlib.MAX_WBITS)
        except zlib.error as e:
            # urllib3's DecodeError (requests' ContentDecodingError) and its text; not a connection error
            raise HTTPError("decode", str((f"Received response with content-encoding: {c}, but failed to decode it.",
                                           e)), e)
    return body


class LineStream:
    """The body of a streaming 2xx response, read record by record (``\n``-terminated lines).

    Handles chunked, ``Content-Length`` and close-delimited bodies and gzip.  :meth:`next_line`
    returns ``None`` when nothing arrived within the read timeout (the stream stays usable: the
    decoder state lives in buffers, nothing is lost) and raises ``EOFError`` at the end.
    """

    def __init__(self, conn: Connection, status: int, reason: str, headers: List[Tuple[str, str]],
                 hmap: Dict[str, str], path: str):
        self.conn = conn
        self.status = status
        self.reason = reason
        self.headers = headers
        self.path = path
        self._chunked = "chunked" in hmap.get("transfer-encoding", "").lower()
        self._left = int(hmap["content-length"]) if (not self._chunked and "content-length" in hmap) else -1
        self._chunk_left = 0       # bytes of the current chunk still to take from the wire buffer
        self._need_size = True     # chunked: expecting a size line next
        self._done = False
        self._body = bytearray()   # decoded body bytes not yet returned as lines
        self._inflate = None
        if hmap.get("content-encoding", "").lower() == "gzip":
            import zlib
            self._inflate = zlib.decompressobj(16 + zlib.MAX_WBITS)

    def _feed(self, data: bytes) -> None:
        self._body += self._inflate.decompress(data) if self._inflate is not None else data

    def _drain_wire(self) -> None:
        """Move every complete piece of the wire buffer into the decoded body buffer."""
        buf = self.conn._buf
        if not self._chunked:
            take = len(buf) if self._left < 0 else min(len(buf), self._left)
            if take:
                self._feed(bytes(buf[:take]))
                del buf[:take]
                if self._left >= 0:
                    self._left -= take
            if self._left == 0:
                self._done = True
            return
        while not self._done:
            if self._need_size:
                i = buf.find(b"\r\n")
                if i < 0:
                    return
                size = int(bytes(buf[:i]).split(b";", 1)[0].strip() or b"0", 16)
                del buf[:i + 2]
                if size == 0:
                    self._done = True  # trailers (if any) are left unread; the stream is closed after
                    return
                self._chunk_left = size
                self._need_size = False
            take = min(len(buf), self._chunk_left)
            if take:
                self._feed(bytes(buf[:take]))
                del buf[:take]
                self._chunk_left -= take
            if self._chunk_left:
                return
            if len(buf) < 2:
                return
            del buf[:2]  # CRLF after the chunk
            self._need_size = True

    def next_line(self) -> Optional[bytes]:
        while True:
            i = self._body.find(b"\n")
            if i >= 0:
                line = bytes(self._body[:i])
                del self._body[:i + 1]
                if line.strip():
                    return line
                continue
            if self._done:
                if self._body.strip():
                    line = bytes(self._body)
                    self._body = bytearray()
                    return line
                raise EOFError
            self._drain_wire()
            if self._body.find(b"\n") >= 0 or self._done:
                continue
            try:
                got = self.conn._recv_more()
            except _socket.timeout:
                return None
            except OSError as e:
                self.conn.close()
                raise self.conn._fail("reset" if isinstance(e, ConnectionResetError) else "aborted", self.path, e)
            if not got:
                if self._chunked or self._left > 0:
                    self.conn.close()
                    raise HTTPError("aborted", "('Connection aborted.', RemoteDisconnected("
                                               "'Remote end closed connection without response'))")
                self._done = True

    def close(self) -> None:
        self.conn.close()


def env_proxy(url: str, environ: Optional[Dict[str, str]] = None) -> Optional[str]:
    """The proxy ``requests`` would use for ``url`` from the environment (``trust_env``; the reference's
    Slack POST goes through it, ``check-gpu-node.py:73``):

    * ``<scheme>_proxy`` then ``all_proxy``, the lower-case spelling winning over the upper-case one
      (``urllib.request.getproxies``); ``HTTP_PROXY`` is ignored under CGI (``REQUEST_METHOD`` set),
      ``http_proxy`` is not;
    * ``no_proxy`` bypasses: ``*``; for an IPv4 host an exact address or a CIDR block; otherwise a
      suffix of the host or of ``host:port`` (so ``example.com`` and ``.example.com`` both match
      ``hooks.example.com``);
    * a proxy given without a scheme is ``http://``.
    """
    env = os.environ if environ is None else environ
    parts = urlsplit(url)
    host = parts.hostname
    if not host:
        return None
    # urllib.request.getproxies_environment: every *_proxy (any case), then the "_proxy"-suffixed
    # spellings again, which win (an empty one removes the entry)
    proxies: Dict[str, str] = {}
    for k, v in env.items():
        if v and k.lower().endswith("_proxy"):
            proxies[k[:-6].lower()] = v
    if "REQUEST_METHOD" in env:  # CGI: HTTP_PROXY may come from a client header (CVE-2016-1000110)
        proxies.pop("http", None)
    for k, v in env.items():
        if k.endswith("_proxy"):
            if v:
                proxies[k[:-6].lower()] = v
            else:
                proxies.pop(k[:-6].lower(), None)
    # requests.utils.should_bypass_proxies, part 1: its own no_proxy lookup and suffix / IP / CIDR test
    no_proxy = env.get("no_proxy") or env.get("NO_PROXY")
    if no_proxy:
        entries = [h for h in no_proxy.replace(" ", "").split(",") if h]
        if _is_ipv4(host):
            for e in entries:
                if ("/" in e and _in_cidr(host, e)) or host == e:
                    return None
        else:
            host_port = f"{host}:{parts.port}" if parts.port else host
            if any(host.endswith(e) or host_port.endswith(e) for e in entries):
                return None
    # part 2: urllib.request.proxy_bypass_environment(hostname) over the merged "no" entry ('*', or a
    # name that is the host or a parent domain of it)
    merged_no = proxies.pop("no", None)
    if merged_no:
        if merged_no == "*":
            return None
        h = host.lower()
        for name in (n.strip() for n in merged_no.split(",")):
            name = name.lstrip(".").lower()
            if name and (h == name or h.endswith("." + name)):
                return None
    proxy = proxies.get(parts.scheme) or proxies.get("all")
    if not proxy:
        return None
    return proxy if "://" in proxy else "http://" + proxy


def _is_ipv4(host: str) -> bool:
    ps = host.split(".")
    return len(ps) == 4 and all(p.isdigit() and int(p) < 256 for p in ps)


def _in_cidr(ip: str, cidr: str) -> bool:
    net, _, bits = cidr.partition("/")
    if not _is_ipv4(net) or not bits.isdigit() or not 0 <= int(bits) <= 32:
        return False

    def num(a: str) -> int:
        x = 0
        for p in a.split("."):
            x = (x << 8) | int(p)
        return x
    mask = (0xFFFFFFFF << (32 - int(bits))) & 0xFFFFFFFF
    return (num(ip) & mask) == (num(net) & mask)


def request(url: str, method: str = "GET", headers: Optional[Dict[str, str]] = None, body: Optional[bytes] = None,
            timeout: float = 30.0, ssl_context=None, proxy_url: Optional[str] = None) -> Response:
    """One-shot request on a fresh connection (through ``proxy_url`` when given)."""
    parts = urlsplit(url)
    if parts.scheme not in ("http", "https"):
        if not parts.scheme:
            raise HTTPError("invalid_url", f"Invalid URL '{url}': No scheme supplied. Perhaps you meant https://{url}?")
        raise HTTPError("invalid_url", f"No connection adapters were found for '{url}'")
    if not parts.hostname:
        raise HTTPError("invalid_url", f"Invalid URL '{url}': No host supplied")
    base = f"{parts.scheme}://{parts.netloc}"
    path = parts.path or "/"
    if parts.query:
        path += "?" + parts.query
    if proxy_url and proxy_url.split("://", 1)[0].lower() not in ("http", "https"):
        # requests' InvalidSchema for socks*:// without PySocks (and any other scheme it has no adapter for)
        raise HTTPError("invalid_url", "Missing dependencies for SOCKS support."
                        if proxy_url.lower().startswith("socks") else f"No connection adapters were found for '{url}'")
    conn = Connection(base, timeout=timeout, ssl_context=ssl_context, proxy_url=proxy_url)
    try:
        return conn.request(method, path, headers, body)
    finally:
        conn.close()
