"""Slack-webhook sink with fault injection.

The URL path selects the behaviour, so one sink serves every test:

==============  =============================================================
``/200``        ``200 ok``
``/500``        ``500 server_error``
``/204``        ``204`` (not a success for the reference, ``:79``)
``/404``        ``404 no_service`` (revoked webhook)
``/429``        ``429 rate_limited`` with ``Retry-After: 1``
``/flakyN``     ``500`` N times (per sink), then ``200``
``/reset``      TCP RST on every attempt (``SO_LINGER {1,0}``)
``/resetflaky`` RST once, then ``200``
``/slow``       sleep ``slow_s`` (default 11 s) before answering ``200``
``/close``      close without a response ("Remote end closed connection")
``/seq/ID/A,B``  scripted: the n-th POST to this exact path gets step n (the last step repeats); a step is
                 ``200``, ``204``, ``404``, ``429``, ``500``, ``reset`` or ``close``; ``ID`` keeps runs apart
``/301`` ...    ``301``, ``302``, ``303``, ``307``, ``308`` redirecting (relative ``Location``) to ``/postonly``
``/postonly``   ``200`` to a POST, ``405 method_not_allowed`` to anything else
``/loop``       ``302`` to itself, forever
``/to/H/MODE``  ``307`` to ``http://H:<this port>/MODE`` (another host name for the same sink)
``/cookie``     ``302`` to ``/200`` setting ``sid=abc`` (path ``/``)
``/loc/S/L``    status ``S`` with ``Location: L`` (percent-decoded; ``{port}`` becomes this sink's port; no header
                when ``L`` is empty): relative, scheme-relative, query, fragment and foreign-scheme targets
``/body/KIND``   ``500`` with a UTF-8 body sent ``gzip`` / ``deflate`` / ``chunked``, as ``euckr`` or ``latin``
                (no charset), with no length (``nolength``), as ``octet`` (guessed), or labelled compressed but
                sent plain (``badgzip`` / ``baddeflate``)
``/raw/NAME``   a malformed or unusual response: ``badstatus``, ``notahttp``, ``truncated`` (body shorter than its
                length), ``badchunk``, ``truncatedchunk``, ``continue`` (100 then 200), ``http10``, ``longheader``,
                ``twolengths``, ``empty200``, ``manyheaders``, ``justenoughheaders``, ``longstatus``,
                ``prematurechunk``, ``badcl``, ``samecl``, ``status99``, ``chunkext``, ``resetbody`` (a 200 head and
                part of its body, then TCP RST: the connection dies mid-body after the server took the POST)
``/locb/S/L``   the same with ``L``'s percent-decoded bytes sent raw (a Location that is not UTF-8)
==============  =============================================================

Every request is logged (path, headers, body) for assertions.
"""

from __future__ import annotations

import json
import socket
import socketserver
import struct
import threading
import time
import urllib.parse
from typing import Any, Dict, List, Optional


# /raw/NAME: responses that break HTTP in one way each (what a proxy or a broken endpoint may send)
_RAW = {
    "badstatus": b"HTTP/1.1 abc Whatever\r\nContent-Length: 2\r\n\r\nok",
    "notahttp": b"hello there\r\n\r\n",
    "truncated": b"HTTP/1.1 500 Internal Server Error\r\nContent-Length: 100\r\nConnection: close\r\n\r\nonly ten b",
    "badchunk": b"HTTP/1.1 500 Internal Server Error\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\nzz\r\nabc\r\n0\r\n\r\n",
    "truncatedchunk": b"HTTP/1.1 500 Internal Server Error\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n10\r\nabc",
    "continue": b"HTTP/1.1 100 Continue\r\n\r\nHTTP/1.1 200 OK\r\nContent-Length: 2\r\nConnection: close\r\n\r\nok",
    "http10": b"HTTP/1.0 200 OK\r\nContent-Type: text/plain\r\n\r\nok",
    "longheader": b"HTTP/1.1 500 Internal Server Error\r\nX-Long: " + b"a" * 70000 + b"\r\nContent-Length: 2\r\n\r\nno",
    "twolengths": b"HTTP/1.1 500 Internal Server Error\r\nContent-Length: 2\r\nContent-Length: 3\r\nConnection: close\r\n\r\nabc",
    "empty200": b"HTTP/1.1 200 OK\r\nConnection: close\r\n\r\n",
    "manyheaders": b"HTTP/1.1 500 Internal Server Error\r\n" + b"".join(b"X-%d: v\r\n" % i for i in range(100))
                   + b"Content-Length: 2\r\n\r\nno",
    "justenoughheaders": b"HTTP/1.1 500 Internal Server Error\r\n" + b"".join(b"X-%d: v\r\n" % i for i in range(98))
                         + b"Content-Length: 2\r\n\r\nno",
    "longstatus": b"HTTP/1.1 500 " + b"x" * 70000 + b"\r\nContent-Length: 2\r\n\r\nno",
    "prematurechunk": b"HTTP/1.1 500 Internal Server Error\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n3\r\nabc\r\n",
    "badcl": b"HTTP/1.1 500 Internal Server Error\r\nContent-Length: abc\r\nConnection: close\r\n\r\nbody",
    "samecl": b"HTTP/1.1 500 Internal Server Error\r\nContent-Length: 3\r\nContent-Length: 3\r\nConnection: close\r\n\r\nabc",
    "status99": b"HTTP/1.1 099 Odd\r\nContent-Length: 2\r\n\r\nno",
    "chunkext": b"HTTP/1.1 500 Internal Server Error\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n3;x=y\r\nabc\r\n0\r\n\r\n",
}


class _SinkHandler(socketserver.BaseRequestHandler):
    server: "WebhookSink"  # type: ignore[assignment]

    def _read_request(self) -> Optional[Dict[str, Any]]:
        sock: socket.socket = self.request
        data = b""
        while b"\r\n\r\n" not in data:
            chunk = sock.recv(65536)
            if not chunk:
                return None
            data += chunk
        head, _, rest = data.partition(b"\r\n\r\n")
        lines = head.decode("latin-1").split("\r\n")
        method, path, _ = lines[0].split(" ", 2)
        headers = {}
        for line in lines[1:]:
            k, _, v = line.partition(":")
            headers[k.strip()] = v.strip()
        n = int(headers.get("Content-Length", "0") or 0)
        while len(rest) < n:
            chunk = sock.recv(65536)
            if not chunk:
                break
            rest += chunk
        return {"method": method, "path": path, "headers": headers, "body": rest[:n], "ts": time.time()}

    def _respond(self, status: int, reason: str, body: bytes, extra: str = "") -> None:
        msg = (f"HTTP/1.1 {status} {reason}\r\nContent-Type: text/plain\r\nContent-Length: {len(body)}\r\n"
               f"{extra}Connection: close\r\n\r\n").encode() + body
        self.request.sendall(msg)

    def _send_body(self, kind: str) -> None:
        text = "서버 오류: rate limited ✗".encode("utf-8")
        head = "HTTP/1.1 500 Internal Server Error\r\nConnection: close\r\n"
        if kind == "gzip":
            import gzip
            body, head = gzip.compress(text), head + "Content-Type: text/plain; charset=utf-8\r\nContent-Encoding: gzip\r\n"
        elif kind == "deflate":
            import zlib
            body, head = zlib.compress(text), head + "Content-Type: text/plain; charset=utf-8\r\nContent-Encoding: deflate\r\n"
        elif kind == "chunked":
            body = b"".join(b"%x\r\n%s\r\n" % (len(text[i:i + 7]), text[i:i + 7]) for i in range(0, len(text), 7))
            body += b"0\r\n\r\n"
            head += "Content-Type: application/json\r\nTransfer-Encoding: chunked\r\n"
        elif kind == "euckr":
            body, head = "서버 오류".encode("euc-kr"), head + "Content-Type: text/plain; charset=euc-kr\r\n"
        elif kind == "latin":  # UTF-8 bytes labelled text/plain without a charset: ISO-8859-1 by requests' rule
            body, head = text, head + "Content-Type: text/plain\r\n"
        elif kind in ("badgzip", "baddeflate"):  # labelled compressed, sent plain: the client cannot decode it
            body = text
            head += f"Content-Type: text/plain; charset=utf-8\r\nContent-Encoding: {kind[3:]}\r\n"
        elif kind == "nolength":  # no Content-Length: the body runs to the close
            body, head = text, head + "Content-Type: application/json\r\n"
            self.request.sendall(head.encode() + b"\r\n" + body)
            return
        else:  # octet-stream: the encoding is guessed
            body, head = text, head + "Content-Type: application/octet-stream\r\n"
        if kind != "chunked":
            head += f"Content-Length: {len(body)}\r\n"
        self.request.sendall(head.encode() + b"\r\n" + body)

    def handle(self) -> None:
        req = self._read_request()
        if req is None:
            return
        srv = self.server
        with srv.lock:
            srv.requests.append(req)
            count = srv.counts.get(req["path"], 0) + 1
            srv.counts[req["path"]] = count
        path = req["path"].split("?", 1)[0]
        if path.startswith("/body/"):  # a 500 whose body is encoded some way: /body/gzip, deflate, chunked, ...
            self._send_body(path[6:])
            return
        if path == "/raw/resetbody":  # the head and 10 of 100 bytes, then RST once the client is reading the body
            self.request.sendall(b"HTTP/1.1 200 OK\r\nContent-Length: 100\r\n\r\nonly ten b")
            time.sleep(0.2)
            self.request.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
            self.request.close()
            return
        if path.startswith("/raw/"):  # a malformed or unusual response (see _RAW)
            self.request.sendall(_RAW[path[5:]])
            if path[5:] in ("truncated", "truncatedchunk"):
                time.sleep(0.05)
            return
        if path.startswith("/locb/"):  # the Location's bytes as given (percent-decoded, not re-encoded)
            _, _, status, loc = req["path"].split("/", 3)
            raw = urllib.parse.unquote_to_bytes(loc)
            self.request.sendall(f"HTTP/1.1 {int(status)} Redirect\r\nContent-Length: 5\r\n".encode() + b"Location: " +
                                 raw + b"\r\nConnection: close\r\n\r\nmoved")
            return
        if path.startswith("/loc/"):
            _, _, status, loc = req["path"].split("/", 3)
            loc = urllib.parse.unquote(loc).replace("{port}", str(srv.server_address[1]))
            self._respond(int(status), "Redirect", b"moved", f"Location: {loc}\r\n" if loc else "")
            return
        if path.startswith("/seq/"):
            steps = path.rsplit("/", 1)[-1].split(",")
            path = "/" + steps[min(count, len(steps)) - 1]
        if path == "/reset" or (path == "/resetflaky" and count == 1):
            self.request.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
            self.request.close()
            return
        if path == "/close":
            self.request.close()
            return
        if path == "/slow":
            time.sleep(srv.slow_s)
        if path in ("/301", "/302", "/303", "/307", "/308"):
            self._respond(int(path[1:]), "Redirect", b"", "Location: /postonly\r\n")
            return
        if path == "/postonly":
            if req["method"] == "POST":
                self._respond(200, "OK", b"ok")
            else:
                self._respond(405, "Method Not Allowed", b"method_not_allowed")
            return
        if path == "/loop":
            self._respond(302, "Found", b"", "Location: /loop\r\n")
            return
        if path.startswith("/to/"):
            _, _, host, mode = path.split("/", 3)
            port = srv.server_address[1]
            self._respond(307, "Temporary Redirect", b"", f"Location: http://{host}:{port}/{mode}\r\n")
            return
        if path == "/cookie":
            self._respond(302, "Found", b"", "Set-Cookie: sid=abc; Path=/\r\nLocation: /200\r\n")
            return
        if path.startswith("/flaky"):
            n = int(path[6:] or 2)
            if count <= n:
                self._respond(500, "Internal Server Error", b"server_error")
                return
            self._respond(200, "OK", b"ok")
            return
        table = {"/200": (200, "OK", b"ok", ""), "/500": (500, "Internal Server Error", b"server_error", ""),
                 "/204": (204, "No Content", b"", ""), "/404": (404, "Not Found", b"no_service", ""),
                 "/429": (429, "Too Many Requests", b"rate_limited", "Retry-After: 1\r\n"),
                 "/slow": (200, "OK", b"ok", ""), "/resetflaky": (200, "OK", b"ok", "")}
        status, reason, body, extra = table.get(path, (404, "Not Found", b"no_such_mode", ""))
        if status == 204:
            self.request.sendall(f"HTTP/1.1 204 No Content\r\n{extra}Connection: close\r\n\r\n".encode())
            return
        self._respond(status, reason, body, extra)


class WebhookSink(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, host: str = "127.0.0.1", port: int = 0, slow_s: float = 11.0):
        super().__init__((host, port), _SinkHandler)
        self.lock = threading.Lock()
        self.requests: List[Dict[str, Any]] = []
        self.counts: Dict[str, int] = {}
        self.slow_s = slow_s

    @property
    def base_url(self) -> str:
        host, port = self.server_address[:2]
        return f"http://{host}:{port}"

    def url(self, mode: str) -> str:
        return f"{self.base_url}/{mode.lstrip('/')}"

    def payloads(self) -> List[Dict[str, Any]]:
        return [json.loads(r["body"]) for r in self.requests if r["body"]]

    def start(self) -> "WebhookSink":
        threading.Thread(target=self.serve_forever, kwargs={"poll_interval": 0.05}, daemon=True).start()
        return self

    def stop(self) -> None:
        self.shutdown()
        self.server_close()

    def __enter__(self) -> "WebhookSink":
        return self.start()

    def __exit__(self, *exc: Any) -> None:
        self.stop()


def main() -> int:
    import argparse
    ap = argparse.ArgumentParser(description="Slack webhook sink with fault injection")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--slow-s", type=float, default=11.0)
    args = ap.parse_args()
    sink = WebhookSink(args.host, args.port, args.slow_s)
    print(json.dumps({"url": sink.base_url}), flush=True)
    try:
        sink.serve_forever(poll_interval=0.2)
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
