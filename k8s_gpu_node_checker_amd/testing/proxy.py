"""An HTTP forward proxy for tests: ``CONNECT`` tunnels (https targets) and absolute-form requests (http
targets), recording every request line and the ``Proxy-Authorization`` it carried."""

from __future__ import annotations

import select
import socket
import socketserver
import threading
from typing import List, Optional, Tuple


class ForwardProxy:
    def __init__(self) -> None:
        self.seen: List[Tuple[str, Optional[str]]] = []  # (request line, Proxy-Authorization)
        owner = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self) -> None:
                data = b""
                while b"\r\n\r\n" not in data:
                    chunk = self.request.recv(4096)
                    if not chunk:
                        return
                    data += chunk
                head, _, rest = data.partition(b"\r\n\r\n")
                lines = head.decode("latin-1").split("\r\n")
                auth = next((ln.split(":", 1)[1].strip() for ln in lines[1:]
                             if ln.lower().startswith("proxy-authorization:")), None)
                owner.seen.append((lines[0], auth))
                method, target = lines[0].split()[:2]
                if method == "CONNECT":
                    host, port = target.rsplit(":", 1)
                    up = socket.create_connection((host, int(port)))
                    self.request.sendall(b"HTTP/1.1 200 Connection established\r\n\r\n")
                else:  # absolute-form: forward the request as origin-form, minus the proxy header
                    hostport = target.split("://", 1)[1].split("/", 1)
                    host, _, port = hostport[0].partition(":")
                    path = "/" + (hostport[1] if len(hostport) > 1 else "")
                    up = socket.create_connection((host, int(port or 80)))
                    kept = [ln for ln in lines[1:] if not ln.lower().startswith("proxy-authorization:")]
                    up.sendall(("\r\n".join([f"{method} {path} HTTP/1.1"] + kept) + "\r\n\r\n").encode("latin-1")
                               + rest)
                socks = [self.request, up]
                try:
                    while True:
                        r, _, _ = select.select(socks, [], [], 5)
                        if not r:
                            break
                        for s in r:
                            chunk = s.recv(65536)
                            if not chunk:
                                return
                            (up if s is self.request else self.request).sendall(chunk)
                finally:
                    up.close()

        class Server(socketserver.ThreadingTCPServer):
            daemon_threads = True
            allow_reuse_address = True
        self.server = Server(("127.0.0.1", 0), Handler)
        self.port = self.server.server_address[1]

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}"

    def __enter__(self) -> "ForwardProxy":
        threading.Thread(target=self.server.serve_forever, daemon=True).start()
        return self

    def __exit__(self, *exc) -> None:
        self.server.shutdown()
        self.server.server_close()
