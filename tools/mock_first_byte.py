#!/usr/bin/env python3
"""The mock kube-apiserver's own latency: a raw-socket GET of the NodeList (no client library), timed to the first
response byte and to the end of the body.  This is the floor under bench.py's ``first_byte`` span: whatever the
checker does, a LIST against this server cannot return sooner.

    python tools/mock_first_byte.py --nodes 1 --reps 300
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1)
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    args = ap.parse_args()
    p = subprocess.Popen([sys.executable, "-m", "k8s_gpu_node_checker_amd.testing.mock_apiserver", "--nodes",
                          str(args.nodes), "--kind", "amd", "--gpus-per-node", "1", "--annotation-encoding", "gzip"],
                         stdout=subprocess.PIPE, text=True, cwd=REPO)
    try:
        url = json.loads(p.stdout.readline())["url"]
        host, port = url.split("//", 1)[1].rstrip("/").rsplit(":", 1)
        req = (f"GET /api/v1/nodes?limit=500 HTTP/1.1\r\nHost: {host}:{port}\r\nAccept: application/json\r\n"
               "Connection: close\r\n\r\n").encode()
        first, total = [], []
        for i in range(args.warmup + args.reps):
            t0 = time.perf_counter()
            s = socket.create_connection((host, int(port)))
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            t1 = time.perf_counter()
            s.sendall(req)
            s.recv(1)
            t2 = time.perf_counter()
            while s.recv(65536):
                pass
            s.close()
            t3 = time.perf_counter()
            if i >= args.warmup:
                first.append((t2 - t1) * 1e3)
                total.append((t3 - t0) * 1e3)
        print(json.dumps({"nodes": args.nodes, "reps": args.reps, "first_byte_ms": round(statistics.median(first), 3),
                          "request_ms": round(statistics.median(total), 3)}))
    finally:
        p.terminate()
        p.wait(timeout=5)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
