#!/usr/bin/env python3
"""Wall clock of the checker's per-node probe fan-out (``--probe-endpoint``, ``parallel/fanout.py``) as the node
count grows: N mock agent endpoints, each answering ``/probe/<node>`` with an 8-GPU MI355X report after a fixed
delay (the remote agent's network and serving time), fetched with the default concurrency and one at a time.

The north star asks for a check whose wall clock stays flat as nodes are added; with a bounded semaphore it
grows in steps of ``ceil(N / concurrency) x delay`` instead of ``N x delay``.  The agents here are Python
servers on the same 8-CPU host, so at hundreds of nodes their serving time adds to the wall; ``checker_cpu_ms``
is the fetching process's own CPU time (connect, read, JSON parse), the part that is the checker's cost.

    python tools/fanout_scaling.py --delay-ms 20 --nodes 1,8,64,256,1000 --out profiles/fanout_scaling_cpu.json
"""
import argparse
import json
import multiprocessing as mp
import os
import statistics
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from k8s_gpu_node_checker_amd.parallel import fanout  # noqa: E402
from k8s_gpu_node_checker_amd.testing import fixtures  # noqa: E402


def agents(delay_s: float) -> ThreadingHTTPServer:
    """A server standing in for many nodes' agents: ``/probe/<node>`` -> that node's report."""
    cache = {}

    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):
            pass

        def do_GET(self):
            name = self.path.rsplit("/", 1)[-1]
            body = cache.get(name)
            if body is None:
                body = cache[name] = json.dumps(fixtures.mi355x_probe_report(name, gpus=8)).encode()
            time.sleep(delay_s)
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

    class S(ThreadingHTTPServer):
        daemon_threads = True
        request_queue_size = 1024

    srv = S(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def _serve(delay_s: float, conn) -> None:
    srv = agents(delay_s)
    conn.send(srv.server_address[1])
    conn.recv()  # parent says stop
    srv.shutdown()
    srv.server_close()


def agent_processes(n: int, delay_s: float):
    """``n`` agent servers in processes of their own, so the fetching process measured here does not share
    an interpreter lock with the servers (a real fleet's agents run on other machines)."""
    ctx = mp.get_context("fork")
    procs = []
    for _ in range(n):
        a, b = ctx.Pipe()
        p = ctx.Process(target=_serve, args=(delay_s, b), daemon=True)
        p.start()
        procs.append((p, a, a.recv()))
    return procs


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--delay-ms", type=float, default=20.0)
    ap.add_argument("--nodes", default="1,8,64,256,1000")
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--servers", type=int, default=6, help="agent server processes the nodes are spread over")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    procs = agent_processes(args.servers, args.delay_ms / 1e3)
    ports = [port for _, _, port in procs]
    rows = []
    try:
        for n in (int(x) for x in args.nodes.split(",")):
            targets = [{"name": f"mi355x-node-{i:04d}",
                        "url": f"http://127.0.0.1:{ports[i % len(ports)]}/probe/mi355x-node-{i:04d}"}
                       for i in range(n)]
            row = {"nodes": n}
            for conc, key in ((args.concurrency, "fanout_ms"), (1, "sequential_ms")):
                if conc == 1 and n > 64:
                    continue  # n x delay: the point is made at small n
                walls, cpu = [], []
                for _ in range(args.runs):
                    t, c = time.perf_counter(), time.process_time()
                    out = fanout.run_coroutine(fanout.fetch_all(targets, conc, timeout=10.0))
                    walls.append((time.perf_counter() - t) * 1e3)
                    cpu.append((time.process_time() - c) * 1e3)
                    bad = [o for o in out if o.get("error")]
                    if bad:
                        raise SystemExit(f"{len(bad)} fetches failed at n={n}: {bad[0]['error']}")
                row[key] = round(statistics.median(walls), 1)
                if conc != 1:  # the checker's own CPU time: what a fleet's real (remote) agents leave of the wall
                    row["checker_cpu_ms"] = round(statistics.median(cpu), 1)
            row["ideal_ms"] = round(-(-n // args.concurrency) * args.delay_ms, 1)
            rows.append(row)
            print(json.dumps(row), flush=True)
    finally:
        for p, a, _ in procs:
            a.send(None)
            p.join(5)
            a.close()
    res = {"delay_ms": args.delay_ms, "concurrency": args.concurrency, "servers": args.servers,
           "report": "8-GPU MI355X probe report", "rows": rows}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
