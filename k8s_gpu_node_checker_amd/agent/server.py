"""The node agent's HTTP side: ``/probe`` (the last report, JSON), ``/metrics`` (Prometheus text), ``/status``
(the report for a human) and ``/healthz`` (the liveness probe), optionally over TLS with client certificates.

Split out of ``agent.py``: everything here reads the agent's state (``agent.last``, ``hung_diagnostic()``,
``hip_lost``) and never changes it.  ``agent.py`` re-exports ``serve``, ``tls_context`` and ``_metrics``.
"""

from __future__ import annotations

import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import TYPE_CHECKING, Any, Dict, List, Optional

from ..utils.http import nodelay
from ..models.health import DEGRADED, HEALTHY, UNHEALTHY, UNKNOWN, driver_release, fw_version_str

if TYPE_CHECKING:
    from .agent import Agent


def _esc(v: Any) -> str:
    """A Prometheus label value (text exposition format escapes)."""
    return str(v).replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def _metrics(rep: Optional[Dict[str, Any]]) -> str:
    """Prometheus text exposition of the last probe.  Samples are collected per metric family and each
    family is written as one group under its ``# TYPE`` line (the format requires it; a per-GPU loop
    that interleaves families makes parsers see the same family twice)."""
    if not rep:
        return "# no probe yet\n"
    fams: Dict[str, List[str]] = {}
    counters = {"mi355x_gpu_pcie_replays", "mi355x_gpu_xgmi_kilobytes", "mi355x_gpu_ecc_correctable"}

    def put(name: str, labels: str, value: Any) -> None:
        fams.setdefault(name, []).append(f"{name}{{{labels}}} {value}" if labels else f"{name} {value}")

    put("mi355x_agent_probe_timestamp_seconds", "", rep.get("ts", 0))
    if isinstance(rep.get("state"), str):
        # the verdict the agent publishes as AMDGPUHealthy, one series per state (1 for the current one)
        for st in (HEALTHY, DEGRADED, UNHEALTHY, UNKNOWN):
            put("mi355x_node_health", f'state="{st}"', 1 if rep["state"] == st else 0)
    drv = rep.get("driver")
    if isinstance(drv, dict) and drv.get("version"):
        put("mi355x_node_driver_info", f'name="{_esc(drv.get("name"))}",version="{_esc(driver_release(drv["version"]))}"', 1)
    for g in rep.get("gpus") or []:
        lbl = f'gpu="{g.get("index")}",bdf="{_esc(g.get("bdf", ""))}"'
        for key, metric in (("ecc_uncorrectable", "ecc_uncorrectable"), ("ecc_correctable", "ecc_correctable"),
                            ("pcie_width", "pcie_width"),
                            ("pcie_replays", "pcie_replays"), ("xgmi_error", "xgmi_error_status"),
                            ("bad_pages", "retired_pages"), ("bad_pages_pending", "retired_pages_pending"),
                            ("bad_pages_unreservable", "retired_pages_unreservable"),
                            ("bad_page_threshold", "retired_page_threshold")):
            if isinstance(g.get(key), int) and not isinstance(g.get(key), bool):
                put(f"mi355x_gpu_{metric}", lbl, g[key])
        if isinstance(g.get("xgmi"), str):
            put("mi355x_gpu_xgmi_links_up", lbl, g["xgmi"].count("U"))
        for key, metric in (("ecc_ce_per_h", "ecc_correctable_per_hour"), ("hotspot_c", "hotspot_celsius"),
                            ("power_w", "power_watts"),
                            ("power_cap_w", "power_cap_watts"), ("hbm_temp_c", "hbm_celsius"),
                            ("gfxclk_mhz", "gfxclk_mhz"), ("vram_used_mb", "vram_used_megabytes"),
                            ("gfx_activity", "gfx_activity_percent")):
            if isinstance(g.get(key), (int, float)) and not isinstance(g.get(key), bool):
                put(f"mi355x_gpu_{metric}", lbl, g[key])
        for kind in ("thermal", "power", "prochot"):
            v = (g.get("throttle") or {}).get(f"{kind}_pct")
            if isinstance(v, (int, float)):
                put("mi355x_gpu_throttle_percent", f'{lbl},kind="{kind}"', v)
        for block, c in ((g.get("ecc_blocks") or {}) if isinstance(g.get("ecc_blocks"), dict) else {}).items():
            for kind in ("ce", "ue", "de"):
                if isinstance(c, dict) and isinstance(c.get(kind), int):
                    put("mi355x_gpu_ecc_block_errors", f'{lbl},block="{_esc(block)}",kind="{kind}"', c[kind])
        cper = g.get("cper")
        if isinstance(cper, dict):
            for sev in ("fatal", "uncorrected", "corrected"):
                if isinstance(cper.get(sev), int):
                    put("mi355x_gpu_cper_records", f'{lbl},severity="{sev}"', cper[sev])
        peers, kb = g.get("xgmi_peers"), g.get("xgmi_kb")
        if isinstance(peers, list) and isinstance(kb, list):
            for peer, rw in zip(peers, kb):
                if isinstance(rw, list) and len(rw) == 2:
                    for d, v in zip(("read", "write"), rw):
                        put("mi355x_gpu_xgmi_kilobytes", f'{lbl},peer="{_esc(peer)}",dir="{d}"', v)
        for image, ver in ((g.get("fw") or {}) if isinstance(g.get("fw"), dict) else {}).items():
            put("mi355x_gpu_firmware_info", f'{lbl},image="{_esc(image)}",version="{_esc(fw_version_str(image, ver))}"', 1)
        if g.get("diag") is not None or g.get("diag_skipped"):
            put("mi355x_gpu_diag_skipped", lbl, 1 if g.get("diag_skipped") else 0)
        proc = g.get("diag_proc")  # process isolation: the diagnostic child's peak host memory (the pod's limit)
        if isinstance(proc, dict) and isinstance(proc.get("peak_rss_mib"), (int, float)):
            put("mi355x_agent_diag_child_peak_rss_bytes", lbl, int(proc["peak_rss_mib"] * 1048576))
        for test, res in (g.get("diag") or {}).items():
            if not isinstance(res, dict):
                continue
            for k in ("tflops", "copy_tbs", "read_tbs", "errors", "h2d_gbps", "d2h_gbps", "fraction",
                      "checksum_bad_tiles"):
                if isinstance(res.get(k), (int, float)) and not isinstance(res.get(k), bool):
                    put(f"mi355x_gpu_diag_{k}", f'{lbl},test="{_esc(test)}"', res[k])
            for xcd, v in ((res.get("alone_tbs") or {}) if isinstance(res.get("alone_tbs"), dict) else {}).items():
                if isinstance(v, (int, float)):
                    put("mi355x_gpu_diag_xcd_hbm_read_tbs", f'{lbl},xcd="{_esc(xcd)}"', v)
            for kind, row in ((res.get("kinds") or {}) if isinstance(res.get("kinds"), dict) else {}).items():
                put("mi355x_gpu_diag_tflops", f'{lbl},test="{_esc(test)}",dtype="{_esc(kind)}"', row.get("tflops", 0))
            # the GPU against its node's other GPUs (models/peers.py) and against its own baseline (models/baseline.py)
            for src, metric in (("peers", "mi355x_gpu_diag_peer_ratio"), ("baseline", "mi355x_gpu_diag_baseline_ratio")):
                ratios = (res.get(src) or {}).get("ratio") if isinstance(res.get(src), dict) else None
                for m, v in (ratios.items() if isinstance(ratios, dict) else ()):
                    if isinstance(v, (int, float)) and not isinstance(v, bool):
                        put(metric, f'{lbl},test="{_esc(test)}",metric="{_esc(m)}"', v)
    node_diag = rep.get("diag_node")
    for f in (node_diag.get("findings") or []) if isinstance(node_diag, dict) else []:
        # a shortfall every GPU shares: the median rate as a fraction of the MI355X reference
        if isinstance(f, dict) and isinstance(f.get("median_fraction"), (int, float)):
            put("mi355x_node_diag_shortfall_fraction", f'test="{_esc(f.get("test"))}",metric="{_esc(f.get("metric"))}"',
                f["median_fraction"])
    fabric = (rep.get("fabric") or {}).get("p2p")
    if isinstance(fabric, dict) and isinstance(fabric.get("median_gbps"), (int, float)):
        put("mi355x_node_xgmi_p2p_gbps", 'stat="median"', fabric["median_gbps"])
        put("mi355x_node_xgmi_p2p_gbps", 'stat="min"', fabric.get("min_gbps", 0))
    rccl = (rep.get("fabric") or {}).get("rccl")
    if isinstance(rccl, dict) and isinstance(rccl.get("best_busbw_by_op"), dict):
        for op, bw in sorted(rccl["best_busbw_by_op"].items()):
            put("mi355x_node_rccl_busbw_gbps", f'op="{_esc(op)}"', bw)
    lines: List[str] = []
    for name, samples in fams.items():
        lines.append(f"# TYPE {name} {'counter' if name in counters else 'gauge'}")
        lines += samples
    return "\n".join(lines) + "\n"


def tls_context(cert_file: str, key_file: str, client_ca: Optional[str] = None) -> Any:
    """Server-side TLS for the agent's port.  With ``client_ca`` a client certificate is requested and, when
    presented, verified against it (``CERT_OPTIONAL``): the kubelet's liveness probe presents none and still
    reaches ``/healthz``; ``serve`` then refuses ``/probe``, ``/metrics`` and ``/status`` (host PIDs, the full
    report) to a client without a verified certificate."""
    import ssl
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.minimum_version = ssl.TLSVersion.TLSv1_2
    ctx.load_cert_chain(cert_file, key_file)
    if client_ca:
        ctx.load_verify_locations(cafile=client_ca)
        ctx.verify_mode = ssl.CERT_OPTIONAL
    return ctx


# a connection that sends no complete request for this long is closed (an idle keep-alive or a stalled client
# would otherwise hold its handler thread for the life of the agent)
IDLE_TIMEOUT_S = 30.0


def serve(agent: Agent, host: str, port: int, stale_after: Optional[float] = None, tls: Any = None,
          require_client_cert: bool = False) -> ThreadingHTTPServer:
    """/probe, /metrics, /status (text) and /healthz; /healthz answers 503 once no probe has completed for
    ``stale_after`` s (a wedged amd-smi call or driver) and, with thread isolation only, once a diagnostic thread
    has outlived HUNG_RESTART_FACTOR x ``diag_timeout`` (a hung HIP queue the process cannot cancel) or after the
    HIP runtime lost its devices, so a livenessProbe restarts the agent as a fresh process (the kubelet starts a
    new container; nothing is re-executed in place).  With process isolation (the DaemonSet's) neither applies:
    a hung diagnostic child is SIGKILLed at its watchdog and every child starts a fresh HIP runtime."""
    started = time.monotonic()

    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"
        timeout = IDLE_TIMEOUT_S

        def log_message(self, *a: Any) -> None:
            pass

        def setup(self) -> None:
            super().setup()
            nodelay(self.connection)

        def do_GET(self) -> None:  # noqa: N802
            if require_client_cert and not self.path.startswith("/healthz"):
                peer = self.connection.getpeercert() if hasattr(self.connection, "getpeercert") else None
                if not peer:
                    body = b"client certificate required\n"
                    self.send_response(403)
                    self.send_header("Content-Type", "text/plain")
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)
                    return
            with agent.lock:
                rep = agent.last
            if self.path.startswith("/probe"):
                body = json.dumps(rep or {"schema": "mi355x-health/v1", "error": "no probe yet"}).encode()
                ctype = "application/json"
            elif self.path.startswith("/metrics"):
                body = _metrics(rep).encode()
                ctype = "text/plain; version=0.0.4"
            elif self.path.startswith("/status"):
                # the last report for a human (kubectl port-forward): verdict, reasons, per-GPU table
                if rep:
                    from ..explain import report_text
                    body = report_text(rep, agent.evaluate(rep)).encode()
                else:
                    body = b"no probe yet\n"
                ctype = "text/plain; charset=utf-8"
            elif self.path.startswith("/healthz"):
                last = agent.last_probe_done if agent.last_probe_done is not None else started
                idle = time.monotonic() - last
                lost = agent.hip_lost
                hung = agent.hung_diagnostic()
                if lost is not None or hung is not None or (stale_after is not None and idle > stale_after):
                    body = (f"HIP runtime lost its devices: {lost}" if lost is not None
                            else hung if hung is not None else f"no probe completed for {idle:.0f} s").encode()
                    self.send_response(503)
                    self.send_header("Content-Type", "text/plain")
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)
                    return
                body, ctype = b"ok", "text/plain"
            else:
                self.send_response(404)
                self.send_header("Content-Length", "0")
                self.end_headers()
                return
            self.send_response(200)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_POST(self) -> None:  # noqa: N802
            """``POST /baseline/reset[?gpu=KEY[,KEY]]``: drop self-baselines (``models/baseline.Baselines.drop``).
            Only from the pod itself -- a loopback peer, which is what ``kubectl port-forward`` and ``kubectl exec``
            arrive as -- so nothing on the pod network (the checker's fan-out, Prometheus) can reset a GPU's
            memory of its own normal."""
            from urllib.parse import parse_qs, urlsplit
            parts = urlsplit(self.path)
            try:
                n = int(self.headers.get("Content-Length") or 0)
            except ValueError:
                n = -1
            if n > 0:
                self.rfile.read(min(n, 65536))
            if n < 0 or n > 65536:  # a malformed or oversized body: answer, then drop the connection
                self.close_connection = True
            peer = self.client_address[0] if self.client_address else ""
            if n < 0:
                code, doc = 400, {"error": "bad Content-Length"}
            elif parts.path != "/baseline/reset":
                code, doc = 404, {"error": "not found"}
            elif not (peer.startswith("127.") or peer in ("::1", "::ffff:127.0.0.1")):
                code, doc = 403, {"error": "baseline reset is only accepted from inside the pod (loopback)"}
            elif agent.baselines is None:
                code, doc = 409, {"error": "self-baselines are off (--no-diag-baseline)"}
            else:
                want = [g for v in parse_qs(parts.query).get("gpu", []) for g in v.split(",") if g.strip()]
                code, doc = 200, {"dropped": agent.baselines.drop(want or None)}
            body = (json.dumps(doc) + "\n").encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

    class Srv(ThreadingHTTPServer):
        daemon_threads = True
        request_queue_size = 128  # the checker's fan-out connects in bursts

        def finish_request(self, request: Any, client_address: Any) -> None:
            if tls is None:
                super().finish_request(request, client_address)
                return
            # the handshake runs on the connection's own thread (never on the accept loop), bounded
            request.settimeout(10.0)
            try:
                conn = tls.wrap_socket(request, server_side=True)
            except OSError:
                request.close()
                return
            conn.settimeout(None)
            try:
                super().finish_request(conn, client_address)
            finally:
                # wrap_socket detached the accepted socket (socketserver closes that empty shell): the TLS one is ours
                try:
                    conn.close()
                except OSError:
                    pass

    srv = Srv((host, port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv
