#!/usr/bin/env python3
"""Writes ``deploy/monitoring/dashboard.yaml``: a Grafana dashboard (ConfigMap with the ``grafana_dashboard``
label the kube-prometheus-stack sidecar loads) over the node agents' ``/metrics`` and the checker's textfile
metrics.  Every series it queries is one the agent (``agent/server.py _metrics``) or the checker
(``utils/prom.py``) emits -- ``tests/test_deploy.py`` checks that -- so the file is generated, not hand-edited:

    python tools/make_dashboard.py
"""
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "deploy", "monitoring", "dashboard.yaml")

# (title, type, unit, [(expr, legend)], width, height)
ROWS = [
    ("Fleet", [
        ("Nodes by MI355X verdict", "stat", "none",
         [('sum by (state) (mi355x_node_health == 1)', "{{state}}")], 8, 5),
        ("GPU nodes / Ready (checker)", "stat", "none",
         [("k8s_gpu_checker_gpu_nodes", "GPU nodes"), ("k8s_gpu_checker_ready_gpu_nodes", "Ready")], 8, 5),
        ("Seconds since each agent's last probe", "timeseries", "s",
         [("time() - mi355x_agent_probe_timestamp_seconds", "{{node}}")], 8, 5),
        ("Nodes not healthy", "table", "none",
         [('mi355x_node_health{state!="healthy"} == 1', "{{node}} {{state}}")], 24, 6),
    ]),
    ("Diagnostics (idle GPUs, every --diag-interval)", [
        ("bf16 / fp8 GEMM TFLOP/s", "timeseries", "none",
         [('mi355x_gpu_diag_tflops{test=~"gemm.*"}', "{{node}} gpu{{gpu}} {{test}}")], 12, 7),
        ("Matrix-core burn-in TFLOP/s by precision", "timeseries", "none",
         [('mi355x_gpu_diag_tflops{test="mfma"}', "{{node}} gpu{{gpu}} {{dtype}}")], 12, 7),
        ("HBM read / copy TB/s", "timeseries", "none",
         [('mi355x_gpu_diag_read_tbs{test="hbm"}', "{{node}} gpu{{gpu}} read"),
          ('mi355x_gpu_diag_copy_tbs{test="hbm"}', "{{node}} gpu{{gpu}} copy")], 12, 7),
        ("HBM read TB/s per XCD, each alone", "timeseries", "none",
         [("mi355x_gpu_diag_xcd_hbm_read_tbs", "{{node}} gpu{{gpu}} xcd{{xcd}}")], 12, 7),
        ("Diagnostic rates as a share of their reference (a lone GPU fails below 0.85, degraded below 0.95)",
         "timeseries", "percentunit", [("mi355x_gpu_diag_fraction", "{{node}} gpu{{gpu}} {{test}}")], 24, 7),
        ("Each GPU against its node's other GPUs (fails below 0.85)", "timeseries", "percentunit",
         [("mi355x_gpu_diag_peer_ratio", "{{node}} gpu{{gpu}} {{test}} {{metric}}")], 12, 7),
        ("Each GPU against its own baseline (drift below 0.90)", "timeseries", "percentunit",
         [("mi355x_gpu_diag_baseline_ratio", "{{node}} gpu{{gpu}} {{test}} {{metric}}")], 12, 7),
        ("Node-wide shortfalls: every GPU slow alike (share of the reference)", "timeseries", "percentunit",
         [("mi355x_node_diag_shortfall_fraction", "{{node}} {{test}} {{metric}}")], 12, 6),
        ("The fleet's median node and its outliers (checker --health-reeval)", "timeseries", "none",
         [("k8s_gpu_checker_diag_fleet_median_fraction", "{{test}} median"),
          ("k8s_gpu_checker_diag_fleet_outlier_nodes", "{{test}} nodes behind")], 12, 6),
        ("Diagnostics skipped (GPU busy or allocated)", "timeseries", "none",
         [("mi355x_gpu_diag_skipped", "{{node}} gpu{{gpu}}")], 12, 6),
        ("Wrong results found by the diagnostics (words, lanes; GEMM output tiles failing their checksums)",
         "timeseries", "none",
         [("mi355x_gpu_diag_errors", "{{node}} gpu{{gpu}} {{test}}"),
          ("mi355x_gpu_diag_checksum_bad_tiles", "{{node}} gpu{{gpu}} {{test}} tiles")], 12, 6),
    ]),
    ("Memory RAS", [
        ("Uncorrectable ECC", "timeseries", "none", [("mi355x_gpu_ecc_uncorrectable", "{{node}} gpu{{gpu}}")], 8, 6),
        ("Correctable ECC per hour", "timeseries", "none",
         [("mi355x_gpu_ecc_correctable_per_hour", "{{node}} gpu{{gpu}}")], 8, 6),
        ("Retired HBM pages vs the driver's threshold", "timeseries", "none",
         [("mi355x_gpu_retired_pages", "{{node}} gpu{{gpu}} retired"),
          ("mi355x_gpu_retired_page_threshold", "{{node}} gpu{{gpu}} threshold")], 8, 6),
        ("CPER records by severity", "timeseries", "none",
         [("mi355x_gpu_cper_records", "{{node}} gpu{{gpu}} {{severity}}")], 12, 6),
        ("ECC errors by RAS block", "timeseries", "none",
         [("sum by (node, block, kind) (mi355x_gpu_ecc_block_errors)", "{{node}} {{block}} {{kind}}")], 12, 6),
    ]),
    ("Fabric", [
        ("xGMI links up (of 7)", "timeseries", "none", [("mi355x_gpu_xgmi_links_up", "{{node}} gpu{{gpu}}")], 8, 6),
        ("xGMI traffic (KB/s, by peer)", "timeseries", "KBs",
         [("sum by (node, gpu, dir) (rate(mi355x_gpu_xgmi_kilobytes[5m]))", "{{node}} gpu{{gpu}} {{dir}}")], 8, 6),
        ("xGMI pair copies GB/s (median / min pair)", "timeseries", "none",
         [("mi355x_node_xgmi_p2p_gbps", "{{node}} {{stat}}")], 8, 6),
        ("RCCL bus bandwidth GB/s by collective", "timeseries", "none",
         [("mi355x_node_rccl_busbw_gbps", "{{node}} {{op}}")], 12, 6),
        ("PCIe width and replays", "timeseries", "none",
         [("mi355x_gpu_pcie_width", "{{node}} gpu{{gpu}} width"),
          ("rate(mi355x_gpu_pcie_replays[15m])", "{{node}} gpu{{gpu}} replays/s")], 12, 6),
    ]),
    ("Power and thermals", [
        ("Power (W) and cap", "timeseries", "watt",
         [("mi355x_gpu_power_watts", "{{node}} gpu{{gpu}}"), ("mi355x_gpu_power_cap_watts", "{{node}} gpu{{gpu}} cap")],
         8, 6),
        ("Hotspot / HBM temperature (C)", "timeseries", "celsius",
         [("mi355x_gpu_hotspot_celsius", "{{node}} gpu{{gpu}} hotspot"),
          ("mi355x_gpu_hbm_celsius", "{{node}} gpu{{gpu}} hbm")], 8, 6),
        ("Throttled share of time (%)", "timeseries", "percent",
         [("mi355x_gpu_throttle_percent", "{{node}} gpu{{gpu}} {{kind}}")], 8, 6),
        ("Graphics clock (MHz) and activity (%)", "timeseries", "none",
         [("mi355x_gpu_gfxclk_mhz", "{{node}} gpu{{gpu}} MHz"),
          ("mi355x_gpu_gfx_activity_percent", "{{node}} gpu{{gpu}} %")], 24, 6),
    ]),
]


def dashboard() -> dict:
    panels, y, pid = [], 0, 1
    for row_title, items in ROWS:
        panels.append({"type": "row", "title": row_title, "id": pid, "collapsed": False,
                       "gridPos": {"h": 1, "w": 24, "x": 0, "y": y}})
        pid += 1
        y += 1
        x, row_h = 0, 0
        for title, ptype, unit, targets, w, h in items:
            if x + w > 24:
                x, y = 0, y + row_h
                row_h = 0
            panels.append({
                "type": ptype, "title": title, "id": pid, "datasource": {"type": "prometheus", "uid": "${datasource}"},
                "gridPos": {"h": h, "w": w, "x": x, "y": y},
                "fieldConfig": {"defaults": {"unit": unit}, "overrides": []},
                "targets": [{"expr": e, "legendFormat": lg, "refId": chr(ord("A") + i),
                             "datasource": {"type": "prometheus", "uid": "${datasource}"},
                             **({"instant": True, "format": "table"} if ptype == "table" else {})}
                            for i, (e, lg) in enumerate(targets)],
            })
            pid += 1
            x += w
            row_h = max(row_h, h)
        y += row_h
    return {
        "uid": "mi355x-node-health", "title": "MI355X node health", "schemaVersion": 39, "version": 1,
        "tags": ["mi355x", "amd", "gpu", "k8s-gpu-node-checker"], "timezone": "utc", "refresh": "1m",
        "time": {"from": "now-24h", "to": "now"},
        "templating": {"list": [{"name": "datasource", "type": "datasource", "query": "prometheus",
                                 "label": "Prometheus"}]},
        "panels": panels,
    }


def main() -> int:
    body = json.dumps(dashboard(), indent=1, sort_keys=True)
    indented = "\n".join("    " + ln for ln in body.splitlines())
    text = ("# Grafana dashboard over the node agents' /metrics and the checker's textfile metrics, as a ConfigMap the\n"
            "# kube-prometheus-stack Grafana sidecar loads (label grafana_dashboard).  Generated by\n"
            "# tools/make_dashboard.py -- edit that, not this; tests/test_deploy.py checks every queried series.\n"
            "apiVersion: v1\nkind: ConfigMap\nmetadata:\n  name: mi355x-node-health-dashboard\n"
            "  namespace: gpu-health\n  labels: {grafana_dashboard: \"1\"}\ndata:\n"
            "  mi355x-node-health.json: |\n" + indented + "\n")
    with open(OUT, "w", encoding="utf-8") as f:
        f.write(text)
    print(OUT)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
