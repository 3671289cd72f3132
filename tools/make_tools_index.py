#!/usr/bin/env python3
"""Writes tools/README.md: every script here with the first paragraph of its docstring or header comment, grouped by
what it measures.  Run after adding a tool."""
import ast
import os

T = os.path.dirname(os.path.abspath(__file__))
GROUPS = [
    ("Checker and bench (CPU or any box)", ("ab_", "baseline_configs", "coldstart", "exit_repro", "extended_modes",
                                            "fanout_scaling", "mock_first_byte", "phase_breakdown", "pin_ab", "bench_",
                                            "make_", "mock_fix", "nodes1000", "sweep_", "watch_")),
    ("Node agent: soaks, memory, isolation", ("agent_", "baseline_soak", "soak", "child_", "first_child", "hip_rss",
                                              "copy_threshold", "scratch_ab", "rccl_rss", "contention", "final_r06",
                                              "telemetry", "sdma_")),
    ("GEMM kernels (diag.hip): A/B, labs, PMC", ("gemm_",)),
    ("HBM / L2 / LDS / MFMA / XCD / host link", ("hbm_", "l2_", "lds_", "mall_", "mfma_", "xcd_", "hostlink",
                                                 "host_link", "fp8_")),
    ("Diagnostics runs and calibration", ("diag_", "cper_", "xgmi_", "explore_amdsmi")),
    ("GPU-box scripts (one gpurun call each)", ("gpu_",)),
]


def describe(f: str) -> str:
    text = open(os.path.join(T, f), errors="replace").read()
    if f.endswith(".py"):
        try:
            doc = ast.get_docstring(ast.parse(text)) or ""
        except SyntaxError:
            doc = ""
        return " ".join(doc.strip().split("\n\n")[0].split())
    lines = []
    for ln in text.splitlines():
        s = ln.strip()
        if s.startswith("#!"):
            continue
        if s.startswith(("//", "#")):
            s = s.lstrip("/#").strip()
            if not s and lines:
                break
            if s:
                lines.append(s)
        elif lines or s:
            break
    return " ".join(lines)


def row(f: str) -> str:
    d = describe(f).replace("|", "\\|") or "(no description)"
    if len(d) > 260:
        d = d[:257].rsplit(" ", 1)[0] + " ..."
    return f"| `{f}` | {d} |"


def main() -> int:
    files = sorted(f for f in os.listdir(T) if os.path.isfile(os.path.join(T, f))
                   and not f.endswith((".bin", ".pyc")) and f != "README.md")
    out = ["# tools/", "",
           "Lab and measurement scripts behind `profiles/` (each profile names the tool and command that made it). Not "
           "shipped", "in the package and not part of the test suite. `.hip` labs build with "
           "`hipcc --offload-arch=gfx950 -O3 <file> -o tools/<name>.bin`",
           "(the `.bin` files are git-ignored); GPU scripts run on an MI355X box through the repository's `gpurun` "
           "workflow.", ""]
    placed = set()
    for title, prefixes in GROUPS + [("Other", ("",))]:
        fs = [f for f in files if f not in placed and f.startswith(prefixes)]
        if fs:
            placed.update(fs)
            out += [f"## {title}", "", "| file | what it does |", "|---|---|"] + [row(f) for f in fs] + [""]
    with open(os.path.join(T, "README.md"), "w") as fh:
        fh.write("\n".join(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
