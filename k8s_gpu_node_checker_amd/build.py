"""Build every native component in-tree (``k8s_gpu_node_checker_amd/_native/``).

``python -m k8s_gpu_node_checker_amd.build [--only fastpath,probe,diag] [--force]``

=====================  ==================================================  ==========================
artefact               source                                              toolchain
=====================  ==================================================  ==========================
``_fastpath*.so``      ``csrc/fastpath/fastpath.cpp`` (CPython ext)        g++ -O3
``libmi355x_probe.so`` ``csrc/probe/probe.cpp`` (C ABI over libamd_smi)     g++ + /opt/rocm/lib/libamd_smi
``mi355x-probe``       ``csrc/probe/probe_main.cpp`` (standalone CLI)       g++ + libamd_smi
``libmi355x_diag.so``  ``csrc/diag/diag.hip`` (HIP kernels, gfx950 only)    hipcc --offload-arch=gfx950
``libmi355x_fabric.so`` ``csrc/fabric/fabric.hip`` (RCCL over xGMI)         hipcc + /opt/rocm/lib/librccl
=====================  ==================================================  ==========================

Outputs are rebuilt only when a source is newer or the build command changed (``--force`` to override).
No JIT cache, nothing outside the tree: the ``.so`` files travel with the
source snapshot to the GPU box.
"""

from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "_native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _targets() -> Dict[str, Dict[str, object]]:
    py_inc = sysconfig.get_paths()["include"]
    cxx = os.environ.get("CXX", "g++")
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    smi = ["-I", os.path.join(ROCM, "include"), "-L", os.path.join(ROCM, "lib"), "-lamd_smi",
           f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"]
    return {
        "fastpath": {
            "sources": [os.path.join(CSRC, "fastpath", "fastpath.cpp")],
            "out": os.path.join(OUT, "_fastpath" + _ext_suffix()),
            # libstdc++ linked in statically: loading the shared one cost ~1.2 ms of a 1-node cold start
            "cmd": [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wextra",
                    "-Wno-missing-field-initializers", "-Wno-cast-function-type", "-ffunction-sections",
                    "-fdata-sections", "-I", py_inc],
            "post": ["-static-libstdc++", "-static-libgcc", "-Wl,--gc-sections"],
        },
        "probe": {
            "sources": [os.path.join(CSRC, "probe", "probe.cpp")],
            "headers": [os.path.join(CSRC, "probe", "probe.h")],
            "out": os.path.join(OUT, "libmi355x_probe.so"),
            "cmd": [cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wextra"],
            "post": smi,
        },
        "probe_cli": {
            "sources": [os.path.join(CSRC, "probe", "probe_main.cpp"), os.path.join(CSRC, "probe", "probe.cpp")],
            "headers": [os.path.join(CSRC, "probe", "probe.h")],
            "out": os.path.join(OUT, "mi355x-probe"),
            "cmd": [cxx, "-O2", "-std=c++17", "-Wall", "-Wextra"],
            "post": smi,
        },
        "diag": {
            "sources": [os.path.join(CSRC, "diag", "diag.hip")],
            "headers": [os.path.join(CSRC, "diag", "v4_plan.h")],
            "out": os.path.join(OUT, "libmi355x_diag.so"),
            "cmd": [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
                    "-Wall", "-Wno-unused-result"],
            "requires": hipcc,
        },
        "fabric": {
            "sources": [os.path.join(CSRC, "fabric", "fabric.hip")],
            "out": os.path.join(OUT, "libmi355x_fabric.so"),
            "cmd": [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
                    "-Wall", "-Wno-unused-result"],
            "post": ["-L", os.path.join(ROCM, "lib"), "-lrccl", f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"],
            "requires": hipcc,
        },
    }


def _stale(out: str, deps: Sequence[str], cmd: str = "") -> bool:
    """Rebuild when the output is missing, older than a source, or was built by a different command."""
    if not os.path.exists(out):
        return True
    try:
        with open(out + ".cmd") as f:
            if f.read() != cmd:
                return True
    except OSError:
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_one(name: str, spec: Dict[str, object], force: bool = False, verbose: bool = False) -> Optional[str]:
    sources: List[str] = list(spec["sources"])  # type: ignore[arg-type]
    out = str(spec["out"])
    deps = sources + list(spec.get("headers", []))  # type: ignore[arg-type]
    req = spec.get("requires")
    if req and not os.path.exists(str(req)):
        return f"{name}: skipped ({req} not found)"
    cmd = list(spec["cmd"]) + sources + ["-o", out + ".tmp"] + list(spec.get("post", []))  # type: ignore[arg-type]
    stamp = " ".join(cmd)
    if not force and not _stale(out, deps, stamp):
        return None
    os.makedirs(OUT, exist_ok=True)
    tmp = out + ".tmp"
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"build of {name} failed:\n{' '.join(cmd)}\n{proc.stdout}")
    os.replace(tmp, out)
    with open(out + ".cmd", "w") as f:
        f.write(stamp)
    return f"{name}: built {os.path.relpath(out, os.path.dirname(PKG))}"


def build(only: Optional[Sequence[str]] = None, force: bool = False, verbose: bool = False) -> List[str]:
    targets = _targets()
    names = [n for n in targets if not only or n in only or (n == "probe_cli" and "probe" in only)]
    msgs: List[str] = []
    with ThreadPoolExecutor(max_workers=min(4, len(names) or 1)) as ex:
        futs = {n: ex.submit(build_one, n, targets[n], force, verbose) for n in names}
        errors = []
        for n, f in futs.items():
            try:
                m = f.result()
                if m:
                    msgs.append(m)
            except Exception as e:  # collect all failures, then raise once
                errors.append(str(e))
    if errors:
        raise RuntimeError("\n\n".join(errors))
    return msgs


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--only", help="comma list of fastpath,probe,diag")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args(argv)
    only = args.only.split(",") if args.only else None
    for m in build(only, args.force, args.verbose):
        print(m)
    return 0


if __name__ == "__main__":
    sys.exit(main())
