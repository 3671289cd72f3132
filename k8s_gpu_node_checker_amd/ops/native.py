"""Locate and load the in-tree native libraries built by :mod:`k8s_gpu_node_checker_amd.build`.

All artefacts live in ``k8s_gpu_node_checker_amd/_native/`` (git-ignored,
but shipped with the source tree to the GPU box).  Nothing is JIT-compiled
into a user cache.

* ``_fastpath*.so``      CPython extension: NodeList scanner + JSON emitter (CPU hot path)
* ``libmi355x_probe.so`` C ABI over ``libamd_smi``: passive MI355X health probe
* ``libmi355x_diag.so``  HIP/gfx950 kernels: active diagnostics (MFMA, HBM, memtest)
"""

from __future__ import annotations

import os
import sys
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Dict, Optional

NATIVE_DIR = os.environ.get("K8SGPU_NATIVE_DIR") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native")

_cache: Dict[str, object] = {}


class NativeUnavailable(RuntimeError):
    """Raised when a required native library is missing or fails to load."""


def native_path(filename: str) -> str:
    return os.path.join(NATIVE_DIR, filename)


def load_extension(name: str):
    """Import a CPython extension module from ``_native`` (returns ``None`` if absent)."""
    key = "ext:" + name
    if key in _cache:
        return _cache[key]
    mod = None
    if os.environ.get("K8SGPU_DISABLE_NATIVE") != "1":
        # the import system's own (frozen, always loaded) machinery: importlib.util / .machinery are
        # thin re-exports of it whose import is ~1 ms of a cold start
        import _imp
        from _frozen_importlib import module_from_spec
        from _frozen_importlib_external import ExtensionFileLoader, spec_from_file_location
        for suffix in _imp.extension_suffixes():
            path = os.path.join(NATIVE_DIR, name + suffix)
            if os.path.exists(path):
                spec = spec_from_file_location(name, path, loader=ExtensionFileLoader(name, path))
                if spec is not None and spec.loader is not None:
                    mod = module_from_spec(spec)
                    spec.loader.exec_module(mod)  # type: ignore[union-attr]
                    sys.modules.setdefault(name, mod)
                break
    _cache[key] = mod
    return mod


def load_cdll(filename: str, required: bool = False) -> "Optional[ctypes.CDLL]":
    """Load a C-ABI shared library from ``_native``; raise loudly when ``required``."""
    key = "dll:" + filename
    if key in _cache and _cache[key] is not None:
        return _cache[key]  # type: ignore[return-value]
    import ctypes  # here, not at module level: the checker's CLI path loads only the CPython extension
    path = native_path(filename)
    lib = None
    err = None
    if os.path.exists(path):
        try:
            # RTLD_LOCAL: libamd_smi.so embeds rocm_smi and exports its rsmi_* symbols.  Loaded into the
            # global scope it would interpose librocm_smi64 for every library loaded after it, and
            # librccl (which links librocm_smi64) then crashed in its load-time initialisers
            # (tools/exit_repro.py, MI355X).  Nothing resolves symbols across these libraries.
            lib = ctypes.CDLL(path, mode=getattr(os, "RTLD_NOW", 2) | ctypes.RTLD_LOCAL)
        except OSError as e:  # missing ROCm runtime, wrong arch, ...
            err = e
    else:
        err = FileNotFoundError(path)
    if lib is None and required:
        raise NativeUnavailable(
            f"native library {filename} not available ({err}); build it with "
            f"`python -m k8s_gpu_node_checker_amd.build`")
    _cache[key] = lib
    return lib
