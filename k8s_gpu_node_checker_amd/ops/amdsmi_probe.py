"""Passive MI355X probe front-end (SURVEY §7.1, §7.2 layer 4).

Sources, in order of preference:

``native``   ``libmi355x_probe.so`` (``csrc/probe/probe.cpp``) over libamd_smi:
             amd-smi initialised once per process, ~1-2 ms per GPU per probe.
``python``   the ``amdsmi`` Python binding (same library, ~50 ms import).
``fixture``  a recorded report (CI / hosts without the amdgpu driver).

All return a ``mi355x-health/v1`` dict (:mod:`models.health`).  Driver or
permission problems come back as ``{"error": ...}`` (verdict ``unknown``),
never as an exception.
"""

from __future__ import annotations

import ctypes
import json
import socket
import time
from typing import Any, Dict, Optional

from ..models.health import SCHEMA
from .native import load_cdll

_lib = None


def _native():
    global _lib
    if _lib is None:
        L = load_cdll("libmi355x_probe.so")
        if L is None:
            return None
        L.mi355x_probe_open.restype = ctypes.c_int
        L.mi355x_probe_json.restype = ctypes.c_void_p
        L.mi355x_probe_json.argtypes = [ctypes.c_char_p]
        L.mi355x_probe_free.argtypes = [ctypes.c_void_p]
        L.mi355x_probe_gpu_count.restype = ctypes.c_int
        _lib = L
    return _lib


def native_available() -> bool:
    return _native() is not None


def close() -> None:
    """Shut amd-smi down (the native probe keeps it initialised between probes); the next probe re-opens."""
    if _lib is not None:
        _lib.mi355x_probe_close()


def probe_native(node: str) -> Dict[str, Any]:
    L = _native()
    if L is None:
        raise RuntimeError("libmi355x_probe.so is not built (python -m k8s_gpu_node_checker_amd.build)")
    ptr = L.mi355x_probe_json(node.encode())
    try:
        return json.loads(ctypes.string_at(ptr).decode())
    finally:
        L.mi355x_probe_free(ptr)


def _xgmi_string(status) -> Optional[str]:
    if not isinstance(status, dict):
        return None
    m = {"U": "U", "D": "D", "X": "X"}
    return "".join(m.get(s, "N") for s in status.get("status", []))


def _int(v: Any) -> Optional[int]:
    """amd-smi's Python binding reports unsupported fields as "N/A" or all-ones sentinels."""
    if isinstance(v, bool) or not isinstance(v, int) or v < 0 or v in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF):
        return None
    return v


def _telemetry_python(A: Any, h: Any, q: Any) -> Dict[str, Any]:
    """The native probe's ``probe_telemetry`` fields (csrc/probe/probe.cpp) from the Python binding."""
    t: Dict[str, Any] = {}
    pw = q(A.amdsmi_get_power_info) or {}
    t["power_w"] = _int(pw.get("current_socket_power"))
    cap = q(A.amdsmi_get_power_cap_info) or {}
    for out_key, key in (("power_cap_w", "power_cap"), ("power_cap_default_w", "default_power_cap")):
        v = _int(cap.get(key))
        if v:  # uW on bare-metal Linux (probe.cpp); a binding that already converted gives W
            t[out_key] = v // 1000000 if v > 100000 else v
    hbm = []
    for name in ("HBM_0", "HBM_1", "HBM_2", "HBM_3", "VRAM"):
        try:
            v = A.amdsmi_get_temp_metric(h, getattr(A.AmdSmiTemperatureType, name),
                                         A.AmdSmiTemperatureMetric.CURRENT)
        except Exception:
            continue
        v = _int(v)
        if v and v < 200:
            hbm.append(v)
    vu = q(A.amdsmi_get_gpu_vram_usage) or {}
    t["vram_used_mb"] = _int(vu.get("vram_used"))
    procs = q(A.amdsmi_get_gpu_process_list)
    t["processes"] = len(procs) if isinstance(procs, list) else None
    if procs and isinstance(procs, list):
        t["procs"] = [{"pid": _int(p.get("pid")),
                       "vram_mb": (_int((p.get("memory_usage") or {}).get("vram_mem")) or 0) >> 20}
                      for p in procs[:64] if isinstance(p, dict)]
    act = q(A.amdsmi_get_gpu_activity) or {}
    gfx = _int(act.get("gfx_activity"))
    t["gfx_activity"] = gfx if gfx is not None and gfx <= 100 else None
    m = q(A.amdsmi_get_gpu_metrics_info) or {}
    th = m.get("temperature_hbm")
    hbm += [x for x in (_int(v) for v in th) if x and x < 200] if isinstance(th, list) else []
    t["hbm_temp_c"] = max(hbm) if hbm else None
    clks = m.get("current_gfxclks")
    clks = [x for x in (_int(v) for v in clks) if x] if isinstance(clks, list) else []
    t["gfxclk_mhz"] = sum(clks) // len(clks) if clks else None
    t["xgmi_width"] = _int(m.get("xgmi_link_width")) or None
    t["xgmi_speed_gbps"] = _int(m.get("xgmi_link_speed")) or None
    n = _int(m.get("accumulation_counter"))
    if n:
        acc = {"n": n}
        for k, src in (("prochot", "prochot_residency_acc"), ("ppt", "ppt_residency_acc"),
                       ("socket_thm", "socket_thm_residency_acc"), ("vr_thm", "vr_thm_residency_acc"),
                       ("hbm_thm", "hbm_thm_residency_acc")):
            v = _int(m.get(src))
            if v is not None:
                acc[k] = v
        t["throttle_acc"] = acc
    return {k: v for k, v in t.items() if v is not None}


# csrc/probe/probe.cpp fw_name() and kRasBlocks: the same images and blocks, under the same names
_FW_NAMES = {"SMU": "smu", "PM": "pm", "PSP_SOSDRV": "psp_sos", "CP_MEC1": "mec", "RLC": "rlc", "SDMA0": "sdma",
             "TA_RAS": "ta_ras", "TA_XGMI": "ta_xgmi", "PLDM_BUNDLE": "pldm_bundle"}
_RAS_BLOCKS = ("UMC", "SDMA", "GFX", "MMHUB", "ATHUB", "PCIE_BIF", "HDP", "XGMI_WAFL", "DF", "SMN", "SEM", "MP0",
               "MP1", "FUSE", "MCA", "VCN", "JPEG", "IH", "MPIO")


def _firmware_python(A: Any, h: Any) -> Optional[Dict[str, int]]:
    """Raw firmware versions (integers, as the native probe reports them): the binding's
    ``amdsmi_get_fw_info`` re-formats some of them as dotted strings, so the C struct is read directly."""
    try:
        W = A.amdsmi_interface.amdsmi_wrapper
        info = W.amdsmi_fw_info_t()
        if W.amdsmi_get_fw_info(h, ctypes.byref(info)) != 0:
            return None
        out = {}
        for i in range(min(int(info.num_fw_info), len(info.fw_info_list))):
            e = info.fw_info_list[i]
            name = A.AmdSmiFwBlock(e.fw_id).name.replace("AMDSMI_FW_ID_", "")
            if name in _FW_NAMES and e.fw_version not in (0, 0xFFFFFFFFFFFFFFFF):
                out[_FW_NAMES[name]] = int(e.fw_version)
        return out or None
    except Exception:
        return None


def _ecc_blocks_python(A: Any, h: Any) -> Optional[Dict[str, Dict[str, int]]]:
    out = {}
    for name in _RAS_BLOCKS:
        try:
            c = A.amdsmi_get_gpu_ecc_count(h, getattr(A.AmdSmiGpuBlock, name))
        except Exception:
            continue
        row = {"ce": _int(c.get("correctable_count")) or 0, "ue": _int(c.get("uncorrectable_count")) or 0,
               "de": _int(c.get("deferred_count")) or 0}
        if any(row.values()):
            out[name.lower()] = row
    return out or None


_CPER_SEV = ("uncorrected", "fatal", "corrected")  # amdsmi_cper_sev_t order


def _status_name(W: Any, st: int) -> str:
    """The library's own text for a status (what the native probe's ``status_name`` reports)."""
    try:
        txt = ctypes.POINTER(ctypes.c_char)()
        if W.amdsmi_status_code_to_string(st, ctypes.byref(txt)) == 0 and txt:
            return ctypes.string_at(txt).decode(errors="replace")
    except Exception:
        pass
    return getattr(W, "amdsmi_status_t__enumvalues", {}).get(st, f"AMDSMI_STATUS_{st}")


def _cper_python(A: Any, h: Any) -> Dict[str, Any]:
    """The native probe's ``probe_cper``: RAS error records by severity and the newest of each
    (``cper``), or ``cper_error`` with the status name when they cannot be read (non-root: NO_PERM)."""
    try:
        W = A.amdsmi_interface.amdsmi_wrapper
        hdr_t = W.amdsmi_cper_hdr_t
    except Exception:
        return {}
    count, last = [0, 0, 0], [0, 0, 0]
    buf = ctypes.create_string_buffer(1 << 20)
    hdrs = (ctypes.POINTER(hdr_t) * 64)()
    cursor = ctypes.c_uint64(0)
    for call in range(256):
        size, n = ctypes.c_uint64(len(buf)), ctypes.c_uint64(len(hdrs))
        st = W.amdsmi_get_gpu_cper_entries(h, ctypes.c_uint32(0x7), buf, ctypes.byref(size),
                                           ctypes.cast(hdrs, ctypes.POINTER(ctypes.POINTER(hdr_t))),
                                           ctypes.byref(n), ctypes.byref(cursor))
        if st not in (0, 39):  # SUCCESS, MORE_DATA
            if call == 0:
                return {"cper_error": _status_name(W, st)}
            break
        base, top = ctypes.addressof(buf), ctypes.addressof(buf) + min(size.value, len(buf))
        for i in range(min(n.value, len(hdrs))):
            if not hdrs[i]:
                continue
            addr = ctypes.cast(hdrs[i], ctypes.c_void_p).value or 0
            if addr < base or addr + ctypes.sizeof(hdr_t) > top:
                continue
            hd = hdrs[i].contents
            sev = int(hd.error_severity)
            if not 0 <= sev <= 2:
                continue
            t = hd.timestamp
            year = t.year + 2000 if t.year < 100 else t.year
            stamp = (((((year * 100 + t.month) * 100 + t.day) * 100 + t.hours) * 100 + t.minutes) * 100) + t.seconds
            count[sev] += 1
            last[sev] = max(last[sev], stamp)
        if st != 39:
            break
    out: Dict[str, Any] = {name: count[i] for i, name in enumerate(_CPER_SEV)}
    for i, name in enumerate(_CPER_SEV):
        if count[i]:
            v = f"{last[i]:014d}"
            out[f"last_{name}"] = f"{v[0:4]}-{v[4:6]}-{v[6:8]}T{v[8:10]}:{v[10:12]}:{v[12:14]}Z"
    return {"cper": out}


def _xgmi_fabric_python(A: Any, h: Any, q: Any) -> Dict[str, Any]:
    """The native probe's xGMI fabric fields: hive id, peer BDF and traffic of every XGMI link."""
    out: Dict[str, Any] = {}
    xi = q(A.amdsmi_get_xgmi_info) or {}
    hive = _int(xi.get("xgmi_hive_id"))
    if hive:
        out["xgmi_hive"] = f"{hive:016x}"
    lm = q(A.amdsmi_get_link_metrics)
    if isinstance(lm, dict) and isinstance(lm.get("links"), list):
        peers, kb = [], []
        xgmi_type = int(getattr(getattr(A, "AmdSmiLinkType", None), "XGMI", 2))
        for link in lm["links"]:
            bdf = str(link.get("bdf") or "").lower()
            if int(link.get("link_type", -1)) != xgmi_type or not bdf or bdf.startswith("ffff"):
                continue
            peers.append(bdf)
            kb.append([_int(link.get("read")) or 0, _int(link.get("write")) or 0])
        out["xgmi_peers"], out["xgmi_kb"] = peers, kb
    return out


def _bad_pages_python(A: Any, h: Any, q: Any) -> Dict[str, Any]:
    """The native probe's ``probe_bad_pages`` fields (csrc/probe/probe.cpp): retired pages by status
    (1 = pending, 2 = unreservable), the driver's threshold and the RAS EEPROM checksum (both root-only)."""
    out: Dict[str, Any] = {}
    bp = q(A.amdsmi_get_gpu_bad_page_info)
    out["bad_pages"] = len(bp) if isinstance(bp, list) else None
    if isinstance(bp, list) and bp:
        st = [r.get("status") if isinstance(r, dict) else None for r in bp]
        out["bad_pages_pending"] = sum(1 for s in st if int(s or 0) == 1)
        out["bad_pages_unreservable"] = sum(1 for s in st if int(s or 0) == 2)
    thr = q(A.amdsmi_get_gpu_bad_page_threshold)
    if isinstance(thr, int) and not isinstance(thr, bool):
        out["bad_page_threshold"] = thr
    try:
        A.amdsmi_gpu_validate_ras_eeprom(h)
        out["ras_eeprom"] = "ok"
    except Exception as e:  # AMDSMI_STATUS_CORRUPTED_EEPROM (56); anything else (NO_PERM, ...) = unknown
        code = e.get_error_code() if hasattr(e, "get_error_code") else None
        if code == 56:
            out["ras_eeprom"] = "corrupted"
    return out


def probe_python(node: str) -> Dict[str, Any]:
    rep: Dict[str, Any] = {"schema": SCHEMA, "node": node, "ts": time.time(), "probe": "python", "gpus": []}
    t0 = time.perf_counter()
    try:
        import amdsmi as A
        A.amdsmi_init()
    except Exception as e:
        rep["error"] = f"amdsmi init: {e}"
        return rep
    try:
        handles = A.amdsmi_get_processor_handles()
        try:
            drv = A.amdsmi_get_gpu_driver_info(handles[0]) if handles else {}
            if drv.get("driver_version") not in (None, "", "N/A"):
                rep["driver"] = {"name": drv.get("driver_name"), "version": drv.get("driver_version")}
        except Exception:
            pass
        for i, h in enumerate(handles):
            g: Dict[str, Any] = {"index": i}

            def q(fn, *a):
                try:
                    return fn(h, *a)
                except Exception:
                    return None
            asic = q(A.amdsmi_get_gpu_asic_info)
            if not asic:
                g["error"] = "asic info unavailable"
                rep["gpus"].append(g)
                continue
            g.update({"bdf": q(A.amdsmi_get_gpu_device_bdf), "uuid": q(A.amdsmi_get_gpu_device_uuid),
                      "gfx": asic.get("target_graphics_version"), "market_name": asic.get("market_name"),
                      "device_id": asic.get("device_id"), "cus": asic.get("num_compute_units")})
            board = q(A.amdsmi_get_gpu_board_info) or {}
            g["product_name"] = board.get("product_name")
            vb = q(A.amdsmi_get_gpu_vbios_info) or {}
            g["vbios_name"] = vb.get("name")
            g["vbios_version"] = vb.get("version") or None
            g["fw"] = _firmware_python(A, h)
            vram = q(A.amdsmi_get_gpu_vram_info) or {}
            g["vram_type"], g["vram_mb"] = vram.get("vram_type"), vram.get("vram_size")
            ecc = q(A.amdsmi_get_gpu_total_ecc_count)
            if ecc:
                g.update({"ecc_correctable": ecc.get("correctable_count"),
                          "ecc_uncorrectable": ecc.get("uncorrectable_count"),
                          "ecc_deferred": ecc.get("deferred_count")})
                if any(_int(ecc.get(k)) for k in ("correctable_count", "uncorrectable_count", "deferred_count")):
                    g["ecc_blocks"] = _ecc_blocks_python(A, h)
            g.update(_bad_pages_python(A, h, q))
            g.update(_cper_python(A, h))
            g["xgmi"] = _xgmi_string(q(A.amdsmi_get_gpu_xgmi_link_status))
            xe = q(A.amdsmi_gpu_xgmi_error_status)
            g["xgmi_error"] = int(xe) if xe is not None else None
            g.update(_xgmi_fabric_python(A, h, q))
            kfd = q(A.amdsmi_get_gpu_kfd_info) or {}
            g["kfd"] = bool(kfd.get("kfd_id") not in (None, "N/A"))
            g["compute_partition"] = q(A.amdsmi_get_gpu_compute_partition)
            g["memory_partition"] = q(A.amdsmi_get_gpu_memory_partition)
            try:
                g["hotspot_c"] = A.amdsmi_get_temp_metric(h, A.AmdSmiTemperatureType.HOTSPOT,
                                                          A.AmdSmiTemperatureMetric.CURRENT)
            except Exception:
                pass
            pcie = q(A.amdsmi_get_pcie_info) or {}
            pst, pmt = pcie.get("pcie_static") or {}, pcie.get("pcie_metric") or {}
            for out_key, src, key in (("pcie_width", pmt, "pcie_width"), ("pcie_max_width", pst, "max_pcie_width"),
                                      ("pcie_speed_mts", pmt, "pcie_speed"),
                                      ("pcie_max_speed_mts", pst, "max_pcie_speed"),
                                      ("pcie_replays", pmt, "pcie_replay_count"),
                                      ("pcie_recoveries", pmt, "pcie_l0_to_recovery_count")):
                if isinstance(src.get(key), int):
                    g[out_key] = src[key]
            g.update(_telemetry_python(A, h, q))
            rep["gpus"].append({k: v for k, v in g.items() if v is not None})
    finally:
        rep["probe_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    return rep


def probe_fixture(path: str, node: str) -> Dict[str, Any]:
    with open(path, encoding="utf-8") as f:
        rep = json.load(f)
    rep["node"] = node
    rep["ts"] = time.time()
    rep.setdefault("schema", SCHEMA)
    rep["probe"] = "fixture"
    return rep


def probe(node: Optional[str] = None, source: str = "auto", fixture: Optional[str] = None) -> Dict[str, Any]:
    node = node or socket.gethostname()
    if source == "fixture" or (source == "auto" and fixture):
        if not fixture:
            raise ValueError("fixture source needs a path")
        return probe_fixture(fixture, node)
    if source == "native" or (source == "auto" and native_available()):
        return probe_native(node)
    return probe_python(node)
