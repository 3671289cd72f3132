"""MI355X health model: probe-report schema, verdicts and the Ready gate.

The reference's only failure signal is NodeCondition ``Ready`` plus "GPU
capacity > 0" (``check-gpu-node.py:172-196``).  It cannot see a node whose
kubelet is fine but whose accelerators are not: a GPU that fell off the bus,
uncorrectable HBM ECC errors, a downed xGMI link, a partition-mode change
that halves the visible VRAM.  The MI355X node agent (``agent/``) runs the
native amd-smi probe (``csrc/probe``) and publishes a compact report as the
node annotation ``amd.com/mi355x-health``; the checker evaluates it here.

Expectations, measured on a real MI355X via ``gpurun`` (amd-smi 26.2.1,
``profiles/amdsmi_mi355x.json``): ``target_graphics_version=gfx950``,
``market_name="AMD Instinct MI355 OAM"``, ``vram_type=5`` (HBM3E),
``vram_size=294896`` MB in SPX/NPS1, xGMI ``status=["X","U"x7]`` (7 of 8
ports Up, one disabled), 256 CUs.

Verdicts: ``healthy`` / ``degraded`` (warnings only, still schedulable) /
``unhealthy`` / ``unknown`` (no report, stale report, or the probe could not
run: driver not loaded, no permission).
"""

from __future__ import annotations

import io
import math
import time
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Dict, List, Optional, Sequence, Tuple

SCHEMA = "mi355x-health/v1"

# --- MI355X / gfx950 expectations (CDNA4) ------------------------------------
GFX_TARGET = "gfx950"
PRODUCT_TOKENS = ("MI355", "MI350")          # product / market / vbios names on gfx950 parts
MI35X_DEVICE_IDS = frozenset(("0x75a3",))     # measured: MI355X OAM (amd-smi DEVICE_ID)
HBM3E_VRAM_TYPE = 5                           # amdsmi.h AMDSMI_VRAM_TYPE_HBM3E
VRAM_MB_FULL = 294896                         # measured vram_size, SPX/NPS1 (288 GB class)
VRAM_MIN_FRACTION = 0.97
XGMI_LINKS_EXPECTED = 7                       # 8-GPU hive: 7 peers per GPU
XGMI_LINK_WIDTH = 16                          # measured: lanes per trained xGMI link
XGMI_LINK_GBPS = 38                           # measured: Gb/s per lane (x16 -> 608 Gb/s, 76 GB/s each way)
NUM_CUS = 256
HOTSPOT_WARN_C = 100
HBM_TEMP_WARN_C = 95                          # HBM3E stacks throttle in the 95-105 C band
PCIE_REPLAY_WARN = 10000                      # link-level retries since boot: a marginal slot or riser
POWER_CAP_MIN_FRACTION = 0.9                  # a cap set below 90 % of the board default
THERMAL_THROTTLE_WARN_PCT = 10.0              # share of a probe interval spent thermally throttled
PROCHOT_WARN_PCT = 1.0                        # PROCHOT is an emergency throttle: any sustained share counts

HEALTHY, DEGRADED, UNHEALTHY, UNKNOWN = "healthy", "degraded", "unhealthy", "unknown"
_OK_STATES = (HEALTHY, DEGRADED)


class HealthExpectations:
    """Tunable thresholds (CLI flags map onto these)."""

    def __init__(self, xgmi_links: int = XGMI_LINKS_EXPECTED, max_age_s: float = 900.0,
                 require_product: bool = True, vram_min_fraction: float = VRAM_MIN_FRACTION,
                 bad_page_limit: int = 64, correctable_warn: int = 1000, cper_window_s: float = 86400.0,
                 ce_rate_warn_per_h: float = 60.0):
        self.xgmi_links = xgmi_links
        self.max_age_s = max_age_s
        self.require_product = require_product
        self.vram_min_fraction = vram_min_fraction
        self.bad_page_limit = bad_page_limit
        self.correctable_warn = correctable_warn
        #: a fatal CPER record newer than this (s, against the report's time) makes the GPU unhealthy
        self.cper_window_s = cper_window_s
        #: correctable ECC errors per hour (the agent's ``ecc_ce_per_h`` over its last hour of probes) at which a
        #: GPU is "degraded": a steady trickle of corrected HBM errors is normal, a burst is a part going bad
        #: before it ever reports an uncorrectable one
        self.ce_rate_warn_per_h = ce_rate_warn_per_h


class Verdict:
    __slots__ = ("state", "reasons", "warnings", "gpus_ok", "gpus_seen", "age_s")

    def __init__(self, state: str, reasons: Optional[List[str]] = None, warnings: Optional[List[str]] = None,
                 gpus_ok: int = 0, gpus_seen: int = 0, age_s: Optional[float] = None):
        self.state = state
        self.reasons = reasons or []
        self.warnings = warnings or []
        self.gpus_ok = gpus_ok
        self.gpus_seen = gpus_seen
        self.age_s = age_s

    @property
    def ok(self) -> bool:
        return self.state in _OK_STATES

    def short(self) -> str:
        if self.state == HEALTHY:
            return f"MI355X {self.gpus_ok}/{self.gpus_seen} healthy" if self.gpus_seen else "MI355X healthy"
        detail = "; ".join(self.reasons or self.warnings)
        return f"MI355X {self.state}" + (f": {detail}" if detail else "")

    def to_dict(self) -> Dict[str, Any]:
        d: Dict[str, Any] = {"state": self.state, "gpus_ok": self.gpus_ok, "gpus_seen": self.gpus_seen}
        if self.reasons:
            d["reasons"] = self.reasons
        if self.warnings:
            d["warnings"] = self.warnings
        if self.age_s is not None:
            d["age_s"] = round(self.age_s, 1)
        return d


def is_mi35x(g: Dict[str, Any]) -> bool:
    """Identify an MI355X/MI350X from any of the names amd-smi reports, or its PCI device id.

    ``market_name`` comes from libdrm's ``amdgpu.ids`` and degrades to "AMD
    Radeon Graphics" when another libdrm copy (e.g. PyTorch's) is loaded first;
    the FRU ``product_name`` and the VBIOS name do not.
    """
    names = " ".join(str(g.get(k) or "") for k in ("product_name", "market_name", "vbios_name"))
    if any(t in names for t in PRODUCT_TOKENS):
        return True
    return str(g.get("device_id", "")).lower() in MI35X_DEVICE_IDS


def _nps(mem_partition: Any) -> int:
    if isinstance(mem_partition, str) and mem_partition.upper().startswith("NPS"):
        try:
            return max(1, int(mem_partition[3:]))
        except ValueError:
            return 1
    return 1


def _num(x: Any) -> float:
    return float(x) if isinstance(x, (int, float)) and not isinstance(x, bool) else 0.0


def throttle_window(prev: Optional[Dict[str, Any]], cur: Optional[Dict[str, Any]],
                    seconds: float) -> Optional[Dict[str, Any]]:
    """Share of the interval between two probes spent throttled, from the firmware's residency
    accumulators (``throttle_acc`` of two consecutive reports; amd-smi's PVIOL / TVIOL formula:
    delta residency * 100 / delta accumulation counter).

    ``thermal_pct`` is the largest of the socket, voltage-regulator and HBM thermal throttlers;
    ``power_pct`` is package-power tracking, the normal operating point of an MI355X under full
    MFMA load (reported, never a warning); ``prochot_pct`` is the emergency throttle.  ``None``
    when either sample is missing or the counters went backwards (driver reload).
    """
    if not isinstance(prev, dict) or not isinstance(cur, dict):
        return None
    dn = _num(cur.get("n")) - _num(prev.get("n"))
    if dn <= 0:
        return None

    def pct(*keys: str) -> Optional[float]:
        vals = []
        for k in keys:
            if isinstance(cur.get(k), int) and isinstance(prev.get(k), int):
                d = cur[k] - prev[k]
                if d < 0:
                    return None
                vals.append(min(100.0, d * 100.0 / dn))
        return round(max(vals), 2) if vals else None
    out: Dict[str, Any] = {"s": round(seconds, 1)}
    for name, keys in (("thermal_pct", ("socket_thm", "vr_thm", "hbm_thm")), ("power_pct", ("ppt",)),
                       ("prochot_pct", ("prochot",))):
        v = pct(*keys)
        if v is not None:
            out[name] = v
    return out if len(out) > 1 else None


#: amdsmi_xgmi_status_t
XGMI_ERROR_STATUS = {0: "no errors", 1: "errors", 2: "multiple errors"}


def _by_block(blocks: Dict[str, Any], kind: str) -> str:
    """`` (umc 3, xgmi_wafl 1)``: the RAS blocks an ECC count comes from (probe ``ecc_blocks``)."""
    parts = [f"{name} {c[kind]}" for name, c in blocks.items()
             if isinstance(c, dict) and isinstance(c.get(kind), int) and c[kind] > 0]
    return f" ({', '.join(parts)})" if parts else ""


_FW_HEX = frozenset(("psp_sos", "ta_ras", "ta_xgmi"))
_FW_DEC = frozenset(("pm", "pldm_bundle"))


def fw_version_str(name: str, v: Any) -> str:
    """A firmware version as ``amd-smi firmware`` prints it: the security-processor images as dotted hex
    bytes (``00.45.00.2F``), PM firmware and the PLDM bundle as dotted decimal bytes (``04.86.15.106``),
    the rest as the plain number."""
    if not isinstance(v, int) or isinstance(v, bool) or v < 0:
        return str(v)
    if name in _FW_HEX or name in _FW_DEC:
        h = f"{v:08x}"
        parts = [h[i:i + 2] for i in range(0, len(h), 2)]
        if name in _FW_HEX:
            return ".".join(parts).upper()
        return ".".join(f"{int(b, 16):02d}" for b in parts)
    return str(v)


def driver_release(version: Any) -> str:
    """The amdgpu driver version as a release string: a DKMS driver reports its own (``6.10.5``); an
    in-tree one reports the kernel's uname with the spaces removed (``Linuxversion6.18.54-ant.1(nixbld@
    ...)#1...``, measured on the MI355X box), of which the kernel release is kept (``6.18.54-ant.1``)."""
    v = str(version or "")
    if not v or v[0].isdigit():
        return v
    i = next((k for k, c in enumerate(v) if c.isdigit()), -1)
    if i < 0:
        return v
    j = i
    while j < len(v) and (v[j].isalnum() or v[j] in ".-"):
        j += 1
    return v[i:j].rstrip(".-") or v


def firmware_mismatch(gpus: Sequence[Any]) -> List[str]:
    """Firmware images whose version differs between the GPUs of one node (probe ``fw``).

    The GPUs of a node are flashed as one bundle; two versions of the same image on one node mean an
    update that stopped half-way, and GPUs that will behave differently under the same job.  One entry
    per image: ``psp_sos: gpu0-6 00.45.00.2F, gpu7 00.45.00.00``; versions are stable, so the condition
    message stays stable probe to probe."""
    fws = [g["fw"] for g in gpus if isinstance(g, dict) and isinstance(g.get("fw"), dict)]
    if not fws or all(f == fws[0] for f in fws):
        return []  # the common case, settled by dict equality
    seen: Dict[str, Dict[Any, List[Any]]] = {}
    for g in gpus:
        if not isinstance(g, dict) or not isinstance(g.get("fw"), dict):
            continue
        for name, ver in g["fw"].items():
            seen.setdefault(name, {}).setdefault(ver, []).append(g.get("index", "?"))
    out = []
    for name in sorted(seen):
        vers = seen[name]
        if len(vers) > 1:
            groups = sorted(vers.items(), key=lambda kv: (-len(kv[1]), str(kv[0])))
            out.append(f"{name}: " + ", ".join(f"gpu{_span(ix)} {fw_version_str(name, v)}" for v, ix in groups))
    return out


_BDF_CACHE: Dict[Any, str] = {}


def _bdf(b: Any) -> str:
    """PCI address, normalised (lower case, domain added); memoised: the same few addresses recur on every
    GPU of every node of a fleet (1000 8-GPU reports carry ~0.5 M of them)."""
    try:
        return _BDF_CACHE[b]
    except (KeyError, TypeError):
        pass
    n = str(b or "").strip().lower()
    n = "0000:" + n if n.count(":") == 1 else n
    if isinstance(b, str) and len(_BDF_CACHE) < 65536:
        _BDF_CACHE[b] = n
    return n


def xgmi_topology(gpus: Sequence[Any], links_expected: int) -> List[str]:
    """Node-level xGMI wiring from the probe's ``xgmi_hive`` and ``xgmi_peers`` (amd-smi link metrics).

    * Every GPU of an 8-GPU board belongs to one hive; GPUs reporting two hive ids cannot run a
      collective over xGMI together (a board that came up split).
    * With the whole board visible (``links_expected + 1`` unpartitioned GPUs), each GPU's Up links
      must reach every other GPU of the node once: a link wired or trained to the wrong peer, or two
      links to the same one, leaves some pair without its direct link -- traffic between them detours
      through a third GPU at half the bandwidth, while every link still reads "Up".
    """
    if links_expected <= 0:
        return []
    gs = [g for g in gpus if isinstance(g, dict) and not g.get("error")]
    out: List[str] = []
    hives: Dict[str, List[Any]] = {}
    for g in gs:
        if isinstance(g.get("xgmi_hive"), str) and g["xgmi_hive"]:
            hives.setdefault(g["xgmi_hive"], []).append(g.get("index", "?"))
    if len(hives) > 1:
        groups = sorted(hives.items(), key=lambda kv: (-len(kv[1]), kv[0]))
        out.append(f"GPUs span {len(hives)} xGMI hives: " + ", ".join(f"gpu{_span(ix)} {h}" for h, ix in groups))
    bdfs = {_bdf(g.get("bdf")): g for g in gs if g.get("bdf")}
    full_board = len(bdfs) == links_expected + 1 and all(
        str(g.get("compute_partition") or "SPX").upper() == "SPX" for g in gs)
    if not full_board:
        return out
    peer_sets = {me: {_bdf(p) for p in g["xgmi_peers"]} for me, g in bdfs.items()
                 if isinstance(g.get("xgmi_peers"), list)}
    board = set(bdfs)
    # a VM that remaps the GPUs' PCI addresses sees its links name host addresses none of its GPUs
    # carry: nothing to match the wiring against, so it is not judged
    if not any(ps & board for ps in peer_sets.values()):
        return out
    for me, ps in peer_sets.items():
        g = bdfs[me]
        reached = ps & (board - {me})
        foreign = sorted(ps - board)
        if len(reached) < links_expected:
            missing = sorted(board - reached - {me})
            out.append(f"gpu{g.get('index', '?')}: xGMI links reach {len(reached)} of the node's {len(bdfs) - 1} "
                       f"other GPUs (no link to {', '.join(missing[:3])}{' ...' if len(missing) > 3 else ''})"
                       + (f", {len(foreign)} to devices outside the node" if foreign else ""))
    return out


def partition_mismatch(gpus: Sequence[Any]) -> List[str]:
    """Compute / memory partition modes that differ between the GPUs of one node.  An 8-GPU board is
    partitioned as a whole (the device plugin advertises one resource shape per node); one GPU left in
    another mode after a repartition hands the scheduler devices of two sizes under one name."""
    out = []
    for key, name in (("compute_partition", "compute"), ("memory_partition", "memory")):
        modes = {g[key] for g in gpus if isinstance(g, dict) and isinstance(g.get(key), str) and g[key]}
        if len(modes) < 2:
            continue  # the common case: one mode across the node
        seen: Dict[str, List[Any]] = {}
        for g in gpus:
            if isinstance(g, dict) and isinstance(g.get(key), str) and g[key]:
                seen.setdefault(g[key], []).append(g.get("index", "?"))
        if len(seen) > 1:
            groups = sorted(seen.items(), key=lambda kv: (-len(kv[1]), kv[0]))
            out.append(f"{name}: " + ", ".join(f"gpu{_span(ix)} {mode}" for mode, ix in groups))
    return out


def _span(ix: List[Any]) -> str:
    """GPU indices as runs: [0, 1, 2, 4, 6, 7] -> "0-2,4,6-7" (non-integers listed as they are)."""
    if not all(isinstance(i, int) for i in ix):
        return ",".join(str(i) for i in ix)
    runs: List[List[int]] = []
    for i in ix:
        if runs and i == runs[-1][1] + 1:
            runs[-1][1] = i
        else:
            runs.append([i, i])
    return ",".join(f"{a}-{b}" if b > a else f"{a}" for a, b in runs)


def _age_s(stamp: Any, now: Optional[float]) -> Optional[float]:
    """Seconds since an RFC 3339 ``...Z`` timestamp (None when either is missing or unparseable)."""
    t = parse_k8s_time(stamp) if isinstance(stamp, str) else None
    return None if t is None or now is None else now - t


def evaluate_gpu(g: Dict[str, Any], exp: HealthExpectations, now: Optional[float] = None,
                 fleet: Optional[Dict[str, Any]] = None) -> Tuple[List[str], List[str]]:
    """Return ``(failures, warnings)`` for one GPU entry of a probe report (``now``: the report's time,
    against which record timestamps are aged; ``fleet``: the node's fleet view, ``models/fleet.py``)."""
    fail: List[str] = []
    warn: List[str] = []
    idx = g.get("index", "?")
    if g.get("error"):
        fail.append(f"gpu{idx}: probe error {g['error']}")
        return fail, warn
    gfx = g.get("gfx")
    if gfx != GFX_TARGET:
        fail.append(f"gpu{idx}: target {gfx!r} is not {GFX_TARGET}")
    if exp.require_product and not is_mi35x(g):
        fail.append(f"gpu{idx}: product {g.get('product_name') or g.get('market_name')!r} is not MI355X/MI350X")
    vt = g.get("vram_type")
    if vt is not None and vt != HBM3E_VRAM_TYPE and vt != "HBM3E":
        fail.append(f"gpu{idx}: VRAM type {vt} is not HBM3E")
    vram = g.get("vram_mb")
    if isinstance(vram, (int, float)):
        need = VRAM_MB_FULL / _nps(g.get("memory_partition")) * exp.vram_min_fraction
        if vram < need:
            fail.append(f"gpu{idx}: VRAM {vram} MB < {need:.0f} MB expected")
    blocks = g.get("ecc_blocks") if isinstance(g.get("ecc_blocks"), dict) else {}
    ue = g.get("ecc_uncorrectable")
    if isinstance(ue, int) and ue > 0:
        fail.append(f"gpu{idx}: {ue} uncorrectable ECC errors{_by_block(blocks, 'ue')}")
    de = g.get("ecc_deferred")
    if isinstance(de, int) and de > 0:
        warn.append(f"gpu{idx}: {de} deferred ECC errors{_by_block(blocks, 'de')}")
    ce = g.get("ecc_correctable")
    if isinstance(ce, int) and ce > exp.correctable_warn:
        warn.append(f"gpu{idx}: {ce} correctable ECC errors{_by_block(blocks, 'ce')}")
    rate = g.get("ecc_ce_per_h")
    if isinstance(rate, (int, float)) and not isinstance(rate, bool) and rate >= exp.ce_rate_warn_per_h > 0:
        warn.append(f"gpu{idx}: correctable ECC errors rising at {rate:.0f}/h{_by_block(blocks, 'ce')}")
    cper = g.get("cper")
    if isinstance(cper, dict):
        # the driver's RAS error records (since it loaded): a recent fatal one means the GPU went through
        # an error reset -- drain and look; an older one is history worth showing
        fatal, last = cper.get("fatal"), cper.get("last_fatal")
        if isinstance(fatal, int) and fatal > 0:
            age = _age_s(last, now)
            if age is None or age <= exp.cper_window_s:
                fail.append(f"gpu{idx}: fatal RAS error record (CPER) at {last or '?'}")
            else:
                warn.append(f"gpu{idx}: {fatal} fatal RAS error record(s) since driver load, last {last}")
        unc, last_u = cper.get("uncorrected"), cper.get("last_uncorrected")
        if isinstance(unc, int) and unc > 0:
            age = _age_s(last_u, now)
            if age is None or age <= exp.cper_window_s:
                warn.append(f"gpu{idx}: uncorrected non-fatal RAS error record (CPER) at {last_u or '?'}")
    bp = g.get("bad_pages")
    if isinstance(bp, int):
        # the driver's own retirement threshold when the probe could read it (root), else the fixed limit;
        # past 90 % of the threshold the GPU is a reset or two from being declared bad by the driver
        thr = g.get("bad_page_threshold")
        limit = thr if isinstance(thr, int) and thr > 0 else None
        if limit is not None and bp >= limit:
            fail.append(f"gpu{idx}: {bp} retired pages reached the driver's threshold {limit}")
        elif limit is None and bp > exp.bad_page_limit:
            fail.append(f"gpu{idx}: {bp} retired pages > {exp.bad_page_limit}")
        elif limit is not None and bp >= 0.9 * limit:
            warn.append(f"gpu{idx}: {bp} retired pages, {limit} is the driver's threshold")
        elif bp > 0:
            warn.append(f"gpu{idx}: {bp} retired pages")
    unres, pend = g.get("bad_pages_unreservable"), g.get("bad_pages_pending")
    if isinstance(unres, int) and unres > 0:
        fail.append(f"gpu{idx}: {unres} bad HBM page(s) could not be retired (still in use)")
    if isinstance(pend, int) and pend > 0:
        warn.append(f"gpu{idx}: {pend} bad HBM page(s) pending retirement (retired at the next GPU reset)")
    if g.get("ras_eeprom") == "corrupted":
        fail.append(f"gpu{idx}: RAS EEPROM checksum invalid (the retired-page list may not survive a reboot)")
    links = g.get("xgmi")
    if isinstance(links, str) and exp.xgmi_links > 0:
        up, down = links.count("U"), links.count("D")
        if down:
            fail.append(f"gpu{idx}: {down} xGMI link(s) down ({links})")
        elif up < exp.xgmi_links and str(g.get("compute_partition") or "SPX").upper() == "SPX":
            # the link count is a property of the whole GPU; how a compute partition (DPX..CPX) of it reports
            # the shared links was not observable here (no partitioned MI355X), so partitions are judged on
            # Down links only
            fail.append(f"gpu{idx}: {up}/{exp.xgmi_links} xGMI links up ({links})")
    if isinstance(links, str) and "U" in links and exp.xgmi_links > 0:
        w, sp = g.get("xgmi_width"), g.get("xgmi_speed_gbps")
        if (isinstance(w, int) and 0 < w < XGMI_LINK_WIDTH) or (isinstance(sp, int) and 0 < sp < XGMI_LINK_GBPS):
            # still "Up", but retrained narrower or slower: every collective through it runs at that rate
            trained = " ".join(x for x in (f"x{w}" if isinstance(w, int) else "",
                                           f"{sp} Gb/s" if isinstance(sp, int) else "") if x)
            warn.append(f"gpu{idx}: xGMI links trained at {trained} (MI355X: x{XGMI_LINK_WIDTH} {XGMI_LINK_GBPS} Gb/s)")
    xe = g.get("xgmi_error")
    if isinstance(xe, int) and xe > 0 and exp.xgmi_links > 0:
        # sticky since the driver loaded: the link PHYs retried or dropped traffic at least once
        warn.append(f"gpu{idx}: xGMI error status {XGMI_ERROR_STATUS.get(xe, xe)}")
    if g.get("kfd") is False:
        fail.append(f"gpu{idx}: no KFD node (not usable by ROCm)")
    cus = g.get("cus")
    if isinstance(cus, int) and g.get("compute_partition", "SPX") == "SPX" and 0 < cus < NUM_CUS:
        fail.append(f"gpu{idx}: {cus} CUs < {NUM_CUS}")
    t = g.get("hotspot_c")
    if isinstance(t, (int, float)) and t >= HOTSPOT_WARN_C:
        warn.append(f"gpu{idx}: hotspot {t} C")
    t = g.get("hbm_temp_c")
    if isinstance(t, (int, float)) and t >= HBM_TEMP_WARN_C:
        warn.append(f"gpu{idx}: HBM {t} C")
    cap, dflt = g.get("power_cap_w"), g.get("power_cap_default_w")
    if isinstance(cap, int) and isinstance(dflt, int) and 0 < cap < POWER_CAP_MIN_FRACTION * dflt:
        warn.append(f"gpu{idx}: power cap {cap} W of {dflt} W default")
    tw = g.get("throttle")
    if isinstance(tw, dict):
        # numbers stay out of the text: the condition message must not change with every probe
        if _num(tw.get("thermal_pct")) >= THERMAL_THROTTLE_WARN_PCT:
            warn.append(f"gpu{idx}: thermally throttled >= {THERMAL_THROTTLE_WARN_PCT:g}% of the last probe interval")
        if _num(tw.get("prochot_pct")) >= PROCHOT_WARN_PCT:
            warn.append(f"gpu{idx}: PROCHOT asserted >= {PROCHOT_WARN_PCT:g}% of the last probe interval")
    w, mw = g.get("pcie_width"), g.get("pcie_max_width")
    if isinstance(w, int) and isinstance(mw, int) and 0 < w < mw:
        warn.append(f"gpu{idx}: PCIe link x{w} of x{mw}")
    rp = g.get("pcie_replays")
    if isinstance(rp, int) and rp >= PCIE_REPLAY_WARN:
        warn.append(f"gpu{idx}: {rp} PCIe replays")
    diag = g.get("diag")
    if isinstance(diag, dict):
        for test, res in diag.items():
            if isinstance(res, dict) and res.get("pass") is False:
                detail = res.get("detail") or ""
                fail.append(f"gpu{idx}: diag {test} failed" + (f" ({detail})" if detail else ""))
            elif isinstance(res, dict) and res.get("degraded"):  # 85-95 % of its reference rate (ops/diag.py)
                if fleet:
                    from .fleet import explains_gpu_result
                    if explains_gpu_result(fleet, test, res, g):
                        continue  # slow alike with the whole fleet: the platform's normal (models/fleet.py)
                detail = res.get("detail") or ""
                warn.append(f"gpu{idx}: diag {test} slow" + (f" ({detail})" if detail else ""))
    return fail, warn


def report_gpus(report: Any) -> List[Any]:
    """The ``gpus`` list of a report, or [] when the report (untrusted JSON) has none or something else there."""
    g = report.get("gpus") if isinstance(report, dict) else None
    return g if isinstance(g, list) else []


def report_gate(report: Any, exp: Optional[HealthExpectations] = None,
                now: Optional[float] = None) -> Optional[Verdict]:
    """The ``unknown`` verdict for a report that cannot be judged at all -- none, not a JSON object, another
    schema, stale or from the future, a failed probe, a malformed ``gpus`` -- else None (judge it)."""
    try:
        return _report_gate(report, exp or HealthExpectations(), now)
    except (TypeError, ValueError, AttributeError, KeyError, IndexError, OverflowError) as e:
        return Verdict(UNKNOWN, [f"malformed probe report ({type(e).__name__}: {str(e)[:80]})"])


def _report_gate(report: Any, exp: HealthExpectations, now: Optional[float]) -> Optional[Verdict]:
    if not report:
        return Verdict(UNKNOWN, ["no probe report"])
    if not isinstance(report, dict):
        return Verdict(UNKNOWN, [f"malformed probe report (a JSON {type(report).__name__}, not an object)"])
    if report.get("schema") != SCHEMA:
        return Verdict(UNKNOWN, [f"unsupported probe schema {report.get('schema')!r}"])
    now = time.time() if now is None else now
    ts = report.get("ts")
    age = (now - float(ts)) if isinstance(ts, (int, float)) and math.isfinite(ts) else None
    if age is None or age > exp.max_age_s:
        return Verdict(UNKNOWN, ["stale probe report" if age is not None else "probe report has no timestamp"],
                       age_s=age)
    if age < -exp.max_age_s:
        # from further in the future than a report may be old: the agent's clock (or the report) is wrong, and
        # such a report would otherwise count as fresh for as long as the clocks disagree
        return Verdict(UNKNOWN, [f"probe report is {-age:.0f} s in the future (clock skew?)"], age_s=age)
    if report.get("error"):
        return Verdict(UNKNOWN, [f"probe failed: {report['error']}"], age_s=age)
    gpus = report.get("gpus") or []
    if not isinstance(gpus, list):
        return Verdict(UNKNOWN, [f"malformed probe report (gpus is a JSON {type(gpus).__name__})"], age_s=age)
    return None


def evaluate_report(report: Optional[Dict[str, Any]], expected_gpus: int,
                    exp: Optional[HealthExpectations] = None, now: Optional[float] = None,
                    fleet: Optional[Dict[str, Any]] = None) -> Verdict:
    """The verdict on one probe report.  A report is untrusted input (an agent endpoint, an annotation): one
    whose fields have the wrong types is ``unknown`` with the reason, never an exception out of the check.
    ``fleet`` is this node's view from ``models/fleet.judge_fleet`` (the checker's fleet-relative judgement)."""
    try:
        return _evaluate_report(report, expected_gpus, exp, now, fleet)
    except (TypeError, ValueError, AttributeError, KeyError, IndexError, OverflowError) as e:
        return Verdict(UNKNOWN, [f"malformed probe report ({type(e).__name__}: {str(e)[:80]})"])


def _evaluate_report(report: Optional[Dict[str, Any]], expected_gpus: int,
                     exp: Optional[HealthExpectations] = None, now: Optional[float] = None,
                     fleet: Optional[Dict[str, Any]] = None) -> Verdict:
    exp = exp or HealthExpectations()
    gate = report_gate(report, exp, now)
    if gate is not None:
        return gate
    now = time.time() if now is None else now
    ts = report["ts"]  # type: ignore[index]
    age = now - float(ts)
    gpus = report.get("gpus") or []  # type: ignore[union-attr]
    fails: List[str] = []
    warns: List[str] = []
    ok = 0
    for g in gpus:
        if not isinstance(g, dict):
            continue
        f, w = evaluate_gpu(g, exp, float(ts) if isinstance(ts, (int, float)) else now, fleet)
        fails += f
        warns += w
        ok += 0 if f else 1
    if expected_gpus and len(gpus) < expected_gpus:
        fails.append(f"{len(gpus)} of {expected_gpus} GPUs visible to amd-smi")
    fails += xgmi_topology(gpus, exp.xgmi_links)
    mism = firmware_mismatch(gpus)
    if mism:
        warns.append("firmware differs across GPUs: " + "; ".join(mism))
    modes = partition_mismatch(gpus)
    if modes:
        warns.append("partition modes differ across GPUs: " + "; ".join(modes))
    node_diag = report.get("diag_node")
    if isinstance(node_diag, dict) and isinstance(node_diag.get("findings"), list):
        # every GPU of the node slow alike (models/peers.judge_node): the node's condition, a warning, never a
        # GPU failure
        from .peers import finding_text
        from .fleet import explains_node_finding
        warns += [finding_text(f) for f in node_diag["findings"]
                  if isinstance(f, dict) and not explains_node_finding(fleet, f)]
    if fleet and fleet.get("findings"):
        # the node against the fleet's other nodes (models/fleet.judge_fleet, in the checker): a warning too
        from .fleet import finding_text as fleet_text
        warns += [fleet_text(f) for f in fleet["findings"]]
    fabric = report.get("fabric")
    if isinstance(fabric, dict):
        for test, res in fabric.items():  # node-level: the xGMI pair matrix (ops/diag.p2p_matrix)
            if isinstance(res, dict) and res.get("pass") is False:
                detail = res.get("detail") or ""
                fails.append(f"xGMI {test} failed" + (f" ({detail})" if detail else ""))
    state = UNHEALTHY if fails else (DEGRADED if warns else HEALTHY)
    return Verdict(state, fails, warns, gpus_ok=ok, gpus_seen=len(gpus), age_s=age)


# --- NodeCondition path (node-problem-detector style) -------------------------
#: Node condition the agent maintains via PATCH /api/v1/nodes/{name}/status.
from .node import HEALTH_CONDITION  # noqa: E402  (single definition)
_REASON = {HEALTHY: "MI355XHealthy", DEGRADED: "MI355XDegraded", UNHEALTHY: "MI355XUnhealthy",
           UNKNOWN: "MI355XProbeFailed"}
_STATE_OF_REASON = {v: k for k, v in _REASON.items()}

#: Taint the agent keeps on its node while the verdict is unhealthy (``--taint-unhealthy``) and removes on
#: recovery: the scheduler stops placing new pods there.  NoSchedule only -- running jobs are left alone,
#: evicting them is an operator's decision.  The checker's ``--require-schedulable`` reads it back.
UNHEALTHY_TAINT = {"key": "amd.com/gpu-unhealthy", "value": "true", "effect": "NoSchedule"}


def condition_reason(state: str) -> str:
    """NodeCondition / Event reason of a verdict state (``MI355XHealthy``, ``MI355XUnhealthy``, ...)."""
    return _REASON[state]


def parse_k8s_time(ts: Optional[str]) -> Optional[float]:
    """RFC 3339 ``2025-10-10T00:00:00Z`` (what the apiserver emits) -> epoch seconds."""
    if not ts or not isinstance(ts, str):
        return None
    try:
        from datetime import datetime
        return datetime.fromisoformat(ts.replace("Z", "+00:00")).timestamp()
    except ValueError:
        return None


def format_k8s_time(epoch: float) -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(epoch))


#: The condition message starts with the GPU counts the verdict was taken on, so the checker can
#: cross-check them against the node's ``amd.com/gpu`` without the report annotation:
#: ``8/8 MI355X GPUs healthy``, ``8/8 MI355X GPUs ok; gpu3: HBM 96 C`` (degraded),
#: ``6/7 MI355X GPUs ok; 7 of 8 GPUs visible to amd-smi; gpu2: ...`` (unhealthy).
#: (parsed by hand, not with ``re``: the regex module is most of this module's import cost)
_COUNTS_TAIL = " MI355X GPUs "


def condition_message(verdict: Verdict) -> str:
    """``AMDGPUHealthy`` message of a verdict: GPU counts first (parseable), then the reasons."""
    if verdict.state == HEALTHY:
        return f"{verdict.gpus_ok}/{verdict.gpus_seen} MI355X GPUs healthy"
    detail = "; ".join(verdict.reasons or verdict.warnings)
    if verdict.state == UNKNOWN and not verdict.gpus_seen:
        return detail  # the probe itself failed: there are no counts to report
    return f"{verdict.gpus_ok}/{verdict.gpus_seen} MI355X GPUs ok" + (f"; {detail}" if detail else "")


def parse_condition_counts(message: Optional[str]) -> Optional[Tuple[int, int]]:
    """``(gpus_ok, gpus_seen)`` from an ``AMDGPUHealthy`` message, None when it carries none
    (an older agent, or a probe failure)."""
    msg = message or ""
    head, sep, rest = msg.partition(_COUNTS_TAIL)
    ok, slash, seen = head.partition("/")
    if not sep or not slash or not ok.isdecimal() or not seen.isdecimal():
        return None
    for word in ("healthy", "ok"):
        if rest.startswith(word):
            nxt = rest[len(word):len(word) + 1]
            if not nxt or not (nxt.isalnum() or nxt == "_"):  # the regex's \b
                return int(ok), int(seen)
    return None


def condition_for(verdict: Verdict, now: Optional[float] = None,
                  previous: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    """The ``AMDGPUHealthy`` NodeCondition the agent publishes for ``verdict``."""
    now = time.time() if now is None else now
    status = "True" if verdict.ok else ("Unknown" if verdict.state == UNKNOWN else "False")
    msg = condition_message(verdict)
    ts = format_k8s_time(now)
    transition = ts
    if previous and previous.get("status") == status and previous.get("lastTransitionTime"):
        transition = previous["lastTransitionTime"]
    return {"type": HEALTH_CONDITION, "status": status, "reason": _REASON[verdict.state], "message": msg[:1024],
            "lastHeartbeatTime": ts, "lastTransitionTime": transition}


_PARTS: Dict[Optional[str], Tuple[Optional[Tuple[int, int]], str]] = {}


def _message_parts(message: Optional[str]) -> Tuple[Optional[Tuple[int, int]], str]:
    """``(counts, detail)`` of a condition message, memoised: across a cluster the agents publish a
    handful of distinct messages ("8/8 MI355X GPUs healthy" on every healthy node)."""
    got = _PARTS.get(message)
    if got is None:
        counts = parse_condition_counts(message)
        detail = message or ""
        if counts:
            detail = detail.split("; ", 1)[1] if "; " in detail else ""
        if len(_PARTS) >= 4096:
            _PARTS.clear()
        got = _PARTS[message] = (counts, detail)
    return got


def verdict_from_condition(cond: Tuple[Optional[str], Optional[str], Optional[str], Optional[float]],
                           max_age_s: float, now: Optional[float] = None, expected_gpus: int = 0) -> Verdict:
    """``(status, reason, message, heartbeat_epoch)`` of an ``AMDGPUHealthy`` condition -> Verdict.

    The cheap path: no annotation JSON to parse, the apiserver already carries
    the agent's verdict in ``status.conditions`` (parsed by the NodeList scan).

    ``expected_gpus`` is the node's ``amd.com/gpu`` count from the same LIST (the reference's
    definition of a GPU node, ``check-gpu-node.py:181-201``).  The message's ``ok/seen`` counts are
    cross-checked against it: an agent that saw fewer GPUs than the device plugin registered --
    a GPU that fell off the bus after registration, or an agent started without the node's
    count -- makes the node unhealthy even when the agent itself said ``True``.
    """
    status, reason, message, hb = cond
    now = time.time() if now is None else now
    age = (now - hb) if hb is not None else None
    if age is None or age > max_age_s:
        return Verdict(UNKNOWN, ["stale AMDGPUHealthy condition" if age is not None
                                 else "AMDGPUHealthy condition has no heartbeat"], age_s=age)
    if age < -max_age_s:  # as for reports: a heartbeat from the future would count as fresh indefinitely
        return Verdict(UNKNOWN, [f"AMDGPUHealthy heartbeat is {-age:.0f} s in the future (clock skew?)"], age_s=age)
    # a fresh condition's verdict depends only on (status, reason, message, expected): across a fleet a handful of
    # distinct ones ("8/8 MI355X GPUs healthy" on every healthy node), so each is worked out once and copied (new
    # lists per node: callers add reasons and warnings to one node's verdict)
    key = (status, reason, message, expected_gpus)
    t = _FRESH.get(key)
    if t is None:
        v = _fresh_condition_verdict(status, reason, message, expected_gpus)
        if len(_FRESH) >= 4096:
            _FRESH.clear()
        t = _FRESH[key] = (v.state, tuple(v.reasons), tuple(v.warnings), v.gpus_ok, v.gpus_seen)
    return Verdict(t[0], list(t[1]), list(t[2]), t[3], t[4], age)


_FRESH: Dict[tuple, tuple] = {}


def _fresh_condition_verdict(status: Optional[str], reason: Optional[str], message: Optional[str],
                             expected_gpus: int) -> Verdict:
    """:func:`verdict_from_condition` of a condition whose heartbeat is fresh (its age filled in by the caller)."""
    age = None
    counts, detail = _message_parts(message)
    ok, seen = counts if counts else (0, 0)
    msg = [detail] if detail else []
    if status == "True":
        state = _STATE_OF_REASON.get(reason or "", HEALTHY)
        state = state if state in _OK_STATES else HEALTHY
        v = Verdict(state, warnings=msg if state == DEGRADED else [], gpus_ok=ok, gpus_seen=seen, age_s=age)
    elif status == "False":
        v = Verdict(UNHEALTHY, msg or ["AMDGPUHealthy=False"], gpus_ok=ok, gpus_seen=seen, age_s=age)
    else:
        return Verdict(UNKNOWN, msg or ["AMDGPUHealthy=Unknown"], gpus_ok=ok, gpus_seen=seen, age_s=age)
    if counts and expected_gpus and seen < expected_gpus:
        missing = f"{seen} of {expected_gpus} GPUs visible to amd-smi"
        if not any(missing in r for r in v.reasons):
            v.reasons.insert(0, missing)
        v.state = UNHEALTHY
    return v


#: prefix of a compressed report annotation: ``gz:`` + base64(gzip(JSON)) (agent ``--annotation-encoding
#: gzip``; an 8-GPU report with level-2 results shrinks 22 KB -> 1.8 KB in every node LIST and watch event)
GZIP_PREFIX = "gz:"


def encode_annotation(report: Dict[str, Any], encoding: str = "json") -> str:
    """The ``amd.com/mi355x-health`` value of a report: compact JSON, or ``gz:`` + base64 of it gzipped."""
    import json
    text = json.dumps(report, separators=(",", ":"))
    if encoding == "json":
        return text
    if encoding != "gzip":
        raise ValueError(f"unknown annotation encoding {encoding!r}")
    import base64
    import gzip
    # mtime=0: the same report always encodes to the same bytes (the agent compares before rewriting)
    return GZIP_PREFIX + base64.b64encode(gzip.compress(text.encode(), 9, mtime=0)).decode("ascii")


# a decompressed report annotation larger than this is refused (a 256 KiB gzip annotation can inflate ~1000x);
# a level-2 report of a 64-partition CPX node is under 256 KiB as JSON
MAX_REPORT_BYTES = 4 << 20


def parse_annotation(raw: Optional[str]) -> Optional[Dict[str, Any]]:
    """A report annotation in either encoding -> the report dict; an undecodable one becomes a probe
    error (verdict unknown), never an exception."""
    if not raw:
        return None
    if raw.startswith(GZIP_PREFIX):
        import base64
        import binascii
        import gzip
        import zlib
        try:
            data = base64.b64decode(raw[len(GZIP_PREFIX):], validate=True)
            try:  # one gzip member, as the agent writes it: zlib directly (GzipFile costs ~3x as much)
                d = zlib.decompressobj(16 + zlib.MAX_WBITS)
                body = d.decompress(data, MAX_REPORT_BYTES + 1)
                if len(body) > MAX_REPORT_BYTES:
                    return {"schema": SCHEMA, "ts": time.time(),
                            "error": f"annotation decompresses to more than {MAX_REPORT_BYTES} bytes"}
                if not d.eof or d.unused_data:
                    raise zlib.error("not a single complete member")
            except zlib.error:
                # several members / trailing data: the general reader decides, on a bounded output
                with gzip.GzipFile(fileobj=io.BytesIO(data)) as f:
                    body = f.read(MAX_REPORT_BYTES + 1)
                if len(body) > MAX_REPORT_BYTES:
                    return {"schema": SCHEMA, "ts": time.time(),
                            "error": f"annotation decompresses to more than {MAX_REPORT_BYTES} bytes"}
            raw = body.decode("utf-8")
        except (binascii.Error, OSError, EOFError, zlib.error, UnicodeDecodeError, ValueError):
            return {"schema": SCHEMA, "error": "annotation is not gzip+base64 JSON", "ts": time.time()}
    from ..ops.fastpath import loads  # native json.loads (falls back to the json package itself)
    try:
        doc = loads(raw)
    except (ValueError, RecursionError):  # RecursionError: nesting deeper than the parser's stack
        return {"schema": SCHEMA, "error": "annotation is not JSON", "ts": time.time()}
    return doc if isinstance(doc, dict) else None


def gate_ready(ready_condition: bool, verdict: Optional[Verdict], policy: str, is_amd: bool,
               unknown_ok: bool = True) -> bool:
    """Combine NodeCondition Ready with the MI355X verdict.

    ``off``     -> Ready condition only (the reference).
    ``auto``    -> nodes that carry a probe report must also be healthy;
                   nodes without one keep the reference semantics.
    ``require`` -> every ``amd.com/gpu`` node needs a healthy, fresh report.
    """
    if not ready_condition or policy == "off" or not is_amd:
        return ready_condition
    if verdict is None:
        return policy != "require"
    if verdict.state == UNKNOWN:
        return unknown_ok and policy != "require"
    return verdict.ok


def summarize(verdicts: Sequence[Optional[Verdict]]) -> Dict[str, int]:
    out = {HEALTHY: 0, DEGRADED: 0, UNHEALTHY: 0, UNKNOWN: 0}
    for v in verdicts:
        out[v.state if v else UNKNOWN] += 1
    return out
