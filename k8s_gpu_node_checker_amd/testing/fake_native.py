"""CPU stand-ins for the C ABIs of ``libmi355x_diag.so`` and ``libmi355x_fabric.so``.

They implement the same calls with the same out-parameter protocol (values written through ctypes
pointers), so ``ops/diag.py`` and ``ops/fabric.py`` run unchanged on CPU with scripted results: a node of
N healthy MI355X by default, with per-GPU rate factors, wrong-result counts, slow or peer-less GPU pairs
and RCCL failures injectable.  Used by the CPU tests of the verdict logic and of whole 8-GPU agent
cycles; the real libraries run under ``tests/test_gpu.py`` on an MI355X.
"""

from __future__ import annotations

import ctypes
import threading
import time
from typing import Dict, List, Optional, Tuple


def _put(ptr, ctype, value) -> None:
    ctypes.cast(ptr, ctypes.POINTER(ctype))[0] = value


class FakeDiagLib:
    """``libmi355x_diag.so`` for a node of ``n`` GPUs.

    rate:        every GEMM / HBM / MFMA / host-link rate = rate x the full-GPU reference (per GPU:
                 ``gpu_rate[d]``; a list ``rates`` overrides it call by call)
    cus/mem_gib: what HIP reports per device (a CPX partition: 32 CUs)
    mfma_errors: ``{(device, kind index): wrong results}``
    p2p_gbps:    rate of every GPU pair; ``slow_pairs[(src, dst)]`` / ``nopeer`` override pairs; a pair in
                 ``hung_pairs`` never completes (with a deadline: returns -4 at it; without: blocks until
                 ``release`` is set); ``p2p_wall_s`` = wall time of each completed pair
    delay_s:     wall time of each GEMM call (the agent's per-GPU threads overlap them)
    gemm_bad_tiles: ``{(device, "gemm" | "gemm_fp8"): {xcd: tiles}}`` failing the GEMM's output checksums
    slow_xcd:    ``{xcd: factor}`` on the burn-in's per-XCD wave time; ``bad_cu[(device, kind)]`` = the CU
                 slot its ``mfma_errors`` come from
    """

    def __init__(self, n: int = 1, rate: float = 1.0, gpu_rate: Optional[Dict[int, float]] = None,
                 rates: Optional[List[float]] = None, cus: int = 256, mem_gib: int = 288, gemm_err: float = 2e-5,
                 mfma: Optional[Dict[int, Tuple[float, int]]] = None,
                 mfma_errors: Optional[Dict[Tuple[int, int], int]] = None, link: Optional[Tuple[float, float]] = None,
                 p2p_gbps: float = 48.0, slow_pairs: Optional[Dict[Tuple[int, int], float]] = None,
                 nopeer: Tuple[Tuple[int, int], ...] = (), rc: int = 0, err: bytes = b"boom", delay_s: float = 0.0,
                 slow_xcd: Optional[Dict[int, float]] = None, bad_cu: Optional[Dict[Tuple[int, int], int]] = None,
                 lds_bad: Optional[Dict[Tuple[int, int], int]] = None,
                 l2_bad: Optional[Dict[Tuple[int, int], int]] = None, slow_cu: Optional[Dict[int, float]] = None,
                 hbm_xcd_slow: Optional[Dict[int, float]] = None, hbm_bad: Optional[Dict[Tuple[int, int], int]] = None,
                 compute_rate: Optional[Dict[int, float]] = None,
                 hung_pairs: Tuple[Tuple[int, int], ...] = (), p2p_wall_s: float = 0.0,
                 gemm_bad_tiles: Optional[Dict[Tuple[int, str], Dict[int, int]]] = None,
                 hang_devices: Tuple[int, ...] = (), abort_devices: Tuple[int, ...] = (),
                 fan_slow: Optional[Dict[Tuple[int, int], float]] = None,
                 fan_errors: Optional[Dict[Tuple[int, int], int]] = None):
        from ..ops import diag
        # the fan pass (diag_p2p_fan_t): fan_slow[(src, dst)] = that pair's rate while every link of src is busy,
        # fan_errors[(src, dst)] = bad words it delivers then
        self.fan_slow = dict(fan_slow or {})
        self.fan_errors = dict(fan_errors or {})
        # hang_devices: a GEMM call on that device never returns (a hung queue: no deadline ends it);
        # abort_devices: it ends the process with SIGABRT, as the HIP runtime does on a GPU memory fault
        self.hang_devices = set(hang_devices)
        self.abort_devices = set(abort_devices)
        self.ref = diag.REFERENCE_RATES
        self.kinds = diag.MFMA_KINDS
        self.n = n
        self.rate = rate
        self.gpu_rate = dict(gpu_rate or {})
        # compute_rate[d]: an extra factor on device d's matrix-core tests only (GEMM, burn-in) -- a lowered
        # power cap slows the core clock, not HBM or the host link
        self.compute_rate = dict(compute_rate or {})
        self.rates = list(rates or [])
        self.cus = cus
        self.mem_gib = mem_gib
        self.gemm_err = gemm_err
        self.gemm_bad_tiles = dict(gemm_bad_tiles or {})
        self.mfma = mfma
        self.mfma_errors = dict(mfma_errors or {})
        self.link = link
        self.p2p_gbps = p2p_gbps
        self.slow_pairs = dict(slow_pairs or {})
        self.nopeer = set(nopeer)
        self.hung_pairs = set(hung_pairs)
        self.p2p_wall_s = p2p_wall_s
        self.p2p_timeouts_ms: List[float] = []
        self.release = threading.Event()
        self.rc = rc
        self.err = err
        self.delay_s = delay_s
        self.slow_xcd = dict(slow_xcd or {})
        self.bad_cu = dict(bad_cu or {})
        self.lds_bad = dict(lds_bad or {})
        # per-XCD HBM: hbm_xcd_slow[xcd] = that XCD's alone rate as a share of the reference; hbm_bad[(device,
        # slot)] = wrong words read there
        self.hbm_xcd_slow = dict(hbm_xcd_slow or {})
        self.hbm_bad = dict(hbm_bad or {})
        self.l2_bad = dict(l2_bad or {})
        self.slow_cu = dict(slow_cu or {})
        self.calls: List[str] = []
        self.threads: Dict[int, set] = {}
        self.lock = threading.Lock()
        # shared host link: with link_shared, concurrent host_link calls split the host's bandwidth (each gets
        # 1/k of it while k run at once, for link_delay_s); in_flight / peak_* record the overlap
        self.link_shared = False
        self.link_delay_s = 0.0
        self.in_flight: Dict[str, int] = {}
        self.peak: Dict[str, int] = {}

    def _enter(self, what: str) -> int:
        with self.lock:
            k = self.in_flight.get(what, 0) + 1
            self.in_flight[what] = k
            self.peak[what] = max(self.peak.get(what, 0), k)
            return k

    def _leave(self, what: str) -> None:
        with self.lock:
            self.in_flight[what] -= 1

    def _rate(self, device: int) -> float:
        with self.lock:
            if self.rates:
                return self.rates.pop(0)
        return self.gpu_rate.get(device, self.rate)

    def _log(self, device: int, what: str) -> None:
        with self.lock:
            self.calls.append(what)
            self.threads.setdefault(device, set()).add(threading.current_thread().name)

    # --- C ABI ------------------------------------------------------------------------------------------
    def diag_last_error(self) -> bytes:
        return self.err

    def diag_device_count(self) -> int:
        return self.n

    def diag_device_arch(self, device, buf, size):
        if not 0 <= device < self.n:
            self.err = b"hipSetDevice: invalid device ordinal"
            return -1
        v = f"gfx950:sramecc+:xnack-|AMD Instinct MI355X|{self.cus}|{self.mem_gib << 30}|0000:{0x05 + 0x10 * device:02x}:00.0"
        ctypes.memmove(buf, v.encode() + b"\0", min(size, len(v) + 1))
        return 0

    def _gemm(self, test, device, size, tflops, err, ms):
        self._log(device, test)
        if device in self.abort_devices:
            import os
            import resource
            resource.setrlimit(resource.RLIMIT_CORE, (0, 0))  # no core file from a scripted abort
            os.abort()
        if device in self.hang_devices:
            while True:
                time.sleep(3600)
        self._enter("gemm")
        if self.delay_s:
            time.sleep(self.delay_s)
        self._leave("gemm")
        table = self.ref[test]
        key = size if size in table else min(table, key=lambda k: abs(k - size))
        _put(tflops, ctypes.c_double, self._rate(device) * self.compute_rate.get(device, 1.0) * table[key])
        _put(err, ctypes.c_double, self.gemm_err)
        _put(ms, ctypes.c_double, 0.1)
        return self.rc

    def diag_gemm_bf16(self, device, m, n, k, warmup, iters, samples, tflops, err, ms):
        return self._gemm("gemm", device, m, tflops, err, ms)

    def _checksums(self, test, device, inject, ck_err, out):
        """Tile checksums: ``gemm_bad_tiles[(device, test)] = {xcd: tiles}``; an injected element = one bad
        tile on XCD 0, as on the GPU (workgroup 0 computes tile (0, 0) on XCD 0)."""
        bad = dict(self.gemm_bad_tiles.get((device, test), {}))
        if inject >= 0:
            bad[0] = bad.get(0, 0) + 1
        vals = [0] * 12
        vals[0] = sum(bad.values())
        vals[1] = 256 * vals[0]
        for x, t in bad.items():
            vals[2 + x] = t
        vals[10], vals[11] = (0, 0) if vals[0] else (-1, -1)
        for i, v in enumerate(vals):
            out[i] = v
        _put(ck_err, ctypes.c_double, 0.4 if vals[0] else 3e-8)

    def diag_gemm_bf16_x(self, device, m, n, k, warmup, iters, samples, inject, tol, tflops, err, ms, ck_err, out):
        rc = self._gemm("gemm", device, m, tflops, err, ms)
        if rc == 0 and tol >= 0:
            self._checksums("gemm", device, inject, ck_err, out)
        return rc

    def diag_gemm_fp8_x(self, device, m, n, k, warmup, iters, samples, inject, tol, tflops, err, ms, ck_err, out):
        rc = self._gemm("gemm_fp8", device, m, tflops, err, ms)
        if rc == 0 and tol >= 0:
            self._checksums("gemm_fp8", device, inject, ck_err, out)
        return rc

    def diag_gemm_fp8(self, device, m, n, k, warmup, iters, samples, tflops, err, ms):
        return self._gemm("gemm_fp8", device, m, tflops, err, ms)

    def diag_hbm_bandwidth(self, device, nbytes, iters, c, r, w):
        self._log(device, "hbm")
        f = self._rate(device)
        _put(c, ctypes.c_double, f * self.ref["hbm"]["copy_tbs"])
        _put(r, ctypes.c_double, f * self.ref["hbm"]["read_tbs"])
        _put(w, ctypes.c_double, f * 6.9)
        return self.rc

    def diag_memtest(self, device, nbytes, seed, passes, errs, first, gbps):
        self._log(device, "memtest")
        _put(errs, ctypes.c_ulonglong, 0)
        _put(gbps, ctypes.c_double, 5400.0)
        return self.rc

    def diag_mfma_burn(self, device, kind, iters, reps, tflops, errors):
        self._log(device, "mfma")
        if self.rc:
            return self.rc
        if self.mfma is not None:
            tf, e = self.mfma[kind]
        else:
            tf, e = (self.gpu_rate.get(device, self.rate) * self.compute_rate.get(device, 1.0)
                     * self.ref["mfma"][self.kinds[kind]], 0)
        _put(tflops, ctypes.c_double, tf)
        _put(errors, ctypes.c_ulonglong, self.mfma_errors.get((device, kind), e))
        return 0

    def diag_mfma_burn_slots(self):
        return 1024

    def diag_mfma_burn_map(self, device, kind, iters, reps, tflops, errors, cu_map):
        """diag_mfma_burn plus the per-CU table: 8 XCDs x 32 CUs (4 SEs x 8), 8 waves per CU and
        launch; ``slow_xcd`` {xcd: time factor} and ``bad_cu`` {(device, kind): slot} shape it."""
        rc = self.diag_mfma_burn(device, kind, iters, reps, tflops, errors)
        if rc or not cu_map:
            return rc
        nerr = self.mfma_errors.get((device, kind), 0)
        bad_slot = self.bad_cu.get((device, kind))
        for xcd in range(8 if self.cus >= 256 else max(1, self.cus // 32)):
            for se in range(4):
                for cu in range(8):
                    slot = (xcd << 7) | (se << 5) | cu
                    waves = 8 * (reps + 1)
                    cu_map[3 * slot] = waves
                    cu_map[3 * slot + 2] = int(waves * 40000 * self.slow_xcd.get(xcd, 1.0) * self.slow_cu.get(slot, 1.0))
        if bad_slot is not None and nerr:
            cu_map[3 * bad_slot + 1] = nerr
        return 0

    def diag_l2_bandwidth(self, device, slice_bytes, passes, blocks_per_cu, seed, tbs, errors, cu_map):
        """Aggregate rate = rate x reference; per-CU table shaped like the burn-in's (``slow_xcd`` applies,
        ``l2_bad[(device, slot)]`` = wrong words read there)."""
        self._log(device, "l2")
        if self.rc:
            return self.rc
        _put(tbs, ctypes.c_double, self._rate(device) * self.ref["l2"]["read_tbs"])
        total = 0
        for xcd in range(8 if self.cus >= 256 else max(1, self.cus // 32)):
            for se in range(4):
                for cu in range(8):
                    slot = (xcd << 7) | (se << 5) | cu
                    waves = 4 * blocks_per_cu
                    cu_map[3 * slot] = waves
                    cu_map[3 * slot + 2] = int(waves * 90000 * self.slow_xcd.get(xcd, 1.0))
                    bad = self.l2_bad.get((device, slot), 0)
                    cu_map[3 * slot + 1] = bad
                    total += bad
        _put(errors, ctypes.c_ulonglong, total)
        return 0

    def diag_hbm_xcd(self, device, slice_bytes, passes, blocks_per_cu, seed, tbs, errors, cu_map, xcd_tbs):
        """All XCDs together at rate x reference; each XCD alone at rate x reference x ``hbm_xcd_slow``."""
        self._log(device, "hbm_xcd")
        if self.rc:
            return self.rc
        r = self._rate(device)
        _put(tbs, ctypes.c_double, r * self.ref["hbm_xcd"]["read_tbs"])
        total = 0
        nx = 8 if self.cus >= 256 else max(1, self.cus // 32)
        for xcd in range(8):
            # an XCD alone reads at its own path's rate whatever the partition: the device's rate share
            # (rate) is normalised by its CU share
            share = min(1.0, self.cus / 256)
            xcd_tbs[xcd] = r / share * 1.31 * self.hbm_xcd_slow.get(xcd, 1.0) if xcd < nx else 0.0
        for xcd in range(nx):
            for se in range(4):
                for cu in range(8):
                    slot = (xcd << 7) | (se << 5) | cu
                    waves = 4 * blocks_per_cu
                    cu_map[3 * slot] = waves
                    cu_map[3 * slot + 2] = waves * 50000
                    bad = self.hbm_bad.get((device, slot), 0)
                    cu_map[3 * slot + 1] = bad
                    total += bad
        _put(errors, ctypes.c_ulonglong, total)
        return 0

    def diag_lds_test(self, device, rounds, seed, inject_block, errors, cu_map, lds_bytes, ms):
        """Every CU of the device runs `rounds` workgroups; ``lds_bad[(device, slot)]`` = bad words there."""
        self._log(device, "lds")
        if self.rc:
            return self.rc
        total = 0
        for xcd in range(8 if self.cus >= 256 else max(1, self.cus // 32)):
            for se in range(4):
                for cu in range(8):
                    slot = (xcd << 7) | (se << 5) | cu
                    cu_map[2 * slot] = rounds
                    bad = self.lds_bad.get((device, slot), 0) + (1 if inject_block >= 0 and slot == 0 else 0)
                    cu_map[2 * slot + 1] = bad
                    total += bad
        _put(errors, ctypes.c_ulonglong, total)
        _put(lds_bytes, ctypes.c_int, 163840 - 16)
        _put(ms, ctypes.c_double, 0.2)
        return 0

    def diag_host_link(self, device, nbytes, iters, h2d, d2h):
        self._log(device, "host_link")
        f = self.gpu_rate.get(device, self.rate)
        k = self._enter("host_link")
        if self.link_delay_s:
            time.sleep(self.link_delay_s)
        k = max(k, self.in_flight.get("host_link", 1))
        self._leave("host_link")
        if self.link_shared:
            f /= k
        h, d = self.link or (f * self.ref["host_link"]["h2d_gbps"], f * self.ref["host_link"]["d2h_gbps"])
        _put(h2d, ctypes.c_double, h)
        _put(d2h, ctypes.c_double, d)
        return self.rc

    def diag_p2p_copy(self, src, dst, nbytes, iters, gbps, errors, peer):
        return self.diag_p2p_copy_t(src, dst, nbytes, iters, 0.0, gbps, errors, peer)

    def diag_p2p_copy_t(self, src, dst, nbytes, iters, timeout_ms, gbps, errors, peer):
        with self.lock:  # node-level: runs on the agent's main thread, after the per-GPU threads
            self.calls.append(f"p2p{src}->{dst}")
            self.p2p_timeouts_ms.append(float(timeout_ms))
        if not (0 <= src < self.n and 0 <= dst < self.n) or src == dst:
            self.err = b"p2p: invalid device pair"
            return -1
        if (src, dst) in self.hung_pairs:
            if timeout_ms > 0 and not self.release.wait(timeout_ms / 1000.0):
                self.err = b"p2p %d->%d: copies did not complete within %d ms (xGMI link or engine hung)" % (
                    src, dst, int(timeout_ms))
                return -4
            self.release.wait()
        elif self.p2p_wall_s:
            time.sleep(self.p2p_wall_s)
        _put(gbps, ctypes.c_double, self.slow_pairs.get((src, dst), self.p2p_gbps))
        _put(errors, ctypes.c_ulonglong, 0)
        _put(peer, ctypes.c_int, 0 if (src, dst) in self.nopeer else 1)
        return 0

    def diag_p2p_fan_t(self, src, dsts, ndst, nbytes, iters, timeout_ms, gbps, errors, peer, total):
        """Every peer of ``src`` at once: a pair's rate is ``fan_slow[(src, dst)]`` when given (a link that holds up
        alone but not under load), else its pair rate (``slow_pairs`` / ``p2p_gbps``)."""
        with self.lock:
            self.calls.append(f"fan{src}")
            self.p2p_timeouts_ms.append(float(timeout_ms))
        peers = [dsts[i] for i in range(ndst)]
        if not 0 <= src < self.n or not peers or any(not 0 <= d < self.n or d == src for d in peers):
            self.err = b"p2p fan: every peer must be a device other than the source"
            return -2
        for d in peers:
            if (src, d) in self.hung_pairs and timeout_ms > 0 and not self.release.wait(timeout_ms / 1000.0):
                self.err = b"p2p fan %d->%d: copies did not complete within %d ms (xGMI link or engine hung)" % (
                    src, d, int(timeout_ms))
                return -4
        for i, d in enumerate(peers):
            gbps[i] = self.fan_slow.get((src, d), self.slow_pairs.get((src, d), self.p2p_gbps))
            errors[i] = self.fan_errors.get((src, d), 0)
            peer[i] = 0 if (src, d) in self.nopeer else 1
        _put(total, ctypes.c_double, float(sum(gbps[i] for i in range(ndst))))
        return 0


class FakeFabricLib:
    """``libmi355x_fabric.so`` (in-process RCCL communicator over the node's GPUs)."""

    def __init__(self, busbw: float = 320.0, errors: int = 0, fail_open: bool = False, version: int = 22707,
                 hang_op: Optional[int] = None, async_error_op: Optional[int] = None, ignore_deadline: bool = False):
        self.busbw, self.errors, self.fail_open, self.version = busbw, errors, fail_open, version
        # ignore_deadline: the hang_op collective never returns, deadline or not (a wait stuck in the driver)
        self.ignore_deadline = ignore_deadline
        # hang_op: that collective never completes -- the call waits out its deadline (or forever without
        # one, until `release` is set) and then "aborts" the communicators like fabric.hip's abort_all
        self.hang_op = hang_op
        # async_error_op: a communicator reports an async error during that collective (a link dropping
        # traffic): fabric.hip's wait_comms / sync_all abort every communicator and return ABORTED
        self.async_error_op = async_error_op
        self.release = threading.Event()
        self.opened: List[List[int]] = []
        self.timeouts_ms: List[float] = []
        self.aborts = 0
        self.closed = 0
        self.err = b"ncclCommInitAll: unhandled system error"

    def fabric_open(self, arr, n, timeout_ms=0.0):
        if self.fail_open:
            return None
        self.opened.append([arr[i] for i in range(n)])
        return 1

    def fabric_run(self, ctx, op, nbytes, iters, warmup, out, timeout_ms=0.0):
        self.timeouts_ms.append(timeout_ms)
        if op == self.hang_op:
            self.release.wait(timeout_ms / 1e3 if timeout_ms > 0 and not self.ignore_deadline else None)
            if not self.release.is_set():
                self.aborts += 1  # ncclCommAbort on every communicator
                self.err = (f"timed collectives: not complete within {timeout_ms:.0f} ms: communicators aborted "
                            "(ncclCommAbort)").encode()
                return -4
        if op == self.async_error_op:
            self.aborts += 1
            self.err = b"collective wait: remote process exited or there was a network error (communicators aborted)"
            return -4
        out[0], out[1], out[2], out[3] = 1.0, self.busbw * 0.57, self.busbw, float(self.errors if op == 3 else 0)
        return 0

    def fabric_aborted(self, ctx):
        return 1 if self.aborts else 0

    def fabric_close(self, ctx):
        self.closed += 1

    def fabric_last_error(self):
        return self.err

    def fabric_rccl_version(self):
        return self.version


class NarrowedDiagLib:
    """A :class:`FakeDiagLib` as a process sees it with ``HIP_VISIBLE_DEVICES=k``: one device, ordinal 0 = GPU k
    (what a per-device diagnostic child of the agent sees, agent/isolation.narrow_to)."""

    _PER_DEVICE = frozenset(("diag_device_arch", "diag_gemm_bf16", "diag_gemm_bf16_x", "diag_gemm_fp8_x",
                             "diag_gemm_fp8", "diag_hbm_bandwidth", "diag_memtest", "diag_memtest_x", "diag_mfma_burn",
                             "diag_mfma_burn_map", "diag_l2_bandwidth", "diag_hbm_xcd", "diag_lds_test",
                             "diag_host_link", "diag_poll_selftest"))

    def __init__(self, lib: FakeDiagLib, physical: int):
        self.lib, self.physical = lib, physical

    def diag_device_count(self) -> int:
        return 1

    def __getattr__(self, name: str):
        fn = getattr(self.lib, name)
        if name not in self._PER_DEVICE:
            return fn

        def on_physical(device, *a):
            if device != 0:
                self.lib.err = b"hipSetDevice: invalid device ordinal"
                return -1
            return fn(self.physical, *a)
        return on_physical


def install(n: int = 1, fabric: Optional[Dict] = None, **diag_kw) -> None:
    """Make this process's ``ops.diag`` and ``ops.fabric`` use the fakes: ``FakeDiagLib(n, **diag_kw)`` and
    ``FakeFabricLib(**fabric)``.  The node agent's diagnostic children run it first when the agent is given
    ``diag_setup=("k8s_gpu_node_checker_amd.testing.fake_native", "install", {...})`` (agent/isolation.py), so the
    child code path runs unchanged on CPU with scripted GPUs; a child narrowed to one GPU (``HIP_VISIBLE_DEVICES``)
    sees only that one, as under HIP."""
    import os
    from ..ops import diag
    from ..ops import fabric as fabric_mod
    lib: object = FakeDiagLib(n=n, **diag_kw)
    vis = os.environ.get("HIP_VISIBLE_DEVICES", "").strip()
    if vis.isdigit() and int(vis) < n:
        lib = NarrowedDiagLib(lib, int(vis))  # type: ignore[arg-type]
    diag.lib = lambda: lib
    fabric_mod._lib = FakeFabricLib(**(fabric or {}))
