"""Disposable diagnostic processes: the resident node agent never initialises HIP.

The reference computes its verdict fresh on every run and keeps nothing between runs
(``/root/reference/check-gpu-node.py:252-293``).  The agent's active diagnostics follow the same model: each
cycle's HIP work runs in short-lived child processes, so

* the agent process itself stays at the size of Python + the amd-smi probe between cycles (no HIP runtime, no
  comgr code-object cache, no kernel-argument pools resident for the hours between two diagnostic runs);
* a diagnostic that outlives ``--diag-timeout`` is ended with SIGKILL and its GPU is reported failed -- the agent
  keeps probing and publishing, and nothing hung stays behind in the agent (no ``/healthz`` restart);
* a GPU fault that aborts the HIP runtime (``hipErrorIllegalAddress`` ends the process) costs one child, reported
  as that GPU's failed ``run``, not the agent;
* a driver reload between cycles is picked up by the next child's fresh HIP runtime.

The children come from a ``multiprocessing`` **forkserver** that :class:`Workers` starts when the agent is
constructed -- before any amd-smi or HIP call -- so every child is forked from a clean interpreter that never
touched the GPU (forking a process that has initialised HIP is undefined; exec'ing from one is refused on the
GPU boxes).  Each child is one of

* :func:`enumerate_main` -- HIP's device count and each ordinal's PCI address (how amd-smi's GPUs map onto HIP
  ordinals);
* :func:`device_main` -- one HIP device's suite (``ops/diag.run``); the suites of one cycle take turns at the
  shared host link through a ``multiprocessing`` lock (``ops/diag.use_host_lock``);
* :func:`fabric_main` -- the node-level xGMI pair matrix and RCCL collectives over every device.

Every child sends one message, ``(result, meta)`` with ``meta`` = its pid, peak RSS and wall time, over a pipe and
exits.  The ``thread`` mode runs the same jobs on threads of the agent process (library use, the benchmark process,
tests that script ``ops.diag`` in-process); there a job that hangs cannot be ended.
"""

from __future__ import annotations

import importlib
import multiprocessing
import os
import resource
import signal
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

ISOLATION = ("process", "thread")
# how long a SIGKILLed child may take to be reaped before it counts as stuck (uninterruptible in the driver)
KILL_GRACE_S = 5.0
# modules the forkserver imports once, so each child starts without re-importing them (pure Python: loading the
# diagnostics library and initialising HIP happen in the child)
PRELOAD = ("k8s_gpu_node_checker_amd.agent.isolation", "k8s_gpu_node_checker_amd.ops.diag",
           "k8s_gpu_node_checker_amd.ops.fabric")

Setup = Optional[Tuple[str, str, Dict[str, Any]]]


def _setup(setup: Setup) -> None:
    """Run ``module.function(**kwargs)`` in the child before its job (tests install the fake C ABIs here)."""
    if setup:
        mod, fn, kw = setup
        getattr(importlib.import_module(mod), fn)(**kw)


def _meta(t0: float) -> Dict[str, Any]:
    # ru_maxrss is in KiB on Linux: the child's own peak, HIP runtime and code objects included
    return {"pid": os.getpid(), "peak_rss_mib": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024, 1),
            "wall_s": round(time.monotonic() - t0, 3)}


def _reply(conn: Any, res: Any, t0: float) -> None:
    try:
        conn.send((res, _meta(t0)))
    finally:
        conn.close()


def _quiet_signals() -> None:
    # the agent's SIGTERM handler finishes its cycle; a child has nothing to finish and ends with the default action
    signal.signal(signal.SIGTERM, signal.SIG_DFL)
    signal.signal(signal.SIGINT, signal.SIG_IGN)


def enumerate_main(conn: Any, setup: Setup = None) -> None:
    """Child: ``{"count": n, "bdf": {ordinal: pci}}`` of the HIP runtime this process sees, or ``{"error": ...}``."""
    t0 = time.monotonic()
    _quiet_signals()
    _setup(setup)
    from ..ops import diag
    try:
        n = diag.device_count()
        bdf: Dict[int, str] = {}
        for d in range(n):
            try:
                bdf[d] = str(diag.device_info(d).get("bdf") or "")
            except Exception:
                bdf[d] = ""
        res: Dict[str, Any] = {"count": n, "bdf": bdf}
    except Exception as e:
        res = {"error": f"{type(e).__name__}: {e}"[:200]}
    _reply(conn, res, t0)


def narrow_to(device: int, environ: Optional[Dict[str, str]] = None) -> Optional[str]:
    """Make HIP ordinal ``device`` of this process's environment the only device a HIP runtime started afterwards
    sees (its ordinal 0): ``HIP_VISIBLE_DEVICES`` set to the entry ``device`` selects -- of an existing
    ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` list when one narrows this process already, else ``device``
    itself.  Returns the selector, or None when the list has no such entry (nothing changed)."""
    env = os.environ if environ is None else environ
    sel = str(device)
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        cur = env.get(var)
        if cur is not None and cur.strip():
            items = [x.strip() for x in cur.split(",") if x.strip()]
            if not 0 <= device < len(items):
                return None
            sel = items[device]
            break
    env["HIP_VISIBLE_DEVICES"] = sel
    env.pop("CUDA_VISIBLE_DEVICES", None)
    return sel


def device_main(conn: Any, setup: Setup, level: int, device: int, kw: Dict[str, Any],
                host_lock: Any = None, host_cell: Any = None) -> None:
    """Child: ``ops/diag.run(level, device, **kw)`` with this child's HIP runtime narrowed to that one GPU
    (:func:`narrow_to`: the process is then what was measured on a one-GPU box, whatever the node's GPU count, and
    touches no other GPU); a run that raises is a failed ``run`` test.  The meta says which PCI address it ran on."""
    t0 = time.monotonic()
    _quiet_signals()
    ordinal = device if narrow_to(device) is None else 0
    from ..ops.diag import uses_dma
    if not uses_dma(level):
        # a suite that times no DMA-engine copy keeps the runtime off the SDMA engines: ~180 MiB less host memory
        # (ops/diag.DMA_TESTS); set before this process starts its HIP runtime
        os.environ.setdefault("HSA_ENABLE_SDMA", "0")
    _setup(setup)
    from ..ops import diag
    if host_lock is not None:
        diag.use_host_lock(host_lock, host_cell, label=device)
    bdf = ""
    try:
        bdf = str(diag.device_info(ordinal).get("bdf") or "")
        res = diag.run(level, ordinal, **kw)
    except Exception as e:  # a broken library or device: a failed test, not a lost report
        res = {"run": {"pass": False, "detail": f"{type(e).__name__}: {e}"[:200]}}
    try:
        conn.send((res, dict(_meta(t0), bdf=bdf)))
    finally:
        conn.close()


def fabric_main(conn: Any, setup: Setup, suite: Callable[..., Dict[str, Any]], devices: List[int],
                timeout_s: Optional[float]) -> None:
    """Child: the node-level suite ``suite(devices, timeout_s)`` over every device."""
    t0 = time.monotonic()
    _quiet_signals()
    _setup(setup)
    _reply(conn, suite(devices, timeout_s), t0)


def describe_exit(code: Optional[int]) -> str:
    """A child's exit status in words (``-9`` is SIGKILL, ``-6`` an abort: HIP ends the process on a GPU fault)."""
    if code is None:
        return "no exit status"
    if code < 0:
        try:
            return f"signal {signal.Signals(-code).name}"
        except ValueError:
            return f"signal {-code}"
    return f"exit code {code}"


class Job:
    """One diagnostic run -- a device's suite, the fabric suite or the enumeration -- on a child process or a thread.

    ``box["res"]`` holds the result once it is in (``died`` supplies one for a child that ended without sending),
    ``box["meta"]`` the child's pid / peak RSS / wall time, ``box["external_kill"]`` the reason when a SIGKILL the
    agent did not send ended the child; ``done`` (shared by a cycle's jobs) is set when it ends.
    """

    def __init__(self, proc: Any = None, thread: Optional[threading.Thread] = None,
                 reader: Optional[threading.Thread] = None, box: Optional[Dict[str, Any]] = None):
        self.proc, self.thread, self.reader = proc, thread, reader
        self.box: Dict[str, Any] = box if box is not None else {}
        self.killed = False

    @property
    def pid(self) -> Optional[int]:
        return self.proc.pid if self.proc is not None else None

    def is_alive(self) -> bool:
        if self.proc is not None:
            return self.proc.is_alive() or bool(self.reader and self.reader.is_alive())
        return bool(self.thread and self.thread.is_alive())

    def kill(self, grace_s: float = KILL_GRACE_S) -> bool:
        """SIGKILL the child and reap it; True when it is gone.  A thread cannot be ended: False."""
        if self.proc is None:
            return not self.is_alive()
        self.killed = True
        try:
            self.proc.kill()
        except (OSError, ValueError):
            pass
        self.proc.join(grace_s)
        if self.reader is not None:
            self.reader.join(grace_s)
        return not self.is_alive()


class Workers:
    """Starts diagnostic jobs: children of a forkserver (``process``) or threads of this process (``thread``).

    ``setup`` -- ``(module, function, kwargs)`` run in each child first (tests: ``testing/fake_native.install``).
    """

    def __init__(self, mode: str = "process", setup: Setup = None, method: str = "forkserver"):
        if mode not in ISOLATION:
            raise ValueError(f"isolation must be one of {ISOLATION}")
        self.mode, self.setup = mode, setup
        self.ctx: Any = None
        self.started: List[Dict[str, Any]] = []  # (pid, what) of every child, for the soak tool and the tests
        if mode == "process":
            self.ctx = multiprocessing.get_context(method)
            if method == "forkserver":
                self.ctx.set_forkserver_preload(list(PRELOAD))
                from multiprocessing import forkserver
                forkserver.ensure_running()  # now: before this process loads amd-smi or HIP

    @property
    def isolated(self) -> bool:
        return self.mode == "process"

    def host_lock(self) -> Tuple[Any, Any]:
        """A fresh (lock, holder cell) for one cycle's device children: a child killed while holding it takes only
        that cycle's lock with it."""
        if not self.isolated:
            return None, None
        return self.ctx.Lock(), self.ctx.Array("d", [-1.0, 0.0], lock=False)

    def _spawn(self, what: str, target: Callable[..., None], args: Sequence[Any], done: threading.Event,
               died: Callable[[str], Any]) -> Job:
        box: Dict[str, Any] = {}
        parent, child = self.ctx.Pipe(duplex=False)
        proc = self.ctx.Process(target=target, args=(child, *args), name=f"mi355x-{what}", daemon=True)
        try:
            proc.start()
        except Exception as e:  # the forkserver is gone, no memory for a child, ...: that job failed, not the agent
            parent.close()
            child.close()
            box["res"] = died(f"could not start the diagnostic process: {type(e).__name__}: {e}")
            done.set()
            return Job(box=box)
        child.close()  # the child's end lives in the child only: its exit closes the pipe (EOF)
        self.started.append({"pid": proc.pid, "what": what})
        holder: List[Job] = []

        def read() -> None:
            try:
                box["res"], box["meta"] = parent.recv()
            except (EOFError, OSError):
                pass
            finally:
                parent.close()
                proc.join()
                if "res" not in box:
                    why = f"diagnostic process {proc.pid} ended before reporting ({describe_exit(proc.exitcode)})"
                    if proc.exitcode == -signal.SIGKILL and not (holder and holder[0].killed):
                        # not the agent's watchdog: the kernel's OOM killer at the pod's memory limit, or an operator
                        # -- not the GPU's finding (box["external_kill"]: the caller skips the result)
                        why += "; not killed by the agent: the pod's memory limit (OOM)?"
                        box["external_kill"] = why
                    box["res"] = died(why)
                done.set()
        reader = threading.Thread(target=read, name=f"{what}-reader", daemon=True)
        job = Job(proc=proc, reader=reader, box=box)
        holder.append(job)
        reader.start()
        return job

    def _thread(self, what: str, fn: Callable[[], Any], done: threading.Event, died: Callable[[str], Any]) -> Job:
        box: Dict[str, Any] = {}

        def work() -> None:
            try:
                box["res"] = fn()
            except Exception as e:
                box["res"] = died(f"{type(e).__name__}: {e}"[:200])
            finally:
                done.set()
        t = threading.Thread(target=work, name=what, daemon=True)
        job = Job(thread=t, box=box)
        t.start()
        return job

    def device(self, level: int, device: int, kw: Dict[str, Any], done: threading.Event,
               host: Tuple[Any, Any] = (None, None)) -> Job:
        def died(why: str) -> Dict[str, Any]:
            return {"run": {"pass": False, "detail": why[:200]}}
        if not self.isolated:
            from ..ops import diag
            return self._thread(f"diag-gpu{device}", lambda: diag.run(level, device, **kw), done, died)
        return self._spawn(f"diag-gpu{device}", device_main, (self.setup, level, device, kw, host[0], host[1]),
                           done, died)

    def fabric(self, suite: Callable[..., Dict[str, Any]], devices: List[int], timeout_s: Optional[float],
               done: threading.Event) -> Job:
        def died(why: str) -> Dict[str, Any]:
            return {"p2p": {"pass": False, "detail": why[:200]}}
        if not self.isolated:
            return self._thread("diag-fabric", lambda: suite(devices, timeout_s), done, died)
        return self._spawn("diag-fabric", fabric_main, (self.setup, suite, devices, timeout_s), done, died)

    def enumerate(self, timeout_s: float) -> Dict[str, Any]:
        """HIP's view of the devices from a child: ``{"count", "bdf"}`` or ``{"error"}`` (one that outlives
        ``timeout_s`` is killed and said so)."""
        done = threading.Event()
        job = self._spawn("hip-enumerate", enumerate_main, (self.setup,), done, lambda why: {"error": why})
        if not done.wait(timeout_s):
            gone = job.kill()
            return {"error": f"HIP device enumeration did not finish within {timeout_s:g} s"
                             + ("" if gone else f" (process {job.pid} did not exit after SIGKILL)")}
        res = job.box.get("res") or {"error": "no result"}
        if isinstance(res.get("bdf"), dict):
            res["bdf"] = {int(k): v for k, v in res["bdf"].items()}
        return res
