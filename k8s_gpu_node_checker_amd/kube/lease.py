"""Leader election on a ``coordination.k8s.io/v1`` Lease, for running the event-driven watcher
(``--watch-events``) as more than one replica: exactly one replica -- the holder of the Lease --
follows the cluster and sends Slack; the others wait, and take over when the holder stops renewing.

The protocol is the one client-go's ``leaderelection`` package speaks, so this process and any other
Kubernetes component can share a Lease correctly:

* the record is ``spec.holderIdentity`` / ``leaseDurationSeconds`` / ``acquireTime`` / ``renewTime`` /
  ``leaseTransitions``, and every write is a ``PUT`` carrying the ``resourceVersion`` it read (a concurrent
  writer gets ``409 Conflict`` and loses that round);
* a candidate may take the Lease only after it has watched the same record stay unchanged for
  ``leaseDurationSeconds`` on its *own* clock (observed time, not the holder's ``renewTime``: no reliance on
  synchronised clocks);
* the holder renews every ``retry_period`` and gives leadership up when it has not managed to renew for
  ``renew_deadline`` (< lease duration), before any candidate can take over;
* a holder that stops cleanly releases the Lease (empty holder, duration 1 s) so the next replica need not
  wait for the lease to expire.

The holder also keeps a small JSON state on the Lease (annotation ``STATE_ANNOTATION``, written with its
renewals: :meth:`LeaderElector.publish_state`), and a replica that takes the Lease over reads it
(:attr:`LeaderElector.inherited_state`).  The watcher keeps its last-notified outcome there, so a failover
neither re-sends the alert the old leader already sent nor loses a recovery that happened during the handover.

The reference has no counterpart: it is a one-shot script (``/root/reference/check-gpu-node.py:296-327``); this
is what running its check as a long-lived, replicated Deployment needs (``deploy/watcher.yaml``).
"""

from __future__ import annotations

import json
import threading
import time
from typing import TYPE_CHECKING, Any, Callable, Dict, Optional, Tuple
from urllib.parse import quote

if TYPE_CHECKING:
    from .client import KubeClient

LEASE_DURATION_S = 15.0  # client-go defaults (kube-controller-manager, kube-scheduler)
RENEW_DEADLINE_S = 10.0
RETRY_PERIOD_S = 2.0
STATE_ANNOTATION = "gpu-health.amd.com/leader-state"
# the apiserver caps an object's annotations at 256 KiB: a state larger than this is not kept on the Lease
# (utils/statefile.compact shrinks an outcome to it first)
from ..utils.statefile import STATE_MAX_BYTES  # noqa: E402


def _micro_time(epoch: float) -> str:
    """``metav1.MicroTime``: RFC 3339 with microseconds."""
    return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(epoch)) + ".%06dZ" % int((epoch % 1) * 1e6)


def _lease_path(namespace: str, name: Optional[str] = None) -> str:
    base = f"/apis/coordination.k8s.io/v1/namespaces/{quote(namespace)}/leases"
    return base + (f"/{quote(name)}" if name else "")


class LeaderElector:
    """Acquire and hold the Lease ``namespace/name`` as ``identity``.

    ``make_client()`` returns a fresh :class:`~k8s_gpu_node_checker_amd.kube.client.KubeClient`; the elector
    keeps one for its thread.  Use :meth:`start` / :meth:`stop`, then :attr:`leading` (an Event set while this
    process holds the Lease) and :attr:`lost` (set once leadership held before was given up).
    """

    def __init__(self, make_client: Callable[[], "KubeClient"], namespace: str, name: str, identity: str,
                 lease_duration: float = LEASE_DURATION_S, renew_deadline: float = RENEW_DEADLINE_S,
                 retry_period: float = RETRY_PERIOD_S, clock: Callable[[], float] = time.monotonic,
                 wall: Callable[[], float] = time.time):
        if not 0 < retry_period < renew_deadline < lease_duration:
            raise ValueError("leader election needs 0 < retry period < renew deadline < lease duration")
        self.make_client = make_client
        self.namespace = namespace
        self.name = name
        self.identity = identity
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.clock = clock
        self.wall = wall
        self.leading = threading.Event()
        self.lost = threading.Event()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._observed: Optional[Tuple[Any, ...]] = None  # (holder, renewTime, acquireTime, transitions)
        self._observed_at = 0.0  # our clock when that record was first seen
        self._last_renew = 0.0
        self.transitions = 0
        self.last_error: Optional[str] = None
        # the leader's shared state: what the holder writes with its renewals, what a new holder found there
        self._state: Optional[str] = None
        self._state_lock = threading.Lock()
        self._wake = threading.Event()
        self.inherited_state: Optional[Dict[str, Any]] = None

    # -- one round -------------------------------------------------------------------------------------
    def try_acquire_or_renew(self, client: "KubeClient") -> bool:
        """One round of client-go's ``tryAcquireOrRenew``: True when this process holds the Lease after it."""
        from .errors import ApiException
        now_wall = self.wall()
        record = {"holderIdentity": self.identity, "leaseDurationSeconds": int(round(self.lease_duration)),
                  "acquireTime": _micro_time(now_wall), "renewTime": _micro_time(now_wall), "leaseTransitions": 0}
        try:
            resp = client.request("GET", _lease_path(self.namespace, self.name))
            lease = json.loads(resp.body)
        except ApiException as e:
            if e.status != 404:
                raise
            body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                    "metadata": {"name": self.name, "namespace": self.namespace}, "spec": record}
            try:
                client.request("POST", _lease_path(self.namespace), json.dumps(body).encode(),
                               content_type="application/json", idempotent=False)
            except ApiException as e2:
                if e2.status == 409:  # another candidate created it first
                    return False
                raise
            self._observe(tuple(record[k] for k in ("holderIdentity", "renewTime", "acquireTime",
                                                    "leaseTransitions")))
            return True
        spec: Dict[str, Any] = lease.get("spec") or {}
        seen = (spec.get("holderIdentity"), spec.get("renewTime"), spec.get("acquireTime"),
                spec.get("leaseTransitions"))
        self._observe(seen)
        holder = spec.get("holderIdentity") or ""
        duration = float(spec.get("leaseDurationSeconds") or self.lease_duration)
        if holder and holder != self.identity and self.clock() < self._observed_at + duration:
            return False  # held, and renewed within the lease duration as far as this process has seen
        if holder == self.identity:
            record["acquireTime"] = spec.get("acquireTime") or record["acquireTime"]
            record["leaseTransitions"] = int(spec.get("leaseTransitions") or 0)
        else:
            record["leaseTransitions"] = int(spec.get("leaseTransitions") or 0) + 1
        lease["spec"] = record
        meta = lease.setdefault("metadata", {})
        found = (meta.get("annotations") or {}).get(STATE_ANNOTATION)
        with self._state_lock:
            mine = self._state
        if mine is not None:
            meta["annotations"] = dict(meta.get("annotations") or {}, **{STATE_ANNOTATION: mine})
        try:
            client.request("PUT", _lease_path(self.namespace, self.name), json.dumps(lease).encode(),
                           content_type="application/json", idempotent=False)
        except ApiException as e:
            if e.status == 409:  # someone else wrote it since our GET
                return False
            raise
        if holder != self.identity:
            self.transitions += 1
            try:  # what the previous holder left: this replica's starting point
                state = json.loads(found) if isinstance(found, str) else None
                self.inherited_state = state if isinstance(state, dict) else None
            except ValueError:
                self.inherited_state = None
        self._observe(tuple(record[k] for k in ("holderIdentity", "renewTime", "acquireTime", "leaseTransitions")))
        return True

    def _observe(self, record: Tuple[Any, ...]) -> None:
        if record != self._observed:
            self._observed = record
            self._observed_at = self.clock()

    def release(self, client: "KubeClient") -> bool:
        """Give the Lease up (holder cleared, 1 s duration) if this process holds it."""
        from .errors import ApiException
        try:
            lease = json.loads(client.request("GET", _lease_path(self.namespace, self.name)).body)
            spec = lease.get("spec") or {}
            if spec.get("holderIdentity") != self.identity:
                return False
            now_wall = self.wall()
            lease["spec"] = dict(spec, holderIdentity="", leaseDurationSeconds=1, renewTime=_micro_time(now_wall),
                                 acquireTime=_micro_time(now_wall))
            client.request("PUT", _lease_path(self.namespace, self.name), json.dumps(lease).encode(),
                           content_type="application/json", idempotent=False)
            return True
        except (ApiException, OSError, ValueError) as e:
            self.last_error = f"release: {e}"[:200]
            return False

    # -- the loop --------------------------------------------------------------------------------------
    def _round(self, client: "KubeClient") -> bool:
        try:
            ok = self.try_acquire_or_renew(client)
            self.last_error = None
            return ok
        except Exception as e:  # apiserver unreachable / refusing: this round failed
            self.last_error = f"{type(e).__name__}: {e}"[:200]
            return False

    def _run(self) -> None:
        client = self.make_client()
        try:
            # acquire: one round every retry_period until the Lease is ours (or we are stopped)
            # a renewal counts from the moment its round *started*: the apiserver applied the write no earlier,
            # so others' lease expiry (observed after the write) is later than ours by at least the write's latency
            while not self._stop.is_set():
                started = self.clock()
                if self._round(client):
                    self._last_renew = started
                    self.leading.set()
                    break
                self._stop.wait(self.retry_period)
            # renew: give up when no round succeeded for renew_deadline
            while not self._stop.is_set() and self.leading.is_set():
                self._wake.wait(self.retry_period)  # a new state to publish renews at once
                self._wake.clear()
                if self._stop.is_set():
                    break
                started = self.clock()
                if self._round(client):
                    self._last_renew = started
                elif self.clock() - self._last_renew >= self.renew_deadline:
                    self.leading.clear()
                    self.lost.set()
            if self._stop.is_set() and self.leading.is_set():
                self.release(client)
                self.leading.clear()
        finally:
            client.close()

    def start(self) -> "LeaderElector":
        self._thread = threading.Thread(target=self._run, name="leader-election", daemon=True)
        self._thread.start()
        return self

    def publish_state(self, state: Dict[str, Any]) -> bool:
        """Keep ``state`` (JSON) on the Lease: written by the next renewal, which is started right away.  A state
        over ``STATE_MAX_BYTES`` (a cluster with thousands of not-Ready node names) is not kept -- the Lease's
        annotations must stay small -- and the previous one is dropped; False then."""
        text = json.dumps(state, sort_keys=True, separators=(",", ":"))
        fits = len(text) <= STATE_MAX_BYTES
        if not fits:
            text = "{}"
        with self._state_lock:
            changed = text != self._state
            self._state = text
        if changed:  # an unchanged state rides on the periodic renewal: no extra Lease write per evaluation
            self._wake.set()
        return fits

    def stop(self, timeout: float = 5.0) -> None:
        """Stop campaigning; a holder releases the Lease on the way out."""
        self._stop.set()
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout)

    def is_leader(self) -> bool:
        """Leadership that is still within its renew deadline: the check a leader makes before it acts."""
        return self.leading.is_set() and self.clock() - self._last_renew < self.renew_deadline


def default_identity() -> str:
    """``$POD_NAME`` (the Downward API, ``deploy/watcher.yaml``), else ``hostname_pid``."""
    import os
    import socket
    return os.environ.get("POD_NAME") or f"{socket.gethostname()}_{os.getpid()}"


def default_namespace() -> str:
    """The pod's own namespace (service-account mount), else ``default``."""
    try:
        with open("/var/run/secrets/kubernetes.io/serviceaccount/namespace", encoding="utf-8") as f:
            ns = f.read().strip()
        return ns or "default"
    except OSError:
        return "default"
