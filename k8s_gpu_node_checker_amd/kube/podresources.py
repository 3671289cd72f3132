"""Kubelet PodResources API client: which GPUs the scheduler has handed to pods on this node.

The node agent must not run active diagnostics on a GPU that is allocated to a pod, even before the pod
touches it (amd-smi shows no process and no VRAM until it does).  The kubelet says which devices it
allocated through the PodResources gRPC service on a node-local unix socket
(``/var/lib/kubelet/pod-resources/kubelet.sock``, ``v1.PodResourcesLister/List``); the ROCm device
plugin registers ``amd.com/gpu`` devices under their PCI address (``0000:05:00.0``), the same BDF the
probe reports per GPU.

The reference has only the scheduler's view (``status.capacity``, ``check-gpu-node.py:186-195``); this is
the node-side view of the same allocations, so the health gate never fights the scheduler.

No generated stubs: the request is an empty message and the response is decoded from the protobuf wire
format here (fields from ``k8s.io/kubelet/pkg/apis/podresources/v1/api.proto``):

    ListPodResourcesResponse { repeated PodResources pod_resources = 1; }
    PodResources             { string name = 1; string namespace = 2; repeated ContainerResources containers = 3; }
    ContainerResources       { string name = 1; repeated ContainerDevices devices = 2; ...;
                               repeated DynamicResource dynamic_resources = 5; }
    ContainerDevices         { string resource_name = 1; repeated string device_ids = 2; ... }
    DynamicResource          { string claim_name = 2; string claim_namespace = 3;
                               repeated ClaimResource claim_resources = 4; }
    ClaimResource            { repeated CDIDevice cdi_devices = 1; string driver_name = 2; string pool_name = 3;
                               string device_name = 4; }
    CDIDevice                { string name = 1; }

Dynamic Resource Allocation: a GPU can reach a pod through a ResourceClaim of a DRA driver instead of the
``amd.com/gpu`` extended resource; the kubelet reports those under ``dynamic_resources``
(KubeletPodResourcesDynamicResources).  A claim device of an AMD GPU DRA driver (``gpu.amd.com`` /
``amd.com``, or a CDI name in those vendors' namespaces) counts as allocated: keyed by the PCI address when
its device or CDI name carries one, else by ``driver/pool/device`` -- an ID the agent cannot map to a local
GPU, which makes it skip every GPU rather than guess (``Agent._unmatched_allocations``).

``grpc`` is optional: without it (or without the socket) :func:`allocated_devices` returns ``None`` and the
agent falls back to its amd-smi VRAM / activity heuristic.
"""

from __future__ import annotations

import os
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

DEFAULT_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
LIST_METHOD = "/v1.PodResourcesLister/List"
GPU_RESOURCES = ("amd.com/gpu",)
DRA_DRIVERS = ("gpu.amd.com", "amd.com")


class PodResourcesError(RuntimeError):
    """The socket exists but the kubelet could not be asked (permission, protocol, timeout)."""


# --- protobuf wire format (varint / length-delimited only: all this API's fields we read) ---------------

def _varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = value = 0
    while True:
        if i >= len(buf):
            raise ValueError("truncated varint")
        b = buf[i]
        i += 1
        value |= (b & 0x7F) << shift
        if not b & 0x80:
            return value, i
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _fields(buf: bytes) -> Iterator[Tuple[int, int, object]]:
    """(field number, wire type, value) for every field of one message; unknown types are skipped."""
    i = 0
    while i < len(buf):
        key, i = _varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
            yield num, wt, v
        elif wt == 2:
            n, i = _varint(buf, i)
            if i + n > len(buf):
                raise ValueError("truncated field")
            yield num, wt, buf[i:i + n]
            i += n
        elif wt == 1:
            i += 8
        elif wt == 5:
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")


def _str(v: object) -> str:
    return bytes(v).decode("utf-8", errors="replace") if isinstance(v, (bytes, bytearray, memoryview)) else ""


def decode_list_response(buf: bytes) -> List[Dict[str, object]]:
    """``ListPodResourcesResponse`` -> ``[{"name", "namespace", "containers": [{"name", "devices":
    [{"resource_name", "device_ids": [...]}]}]}]``."""
    pods = []
    for num, wt, v in _fields(buf):
        if num != 1 or wt != 2:
            continue
        pod: Dict[str, object] = {"name": "", "namespace": "", "containers": []}
        for pn, pw, pv in _fields(bytes(v)):  # type: ignore[arg-type]
            if pn == 1 and pw == 2:
                pod["name"] = _str(pv)
            elif pn == 2 and pw == 2:
                pod["namespace"] = _str(pv)
            elif pn == 3 and pw == 2:
                ctr: Dict[str, object] = {"name": "", "devices": []}
                for cn, cw, cv in _fields(bytes(pv)):  # type: ignore[arg-type]
                    if cn == 1 and cw == 2:
                        ctr["name"] = _str(cv)
                    elif cn == 2 and cw == 2:
                        dev: Dict[str, object] = {"resource_name": "", "device_ids": []}
                        for dn, dw, dv in _fields(bytes(cv)):  # type: ignore[arg-type]
                            if dn == 1 and dw == 2:
                                dev["resource_name"] = _str(dv)
                            elif dn == 2 and dw == 2:
                                dev["device_ids"].append(_str(dv))  # type: ignore[union-attr]
                        ctr["devices"].append(dev)  # type: ignore[union-attr]
                    elif cn == 5 and cw == 2:
                        ctr.setdefault("dynamic", []).append(_decode_dynamic(bytes(cv)))  # type: ignore[union-attr]
                pod["containers"].append(ctr)  # type: ignore[union-attr]
        pods.append(pod)
    return pods


def _decode_dynamic(buf: bytes) -> Dict[str, object]:
    """``DynamicResource`` -> ``{"claim_name", "claim_namespace", "devices": [{"driver", "pool", "device",
    "cdi": [...]}]}``."""
    out: Dict[str, object] = {"claim_name": "", "claim_namespace": "", "devices": []}
    for n, w, v in _fields(buf):
        if n == 2 and w == 2:
            out["claim_name"] = _str(v)
        elif n == 3 and w == 2:
            out["claim_namespace"] = _str(v)
        elif n == 4 and w == 2:
            dev: Dict[str, object] = {"driver": "", "pool": "", "device": "", "cdi": []}
            for rn, rw, rv in _fields(bytes(v)):  # type: ignore[arg-type]
                if rn == 1 and rw == 2:
                    for cn, cw, cv in _fields(bytes(rv)):  # type: ignore[arg-type]
                        if cn == 1 and cw == 2:
                            dev["cdi"].append(_str(cv))  # type: ignore[union-attr]
                elif rn == 2 and rw == 2:
                    dev["driver"] = _str(rv)
                elif rn == 3 and rw == 2:
                    dev["pool"] = _str(rv)
                elif rn == 4 and rw == 2:
                    dev["device"] = _str(rv)
            out["devices"].append(dev)  # type: ignore[union-attr]
    return out


def _enc_varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def _enc_bytes(num: int, payload: bytes) -> bytes:
    return _enc_varint(num << 3 | 2) + _enc_varint(len(payload)) + payload


def encode_list_response(pods: Sequence[Dict[str, object]]) -> bytes:
    """Inverse of :func:`decode_list_response` (the fake kubelet in the tests serves this)."""
    out = bytearray()
    for pod in pods:
        p = _enc_bytes(1, str(pod.get("name", "")).encode()) + _enc_bytes(2, str(pod.get("namespace", "")).encode())
        for ctr in pod.get("containers") or []:  # type: ignore[union-attr]
            c = _enc_bytes(1, str(ctr.get("name", "")).encode())
            for dev in ctr.get("devices") or []:
                d = _enc_bytes(1, str(dev.get("resource_name", "")).encode())
                for did in dev.get("device_ids") or []:
                    d += _enc_bytes(2, str(did).encode())
                c += _enc_bytes(2, d)
            for dyn in ctr.get("dynamic") or []:
                r = _enc_bytes(2, str(dyn.get("claim_name", "")).encode()) + \
                    _enc_bytes(3, str(dyn.get("claim_namespace", "")).encode())
                for dev in dyn.get("devices") or []:
                    cr = b"".join(_enc_bytes(1, _enc_bytes(1, str(name).encode())) for name in dev.get("cdi") or [])
                    cr += _enc_bytes(2, str(dev.get("driver", "")).encode()) + \
                        _enc_bytes(3, str(dev.get("pool", "")).encode()) + \
                        _enc_bytes(4, str(dev.get("device", "")).encode())
                    r += _enc_bytes(4, cr)
                c += _enc_bytes(5, r)
            p += _enc_bytes(3, c)
        out += _enc_bytes(1, p)
    return bytes(out)


# --- the kubelet call ---------------------------------------------------------------------------------

def list_pod_resources(socket_path: str = DEFAULT_SOCKET, timeout: float = 5.0) -> List[Dict[str, object]]:
    """One ``List`` call against the kubelet.  Raises :class:`PodResourcesError` on any failure."""
    try:
        import grpc
    except ImportError as e:  # pragma: no cover - grpc is in the image; stay usable without it
        raise PodResourcesError(f"grpc not importable: {e}") from e
    try:
        with grpc.insecure_channel(f"unix://{socket_path}") as ch:
            call = ch.unary_unary(LIST_METHOD, request_serializer=lambda _: b"",
                                  response_deserializer=decode_list_response)
            return call(None, timeout=timeout)
    except grpc.RpcError as e:
        code = e.code() if hasattr(e, "code") else None
        raise PodResourcesError(f"PodResources List failed: {getattr(code, 'name', code)}: "
                                f"{e.details() if hasattr(e, 'details') else e}") from e
    except ValueError as e:
        raise PodResourcesError(f"PodResources List: bad response ({e})") from e


def _pci_address(text: str) -> Optional[str]:
    """The first PCI address (``0000:05:00.0`` or ``05:00.0``) inside a device or CDI name, lower case."""
    t = text.lower()
    for i in range(len(t)):
        for width in (12, 7):  # dddd:bb:dd.f / bb:dd.f
            cand = t[i:i + width]
            if len(cand) != width or (i and t[i - 1] in "0123456789abcdef:"):
                continue
            if width == 12 and not (cand[4] == ":" and cand[7] == ":" and cand[10] == "."):
                continue
            if width == 7 and not (cand[2] == ":" and cand[5] == "."):
                continue
            hexpart = cand.replace(":", "").replace(".", "")
            if all(c in "0123456789abcdef" for c in hexpart) and cand[-1] in "01234567":
                if i + width < len(t) and t[i + width] in "0123456789abcdef":
                    continue
                return cand
    return None


def _is_amd_claim_device(dev: Dict[str, object], drivers: Sequence[str]) -> bool:
    if str(dev.get("driver") or "") in drivers:
        return True
    return any(str(c).split("/", 1)[0] in drivers for c in dev.get("cdi") or [])  # type: ignore[union-attr]


def allocated_devices(socket_path: str = DEFAULT_SOCKET, resources: Sequence[str] = GPU_RESOURCES,
                      timeout: float = 5.0, dra_drivers: Sequence[str] = DRA_DRIVERS) -> Optional[Dict[str, str]]:
    """``{device id (lower case): "namespace/pod"}`` for every device of ``resources`` the kubelet has
    allocated, and every AMD GPU a DRA claim gave a pod (by PCI address when its name carries one, else
    ``driver/pool/device``); ``None`` when the node has no PodResources socket (not a kubelet host / not
    mounted)."""
    if not os.path.exists(socket_path):
        return None
    out: Dict[str, str] = {}
    for pod in list_pod_resources(socket_path, timeout):
        owner = f"{pod.get('namespace')}/{pod.get('name')}"
        for ctr in pod.get("containers") or []:  # type: ignore[union-attr]
            for dev in ctr.get("devices") or []:
                if dev.get("resource_name") in resources:
                    for did in dev.get("device_ids") or []:
                        out[str(did).lower()] = owner
            for dyn in ctr.get("dynamic") or []:
                claim = f"{owner} (claim {dyn.get('claim_namespace') or pod.get('namespace')}/{dyn.get('claim_name')})"
                for dev in dyn.get("devices") or []:  # type: ignore[union-attr]
                    if not _is_amd_claim_device(dev, dra_drivers):
                        continue
                    names = [str(dev.get("device") or "")] + [str(c) for c in dev.get("cdi") or []]  # type: ignore[union-attr]
                    bdf = next((a for a in map(_pci_address, names) if a), None)
                    key = bdf or "/".join(str(dev.get(k) or "") for k in ("driver", "pool", "device")).lower()
                    out[key] = claim
    return out
