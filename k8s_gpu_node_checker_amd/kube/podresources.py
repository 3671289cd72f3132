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
    ContainerResources       { string name = 1; repeated ContainerDevices devices = 2; ... }
    ContainerDevices         { string resource_name = 1; repeated string device_ids = 2; ... }

``grpc`` is optional: without it (or without the socket) :func:`allocated_devices` returns ``None`` and the
agent falls back to its amd-smi VRAM / activity heuristic.
"""

from __future__ import annotations

import os
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

DEFAULT_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
LIST_METHOD = "/v1.PodResourcesLister/List"
GPU_RESOURCES = ("amd.com/gpu",)


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
                pod["containers"].append(ctr)  # type: ignore[union-attr]
        pods.append(pod)
    return pods


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


def allocated_devices(socket_path: str = DEFAULT_SOCKET, resources: Sequence[str] = GPU_RESOURCES,
                      timeout: float = 5.0) -> Optional[Dict[str, str]]:
    """``{device id (lower case): "namespace/pod"}`` for every device of ``resources`` the kubelet has
    allocated; ``None`` when the node has no PodResources socket (not a kubelet host / not mounted)."""
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
    return out
