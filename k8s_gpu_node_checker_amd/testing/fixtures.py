"""Synthetic Kubernetes ``Node`` objects for tests and the bench.

``realistic_node`` produces a ~5.9 KB object shaped like a real kubelet-
registered node (14 labels, 6 annotations, 5 conditions with timestamps, 20
container images, ``nodeInfo``, addresses), matching the survey's proxy
harness so bench numbers compare with BASELINE.md.

The small golden clusters (``readme``, ``nogpu``, ``notready``, ``edge``,
``empty``, ``nometa``) reproduce the survey fixtures behind Appendix A.
"""

from __future__ import annotations

import hashlib
import json
import time
from typing import Any, Dict, List, Optional, Sequence

from ..models.node import HEALTH_ANNOTATION

_TS = "2025-10-10T00:00:00Z"


def _cond(ctype: str, status: str, reason: str, message: str) -> Dict[str, Any]:
    return {"type": ctype, "status": status, "lastHeartbeatTime": _TS, "lastTransitionTime": _TS,
            "reason": reason, "message": message}


def realistic_node(name: str, gpu_key: Optional[str] = "amd.com/gpu", gpu_count: int = 8, ready: bool = True,
                   index: int = 0, annotations: Optional[Dict[str, str]] = None,
                   taints: Optional[List[Dict[str, Any]]] = None, allocatable_gpus: Optional[int] = None,
                   instance_type: str = "mi355x.8x",
                   extra_conditions: Optional[List[Dict[str, Any]]] = None) -> Dict[str, Any]:
    h = hashlib.sha1(name.encode()).hexdigest()
    ip = f"10.{(index >> 16) & 255}.{(index >> 8) & 255}.{index & 255}"
    labels = {
        "beta.kubernetes.io/arch": "amd64",
        "beta.kubernetes.io/instance-type": instance_type,
        "beta.kubernetes.io/os": "linux",
        "failure-domain.beta.kubernetes.io/region": "us-central",
        "failure-domain.beta.kubernetes.io/zone": f"us-central-{'abc'[index % 3]}",
        "kubernetes.io/arch": "amd64",
        "kubernetes.io/hostname": name,
        "kubernetes.io/os": "linux",
        "node.kubernetes.io/instance-type": instance_type,
        "topology.kubernetes.io/region": "us-central",
        "topology.kubernetes.io/zone": f"us-central-{'abc'[index % 3]}",
        "node-role.kubernetes.io/gpu": "",
        "amd.com/gpu.family": "MI355X" if gpu_key == "amd.com/gpu" else "none",
        "pool": "training",
    }
    ann = {
        "node.alpha.kubernetes.io/ttl": "0",
        "volumes.kubernetes.io/controller-managed-attach-detach": "true",
        "kubeadm.alpha.kubernetes.io/cri-socket": "unix:///run/containerd/containerd.sock",
        "projectcalico.org/IPv4Address": ip + "/16",
        "csi.volume.kubernetes.io/nodeid": json.dumps({"ebs.csi.aws.com": "i-" + h[:17]}),
        "cluster.x-k8s.io/machine": "machine-" + h[:10],
    }
    if annotations:
        ann.update(annotations)
    capacity = {"cpu": "192", "ephemeral-storage": "3750000000Ki", "hugepages-1Gi": "0", "hugepages-2Mi": "0",
                "memory": "3170000000Ki", "pods": "110"}
    allocatable = {"cpu": "191500m", "ephemeral-storage": "3456000000000", "hugepages-1Gi": "0",
                   "hugepages-2Mi": "0", "memory": "3160000000Ki", "pods": "110"}
    if gpu_key:
        capacity[gpu_key] = str(gpu_count)
        allocatable[gpu_key] = str(gpu_count if allocatable_gpus is None else allocatable_gpus)
    images = [{"names": [f"registry.example.com/ml/image-{i}@sha256:{hashlib.sha256((h + str(i)).encode()).hexdigest()}",
                         f"registry.example.com/ml/image-{i}:v{i}.0"], "sizeBytes": 100000000 + i * 7919}
              for i in range(20)]
    conds = [
        _cond("MemoryPressure", "False", "KubeletHasSufficientMemory", "kubelet has sufficient memory available"),
        _cond("DiskPressure", "False", "KubeletHasNoDiskPressure", "kubelet has no disk pressure"),
        _cond("PIDPressure", "False", "KubeletHasSufficientPID", "kubelet has sufficient PID available"),
        _cond("NetworkUnavailable", "False", "CalicoIsUp", "Calico is running on this node"),
        _cond("Ready", "True" if ready else "False", "KubeletReady" if ready else "KubeletNotReady",
              "kubelet is posting ready status" if ready else "container runtime network not ready"),
    ] + list(extra_conditions or [])
    node = {
        "metadata": {
            "name": name, "uid": f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:32]}",
            "resourceVersion": str(1000 + index), "creationTimestamp": _TS,
            "labels": labels, "annotations": ann,
        },
        "spec": {"podCIDR": f"192.168.{index % 256}.0/24", "podCIDRs": [f"192.168.{index % 256}.0/24"],
                 "providerID": f"aws:///us-central-1a/i-{h[:17]}"},
        "status": {
            "capacity": capacity, "allocatable": allocatable, "conditions": conds,
            "addresses": [{"type": "InternalIP", "address": ip}, {"type": "Hostname", "address": name}],
            "daemonEndpoints": {"kubeletEndpoint": {"Port": 10250}},
            "nodeInfo": {"machineID": h, "systemUUID": h[:32], "bootID": h[::-1],
                         "kernelVersion": "6.8.0-1015-amd", "osImage": "Ubuntu 22.04.4 LTS",
                         "containerRuntimeVersion": "containerd://1.7.20", "kubeletVersion": "v1.31.2",
                         "kubeProxyVersion": "v1.31.2", "operatingSystem": "linux", "architecture": "amd64"},
            "images": images,
        },
    }
    if taints:
        node["spec"]["taints"] = taints
    return node


#: firmware image versions amd-smi reported on an MI355X box (csrc/probe fw_name(); round 2)
MI355X_FW = {"mec": 44, "rlc": 43, "sdma": 14, "psp_sos": 4522031, "ta_ras": 457506826, "ta_xgmi": 536870932,
             "pm": 72748906, "pldm_bundle": 18419975}
MI355X_DRIVER = {"name": "amdgpu", "version": "6.18.54"}
MI355X_HIVE = "bbf0a3c1d2e4f5fe"


def mi355x_probe_report(node: str, gpus: int = 8, ts: Optional[float] = None, **overrides: Any) -> Dict[str, Any]:
    """A probe report as the node agent publishes it (values measured on a real MI355X)."""
    entries = []
    for i in range(gpus):
        g = {"index": i, "bdf": f"0000:{0x05 + 0x10 * i:02x}:00.0", "gfx": "gfx950",
             "market_name": "AMD Instinct MI355 OAM", "product_name": "AMD Instinct MI355 OAM",
             "vbios_name": "AMD MI355X", "device_id": "0x75a3",
             "cus": 256, "vram_type": 5, "vram_mb": 294896, "ecc_correctable": 0, "ecc_uncorrectable": 0,
             "ecc_deferred": 0, "bad_pages": 0, "xgmi": "XUUUUUUU", "kfd": True,
             "compute_partition": "SPX", "memory_partition": "NPS1", "hotspot_c": 45,
             "pcie_width": 16, "pcie_max_width": 16, "pcie_speed_mts": 32000, "pcie_max_speed_mts": 32000,
             "pcie_replays": 0, "pcie_recoveries": 0, "power_w": 260, "power_cap_w": 1400,
             "power_cap_default_w": 1400, "hbm_temp_c": 34, "gfxclk_mhz": 157, "vram_used_mb": 283,
             "processes": 0, "throttle_acc": {"n": 499923464, "prochot": 0, "ppt": 1486216, "socket_thm": 0,
                                              "vr_thm": 0, "hbm_thm": 0},
             "vbios_version": "00175784", "fw": dict(MI355X_FW), "xgmi_hive": MI355X_HIVE,
             "xgmi_width": 16, "xgmi_speed_gbps": 38,
             "xgmi_peers": [f"0000:{0x05 + 0x10 * j:02x}:00.0" for j in range(gpus) if j != i]}
        g.update(overrides.get(f"gpu{i}", {}))
        entries.append(g)
    rep = {"schema": "mi355x-health/v1", "node": node, "ts": time.time() if ts is None else ts,
           "probe": "fixture", "driver": dict(MI355X_DRIVER), "gpus": entries}
    for k, v in overrides.items():
        if not k.startswith("gpu"):
            rep[k] = v
    return rep


def health_annotation(report: Dict[str, Any], encoding: str = "json") -> Dict[str, str]:
    """The report annotation as an agent with ``--annotation-encoding <encoding>`` writes it."""
    from ..models.health import encode_annotation
    return {HEALTH_ANNOTATION: encode_annotation(report, encoding)}


def health_condition(report: Dict[str, Any], expected_gpus: int = 0) -> Dict[str, Any]:
    """The ``AMDGPUHealthy`` NodeCondition an agent would publish for ``report``."""
    from ..models.health import condition_for, evaluate_report
    return condition_for(evaluate_report(report, expected_gpus))


def cluster(n: int, kind: str = "amd", not_ready: Sequence[int] = (), gpus_per_node: int = 8,
            with_health: bool = False, prefix: str = "mi355x-node",
            annotation_encoding: str = "json") -> List[Dict[str, Any]]:
    """``kind``: ``amd`` | ``nvidia`` | ``mixed`` (alternating, as the survey's 1000-node run) | ``cpu``."""
    nodes = []
    for i in range(n):
        if kind == "cpu":
            key = None
        elif kind == "nvidia":
            key = "nvidia.com/gpu"
        elif kind == "mixed":
            key = "amd.com/gpu" if i % 2 == 0 else "nvidia.com/gpu"
        else:
            key = "amd.com/gpu"
        name = f"{prefix}-{i:04d}" if kind != "cpu" else f"cpu-node-{i:04d}"
        ann, conds = None, None
        if with_health and key == "amd.com/gpu":
            rep = mi355x_probe_report(name, gpus_per_node)
            ann, conds = health_annotation(rep, annotation_encoding), [health_condition(rep, gpus_per_node)]
        nodes.append(realistic_node(name, key, gpus_per_node, ready=i not in not_ready, index=i, annotations=ann,
                                    extra_conditions=conds))
    return nodes


def _simple(name: Optional[str], caps: Optional[Dict[str, Any]], ready: Optional[bool] = True,
            labels: Optional[Dict[str, str]] = None, taints: Optional[List[Dict[str, Any]]] = None,
            allocatable: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    node: Dict[str, Any] = {"metadata": {"name": name}, "spec": {}, "status": {}}
    if labels is not None:
        node["metadata"]["labels"] = labels
    if caps is not None:
        node["status"]["capacity"] = caps
    if allocatable is not None:
        node["status"]["allocatable"] = allocatable
    if ready is not None:
        node["status"]["conditions"] = [{"type": "Ready", "status": "True" if ready else "False"}]
    if taints is not None:
        node["spec"]["taints"] = taints
    return node


def golden(name: str) -> List[Dict[str, Any]]:
    """Survey §4.3 fixtures (inputs of Appendix A)."""
    if name == "readme":
        return [_simple("gpu-node-1", {"nvidia.com/gpu": "4"}, labels={"node.kubernetes.io/instance-type": "g4dn.xlarge"}),
                _simple("gpu-node-2", {"nvidia.com/gpu": "8"})]
    if name == "nogpu":
        return [_simple(f"cpu-{i}", {"cpu": "8"}) for i in range(3)]
    if name == "notready":
        return [_simple("gpu-a", {"amd.com/gpu": "8"}, ready=False), _simple("gpu-b", {"amd.com/gpu": "8"}, ready=None)]
    if name == "edge":
        return [
            _simple("zero-and-amd", {"nvidia.com/gpu": "0", "amd.com/gpu": "8"}),
            _simple("only-zero", {"nvidia.com/gpu": "0"}),
            _simple("weird-qty", {"amd.com/gpu": "1k", "intel.com/gpu": "2"}, labels={"k": "한글"}),
            _simple("mixed-all-keys", {"intel.com/gpu": "1", "gpu.intel.com/i915": "2", "amd.com/gpu": "3",
                                       "nvidia.com/gpu": "4"},
                    taints=[{"key": "amd.com/gpu", "effect": "NoSchedule"},
                            {"key": "dedicated", "value": "ml", "effect": "NoExecute", "timeAdded": _TS}]),
            _simple("alloc-only", {"cpu": "8"}, allocatable={"amd.com/gpu": "8"}),
            _simple("a-very-long-node-name-0123456789", {"amd.com/gpu": "8"}, ready=False),
        ]
    if name == "empty":
        return []
    if name == "nometa":
        return [{"metadata": None, "spec": None, "status": {"capacity": {"amd.com/gpu": "2"},
                                                           "conditions": [{"type": "Ready", "status": "True"}]}}]
    raise KeyError(name)


GOLDEN = ("readme", "nogpu", "notready", "edge", "empty", "nometa")


def node_list(items: List[Dict[str, Any]], cont: Optional[str] = None, rv: str = "12345") -> Dict[str, Any]:
    meta: Dict[str, Any] = {"resourceVersion": rv}
    if cont:
        meta["continue"] = cont
    return {"kind": "NodeList", "apiVersion": "v1", "metadata": meta, "items": items}
