"""Kubelet PodResources API (kube/podresources.py) and the agent's use of it: a fake kubelet serves
``v1.PodResourcesLister/List`` over a unix socket with grpc; the agent must skip the GPU allocated to a pod
(even though amd-smi shows it idle) and diagnose the free one."""
import os
import tempfile
import time
from concurrent import futures

import pytest

from k8s_gpu_node_checker_amd.agent import agent as A
from k8s_gpu_node_checker_amd.kube import podresources as PR
from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag
from k8s_gpu_node_checker_amd.testing import fixtures

grpc = pytest.importorskip("grpc")

PODS = [
    {"name": "trainer-0", "namespace": "ml", "containers": [
        {"name": "main", "devices": [{"resource_name": "amd.com/gpu", "device_ids": ["0000:15:00.0"]},
                                     {"resource_name": "example.com/nic", "device_ids": ["0000:05:00.0"]}]}]},
    {"name": "idle-pod", "namespace": "default", "containers": [{"name": "c", "devices": []}]},
]


class FakeKubelet:
    def __init__(self, pods, code=None):
        self.pods = pods
        self.code = code
        self.calls = 0
        self.dir = tempfile.mkdtemp(prefix="podres")  # short path: unix socket names are <= 107 bytes
        self.sock = os.path.join(self.dir, "kubelet.sock")

    def __enter__(self):
        def handle(req, ctx):
            self.calls += 1
            assert req == b""
            if self.code is not None:
                ctx.abort(self.code, "denied by the fake kubelet")
            return PR.encode_list_response(self.pods)
        handler = grpc.method_handlers_generic_handler("v1.PodResourcesLister", {
            "List": grpc.unary_unary_rpc_method_handler(handle, request_deserializer=lambda b: b,
                                                        response_serializer=lambda b: b)})
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        self.server.add_generic_rpc_handlers((handler,))
        self.server.add_insecure_port(f"unix://{self.sock}")
        self.server.start()
        return self

    def __exit__(self, *a):
        self.server.stop(None)


def test_wire_roundtrip_and_unknown_fields():
    buf = PR.encode_list_response(PODS)
    assert PR.decode_list_response(buf) == [
        {"name": "trainer-0", "namespace": "ml", "containers": [
            {"name": "main", "devices": [{"resource_name": "amd.com/gpu", "device_ids": ["0000:15:00.0"]},
                                         {"resource_name": "example.com/nic", "device_ids": ["0000:05:00.0"]}]}]},
        {"name": "idle-pod", "namespace": "default", "containers": [{"name": "c", "devices": []}]}]
    # fields this client does not read (cpu_ids varint list, topology, fixed64) are skipped
    extra = PR._enc_varint(3 << 3 | 0) + PR._enc_varint(7) + PR._enc_varint(9 << 3 | 1) + b"\0" * 8
    pod = PR._enc_bytes(1, b"p") + PR._enc_bytes(2, b"ns") + PR._enc_bytes(3, PR._enc_bytes(1, b"c") + extra)
    assert PR.decode_list_response(PR._enc_bytes(1, pod))[0]["containers"] == [{"name": "c", "devices": []}]
    with pytest.raises(ValueError):
        PR.decode_list_response(PR._enc_bytes(1, pod)[:-3])


def test_allocated_devices_from_a_fake_kubelet():
    with FakeKubelet(PODS) as k:
        assert PR.allocated_devices(k.sock) == {"0000:15:00.0": "ml/trainer-0"}
        assert PR.allocated_devices(k.sock, ("example.com/nic",)) == {"0000:05:00.0": "ml/trainer-0"}
    assert PR.allocated_devices("/nonexistent/kubelet.sock") is None
    with FakeKubelet(PODS, code=grpc.StatusCode.PERMISSION_DENIED) as k:
        with pytest.raises(PR.PodResourcesError, match="PERMISSION_DENIED"):
            PR.allocated_devices(k.sock)


def _world(monkeypatch, n=2):
    gpus = []
    for i in range(n):
        g = dict(fixtures.mi355x_probe_report("n", gpus=n)["gpus"][i])
        g.update({"index": i, "bdf": f"0000:{0x05 + 0x10 * i:02x}:00.0", "procs": [], "processes": 0,
                  "vram_used_mb": 280, "gfx_activity": 0})  # amd-smi: both GPUs idle
        gpus.append(g)
    runs = []
    monkeypatch.setattr(amdsmi_probe, "probe", lambda node, src, fx: {
        "schema": "mi355x-health/v1", "node": node, "ts": time.time(), "probe": "fake", "gpus": [dict(g) for g in gpus]})
    monkeypatch.setattr(diag, "device_count", lambda: n)
    monkeypatch.setattr(diag, "device_info", lambda d: {"bdf": f"0000:{0x05 + 0x10 * d:02x}:00.0"})

    def run(level, d, memory_partition=None, **kw):
        runs.append(d)
        return {"gemm": {"pass": True, "tflops": 1220.0}}
    monkeypatch.setattr(diag, "run", run)
    return runs


def test_agent_skips_the_gpu_a_pod_was_allocated(monkeypatch):
    runs = _world(monkeypatch)
    with FakeKubelet(PODS) as k:
        ag = A.Agent("n", source="fake", diag_level=1, pod_resources_socket=k.sock)
        rep = ag.probe_once()
        assert k.calls == 1
    assert runs == [0]
    g0, g1 = rep["gpus"]
    assert g0["diag"]["gemm"]["pass"] and "diag_skipped" not in g0
    assert g1["diag_skipped"] == "allocated to pod ml/trainer-0" and "diag" not in g1
    assert rep["pod_resources"] == "ok" and rep["state"] == "healthy"
    # the node-level fabric test waits for a node with no allocated GPU
    assert "fabric" not in rep


def test_agent_falls_back_to_the_heuristic(monkeypatch, capsys):
    runs = _world(monkeypatch)
    ag = A.Agent("n", source="fake", diag_level=1, pod_resources_socket="/nonexistent/kubelet.sock")
    rep = ag.probe_once()
    assert sorted(runs) == [0, 1] and rep["pod_resources"] == "absent"
    runs.clear()
    with FakeKubelet(PODS, code=grpc.StatusCode.UNAVAILABLE) as k:
        ag = A.Agent("n", source="fake", diag_level=1, pod_resources_socket=k.sock)
        rep = ag.probe_once()
    assert sorted(runs) == [0, 1] and rep["pod_resources"].startswith("error: PodResources List failed: UNAVAILABLE")
    assert "using the amd-smi busy heuristic" in capsys.readouterr().err


def test_domainless_device_ids_match():
    assert A.normalize_bdf("15:00.0") == "0000:15:00.0" and A.normalize_bdf("0000:DC:00.0") == "0000:dc:00.0"
    assert A.normalize_bdf(None) == ""


def test_agent_cli_flags():
    a = A.build_parser().parse_args(["--pod-resources-socket", "/var/lib/kubelet/pod-resources/kubelet.sock",
                                     "--gpu-resource", "amd.com/gpu", "--gpu-resource", "amd.com/gpu-cpx"])
    assert a.pod_resources_socket.endswith("kubelet.sock") and a.gpu_resource == ["amd.com/gpu", "amd.com/gpu-cpx"]


DRA_PODS = [
    {"name": "dra-trainer", "namespace": "ml", "containers": [
        {"name": "main", "devices": [], "dynamic": [
            {"claim_name": "gpu-claim", "claim_namespace": "ml", "devices": [
                {"driver": "gpu.amd.com", "pool": "node-a", "device": "gpu-0000-15-00-0",
                 "cdi": ["gpu.amd.com/gpu=0000:15:00.0"]},
                {"driver": "example.com", "pool": "p", "device": "nic-0", "cdi": ["example.com/nic=0000:05:00.0"]}]}]}]},
]


def test_dra_wire_roundtrip_and_allocation():
    buf = PR.encode_list_response(DRA_PODS)
    got = PR.decode_list_response(buf)
    assert got[0]["containers"][0]["dynamic"] == DRA_PODS[0]["containers"][0]["dynamic"]
    assert PR._pci_address("gpu.amd.com/gpu=0000:15:00.0") == "0000:15:00.0"
    assert PR._pci_address("card-15:00.0") == "15:00.0"
    assert PR._pci_address("gpu-0") is None and PR._pci_address("00000:15:00.0x") is None


def test_agent_skips_a_gpu_allocated_only_through_dra(monkeypatch):
    """a GPU handed to a pod by a DRA driver (no amd.com/gpu extended resource) is not
    diagnosed; the other GPU is."""
    ran = []
    two = fixtures.mi355x_probe_report("n", gpus=2)
    two["gpus"][0]["bdf"], two["gpus"][1]["bdf"] = "0000:05:00.0", "0000:15:00.0"
    monkeypatch.setattr(amdsmi_probe, "probe", lambda node, src, fx: two)
    monkeypatch.setattr(diag, "device_count", lambda: 2)
    monkeypatch.setattr(diag, "device_info", lambda d: {"bdf": ["0000:05:00.0", "0000:15:00.0"][d]})
    monkeypatch.setattr(diag, "run", lambda level, d, **kw: (ran.append(d), {"gemm": {"pass": True}})[1])
    with FakeKubelet(DRA_PODS) as kub:
        got = PR.allocated_devices(kub.sock)
        assert got == {"0000:15:00.0": "ml/dra-trainer (claim ml/gpu-claim)"}
        ag = A.Agent("n", source="fake", diag_level=1, pod_resources_socket=kub.sock)
        rep = ag.probe_once()
    assert ran == [0]
    assert rep["gpus"][1]["diag_skipped"] == "allocated to pod ml/dra-trainer (claim ml/gpu-claim)"


def test_dra_device_without_a_pci_address_makes_the_agent_fail_safe(monkeypatch):
    pods = [{"name": "p", "namespace": "ml", "containers": [{"name": "c", "devices": [], "dynamic": [
        {"claim_name": "c1", "claim_namespace": "ml", "devices": [
            {"driver": "gpu.amd.com", "pool": "node-a", "device": "gpu-3", "cdi": ["gpu.amd.com/gpu=gpu-3"]}]}]}]}]
    ran = []
    monkeypatch.setattr(amdsmi_probe, "probe", lambda node, src, fx: fixtures.mi355x_probe_report("n", gpus=2))
    monkeypatch.setattr(diag, "device_count", lambda: 2)
    monkeypatch.setattr(diag, "device_info", lambda d: {"bdf": ["0000:05:00.0", "0000:15:00.0"][d]})
    monkeypatch.setattr(diag, "run", lambda level, d, **kw: (ran.append(d), {"gemm": {"pass": True}})[1])
    with FakeKubelet(pods) as kub:
        assert PR.allocated_devices(kub.sock) == {"gpu.amd.com/node-a/gpu-3": "ml/p (claim ml/c1)"}
        rep = A.Agent("n", source="fake", diag_level=1, pod_resources_socket=kub.sock).probe_once()
    assert ran == []
    assert all("matching no local PCI address" in g["diag_skipped"] for g in rep["gpus"])


def test_one_mappable_and_one_unmappable_allocation_still_fail_safe(monkeypatch):
    """a device-plugin allocation that maps to a local PCI address next to a DRA claim keyed by
    driver/pool/device: the claim may be any GPU, so no GPU is diagnosed (it used to diagnose all but the mapped
    one, possibly under a running pod)."""
    pods = [{"name": "a", "namespace": "ml", "containers": [{"name": "c", "devices": [
                {"resource_name": "amd.com/gpu", "device_ids": ["0000:05:00.0"]}], "dynamic": []}]},
            {"name": "p", "namespace": "ml", "containers": [{"name": "c", "devices": [], "dynamic": [
                {"claim_name": "c1", "claim_namespace": "ml", "devices": [
                    {"driver": "gpu.amd.com", "pool": "node-a", "device": "gpu-3", "cdi": ["gpu.amd.com/gpu=gpu-3"]}]}]}]}]
    ran = []
    monkeypatch.setattr(amdsmi_probe, "probe", lambda node, src, fx: fixtures.mi355x_probe_report("n", gpus=2))
    monkeypatch.setattr(diag, "device_count", lambda: 2)
    monkeypatch.setattr(diag, "device_info", lambda d: {"bdf": ["0000:05:00.0", "0000:15:00.0"][d]})
    monkeypatch.setattr(diag, "run", lambda level, d, **kw: (ran.append(d), {"gemm": {"pass": True}})[1])
    with FakeKubelet(pods) as kub:
        got = PR.allocated_devices(kub.sock)
        assert got == {"0000:05:00.0": "ml/a", "gpu.amd.com/node-a/gpu-3": "ml/p (claim ml/c1)"}
        rep = A.Agent("n", source="fake", diag_level=1, pod_resources_socket=kub.sock).probe_once()
    assert ran == []
    assert all("gpu.amd.com/node-a/gpu-3" in g["diag_skipped"] and "matching no local PCI address" in g["diag_skipped"]
               for g in rep["gpus"])
