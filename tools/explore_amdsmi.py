"""One-off exploration: dump what amd-smi reports on the GPU box (non-root)."""
import json, time, os
t0 = time.perf_counter()
import amdsmi as A
t1 = time.perf_counter()
out = {"import_ms": (t1 - t0) * 1e3}
def call(name, fn, *a):
    s = time.perf_counter()
    try:
        r = fn(*a)
        out.setdefault("calls", {})[name] = {"ms": (time.perf_counter() - s) * 1e3, "value": r}
    except Exception as e:
        out.setdefault("calls", {})[name] = {"ms": (time.perf_counter() - s) * 1e3, "error": repr(e)}
s = time.perf_counter()
A.amdsmi_init()
out["init_ms"] = (time.perf_counter() - s) * 1e3
hs = A.amdsmi_get_processor_handles()
out["n_handles"] = len(hs)
for i, h in enumerate(hs[:2]):
    for nm in ["amdsmi_get_gpu_asic_info", "amdsmi_get_gpu_vram_info", "amdsmi_get_gpu_total_ecc_count",
               "amdsmi_get_gpu_xgmi_link_status", "amdsmi_get_gpu_kfd_info", "amdsmi_get_gpu_device_bdf",
               "amdsmi_get_gpu_device_uuid", "amdsmi_get_gpu_board_info", "amdsmi_get_gpu_driver_info",
               "amdsmi_get_gpu_compute_partition", "amdsmi_get_gpu_memory_partition", "amdsmi_get_gpu_enumeration_info",
               "amdsmi_get_gpu_bad_page_info", "amdsmi_get_gpu_vbios_info", "amdsmi_get_power_info",
               "amdsmi_get_gpu_activity", "amdsmi_get_link_metrics", "amdsmi_get_gpu_ras_block_features_enabled",
               "amdsmi_get_gpu_ecc_enabled", "amdsmi_get_gpu_metrics_info", "amdsmi_get_violation_status"]:
        call(f"{i}:{nm}", getattr(A, nm), h)
    call(f"{i}:mem_total_vram", A.amdsmi_get_gpu_memory_total, h, A.AmdSmiMemoryType.VRAM)
    call(f"{i}:temp_hotspot", A.amdsmi_get_temp_metric, h, A.AmdSmiTemperatureType.HOTSPOT, A.AmdSmiTemperatureMetric.CURRENT)
    # repeat timing for the hot probe calls
    for nm in ["amdsmi_get_gpu_total_ecc_count", "amdsmi_get_gpu_xgmi_link_status", "amdsmi_get_gpu_asic_info", "amdsmi_get_gpu_vram_info"]:
        s = time.perf_counter()
        for _ in range(20):
            try: getattr(A, nm)(h)
            except Exception: pass
        out.setdefault("repeat_ms", {})[f"{i}:{nm}"] = (time.perf_counter() - s) * 1e3 / 20
out["env"] = {k: os.environ.get(k) for k in ["HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_MAX_HW_QUEUES"]}
out["uid"] = os.getuid()
try:
    out["kfd_nodes"] = sorted(os.listdir("/sys/class/kfd/kfd/topology/nodes"))
except Exception as e:
    out["kfd_nodes"] = repr(e)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/amdsmi_explore.json", "w"), indent=1, default=str)
print(json.dumps({k: v for k, v in out.items() if k != "calls"}, default=str))
