"""Dump what the amd-smi Python binding reports about xGMI links, RAS and ECC on GPU 0 (exploration behind the native
probe's link fields, profiles/amdsmi_xgmi_link_metrics_mi355x.json)."""
import json, amdsmi as A
A.amdsmi_init()
h = A.amdsmi_get_processor_handles()[0]
out = {}
try:
    out["link_metrics"] = A.amdsmi_get_link_metrics(h)
except Exception as e:
    out["link_metrics"] = repr(e)
m = A.amdsmi_get_gpu_metrics_info(h)
out["metrics_xgmi"] = {k: v for k, v in m.items() if "xgmi" in k or "link" in k}
for fn in ("amdsmi_get_gpu_xgmi_link_status", "amdsmi_gpu_xgmi_error_status", "amdsmi_get_xgmi_info",
           "amdsmi_get_gpu_ras_feature_info", "amdsmi_get_gpu_bad_page_threshold", "amdsmi_get_gpu_ecc_enabled",
           "amdsmi_get_gpu_ecc_status", "amdsmi_get_gpu_total_ecc_count"):
    try:
        out[fn] = getattr(A, fn)(h)
    except Exception as e:
        out[fn] = repr(e)
try:
    out["topo"] = A.amdsmi_topo_get_link_type(h, h)
except Exception as e:
    out["topo"] = repr(e)
print(json.dumps(out, default=str, indent=1))
