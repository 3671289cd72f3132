// MI355X passive health probe over libamd_smi (C ABI, loaded by ctypes and by mi355x-probe).
//
// One report per call, schema "mi355x-health/v1" (see models/health.py):
//   {"schema","node","ts","probe":"native","amdsmi":"x.y.z","probe_ms",
//    "gpus":[{"index","bdf","uuid","gfx","market_name","vbios_name","device_id","cus",
//             "vram_type","vram_mb","ecc_correctable","ecc_uncorrectable","ecc_deferred",
//             "bad_pages","xgmi","kfd","kfd_node","compute_partition","memory_partition",
//             "hotspot_c"}...],
//    "error": null | "<amdsmi status name>"}
// amd-smi stays initialised between calls (the node agent probes on a cadence;
// the first query after init costs ~0.7 s on MI355X, later full probes 2-5 ms/GPU).
#pragma once

#ifdef __cplusplus
extern "C" {
#endif

// Initialise amd-smi (idempotent). Returns the amdsmi_status_t value (0 = success).
int mi355x_probe_open(void);
// Probe every GPU; returns a malloc'd NUL-terminated JSON document (free with mi355x_probe_free).
char* mi355x_probe_json(const char* node_name);
void mi355x_probe_free(char* doc);
// Shut amd-smi down (optional; safe to call when not open).
void mi355x_probe_close(void);
// Number of GPU processors seen by the last successful open (or -1).
int mi355x_probe_gpu_count(void);
// Re-enumerate (shut amd-smi down and initialise it again) when the session is this old at a probe, so a
// driver reload, GPU reset or repartition is seen; 0 = never.  Default 600 s or MI355X_PROBE_REOPEN_S.
// A probe in which a GPU stopped answering also re-enumerates at the next call.
void mi355x_probe_set_reopen_interval(double seconds);

#ifdef __cplusplus
}
#endif
