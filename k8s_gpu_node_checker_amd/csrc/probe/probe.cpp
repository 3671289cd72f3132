// MI355X passive health probe: libamd_smi -> "mi355x-health/v1" JSON (see probe.h).
//
// Checks what SURVEY §7.1 lists (ASIC/gfx950, HBM3E VRAM size, ECC, xGMI links,
// KFD node) plus bad pages, partition modes, hotspot temperature, the PCIe link,
// the driver and firmware versions, the RAS block behind any ECC count, the xGMI error
// status and operating telemetry (power, HBM temperature, clock, throttle residency).  Every
// amd-smi status other than success is recorded, never thrown: a node whose
// driver is not loaded (AMDSMI_STATUS_DRIVER_NOT_LOADED) or that denies access
// (AMDSMI_STATUS_NO_PERM) yields a report with "error" set, which the checker
// maps to verdict "unknown" (models/health.py), not to a crash.
#include "probe.h"

#include <algorithm>
#include <amd_smi/amdsmi.h>

#include <atomic>

#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace {

std::mutex g_mu;
bool g_open = false;
std::atomic<int> g_gpus{-1};  // read without the lock by mi355x_probe_gpu_count
std::vector<amdsmi_processor_handle> g_handles;
// per-handle firmware JSON object; firmware only changes across a driver reload, which also
// invalidates the handles, so it is read once per open (amdsmi_get_fw_info reads ~80 sysfs files)
std::vector<std::string> g_fw;
// per-handle RAS retirement state that is costly or static: the driver's bad-page threshold (a module
// parameter, fixed per load) and the RAS EEPROM checksum, validated again only when the retired-page
// count moved (the driver writes the EEPROM when it retires a page).  Both need root; -1 = not known.
struct RasCache {
  bool threshold_read = false;
  int64_t threshold = -1;
  int64_t eeprom = -1;  // 1 valid, 0 corrupted
  int64_t eeprom_pages = -1;
};
std::vector<RasCache> g_ras;
// The processor list is enumerated at amdsmi_init.  A driver reload, a GPU reset or a repartition (SPX ->
// CPX turns one GPU into eight processors) changes it under a long-lived session, so the session is
// re-opened every g_reopen_s seconds (MI355X_PROBE_REOPEN_S, default 600; 0 = never) and right after a
// probe in which a GPU stopped answering (its handle may be stale).
double g_reopen_s = -1.0;  // < 0: not read from the environment yet
bool g_reenumerate = false;
std::chrono::steady_clock::time_point g_opened_at;

void jstr(std::string& o, const char* s) {
  o.push_back('"');
  for (const unsigned char* p = reinterpret_cast<const unsigned char*>(s); *p; ++p) {
    unsigned char c = *p;
    if (c == '"' || c == '\\') {
      o.push_back('\\');
      o.push_back(static_cast<char>(c));
    } else if (c < 0x20) {
      char buf[8];
      snprintf(buf, sizeof buf, "\\u%04x", c);
      o += buf;
    } else {
      o.push_back(static_cast<char>(c));
    }
  }
  o.push_back('"');
}

void key(std::string& o, const char* k) {
  if (o.back() != '{') o.push_back(',');
  jstr(o, k);
  o.push_back(':');
}

void kv_str(std::string& o, const char* k, const char* v) {
  key(o, k);
  jstr(o, v);
}

void kv_u64(std::string& o, const char* k, uint64_t v) {
  key(o, k);
  o += std::to_string(v);
}

void kv_i64(std::string& o, const char* k, int64_t v) {
  key(o, k);
  o += std::to_string(v);
}

void kv_null(std::string& o, const char* k) {
  key(o, k);
  o += "null";
}

const char* status_name(amdsmi_status_t st) {
  const char* s = nullptr;
  if (amdsmi_status_code_to_string(st, &s) == AMDSMI_STATUS_SUCCESS && s) return s;
  return "AMDSMI_STATUS_UNKNOWN";
}

void close_locked() {
  if (!g_open) return;
  amdsmi_shut_down();
  g_open = false;
  g_handles.clear();
  g_fw.clear();
  g_ras.clear();
}

int open_locked() {
  if (g_open) return 0;
  amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) return static_cast<int>(st);
  uint32_t nsock = 0;
  st = amdsmi_get_socket_handles(&nsock, nullptr);
  if (st != AMDSMI_STATUS_SUCCESS) {
    amdsmi_shut_down();
    return static_cast<int>(st);
  }
  std::vector<amdsmi_socket_handle> socks(nsock);
  st = amdsmi_get_socket_handles(&nsock, socks.data());
  g_handles.clear();
  for (uint32_t s = 0; st == AMDSMI_STATUS_SUCCESS && s < nsock; ++s) {
    uint32_t n = 0;
    if (amdsmi_get_processor_handles(socks[s], &n, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> hs(n);
    if (amdsmi_get_processor_handles(socks[s], &n, hs.data()) != AMDSMI_STATUS_SUCCESS) continue;
    for (uint32_t i = 0; i < n; ++i) {
      processor_type_t t;
      if (amdsmi_get_processor_type(hs[i], &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
        g_handles.push_back(hs[i]);
    }
  }
  g_fw.assign(g_handles.size(), std::string());
  g_ras.assign(g_handles.size(), RasCache());
  g_open = true;
  g_reenumerate = false;
  g_opened_at = std::chrono::steady_clock::now();
  g_gpus.store(static_cast<int>(g_handles.size()), std::memory_order_relaxed);
  return 0;
}

// The firmware images that decide how a GPU behaves under load and under faults: power management
// (SMU / PM firmware), the security processor's OS, the compute queues (MEC), RLC, SDMA, and the RAS / xGMI
// trusted apps.  All GPUs of a node are flashed together, so a difference between them is a node
// that was half-updated (models/health.py compares them).
const char* fw_name(amdsmi_fw_block_t id) {
  switch (id) {
    case AMDSMI_FW_ID_SMU: return "smu";
    case AMDSMI_FW_ID_PM: return "pm";
    case AMDSMI_FW_ID_PSP_SOSDRV: return "psp_sos";
    case AMDSMI_FW_ID_CP_MEC1: return "mec";
    case AMDSMI_FW_ID_RLC: return "rlc";
    case AMDSMI_FW_ID_SDMA0: return "sdma";
    case AMDSMI_FW_ID_TA_RAS: return "ta_ras";
    case AMDSMI_FW_ID_TA_XGMI: return "ta_xgmi";
    case AMDSMI_FW_ID_PLDM_BUNDLE: return "pldm_bundle";
    default: return nullptr;
  }
}

const std::string& firmware_locked(size_t i) {
  std::string& s = g_fw[i];
  if (!s.empty()) return s;
  amdsmi_fw_info_t fw;
  memset(&fw, 0, sizeof fw);
  s = "{";
  if (amdsmi_get_fw_info(g_handles[i], &fw) == AMDSMI_STATUS_SUCCESS) {
    const size_t n = std::min<size_t>(fw.num_fw_info, AMDSMI_FW_ID__MAX);
    for (size_t k = 0; k < n; ++k) {
      const char* name = fw_name(fw.fw_info_list[k].fw_id);
      if (name && fw.fw_info_list[k].fw_version != 0 && fw.fw_info_list[k].fw_version != UINT64_MAX)
        kv_u64(s, name, fw.fw_info_list[k].fw_version);
    }
  }
  s.push_back('}');
  return s;
}

// Retired HBM pages: the total, and by status -- "pending" pages are marked bad and leave service at the
// next reset window, "unreservable" ones the driver could not take out of service (a bad page still in
// use).  Then the driver's retirement threshold (the GPU is declared bad once the count reaches it) and
// whether the RAS EEPROM that persists the list across reboots still checksums.
void probe_bad_pages(std::string& o, amdsmi_processor_handle h, RasCache& rc) {
  uint32_t n = 0;
  if (amdsmi_get_gpu_bad_page_info(h, &n, nullptr) == AMDSMI_STATUS_SUCCESS) {
    kv_u64(o, "bad_pages", n);
    if (n > 0) {
      std::vector<amdsmi_retired_page_record_t> rec(std::min<uint32_t>(n, 1u << 16));
      uint32_t got = static_cast<uint32_t>(rec.size());
      if (amdsmi_get_gpu_bad_page_info(h, &got, rec.data()) == AMDSMI_STATUS_SUCCESS) {
        uint64_t pending = 0, unreservable = 0;
        for (uint32_t i = 0; i < got && i < rec.size(); ++i) {
          pending += rec[i].status == AMDSMI_MEM_PAGE_STATUS_PENDING;
          unreservable += rec[i].status == AMDSMI_MEM_PAGE_STATUS_UNRESERVABLE;
        }
        kv_u64(o, "bad_pages_pending", pending);
        kv_u64(o, "bad_pages_unreservable", unreservable);
      }
    }
  }
  if (!rc.threshold_read) {
    rc.threshold_read = true;
    uint32_t t = 0;
    if (amdsmi_get_gpu_bad_page_threshold(h, &t) == AMDSMI_STATUS_SUCCESS) rc.threshold = t;
  }
  if (rc.threshold >= 0) kv_u64(o, "bad_page_threshold", static_cast<uint64_t>(rc.threshold));
  if (rc.eeprom_pages != static_cast<int64_t>(n)) {
    rc.eeprom_pages = n;
    const amdsmi_status_t st = amdsmi_gpu_validate_ras_eeprom(h);
    rc.eeprom = st == AMDSMI_STATUS_SUCCESS ? 1 : st == AMDSMI_STATUS_CORRUPTED_EEPROM ? 0 : -1;
  }
  if (rc.eeprom >= 0) kv_str(o, "ras_eeprom", rc.eeprom ? "ok" : "corrupted");
}

// RAS blocks, named as the kernel's ras sysfs does; asked only when the totals are non-zero, so a clean
// GPU costs no extra reads
const struct {
  amdsmi_gpu_block_t block;
  const char* name;
} kRasBlocks[] = {{AMDSMI_GPU_BLOCK_UMC, "umc"},     {AMDSMI_GPU_BLOCK_SDMA, "sdma"},
                  {AMDSMI_GPU_BLOCK_GFX, "gfx"},     {AMDSMI_GPU_BLOCK_MMHUB, "mmhub"},
                  {AMDSMI_GPU_BLOCK_ATHUB, "athub"}, {AMDSMI_GPU_BLOCK_PCIE_BIF, "pcie_bif"},
                  {AMDSMI_GPU_BLOCK_HDP, "hdp"},     {AMDSMI_GPU_BLOCK_XGMI_WAFL, "xgmi_wafl"},
                  {AMDSMI_GPU_BLOCK_DF, "df"},       {AMDSMI_GPU_BLOCK_SMN, "smn"},
                  {AMDSMI_GPU_BLOCK_SEM, "sem"},     {AMDSMI_GPU_BLOCK_MP0, "mp0"},
                  {AMDSMI_GPU_BLOCK_MP1, "mp1"},     {AMDSMI_GPU_BLOCK_FUSE, "fuse"},
                  {AMDSMI_GPU_BLOCK_MCA, "mca"},     {AMDSMI_GPU_BLOCK_VCN, "vcn"},
                  {AMDSMI_GPU_BLOCK_JPEG, "jpeg"},   {AMDSMI_GPU_BLOCK_IH, "ih"},
                  {AMDSMI_GPU_BLOCK_MPIO, "mpio"}};

// {"umc":{"ce":..,"ue":..,"de":..},...}: which hardware block the ECC errors come from (HBM behind the
// memory controller, the xGMI PHYs, the GFX engines...)
void ecc_blocks(std::string& o, amdsmi_processor_handle h) {
  std::string b = "{";
  for (const auto& rb : kRasBlocks) {
    amdsmi_error_count_t ec;
    memset(&ec, 0, sizeof ec);
    if (amdsmi_get_gpu_ecc_count(h, rb.block, &ec) != AMDSMI_STATUS_SUCCESS) continue;
    if (!ec.correctable_count && !ec.uncorrectable_count && !ec.deferred_count) continue;
    key(b, rb.name);
    b.push_back('{');
    kv_u64(b, "ce", ec.correctable_count);
    kv_u64(b, "ue", ec.uncorrectable_count);
    kv_u64(b, "de", ec.deferred_count);
    b.push_back('}');
  }
  b.push_back('}');
  if (b.size() > 2) {
    key(o, "ecc_blocks");
    o += b;
  }
}

// RAS error records (CPER) the driver keeps for this GPU, by severity, with the newest timestamp of each:
// {"fatal":n,"uncorrected":n,"corrected":n,"last_fatal":"2026-10-16T10:00:00Z",...}.  Reading them needs
// root (the DaemonSet is privileged); any other status is reported as "cper_error", not judged.
void probe_cper(std::string& o, amdsmi_processor_handle h) {
  static const char* kSev[3] = {"uncorrected", "fatal", "corrected"};  // amdsmi_cper_sev_t order
  std::vector<char> buf(1 << 20);
  std::vector<amdsmi_cper_hdr_t*> hdrs(64);
  uint64_t count[3] = {0, 0, 0}, last[3] = {0, 0, 0};  // last: YYYYMMDDhhmmss, comparable
  uint64_t cursor = 0;
  for (int call = 0; call < 256; ++call) {
    uint64_t size = buf.size(), n = hdrs.size();
    std::fill(hdrs.begin(), hdrs.end(), nullptr);
    const amdsmi_status_t st = amdsmi_get_gpu_cper_entries(h, 0x7, buf.data(), &size, hdrs.data(), &n, &cursor);
    if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_MORE_DATA) {
      if (call == 0) kv_str(o, "cper_error", status_name(st));
      if (call == 0) return;
      break;
    }
    const char* lo = buf.data();
    const char* hi = buf.data() + std::min<uint64_t>(size, buf.size());
    for (uint64_t i = 0; i < std::min<uint64_t>(n, hdrs.size()); ++i) {
      const char* p = reinterpret_cast<const char*>(hdrs[i]);
      if (p == nullptr || p < lo || p + sizeof(amdsmi_cper_hdr_t) > hi) continue;  // only headers inside buf
      amdsmi_cper_hdr_t hd;
      memcpy(&hd, p, sizeof hd);  // packed struct: copied out, never read through a misaligned pointer
      const unsigned sev = static_cast<unsigned>(hd.error_severity);
      if (sev > 2) continue;
      ++count[sev];
      const amdsmi_cper_timestamp_t& t = hd.timestamp;
      const uint64_t year = t.year < 100 ? 2000u + t.year : t.year;
      const uint64_t stamp = ((((year * 100 + t.month) * 100 + t.day) * 100 + t.hours) * 100 + t.minutes) * 100 + t.seconds;
      last[sev] = std::max(last[sev], stamp);
    }
    if (st != AMDSMI_STATUS_MORE_DATA) break;
  }
  key(o, "cper");
  o.push_back('{');
  for (int sv = 0; sv < 3; ++sv) kv_u64(o, kSev[sv], count[sv]);
  for (int sv = 0; sv < 3; ++sv) {
    if (!count[sv]) continue;
    const uint64_t v = last[sv];
    char ts[32];
    snprintf(ts, sizeof ts, "%04u-%02u-%02uT%02u:%02u:%02uZ", static_cast<unsigned>(v / 10000000000ull),
             static_cast<unsigned>(v / 100000000ull % 100), static_cast<unsigned>(v / 1000000ull % 100),
             static_cast<unsigned>(v / 10000ull % 100), static_cast<unsigned>(v / 100ull % 100),
             static_cast<unsigned>(v % 100));
    std::string k = std::string("last_") + kSev[sv];
    kv_str(o, k.c_str(), ts);
  }
  o.push_back('}');
}

// Operating state, not identity: power against its cap, HBM stack temperature, clock, VRAM in use,
// processes holding the device, and the firmware's throttle-residency accumulators.
// The accumulators count since driver load; the agent turns two consecutive probes into the share
// of the interval spent throttled (PVIOL / TVIOL in amd-smi terms).  A field the firmware does not
// report (all-ones sentinel) is left out.
void probe_telemetry(std::string& o, amdsmi_processor_handle h) {
  amdsmi_power_info_t pw;
  memset(&pw, 0, sizeof pw);
  if (amdsmi_get_power_info(h, &pw) == AMDSMI_STATUS_SUCCESS && pw.current_socket_power != UINT32_MAX &&
      pw.current_socket_power != UINT16_MAX)
    kv_u64(o, "power_w", pw.current_socket_power);
  // the cap in uW on bare-metal Linux (power_info's power_limit is documented in W but reads in uW too)
  amdsmi_power_cap_info_t cap;
  memset(&cap, 0, sizeof cap);
  if (amdsmi_get_power_cap_info(h, 0, &cap) == AMDSMI_STATUS_SUCCESS && cap.power_cap != UINT64_MAX &&
      cap.power_cap > 0) {
    kv_u64(o, "power_cap_w", cap.power_cap / 1000000);
    if (cap.default_power_cap != UINT64_MAX && cap.default_power_cap > 0)
      kv_u64(o, "power_cap_default_w", cap.default_power_cap / 1000000);
  }
  // HBM stacks: per-stack sensors, then the VRAM sensor; the hottest one counts
  int64_t hbm = -1;
  for (amdsmi_temperature_type_t t : {AMDSMI_TEMPERATURE_TYPE_HBM_0, AMDSMI_TEMPERATURE_TYPE_HBM_1,
                                      AMDSMI_TEMPERATURE_TYPE_HBM_2, AMDSMI_TEMPERATURE_TYPE_HBM_3,
                                      AMDSMI_TEMPERATURE_TYPE_VRAM}) {
    int64_t v = 0;
    if (amdsmi_get_temp_metric(h, t, AMDSMI_TEMP_CURRENT, &v) == AMDSMI_STATUS_SUCCESS && v > 0 && v < 200 &&
        v > hbm)
      hbm = v;
  }
  amdsmi_vram_usage_t vu;
  memset(&vu, 0, sizeof vu);
  if (amdsmi_get_gpu_vram_usage(h, &vu) == AMDSMI_STATUS_SUCCESS && vu.vram_used != UINT32_MAX)
    kv_u64(o, "vram_used_mb", vu.vram_used);
  // processes holding the device (PIDs of the host namespace, the VRAM each holds) and how busy the
  // graphics engine is: the agent runs its active diagnostics only on GPUs no workload holds
  uint32_t nproc = 0;
  if (amdsmi_get_gpu_process_list(h, &nproc, nullptr) == AMDSMI_STATUS_SUCCESS) {
    kv_u64(o, "processes", nproc);
    if (nproc > 0) {
      std::vector<amdsmi_proc_info_t> pl(std::min<uint32_t>(nproc, 64));
      uint32_t cap = static_cast<uint32_t>(pl.size());
      const amdsmi_status_t st = amdsmi_get_gpu_process_list(h, &cap, pl.data());
      if (st == AMDSMI_STATUS_SUCCESS || st == AMDSMI_STATUS_OUT_OF_RESOURCES) {
        key(o, "procs");
        o.push_back('[');
        const size_t n = std::min<size_t>(cap, pl.size());
        for (size_t i = 0; i < n; ++i) {
          if (i) o.push_back(',');
          o.push_back('{');
          kv_u64(o, "pid", pl[i].pid);
          kv_u64(o, "vram_mb", pl[i].memory_usage.vram_mem >> 20);
          o.push_back('}');
        }
        o.push_back(']');
      }
    }
  }
  amdsmi_engine_usage_t act;
  memset(&act, 0xFF, sizeof act);
  if (amdsmi_get_gpu_activity(h, &act) == AMDSMI_STATUS_SUCCESS && act.gfx_activity <= 100)
    kv_u64(o, "gfx_activity", act.gfx_activity);
  // all-ones first: whatever the library does not fill reads as the not-reported sentinel
  amdsmi_gpu_metrics_t m;
  memset(&m, 0xFF, sizeof m);
  const bool have_m = amdsmi_get_gpu_metrics_info(h, &m) == AMDSMI_STATUS_SUCCESS;
  for (int i = 0; have_m && i < AMDSMI_NUM_HBM_INSTANCES; ++i) {
    const uint16_t t = m.temperature_hbm[i];
    if (t != UINT16_MAX && t > 0 && t < 200 && static_cast<int64_t>(t) > hbm) hbm = t;
  }
  if (hbm > 0) kv_i64(o, "hbm_temp_c", hbm);
  if (!have_m) return;
  uint64_t clk_sum = 0, clk_n = 0;
  for (int i = 0; i < AMDSMI_MAX_NUM_GFX_CLKS; ++i) {
    const uint16_t c = m.current_gfxclks[i];
    if (c != UINT16_MAX && c > 0) {
      clk_sum += c;
      ++clk_n;
    }
  }
  if (clk_n) kv_u64(o, "gfxclk_mhz", clk_sum / clk_n);
  // the trained xGMI link: lanes and per-lane rate (MI355X: x16 at 38 Gb/s); a link that retrained
  // lower still reports Up
  if (m.xgmi_link_width != UINT16_MAX && m.xgmi_link_width > 0) kv_u64(o, "xgmi_width", m.xgmi_link_width);
  if (m.xgmi_link_speed != UINT16_MAX && m.xgmi_link_speed > 0) kv_u64(o, "xgmi_speed_gbps", m.xgmi_link_speed);
  if (m.accumulation_counter != UINT64_MAX && m.accumulation_counter != 0) {
    key(o, "throttle_acc");
    o.push_back('{');
    kv_u64(o, "n", m.accumulation_counter);
    const struct {
      const char* k;
      uint64_t v;
    } acc[] = {{"prochot", m.prochot_residency_acc},       {"ppt", m.ppt_residency_acc},
               {"socket_thm", m.socket_thm_residency_acc}, {"vr_thm", m.vr_thm_residency_acc},
               {"hbm_thm", m.hbm_thm_residency_acc}};
    for (const auto& a : acc)
      if (a.v != UINT64_MAX) kv_u64(o, a.k, a.v);
    o.push_back('}');
  }
}

bool probe_gpu(std::string& o, int index, amdsmi_processor_handle h) {
  auto t0 = std::chrono::steady_clock::now();
  o.push_back('{');
  kv_i64(o, "index", index);
  amdsmi_bdf_t bdf;
  if (amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) {
    char buf[32];
    snprintf(buf, sizeof buf, "%04" PRIx64 ":%02x:%02x.%x", static_cast<uint64_t>(bdf.domain_number),
             static_cast<unsigned>(bdf.bus_number), static_cast<unsigned>(bdf.device_number),
             static_cast<unsigned>(bdf.function_number));
    kv_str(o, "bdf", buf);
  }
  char uuid[AMDSMI_GPU_UUID_SIZE + 2] = {0};
  unsigned int ulen = sizeof uuid;
  if (amdsmi_get_gpu_device_uuid(h, &ulen, uuid) == AMDSMI_STATUS_SUCCESS) kv_str(o, "uuid", uuid);

  amdsmi_asic_info_t asic;
  memset(&asic, 0, sizeof asic);
  amdsmi_status_t st = amdsmi_get_gpu_asic_info(h, &asic);
  if (st != AMDSMI_STATUS_SUCCESS) {
    kv_str(o, "error", status_name(st));
    o.push_back('}');
    return false;
  }
  if (asic.target_graphics_version != UINT64_MAX) {
    char buf[32];
    snprintf(buf, sizeof buf, "gfx%" PRIx64, asic.target_graphics_version);
    kv_str(o, "gfx", buf);
  } else {
    kv_null(o, "gfx");
  }
  kv_str(o, "market_name", asic.market_name);
  {
    char buf[24];
    snprintf(buf, sizeof buf, "0x%04" PRIx64, asic.device_id);
    kv_str(o, "device_id", buf);
  }
  if (asic.num_of_compute_units != UINT32_MAX) kv_u64(o, "cus", asic.num_of_compute_units);
  amdsmi_board_info_t board;
  memset(&board, 0, sizeof board);
  // FRU product name does not depend on libdrm's amdgpu.ids (market_name does:
  // inside a process that loaded another libdrm it degrades to "AMD Radeon Graphics")
  if (amdsmi_get_gpu_board_info(h, &board) == AMDSMI_STATUS_SUCCESS) kv_str(o, "product_name", board.product_name);
  amdsmi_vbios_info_t vb;
  memset(&vb, 0, sizeof vb);
  if (amdsmi_get_gpu_vbios_info(h, &vb) == AMDSMI_STATUS_SUCCESS) {
    kv_str(o, "vbios_name", vb.name);
    if (vb.version[0]) kv_str(o, "vbios_version", vb.version);
  }
  const std::string& fw = firmware_locked(static_cast<size_t>(index));
  if (fw.size() > 2) {
    key(o, "fw");
    o += fw;
  }

  amdsmi_vram_info_t vram;
  memset(&vram, 0, sizeof vram);
  if (amdsmi_get_gpu_vram_info(h, &vram) == AMDSMI_STATUS_SUCCESS) {
    kv_i64(o, "vram_type", static_cast<int64_t>(vram.vram_type));
    kv_u64(o, "vram_mb", vram.vram_size);
  }
  amdsmi_error_count_t ec;
  memset(&ec, 0, sizeof ec);
  if (amdsmi_get_gpu_total_ecc_count(h, &ec) == AMDSMI_STATUS_SUCCESS) {
    kv_u64(o, "ecc_correctable", ec.correctable_count);
    kv_u64(o, "ecc_uncorrectable", ec.uncorrectable_count);
    kv_u64(o, "ecc_deferred", ec.deferred_count);
    if (ec.correctable_count || ec.uncorrectable_count || ec.deferred_count) ecc_blocks(o, h);
  } else {
    kv_null(o, "ecc_uncorrectable");
  }
  probe_bad_pages(o, h, g_ras[static_cast<size_t>(index)]);
  probe_cper(o, h);

  amdsmi_xgmi_link_status_t xs;
  memset(&xs, 0, sizeof xs);
  if (amdsmi_get_gpu_xgmi_link_status(h, &xs) == AMDSMI_STATUS_SUCCESS) {
    std::string links;
    for (uint32_t i = 0; i < xs.total_links && i < AMDSMI_MAX_NUM_XGMI_LINKS; ++i) {
      switch (xs.status[i]) {
        case AMDSMI_XGMI_LINK_UP: links.push_back('U'); break;
        case AMDSMI_XGMI_LINK_DOWN: links.push_back('D'); break;
        case AMDSMI_XGMI_LINK_DISABLE: links.push_back('X'); break;
        default: links.push_back('N');
      }
    }
    kv_str(o, "xgmi", links.c_str());
  } else {
    kv_null(o, "xgmi");
  }
  // the fabric this GPU is wired into: its hive (every GPU of an 8-GPU board shares one) and, per xGMI
  // link, the PCI address of the GPU at the other end and the traffic it has carried (KB since load)
  amdsmi_xgmi_info_t xi;
  memset(&xi, 0, sizeof xi);
  if (amdsmi_get_xgmi_info(h, &xi) == AMDSMI_STATUS_SUCCESS && xi.xgmi_hive_id != 0 && xi.xgmi_hive_id != UINT64_MAX) {
    char buf[24];
    snprintf(buf, sizeof buf, "%016" PRIx64, xi.xgmi_hive_id);
    kv_str(o, "xgmi_hive", buf);
  }
  amdsmi_link_metrics_t lm;
  memset(&lm, 0, sizeof lm);
  if (amdsmi_get_link_metrics(h, &lm) == AMDSMI_STATUS_SUCCESS) {
    std::string peers = "[", kb = "[";
    // num_links counts the connected links, but the table also holds the disabled port (all-ones BDF)
    // ahead of them (MI355X: num_links 7, entries 0..7), so every entry is scanned; the memset leaves
    // the unused ones as type INTERNAL
    for (uint32_t i = 0; i < AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK; ++i) {
      const auto& l = lm.links[i];
      if (l.link_type != AMDSMI_LINK_TYPE_XGMI || l.bdf.as_uint == UINT64_MAX) continue;  // a disabled port
      char buf[32];
      snprintf(buf, sizeof buf, "%04" PRIx64 ":%02x:%02x.%x", static_cast<uint64_t>(l.bdf.domain_number),
               static_cast<unsigned>(l.bdf.bus_number), static_cast<unsigned>(l.bdf.device_number),
               static_cast<unsigned>(l.bdf.function_number));
      if (peers.size() > 1) {
        peers.push_back(',');
        kb.push_back(',');
      }
      jstr(peers, buf);
      kb += "[" + std::to_string(l.read) + "," + std::to_string(l.write) + "]";
    }
    peers.push_back(']');
    kb.push_back(']');
    key(o, "xgmi_peers");
    o += peers;
    key(o, "xgmi_kb");
    o += kb;
  }
  // sticky until reset: the xGMI PHYs saw errors (one, or several) since the driver loaded
  amdsmi_xgmi_status_t xe = AMDSMI_XGMI_STATUS_NO_ERRORS;
  if (amdsmi_gpu_xgmi_error_status(h, &xe) == AMDSMI_STATUS_SUCCESS) kv_u64(o, "xgmi_error", static_cast<uint64_t>(xe));
  amdsmi_kfd_info_t kfd;
  memset(&kfd, 0, sizeof kfd);
  bool kfd_ok = amdsmi_get_gpu_kfd_info(h, &kfd) == AMDSMI_STATUS_SUCCESS && kfd.kfd_id != UINT64_MAX &&
                kfd.node_id != UINT32_MAX;
  key(o, "kfd");
  o += kfd_ok ? "true" : "false";
  if (kfd_ok) kv_u64(o, "kfd_node", kfd.node_id);
  char part[64] = {0};
  if (amdsmi_get_gpu_compute_partition(h, part, sizeof part) == AMDSMI_STATUS_SUCCESS) kv_str(o, "compute_partition", part);
  memset(part, 0, sizeof part);
  if (amdsmi_get_gpu_memory_partition(h, part, sizeof part) == AMDSMI_STATUS_SUCCESS) kv_str(o, "memory_partition", part);
  int64_t temp = 0;
  if (amdsmi_get_temp_metric(h, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &temp) == AMDSMI_STATUS_SUCCESS)
    kv_i64(o, "hotspot_c", temp);
  // PCIe host link: a slot trained down (x8, Gen4) halves host<->GPU bandwidth without any error;
  // the current speed may drop at idle (link power management), the width does not.
  amdsmi_pcie_info_t pcie;
  memset(&pcie, 0, sizeof pcie);
  if (amdsmi_get_pcie_info(h, &pcie) == AMDSMI_STATUS_SUCCESS) {
    kv_u64(o, "pcie_width", pcie.pcie_metric.pcie_width);
    kv_u64(o, "pcie_max_width", pcie.pcie_static.max_pcie_width);
    kv_u64(o, "pcie_speed_mts", pcie.pcie_metric.pcie_speed);
    kv_u64(o, "pcie_max_speed_mts", pcie.pcie_static.max_pcie_speed);  // header says GT/s; MI355X reports 32000
    if (pcie.pcie_metric.pcie_replay_count != UINT64_MAX) kv_u64(o, "pcie_replays", pcie.pcie_metric.pcie_replay_count);
    if (pcie.pcie_metric.pcie_l0_to_recovery_count != UINT64_MAX)
      kv_u64(o, "pcie_recoveries", pcie.pcie_metric.pcie_l0_to_recovery_count);
  }
  probe_telemetry(o, h);
  double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  key(o, "probe_us");
  o += std::to_string(static_cast<int64_t>(us));
  o.push_back('}');
  return true;
}

char* dup(const std::string& s) {
  char* p = static_cast<char*>(malloc(s.size() + 1));
  if (p) memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

}  // namespace

extern "C" int mi355x_probe_open(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return open_locked();
}

extern "C" int mi355x_probe_gpu_count(void) { return g_gpus.load(std::memory_order_relaxed); }

extern "C" char* mi355x_probe_json(const char* node_name) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto t0 = std::chrono::steady_clock::now();
  double now = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
  std::string o = "{";
  kv_str(o, "schema", "mi355x-health/v1");
  kv_str(o, "node", node_name ? node_name : "");
  {
    char buf[40];
    snprintf(buf, sizeof buf, "%.3f", now);
    key(o, "ts");
    o += buf;
  }
  kv_str(o, "probe", "native");
  amdsmi_version_t ver;
  if (amdsmi_get_lib_version(&ver) == AMDSMI_STATUS_SUCCESS) {
    char buf[64];
    snprintf(buf, sizeof buf, "%u.%u.%u", ver.major, ver.minor, ver.release);
    kv_str(o, "amdsmi", buf);
  }
  if (g_reopen_s < 0) {
    const char* e = getenv("MI355X_PROBE_REOPEN_S");
    g_reopen_s = e && *e ? std::max(0.0, atof(e)) : 600.0;
  }
  if (g_open && (g_reenumerate ||
                 (g_reopen_s > 0 &&
                  std::chrono::duration<double>(std::chrono::steady_clock::now() - g_opened_at).count() >= g_reopen_s)))
    close_locked();  // enumerate again: the processor list may have changed under the session
  const bool fresh = !g_open;
  int st = open_locked();
  if (st != 0) {
    kv_str(o, "error", status_name(static_cast<amdsmi_status_t>(st)));
    key(o, "gpus");
    o += "[]}";
    return dup(o);
  }
  if (!g_handles.empty()) {
    amdsmi_driver_info_t drv;
    memset(&drv, 0, sizeof drv);
    if (amdsmi_get_gpu_driver_info(g_handles[0], &drv) == AMDSMI_STATUS_SUCCESS && drv.driver_version[0]) {
      drv.driver_name[sizeof drv.driver_name - 1] = '\0';
      drv.driver_version[sizeof drv.driver_version - 1] = '\0';
      key(o, "driver");
      o.push_back('{');
      kv_str(o, "name", drv.driver_name);
      kv_str(o, "version", drv.driver_version);
      o.push_back('}');
    }
  }
  key(o, "gpus");
  o.push_back('[');
  for (size_t i = 0; i < g_handles.size(); ++i) {
    if (i) o.push_back(',');
    // a GPU that stops answering in an older session: enumerate again at the next probe (once: if it
    // still fails in the fresh session, only the periodic re-open retries it)
    if (!probe_gpu(o, static_cast<int>(i), g_handles[i]) && !fresh) g_reenumerate = true;
  }
  o.push_back(']');
  double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  char buf[40];
  snprintf(buf, sizeof buf, "%.3f", ms);
  key(o, "probe_ms");
  o += buf;
  o.push_back('}');
  return dup(o);
}

extern "C" void mi355x_probe_free(char* doc) { free(doc); }

extern "C" void mi355x_probe_close(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  close_locked();
}

extern "C" void mi355x_probe_set_reopen_interval(double seconds) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_reopen_s = seconds < 0 ? 0.0 : seconds;
}
