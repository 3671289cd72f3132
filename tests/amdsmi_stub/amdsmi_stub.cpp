// Replay stub of libamd_smi for host-side sanitizer builds of csrc/probe/probe.cpp (tests/test_sanitizers.py).
//
// Compiled against the real <amd_smi/amdsmi.h>, so every signature the probe links against is checked
// by the compiler.  The values come from a flat "key=value" scenario file named by AMDSMI_STUB_SCENARIO
// (the test writes it from a recorded MI355X probe, profiles/probe_cli_mi355x.jsonl):
//
//   init_status=0|10|34              amdsmi_init result (NO_PERM, DRIVER_NOT_LOADED, ...)
//   sockets_status=0                 amdsmi_get_socket_handles result
//   gpus=N                           GPU processors (one socket each)
//   gpu.<i>.<field>=<value>          one recorded field of GPU i (names as in the probe's JSON)
//   gpu.<i>.asic_status=<status>     make amdsmi_get_gpu_asic_info fail for GPU i
//   gpu.<i>.nprocs=<n>               synthesise n processes (exercises the probe's 64-entry cap)
//   gpu.<i>.fw.<name>=<version>      firmware versions; gpu.<i>.ecc_blocks.<block>.ce|ue|de per-block ECC
//   driver_version=<v>               amdsmi_get_gpu_driver_info (absent: NOT_SUPPORTED)
//   gpu.<i>.xgmi_hive=<hex>, gpu.<i>.xgmi_peers=<bdf>,...   amdsmi_get_xgmi_info / amdsmi_get_link_metrics
//
// Output buffers are written exactly as the real library documents (length-checked), so a probe that
// passes a short buffer or reads past what was written shows up under ASan.
#include <amd_smi/amdsmi.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace {

struct Gpu {
  std::map<std::string, std::string> f;
  bool has(const char* k) const { return f.count(k) != 0; }
  std::string s(const char* k, const char* d = "") const {
    auto it = f.find(k);
    return it == f.end() ? d : it->second;
  }
  uint64_t u(const char* k, uint64_t d = 0) const {
    auto it = f.find(k);
    return it == f.end() ? d : strtoull(it->second.c_str(), nullptr, 0);
  }
};

struct World {
  bool loaded = false;
  int init_status = 0;
  int sockets_status = 0;
  std::string driver_version;
  bool open = false;
  std::vector<Gpu> gpus;
};

World g_world;

void load() {
  if (g_world.loaded) return;
  g_world.loaded = true;
  const char* path = getenv("AMDSMI_STUB_SCENARIO");
  if (!path) return;
  FILE* fp = fopen(path, "r");
  if (!fp) return;
  char line[4096];
  while (fgets(line, sizeof line, fp)) {
    std::string l(line);
    while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
    const size_t eq = l.find('=');
    if (eq == std::string::npos) continue;
    const std::string k = l.substr(0, eq), v = l.substr(eq + 1);
    if (k == "init_status") {
      g_world.init_status = atoi(v.c_str());
    } else if (k == "sockets_status") {
      g_world.sockets_status = atoi(v.c_str());
    } else if (k == "driver_version") {
      g_world.driver_version = v;
    } else if (k == "gpus") {
      g_world.gpus.resize(static_cast<size_t>(atoi(v.c_str())));
    } else if (k.rfind("gpu.", 0) == 0) {
      const size_t dot = k.find('.', 4);
      if (dot == std::string::npos) continue;
      const size_t i = static_cast<size_t>(atoi(k.substr(4, dot - 4).c_str()));
      if (i < g_world.gpus.size()) g_world.gpus[i].f[k.substr(dot + 1)] = v;
    }
  }
  fclose(fp);
}

const Gpu* gpu_of(amdsmi_processor_handle h) {
  for (const Gpu& g : g_world.gpus)
    if (static_cast<const void*>(&g) == h) return &g;
  return nullptr;
}

// copy a string into a caller buffer of `len` bytes, NUL-terminated and truncated like strncpy + term
void put(char* dst, size_t len, const std::string& v) {
  if (!len) return;
  const size_t n = v.size() < len - 1 ? v.size() : len - 1;
  memcpy(dst, v.data(), n);
  dst[n] = '\0';
}

#define GPU_OR_FAIL(h)                                   \
  const Gpu* g = gpu_of(h);                              \
  if (!g_world.open) return AMDSMI_STATUS_NOT_INIT;      \
  if (!g) return AMDSMI_STATUS_INVAL

#define FIELD_OR_NA(k) \
  if (!g->has(k)) return AMDSMI_STATUS_NOT_SUPPORTED

}  // namespace

extern "C" {

amdsmi_status_t amdsmi_init(uint64_t) {
  if (const char* log = getenv("AMDSMI_STUB_INIT_LOG")) {
    if (FILE* fp = fopen(log, "a")) {
      fputs("init\n", fp);
      fclose(fp);
    }
  }
  load();
  if (g_world.init_status) return static_cast<amdsmi_status_t>(g_world.init_status);
  g_world.open = true;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_shut_down(void) {
  // the next init reads the scenario again (a changed file = a driver reload / repartition); handles of
  // this session become invalid, as with the real library
  g_world = World();
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_status_code_to_string(amdsmi_status_t status, const char** status_string) {
  switch (status) {
    case AMDSMI_STATUS_SUCCESS: *status_string = "AMDSMI_STATUS_SUCCESS"; break;
    case AMDSMI_STATUS_NO_PERM: *status_string = "AMDSMI_STATUS_NO_PERM"; break;
    case AMDSMI_STATUS_DRIVER_NOT_LOADED: *status_string = "AMDSMI_STATUS_DRIVER_NOT_LOADED"; break;
    case AMDSMI_STATUS_NOT_SUPPORTED: *status_string = "AMDSMI_STATUS_NOT_SUPPORTED"; break;
    default: *status_string = "AMDSMI_STATUS_UNKNOWN_ERROR";
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_lib_version(amdsmi_version_t* version) {
  version->major = 26;
  version->minor = 2;
  version->release = 1;
  version->build = "26.2.1-stub";
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_socket_handles(uint32_t* socket_count, amdsmi_socket_handle* socket_handles) {
  if (!g_world.open) return AMDSMI_STATUS_NOT_INIT;
  if (g_world.sockets_status) return static_cast<amdsmi_status_t>(g_world.sockets_status);
  const uint32_t n = static_cast<uint32_t>(g_world.gpus.size());
  if (socket_handles) {
    const uint32_t cap = *socket_count < n ? *socket_count : n;
    for (uint32_t i = 0; i < cap; ++i) socket_handles[i] = &g_world.gpus[i].f;  // any distinct non-null
    *socket_count = cap;
  } else {
    *socket_count = n;
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle socket_handle, uint32_t* processor_count,
                                             amdsmi_processor_handle* processor_handles) {
  for (Gpu& g : g_world.gpus) {
    if (static_cast<void*>(&g.f) != socket_handle) continue;
    if (processor_handles && *processor_count >= 1) processor_handles[0] = &g;
    *processor_count = 1;
    return AMDSMI_STATUS_SUCCESS;
  }
  return AMDSMI_STATUS_INVAL;
}

amdsmi_status_t amdsmi_get_processor_type(amdsmi_processor_handle processor_handle, processor_type_t* processor_type) {
  GPU_OR_FAIL(processor_handle);
  (void)g;
  *processor_type = AMDSMI_PROCESSOR_TYPE_AMD_GPU;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_bdf(amdsmi_processor_handle processor_handle, amdsmi_bdf_t* bdf) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("bdf");
  unsigned dom = 0, bus = 0, dev = 0, fn = 0;
  if (sscanf(g->s("bdf").c_str(), "%x:%x:%x.%x", &dom, &bus, &dev, &fn) != 4) return AMDSMI_STATUS_INVAL;
  bdf->as_uint = 0;
  bdf->domain_number = dom;
  bdf->bus_number = bus;
  bdf->device_number = dev;
  bdf->function_number = fn;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_uuid(amdsmi_processor_handle processor_handle, unsigned int* uuid_length,
                                           char* uuid) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("uuid");
  if (*uuid_length < AMDSMI_GPU_UUID_SIZE) return AMDSMI_STATUS_INSUFFICIENT_SIZE;
  put(uuid, *uuid_length, g->s("uuid"));
  *uuid_length = static_cast<unsigned>(g->s("uuid").size());
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_asic_info(amdsmi_processor_handle processor_handle, amdsmi_asic_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  if (g->has("asic_status")) return static_cast<amdsmi_status_t>(g->u("asic_status"));
  memset(info, 0, sizeof *info);
  put(info->market_name, sizeof info->market_name, g->s("market_name"));
  info->device_id = g->u("device_id", 0);
  const std::string gfx = g->s("gfx");  // "gfx950" -> 0x950
  info->target_graphics_version = gfx.rfind("gfx", 0) == 0 ? strtoull(gfx.c_str() + 3, nullptr, 16) : UINT64_MAX;
  info->num_of_compute_units = g->has("cus") ? static_cast<uint32_t>(g->u("cus")) : UINT32_MAX;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_board_info(amdsmi_processor_handle processor_handle, amdsmi_board_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("product_name");
  memset(info, 0, sizeof *info);
  put(info->product_name, sizeof info->product_name, g->s("product_name"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_vbios_info(amdsmi_processor_handle processor_handle, amdsmi_vbios_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("vbios_name");
  memset(info, 0, sizeof *info);
  put(info->name, sizeof info->name, g->s("vbios_name"));
  put(info->version, sizeof info->version, g->s("vbios_version"));
  return AMDSMI_STATUS_SUCCESS;
}

// gpu.<i>.fw.<name>=<version>, names as the probe emits them
amdsmi_status_t amdsmi_get_fw_info(amdsmi_processor_handle processor_handle, amdsmi_fw_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  static const struct {
    amdsmi_fw_block_t id;
    const char* key;
  } ids[] = {{AMDSMI_FW_ID_SMU, "fw.smu"},       {AMDSMI_FW_ID_CP_ME, "fw.me"}, {AMDSMI_FW_ID_PM, "fw.pm"},
             {AMDSMI_FW_ID_PSP_SOSDRV, "fw.psp_sos"}, {AMDSMI_FW_ID_CP_MEC1, "fw.mec"},
             {AMDSMI_FW_ID_RLC, "fw.rlc"},       {AMDSMI_FW_ID_SDMA0, "fw.sdma"},
             {AMDSMI_FW_ID_TA_RAS, "fw.ta_ras"}, {AMDSMI_FW_ID_TA_XGMI, "fw.ta_xgmi"},
             {AMDSMI_FW_ID_PLDM_BUNDLE, "fw.pldm_bundle"}};
  memset(info, 0, sizeof *info);
  uint8_t n = 0;
  for (const auto& e : ids) {
    if (!g->has(e.key) && e.id != AMDSMI_FW_ID_CP_ME) continue;
    info->fw_info_list[n].fw_id = e.id;
    info->fw_info_list[n].fw_version = g->u(e.key, 0x1234);  // CP_ME: a block the probe does not report
    ++n;
  }
  info->num_fw_info = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_xgmi_info(amdsmi_processor_handle processor_handle, amdsmi_xgmi_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("xgmi_hive");
  memset(info, 0, sizeof *info);
  info->xgmi_hive_id = strtoull(g->s("xgmi_hive").c_str(), nullptr, 16);
  info->xgmi_lanes = 0;  // what the MI355X box reports
  return AMDSMI_STATUS_SUCCESS;
}

// gpu.<i>.xgmi_peers=<bdf>,<bdf>,...: one XGMI link per peer, plus the disabled port (all-ones BDF) first,
// as the MI355X box reports them
amdsmi_status_t amdsmi_get_link_metrics(amdsmi_processor_handle processor_handle, amdsmi_link_metrics_t* lm) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("xgmi_peers");
  memset(lm, 0, sizeof *lm);
  uint32_t n = 0;
  lm->links[n].bdf.as_uint = UINT64_MAX;
  lm->links[n].link_type = AMDSMI_LINK_TYPE_XGMI;
  ++n;
  const std::string s = g->s("xgmi_peers");
  size_t pos = 0;
  while (pos < s.size() && n < AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK) {
    size_t end = s.find(',', pos);
    if (end == std::string::npos) end = s.size();
    unsigned dom = 0, bus = 0, dev = 0, fn = 0;
    if (sscanf(s.substr(pos, end - pos).c_str(), "%x:%x:%x.%x", &dom, &bus, &dev, &fn) == 4) {
      auto& l = lm->links[n++];
      l.bdf.domain_number = dom;
      l.bdf.bus_number = bus;
      l.bdf.device_number = dev;
      l.bdf.function_number = fn;
      l.bit_rate = static_cast<uint32_t>(g->u("xgmi_speed_gbps", 38));
      l.max_bandwidth = 16 * l.bit_rate;
      l.link_type = AMDSMI_LINK_TYPE_XGMI;
      l.read = 1000 * n;
      l.write = 2000 * n;
    }
    pos = end + 1;
  }
  lm->num_links = n - 1;  // as the real library: the disabled port is in the table but not counted
  return AMDSMI_STATUS_SUCCESS;
}

// gpu.<i>.cper_entries=<sev>@<YYYYMMDDhhmmss>,... : records laid out back to back in cper_data (header +
// 32 payload bytes each), paged by the caller's header-array length and buffer size with the cursor;
// gpu.<i>.cper_error=... : NO_PERM (what a non-root caller gets on the MI355X box)
amdsmi_status_t amdsmi_get_gpu_cper_entries(amdsmi_processor_handle processor_handle, uint32_t severity_mask,
                                            char* cper_data, uint64_t* buf_size, amdsmi_cper_hdr_t** cper_hdrs,
                                            uint64_t* entry_count, uint64_t* cursor) {
  GPU_OR_FAIL(processor_handle);
  if (g->has("cper_error")) return AMDSMI_STATUS_NO_PERM;
  FIELD_OR_NA("cper_entries");
  struct Rec {
    unsigned sev;
    uint64_t stamp;
  };
  std::vector<Rec> recs;
  const std::string s = g->s("cper_entries");
  size_t pos = 0;
  while (pos < s.size()) {
    size_t end = s.find(',', pos);
    if (end == std::string::npos) end = s.size();
    unsigned sev = 0;
    unsigned long long stamp = 0;
    if (sscanf(s.substr(pos, end - pos).c_str(), "%u@%llu", &sev, &stamp) == 2 && ((severity_mask >> sev) & 1u))
      recs.push_back({sev, stamp});
    pos = end + 1;
  }
  const size_t rec_len = sizeof(amdsmi_cper_hdr_t) + 32;
  uint64_t n = 0, used = 0, i = *cursor;
  for (; i < recs.size() && n < *entry_count && used + rec_len <= *buf_size; ++i, ++n) {
    amdsmi_cper_hdr_t h;
    memset(&h, 0, sizeof h);
    memcpy(h.signature, "CPER", 4);
    h.signature_end = 0xFFFFFFFFu;
    h.sec_cnt = 1;
    h.error_severity = static_cast<amdsmi_cper_sev_t>(recs[i].sev);
    h.record_length = static_cast<uint32_t>(rec_len);
    const uint64_t t = recs[i].stamp;
    h.timestamp.year = static_cast<uint8_t>(t / 10000000000ull % 100);  // two digits, as the driver fills it
    h.timestamp.month = static_cast<uint8_t>(t / 100000000ull % 100);
    h.timestamp.day = static_cast<uint8_t>(t / 1000000ull % 100);
    h.timestamp.hours = static_cast<uint8_t>(t / 10000ull % 100);
    h.timestamp.minutes = static_cast<uint8_t>(t / 100ull % 100);
    h.timestamp.seconds = static_cast<uint8_t>(t % 100);
    memcpy(cper_data + used, &h, sizeof h);
    memset(cper_data + used + sizeof h, 0xAB, 32);
    cper_hdrs[n] = reinterpret_cast<amdsmi_cper_hdr_t*>(cper_data + used);
    used += rec_len;
  }
  *entry_count = n;
  *buf_size = used;
  *cursor = i;
  return i < recs.size() ? AMDSMI_STATUS_MORE_DATA : AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_gpu_xgmi_error_status(amdsmi_processor_handle processor_handle, amdsmi_xgmi_status_t* status) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("xgmi_error");
  *status = static_cast<amdsmi_xgmi_status_t>(g->u("xgmi_error"));
  return AMDSMI_STATUS_SUCCESS;
}

// gpu.<i>.ecc_blocks.<block>.{ce,ue,de}; blocks without a line read as zero counts
amdsmi_status_t amdsmi_get_gpu_ecc_count(amdsmi_processor_handle processor_handle, amdsmi_gpu_block_t block,
                                         amdsmi_error_count_t* ec) {
  GPU_OR_FAIL(processor_handle);
  static const struct {
    amdsmi_gpu_block_t b;
    const char* name;
  } names[] = {{AMDSMI_GPU_BLOCK_UMC, "umc"}, {AMDSMI_GPU_BLOCK_GFX, "gfx"}, {AMDSMI_GPU_BLOCK_SDMA, "sdma"},
               {AMDSMI_GPU_BLOCK_MMHUB, "mmhub"}, {AMDSMI_GPU_BLOCK_XGMI_WAFL, "xgmi_wafl"},
               {AMDSMI_GPU_BLOCK_PCIE_BIF, "pcie_bif"}};
  if (!ec) return AMDSMI_STATUS_INVAL;
  memset(ec, 0, sizeof *ec);
  for (const auto& n : names) {
    if (n.b != block) continue;
    const std::string k = std::string("ecc_blocks.") + n.name + ".";
    ec->correctable_count = g->u((k + "ce").c_str());
    ec->uncorrectable_count = g->u((k + "ue").c_str());
    ec->deferred_count = g->u((k + "de").c_str());
    return AMDSMI_STATUS_SUCCESS;
  }
  return AMDSMI_STATUS_NOT_SUPPORTED;
}

amdsmi_status_t amdsmi_get_gpu_driver_info(amdsmi_processor_handle processor_handle, amdsmi_driver_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  (void)g;
  if (g_world.driver_version.empty()) return AMDSMI_STATUS_NOT_SUPPORTED;
  memset(info, 0, sizeof *info);
  put(info->driver_name, sizeof info->driver_name, "amdgpu");
  put(info->driver_version, sizeof info->driver_version, g_world.driver_version);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_vram_info(amdsmi_processor_handle processor_handle, amdsmi_vram_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("vram_mb");
  memset(info, 0, sizeof *info);
  info->vram_type = static_cast<amdsmi_vram_type_t>(g->u("vram_type"));
  info->vram_size = g->u("vram_mb");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_total_ecc_count(amdsmi_processor_handle processor_handle, amdsmi_error_count_t* ec) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("ecc_uncorrectable");
  memset(ec, 0, sizeof *ec);
  ec->correctable_count = g->u("ecc_correctable");
  ec->uncorrectable_count = g->u("ecc_uncorrectable");
  ec->deferred_count = g->u("ecc_deferred");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_bad_page_info(amdsmi_processor_handle processor_handle, uint32_t* num_pages,
                                             amdsmi_retired_page_record_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("bad_pages");
  const uint32_t n = static_cast<uint32_t>(g->u("bad_pages"));
  if (info) {
    const uint32_t cap = *num_pages < n ? *num_pages : n;
    for (uint32_t i = 0; i < cap; ++i) {
      memset(&info[i], 0, sizeof info[i]);
      info[i].page_address = 0x1000ull * (i + 1);
      info[i].page_size = 4096;
      // bad_page_status: one letter per record, r(eserved) p(ending) u(nreservable); reserved by default
      const std::string st = g->s("bad_page_status");
      const char c = i < st.size() ? st[i] : 'r';
      info[i].status = c == 'p' ? AMDSMI_MEM_PAGE_STATUS_PENDING
                     : c == 'u' ? AMDSMI_MEM_PAGE_STATUS_UNRESERVABLE : AMDSMI_MEM_PAGE_STATUS_RESERVED;
    }
    *num_pages = cap;
  } else {
    *num_pages = n;
  }
  return AMDSMI_STATUS_SUCCESS;
}

// bad_page_threshold=N, or bad_page_threshold=noperm (non-root, as on a real box)
amdsmi_status_t amdsmi_get_gpu_bad_page_threshold(amdsmi_processor_handle processor_handle, uint32_t* threshold) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("bad_page_threshold");
  if (g->s("bad_page_threshold") == "noperm") return AMDSMI_STATUS_NO_PERM;
  *threshold = static_cast<uint32_t>(g->u("bad_page_threshold"));
  return AMDSMI_STATUS_SUCCESS;
}

// ras_eeprom=ok|corrupted|noperm; validations counted in the scenario-visible call log
amdsmi_status_t amdsmi_gpu_validate_ras_eeprom(amdsmi_processor_handle processor_handle) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("ras_eeprom");
  const std::string v = g->s("ras_eeprom");
  if (const char* log = getenv("AMDSMI_STUB_EEPROM_LOG")) {
    if (FILE* fp = fopen(log, "a")) {
      fputs("validate\n", fp);
      fclose(fp);
    }
  }
  return v == "ok" ? AMDSMI_STATUS_SUCCESS : v == "corrupted" ? AMDSMI_STATUS_CORRUPTED_EEPROM : AMDSMI_STATUS_NO_PERM;
}

amdsmi_status_t amdsmi_get_gpu_xgmi_link_status(amdsmi_processor_handle processor_handle,
                                                amdsmi_xgmi_link_status_t* link_status) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("xgmi");
  memset(link_status, 0, sizeof *link_status);
  const std::string s = g->s("xgmi");
  const uint32_t n = s.size() < AMDSMI_MAX_NUM_XGMI_LINKS ? static_cast<uint32_t>(s.size()) : AMDSMI_MAX_NUM_XGMI_LINKS;
  link_status->total_links = n;
  for (uint32_t i = 0; i < n; ++i)
    link_status->status[i] = s[i] == 'U' ? AMDSMI_XGMI_LINK_UP
                             : s[i] == 'D' ? AMDSMI_XGMI_LINK_DOWN
                                           : AMDSMI_XGMI_LINK_DISABLE;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_kfd_info(amdsmi_processor_handle processor_handle, amdsmi_kfd_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("kfd_node");
  memset(info, 0, sizeof *info);
  info->kfd_id = 1000 + g->u("kfd_node");
  info->node_id = static_cast<uint32_t>(g->u("kfd_node"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_compute_partition(amdsmi_processor_handle processor_handle, char* compute_partition,
                                                 uint32_t len) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("compute_partition");
  if (len < g->s("compute_partition").size() + 1) return AMDSMI_STATUS_INSUFFICIENT_SIZE;
  put(compute_partition, len, g->s("compute_partition"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_partition(amdsmi_processor_handle processor_handle, char* memory_partition,
                                                uint32_t len) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("memory_partition");
  if (len < g->s("memory_partition").size() + 1) return AMDSMI_STATUS_INSUFFICIENT_SIZE;
  put(memory_partition, len, g->s("memory_partition"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_temp_metric(amdsmi_processor_handle processor_handle, amdsmi_temperature_type_t sensor_type,
                                       amdsmi_temperature_metric_t metric, int64_t* temperature) {
  GPU_OR_FAIL(processor_handle);
  if (metric != AMDSMI_TEMP_CURRENT) return AMDSMI_STATUS_NOT_SUPPORTED;
  if (sensor_type == AMDSMI_TEMPERATURE_TYPE_HOTSPOT && g->has("hotspot_c")) {
    *temperature = static_cast<int64_t>(g->u("hotspot_c"));
    return AMDSMI_STATUS_SUCCESS;
  }
  if (sensor_type == AMDSMI_TEMPERATURE_TYPE_HBM_0 && g->has("hbm_temp_c")) {
    *temperature = static_cast<int64_t>(g->u("hbm_temp_c"));
    return AMDSMI_STATUS_SUCCESS;
  }
  return AMDSMI_STATUS_NOT_SUPPORTED;
}

amdsmi_status_t amdsmi_get_pcie_info(amdsmi_processor_handle processor_handle, amdsmi_pcie_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("pcie_width");
  memset(info, 0, sizeof *info);
  info->pcie_metric.pcie_width = static_cast<uint16_t>(g->u("pcie_width"));
  info->pcie_metric.pcie_speed = static_cast<uint32_t>(g->u("pcie_speed_mts"));
  info->pcie_static.max_pcie_width = static_cast<uint16_t>(g->u("pcie_max_width"));
  info->pcie_static.max_pcie_speed = static_cast<uint32_t>(g->u("pcie_max_speed_mts"));
  info->pcie_metric.pcie_replay_count = g->u("pcie_replays", UINT64_MAX);
  info->pcie_metric.pcie_l0_to_recovery_count = g->u("pcie_recoveries", UINT64_MAX);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_power_info(amdsmi_processor_handle processor_handle, amdsmi_power_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("power_w");
  memset(info, 0, sizeof *info);
  info->current_socket_power = static_cast<uint32_t>(g->u("power_w"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_power_cap_info(amdsmi_processor_handle processor_handle, uint32_t,
                                          amdsmi_power_cap_info_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("power_cap_w");
  memset(info, 0, sizeof *info);
  info->power_cap = g->u("power_cap_w") * 1000000ull;  // uW, as the real library reports on Linux
  info->default_power_cap = g->u("power_cap_default_w") * 1000000ull;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_vram_usage(amdsmi_processor_handle processor_handle, amdsmi_vram_usage_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("vram_used_mb");
  memset(info, 0, sizeof *info);
  info->vram_total = static_cast<uint32_t>(g->u("vram_mb"));
  info->vram_used = static_cast<uint32_t>(g->u("vram_used_mb"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_process_list(amdsmi_processor_handle processor_handle, uint32_t* max_processes,
                                            amdsmi_proc_info_t* list) {
  GPU_OR_FAIL(processor_handle);
  // "procs" = "pid:vram_mb,pid:vram_mb"; or nprocs=N synthetic entries
  std::vector<std::pair<uint32_t, uint64_t>> procs;
  if (g->has("nprocs")) {
    for (uint64_t i = 0; i < g->u("nprocs"); ++i) procs.push_back({static_cast<uint32_t>(5000 + i), i});
  } else {
    const std::string s = g->s("procs");
    size_t p = 0;
    while (p < s.size()) {
      size_t e = s.find(',', p);
      if (e == std::string::npos) e = s.size();
      unsigned pid = 0;
      unsigned long long mb = 0;
      if (sscanf(s.substr(p, e - p).c_str(), "%u:%llu", &pid, &mb) == 2) procs.push_back({pid, mb});
      p = e + 1;
    }
  }
  const uint32_t n = static_cast<uint32_t>(procs.size());
  if (!list) {
    *max_processes = n;
    return AMDSMI_STATUS_SUCCESS;
  }
  const uint32_t cap = *max_processes < n ? *max_processes : n;
  for (uint32_t i = 0; i < cap; ++i) {
    memset(&list[i], 0, sizeof list[i]);
    list[i].pid = procs[i].first;
    list[i].memory_usage.vram_mem = procs[i].second << 20;
  }
  *max_processes = cap;
  return cap < n ? AMDSMI_STATUS_OUT_OF_RESOURCES : AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_activity(amdsmi_processor_handle processor_handle, amdsmi_engine_usage_t* info) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("gfx_activity");
  memset(info, 0, sizeof *info);
  info->gfx_activity = static_cast<uint32_t>(g->u("gfx_activity"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_metrics_info(amdsmi_processor_handle processor_handle,
                                            amdsmi_gpu_metrics_t* pgpu_metrics) {
  GPU_OR_FAIL(processor_handle);
  FIELD_OR_NA("gfxclk_mhz");
  // the real library fills only what the firmware reports; the rest keeps the caller's all-ones
  if (g->has("xgmi_width")) pgpu_metrics->xgmi_link_width = static_cast<uint16_t>(g->u("xgmi_width"));
  if (g->has("xgmi_speed_gbps")) pgpu_metrics->xgmi_link_speed = static_cast<uint16_t>(g->u("xgmi_speed_gbps"));
  pgpu_metrics->current_gfxclks[0] = static_cast<uint16_t>(g->u("gfxclk_mhz"));
  pgpu_metrics->current_gfxclks[1] = static_cast<uint16_t>(g->u("gfxclk_mhz"));
  if (g->has("throttle_acc.n")) {
    pgpu_metrics->accumulation_counter = g->u("throttle_acc.n");
    pgpu_metrics->prochot_residency_acc = g->u("throttle_acc.prochot");
    pgpu_metrics->ppt_residency_acc = g->u("throttle_acc.ppt");
    pgpu_metrics->socket_thm_residency_acc = g->u("throttle_acc.socket_thm");
    pgpu_metrics->vr_thm_residency_acc = g->u("throttle_acc.vr_thm");
    pgpu_metrics->hbm_thm_residency_acc = g->u("throttle_acc.hbm_thm");
  }
  return AMDSMI_STATUS_SUCCESS;
}

}  // extern "C"
