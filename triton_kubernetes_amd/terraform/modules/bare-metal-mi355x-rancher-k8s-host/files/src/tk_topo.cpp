// amdgpu-topo-labeller (N1): enumerate the node's AMD GPUs
// through libamd_smi and emit one JSON document describing each GPU and every
// GPU<->GPU link.  triton_kubernetes_amd.node.labels turns it into Kubernetes
// node labels (product, count, CU count, VRAM, partition modes, xGMI hive id,
// links per GPU, fully-connected flag) used by the device plugin, the
// readiness waiter and xGMI-aware pod affinity.
//
// Built twice from this file: libtk_topo.so (C ABI, loaded with ctypes) and the
// stand-alone `amdgpu-topo-labeller` executable (-DTK_TOPO_MAIN) that the
// bare-metal host bootstrap runs on nodes without Python tooling.

#include <amd_smi/amdsmi.h>

#include <cinttypes>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

std::string esc(const char* s) {
  std::string o;
  for (const char* p = s; *p; ++p) {
    const unsigned char c = static_cast<unsigned char>(*p);
    if (c == '"' || c == '\\') { o += '\\'; o += static_cast<char>(c); }
    else if (c < 0x20) { char b[8]; snprintf(b, sizeof(b), "\\u%04x", c); o += b; }
    else o += static_cast<char>(c);
  }
  return o;
}

const char* link_name(amdsmi_link_type_t t) {
  switch (t) {
    case AMDSMI_LINK_TYPE_INTERNAL: return "INTERNAL";
    case AMDSMI_LINK_TYPE_PCIE: return "PCIE";
    case AMDSMI_LINK_TYPE_XGMI: return "XGMI";
    case AMDSMI_LINK_TYPE_NOT_APPLICABLE: return "NA";
    default: return "UNKNOWN";
  }
}

struct Gpu {
  amdsmi_processor_handle h;
};

void appendf(std::string& o, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void appendf(std::string& o, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  o += buf;
}

std::string topology_json(int* status) {
  std::string o;
  amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    const char* msg = nullptr;
    amdsmi_status_code_to_string(st, &msg);
    appendf(o, "{\"source\":\"amd_smi\",\"error\":\"amdsmi_init: %s\",\"gpus\":[]}", msg ? msg : "?");
    *status = static_cast<int>(st);
    return o;
  }
  std::vector<Gpu> gpus;
  uint32_t nsock = 0;
  amdsmi_get_socket_handles(&nsock, nullptr);
  std::vector<amdsmi_socket_handle> socks(nsock);
  if (nsock) amdsmi_get_socket_handles(&nsock, socks.data());
  for (uint32_t s = 0; s < nsock; ++s) {
    uint32_t np = 0;
    amdsmi_get_processor_handles(socks[s], &np, nullptr);
    std::vector<amdsmi_processor_handle> ph(np);
    if (np) amdsmi_get_processor_handles(socks[s], &np, ph.data());
    for (auto h : ph) {
      processor_type_t t;
      if (amdsmi_get_processor_type(h, &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
        gpus.push_back({h});
    }
  }
  o += "{\"source\":\"amd_smi\",";
  amdsmi_driver_info_t drv{};
  if (!gpus.empty() && amdsmi_get_gpu_driver_info(gpus[0].h, &drv) == AMDSMI_STATUS_SUCCESS)
    appendf(o, "\"driver\":{\"name\":\"%s\",\"version\":\"%s\"},", esc(drv.driver_name).c_str(),
            esc(drv.driver_version).c_str());
  o += "\"gpus\":[";
  for (size_t i = 0; i < gpus.size(); ++i) {
    auto h = gpus[i].h;
    if (i) o += ",";
    appendf(o, "{\"index\":%zu", i);
    amdsmi_enumeration_info_t en{};
    if (amdsmi_get_gpu_enumeration_info(h, &en) == AMDSMI_STATUS_SUCCESS)
      appendf(o, ",\"hip_id\":%u,\"drm_render\":%u,\"drm_card\":%u", en.hip_id, en.drm_render, en.drm_card);
    amdsmi_bdf_t bdf{};
    if (amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS)
      appendf(o, ",\"bdf\":\"%04" PRIx64 ":%02" PRIx64 ":%02" PRIx64 ".%" PRIx64 "\"",
              (uint64_t)bdf.domain_number, (uint64_t)bdf.bus_number, (uint64_t)bdf.device_number,
              (uint64_t)bdf.function_number);
    amdsmi_asic_info_t asic{};
    if (amdsmi_get_gpu_asic_info(h, &asic) == AMDSMI_STATUS_SUCCESS) {
      appendf(o, ",\"market_name\":\"%s\",\"vendor_id\":\"0x%x\",\"device_id\":\"0x%" PRIx64 "\",\"rev_id\":%u",
              esc(asic.market_name).c_str(), asic.vendor_id, asic.device_id, asic.rev_id);
      appendf(o, ",\"asic_serial\":\"%s\"", esc(asic.asic_serial).c_str());
      if (asic.num_of_compute_units != 0xFFFFFFFFu) appendf(o, ",\"compute_units\":%u", asic.num_of_compute_units);
      if (asic.oam_id != 0xFFFFFFFFu) appendf(o, ",\"oam_id\":%u", asic.oam_id);
      if (asic.target_graphics_version != 0xFFFFFFFFFFFFFFFFull)
        appendf(o, ",\"target_graphics_version\":\"gfx%" PRIx64 "\"", asic.target_graphics_version);
    }
    amdsmi_vram_info_t vram{};
    if (amdsmi_get_gpu_vram_info(h, &vram) == AMDSMI_STATUS_SUCCESS)
      appendf(o, ",\"vram_mb\":%" PRIu64 ",\"vram_bit_width\":%u", vram.vram_size, vram.vram_bit_width);
    uint32_t numa = 0;
    if (amdsmi_topo_get_numa_node_number(h, &numa) == AMDSMI_STATUS_SUCCESS) appendf(o, ",\"numa_node\":%u", numa);
    char part[64] = {0};
    if (amdsmi_get_gpu_compute_partition(h, part, sizeof(part)) == AMDSMI_STATUS_SUCCESS)
      appendf(o, ",\"compute_partition\":\"%s\"", esc(part).c_str());
    memset(part, 0, sizeof(part));
    if (amdsmi_get_gpu_memory_partition(h, part, sizeof(part)) == AMDSMI_STATUS_SUCCESS)
      appendf(o, ",\"memory_partition\":\"%s\"", esc(part).c_str());
    amdsmi_xgmi_info_t xg{};
    if (amdsmi_get_xgmi_info(h, &xg) == AMDSMI_STATUS_SUCCESS)
      appendf(o, ",\"xgmi_hive_id\":\"0x%" PRIx64 "\",\"xgmi_node_id\":\"0x%" PRIx64 "\",\"xgmi_lanes\":%u",
              xg.xgmi_hive_id, xg.xgmi_node_id, (unsigned)xg.xgmi_lanes);
    amdsmi_error_count_t ec{};
    if (amdsmi_get_gpu_total_ecc_count(h, &ec) == AMDSMI_STATUS_SUCCESS)
      appendf(o, ",\"ecc_correctable\":%" PRIu64 ",\"ecc_uncorrectable\":%" PRIu64, ec.correctable_count,
              ec.uncorrectable_count);
    o += ",\"links\":[";
    bool first = true;
    for (size_t j = 0; j < gpus.size(); ++j) {
      if (j == i) continue;
      uint64_t hops = 0;
      amdsmi_link_type_t lt = AMDSMI_LINK_TYPE_UNKNOWN;
      if (amdsmi_topo_get_link_type(h, gpus[j].h, &hops, &lt) != AMDSMI_STATUS_SUCCESS) continue;
      bool p2p = false;
      amdsmi_is_P2P_accessible(h, gpus[j].h, &p2p);
      appendf(o, "%s{\"peer\":%zu,\"type\":\"%s\",\"hops\":%" PRIu64 ",\"p2p\":%s}", first ? "" : ",", j,
              link_name(lt), hops, p2p ? "true" : "false");
      first = false;
    }
    o += "]}";
  }
  o += "]}";
  amdsmi_shut_down();
  *status = 0;
  return o;
}

}  // namespace

// Writes the JSON document into buf (NUL-terminated).  Returns 0 on success,
// the amdsmi status on init failure (buf still holds a JSON error document),
// or -(required size) if buf is too small.
extern "C" int tkt_topology_json(char* buf, size_t len) {
  int status = 0;
  const std::string j = topology_json(&status);
  if (j.size() + 1 > len) return -static_cast<int>(j.size() + 1);
  memcpy(buf, j.c_str(), j.size() + 1);
  return status;
}

#ifdef TK_TOPO_MAIN
int main() {
  int status = 0;
  const std::string j = topology_json(&status);
  fputs(j.c_str(), stdout);
  fputc('\n', stdout);
  return status == 0 ? 0 : 2;
}
#endif
