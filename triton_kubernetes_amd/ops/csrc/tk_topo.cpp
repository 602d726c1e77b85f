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

#include <algorithm>
#include <cctype>
#include <cinttypes>
#include <climits>
#include <cstdint>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
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

struct Link {
  size_t peer;
  const char* type;
  uint64_t hops;
  bool p2p;
};

// Everything the labeller knows about one GPU; the JSON document and the
// label set are both rendered from this.
struct GpuInfo {
  amdsmi_processor_handle h{};
  bool has_enum = false, has_bdf = false, has_asic = false, has_vram = false, has_numa = false;
  bool has_xgmi = false, has_ecc = false;
  amdsmi_enumeration_info_t en{};
  amdsmi_bdf_t bdf{};
  amdsmi_asic_info_t asic{};
  amdsmi_vram_info_t vram{};
  uint32_t numa = 0;
  std::string compute_partition, memory_partition;
  amdsmi_xgmi_info_t xg{};
  amdsmi_error_count_t ec{};
  std::vector<Link> links;
};

struct Topology {
  int status = 0;
  std::string error;
  bool has_driver = false;
  amdsmi_driver_info_t drv{};
  std::vector<GpuInfo> gpus;
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

Topology collect() {
  Topology t;
  amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    const char* msg = nullptr;
    amdsmi_status_code_to_string(st, &msg);
    t.error = std::string("amdsmi_init: ") + (msg ? msg : "?");
    t.status = static_cast<int>(st);
    return t;
  }
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
      processor_type_t pt;
      if (amdsmi_get_processor_type(h, &pt) == AMDSMI_STATUS_SUCCESS && pt == AMDSMI_PROCESSOR_TYPE_AMD_GPU) {
        t.gpus.emplace_back();
        t.gpus.back().h = h;
      }
    }
  }
  if (!t.gpus.empty())
    t.has_driver = amdsmi_get_gpu_driver_info(t.gpus[0].h, &t.drv) == AMDSMI_STATUS_SUCCESS;
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    GpuInfo& g = t.gpus[i];
    auto h = g.h;
    g.has_enum = amdsmi_get_gpu_enumeration_info(h, &g.en) == AMDSMI_STATUS_SUCCESS;
    g.has_bdf = amdsmi_get_gpu_device_bdf(h, &g.bdf) == AMDSMI_STATUS_SUCCESS;
    g.has_asic = amdsmi_get_gpu_asic_info(h, &g.asic) == AMDSMI_STATUS_SUCCESS;
    g.has_vram = amdsmi_get_gpu_vram_info(h, &g.vram) == AMDSMI_STATUS_SUCCESS;
    g.has_numa = amdsmi_topo_get_numa_node_number(h, &g.numa) == AMDSMI_STATUS_SUCCESS;
    char part[64] = {0};
    if (amdsmi_get_gpu_compute_partition(h, part, sizeof(part)) == AMDSMI_STATUS_SUCCESS) g.compute_partition = part;
    memset(part, 0, sizeof(part));
    if (amdsmi_get_gpu_memory_partition(h, part, sizeof(part)) == AMDSMI_STATUS_SUCCESS) g.memory_partition = part;
    g.has_xgmi = amdsmi_get_xgmi_info(h, &g.xg) == AMDSMI_STATUS_SUCCESS;
    g.has_ecc = amdsmi_get_gpu_total_ecc_count(h, &g.ec) == AMDSMI_STATUS_SUCCESS;
    for (size_t j = 0; j < t.gpus.size(); ++j) {
      if (j == i) continue;
      uint64_t hops = 0;
      amdsmi_link_type_t lt = AMDSMI_LINK_TYPE_UNKNOWN;
      if (amdsmi_topo_get_link_type(h, t.gpus[j].h, &hops, &lt) != AMDSMI_STATUS_SUCCESS) continue;
      bool p2p = false;
      amdsmi_is_P2P_accessible(h, t.gpus[j].h, &p2p);
      g.links.push_back({j, link_name(lt), hops, p2p});
    }
  }
  amdsmi_shut_down();
  return t;
}

std::string render_json(const Topology& t) {
  std::string o;
  if (t.status != 0) {
    appendf(o, "{\"source\":\"amd_smi\",\"error\":\"%s\",\"gpus\":[]}", esc(t.error.c_str()).c_str());
    return o;
  }
  o += "{\"source\":\"amd_smi\",";
  if (t.has_driver)
    appendf(o, "\"driver\":{\"name\":\"%s\",\"version\":\"%s\"},", esc(t.drv.driver_name).c_str(),
            esc(t.drv.driver_version).c_str());
  o += "\"gpus\":[";
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    const GpuInfo& g = t.gpus[i];
    if (i) o += ",";
    appendf(o, "{\"index\":%zu", i);
    if (g.has_enum)
      appendf(o, ",\"hip_id\":%u,\"drm_render\":%u,\"drm_card\":%u", g.en.hip_id, g.en.drm_render, g.en.drm_card);
    if (g.has_bdf)
      appendf(o, ",\"bdf\":\"%04" PRIx64 ":%02" PRIx64 ":%02" PRIx64 ".%" PRIx64 "\"",
              (uint64_t)g.bdf.domain_number, (uint64_t)g.bdf.bus_number, (uint64_t)g.bdf.device_number,
              (uint64_t)g.bdf.function_number);
    if (g.has_asic) {
      const amdsmi_asic_info_t& a = g.asic;
      appendf(o, ",\"market_name\":\"%s\",\"vendor_id\":\"0x%x\",\"device_id\":\"0x%" PRIx64 "\",\"rev_id\":%u",
              esc(a.market_name).c_str(), a.vendor_id, a.device_id, a.rev_id);
      appendf(o, ",\"asic_serial\":\"%s\"", esc(a.asic_serial).c_str());
      if (a.num_of_compute_units != 0xFFFFFFFFu) appendf(o, ",\"compute_units\":%u", a.num_of_compute_units);
      if (a.oam_id != 0xFFFFFFFFu) appendf(o, ",\"oam_id\":%u", a.oam_id);
      if (a.target_graphics_version != 0xFFFFFFFFFFFFFFFFull)
        appendf(o, ",\"target_graphics_version\":\"gfx%" PRIx64 "\"", a.target_graphics_version);
    }
    if (g.has_vram)
      appendf(o, ",\"vram_mb\":%" PRIu64 ",\"vram_bit_width\":%u", g.vram.vram_size, g.vram.vram_bit_width);
    if (g.has_numa) appendf(o, ",\"numa_node\":%u", g.numa);
    if (!g.compute_partition.empty())
      appendf(o, ",\"compute_partition\":\"%s\"", esc(g.compute_partition.c_str()).c_str());
    if (!g.memory_partition.empty())
      appendf(o, ",\"memory_partition\":\"%s\"", esc(g.memory_partition.c_str()).c_str());
    if (g.has_xgmi)
      appendf(o, ",\"xgmi_hive_id\":\"0x%" PRIx64 "\",\"xgmi_node_id\":\"0x%" PRIx64 "\",\"xgmi_lanes\":%u",
              g.xg.xgmi_hive_id, g.xg.xgmi_node_id, (unsigned)g.xg.xgmi_lanes);
    if (g.has_ecc)
      appendf(o, ",\"ecc_correctable\":%" PRIu64 ",\"ecc_uncorrectable\":%" PRIu64, g.ec.correctable_count,
              g.ec.uncorrectable_count);
    o += ",\"links\":[";
    for (size_t k = 0; k < g.links.size(); ++k) {
      const Link& l = g.links[k];
      appendf(o, "%s{\"peer\":%zu,\"type\":\"%s\",\"hops\":%" PRIu64 ",\"p2p\":%s}", k ? "," : "", l.peer, l.type,
              l.hops, l.p2p ? "true" : "false");
    }
    o += "]}";
  }
  o += "]}";
  return o;
}

// --- node labels -----------------------------------------------------------
// Same rules as triton_kubernetes_amd/node/labels.py:labels_from_topology (the
// Python side is the spec and is unit-tested; tests/test_labels.py checks this
// renderer against it on the box).

// Kubernetes label value: [A-Za-z0-9._-], trimmed of leading/trailing '-._', <= 63.
std::string label_value(const std::string& v) {
  std::string s;
  for (char c : v) s += (isalnum(static_cast<unsigned char>(c)) || c == '.' || c == '_' || c == '-') ? c : '-';
  size_t b = s.find_first_not_of("-._"), e = s.find_last_not_of("-._");
  if (b == std::string::npos) return "";
  s = s.substr(b, e - b + 1);
  return s.size() > 63 ? s.substr(0, 63) : s;
}

// PCI device id -> product, for parts whose market name is not the SKU name
// (amd_smi reports an MI355X as "AMD Instinct MI355 OAM").
const char* product_from_device_id(uint64_t id) {
  switch (id) {
    case 0x75a3: return "MI355X";
    case 0x74a5: return "MI325X";
    case 0x74a1: return "MI300X";
    default: return nullptr;
  }
}

std::string product_name(const GpuInfo& g) {
  if (const char* p = product_from_device_id(g.asic.device_id)) return p;
  const char* m = g.asic.market_name;
  for (const char* p = m; *p; ++p) {
    if (p[0] == 'M' && p[1] == 'I' && isdigit((unsigned char)p[2]) && isdigit((unsigned char)p[3]) &&
        isdigit((unsigned char)p[4])) {
      const char* e = p + 5;
      while (*e >= 'A' && *e <= 'Z') ++e;
      return std::string(p, e);
    }
  }
  return label_value(m);
}

std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
  return s;
}

std::string render_labels(const Topology& t) {
  std::map<std::string, std::string> L;
  const auto& gs = t.gpus;
  if (gs.empty()) {
    L["amd.com/gpu.present"] = "false";
  } else {
    L["amd.com/gpu.present"] = "true";
    L["amd.com/gpu.count"] = std::to_string(gs.size());
    std::set<std::string> names, dev_ids, targets, cparts, mparts, hives;
    uint32_t min_cu = UINT32_MAX;
    uint64_t min_vram = UINT64_MAX;
    size_t min_xgmi = SIZE_MAX;
    uint64_t ecc = 0;
    for (const auto& g : gs) {
      if (g.has_asic) {
        if (g.asic.market_name[0] || product_from_device_id(g.asic.device_id)) names.insert(product_name(g));
        char b[32];
        snprintf(b, sizeof(b), "0x%" PRIx64, g.asic.device_id);
        if (g.asic.device_id) dev_ids.insert(b);
        if (g.asic.num_of_compute_units != 0xFFFFFFFFu && g.asic.num_of_compute_units)
          min_cu = std::min(min_cu, g.asic.num_of_compute_units);
        if (g.asic.target_graphics_version != 0xFFFFFFFFFFFFFFFFull) {
          snprintf(b, sizeof(b), "gfx%" PRIx64, g.asic.target_graphics_version);
          targets.insert(b);
        }
      }
      if (g.has_vram && g.vram.vram_size) min_vram = std::min<uint64_t>(min_vram, g.vram.vram_size);
      if (!g.compute_partition.empty()) cparts.insert(lower(g.compute_partition));
      if (!g.memory_partition.empty()) mparts.insert(lower(g.memory_partition));
      if (g.has_xgmi && g.xg.xgmi_hive_id) {
        char b[32];
        snprintf(b, sizeof(b), "0x%" PRIx64, g.xg.xgmi_hive_id);
        hives.insert(b);
      }
      std::set<size_t> peers;
      for (const auto& l : g.links)
        if (strcmp(l.type, "XGMI") == 0) peers.insert(l.peer);
      min_xgmi = std::min(min_xgmi, peers.size());
      if (g.has_ecc) ecc += g.ec.uncorrectable_count;
    }
    if (names.size() == 1) {
      const std::string n = *names.begin();
      L["amd.com/gpu.product-name"] = label_value(n);
      if (n.rfind("MI", 0) == 0) L["amd.com/gpu.family"] = "AI";
    }
    if (dev_ids.size() == 1) L["amd.com/gpu.device-id"] = label_value(*dev_ids.begin());
    if (min_cu != UINT32_MAX) L["amd.com/gpu.cu-count"] = std::to_string(min_cu);
    if (min_vram != UINT64_MAX) L["amd.com/gpu.vram"] = std::to_string(min_vram / 1024) + "G";
    if (targets.size() == 1) L["amd.com/gpu.target"] = label_value(*targets.begin());
    if (cparts.size() == 1) L["amd.com/gpu.compute-partition"] = label_value(*cparts.begin());
    if (mparts.size() == 1) L["amd.com/gpu.memory-partition"] = label_value(*mparts.begin());
    if (hives.size() == 1) L["amd.com/xgmi.hive-id"] = label_value(*hives.begin());
    L["amd.com/xgmi.links-per-gpu"] = std::to_string(min_xgmi);
    L["amd.com/xgmi.fully-connected"] = (gs.size() > 1 && min_xgmi == gs.size() - 1) ? "true" : "false";
    L["amd.com/gpu.ecc-uncorrectable"] = std::to_string(ecc);
  }
  std::string o;
  for (const auto& kv : L) o += kv.first + "=" + kv.second + "\n";
  return o;
}

}  // namespace

// Writes the JSON document into buf (NUL-terminated).  Returns 0 on success,
// the amdsmi status on init failure (buf still holds a JSON error document),
// or -(required size) if buf is too small.
extern "C" int tkt_topology_json(char* buf, size_t len) {
  const Topology t = collect();
  const std::string j = render_json(t);
  if (j.size() + 1 > len) return -static_cast<int>(j.size() + 1);
  memcpy(buf, j.c_str(), j.size() + 1);
  return t.status;
}

// Same contract as tkt_topology_json, but the payload is the `key=value\n`
// node label set.
extern "C" int tkt_topology_labels(char* buf, size_t len) {
  const Topology t = collect();
  const std::string j = t.status == 0 ? render_labels(t) : std::string();
  if (j.size() + 1 > len) return -static_cast<int>(j.size() + 1);
  memcpy(buf, j.c_str(), j.size() + 1);
  return t.status;
}

#ifdef TK_TOPO_MAIN
// amdgpu-topo-labeller            topology JSON on stdout
// amdgpu-topo-labeller --labels   one `amd.com/...=value` node label per line
int main(int argc, char** argv) {
  bool labels = false;
  for (int i = 1; i < argc; ++i) {
    if (strcmp(argv[i], "--labels") == 0) {
      labels = true;
    } else {
      fprintf(stderr, "usage: %s [--labels]\n", argv[0]);
      return 64;
    }
  }
  const Topology t = collect();
  if (labels) {
    if (t.status != 0) {
      fprintf(stderr, "amdgpu-topo-labeller: %s\n", t.error.c_str());
      return 2;
    }
    fputs(render_labels(t).c_str(), stdout);
    return 0;
  }
  fputs(render_json(t).c_str(), stdout);
  fputc('\n', stdout);
  return t.status == 0 ? 0 : 2;
}
#endif
