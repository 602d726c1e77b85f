// amdgpu-topo-labeller (N1): describe the node's AMD GPUs and
// every GPU<->GPU link as one JSON document, or as the Kubernetes node labels
// derived from it (product, count, CU count, VRAM, partition modes, xGMI hive
// id, links per GPU, fully-connected flag, RDMA NICs) used by the device plugin,
// the readiness waiter, xGMI-aware pod affinity and the inter-node RCCL settings.
//
// Two collectors fill the same GpuInfo records:
//   amdsmi  libamd_smi (amdsmi_init + per-processor queries);
//   sysfs   the KFD topology (/sys/class/kfd/kfd/topology/nodes) joined with
//           the DRM device attributes (/sys/class/drm/renderD<minor>/device):
//           plain file reads, no library state — ~1 ms instead of the tens of
//           ms amdsmi_init costs, and safe inside a process that also runs HIP.
// tests/test_gpu_probes.py checks on an MI355X that both give identical labels.
//
// Built twice from this file:
//   libtk_topo.so          C ABI for ctypes, sysfs collector only.  It is loaded
//                          into processes that also run HIP and RCCL, so it
//                          does not link libamd_smi at all (amd_smi's library
//                          state next to librccl crashed dlopen on the box).
//   amdgpu-topo-labeller   stand-alone executable (-DTK_TOPO_MAIN
//                          -DTK_TOPO_AMDSMI): both collectors; the agent and
//                          the bare-metal host bootstrap run it as a child.

#ifdef TK_TOPO_AMDSMI
#include <amd_smi/amdsmi.h>
#endif
#include <dirent.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cinttypes>
#include <climits>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace {

// Length of the well-formed UTF-8 sequence at s[i] (RFC 3629: no overlong forms, no
// surrogates, nothing past U+10FFFF), 0 when the bytes there are not one.
size_t utf8_len(const std::string& s, size_t i) {
  const auto b = [&](size_t k) { return i + k < s.size() ? static_cast<unsigned char>(s[i + k]) : 0u; };
  const unsigned c = b(0);
  const auto cont = [&](size_t k) { return (b(k) & 0xC0) == 0x80; };
  if (c >= 0xC2 && c <= 0xDF) return cont(1) ? 2 : 0;
  if (c >= 0xE0 && c <= 0xEF) {
    const unsigned lo = c == 0xE0 ? 0xA0 : 0x80, hi = c == 0xED ? 0x9F : 0xBF;
    return b(1) >= lo && b(1) <= hi && cont(2) ? 3 : 0;
  }
  if (c >= 0xF0 && c <= 0xF4) {
    const unsigned lo = c == 0xF0 ? 0x90 : 0x80, hi = c == 0xF4 ? 0x8F : 0xBF;
    return b(1) >= lo && b(1) <= hi && cont(2) && cont(3) ? 4 : 0;
  }
  return 0;
}

// A JSON string body.  sysfs attributes are bytes: a byte that does not start a
// well-formed UTF-8 sequence becomes U+FFFD, so the document always parses.
std::string esc(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = static_cast<unsigned char>(s[i]);
    if (c == '"' || c == '\\') { o += '\\'; o += static_cast<char>(c); ++i; }
    else if (c < 0x20 || c == 0x7F) { char b[8]; snprintf(b, sizeof(b), "\\u%04x", c); o += b; ++i; }
    else if (c < 0x80) { o += static_cast<char>(c); ++i; }
    else if (const size_t n = utf8_len(s, i)) { o.append(s, i, n); i += n; }
    else { o += "\\ufffd"; ++i; }
  }
  return o;
}

void appendf(std::string& o, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void appendf(std::string& o, const char* fmt, ...) {
  char buf[1024];
  va_list ap, again;
  va_start(ap, fmt);
  va_copy(again, ap);
  const int n = vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (n >= static_cast<int>(sizeof(buf))) {  // longer than the stack buffer: format again, sized exactly
    std::string big(static_cast<size_t>(n) + 1, '\0');
    vsnprintf(&big[0], big.size(), fmt, again);
    big.resize(static_cast<size_t>(n));
    o += big;
  } else if (n > 0) {
    o.append(buf, static_cast<size_t>(n));
  }
  va_end(again);
}

struct Link {
  size_t peer;
  std::string type;  // XGMI | PCIE | ...
  uint64_t hops;
  bool p2p;
};

// Everything the labeller knows about one GPU, collector-independent.
struct GpuInfo {
  int64_t hip_id = -1, drm_render = -1, drm_card = -1;
  std::string bdf, market_name, vendor_id, device_id, serial, gfx, compute_partition, memory_partition;
  std::string vbios;  // VBIOS version (e.g. "113-M355-01-1K1-020F"); "" not reported
  int64_t rev_id = -1, compute_units = -1, oam_id = -1, numa_node = -1;
  uint64_t vram_mb = 0;
  uint32_t vram_bit_width = 0;
  bool has_xgmi = false, has_ecc = false;
  uint64_t hive_id = 0, xgmi_node_id = 0;
  uint32_t xgmi_lanes = 0;
  uint64_t ecc_correctable = 0, ecc_uncorrectable = 0;
  // retired VRAM pages (the driver's bad-page records; -1: not reported), of which pending
  // (marked bad, reserved at the next reset)
  int64_t bad_pages = -1, bad_pages_pending = -1;
  // the GPU's PCIe link to the host (its PCI function; partitions have none): lanes and
  // GT/s, current and the most the device supports (-1: not reported)
  int64_t pcie_width = -1, pcie_max_width = -1;
  double pcie_gts = -1.0, pcie_max_gts = -1.0;
  // board power cap and its default, watts (the PCI function's hwmon; -1: not reported)
  int64_t power_cap_w = -1, power_cap_default_w = -1;
  std::vector<Link> links;
};

// One RDMA device (/sys/class/infiniband/<name>): the inter-node fabric RCCL uses
// between MI355X nodes (RoCE or InfiniBand NICs).
struct NicInfo {
  std::string name, link_layer, netdev, bdf;
  int port = 0;             // first ACTIVE port (0: none active)
  uint64_t rate_gbps = 0;   // of that port
  int gid_index = -1;       // RoCE v2 GID of that port (IPv4-mapped first); -1: none / not RoCE
  int64_t numa_node = -1;
};

struct Topology {
  std::string source;
  int status = 0;
  std::string error;
  std::string driver_name, driver_version;
  std::string rocm_version;  // the node's ROCm userspace (<ROCM_PATH>/.info/version)
  std::vector<GpuInfo> gpus;
  std::vector<NicInfo> nics;
};

std::string hex64(uint64_t v) {
  char b[32];
  snprintf(b, sizeof(b), "0x%" PRIx64, v);
  return b;
}

// ---------------------------------------------------------------- amd_smi --
#ifdef TK_TOPO_AMDSMI
const char* link_name(amdsmi_link_type_t t) {
  switch (t) {
    case AMDSMI_LINK_TYPE_INTERNAL: return "INTERNAL";
    case AMDSMI_LINK_TYPE_PCIE: return "PCIE";
    case AMDSMI_LINK_TYPE_XGMI: return "XGMI";
    case AMDSMI_LINK_TYPE_NOT_APPLICABLE: return "NA";
    default: return "UNKNOWN";
  }
}

Topology collect_amdsmi() {
  Topology t;
  t.source = "amd_smi";
  amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    const char* msg = nullptr;
    amdsmi_status_code_to_string(st, &msg);
    t.error = std::string("amdsmi_init: ") + (msg ? msg : "?");
    t.status = static_cast<int>(st);
    return t;
  }
  std::vector<amdsmi_processor_handle> hs;
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
      if (amdsmi_get_processor_type(h, &pt) == AMDSMI_STATUS_SUCCESS && pt == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
        hs.push_back(h);
    }
  }
  amdsmi_driver_info_t drv{};
  if (!hs.empty() && amdsmi_get_gpu_driver_info(hs[0], &drv) == AMDSMI_STATUS_SUCCESS) {
    t.driver_name = drv.driver_name;
    t.driver_version = drv.driver_version;
    // an in-tree amdgpu has no module version; amd_smi then reports the kernel banner
    // ("Linux version ..."): report none, as /sys/module/amdgpu/version does
    if (t.driver_version.rfind("Linux", 0) == 0) t.driver_version.clear();
  }
  for (size_t i = 0; i < hs.size(); ++i) {
    auto h = hs[i];
    GpuInfo g;
    amdsmi_enumeration_info_t en{};
    if (amdsmi_get_gpu_enumeration_info(h, &en) == AMDSMI_STATUS_SUCCESS) {
      g.hip_id = en.hip_id;
      g.drm_render = en.drm_render;
      g.drm_card = en.drm_card;
    }
    amdsmi_bdf_t bdf{};
    if (amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) {
      char b[32];
      snprintf(b, sizeof(b), "%04" PRIx64 ":%02" PRIx64 ":%02" PRIx64 ".%" PRIx64, (uint64_t)bdf.domain_number,
               (uint64_t)bdf.bus_number, (uint64_t)bdf.device_number, (uint64_t)bdf.function_number);
      g.bdf = b;
    }
    amdsmi_asic_info_t a{};
    if (amdsmi_get_gpu_asic_info(h, &a) == AMDSMI_STATUS_SUCCESS) {
      g.market_name = a.market_name;
      char b[16];
      snprintf(b, sizeof(b), "0x%x", a.vendor_id);
      g.vendor_id = b;
      g.device_id = hex64(a.device_id);
      g.rev_id = a.rev_id;
      g.serial = a.asic_serial;
      if (a.num_of_compute_units != 0xFFFFFFFFu) g.compute_units = a.num_of_compute_units;
      if (a.oam_id != 0xFFFFFFFFu) g.oam_id = a.oam_id;
      if (a.target_graphics_version != 0xFFFFFFFFFFFFFFFFull) {
        char gb[32];
        snprintf(gb, sizeof(gb), "gfx%" PRIx64, a.target_graphics_version);
        g.gfx = gb;
      }
    }
    amdsmi_power_cap_info_t pc{};
    if (amdsmi_get_power_cap_info(h, 0, &pc) == AMDSMI_STATUS_SUCCESS && pc.power_cap > 0) {  // uW on bare metal
      g.power_cap_w = static_cast<int64_t>((pc.power_cap + 500000) / 1000000);
      if (pc.default_power_cap > 0) g.power_cap_default_w = static_cast<int64_t>((pc.default_power_cap + 500000) / 1000000);
    }
    amdsmi_vbios_info_t vb{};
    // sysfs vbios_version is amd_smi's part_number ("113-M355-01-1K1-020F" on the box);
    // amd_smi's version field is a build number
    if (amdsmi_get_gpu_vbios_info(h, &vb) == AMDSMI_STATUS_SUCCESS) g.vbios = vb.part_number[0] ? vb.part_number : vb.version;
    amdsmi_vram_info_t vram{};
    if (amdsmi_get_gpu_vram_info(h, &vram) == AMDSMI_STATUS_SUCCESS) {
      g.vram_mb = vram.vram_size;
      g.vram_bit_width = vram.vram_bit_width;
    }
    uint32_t numa = 0;
    if (amdsmi_topo_get_numa_node_number(h, &numa) == AMDSMI_STATUS_SUCCESS) g.numa_node = numa;
    char part[64] = {0};
    if (amdsmi_get_gpu_compute_partition(h, part, sizeof(part)) == AMDSMI_STATUS_SUCCESS) g.compute_partition = part;
    memset(part, 0, sizeof(part));
    if (amdsmi_get_gpu_memory_partition(h, part, sizeof(part)) == AMDSMI_STATUS_SUCCESS) g.memory_partition = part;
    amdsmi_xgmi_info_t xg{};
    if (amdsmi_get_xgmi_info(h, &xg) == AMDSMI_STATUS_SUCCESS) {
      g.has_xgmi = true;
      g.hive_id = xg.xgmi_hive_id;
      g.xgmi_node_id = xg.xgmi_node_id;
      g.xgmi_lanes = xg.xgmi_lanes;
    }
    amdsmi_error_count_t ec{};
    if (amdsmi_get_gpu_total_ecc_count(h, &ec) == AMDSMI_STATUS_SUCCESS) {
      g.has_ecc = true;
      g.ecc_correctable = ec.correctable_count;
      g.ecc_uncorrectable = ec.uncorrectable_count;
    }
    amdsmi_pcie_info_t pcie{};
    if (amdsmi_get_pcie_info(h, &pcie) == AMDSMI_STATUS_SUCCESS) {
      // speeds come as MT/s (current) and GT/s or MT/s (max, by release): GT/s here
      auto gts = [](uint32_t v) { return v > 1000 ? v / 1000.0 : (double)v; };
      if (pcie.pcie_metric.pcie_width && pcie.pcie_metric.pcie_width != 0xFFFF) g.pcie_width = pcie.pcie_metric.pcie_width;
      if (pcie.pcie_static.max_pcie_width && pcie.pcie_static.max_pcie_width != 0xFFFF)
        g.pcie_max_width = pcie.pcie_static.max_pcie_width;
      if (pcie.pcie_metric.pcie_speed && pcie.pcie_metric.pcie_speed != 0xFFFFFFFFu) g.pcie_gts = gts(pcie.pcie_metric.pcie_speed);
      if (pcie.pcie_static.max_pcie_speed && pcie.pcie_static.max_pcie_speed != 0xFFFFFFFFu)
        g.pcie_max_gts = gts(pcie.pcie_static.max_pcie_speed);
    }
    uint32_t nbad = 0;
    if (amdsmi_get_gpu_bad_page_info(h, &nbad, nullptr) == AMDSMI_STATUS_SUCCESS) {
      g.bad_pages = nbad;
      g.bad_pages_pending = 0;
      if (nbad) {
        std::vector<amdsmi_retired_page_record_t> rec(nbad);
        uint32_t got = nbad;
        if (amdsmi_get_gpu_bad_page_info(h, &got, rec.data()) == AMDSMI_STATUS_SUCCESS)
          for (uint32_t k = 0; k < std::min(got, nbad); ++k)
            g.bad_pages_pending += rec[k].status == AMDSMI_MEM_PAGE_STATUS_PENDING;
      }
    }
    for (size_t j = 0; j < hs.size(); ++j) {
      if (j == i) continue;
      uint64_t hops = 0;
      amdsmi_link_type_t lt = AMDSMI_LINK_TYPE_UNKNOWN;
      if (amdsmi_topo_get_link_type(h, hs[j], &hops, &lt) != AMDSMI_STATUS_SUCCESS) continue;
      bool p2p = false;
      amdsmi_is_P2P_accessible(h, hs[j], &p2p);
      g.links.push_back({j, link_name(lt), hops, p2p});
    }
    t.gpus.push_back(std::move(g));
  }
  amdsmi_shut_down();
  return t;
}
#else
Topology collect_amdsmi() {
  Topology t;
  t.source = "amd_smi";
  t.status = 3;
  t.error = "amd_smi collector not built into this library (run amdgpu-topo-labeller --source amdsmi)";
  return t;
}
#endif

// ------------------------------------------------------------------ sysfs --
bool read_file(const std::string& path, std::string* out) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  out->clear();
  char buf[4096];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), f)) > 0) out->append(buf, n);  // the whole file
  fclose(f);
  while (!out->empty() && (out->back() == '\n' || out->back() == ' ')) out->pop_back();
  return true;
}

// "key value" lines (KFD properties files).
std::map<std::string, uint64_t> read_props(const std::string& path) {
  std::map<std::string, uint64_t> m;
  std::string s;
  if (!read_file(path, &s)) return m;
  size_t pos = 0;
  while (pos < s.size()) {
    size_t e = s.find('\n', pos);
    if (e == std::string::npos) e = s.size();
    const std::string line = s.substr(pos, e - pos);
    pos = e + 1;
    const size_t sp = line.find(' ');
    if (sp == std::string::npos) continue;
    char* end = nullptr;
    const std::string v = line.substr(sp + 1);
    const unsigned long long x = strtoull(v.c_str(), &end, 10);
    if (end && *end == 0) m[line.substr(0, sp)] = x;
  }
  return m;
}

std::vector<int> numeric_entries(const std::string& dir) {
  std::vector<int> ids;
  DIR* d = opendir(dir.c_str());
  if (!d) return ids;
  while (dirent* e = readdir(d)) {
    const char* n = e->d_name;
    if (!*n) continue;
    bool num = true;
    for (const char* p = n; *p; ++p) num = num && isdigit(static_cast<unsigned char>(*p));
    if (num) ids.push_back(atoi(n));
  }
  closedir(d);
  std::sort(ids.begin(), ids.end());
  return ids;
}

uint64_t prop(const std::map<std::string, uint64_t>& m, const char* k, uint64_t dflt = 0) {
  auto it = m.find(k);
  return it == m.end() ? dflt : it->second;
}

// gfx_target_version 90500 -> "gfx950" (major*10000 + minor*100 + stepping; minor/stepping print as hex digits)
std::string gfx_name(uint64_t v) {
  if (!v) return "";
  char b[32];
  snprintf(b, sizeof(b), "gfx%" PRIu64 "%" PRIx64 "%" PRIx64, v / 10000, (v / 100) % 100, v % 100);
  return b;
}

// PCI device id -> market name, for the sysfs path (amd_smi reads it from the
// ASIC).  Mirrored in node/labels.py:DEVICE_PRODUCTS.
const char* market_from_device_id(uint64_t id) {
  switch (id) {
    case 0x75a3: return "AMD Instinct MI355X";
    case 0x75a0: return "AMD Instinct MI350X";
    case 0x74a5: return "AMD Instinct MI325X";
    case 0x74a1: return "AMD Instinct MI300X";
    default: return nullptr;
  }
}

Topology collect_sysfs(const std::string& root) {
  Topology t;
  t.source = "sysfs";
  const std::string kfd = root + "/sys/class/kfd/kfd/topology/nodes";
  struct Node {
    int kfd_node;
    std::map<std::string, uint64_t> p;
  };
  const std::vector<int> all = numeric_entries(kfd);
  if (all.empty()) {
    t.status = 2;
    t.error = "no KFD topology at " + kfd;
    return t;
  }
  std::vector<Node> nodes;
  for (int id : all) {
    auto p = read_props(kfd + "/" + std::to_string(id) + "/properties");
    if (prop(p, "simd_count") > 0) nodes.push_back({id, std::move(p)});
  }
  std::map<int, size_t> kfd_to_index;
  for (size_t i = 0; i < nodes.size(); ++i) kfd_to_index[nodes[i].kfd_node] = i;
  std::string ver;
  if (read_file(root + "/sys/module/amdgpu/version", &ver)) t.driver_version = ver;
  t.driver_name = "amdgpu";
  for (size_t i = 0; i < nodes.size(); ++i) {
    const auto& p = nodes[i].p;
    GpuInfo g;
    g.hip_id = static_cast<int64_t>(i);
    const uint64_t minor = prop(p, "drm_render_minor", UINT64_MAX);
    if (minor != UINT64_MAX) g.drm_render = static_cast<int64_t>(minor);
    const uint64_t loc = prop(p, "location_id");
    char b[64];
    snprintf(b, sizeof(b), "%04" PRIx64 ":%02" PRIx64 ":%02" PRIx64 ".%" PRIx64, prop(p, "domain"),
             (loc >> 8) & 0xff, (loc >> 3) & 0x1f, loc & 7);
    g.bdf = b;
    const uint64_t did = prop(p, "device_id");
    snprintf(b, sizeof(b), "0x%" PRIx64, prop(p, "vendor_id"));
    g.vendor_id = b;
    g.device_id = hex64(did);
    const uint64_t spc = prop(p, "simd_per_cu", 4) ? prop(p, "simd_per_cu", 4) : 4;
    g.compute_units = static_cast<int64_t>(prop(p, "simd_count") / spc);
    g.gfx = gfx_name(prop(p, "gfx_target_version"));
    if (p.count("hive_id")) {
      g.has_xgmi = true;
      g.hive_id = prop(p, "hive_id");
    }
    if (const uint64_t uid = prop(p, "unique_id")) {
      snprintf(b, sizeof(b), "%" PRIx64, uid);
      g.serial = b;
    }
    // local memory: the KFD mem bank(s) of this node
    const std::string nd = kfd + "/" + std::to_string(nodes[i].kfd_node);
    uint64_t vram = 0;
    for (int mb : numeric_entries(nd + "/mem_banks")) {
      auto mp = read_props(nd + "/mem_banks/" + std::to_string(mb) + "/properties");
      vram += prop(mp, "size_in_bytes");
      if (!g.vram_bit_width) g.vram_bit_width = static_cast<uint32_t>(prop(mp, "width"));
    }
    // DRM device attributes (partition modes, VRAM total, NUMA node, RAS counters)
    const std::string dev = root + "/sys/class/drm/renderD" + std::to_string(minor) + "/device";
    std::string s;
    if (read_file(dev + "/mem_info_vram_total", &s)) vram = strtoull(s.c_str(), nullptr, 10);
    g.vram_mb = vram >> 20;
    if (read_file(dev + "/current_compute_partition", &s)) g.compute_partition = s;
    if (read_file(dev + "/current_memory_partition", &s)) g.memory_partition = s;
    if (read_file(dev + "/numa_node", &s)) g.numa_node = std::max<int64_t>(0, atoll(s.c_str()));
    if (read_file(dev + "/product_name", &s) && !s.empty()) g.market_name = s;
    if (read_file(dev + "/vbios_version", &s)) g.vbios = s;
    // board power cap (hwmon of the PCI function, microwatts)
    if (DIR* hw = opendir((dev + "/hwmon").c_str())) {
      while (dirent* e = readdir(hw)) {
        if (strncmp(e->d_name, "hwmon", 5) != 0) continue;
        const std::string hd = dev + "/hwmon/" + e->d_name;
        if (read_file(hd + "/power1_cap", &s) && isdigit((unsigned char)s[0]))
          g.power_cap_w = static_cast<int64_t>((strtoull(s.c_str(), nullptr, 10) + 500000) / 1000000);
        if (read_file(hd + "/power1_cap_default", &s) && isdigit((unsigned char)s[0]))
          g.power_cap_default_w = static_cast<int64_t>((strtoull(s.c_str(), nullptr, 10) + 500000) / 1000000);
        break;
      }
      closedir(hw);
    }
    // PCIe link (the PCI function's attributes, e.g. "32.0 GT/s PCIe" and "16")
    if (read_file(dev + "/current_link_width", &s) && isdigit((unsigned char)s[0])) g.pcie_width = atoll(s.c_str());
    if (read_file(dev + "/max_link_width", &s) && isdigit((unsigned char)s[0])) g.pcie_max_width = atoll(s.c_str());
    if (read_file(dev + "/current_link_speed", &s) && isdigit((unsigned char)s[0])) g.pcie_gts = atof(s.c_str());
    if (read_file(dev + "/max_link_speed", &s) && isdigit((unsigned char)s[0])) g.pcie_max_gts = atof(s.c_str());
    if (g.market_name.empty()) {
      const char* m = market_from_device_id(did);
      g.market_name = m ? m : "";
    }
    DIR* ras = opendir((dev + "/ras").c_str());
    if (ras) {
      // per-block error counters, "ue: N\nce: N[\nde: N]": aca_<block> on parts with the
      // Accelerator Check Architecture (MI300 / MI350 series), <block>_err_count before it;
      // when a driver exposes both, the ACA view is the one counted
      std::vector<std::string> aca, legacy;
      while (dirent* e = readdir(ras)) {
        const std::string n = e->d_name;
        if (n.rfind("aca_", 0) == 0) aca.push_back(n);
        else if (n.size() > 10 && n.compare(n.size() - 10, 10, "_err_count") == 0) legacy.push_back(n);
      }
      closedir(ras);
      for (const auto& n : aca.empty() ? legacy : aca) {
        std::string c;
        if (!read_file(dev + "/ras/" + n, &c)) continue;
        unsigned long long ue = 0, ce = 0;
        const char* q = strstr(c.c_str(), "ue:");
        if (q) ue = strtoull(q + 3, nullptr, 10);
        q = strstr(c.c_str(), "ce:");
        if (q) ce = strtoull(q + 3, nullptr, 10);
        g.has_ecc = true;
        g.ecc_uncorrectable += ue;
        g.ecc_correctable += ce;
      }
      // the driver's bad-page records, one "0x<page> : 0x<size> : R|P|F" line each
      // (R reserved, P pending until the next reset, F could not be reserved)
      FILE* f = fopen((dev + "/ras/gpu_vram_bad_pages").c_str(), "r");
      if (f) {
        g.bad_pages = g.bad_pages_pending = 0;
        char line[256];
        while (fgets(line, sizeof(line), f)) {
          const char* c = strrchr(line, ':');
          if (!c || !strstr(line, "0x")) continue;
          while (*++c == ' ') {
          }
          ++g.bad_pages;
          g.bad_pages_pending += *c == 'P';
        }
        fclose(f);
      }
    }
    // links to other GPU nodes (io_links: direct; p2p_links: indirect peers)
    std::set<size_t> seen;
    for (const char* sub : {"io_links", "p2p_links"}) {
      for (int l : numeric_entries(nd + "/" + sub)) {
        auto lp = read_props(nd + "/" + sub + "/" + std::to_string(l) + "/properties");
        auto it = kfd_to_index.find(static_cast<int>(prop(lp, "node_to", UINT64_MAX)));
        if (it == kfd_to_index.end() || it->second == i || seen.count(it->second)) continue;
        seen.insert(it->second);
        const uint64_t type = prop(lp, "type");
        const bool xgmi = type == 11;
        g.links.push_back({it->second, xgmi ? "XGMI" : (type == 2 ? "PCIE" : "OTHER"), 1, xgmi});
      }
    }
    t.gpus.push_back(std::move(g));
  }
  return t;
}

// The RoCE v2 GID index of a port (ports/<n>/gid_attrs/types/<i> == "RoCE v2" and a
// non-zero ports/<n>/gids/<i>), the first IPv4-mapped one (::ffff:a.b.c.d) if any, else the
// first IPv6 one; -1 when the port has none (InfiniBand, or no address configured).
int roce_v2_gid(const std::string& port_dir) {
  int v6 = -1;
  for (int i : numeric_entries(port_dir + "/gid_attrs/types")) {
    std::string type, gid;
    if (!read_file(port_dir + "/gid_attrs/types/" + std::to_string(i), &type) || type != "RoCE v2") continue;
    if (!read_file(port_dir + "/gids/" + std::to_string(i), &gid)) continue;
    if (gid.find_first_not_of("0:") == std::string::npos) continue;  // an empty slot
    if (gid.rfind("0000:0000:0000:0000:0000:ffff:", 0) == 0) return i;
    if (v6 < 0) v6 = i;
  }
  return v6;
}

// RDMA NICs: /sys/class/infiniband/<dev>/ports/<n>/{state,link_layer,rate}, the netdev
// under <dev>/device/net and the PCI function <dev>/device points at.  Same for both
// collectors (amd_smi does not describe NICs).  Mirrored in ops/topo.py:rdma_nics.
std::vector<NicInfo> collect_nics(const std::string& root) {
  std::vector<NicInfo> out;
  const std::string ib = root + "/sys/class/infiniband";
  DIR* d = opendir(ib.c_str());
  if (!d) return out;
  std::vector<std::string> names;
  while (dirent* e = readdir(d))
    if (e->d_name[0] != '.') names.push_back(e->d_name);
  closedir(d);
  std::sort(names.begin(), names.end());
  for (const auto& n : names) {
    NicInfo nic;
    nic.name = n;
    const std::string dev = ib + "/" + n;
    std::string s;
    for (int port : numeric_entries(dev + "/ports")) {
      const std::string pd = dev + "/ports/" + std::to_string(port);
      if (!read_file(pd + "/state", &s) || s.find("ACTIVE") == std::string::npos) {
        if (nic.link_layer.empty() && read_file(pd + "/link_layer", &s)) nic.link_layer = s;
        continue;
      }
      nic.port = port;
      if (read_file(pd + "/link_layer", &s)) nic.link_layer = s;
      if (read_file(pd + "/rate", &s)) nic.rate_gbps = strtoull(s.c_str(), nullptr, 10);
      nic.gid_index = roce_v2_gid(pd);
      break;
    }
    if (read_file(dev + "/device/numa_node", &s)) nic.numa_node = atoll(s.c_str());
    DIR* nd = opendir((dev + "/device/net").c_str());
    if (nd) {
      std::vector<std::string> nets;
      while (dirent* e = readdir(nd))
        if (e->d_name[0] != '.') nets.push_back(e->d_name);
      closedir(nd);
      std::sort(nets.begin(), nets.end());
      if (!nets.empty()) nic.netdev = nets.front();
    }
    char link[4096];
    const ssize_t k = readlink((dev + "/device").c_str(), link, sizeof(link) - 1);
    if (k > 0) {
      link[k] = 0;
      const char* base = strrchr(link, '/');
      nic.bdf = base ? base + 1 : link;
    }
    out.push_back(std::move(nic));
  }
  return out;
}

// ------------------------------------------------------------ renderers ----
std::string render_json(const Topology& t) {
  std::string o;
  if (t.status != 0) {
    appendf(o, "{\"source\":\"%s\",\"error\":\"%s\",\"gpus\":[]}", t.source.c_str(), esc(t.error).c_str());
    return o;
  }
  appendf(o, "{\"source\":\"%s\",", t.source.c_str());
  if (!t.driver_name.empty())
    appendf(o, "\"driver\":{\"name\":\"%s\",\"version\":\"%s\"},", esc(t.driver_name).c_str(),
            esc(t.driver_version).c_str());
  if (!t.rocm_version.empty()) appendf(o, "\"rocm\":{\"version\":\"%s\"},", esc(t.rocm_version).c_str());
  o += "\"gpus\":[";
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    const GpuInfo& g = t.gpus[i];
    if (i) o += ",";
    appendf(o, "{\"index\":%zu", i);
    if (g.hip_id >= 0) appendf(o, ",\"hip_id\":%" PRId64, g.hip_id);
    if (g.drm_render >= 0) appendf(o, ",\"drm_render\":%" PRId64, g.drm_render);
    if (g.drm_card >= 0) appendf(o, ",\"drm_card\":%" PRId64, g.drm_card);
    if (!g.bdf.empty()) appendf(o, ",\"bdf\":\"%s\"", g.bdf.c_str());
    if (!g.market_name.empty()) appendf(o, ",\"market_name\":\"%s\"", esc(g.market_name).c_str());
    if (!g.vendor_id.empty()) appendf(o, ",\"vendor_id\":\"%s\"", g.vendor_id.c_str());
    if (!g.device_id.empty()) appendf(o, ",\"device_id\":\"%s\"", g.device_id.c_str());
    if (g.rev_id >= 0) appendf(o, ",\"rev_id\":%" PRId64, g.rev_id);
    if (!g.serial.empty()) appendf(o, ",\"asic_serial\":\"%s\"", esc(g.serial).c_str());
    if (!g.vbios.empty()) appendf(o, ",\"vbios_version\":\"%s\"", esc(g.vbios).c_str());
    if (g.power_cap_w > 0) appendf(o, ",\"power_cap_w\":%" PRId64, g.power_cap_w);
    if (g.power_cap_default_w > 0) appendf(o, ",\"power_cap_default_w\":%" PRId64, g.power_cap_default_w);
    if (g.compute_units >= 0) appendf(o, ",\"compute_units\":%" PRId64, g.compute_units);
    if (g.oam_id >= 0) appendf(o, ",\"oam_id\":%" PRId64, g.oam_id);
    if (!g.gfx.empty()) appendf(o, ",\"target_graphics_version\":\"%s\"", g.gfx.c_str());
    if (g.vram_mb) appendf(o, ",\"vram_mb\":%" PRIu64 ",\"vram_bit_width\":%u", g.vram_mb, g.vram_bit_width);
    if (g.numa_node >= 0) appendf(o, ",\"numa_node\":%" PRId64, g.numa_node);
    if (!g.compute_partition.empty())
      appendf(o, ",\"compute_partition\":\"%s\"", esc(g.compute_partition).c_str());
    if (!g.memory_partition.empty()) appendf(o, ",\"memory_partition\":\"%s\"", esc(g.memory_partition).c_str());
    if (g.has_xgmi)
      appendf(o, ",\"xgmi_hive_id\":\"%s\",\"xgmi_node_id\":\"%s\",\"xgmi_lanes\":%u", hex64(g.hive_id).c_str(),
              hex64(g.xgmi_node_id).c_str(), g.xgmi_lanes);
    if (g.has_ecc)
      appendf(o, ",\"ecc_correctable\":%" PRIu64 ",\"ecc_uncorrectable\":%" PRIu64, g.ecc_correctable,
              g.ecc_uncorrectable);
    if (g.bad_pages >= 0)
      appendf(o, ",\"bad_pages\":%" PRId64 ",\"bad_pages_pending\":%" PRId64, g.bad_pages, g.bad_pages_pending);
    if (g.pcie_width >= 0) appendf(o, ",\"pcie_width\":%" PRId64, g.pcie_width);
    if (g.pcie_max_width >= 0) appendf(o, ",\"pcie_max_width\":%" PRId64, g.pcie_max_width);
    if (g.pcie_gts >= 0) appendf(o, ",\"pcie_speed_gts\":%.1f", g.pcie_gts);
    if (g.pcie_max_gts >= 0) appendf(o, ",\"pcie_max_speed_gts\":%.1f", g.pcie_max_gts);
    o += ",\"links\":[";
    for (size_t k = 0; k < g.links.size(); ++k) {
      const Link& l = g.links[k];
      appendf(o, "%s{\"peer\":%zu,\"type\":\"%s\",\"hops\":%" PRIu64 ",\"p2p\":%s}", k ? "," : "", l.peer,
              l.type.c_str(), l.hops, l.p2p ? "true" : "false");
    }
    o += "]}";
  }
  o += "],\"nics\":[";
  for (size_t i = 0; i < t.nics.size(); ++i) {
    const NicInfo& n = t.nics[i];
    appendf(o, "%s{\"name\":\"%s\",\"port\":%d,\"active\":%s,\"link_layer\":\"%s\",\"rate_gbps\":%" PRIu64,
            i ? "," : "", esc(n.name).c_str(), n.port, n.port > 0 ? "true" : "false", esc(n.link_layer).c_str(),
            n.rate_gbps);
    if (!n.netdev.empty()) appendf(o, ",\"netdev\":\"%s\"", esc(n.netdev).c_str());
    if (!n.bdf.empty()) appendf(o, ",\"bdf\":\"%s\"", esc(n.bdf).c_str());
    if (n.gid_index >= 0) appendf(o, ",\"roce_v2_gid_index\":%d", n.gid_index);
    if (n.numa_node >= 0) appendf(o, ",\"numa_node\":%" PRId64, n.numa_node);
    o += "}";
  }
  o += "]}";
  return o;
}

// --- GPU health ------------------------------------------------------------
// Same rules as triton_kubernetes_amd/node/health.py:evaluate (tests compare the two on
// fixture trees).  Judged per physical GPU -- its compute partitions share the PCI function
// and report the same device's RAS counters, so the max over partitions counts once: a GPU
// is unhealthy when its uncorrectable ECC errors exceed max_ue, or its retired VRAM pages
// exceed max_bad (< 0: the amdgpu driver's default bad-page threshold, one page per 100 MiB
// of VRAM rounded up, RAS_BAD_PAGE_COVER in amdgpu_ras.c).
struct PhysGpu {
  std::string bdf;
  bool has_ecc = false;
  uint64_t ue = 0, ce = 0, vram_mb = 0;
  int64_t bad = -1, pending = -1;
  int64_t width = -1, max_width = -1;
};

std::vector<PhysGpu> physical_gpus(const Topology& t) {
  std::vector<PhysGpu> out;
  std::map<std::string, size_t> at;
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    const GpuInfo& g = t.gpus[i];
    const std::string key = g.bdf.empty() ? "#" + std::to_string(i) : g.bdf;
    auto it = at.find(key);
    if (it == at.end()) {
      it = at.emplace(key, out.size()).first;
      out.emplace_back();
      out.back().bdf = g.bdf;
    }
    PhysGpu& p = out[it->second];
    p.has_ecc = p.has_ecc || g.has_ecc;
    p.ue = std::max(p.ue, g.ecc_uncorrectable);
    p.ce = std::max(p.ce, g.ecc_correctable);
    p.vram_mb = std::max(p.vram_mb, g.vram_mb);
    p.bad = std::max(p.bad, g.bad_pages);
    p.pending = std::max(p.pending, g.bad_pages_pending);
    p.width = std::max(p.width, g.pcie_width);
    p.max_width = std::max(p.max_width, g.pcie_max_width);
  }
  return out;
}

int64_t bad_page_limit(const PhysGpu& p, int64_t max_bad) {
  if (max_bad >= 0) return max_bad;
  return p.vram_mb ? static_cast<int64_t>((p.vram_mb + 99) / 100) : -1;  // -1: no limit known
}

struct HealthRow {
  PhysGpu p;
  int64_t limit = -1;
  bool ok = true;
};

struct Verdict {
  std::vector<HealthRow> rows;
  std::vector<std::string> reasons;
  size_t bad_gpus = 0;
};

Verdict judge(const Topology& t, int64_t max_ue, int64_t max_bad) {
  Verdict v;
  const auto phys = physical_gpus(t);
  for (size_t i = 0; i < phys.size(); ++i) {
    HealthRow r;
    r.p = phys[i];
    const PhysGpu& p = r.p;
    r.limit = bad_page_limit(p, max_bad);
    const std::string who = "GPU " + std::to_string(i) + (p.bdf.empty() ? "" : " (" + p.bdf + ")");
    char b[256];
    if (p.has_ecc && static_cast<int64_t>(p.ue) > max_ue) {
      snprintf(b, sizeof(b), "%s: %" PRIu64 " uncorrectable ECC errors (max %" PRId64 ")", who.c_str(), p.ue, max_ue);
      v.reasons.push_back(b);
      r.ok = false;
    }
    if (p.bad >= 0 && r.limit >= 0 && p.bad > r.limit) {
      snprintf(b, sizeof(b), "%s: %" PRId64 " retired VRAM pages (max %" PRId64 ")", who.c_str(), p.bad, r.limit);
      v.reasons.push_back(b);
      r.ok = false;
    }
    if (p.width > 0 && p.max_width > 0 && p.width < p.max_width) {
      snprintf(b, sizeof(b), "%s: PCIe link trained at x%" PRId64 ", the device supports x%" PRId64, who.c_str(),
               p.width, p.max_width);
      v.reasons.push_back(b);
      r.ok = false;
    }
    v.bad_gpus += !r.ok;
    v.rows.push_back(r);
  }
  return v;
}

std::string render_health(const Topology& t, int64_t max_ue, int64_t max_bad, bool labels) {
  const Verdict v = judge(t, max_ue, max_bad);
  const bool healthy = v.reasons.empty();
  if (labels) {
    std::string o = std::string("amd.com/gpu.health=") + (healthy ? "healthy" : "unhealthy") + "\n";
    o += "amd.com/gpu.unhealthy-count=" + std::to_string(v.bad_gpus) + "\n";
    return o;
  }
  std::string gpus;
  for (size_t i = 0; i < v.rows.size(); ++i) {
    const PhysGpu& p = v.rows[i].p;
    appendf(gpus, "%s{\"gpu\":%zu,\"bdf\":\"%s\",\"ok\":%s", i ? "," : "", i, esc(p.bdf).c_str(),
            v.rows[i].ok ? "true" : "false");
    if (p.has_ecc)
      appendf(gpus, ",\"ecc_uncorrectable\":%" PRIu64 ",\"ecc_correctable\":%" PRIu64, p.ue, p.ce);
    if (p.bad >= 0)
      appendf(gpus, ",\"bad_pages\":%" PRId64 ",\"bad_pages_pending\":%" PRId64, p.bad, p.pending);
    if (v.rows[i].limit >= 0) appendf(gpus, ",\"bad_page_limit\":%" PRId64, v.rows[i].limit);
    if (p.width >= 0) appendf(gpus, ",\"pcie_width\":%" PRId64, p.width);
    if (p.max_width >= 0) appendf(gpus, ",\"pcie_max_width\":%" PRId64, p.max_width);
    gpus += "}";
  }
  std::string o;
  appendf(o, "{\"status\":\"%s\",\"max_uncorrectable\":%" PRId64 ",\"max_bad_pages\":", healthy ? "healthy" : "unhealthy",
          max_ue);
  if (max_bad >= 0) appendf(o, "%" PRId64, max_bad);
  else o += "\"auto\"";
  appendf(o, ",\"unhealthy_gpus\":%zu,\"reasons\":[", v.bad_gpus);
  for (size_t i = 0; i < v.reasons.size(); ++i) appendf(o, "%s\"%s\"", i ? "," : "", esc(v.reasons[i]).c_str());
  o += "],\"gpus\":[" + gpus + "]}";
  return o;
}

// --- Prometheus text ----------------------------------------------------------
// The GPU families of triton_kubernetes_amd/node/metrics.py:gpu_metrics -- same names, help
// strings, label order and samples (tests compare the two) -- for node_exporter's textfile
// collector on SSH / Terraform nodes.
// A label value (the exposition format is UTF-8: a byte that does not start a well-formed
// sequence becomes U+FFFD, or node_exporter drops the whole textfile).
std::string prom_esc(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size();) {
    const char c = s[i];
    if (c == '\\') { o += "\\\\"; ++i; }
    else if (c == '\n') { o += "\\n"; ++i; }
    else if (c == '"') { o += "\\\""; ++i; }
    else if (!(static_cast<unsigned char>(c) & 0x80)) { o += c; ++i; }
    else if (const size_t n = utf8_len(s, i)) { o.append(s, i, n); i += n; }
    else { o += "\xEF\xBF\xBD"; ++i; }
  }
  return o;
}

std::string render_prom(const Topology& t, int64_t max_ue, int64_t max_bad, const std::string& node) {
  const Verdict v = judge(t, max_ue, max_bad);
  struct Family {
    const char* name;
    const char* help;
  };
  static const Family fams[] = {
      {"tk_gpu_healthy", "1 if the GPU passes the node's health rules, else 0"},
      {"tk_gpu_ecc_uncorrectable_errors", "Uncorrectable ECC errors, summed over RAS blocks"},
      {"tk_gpu_ecc_correctable_errors", "Correctable ECC errors, summed over RAS blocks"},
      {"tk_gpu_retired_pages", "Retired VRAM pages (driver bad-page records)"},
      {"tk_gpu_retired_pages_pending", "VRAM pages pending retirement"},
      {"tk_gpu_retired_pages_limit", "Retired-page limit of the health rules"},
      {"tk_gpu_pcie_link_width", "Trained PCIe link width (lanes)"},
      {"tk_gpu_pcie_link_max_width", "PCIe link width the device supports (lanes)"},
      {"tk_node_unhealthy_gpus", "Unhealthy physical GPUs on the node"},
  };
  const size_t nfam = sizeof(fams) / sizeof(fams[0]);
  std::vector<std::string> rows(nfam);
  const std::string n = prom_esc(node);
  for (size_t i = 0; i < v.rows.size(); ++i) {
    const HealthRow& r = v.rows[i];
    const PhysGpu& p = r.p;
    // any length: a node name is a host name (<= 253 bytes) but escaping can double it
    const std::string lab = "{node=\"" + n + "\",gpu=\"" + std::to_string(i) + "\",bdf=\"" + prom_esc(p.bdf) + "\"}";
    auto add = [&](size_t f, int64_t val) {
      if (val < 0) return;
      rows[f] += std::string(fams[f].name) + lab + " " + std::to_string(val) + "\n";
    };
    add(0, r.ok ? 1 : 0);
    if (p.has_ecc) {
      add(1, static_cast<int64_t>(p.ue));
      add(2, static_cast<int64_t>(p.ce));
    }
    if (p.bad >= 0) {
      add(3, p.bad);
      add(4, p.pending);
    }
    add(5, r.limit);
    add(6, p.width);
    add(7, p.max_width);
  }
  rows[8] += "tk_node_unhealthy_gpus{node=\"" + n + "\"} " + std::to_string(v.bad_gpus) + "\n";
  std::string o;
  for (size_t f = 0; f < nfam; ++f) {
    if (rows[f].empty()) continue;
    appendf(o, "# HELP %s %s\n# TYPE %s gauge\n", fams[f].name, fams[f].help, fams[f].name);
    o += rows[f];
  }
  return o;
}

// --- node labels -----------------------------------------------------------
// Same rules as triton_kubernetes_amd/node/labels.py:labels_from_topology (the
// Python side is the spec; tests compare the two on fixtures and on the box).

// Kubernetes label value: [A-Za-z0-9._-], at most 63, alphanumeric at both ends.  Any other
// character becomes one '-' (a UTF-8 sequence is one character, as in the Python spec: its
// continuation bytes add nothing); trimmed of '-._' at both ends, and again after the cut.
std::string label_value(const std::string& v) {
  std::string s;
  for (char c : v) {
    const unsigned char u = static_cast<unsigned char>(c);
    if ((u & 0xC0) == 0x80) continue;  // UTF-8 continuation byte
    s += (u < 0x80 && (isalnum(u) || c == '.' || c == '_' || c == '-')) ? c : '-';
  }
  auto trim = [](const std::string& x) {
    size_t b = x.find_first_not_of("-._"), e = x.find_last_not_of("-._");
    return b == std::string::npos ? std::string() : x.substr(b, e - b + 1);
  };
  s = trim(s);
  return s.size() > 63 ? trim(s.substr(0, 63)) : s;
}

// PCI device id -> product, for parts whose market name is not the SKU name
// (amd_smi reports an MI355X as "AMD Instinct MI355 OAM").
const char* product_from_device_id(const std::string& id) {
  static const std::map<std::string, const char*> m = {
      {"0x75a3", "MI355X"}, {"0x75a0", "MI350X"}, {"0x74a5", "MI325X"}, {"0x74a1", "MI300X"}};
  auto it = m.find(id);
  return it == m.end() ? nullptr : it->second;
}

std::string product_name(const GpuInfo& g) {
  if (const char* p = product_from_device_id(g.device_id)) return p;
  const std::string& m = g.market_name;
  for (size_t i = 0; i + 4 < m.size(); ++i) {
    if (m[i] == 'M' && m[i + 1] == 'I' && isdigit((unsigned char)m[i + 2]) && isdigit((unsigned char)m[i + 3]) &&
        isdigit((unsigned char)m[i + 4])) {
      size_t e = i + 5;
      while (e < m.size() && m[e] >= 'A' && m[e] <= 'Z') ++e;
      return m.substr(i, e - i);
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
    if (!t.rocm_version.empty()) L["amd.com/rocm.version"] = label_value(t.rocm_version);
    // physical GPUs = distinct PCI functions (a GPU's compute partitions share one);
    // = node/labels.py and node/partition.py:physical_count
    std::set<std::string> bdfs;
    for (size_t i = 0; i < gs.size(); ++i) bdfs.insert(gs[i].bdf.empty() ? "#" + std::to_string(i) : gs[i].bdf);
    const size_t physical = bdfs.size();
    L["amd.com/gpu.count"] = std::to_string(physical);
    L["amd.com/gpu.logical-count"] = std::to_string(gs.size());
    if (gs.size() % physical == 0) L["amd.com/gpu.partitions-per-gpu"] = std::to_string(gs.size() / physical);
    std::set<std::string> names, dev_ids, targets, cparts, mparts, hives, vbioses;
    int64_t min_cap = INT64_MAX;
    int64_t min_cu = INT64_MAX;
    uint64_t min_vram = UINT64_MAX;
    size_t min_xgmi = SIZE_MAX;
    for (const auto& g : gs) {
      if (!g.market_name.empty() || product_from_device_id(g.device_id)) names.insert(product_name(g));
      if (!g.device_id.empty() && g.device_id != "0x0") dev_ids.insert(g.device_id);
      if (g.compute_units > 0) min_cu = std::min(min_cu, g.compute_units);
      if (g.vram_mb) min_vram = std::min(min_vram, g.vram_mb);
      if (!g.gfx.empty()) targets.insert(g.gfx);
      if (!g.compute_partition.empty()) cparts.insert(lower(g.compute_partition));
      if (!g.memory_partition.empty()) mparts.insert(lower(g.memory_partition));
      if (g.has_xgmi && g.hive_id) hives.insert(hex64(g.hive_id));
      if (!g.vbios.empty()) vbioses.insert(g.vbios);
      if (g.power_cap_w > 0) min_cap = std::min(min_cap, g.power_cap_w);
      std::set<size_t> peers;
      for (const auto& l : g.links)
        if (l.type == "XGMI") peers.insert(l.peer);
      min_xgmi = std::min(min_xgmi, peers.size());
    }
    if (names.size() == 1) {
      const std::string n = *names.begin();
      L["amd.com/gpu.product-name"] = label_value(n);
      if (n.rfind("MI", 0) == 0) L["amd.com/gpu.family"] = "AI";
    }
    if (dev_ids.size() == 1) L["amd.com/gpu.device-id"] = label_value(*dev_ids.begin());
    if (min_cu != INT64_MAX) L["amd.com/gpu.cu-count"] = std::to_string(min_cu);
    // nearest GiB: the 294896 MiB an MI355X reports reads as 288G
    if (min_vram != UINT64_MAX) L["amd.com/gpu.vram"] = std::to_string((min_vram + 512) / 1024) + "G";
    if (targets.size() == 1) L["amd.com/gpu.target"] = label_value(*targets.begin());
    if (cparts.size() == 1) L["amd.com/gpu.compute-partition"] = label_value(*cparts.begin());
    if (mparts.size() == 1) L["amd.com/gpu.memory-partition"] = label_value(*mparts.begin());
    if (hives.size() == 1) L["amd.com/xgmi.hive-id"] = label_value(*hives.begin());
    // one VBIOS on every GPU, or "mixed" (a node whose GPUs were flashed apart)
    if (!vbioses.empty()) L["amd.com/gpu.vbios"] = vbioses.size() == 1 ? label_value(*vbioses.begin()) : "mixed";
    if (min_cap != INT64_MAX) L["amd.com/gpu.power-cap"] = std::to_string(min_cap);  // watts, lowest GPU
    L["amd.com/xgmi.links-per-gpu"] = std::to_string(min_xgmi);
    // a compute partition is not a whole GPU with its own xGMI links: SPX only
    const bool whole = (cparts.empty() || (cparts.size() == 1 && *cparts.begin() == "spx")) && physical == gs.size();
    L["amd.com/xgmi.fully-connected"] = (whole && gs.size() > 1 && min_xgmi == gs.size() - 1) ? "true" : "false";
    // RAS counters per physical GPU (its partitions report the same device's counters)
    uint64_t ecc = 0;
    int64_t bad = 0, width = INT64_MAX;
    bool bad_known = false;
    for (const auto& p : physical_gpus(t)) {
      ecc += p.ue;
      if (p.bad >= 0) bad += p.bad, bad_known = true;
      if (p.width > 0) width = std::min(width, p.width);
    }
    L["amd.com/gpu.ecc-uncorrectable"] = std::to_string(ecc);
    if (bad_known) L["amd.com/gpu.bad-pages"] = std::to_string(bad);
    if (width != INT64_MAX) L["amd.com/gpu.pcie-width"] = std::to_string(width);  // narrowest GPU link
  }
  // inter-node fabric: active RDMA ports
  size_t active = 0;
  std::set<std::string> layers;
  uint64_t min_rate = UINT64_MAX;
  for (const auto& n : t.nics) {
    if (n.port <= 0) continue;
    ++active;
    if (!n.link_layer.empty()) layers.insert(lower(n.link_layer));
    if (n.rate_gbps) min_rate = std::min(min_rate, n.rate_gbps);
  }
  L["amd.com/rdma.count"] = std::to_string(active);
  if (layers.size() == 1) L["amd.com/rdma.link-layer"] = label_value(*layers.begin());
  if (min_rate != UINT64_MAX) L["amd.com/rdma.rate-gbps"] = std::to_string(min_rate);
  std::string o;
  for (const auto& kv : L) o += kv.first + "=" + kv.second + "\n";
  return o;
}

// RCCL/NCCL settings for the inter-node fabric, one KEY="value" line each (sourced after
// the static /etc/rccl/rccl.env defaults; explicit per-node overrides come later and win).
// Mirrored in parallel/rccl_env.py:site_env_from_topology.
// NCCL_IB_GID_INDEX is set only when every active RoCE port has its RoCE v2 GID at the
// same index; otherwise RCCL picks one per port itself (RoCE v2, IPv4 first, by default).
// A plain device name (sysfs: mlx5_0, bnxt_re1, irdma0, ...): anything else is left to RCCL's
// own detection rather than written into a file the node's services load as root
// (parallel/rccl_env.py:site_env_from_topology applies the same rule).
static bool plain_device_name(const std::string& s) {
  if (s.empty() || s.size() > 64) return false;
  for (char c : s)
    if (!(std::isalnum(static_cast<unsigned char>(c)) || c == '_' || c == '.' || c == '-')) return false;
  return true;
}

std::string render_rccl_env(const Topology& t) {
  std::string hca;
  std::set<int> gids;
  for (const auto& n : t.nics) {
    if (n.port <= 0 || !plain_device_name(n.name)) continue;
    hca += (hca.empty() ? "" : ",") + n.name + ":" + std::to_string(n.port);
    if (lower(n.link_layer) == "ethernet") gids.insert(n.gid_index);
  }
  std::string o;
  if (hca.empty()) return o;
  o += "NCCL_IB_HCA=\"=" + hca + "\"\n";  // leading '=': exact device names, not prefixes
  if (gids.size() == 1 && *gids.begin() >= 0) o += "NCCL_IB_GID_INDEX=\"" + std::to_string(*gids.begin()) + "\"\n";
  return o;
}

Topology collect_gpus(const std::string& src, const std::string& r) {
  if (src == "sysfs") return collect_sysfs(r);
  if (src == "amdsmi") return collect_amdsmi();
  Topology t = collect_amdsmi();
  if (t.status != 0 || t.gpus.empty()) {
    Topology s = collect_sysfs(r);
    if (s.status == 0) return s;
  }
  return t;
}

Topology collect(const char* source, const char* root) {
  const std::string r = (root && *root) ? root : "";
  Topology t = collect_gpus(source ? source : "auto", r);
  t.nics = collect_nics(r);
  // ROCm userspace version: the live system's ROCM_PATH, a fixture tree's /opt/rocm
  const char* rp = getenv("ROCM_PATH");
  const std::string info = r.empty() ? std::string(rp && *rp ? rp : "/opt/rocm") + "/.info/version"
                                     : r + "/opt/rocm/.info/version";
  std::string v;
  if (read_file(info, &v)) t.rocm_version = v;
  return t;
}

int copy_out(const std::string& j, char* buf, size_t len) {
  if (j.size() + 1 > len) return -static_cast<int>(j.size() + 1);
  memcpy(buf, j.c_str(), j.size() + 1);
  return 0;
}

}  // namespace

// Writes the JSON document into buf (NUL-terminated).  source: "amdsmi",
// "sysfs" or "auto" (amd_smi, sysfs when it fails); root prefixes the sysfs
// paths (fixture trees in tests; NULL/"" for the live system).  Returns 0 on
// success, the collector status on failure (buf still holds a JSON error
// document), or -(required size) if buf is too small.
extern "C" int tkt_topology_json_src(const char* source, const char* root, char* buf, size_t len) {
  const Topology t = collect(source, root);
  const int rc = copy_out(render_json(t), buf, len);
  return rc < 0 ? rc : t.status;
}

// Same contract; the payload is the `key=value\n` node label set.
extern "C" int tkt_topology_labels_src(const char* source, const char* root, char* buf, size_t len) {
  const Topology t = collect(source, root);
  const int rc = copy_out(t.status == 0 ? render_labels(t) : std::string(), buf, len);
  return rc < 0 ? rc : t.status;
}

// Same contract; the payload is the inter-node RCCL environment (KEY="value" lines).
extern "C" int tkt_rccl_env_src(const char* root, char* buf, size_t len) {
  Topology t;
  t.nics = collect_nics((root && *root) ? root : "");
  return copy_out(render_rccl_env(t), buf, len);
}

// Same contract; the payload is the health verdict JSON (labels: the health label set).
extern "C" int tkt_health_src(const char* source, const char* root, long long max_ue, long long max_bad, int labels,
                              char* buf, size_t len) {
  const Topology t = collect(source, root);
  const int rc = copy_out(t.status == 0 ? render_health(t, max_ue, max_bad, labels != 0) : std::string(), buf, len);
  return rc < 0 ? rc : t.status;
}

extern "C" int tkt_topology_json(char* buf, size_t len) { return tkt_topology_json_src("amdsmi", "", buf, len); }

extern "C" int tkt_topology_labels(char* buf, size_t len) { return tkt_topology_labels_src("amdsmi", "", buf, len); }

#ifdef TK_TOPO_MAIN
// A whole decimal int64 ("12", "-1"); "", "abc", "3x" and out-of-range values are not.
static bool whole_int(const char* s, long long* out) {
  if (!*s) return false;
  char* end = nullptr;
  errno = 0;
  const long long v = strtoll(s, &end, 10);
  if (*end || errno == ERANGE || isspace((unsigned char)*s)) return false;
  *out = v;
  return true;
}

// amdgpu-topo-labeller [--labels|--rccl-env|--health|--prom] [--source auto|amdsmi|sysfs] [--sysfs-root DIR]
//                      [--max-uncorrectable N] [--max-bad-pages N|auto] [--node NAME]
//   default: topology JSON on stdout; --labels: one `amd.com/...=value` per line;
//   --rccl-env: the inter-node RCCL settings for the node's active RDMA ports;
//   --health: the GPU health verdict (JSON; with --labels the health labels), exit 3 when
//   a GPU is unhealthy;
//   --prom: the GPU health families as Prometheus text (node_exporter textfile collector;
//   label node=NAME, default the host name), exit 0 whatever the verdict
int main(int argc, char** argv) {
  bool labels = false, rccl_env = false, health = false, prom = false;
  std::string node;
  long long max_ue = 0, max_bad = -1;
  const char* source = "auto";
  const char* root = "";
  for (int i = 1; i < argc; ++i) {
    if (strcmp(argv[i], "--labels") == 0) {
      labels = true;
    } else if (strcmp(argv[i], "--rccl-env") == 0) {
      rccl_env = true;
    } else if (strcmp(argv[i], "--health") == 0) {
      health = true;
    } else if (strcmp(argv[i], "--prom") == 0) {
      prom = true;
    } else if (strcmp(argv[i], "--node") == 0 && i + 1 < argc) {
      node = argv[++i];
    } else if (strcmp(argv[i], "--max-uncorrectable") == 0 && i + 1 < argc && whole_int(argv[i + 1], &max_ue)) {
      ++i;
    } else if (strcmp(argv[i], "--max-bad-pages") == 0 && i + 1 < argc &&
               (strcmp(argv[i + 1], "auto") == 0 || whole_int(argv[i + 1], &max_bad))) {
      if (strcmp(argv[++i], "auto") == 0) max_bad = -1;
    } else if (strcmp(argv[i], "--source") == 0 && i + 1 < argc) {
      source = argv[++i];
    } else if (strcmp(argv[i], "--sysfs-root") == 0 && i + 1 < argc) {
      root = argv[++i];
    } else {
      fprintf(stderr,
              "usage: %s [--labels|--rccl-env|--health|--prom] [--source auto|amdsmi|sysfs] [--sysfs-root DIR] "
              "[--max-uncorrectable N] [--max-bad-pages N|auto] [--node NAME]\n",
              argv[0]);
      return 64;
    }
  }
  if (strcmp(source, "auto") != 0 && strcmp(source, "amdsmi") != 0 && strcmp(source, "sysfs") != 0) {
    fprintf(stderr, "unknown --source '%s'\n", source);
    return 64;
  }
  if (rccl_env) {  // NIC-only: no GPU collector runs
    Topology t;
    t.nics = collect_nics(root);
    fputs(render_rccl_env(t).c_str(), stdout);
    return 0;
  }
  const Topology t = collect(source, root);
  if (prom) {
    if (t.status != 0) {
      fprintf(stderr, "amdgpu-topo-labeller: %s\n", t.error.c_str());
      return 2;
    }
    if (node.empty()) {
      char host[256] = {0};
      if (gethostname(host, sizeof(host) - 1) == 0) node = host;
    }
    fputs(render_prom(t, max_ue, max_bad, node).c_str(), stdout);
    return 0;
  }
  if (health) {
    if (t.status != 0) {
      fprintf(stderr, "amdgpu-topo-labeller: %s\n", t.error.c_str());
      return 2;
    }
    const std::string verdict = render_health(t, max_ue, max_bad, false);
    fputs(labels ? render_health(t, max_ue, max_bad, true).c_str() : (verdict + "\n").c_str(), stdout);
    return verdict.find("\"status\":\"healthy\"") != std::string::npos ? 0 : 3;
  }
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
