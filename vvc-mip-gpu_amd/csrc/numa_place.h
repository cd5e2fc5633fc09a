// numa_place.h -- NUMA placement of an engine's host side (round 6).
//
// On a multi-socket host each GPU hangs off one socket's PCIe root; page-locked buffers on
// the other socket cost every DMA a trip over the inter-socket link, and copy threads there
// read and write remote DRAM.  Eight GPUs fed with full cost tables move ~0.9 TB/s of host
// DRAM traffic, so the engine keeps its host side on its GPU's node:
//   * the node: /sys/bus/pci/devices/<PCI bus id>/numa_node (the bus id from
//     hipDeviceGetPCIBusId; -1 or a one-node host: no placement);
//   * its CPUs: /sys/devices/system/node/node<N>/cpulist, intersected with the CPUs the
//     process may run on (containers);
//   * page-locked allocations (bounce ring, mip_host_alloc_near) are made under a
//     "preferred node" memory policy with hipHostMallocNumaUser, so the pages come from that
//     node;
//   * the engine's host threads (bounce-ring copy pool and completion thread, the merge
//     flusher) and, on request (mip_bind_thread), the caller's thread run on its CPUs.
// No HIP dependency: tests/cpp/test_numa_place.cpp runs it over a fake sysfs tree
// (MIPGPU_SYSFS_ROOT).
#pragma once
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace mipgpu {

struct NumaPlace {
  int node = -1;          // -1: unknown, or nothing to place (one node)
  std::vector<int> cpus;  // the node's CPUs this process may use
  bool active() const { return node >= 0 && !cpus.empty(); }
};

inline std::string sysfs_root() {
  const char *r = getenv("MIPGPU_SYSFS_ROOT");  // tests: a fake sysfs tree
  return r && *r ? r : "/sys";
}

inline bool read_text(const std::string &path, std::string *out) {
  FILE *f = fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096];
  const size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  *out = buf;
  while (!out->empty() && isspace((unsigned char)out->back())) out->pop_back();
  return true;
}

// Linux cpulist / nodelist syntax: "0-15,32-47", "3", "" -> the listed numbers.
inline std::vector<int> parse_cpulist(const std::string &s) {
  std::vector<int> v;
  size_t i = 0;
  while (i < s.size()) {
    char *end = nullptr;
    const long a = strtol(s.c_str() + i, &end, 10);
    if (end == s.c_str() + i) break;
    long b = a;
    i = end - s.c_str();
    if (i < s.size() && s[i] == '-') {
      b = strtol(s.c_str() + i + 1, &end, 10);
      i = end - s.c_str();
    }
    for (long c = a; c <= b && c - a < 65536; c++) v.push_back((int)c);
    while (i < s.size() && (s[i] == ',' || isspace((unsigned char)s[i]))) i++;
  }
  return v;
}

inline std::vector<int> allowed_cpus() {
  std::vector<int> v;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof set, &set) != 0) return v;
  for (int c = 0; c < CPU_SETSIZE; c++)
    if (CPU_ISSET(c, &set)) v.push_back(c);
  return v;
}

// NUMA placement of the PCI device `busid` ("0000:C1:00.0", any case).
inline NumaPlace numa_place_of_pci(std::string busid, const std::string &root = sysfs_root()) {
  NumaPlace p;
  for (char &c : busid) c = (char)tolower((unsigned char)c);
  std::string t;
  if (!read_text(root + "/bus/pci/devices/" + busid + "/numa_node", &t) || t.empty()) return p;
  const int node = atoi(t.c_str());
  if (node < 0) return p;
  if (read_text(root + "/devices/system/node/online", &t) && parse_cpulist(t).size() < 2) return p;  // one node
  if (!read_text(root + "/devices/system/node/node" + std::to_string(node) + "/cpulist", &t)) return p;
  const std::vector<int> node_cpus = parse_cpulist(t), ok = allowed_cpus();
  for (int c : node_cpus)
    for (int a : ok)
      if (a == c) {
        p.cpus.push_back(c);
        break;
      }
  if (!p.cpus.empty()) p.node = node;
  return p;
}

// Run the calling thread on the place's CPUs (false: nothing to do or refused).
inline bool bind_current_thread(const NumaPlace &p) {
  if (!p.active()) return false;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : p.cpus)
    if (c < CPU_SETSIZE) CPU_SET(c, &set);
  return sched_setaffinity(0, sizeof set, &set) == 0;
}

// The calling thread's memory policy is "prefer the place's node" for the scope (page-locked
// allocations made with hipHostMallocNumaUser follow it), then the previous policy again.
class ScopedNodePolicy {
 public:
  static constexpr int kMpolDefault = 0, kMpolPreferred = 1;
  static constexpr unsigned long kMaxNode = 1024;
  explicit ScopedNodePolicy(const NumaPlace &p) {
    if (!p.active() || p.node >= (int)kMaxNode) return;
    if (syscall(SYS_get_mempolicy, &old_mode_, old_mask_, kMaxNode, nullptr, 0UL) != 0) return;
    unsigned long mask[kMaxNode / (8 * sizeof(unsigned long))] = {};
    mask[p.node / (8 * sizeof(unsigned long))] = 1UL << (p.node % (8 * sizeof(unsigned long)));
    set_ = syscall(SYS_set_mempolicy, kMpolPreferred, mask, kMaxNode) == 0;
  }
  ~ScopedNodePolicy() {
    if (set_) (void)syscall(SYS_set_mempolicy, old_mode_, old_mode_ == kMpolDefault ? nullptr : old_mask_, kMaxNode);
  }
  bool applied() const { return set_; }
  ScopedNodePolicy(const ScopedNodePolicy &) = delete;
  ScopedNodePolicy &operator=(const ScopedNodePolicy &) = delete;

 private:
  int old_mode_ = kMpolDefault;
  unsigned long old_mask_[kMaxNode / (8 * sizeof(unsigned long))] = {};
  bool set_ = false;
};

}  // namespace mipgpu
