// devmem.cpp — process-wide caching device allocator (devmem.h).
#include "devmem.h"

#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace vts {
namespace {

constexpr size_t kCacheMin = 64 << 10;  // smaller blocks go straight back to HIP
constexpr size_t kRound = 2 << 20;      // cached sizes rounded up to 2 MiB

struct Block {
  void *p;
  size_t n;
  int dev;
};
std::mutex g_mu;
std::unordered_map<void *, Block> g_live;          // allocations handed out (cacheable sizes)
std::map<int, std::multimap<size_t, void *>> g_free;  // per device: size -> block
std::map<int, size_t> g_cached;

void release_device_locked(int dev) {
  auto &fm = g_free[dev];
  for (auto &kv : fm) (void)hipFree(kv.second);
  fm.clear();
  g_cached[dev] = 0;
}

}  // namespace

hipError_t dmalloc_raw(void **p, size_t n) {
  *p = nullptr;
  if (n < kCacheMin) return hipMalloc(p, n ? n : 1);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const size_t want = (n + kRound - 1) / kRound * kRound;
  std::lock_guard<std::mutex> lk(g_mu);
  auto &fm = g_free[dev];
  auto it = fm.lower_bound(want);
  if (it != fm.end() && it->first <= 2 * want) {
    *p = it->second;
    g_live[*p] = Block{*p, it->first, dev};
    g_cached[dev] -= it->first;
    fm.erase(it);
    return hipSuccess;
  }
  e = hipMalloc(p, want);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    release_device_locked(dev);
    e = hipMalloc(p, want);
    if (e != hipSuccess) return e;
  }
  g_live[*p] = Block{*p, want, dev};
  return hipSuccess;
}

void dfree(void *p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_live.find(p);
  if (it == g_live.end()) {
    (void)hipFree(p);
    return;
  }
  const Block b = it->second;
  g_live.erase(it);
  g_free[b.dev].emplace(b.n, b.p);
  g_cached[b.dev] += b.n;
}

size_t dmem_cached(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_cached.find(device);
  return it == g_cached.end() ? 0 : it->second;
}

hipError_t dmem_free(size_t *free_b, size_t *total_b) {
  const hipError_t e = hipMemGetInfo(free_b, total_b);
  if (e != hipSuccess) return e;
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) *free_b += dmem_cached(dev);
  return hipSuccess;
}

}  // namespace vts

extern "C" int vts_empty_cache(int device) {
  std::lock_guard<std::mutex> lk(vts::g_mu);
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return vts::fail(VTS_E_HIP, "hipGetDevice");
  if (hipSetDevice(device) != hipSuccess) return vts::fail(VTS_E_NODEVICE, "device %d", device);
  vts::release_device_locked(device);
  (void)hipSetDevice(cur);
  return VTS_OK;
}
