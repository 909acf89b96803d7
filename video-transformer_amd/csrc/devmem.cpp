// devmem.cpp — process-wide caching device allocator (devmem.h).
//
// Large requests (>= kVmmMin) are built from physical chunks of kChunk bytes
// (hipMemCreate) mapped back to back into a fresh virtual range
// (hipMemAddressReserve / hipMemMap / hipMemSetAccess); freeing unmaps the
// range and keeps the chunks.  Any later request, of any size or shape, maps
// whichever chunks are idle: no fragmentation, and HBM never goes back to the
// driver between sessions — memory handed back is cleared by the driver
// before it is handed out again (~45 GB/s: 2.8 s of a 2-h video's open in the
// bench after other sessions' buffers), chunks re-mapped are not (16 GB in
// 3.6 ms, tools/micro/vmm_probe.hip; copy bandwidth equal to hipMalloc's).
// Where VMM is unavailable, large requests take the segment path below.
//
// Smaller requests: segments are hipMalloc'd blocks; a segment is cut into
// ranges.  A request takes the smallest free range that holds it (any
// segment) when that range is a close fit or the request is large (devmem.h),
// splitting off the rest as a new free range; a released range merges with
// its free neighbours of the same segment.  Segments go back to HIP only when
// wholly free: on a failed allocation (as much as it needs) or
// vts_empty_cache().
#include "devmem.h"

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "common.h"

namespace vts {
namespace {

constexpr size_t kCacheMin = 64 << 10;  // smaller blocks go straight to / back to HIP
constexpr size_t kRound = 2 << 20;      // ranges are multiples of 2 MiB (so they stay 2 MiB aligned)
constexpr size_t kCarveMin = size_t(256) << 20;  // requests this large may be cut from any larger free range
constexpr size_t kVmmMin = size_t(256) << 20;    // requests this large are mapped physical chunks
constexpr size_t kChunk = size_t(128) << 20;     // physical chunk size of the mapped requests

struct Range {
  size_t n;
  char *base;  // the segment's hipMalloc pointer
  bool free;
};
struct Mapped {
  size_t n;                                        // reserved and mapped bytes (chunks x kChunk)
  std::vector<hipMemGenericAllocationHandle_t> h;  // the chunks, in address order
};
struct Device {
  std::map<char *, Range> ranges;             // every range of every segment, by address
  std::multimap<size_t, char *> free_by_size;  // the free ranges
  std::map<char *, size_t> segments;          // base -> bytes
  std::map<char *, Mapped> mapped;            // mapped requests, by address
  std::vector<hipMemGenericAllocationHandle_t> idle_chunks;
  int vmm = -1;                               // VMM usable (-1: not probed yet)
  size_t cached = 0;                          // bytes in free ranges and idle chunks
  size_t in_use = 0;                          // bytes handed out (ranges not free, mapped requests)
};
std::mutex g_mu;
std::map<int, Device> g_dev;

// VTS_DEVMEM_LOG=1: every fresh hipMalloc and every release of cached
// segments to HIP on stderr, with its time (measurement)
bool log_on() {
  static const bool on = [] {
    const char *e = std::getenv("VTS_DEVMEM_LOG");
    return e && std::atoi(e) != 0;
  }();
  return on;
}
double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void free_list_erase(Device &d, size_t n, char *p) {
  auto r = d.free_by_size.equal_range(n);
  for (auto it = r.first; it != r.second; ++it)
    if (it->second == p) {
      d.free_by_size.erase(it);
      return;
    }
}

// hand wholly free segments back to HIP, smallest first, until `want` bytes
// went back (all of them for want = SIZE_MAX): HBM that goes back is cleared
// by the driver when it is handed out again (~45 GB/s measured), so a miss
// gives back no more than it needs
void release_free_segments_locked(Device &d, size_t want = SIZE_MAX) {
  const auto t0 = std::chrono::steady_clock::now();
  size_t nseg = 0, bytes = 0;
  std::vector<std::pair<size_t, char *>> idle;  // wholly free segments by size
  for (const auto &sg : d.segments) {
    auto r = d.ranges.find(sg.first);
    if (r != d.ranges.end() && r->second.free && r->second.n == sg.second) idle.emplace_back(sg.second, sg.first);
  }
  std::sort(idle.begin(), idle.end());
  for (const auto &sg : idle) {
    if (bytes >= want) break;
    auto r = d.ranges.find(sg.second);
    free_list_erase(d, r->second.n, r->first);
    d.cached -= r->second.n;
    d.ranges.erase(r);
    (void)hipFree(sg.second);
    d.segments.erase(sg.second);
    ++nseg;
    bytes += sg.first;
  }
  if (log_on())
    std::fprintf(stderr, "[devmem] released %zu segments, %.2f GB to HIP in %.1f ms (cached %.2f GB, in use %.2f GB)\n",
                 nseg, bytes / 1e9, ms_since(t0), d.cached / 1e9, d.in_use / 1e9);
}

// take `want` bytes from the front of free range p (splitting off the rest)
void *take_locked(Device &d, char *p, size_t want) {
  Range &r = d.ranges[p];
  free_list_erase(d, r.n, p);
  d.cached -= r.n;
  if (r.n > want) {
    char *rest = p + want;
    d.ranges[rest] = Range{r.n - want, r.base, true};
    d.free_by_size.emplace(r.n - want, rest);
    d.cached += r.n - want;
    r.n = want;
  }
  r.free = false;
  d.in_use += want;
  return p;
}

// hand idle physical chunks back to HIP until `want` bytes went back
void release_idle_chunks_locked(Device &d, size_t want = SIZE_MAX) {
  size_t bytes = 0;
  while (!d.idle_chunks.empty() && bytes < want) {
    (void)hipMemRelease(d.idle_chunks.back());
    d.idle_chunks.pop_back();
    d.cached -= kChunk;
    bytes += kChunk;
  }
}

bool vmm_usable(Device &d, int dev) {
  if (d.vmm < 0) {
    int v = 0;
    d.vmm = (hipDeviceGetAttribute(&v, hipDeviceAttributeVirtualMemoryManagementSupported, dev) == hipSuccess && v) ? 1 : 0;
    const char *e = std::getenv("VTS_DEVMEM_VMM");
    if (e && std::atoi(e) == 0) d.vmm = 0;
    (void)hipGetLastError();
  }
  return d.vmm == 1;
}

hipMemAllocationProp chunk_prop(int dev) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  return prop;
}

// a large request: idle chunks first, new ones for the rest (idle hipMalloc
// segments go back first if HIP has no room), mapped back to back
hipError_t vmm_alloc_locked(Device &d, int dev, void **p, size_t n) {
  const auto t0 = std::chrono::steady_clock::now();
  const size_t k = (n + kChunk - 1) / kChunk, bytes = k * kChunk;
  std::vector<hipMemGenericAllocationHandle_t> h;
  h.reserve(k);
  size_t fresh = 0;
  const hipMemAllocationProp prop = chunk_prop(dev);
  auto undo = [&](hipError_t e) {
    for (auto x : h) d.idle_chunks.push_back(x);
    d.cached += h.size() * kChunk;
    return e;
  };
  while (h.size() < k) {
    if (!d.idle_chunks.empty()) {
      h.push_back(d.idle_chunks.back());
      d.idle_chunks.pop_back();
      d.cached -= kChunk;
      continue;
    }
    hipMemGenericAllocationHandle_t x{};
    hipError_t e = hipMemCreate(&x, kChunk, &prop, 0);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      release_free_segments_locked(d, (k - h.size()) * kChunk);
      e = hipMemCreate(&x, kChunk, &prop, 0);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        return undo(e);
      }
    }
    h.push_back(x);
    ++fresh;
  }
  void *va = nullptr;
  hipError_t e = hipMemAddressReserve(&va, bytes, 0, nullptr, 0);
  if (e != hipSuccess) return undo(e);
  size_t mapped = 0;
  for (; mapped < k; ++mapped) {
    e = hipMemMap(static_cast<char *>(va) + mapped * kChunk, kChunk, 0, h[mapped], 0);
    if (e != hipSuccess) break;
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if (e == hipSuccess) e = hipMemSetAccess(va, bytes, &acc, 1);
  if (e != hipSuccess) {
    if (mapped) (void)hipMemUnmap(va, mapped * kChunk);
    (void)hipMemAddressFree(va, bytes);
    return undo(e);
  }
  d.mapped[static_cast<char *>(va)] = Mapped{bytes, std::move(h)};
  d.in_use += bytes;
  *p = va;
  if (log_on())
    std::fprintf(stderr, "[devmem] mapped %.3f GB (%zu new chunks) in %.1f ms (cached %.2f GB, in use %.2f GB)\n",
                 bytes / 1e9, fresh, ms_since(t0), d.cached / 1e9, d.in_use / 1e9);
  return hipSuccess;
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
  Device &d = g_dev[dev];
  if (n >= kVmmMin && vmm_usable(d, dev)) return vmm_alloc_locked(d, dev, p, n);
  auto it = d.free_by_size.lower_bound(want);
  // a close fit, or a large request (a fresh hipMalloc of recycled memory
  // waits for the driver's clear): take it from the cache
  if (it != d.free_by_size.end() && (it->first <= 2 * want || it->first <= want + (64u << 20) || want >= kCarveMin)) {
    *p = take_locked(d, it->second, want);
    return hipSuccess;
  }
  const auto t0 = std::chrono::steady_clock::now();
  e = hipMalloc(p, want);
  if (log_on())
    std::fprintf(stderr, "[devmem] hipMalloc %.3f GB: %s in %.1f ms (cached %.2f GB, in use %.2f GB)\n", want / 1e9,
                 e == hipSuccess ? "ok" : "failed", ms_since(t0), d.cached / 1e9, d.in_use / 1e9);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    if (it != d.free_by_size.end()) {  // no fresh memory: carve the large range after all
      *p = take_locked(d, it->second, want);
      return hipSuccess;
    }
    // give back what the request needs (smallest idle segments first), more
    // only if that was not enough
    release_free_segments_locked(d, want);
    e = hipMalloc(p, want);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      release_free_segments_locked(d);
      release_idle_chunks_locked(d, want);
      e = hipMalloc(p, want);
      if (e != hipSuccess) return e;
    }
  }
  char *b = static_cast<char *>(*p);
  d.segments[b] = want;
  d.ranges[b] = Range{want, b, false};
  d.in_use += want;
  return hipSuccess;
}

void dfree(void *p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_mu);
  int dev = 0;
  (void)hipGetDevice(&dev);
  // a mapped request: unmap it, keep its chunks
  for (auto &kv : g_dev) {
    auto m = kv.second.mapped.find(static_cast<char *>(p));
    if (m == kv.second.mapped.end()) continue;
    Device &dd = kv.second;
    (void)hipMemUnmap(p, m->second.n);
    (void)hipMemAddressFree(p, m->second.n);
    for (auto x : m->second.h) dd.idle_chunks.push_back(x);
    dd.in_use -= m->second.n;
    dd.cached += m->second.n;
    dd.mapped.erase(m);
    return;
  }
  // the range may belong to any device's segments: look in the current one first
  Device *d = nullptr;
  std::map<char *, Range>::iterator it;
  auto look = [&](Device &dd) {
    auto f = dd.ranges.find(static_cast<char *>(p));
    if (f == dd.ranges.end() || f->second.free) return false;
    d = &dd;
    it = f;
    return true;
  };
  if (!look(g_dev[dev]))
    for (auto &kv : g_dev)
      if (look(kv.second)) break;
  if (!d) {
    (void)hipFree(p);
    return;
  }
  char *q = it->first;
  Range r = it->second;
  r.free = true;
  d->in_use -= r.n;
  // merge with the next range of the same segment
  auto nx = std::next(it);
  if (nx != d->ranges.end() && nx->second.free && nx->second.base == r.base && nx->first == q + r.n) {
    free_list_erase(*d, nx->second.n, nx->first);
    d->cached -= nx->second.n;
    r.n += nx->second.n;
    d->ranges.erase(nx);
  }
  // ... and with the previous one
  if (it != d->ranges.begin()) {
    auto pv = std::prev(it);
    if (pv->second.free && pv->second.base == r.base && pv->first + pv->second.n == q) {
      free_list_erase(*d, pv->second.n, pv->first);
      d->cached -= pv->second.n;
      pv->second.n += r.n;
      d->ranges.erase(it);
      d->free_by_size.emplace(pv->second.n, pv->first);
      d->cached += pv->second.n;
      return;
    }
  }
  it->second = r;
  d->free_by_size.emplace(r.n, q);
  d->cached += r.n;
}

size_t dmem_cached(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_dev.find(device);
  return it == g_dev.end() ? 0 : it->second.cached;
}

size_t dmem_in_use(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_dev.find(device);
  return it == g_dev.end() ? 0 : it->second.in_use;
}

hipError_t dmem_free(size_t *free_b, size_t *total_b) {
  const hipError_t e = hipMemGetInfo(free_b, total_b);
  if (e != hipSuccess) return e;
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) *free_b += dmem_cached(dev);
  return hipSuccess;
}

}  // namespace vts

extern "C" int64_t vts_device_bytes(int device) { return static_cast<int64_t>(vts::dmem_in_use(device)); }

extern "C" int vts_empty_cache(int device) {
  std::lock_guard<std::mutex> lk(vts::g_mu);
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return vts::fail(VTS_E_HIP, "hipGetDevice");
  if (hipSetDevice(device) != hipSuccess) return vts::fail(VTS_E_NODEVICE, "device %d", device);
  vts::release_free_segments_locked(vts::g_dev[device]);
  vts::release_idle_chunks_locked(vts::g_dev[device]);
  (void)hipSetDevice(cur);
  return VTS_OK;
}
