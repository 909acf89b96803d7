// devmem.h — the sessions' device memory: a process-wide caching allocator.
//
// A session allocates tens of GB (decoded-surface rings, macroblock records,
// the coefficient arena).  hipMalloc of memory another allocation released
// waits while the driver clears it (vts_open of the general decoder after a
// closed session: 4-6 s in the allocation stage, against 7 ms on fresh
// memory; profiles/r04c_open_stages.json), so released blocks of >= 64 KiB
// stay mapped in a per-device cache and the next session takes them back.
// Placement: the smallest free range that holds the request; a range more
// than twice the request (and 64 MiB over it) is carved only for requests of
// >= 256 MiB, or when a fresh hipMalloc fails, so small buffers do not pin a
// large cached segment (a segment goes back to HIP only when wholly free).  A
// failed hipMalloc empties the device's wholly free segments and tries once
// more.  Window sizing counts cached bytes as free (vts::dmem_free: the free
// ranges, which large requests may carve).  vts_empty_cache() hands the
// cache back.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstddef>

namespace vts {

hipError_t dmalloc_raw(void **p, size_t n);
template <typename T>
inline hipError_t dmalloc(T **p, size_t n) {
  return dmalloc_raw(reinterpret_cast<void **>(p), n);
}
void dfree(void *p);                 // null-safe; the block's stream work must be finished
size_t dmem_cached(int device);      // bytes held in the device's cache
size_t dmem_in_use(int device);      // bytes of the device's cached ranges handed out (sessions' buffers)
hipError_t dmem_free(size_t *free_b, size_t *total_b);  // hipMemGetInfo + the cache

}  // namespace vts
