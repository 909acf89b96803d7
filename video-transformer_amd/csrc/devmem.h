// devmem.h — the sessions' device memory: a process-wide caching allocator.
//
// A session allocates tens of GB (decoded-surface rings, macroblock records,
// the coefficient arena).  HBM handed back to HIP is cleared by the driver
// before it is handed out again (~45 GB/s; vts_open of a session after
// differently shaped ones: seconds in the allocation stage), so nothing goes
// back between sessions:
//  - requests of >= 256 MiB are physical 128 MiB chunks (hipMemCreate)
//    mapped back to back into a fresh virtual range; on release the range is
//    unmapped and the chunks kept, and any later request maps whichever are
//    idle — no fragmentation, whatever the sessions' shapes (devmem.cpp);
//  - smaller blocks of >= 64 KiB stay in a per-device cache of hipMalloc
//    segments: the smallest free range that holds the request, a range more
//    than twice the request (and 64 MiB over it) carved only when a fresh
//    hipMalloc fails; a segment goes back to HIP only when wholly free, and
//    a failed allocation gives back only as much as it needs, smallest idle
//    segments / chunks first.
// Window sizing counts cached bytes as free (vts::dmem_free).
// vts_empty_cache() hands everything idle back; VTS_DEVMEM_LOG=1 logs every
// fresh allocation and give-back, VTS_DEVMEM_VMM=0 turns the mapped path off.
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
