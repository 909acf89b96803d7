// Experiment only (never in the product build): start and end of every
// workgroup of the one-workgroup-per-picture kernels (decode_full.hip's
// VTS_WG_TRACE points: kernel 0 h264_deblock_plane, 1 h264_intra_v2), on the
// 100 MHz real-time counter every XCD shares.  Built into a variant by
//   bash tools/exp/build_full_variants.sh wg:"-include $PWD/tools/exp/wg_trace.h -DVTS_WG_TRACE(k,e,key)=vts_wg_tp(k,e,key)"
// vts_wg_dump() reads the records back (and resets the counter).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

struct VtsWgRec {
  unsigned long long key;    // the launch's picture list (one per level launch) | kernel
  unsigned long long t0, t1;  // s_memrealtime at the workgroup's start / end (thread 0)
  unsigned int block, grid;
};
constexpr unsigned kWgRecs = 1u << 18;
__device__ VtsWgRec vts_wg_out[kWgRecs];
__device__ unsigned int vts_wg_n;

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void vts_wg_tp(int k, int end, const void *key) {
  __shared__ unsigned int slot;
  if (threadIdx.x != 0 || threadIdx.y != 0) return;
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  if (!end) {
    slot = atomicAdd(&vts_wg_n, 1u);
    if (slot < kWgRecs) {
      vts_wg_out[slot].key = reinterpret_cast<unsigned long long>(key) | static_cast<unsigned long long>(k);
      vts_wg_out[slot].t0 = t;
      vts_wg_out[slot].block = blockIdx.x;
      vts_wg_out[slot].grid = gridDim.x;
    }
  } else if (slot < kWgRecs) {
    vts_wg_out[slot].t1 = t;
  }
}
#else
__device__ inline void vts_wg_tp(int, int, const void *) {}
#endif

extern "C" __attribute__((visibility("default"))) int vts_wg_dump(void *out, int cap) {
  unsigned int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(vts_wg_n), sizeof(n), 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (n > kWgRecs) n = kWgRecs;
  if (static_cast<int>(n) > cap) n = static_cast<unsigned>(cap);
  if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(vts_wg_out), sizeof(VtsWgRec) * n, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  const unsigned int z = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(vts_wg_n), &z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess) return -1;
  return static_cast<int>(n);
}
