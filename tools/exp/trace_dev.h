// Experiment only (never in the product build): per-wave section timing of
// the CABAC slice parser through its VTS_PARSE_TRACE points (parse_cabac.h),
// which the product compiles to nothing.  Built into a variant library by
//   bash tools/exp/build_full_variants.sh trace:"-include $PWD/tools/exp/trace_dev.h -DVTS_PARSE_TRACE(k)=vts_tp(k)"
// Each trace point adds the shader clock since the previous one to that
// point's bucket (lane 0, LDS) and counts the visit; point 15 (slice start)
// resets, 0 (every macroblock) and 16 (slice end) copy the buckets to
// vts_tr_out[workgroup][2 x kTrPoints] (cycles, visits), which
// vts_trace_dump() reads back.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

constexpr int kTrPoints = 20;
constexpr int kTrWaves = 4096;
__device__ unsigned long long vts_tr_out[kTrWaves * 2 * kTrPoints];

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void vts_tp(int k) {
  __shared__ unsigned long long acc[2 * kTrPoints + 2];  // cycles, visits, last time, last point
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    if (k == 15) {
      for (int i = 0; i < 2 * kTrPoints; ++i) acc[i] = 0;
      acc[2 * kTrPoints] = t;
      acc[2 * kTrPoints + 1] = 15;
    } else {
      const int lk = static_cast<int>(acc[2 * kTrPoints + 1]);
      acc[lk] += t - acc[2 * kTrPoints];
      acc[kTrPoints + lk] += 1;
      acc[2 * kTrPoints] = t;
      acc[2 * kTrPoints + 1] = static_cast<unsigned long long>(k);
      if ((k == 0 || k == 16) && blockIdx.x < kTrWaves)
        for (int i = 0; i < 2 * kTrPoints; ++i) vts_tr_out[blockIdx.x * 2 * kTrPoints + i] = acc[i];
    }
  }
}
#else
inline void vts_tp(int) {}
#endif

// host: copy the buckets of the first n workgroups (n <= kTrWaves)
extern "C" __attribute__((visibility("default"))) int vts_trace_dump(unsigned long long *out, int n) {
  if (n > kTrWaves) n = kTrWaves;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(vts_tr_out), sizeof(unsigned long long) * 2 * kTrPoints * n, 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? n
             : -1;
}
