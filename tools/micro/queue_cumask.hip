// Micro-probe: do streams run their kernels concurrently when a process has
// more streams than hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4)?
// Each of n streams gets one single-workgroup kernel that spins ~t ms on the
// constant 100 MHz clock (exit condition reached by every wave).  Wall time
// ~t: the kernels overlapped; ~n/4 x t: streams sharing a queue serialised.
// Variants: plain streams (hipStreamCreateWithFlags), CU-masked streams
// (hipExtStreamCreateWithCUMask, every CU enabled), and high-priority streams.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/queue_cumask.hip -o /tmp/qprobe
//   GPU_MAX_HW_QUEUES=4 /tmp/qprobe 8 20
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void spin(uint64_t ticks, uint32_t *out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t n = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    ++n;
  }
  if (threadIdx.x == 0) out[blockIdx.x] = n;
}

static double run(std::vector<hipStream_t> &ss, uint64_t ticks, uint32_t *d) {
  for (auto s : ss) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, ticks / 10, d);  // warm
  (void)hipDeviceSynchronize();
  const auto t0 = std::chrono::steady_clock::now();
  for (auto s : ss) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, ticks, d);
  (void)hipDeviceSynchronize();
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 8;
  const double ms = argc > 2 ? std::atof(argv[2]) : 20.0;
  const uint64_t ticks = static_cast<uint64_t>(ms * 1e5);  // 100 MHz
  uint32_t *d = nullptr;
  (void)hipMalloc(&d, 4096);
  const char *q = std::getenv("GPU_MAX_HW_QUEUES");
  std::vector<hipStream_t> plain(n), masked(n), prio(n);
  for (auto &s : plain) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  std::printf("{\"hw_queues\": \"%s\", \"streams\": %d, \"kernel_ms\": %.1f, \"plain_ms\": %.1f", q ? q : "unset", n,
              ms, run(plain, ticks, d));
  std::vector<uint32_t> mask(8, 0xffffffffu);  // 256 CUs
  bool ok = true;
  for (auto &s : masked)
    ok &= hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data()) == hipSuccess;
  std::printf(", \"cumask_ok\": %s, \"cumask_ms\": %.1f", ok ? "true" : "false", ok ? run(masked, ticks, d) : -1.0);
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  for (int i = 0; i < n; ++i) (void)hipStreamCreateWithPriority(&prio[i], hipStreamNonBlocking, i % 2 ? lo : hi);
  std::printf(", \"prio_range\": [%d, %d], \"mixed_prio_ms\": %.1f", lo, hi, run(prio, ticks, d));
  // plain and masked together: does a masked stream still get its own queue
  // once the plain ones hold all of them?
  std::vector<hipStream_t> both(plain.begin(), plain.end());
  both.insert(both.end(), masked.begin(), masked.end());
  std::printf(", \"plain_plus_cumask_ms\": %.1f}\n", ok ? run(both, ticks, d) : -1.0);
  return 0;
}
