// VMM probe: physical chunks (hipMemCreate) mapped into one reserved VA range
// vs one hipMalloc block — map / unmap / remap times and a copy kernel's
// bandwidth over each.  hipcc --offload-arch=gfx950 -O3 vmm_probe.hip -o vmm_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s failed: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
__global__ void copy4(const uint4 *a, uint4 *b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
double bw(const void *src, void *dst, size_t bytes) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const size_t n = bytes / 16;
  copy4<<<4096, 256>>>((const uint4 *)src, (uint4 *)dst, n);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) copy4<<<4096, 256>>>((const uint4 *)src, (uint4 *)dst, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return 2.0 * bytes * 5 / (ms / 1e3) / 1e9;
}
int main() {
  CK(hipSetDevice(0));
  int vmm = 0;
  CK(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, 0));
  std::printf("vmm supported %d\n", vmm);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  size_t rec = 0;
  CK(hipMemGetAllocationGranularity(&rec, &prop, hipMemAllocationGranularityRecommended));
  std::printf("granularity min %zu recommended %zu\n", gran, rec);
  const size_t G = 128ull << 20, total = 16ull << 30, k = total / G;
  std::vector<hipMemGenericAllocationHandle_t> h(k);
  double t0 = now();
  for (size_t i = 0; i < k; ++i) CK(hipMemCreate(&h[i], G, &prop, 0));
  double t1 = now();
  void *va = nullptr;
  CK(hipMemAddressReserve(&va, total, 0, nullptr, 0));
  for (size_t i = 0; i < k; ++i) CK(hipMemMap((char *)va + i * G, G, 0, h[i], 0));
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(va, total, &acc, 1));
  double t2 = now();
  void *pm = nullptr;
  CK(hipMalloc(&pm, total));
  CK(hipMemset(pm, 1, total));
  CK(hipMemset(va, 1, total));
  CK(hipDeviceSynchronize());
  const size_t half = total / 2;
  std::printf("create %zu x %zu MB: %.1f ms; reserve+map+access: %.1f ms\n", k, G >> 20, (t1 - t0) * 1e3, (t2 - t1) * 1e3);
  std::printf("copy bw hipMalloc %.0f GB/s, vmm %.0f GB/s\n", bw(pm, (char *)pm + half, half), bw(va, (char *)va + half, half));
  double t3 = now();
  CK(hipMemUnmap(va, total));
  CK(hipMemAddressFree(va, total));
  void *va2 = nullptr;
  CK(hipMemAddressReserve(&va2, total, 0, nullptr, 0));
  for (size_t i = 0; i < k; ++i) CK(hipMemMap((char *)va2 + i * G, G, 0, h[(i * 7) % k], 0));
  CK(hipMemSetAccess(va2, total, &acc, 1));
  double t4 = now();
  std::printf("unmap + remap (permuted chunks): %.1f ms; bw %.0f GB/s\n", (t4 - t3) * 1e3, bw(va2, (char *)va2 + half, half));
  return 0;
}
