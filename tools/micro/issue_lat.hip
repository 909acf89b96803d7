// Micro-benchmark: issue cost of instruction chains on one lone wave (the
// CABAC parser's regime: a 57 KB I slice is one wave's serial chain).
// Every asm block declares SCC clobbered (the loop's own compare must not
// live across it: without that the r06g run's loop never ended).
// Each test runs 32 copies of one short sequence per loop iteration, 2000
// iterations, timed with s_memtime; prints cycles per copy.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/issue_lat.hip -o tools/micro/issue_lat
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define R4(x) x x x x
#define R32(x) R4(R4(x)) R4(x) R4(x)

template <int T>
__global__ void __launch_bounds__(64) lat(uint32_t seed, uint32_t *out, unsigned long long *cyc) {
  uint32_t s = seed, s2 = seed + 1, s3 = seed + 2, s4 = seed + 3;
  uint32_t v = threadIdx.x + seed, v2 = v + 1;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 2000; ++it) {
    if constexpr (T == 0) {  // dependent SALU adds
      asm volatile(R32("s_add_u32 %0, %0, 1\n") : "+s"(s)::"scc");
    } else if constexpr (T == 1) {  // independent SALU adds (4 chains)
      asm volatile(R32("s_add_u32 %0, %0, 1\ns_add_u32 %1, %1, 1\ns_add_u32 %2, %2, 1\ns_add_u32 %3, %3, 1\n")
                   : "+s"(s), "+s"(s2), "+s"(s3), "+s"(s4)::"scc");
    } else if constexpr (T == 2) {  // dependent VALU adds
      asm volatile(R32("v_add_u32 %0, %0, 1\n") : "+v"(v));
    } else if constexpr (T == 3) {  // independent VALU adds (2 chains)
      asm volatile(R32("v_add_u32 %0, %0, 1\nv_add_u32 %1, %1, 1\n") : "+v"(v), "+v"(v2));
    } else if constexpr (T == 4) {  // VGPR -> SGPR -> VGPR round trip: readfirstlane, s_add, v_add with SGPR
      asm volatile(R32("v_readfirstlane_b32 %1, %0\ns_add_u32 %1, %1, 1\nv_add_u32 %0, %1, %0\n")
                   : "+v"(v), "+s"(s)::"scc");
    } else if constexpr (T == 5) {  // v_readlane with a SALU-computed lane select, dependent
      asm volatile(R32("s_and_b32 %1, %1, 63\nv_readlane_b32 %1, %0, %1\n") : "+v"(v), "+s"(s)::"scc");
    } else if constexpr (T == 6) {  // compare + branch not taken (scc from SALU)
      asm volatile(R32("s_cmp_eq_u32 %0, 12345\ns_cbranch_scc1 1f\ns_add_u32 %0, %0, 1\n") "1:\n" : "+s"(s)::"scc");
    } else if constexpr (T == 7) {  // v_cmp -> vcc -> s_cbranch_vccnz not taken
      asm volatile(R32("v_cmp_eq_u32 vcc, 12345, %0\ns_cbranch_vccnz 1f\nv_add_u32 %0, %0, 1\n") "1:\n"
                   : "+v"(v)::"vcc", "scc");
    } else if constexpr (T == 8) {  // v_writelane then v_readlane of the same VGPR (LaneTab set / get)
      asm volatile(R32("v_writelane_b32 %0, %1, 5\nv_readlane_b32 %1, %0, 5\ns_add_u32 %1, %1, 1\n")
                   : "+v"(v), "+s"(s)::"scc");
    } else if constexpr (T == 9) {  // SALU chain with s_cselect (scc dependence)
      asm volatile(R32("s_cmp_ge_u32 %0, %1\ns_cselect_b32 %0, %1, %0\ns_add_u32 %0, %0, 1\n") : "+s"(s), "+s"(s2)::"scc");
    } else if constexpr (T == 10) {  // s_flbit + shifts (renormalisation)
      asm volatile(R32("s_flbit_i32_b32 %1, %0\ns_lshl_b32 %0, %0, %1\ns_or_b32 %0, %0, 1\n") : "+s"(s), "+s"(s2)::"scc");
    } else if constexpr (T == 12) {  // compare + branch TAKEN over one instruction
      asm volatile(R32("s_cmp_lg_u32 %0, 12345\ns_cbranch_scc1 1f\ns_add_u32 %0, %0, 7\n1:\ns_add_u32 %0, %0, 1\n")
                   : "+s"(s)::"scc");
    } else if constexpr (T == 13) {  // readlane -> SALU -> readlane chain (state -> lps table)
      asm volatile(R32("v_readlane_b32 %1, %0, %1\ns_lshr_b32 %1, %1, 1\ns_and_b32 %1, %1, 63\n") : "+v"(v), "+s"(s)::"scc");
    } else if constexpr (T == 14) {  // unconditional jump to the next instruction block
      asm volatile(R32("s_branch 1f\ns_add_u32 %0, %0, 7\n1:\ns_add_u32 %0, %0, 1\n") : "+s"(s)::"scc");
    } else if constexpr (T == 11) {  // ds_read after ds_write, waited (LDS round trip)
      __shared__ uint32_t l[64];
      asm volatile(R32("ds_write_b32 %1, %0\nds_read_b32 %0, %1\ns_waitcnt lgkmcnt(0)\n")
                   : "+v"(v) : "v"(threadIdx.x * 4));
      (void)l;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = s + s2 + s3 + s4 + v + v2;
    cyc[0] = t1 - t0;
  }
}

template <int T>
static void run(const char *name, int per, uint32_t *d, unsigned long long *dc) {
  hipLaunchKernelGGL(lat<T>, dim3(1), dim3(64), 0, 0, 1u, d, dc);
  hipLaunchKernelGGL(lat<T>, dim3(1), dim3(64), 0, 0, 1u, d, dc);
  unsigned long long c = 0;
  (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  std::printf("{\"test\": \"%s\", \"cycles_per_copy\": %.2f, \"instructions_per_copy\": %d}\n", name,
              static_cast<double>(c) / (2000.0 * 32), per);
  std::fflush(stdout);
}

int main(int argc, char **argv) {
  const int only = argc > 1 ? std::atoi(argv[1]) : -1;
  uint32_t *d = nullptr;
  unsigned long long *dc = nullptr;
  (void)hipMalloc(&d, 64);
  (void)hipMalloc(&dc, 8);
  if (only < 0 || only == 0) run<0>("salu_dep", 1, d, dc);
  if (only < 0 || only == 1) run<1>("salu_indep4", 4, d, dc);
  if (only < 0 || only == 2) run<2>("valu_dep", 1, d, dc);
  if (only < 0 || only == 3) run<3>("valu_indep2", 2, d, dc);
  if (only < 0 || only == 4) run<4>("readfirstlane_salu_valu", 3, d, dc);
  if (only < 0 || only == 5) run<5>("salu_lane_readlane", 2, d, dc);
  if (only < 0 || only == 6) run<6>("scmp_branch_salu", 3, d, dc);
  if (only < 0 || only == 7) run<7>("vcmp_vccbranch_valu", 3, d, dc);
  if (only < 0 || only == 8) run<8>("writelane_readlane_salu", 3, d, dc);
  if (only < 0 || only == 9) run<9>("scmp_cselect_add", 3, d, dc);
  if (only < 0 || only == 10) run<10>("flbit_lshl_or", 3, d, dc);
  if (only < 0 || only == 11) run<11>("lds_write_read_wait", 3, d, dc);
  if (only < 0 || only == 12) run<12>("scmp_branch_taken_salu", 3, d, dc);
  if (only < 0 || only == 13) run<13>("readlane_salu_chain", 3, d, dc);
  if (only < 0 || only == 14) run<14>("s_branch_salu", 2, d, dc);
  return 0;
}
