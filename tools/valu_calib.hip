// VALU issue-rate calibration for the roofline of this repo's integer kernels (bench.py
// valu_cycles(), profiles/valu_calibration.json).  MI355X_MICROARCH.md: a wave64 VALU
// instruction occupies a SIMD-32 for 2 cycles; one wave alone sustains one per 4.  This program
// measures what a saturated SIMD sustains for the instruction kinds k_fast_tile / k_cvfast /
// k_blur issue (32-bit add, packed u16 max/sub, v_perm, bitfield extract, 3-operand adds,
// compares into SGPR masks, v_cndmask), at 1, 2, 4 and 8 waves per SIMD: every wave runs 8
// independent chains of one instruction kind (no dependency stalls), the grid puts W waves on
// each of the 1024 SIMDs, and
//   cycles per instruction per SIMD = elapsed x clock x 1024 / (total wave instructions)
// from HIP events, cross-checked by the in-kernel shader clock (s_memtime ticks = shader
// cycles, MI355X_MICROARCH.md constants table): wave lifetime / (W x instructions per wave).
// Build: hipcc -O3 --offload-arch=gfx950 tools/valu_calib.hip -o tools/_bin/valu_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                  \
  do {                                                         \
    hipError_t e_ = (x);                                       \
    if (e_ != hipSuccess) {                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));  \
      return 1;                                                \
    }                                                          \
  } while (0)

constexpr int kChains = 8;
constexpr int kUnroll = 16;

template <int OP>
__device__ __forceinline__ void op(uint32_t& a, uint64_t& a2, uint32_t b, uint64_t b2, uint32_t c, uint64_t msk, uint64_t& sa, uint32_t& s32) {
  if constexpr (OP == 0) { asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 1) { asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 2) { asm volatile("v_pk_sub_u16 %0, %0, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 3) { asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)); }
  if constexpr (OP == 4) { asm volatile("v_bfe_u32 %0, %0, %1, 8" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 5) { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)); }
  if constexpr (OP == 6) { uint64_t m; asm volatile("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(m) : "v"(a), "v"(b)); asm volatile("" ::"s"(m)); }
  if constexpr (OP == 7) { asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(msk)); }
  if constexpr (OP == 8) { asm volatile("v_max_u32 %0, %0, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 9) { asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)); }
  if constexpr (OP == 10) { asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 11) { asm volatile("v_and_b32 %0, %0, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 12) { asm volatile("v_or_b32 %0, %0, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 13) { asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 14) { asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 15) { asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(b ^ a)); }
  if constexpr (OP == 16) { asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 17) { asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)); }
  if constexpr (OP == 18) { asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a2) : "v"(b2)); }
  if constexpr (OP == 19) { asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)); }
  if constexpr (OP == 20) { asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a), "v"(b) : "vcc"); }
  if constexpr (OP == 21) { asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c)); }
  if constexpr (OP == 22) { asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 23) { asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 24) { asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c)); }
  if constexpr (OP == 25) { asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(a) : "v"(b)); }
  if constexpr (OP == 26) { asm volatile("s_and_b64 %0, %0, %1" : "+s"(sa) : "s"(msk) : "scc"); }
  if constexpr (OP == 27) { asm volatile("s_add_u32 %0, %0, %1" : "+s"(s32) : "s"((uint32_t)msk) : "scc"); }
  if constexpr (OP == 28) { uint64_t m; asm volatile("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(m) : "v"(a), "v"(b)); asm volatile("s_and_b64 %0, %0, %1\n s_or_b64 %0, %0, %1" : "+s"(sa) : "s"(m) : "scc"); }
  if constexpr (OP == 29) { asm volatile("v_add_u32 %0, %0, %2\n s_and_b64 %1, %1, %3" : "+v"(a), "+s"(sa) : "v"(b), "s"(msk) : "scc"); }
}

template <int OP>
__global__ __launch_bounds__(256) void k_valu(uint32_t* __restrict__ sink, int iters,
                                              uint32_t magic, unsigned long long* __restrict__ cyc) {
  uint32_t a[kChains];
  uint64_t a2[kChains];
#pragma unroll
  for (int k = 0; k < kChains; k++) a[k] = threadIdx.x * 7 + k;
#pragma unroll
  for (int k = 0; k < kChains; k++) a2[k] = ((uint64_t)a[k] << 32) | a[k];
  const uint64_t b2 = ((uint64_t)magic << 32) | threadIdx.x;
  uint64_t sa[kChains];
  uint32_t s32[kChains];
#pragma unroll
  for (int k = 0; k < kChains; k++) {
    sa[k] = __builtin_amdgcn_readfirstlane(blockIdx.x + k) * 0x100000001ull;
    s32[k] = __builtin_amdgcn_readfirstlane(blockIdx.x * 3 + k);
  }
  const uint32_t b = blockIdx.x | 0x10001u, c = 0x05040100u ^ threadIdx.x;
  const uint64_t msk = ((uint64_t)magic << 32) | blockIdx.x;  // wave-uniform lane mask
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
#pragma unroll
      for (int k = 0; k < kChains; k++) op<OP>(a[k], a2[k], b, b2, c, msk, sa[k], s32[k]);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < kChains; k++) x ^= a[k] ^ (uint32_t)a2[k] ^ (uint32_t)sa[k] ^ s32[k];
  if (x == magic) sink[blockIdx.x * 256 + threadIdx.x] = x;  // magic is a runtime value
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

static const char* kNames[] = {"v_add_u32", "v_pk_max_u16", "v_pk_sub_u16", "v_perm_b32", "v_bfe_u32", "v_add3_u32", "v_cmp_gt_u32_e64", "v_cndmask_b32", "v_max_u32", "v_and_or_b32", "v_sub_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_lshlrev_b32", "v_mov_b32", "v_add_f32", "v_fma_f32", "v_pk_add_f32", "v_mad_u32_u24", "v_cmp_gt_u32_vcc", "v_min3_u32", "v_lshl_or_b32", "v_pk_add_u16", "v_dot4_u32_u8", "v_bcnt_u32_b32", "s_and_b64", "s_add_u32", "v_cmp_e64+2salu", "v_add_u32+s_and_b64"};

template <int OP>
int run(uint32_t* sink, unsigned long long* cyc, int waves_per_simd, int iters, bool print) {
  const int blocks = 256 * waves_per_simd;  // 4 waves per block: one per SIMD of a CU
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, sink, iters, 0xFFFFFFFFu, cyc);
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, sink, iters, 0xFFFFFFFFu, cyc);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipGetLastError());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h((size_t)blocks * 4);
  CK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  double avg = 0;
  for (auto v : h) avg += (double)v;
  avg /= h.size();
  const double per_wave = (double)iters * kUnroll * kChains;
  const double total = per_wave * blocks * 4;
  const double cyc_event = ms * 1e-3 * 2.4e9 * 1024 / total;  // at the 2.4 GHz peak clock
  const double cyc_clock = avg / (waves_per_simd * per_wave);
  if (print)
    printf("  {\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"wave_instr\": %.0f, "
           "\"cycles_per_instr_event_2p4GHz\": %.4f, \"cycles_per_instr_shader_clock\": %.4f},\n",
           kNames[OP], waves_per_simd, ms, total, cyc_event, cyc_clock);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return 0;
}

template <int OP>
int sweep(uint32_t* sink, unsigned long long* cyc) {
  for (int w : {1, 2, 8})
    if (run<OP>(sink, cyc, w, 1024, true)) return 1;
  return 0;
}

int main() {
  uint32_t* sink = nullptr;
  unsigned long long* cyc = nullptr;
  CK(hipMalloc(&sink, 256 * 8 * 256 * 4));
  CK(hipMalloc(&cyc, 256 * 8 * 4 * 8));
  setvbuf(stdout, nullptr, _IOLBF, 0);  // a line per run reaches the file even if a run stalls
  printf("{\"runs\": [\n");
  if (sweep<0>(sink, cyc) ||
      sweep<1>(sink, cyc) ||
      sweep<2>(sink, cyc) ||
      sweep<3>(sink, cyc) ||
      sweep<4>(sink, cyc) ||
      sweep<5>(sink, cyc) ||
      sweep<6>(sink, cyc) ||
      sweep<7>(sink, cyc) ||
      sweep<8>(sink, cyc) ||
      sweep<9>(sink, cyc) ||
      sweep<10>(sink, cyc) ||
      sweep<11>(sink, cyc) ||
      sweep<12>(sink, cyc) ||
      sweep<13>(sink, cyc) ||
      sweep<14>(sink, cyc) ||
      sweep<15>(sink, cyc) ||
      sweep<16>(sink, cyc) ||
      sweep<17>(sink, cyc) ||
      sweep<18>(sink, cyc) ||
      sweep<19>(sink, cyc) ||
      sweep<20>(sink, cyc) ||
      sweep<21>(sink, cyc) ||
      sweep<22>(sink, cyc) ||
      sweep<23>(sink, cyc) ||
      sweep<24>(sink, cyc) ||
      sweep<25>(sink, cyc) ||
      sweep<26>(sink, cyc) || sweep<27>(sink, cyc) || sweep<28>(sink, cyc) || sweep<29>(sink, cyc))
    return 1;
  printf("  {}]}\n");
  CK(hipFree(sink));
  CK(hipFree(cyc));
  return 0;
}
