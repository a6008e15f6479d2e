// VALU issue-rate probe (round 5): wave64 instructions per SIMD per cycle for
// the instruction kinds of k_map, measured with 8 independent chains per lane
// and 4 waves per SIMD (1024-thread workgroups, one per CU, as k_map runs).
//   hipcc -O3 --offload-arch=gfx950 tools/probe_valu.hip -o build/probe_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 4096;
#define CH 8

#define OP_KERNEL(NAME, BODY)                                                      \
  __global__ __launch_bounds__(1024) void NAME(uint32_t* out, uint32_t seed) {   \
    uint32_t a[CH];                                                                \
    uint64_t q[CH];                                                                \
    for (int i = 0; i < CH; i++) { a[i] = seed * (threadIdx.x + i + 1); q[i] = a[i] * 0x9E3779B97F4A7C15ull; } \
    const uint32_t b = seed ^ threadIdx.x;                                         \
    for (int it = 0; it < ITERS; it++) {                                           \
      _Pragma("unroll") for (int i = 0; i < CH; i++) { BODY; }                     \
    }                                                                              \
    uint32_t r = 0;                                                                \
    for (int i = 0; i < CH; i++) r ^= a[i] ^ (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32); \
    if (r == 0x12345678u) out[blockIdx.x] = r;                                     \
  }

OP_KERNEL(k_add, asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_xor, asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_bitop3, asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_perm, asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_lshladd64, asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(q[i])))
OP_KERNEL(k_mullo, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_mulu24, asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_mad64, asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(q[i]) : "v"(a[i]), "v"(b) : "s0", "s1"))
OP_KERNEL(k_ffbl, asm volatile("v_ffbl_b32 %0, %0" : "+v"(a[i])))
OP_KERNEL(k_bcnt, asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_dpp, asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[i])))
OP_KERNEL(k_cmp64, asm volatile("v_cmp_eq_u64 vcc, %0, %1\n\tv_cndmask_b32 %2, %2, %3, vcc" : : "v"(q[i]), "v"(q[(i + 1) % CH]), "v"(a[i]), "v"(b) : "vcc"))
OP_KERNEL(k_cmp32cnd, asm volatile("v_cmp_eq_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc"))
OP_KERNEL(k_alignbit, asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_lshr, asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[i])))
OP_KERNEL(k_fma, asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_pkadd16, asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_add3, asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_and, asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_or, asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_lshl, asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a[i])))
OP_KERNEL(k_sub, asm volatile("v_sub_u32 %0, %1, %0" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_mov, asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 1) % CH])))
OP_KERNEL(k_andor, asm volatile("v_and_or_b32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_lshlor, asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_lshladd, asm volatile("v_lshl_add_u32 %0, %0, 7, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_or3, asm volatile("v_or3_b32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_bfi, asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_bfe, asm volatile("v_bfe_u32 %0, %0, 3, 9" : "+v"(a[i])))
OP_KERNEL(k_cnd, asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_cmp32, asm volatile("v_cmp_eq_u32 vcc, %0, %1" : : "v"(a[i]), "v"(b) : "vcc"))
OP_KERNEL(k_cmp64only, asm volatile("v_cmp_eq_u64 vcc, %0, %1" : : "v"(q[i]), "v"(q[(i + 1) % CH]) : "vcc"))
OP_KERNEL(k_lshlsdwa, asm volatile("v_lshlrev_b32_sdwa %0, 4, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(a[i])))
OP_KERNEL(k_mulsdwa, asm volatile("v_mul_u32_u24_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_mad24, asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_mulhi24, asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_xad, asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_addlshl, asm volatile("v_add_lshl_u32 %0, %0, %1, 4" : "+v"(a[i]) : "v"(b)))
OP_KERNEL(k_dppmov, asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[i])))
OP_KERNEL(k_lshr64, asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(q[i])))
OP_KERNEL(k_readlane, asm volatile("v_readlane_b32 s0, %0, 5" : : "v"(a[i]) : "s0"))

// the shader clock: s_memtime ticks over a fixed spin, against the wall clock
__global__ void k_clock(unsigned long long* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < 50000000ull) t = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = t - t0; out[1] = r1 - r0; }
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 4096 * 4);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct { const char* n; void (*k)(uint32_t*, uint32_t); int ops; } ks[] = {
      {"v_add_u32", k_add, 1}, {"v_xor_b32", k_xor, 1}, {"v_bitop3_b32", k_bitop3, 1}, {"v_perm_b32", k_perm, 1},
      {"v_lshl_add_u64", k_lshladd64, 1}, {"v_mul_lo_u32", k_mullo, 1}, {"v_mul_u32_u24", k_mulu24, 1},
      {"v_mad_u64_u32", k_mad64, 1}, {"v_ffbl_b32", k_ffbl, 1}, {"v_bcnt_u32_b32", k_bcnt, 1},
      {"v_add_u32_dpp", k_dpp, 1}, {"v_cmp_eq_u64+cndmask", k_cmp64, 2}, {"v_cmp_eq_u32+cndmask", k_cmp32cnd, 2},
      {"v_alignbit_b32", k_alignbit, 1}, {"v_lshrrev_b32", k_lshr, 1}, {"v_fma_f32", k_fma, 1}, {"v_pk_add_u16", k_pkadd16, 1},
      {"v_add3_u32", k_add3, 1}, {"v_and_b32", k_and, 1}, {"v_or_b32", k_or, 1}, {"v_lshlrev_b32", k_lshl, 1},
      {"v_sub_u32", k_sub, 1}, {"v_mov_b32", k_mov, 1}, {"v_and_or_b32", k_andor, 1}, {"v_lshl_or_b32", k_lshlor, 1},
      {"v_lshl_add_u32", k_lshladd, 1}, {"v_or3_b32", k_or3, 1}, {"v_bfi_b32", k_bfi, 1}, {"v_bfe_u32", k_bfe, 1},
      {"v_cndmask_b32 (vcc)", k_cnd, 1}, {"v_cmp_eq_u32", k_cmp32, 1}, {"v_cmp_eq_u64", k_cmp64only, 1},
      {"v_lshlrev_b32_sdwa", k_lshlsdwa, 1}, {"v_mul_u32_u24_sdwa", k_mulsdwa, 1}, {"v_mad_u32_u24", k_mad24, 1},
      {"v_mul_hi_u32_u24", k_mulhi24, 1}, {"v_xad_u32", k_xad, 1}, {"v_add_lshl_u32", k_addlshl, 1},
      {"v_mov_b32_dpp", k_dppmov, 1}, {"v_lshrrev_b64", k_lshr64, 1}, {"v_readlane_b32", k_readlane, 1}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.k, dim3(cus), dim3(1024), 0, 0, out, 12345u + rep);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) {
        const double wave_instr = (double)cus * 16 * ITERS * CH * k.ops;  // per CU: 16 waves
        const double per_simd = wave_instr / (cus * 4.0);
        printf("%-24s %8.3f ms  %6.2f ns per wave-instr per SIMD  (%.2f cycles at 2.4 GHz)\n", k.n, ms,
               ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
      }
    }
  }
  {
    unsigned long long* d;
    hipMalloc(&d, 16);
    hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, 0, d);
    unsigned long long h[2];
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("s_memtime %llu ticks in %llu s_memrealtime ticks (100 MHz): %.3f GHz\n", h[0], h[1], h[0] / (h[1] * 10.0));
  }
  return 0;
}
