// isabench.hip — issue throughput of the integer VALU instructions the hash
// path uses, on gfx950 (wave64).  Each kernel runs 8 independent chains of one
// instruction per lane so dependency latency is hidden; the grid fills every
// SIMD with 8 waves.  Reports wave-instructions per SIMD per shader clock
// (clock from s_memtime / s_memrealtime in the same kernel).
//   hipcc --offload-arch=gfx950 -O3 -o isabench tools/isabench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096

#define CHAIN8(ASM)                                                                       \
  asm volatile(ASM : "+v"(a0) : "v"(b0), "v"(c0)); asm volatile(ASM : "+v"(a1) : "v"(b0), "v"(c0)); \
  asm volatile(ASM : "+v"(a2) : "v"(b0), "v"(c0)); asm volatile(ASM : "+v"(a3) : "v"(b0), "v"(c0)); \
  asm volatile(ASM : "+v"(a4) : "v"(b0), "v"(c0)); asm volatile(ASM : "+v"(a5) : "v"(b0), "v"(c0)); \
  asm volatile(ASM : "+v"(a6) : "v"(b0), "v"(c0)); asm volatile(ASM : "+v"(a7) : "v"(b0), "v"(c0));

#define CHAIN8S(ASM)                                                                      \
  asm volatile(ASM : "+v"(a0) : "s"(s0)); asm volatile(ASM : "+v"(a1) : "s"(s0));         \
  asm volatile(ASM : "+v"(a2) : "s"(s0)); asm volatile(ASM : "+v"(a3) : "s"(s0));         \
  asm volatile(ASM : "+v"(a4) : "s"(s0)); asm volatile(ASM : "+v"(a5) : "s"(s0));         \
  asm volatile(ASM : "+v"(a6) : "s"(s0)); asm volatile(ASM : "+v"(a7) : "s"(s0));

template <int OP>
__global__ __launch_bounds__(256) void kop(uint32_t *out, uint64_t *clk) {
  uint32_t b0 = threadIdx.x * 7 + 1, c0 = threadIdx.x ^ 0x55;
  uint32_t s0 = __builtin_amdgcn_readfirstlane(b0 ^ 0x74656462u);
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7;
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < ITERS; ++i) {
    if (OP == 0) { CHAIN8("v_xor_b32 %0, %0, %1") }
    if (OP == 1) { CHAIN8("v_alignbit_b32 %0, %0, %1, 13") }
    if (OP == 2) { CHAIN8("v_add_u32 %0, %0, %1") }
    if (OP == 3) { CHAIN8("v_mul_lo_u32 %0, %0, %1") }
    if (OP == 4) { CHAIN8("v_mul_hi_u32 %0, %0, %1") }
    if (OP == 5) { CHAIN8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96") }
    if (OP == 6) { CHAIN8("v_lshlrev_b32 %0, 13, %0") }
    if (OP == 7) { CHAIN8("v_perm_b32 %0, %0, %1, %2") }
    if (OP == 8) { CHAIN8("v_alignbyte_b32 %0, %0, %1, 2") }
    if (OP == 9) { CHAIN8("v_pack_b32_f16 %0, %0, %1 op_sel:[1,0]") }
    if (OP == 10) { CHAIN8("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1") }
    if (OP == 11) { CHAIN8("v_lshl_or_b32 %0, %0, 13, %1") }
    if (OP == 12) { CHAIN8("v_add_co_u32 %0, vcc, %0, %1") }
    if (OP == 13) { CHAIN8("v_addc_co_u32 %0, vcc, %0, %1, vcc") }
    if (OP == 14) { CHAIN8("v_add3_u32 %0, %0, %1, %2") }
    if (OP == 15) { CHAIN8("v_xad_u32 %0, %0, %1, %2") }
    if (OP == 16) { CHAIN8("v_mov_b32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0") }
    if (OP == 17) { CHAIN8("v_lshrrev_b32_e32 %0, 13, %0") }
    if (OP == 18) { CHAIN8("v_cndmask_b32 %0, %0, %1, vcc") }
    if (OP == 19) { CHAIN8("v_pk_add_u16 %0, %0, %1") }
    if (OP == 20) { CHAIN8("v_and_or_b32 %0, %0, %1, %2") }
    if (OP == 21) { CHAIN8("v_mul_u32_u24 %0, %0, %1") }
    if (OP == 22) { CHAIN8("v_mov_b32_e32 %0, %1") }
    if (OP == 23) {
#define SWP(A, B) asm volatile("v_swap_b32 %0, %1" : "+v"(A), "+v"(B));
      SWP(a0, a1) SWP(a2, a3) SWP(a4, a5) SWP(a6, a7) SWP(a1, a2) SWP(a3, a4) SWP(a5, a6) SWP(a7, a0)
    }
    if (OP == 25) { CHAIN8("v_xor_b32_e32 %0, 0x74656462, %0") }
    if (OP == 26) { CHAIN8S("v_xor_b32_e32 %0, %1, %0") }
    if (OP == 27) { CHAIN8("v_lshlrev_b32_e32 %0, 13, %0") }
    if (OP == 28) { CHAIN8("v_cndmask_b32_e32 %0, %0, %1, vcc") }
    if (OP == 29) { CHAIN8("v_and_b32_e32 %0, 0x3fffffff, %0") }
    if (OP == 30) { CHAIN8("v_min_u32_e32 %0, %0, %1") }
    if (OP == 31) { CHAIN8("v_sub_u32_e32 %0, %0, %1") }
    if (OP == 32) { CHAIN8("v_lshlrev_b32_e64 %0, 13, %0") }
    if (OP == 33) { CHAIN8("v_xor_b32_e64 %0, %0, %1") }
    if (OP == 34) {  // canonical min as compiled: v_cmp_lt_u64 -> SGPR pair, two v_cndmask
#define CMIN(A, B) asm volatile("v_cmp_lt_u64_e64 s[40:41], %0, %1\n\tv_cndmask_b32_e64 %0, %1, %0, s[40:41]" : "+v"(A) : "v"(B) : "s40", "s41");
      uint64_t p0 = ((uint64_t)a1 << 32) | a0, p1 = ((uint64_t)a3 << 32) | a2;
      uint64_t q0 = ((uint64_t)b0 << 32) | c0;
      asm volatile("v_cmp_lt_u64_e64 s[40:41], %0, %2\n\tv_cndmask_b32_e64 %1, %1, %3, s[40:41]" : "+v"(p0), "+v"(a4) : "v"(q0), "v"(b0) : "s40", "s41");
      asm volatile("v_cmp_lt_u64_e64 s[42:43], %0, %2\n\tv_cndmask_b32_e64 %1, %1, %3, s[42:43]" : "+v"(p1), "+v"(a5) : "v"(q0), "v"(c0) : "s42", "s43");
      asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]\n\tv_cndmask_b32_e64 %2, %2, %1, s[42:43]" : "+v"(a6), "+v"(b0), "+v"(a7) :: "s40", "s41", "s42", "s43");
      asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]\n\tv_cndmask_b32_e64 %2, %2, %1, s[42:43]" : "+v"(a0), "+v"(c0), "+v"(a1) :: "s40", "s41", "s42", "s43");
      a2 ^= (uint32_t)p0; a3 ^= (uint32_t)p1;
    }
    if (OP == 35) { CHAIN8("v_cndmask_b32_e64 %0, %0, %1, s[4:5]") }
    if (OP == 36) {  // mix: 4 v_xor + 4 v_alignbit
      asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a0) : "v"(b0)); asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(a1) : "v"(b0));
      asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a2) : "v"(b0)); asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(a3) : "v"(b0));
      asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a4) : "v"(b0)); asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(a5) : "v"(b0));
      asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a6) : "v"(b0)); asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(a7) : "v"(b0));
    }
    if (OP == 37) { CHAIN8("v_lshlrev_b32_e32 %0, 2, %0") }
    if (OP == 38) { CHAIN8("v_add_lshl_u32 %0, %0, %1, 2") }
    if (OP == 39) { CHAIN8("v_mov_b32_e32 %0, %0") }
    if (OP == 24) {  // 64-bit add as a VOP2 carry pair through VCC
#define ADC(L, H) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %2\n\tv_addc_co_u32_e32 %1, vcc, %1, %3, vcc" : "+v"(L), "+v"(H) : "v"(b0), "v"(c0) : "vcc");
      ADC(a0, a1) ADC(a2, a3) ADC(a4, a5) ADC(a6, a7)
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

// 64-bit ops need register pairs
#define CHAIN8_64(ASM)                                                                     \
  asm volatile(ASM : "+v"(a0) : "v"(b0)); asm volatile(ASM : "+v"(a1) : "v"(b0));          \
  asm volatile(ASM : "+v"(a2) : "v"(b0)); asm volatile(ASM : "+v"(a3) : "v"(b0));          \
  asm volatile(ASM : "+v"(a4) : "v"(b0)); asm volatile(ASM : "+v"(a5) : "v"(b0));          \
  asm volatile(ASM : "+v"(a6) : "v"(b0)); asm volatile(ASM : "+v"(a7) : "v"(b0));

template <int OP>
__global__ __launch_bounds__(256) void kop64(uint64_t *out, uint64_t *clk) {
  uint64_t b0 = threadIdx.x * 7 + 1;
  uint32_t bl = threadIdx.x * 3 + 1, bh = threadIdx.x + 9;
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7;
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < ITERS; ++i) {
    if (OP == 0) { CHAIN8_64("v_lshl_add_u64 %0, %0, 0, %1") }
    if (OP == 1) { CHAIN8_64("v_lshlrev_b64 %0, 13, %0") }
    if (OP == 2) {
#define MAD(A) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(A) : "v"(bl), "v"(bh) : "vcc");
      MAD(a0) MAD(a1) MAD(a2) MAD(a3) MAD(a4) MAD(a5) MAD(a6) MAD(a7)
    }
    if (OP == 3) { CHAIN8_64("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]") }
    if (OP == 4) { CHAIN8_64("v_mov_b64_e32 %0, %1") }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <typename T>
static void run(const char *name, void (*kern)(T *, uint64_t *), void *out, uint64_t *clk) {
  const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e9;
  uint64_t hc[2] = {0, 0};
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, (T *)out, clk);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) {
      best = ms;
      (void)hipMemcpy(hc, clk, 16, hipMemcpyDeviceToHost);
    }
  }
  double winstr = (double)blocks * 4 * ITERS * 8;  // wave-instructions chip-wide
  double per_simd_s = winstr / (256.0 * 4) / (best * 1e-3);
  double ghz = (double)hc[0] / ((double)hc[1] / 100e6) / 1e9;
  printf("%-28s %8.3f ms  clk %.2f GHz  %.3f wave-instr/SIMD/clk  (%.2f clk per instr)\n", name, best,
         ghz, per_simd_s / (ghz * 1e9), (ghz * 1e9) / per_simd_s);
}

int main() {
  void *out;
  uint64_t *clk;
  (void)hipMalloc(&out, 256 * 8 * 256 * 8);
  (void)hipMalloc(&clk, 16);
  run("v_xor_b32", kop<0>, out, clk);
  run("v_alignbit_b32", kop<1>, out, clk);
  run("v_add_u32", kop<2>, out, clk);
  run("v_mul_lo_u32", kop<3>, out, clk);
  run("v_mul_hi_u32", kop<4>, out, clk);
  run("v_bitop3_b32", kop<5>, out, clk);
  run("v_lshlrev_b32", kop<6>, out, clk);
  run("v_perm_b32", kop<7>, out, clk);
  run("v_alignbyte_b32", kop<8>, out, clk);
  run("v_pack_b32_f16 op_sel", kop<9>, out, clk);
  run("v_or_b32_sdwa", kop<10>, out, clk);
  run("v_lshl_or_b32", kop<11>, out, clk);
  run("v_add_co_u32", kop<12>, out, clk);
  run("v_addc_co_u32", kop<13>, out, clk);
  run("v_add3_u32", kop<14>, out, clk);
  run("v_xad_u32", kop<15>, out, clk);
  run("v_mov_b32_sdwa", kop<16>, out, clk);
  run("v_lshrrev_b32_e32", kop<17>, out, clk);
  run("v_cndmask_b32", kop<18>, out, clk);
  run("v_pk_add_u16", kop<19>, out, clk);
  run("v_and_or_b32", kop<20>, out, clk);
  run("v_mul_u32_u24", kop<21>, out, clk);
  run("v_mov_b32_e32", kop<22>, out, clk);
  run("v_swap_b32 (8/iter)", kop<23>, out, clk);
  run("add_co+addc_co e32 (4 pairs)", kop<24>, out, clk);
  run("v_xor_b32_e32 literal", kop<25>, out, clk);
  run("v_xor_b32_e32 sgpr", kop<26>, out, clk);
  run("v_lshlrev_b32_e32", kop<27>, out, clk);
  run("v_cndmask_b32_e32 vcc", kop<28>, out, clk);
  run("v_and_b32_e32 literal", kop<29>, out, clk);
  run("v_min_u32_e32", kop<30>, out, clk);
  run("v_sub_u32_e32", kop<31>, out, clk);
  run("v_lshlrev_b32_e64", kop<32>, out, clk);
  run("v_xor_b32_e64", kop<33>, out, clk);
  run("cmp_lt_u64 + cndmask (mix)", kop<34>, out, clk);
  run("v_cndmask_b32_e64 s[4:5]", kop<35>, out, clk);
  run("4 xor + 4 alignbit", kop<36>, out, clk);
  run("v_lshlrev_b32_e32 by 2", kop<37>, out, clk);
  run("v_add_lshl_u32", kop<38>, out, clk);
  run("v_mov_b32 self", kop<39>, out, clk);
  run("v_lshl_add_u64", kop64<0>, out, clk);
  run("v_pk_mov_b32 swap", kop64<3>, out, clk);
  run("v_mov_b64_e32", kop64<4>, out, clk);
  run("v_lshlrev_b64", kop64<1>, out, clk);
  run("v_mad_u64_u32", kop64<2>, out, clk);
  return 0;
}
