// Issue-cost microbenchmark for the Montgomery inner-loop instructions on
// gfx950 (tools only).  Each kernel runs REP x 8 independent copies of one
// instruction pattern per loop trip (8 independent accumulators, so the
// stream is throughput- not latency-bound) and reports chip-wide wave-
// instructions per SIMD-cycle-equivalent: ns per 1e9 lane-instructions.
//   mad      v_mad_u64_u32 (carry-out to an SGPR pair, discarded)
//   addc     v_addc_co_u32_e64 (carry-in/out in an SGPR pair)
//   madaddc  the fmul step: mad + addc on the mad's carry
//   madaddcn the fmul step as hipcc emits it: mad + addc + s_nop 0
//   add      v_add_u32 (plain 32-bit op)
//   add64    v_lshl_add_u64 (64-bit add, shift 0)
//   bfe      v_alignbit_b32 (radix-change helper)
//   and the other non-MAD ops of the reduced-radix products: 64-bit shift,
//   and/sub/shift/mov (32-bit), cndmask with an SGPR mask, mad with an SGPR
//   operand, and_or
// Build: hipcc --offload-arch=gfx950 -O3 -o issue_bench issue_bench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;

#define MAD(i) "v_mad_u64_u32 %[a" #i "], s[40:41], %[x], %[y], %[a" #i "]\n\t"
#define ADDC(i) "v_addc_co_u32_e64 %[t" #i "], s[42:43], %[t" #i "], 0, s[42:43]\n\t"
#define MADADDC(i) "v_mad_u64_u32 %[a" #i "], s[40:41], %[x], %[y], %[a" #i "]\n\t" \
                   "v_addc_co_u32_e64 %[t" #i "], s[40:41], %[t" #i "], 0, s[40:41]\n\t"
#define MADADDCD(i, S) "v_mad_u64_u32 %[a" #i "], " S ", %[x], %[y], %[a" #i "]\n\t" \
                   "v_addc_co_u32_e64 %[t" #i "], " S ", %[t" #i "], 0, " S "\n\t"
#define MADADDCV(i) "v_mad_u64_u32 %[a" #i "], vcc, %[x], %[y], %[a" #i "]\n\t" \
                    "v_addc_co_u32_e32 %[t" #i "], vcc, 0, %[t" #i "], vcc\n\t"
#define ADDCV(i) "v_addc_co_u32_e32 %[t" #i "], vcc, %[x], %[t" #i "], vcc\n\t"
#define ADDCO(i) "v_add_co_u32_e32 %[t" #i "], vcc, %[x], %[t" #i "]\n\t"
#define ADD3(i) "v_add3_u32 %[t" #i "], %[t" #i "], %[x], %[y]\n\t"
#define MUL24(i) "v_mul_u32_u24 %[t" #i "], %[t" #i "], %[x]\n\t"
#define MULHI24(i) "v_mul_hi_u32_u24 %[t" #i "], %[t" #i "], %[x]\n\t"
#define MULLO(i) "v_mul_lo_u32 %[t" #i "], %[t" #i "], %[x]\n\t"
#define MULHI(i) "v_mul_hi_u32 %[t" #i "], %[t" #i "], %[x]\n\t"
#define CND(i) "v_cndmask_b32_e32 %[t" #i "], %[t" #i "], %[x], vcc\n\t"
#define FMA64(i) "v_fma_f64 %[a" #i "], %[a" #i "], %[a" #i "], %[a" #i "]\n\t"
#define MADADDCN(i) MADADDC(i) "s_nop 0\n\t"
#define ADD(i) "v_add_u32 %[t" #i "], %[t" #i "], %[x]\n\t"
#define ADD64(i) "v_lshl_add_u64 %[a" #i "], %[a" #i "], 0, %[a" #i "]\n\t"
#define BFE(i) "v_alignbit_b32 %[t" #i "], %[t" #i "], %[x], 29\n\t"
#define SHR64(i) "v_lshrrev_b64 %[a" #i "], 29, %[a" #i "]\n\t"
#define AND(i) "v_and_b32 %[t" #i "], %[t" #i "], %[x]\n\t"
#define SUB(i) "v_sub_u32 %[t" #i "], %[t" #i "], %[x]\n\t"
#define SHR32(i) "v_lshrrev_b32 %[t" #i "], 29, %[t" #i "]\n\t"
#define MOV(i) "v_mov_b32 %[t" #i "], %[x]\n\t"
#define CND64(i) "v_cndmask_b32_e64 %[t" #i "], %[t" #i "], %[x], s[40:41]\n\t"
#define MADS(i) "v_mad_u64_u32 %[a" #i "], s[40:41], %[x], s44, %[a" #i "]\n\t"
#define ANDOR(i) "v_and_or_b32 %[t" #i "], %[t" #i "], %[x], %[y]\n\t"
#define X8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)

#define KERNEL(NAME, BODY)                                                                         \
  __global__ void NAME(uint64_t* out, uint32_t s) {                                              \
    uint64_t a0 = s, a1 = s + 1, a2 = s + 2, a3 = s + 3, a4 = s + 4, a5 = s + 5, a6 = s + 6, a7 = s + 7; \
    uint32_t t0 = s, t1 = s ^ 1, t2 = s ^ 2, t3 = s ^ 3, t4 = s ^ 4, t5 = s ^ 5, t6 = s ^ 6, t7 = s ^ 7; \
    uint32_t x = threadIdx.x | 1, y = s | 3;                                                      \
    for (int i = 0; i < ITERS; i++) {                                                             \
      asm volatile(BODY BODY                                                                      \
                   : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [a4] "+v"(a4),  \
                     [a5] "+v"(a5), [a6] "+v"(a6), [a7] "+v"(a7), [t0] "+v"(t0), [t1] "+v"(t1),  \
                     [t2] "+v"(t2), [t3] "+v"(t3), [t4] "+v"(t4), [t5] "+v"(t5), [t6] "+v"(t6),  \
                     [t7] "+v"(t7)                                                               \
                   : [x] "v"(x), [y] "v"(y)                                                     \
                   : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", \
                     "s51", "s52", "s53", "s54", "s55", "vcc");                                                \
    }                                                                                             \
    out[blockIdx.x * blockDim.x + threadIdx.x] =                                                  \
        a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ t0 ^ t1 ^ t2 ^ t3 ^ t4 ^ t5 ^ t6 ^ t7;            \
  }

KERNEL(k_mad, X8(MAD))
KERNEL(k_addc, X8(ADDC))
KERNEL(k_madaddc, X8(MADADDC))
KERNEL(k_madaddcn, X8(MADADDCN))
KERNEL(k_madaddcd, MADADDCD(0, "s[40:41]") MADADDCD(1, "s[42:43]") MADADDCD(2, "s[44:45]")
       MADADDCD(3, "s[46:47]") MADADDCD(4, "s[48:49]") MADADDCD(5, "s[50:51]") MADADDCD(6, "s[52:53]")
       MADADDCD(7, "s[54:55]"))
KERNEL(k_add, X8(ADD))
KERNEL(k_madaddcv, X8(MADADDCV))
KERNEL(k_addcv, X8(ADDCV))
KERNEL(k_addco, X8(ADDCO))
KERNEL(k_add3, X8(ADD3))
KERNEL(k_mul24, X8(MUL24))
KERNEL(k_mulhi24, X8(MULHI24))
KERNEL(k_mullo, X8(MULLO))
KERNEL(k_mulhi, X8(MULHI))
KERNEL(k_cnd, X8(CND))
KERNEL(k_fma64, X8(FMA64))
KERNEL(k_add64, X8(ADD64))
KERNEL(k_bfe, X8(BFE))
KERNEL(k_shr64, X8(SHR64))
KERNEL(k_and, X8(AND))
KERNEL(k_sub, X8(SUB))
KERNEL(k_shr32, X8(SHR32))
KERNEL(k_mov, X8(MOV))
KERNEL(k_cnd64, X8(CND64))
KERNEL(k_mads, X8(MADS))
KERNEL(k_andor, X8(ANDOR))

typedef void (*kern_t)(uint64_t*, uint32_t);

int main() {
  struct { const char* name; kern_t k; int instr; } ks[] = {
      {"mad", k_mad, 16},         {"addc", k_addc, 16},   {"mad+addc", k_madaddc, 32},
      {"mad+addc+nop", k_madaddcn, 48}, {"mad+addc dsgpr", k_madaddcd, 32}, {"add_u32", k_add, 16}, {"add64", k_add64, 16},
      {"alignbit", k_bfe, 16}, {"mad+addc vcc", k_madaddcv, 32}, {"addc_e32 vcc", k_addcv, 16},
      {"add_co_e32", k_addco, 16}, {"add3", k_add3, 16}, {"mul_u32_u24", k_mul24, 16},
      {"mul_hi_u24", k_mulhi24, 16}, {"mul_lo_u32", k_mullo, 16}, {"mul_hi_u32", k_mulhi, 16},
      {"cndmask_e32", k_cnd, 16}, {"fma_f64", k_fma64, 16},
      {"lshrrev_b64", k_shr64, 16}, {"and_b32", k_and, 16}, {"sub_u32", k_sub, 16}, {"lshrrev_b32", k_shr32, 16},
      {"mov_b32", k_mov, 16}, {"cndmask_e64 sgpr", k_cnd64, 16}, {"mad sgpr operand", k_mads, 16},
      {"and_or_b32", k_andor, 16},
  };
  uint64_t* out;
  CHK(hipMalloc(&out, sizeof(uint64_t) << 24));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  int ncu = 256;
  for (int wps : {2, 4}) {
    const int blocks = ncu * wps, threads = 256;  // 256 threads = 1 wave per SIMD per block
    for (auto& k : ks) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; rep++) {
        CHK(hipEventRecord(a));
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, out, 7u);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
      }
      const double waves = (double)blocks * threads / 64;
      const double winstr = waves * ITERS * k.instr;  // wave-instructions (nop counted)
      // cycles per wave-instruction per SIMD at 2.4 GHz
      const double cyc = best * 1e-3 * 2.4e9 * ncu * 4 / winstr;
      printf("waves/SIMD %d  %-14s %8.3f ms  %6.2f SIMD-cyc per wave-instr (2.4 GHz)  %6.2f T lane-instr/s\n", wps,
             k.name, best, cyc, winstr * 64 / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
