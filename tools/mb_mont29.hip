// Microbenchmark: radix-2^29 Montgomery product (field29.hpp) throughput on gfx950 as a function of
// waves per SIMD (occupancy, forced with dynamic LDS) and independent products in flight per thread
// (ILP).  Answers: is the NTT's VALU time issue-bound or latency-bound at its 2 waves/SIMD?
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/mb_mont29.hip -o tools/mb_mont29
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../ntt_amd/csrc/field29.hpp"

#define CHECK(x)                                                                            \
  do {                                                                                      \
    hipError_t e = (x);                                                                     \
    if (e != hipSuccess) {                                                                  \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);         \
      return 1;                                                                             \
    }                                                                                       \
  } while (0)

using namespace ntt;
constexpr int L = 9;
constexpr int ITERS = 64;

// VAR 0: mont29 (compiler-scheduled), 1: mont29_chain (asm single chain), 2: mulc29 (Shoup, asm)
template <int ILP, int VAR>
__global__ __launch_bounds__(256) void k_mont(uint64_t* out, Mod29<L> M, Mod29<L> S, uint32_t seed) {
  extern __shared__ uint32_t pad[];  // occupancy control only
  uint32_t x[ILP][L], w[L], ws[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    w[i] = (i * 0x9e3779b9u + seed + threadIdx.x) & 0x0fffffffu;
    ws[i] = (i * 0x85ebca6bu + seed + threadIdx.x) & 0x1fffffffu;
#pragma unroll
    for (int k = 0; k < ILP; ++k) x[k][i] = (threadIdx.x * 2654435761u + i * 40503u + k * 7u) & 0x0fffffffu;
  }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < ILP; ++k) {
      uint32_t r[L];
      if constexpr (VAR == 0) mont29<L>(r, x[k], w, M);
      else if constexpr (VAR == 1) mont29_chain<L>(r, x[k], w, M);
      else if constexpr (VAR == 2) mulc29<L>(r, x[k], w, ws, S.p);
      else if constexpr (VAR == 3) mulc29_cc<L>(r, x[k], w, ws, S.p);
      else mulc29_blk<L>(r, x[k], w, ws, S.p);
#pragma unroll
      for (int i = 0; i < L; ++i) x[k][i] = r[i];
    }
  }
  uint64_t h = 0;
#pragma unroll
  for (int k = 0; k < ILP; ++k)
#pragma unroll
    for (int i = 0; i < L; ++i) h ^= (uint64_t)x[k][i] << (i & 31);
  if (h == 0x123456789ull) pad[threadIdx.x] = 1;
  out[blockIdx.x * blockDim.x + threadIdx.x] = h;
}


// Issue cost of the non-multiply instructions the field code leans on (8 independent chains).
#define KOP(NAME, BODY, T)                                                                          \
  __global__ void NAME(uint64_t* out, uint32_t s) {                                                 \
    T a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, \
      a7 = a0 + 7;                                                                                  \
    uint32_t y = s * 13 + 5, z = s * 7 + 3;                                                         \
    for (int i = 0; i < 2048; ++i) {                                                                \
      asm volatile(BODY("%0") BODY("%1") BODY("%2") BODY("%3") BODY("%4") BODY("%5") BODY("%6")       \
                       BODY("%7")                                                                   \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                   : "v"(y), "v"(z));                                                               \
    }                                                                                               \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);  \
  }
#define B_LSHR64(r) "v_lshrrev_b64 " r ", 29, " r "\n\t"
#define B_ALIGN(r) "v_alignbit_b32 " r ", " r ", %8, 29\n\t"
#define B_ADD3(r) "v_add3_u32 " r ", " r ", %8, %9\n\t"
#define B_BFE(r) "v_bfe_u32 " r ", " r ", 29, 3\n\t"
#define B_ANDOR(r) "v_and_or_b32 " r ", " r ", %8, %9\n\t"
#define B_LSHLOR(r) "v_lshl_or_b32 " r ", " r ", 3, %8\n\t"
#define B_MAD32(r) "v_mad_u32_u24 " r ", " r ", %8, %9\n\t"
#define B_ASHR(r) "v_ashrrev_i32 " r ", 29, " r "\n\t"
KOP(k_lshr64, B_LSHR64, uint64_t)
KOP(k_align, B_ALIGN, uint32_t)
KOP(k_add3, B_ADD3, uint32_t)
KOP(k_bfe, B_BFE, uint32_t)
KOP(k_andor, B_ANDOR, uint32_t)
KOP(k_lshlor, B_LSHLOR, uint32_t)
KOP(k_mad24, B_MAD32, uint32_t)
KOP(k_ashr, B_ASHR, uint32_t)

static int run_op(const char* name, void (*f)(uint64_t*, uint32_t), uint64_t* d) {
  const int blocks = 2048, threads = 256;
  hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double rate = 5.0 * blocks * threads * 2048.0 * 8 / (ms * 1e-3);
  printf("{\"instr\": \"%s\", \"cyc_per_wave_instr_per_simd@2.4GHz\": %.2f}\n", name, 1024.0 * 2.4e9 / (rate / 64.0));
  return 0;
}

template <int ILP, int VAR>
static int run(Mod29<L> M, Mod29<L> S, uint64_t* d, int wg_per_cu) {
  const int threads = 256, blocks = 256 * wg_per_cu * 4;  // 4 rounds of full-chip residency
  const size_t lds = (160 * 1024) / wg_per_cu - 1024;
  CHECK(hipFuncSetAttribute((const void*)(k_mont<ILP, VAR>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((k_mont<ILP, VAR>), dim3(blocks), dim3(threads), lds, 0, d, M, S, 1u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_mont<ILP, VAR>), dim3(blocks), dim3(threads), lds, 0, d, M, S, 1u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double muls = 3.0 * blocks * threads * (double)ITERS * ILP;
  const double rate = muls / (ms * 1e-3);
  const double cyc = 1024.0 * 2.4e9 / (rate / 64.0);  // SIMD cycles per wave-level product @2.4 GHz
  static const char* names[] = {"mont29", "mont29_chain", "mulc29_shoup", "mulc29_shoup_cc", "mulc29_shoup_blk"};
  printf("{\"variant\": \"%s\", \"ilp\": %d, \"waves_per_simd\": %d, \"Gmul_per_s\": %.2f, "
         "\"simd_cycles_per_wave_mul\": %.1f}\n", names[VAR], ILP, wg_per_cu, rate / 1e9, cyc);
  return 0;
}

int main() {
  // BN254 Fr in radix-2^29 limbs
  const uint32_t bn[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                          0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  Mod29<L> M{};
  pack29<L, 8>(M.p, bn);
  uint32_t inv = 1;
  for (int i = 0; i < 5; ++i) inv *= 2 - M.p[0] * inv;
  M.pinv = (0u - inv) & kMask29;
  uint64_t* d;
  CHECK(hipMalloc(&d, (size_t)256 * 8 * 4 * 256 * 8));
  if (run_op("v_lshrrev_b64", k_lshr64, d) || run_op("v_alignbit_b32", k_align, d) ||
      run_op("v_add3_u32", k_add3, d) || run_op("v_bfe_u32", k_bfe, d) || run_op("v_and_or_b32", k_andor, d) ||
      run_op("v_lshl_or_b32", k_lshlor, d) || run_op("v_mad_u32_u24", k_mad24, d) || run_op("v_ashrrev_i32", k_ashr, d))
    return 1;
  Mod29<L> S{};  // S.p = pbar = 2^(29L) - p
  {
    uint32_t borrow = 1;
    for (int i = 0; i < L; ++i) {
      uint32_t v = (kMask29 - M.p[i]) + borrow;
      S.p[i] = v & kMask29;
      borrow = v >> 29;
    }
  }
  for (int occ : {2, 3}) {
    if (run<1, 0>(M, S, d, occ) || run<2, 0>(M, S, d, occ)) return 1;
    if (run<1, 2>(M, S, d, occ) || run<2, 2>(M, S, d, occ)) return 1;
    if (run<1, 3>(M, S, d, occ) || run<2, 3>(M, S, d, occ)) return 1;
    if (run<1, 4>(M, S, d, occ) || run<2, 4>(M, S, d, occ)) return 1;
  }
  return 0;
}
