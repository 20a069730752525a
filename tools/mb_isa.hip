// Microbenchmark: integer / fp64 instruction throughput on gfx950, and 256/384-bit Montgomery
// multiply throughput with the field.hpp implementation.  Used to size the NTT's VALU roofline
// (DESIGN.md "VALU bound").  Build: hipcc -O3 --offload-arch=gfx950 tools/mb_isa.hip -o mb_isa
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include "../ntt_amd/csrc/field.hpp"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;

// 8 independent chains of the instruction under test per iteration.
__global__ void k_mad64(uint64_t* out, uint32_t s) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t x = threadIdx.x * 7 + s, y = s * 13 + 5;
  uint64_t sc;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_mad_u64_u32 %0, %8, %9, %10, %0\n\t"
        "v_mad_u64_u32 %1, %8, %9, %10, %1\n\t"
        "v_mad_u64_u32 %2, %8, %9, %10, %2\n\t"
        "v_mad_u64_u32 %3, %8, %9, %10, %3\n\t"
        "v_mad_u64_u32 %4, %8, %9, %10, %4\n\t"
        "v_mad_u64_u32 %5, %8, %9, %10, %5\n\t"
        "v_mad_u64_u32 %6, %8, %9, %10, %6\n\t"
        "v_mad_u64_u32 %7, %8, %9, %10, %7\n\t"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "=s"(sc)
        : "v"(x), "v"(y));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

#define K32(NAME, INSTR)                                                                          \
  __global__ void NAME(uint64_t* out, uint32_t s) {                                               \
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,     \
             a6 = a0 + 6, a7 = a0 + 7;                                                            \
    uint32_t y = s * 13 + 5;                                                                      \
    for (int i = 0; i < ITERS; ++i) {                                                             \
      asm volatile(INSTR " %0, %0, %8\n\t" INSTR " %1, %1, %8\n\t" INSTR " %2, %2, %8\n\t" INSTR     \
                         " %3, %3, %8\n\t" INSTR " %4, %4, %8\n\t" INSTR " %5, %5, %8\n\t" INSTR     \
                         " %6, %6, %8\n\t" INSTR " %7, %7, %8\n\t"                                  \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                   : "v"(y));                                                                     \
    }                                                                                             \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
  }

K32(k_mullo, "v_mul_lo_u32")
K32(k_mulhi, "v_mul_hi_u32")
K32(k_add, "v_add_u32")
K32(k_mul24, "v_mul_u32_u24")
K32(k_mulhi24, "v_mul_hi_u32_u24")
K32(k_xor, "v_xor_b32")

__global__ void k_lshladd64(uint64_t* out, uint32_t s) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint64_t y = s * 13ull + 5;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_lshl_add_u64 %0, %0, 0, %8\n\t"
        "v_lshl_add_u64 %1, %1, 0, %8\n\t"
        "v_lshl_add_u64 %2, %2, 0, %8\n\t"
        "v_lshl_add_u64 %3, %3, 0, %8\n\t"
        "v_lshl_add_u64 %4, %4, 0, %8\n\t"
        "v_lshl_add_u64 %5, %5, 0, %8\n\t"
        "v_lshl_add_u64 %6, %6, 0, %8\n\t"
        "v_lshl_add_u64 %7, %7, 0, %8\n\t"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        : "v"(y));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_addc(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 13 + 5;
  uint64_t sc;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_add_co_u32 %0, vcc, %0, %9\n\t"
        "v_addc_co_u32 %1, vcc, %1, %9, vcc\n\t"
        "v_addc_co_u32 %2, vcc, %2, %9, vcc\n\t"
        "v_addc_co_u32 %3, vcc, %3, %9, vcc\n\t"
        "v_add_co_u32 %4, %8, %4, %9\n\t"
        "v_addc_co_u32 %5, %8, %5, %9, %8\n\t"
        "v_addc_co_u32 %6, %8, %6, %9, %8\n\t"
        "v_addc_co_u32 %7, %8, %7, %9, %8\n\t"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "=s"(sc)
        : "v"(y)
        : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_fma64(uint64_t* out, uint32_t s) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  double y = 1.0000001 + s * 1e-9, z = 1e-7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_fma_f64 %0, %0, %8, %9\n\t"
        "v_fma_f64 %1, %1, %8, %9\n\t"
        "v_fma_f64 %2, %2, %8, %9\n\t"
        "v_fma_f64 %3, %3, %8, %9\n\t"
        "v_fma_f64 %4, %4, %8, %9\n\t"
        "v_fma_f64 %5, %5, %8, %9\n\t"
        "v_fma_f64 %6, %6, %8, %9\n\t"
        "v_fma_f64 %7, %7, %8, %9\n\t"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        : "v"(y), "v"(z));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

constexpr int MM_ITERS = 64;
template <int N, bool FIPS>
__global__ void k_montmul(uint64_t* out, ntt::Modulus<N> M) {
  uint32_t x[N], y[N], w[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    x[i] = (threadIdx.x * 2654435761u + i * 40503u) & 0x0fffffffu;
    y[i] = (blockIdx.x * 97u + i * 31337u) & 0x0fffffffu;
    w[i] = (i * 0x9e3779b9u + threadIdx.x * 0x85ebca6bu) & 0x0fffffffu;
  }
  for (int it = 0; it < MM_ITERS; ++it) {
    if (FIPS) {
      ntt::mont_mul_fips<N>(x, x, w, M);
      ntt::mont_mul_fips<N>(y, y, w, M);
    } else {
      ntt::mont_mul_cios<N>(x, x, w, M);
      ntt::mont_mul_cios<N>(y, y, w, M);
    }
  }
  uint64_t h = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) h ^= x[i] ^ ((uint64_t)y[i] << 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = h;
}

__global__ void k_clock(uint64_t* out) {
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t a = threadIdx.x;
  for (int i = 0; i < (1 << 20); ++i) asm volatile("v_add_u32 %0, %0, 1" : "+v"(a));
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = r1 - r0; }
  if (a == 0xdeadbeef) out[0] = a;
}

typedef void (*kfn)(uint64_t*, uint32_t);

int main() {
  const int blocks = 2048, threads = 256;
  uint64_t* d;
  CHECK(hipMalloc(&d, (size_t)blocks * threads * 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));

  // clock
  hipLaunchKernelGGL(k_clock, dim3(256), dim3(64), 0, 0, d);
  CHECK(hipDeviceSynchronize());
  std::vector<uint64_t> h(512);
  CHECK(hipMemcpy(h.data(), d, 512 * 8, hipMemcpyDeviceToHost));
  double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
  printf("{\"shader_clock_ghz_single_wave\": %.3f}\n", ghz);

  struct { const char* name; kfn f; } ks[] = {
      {"v_mad_u64_u32", k_mad64}, {"v_mul_lo_u32", k_mullo},   {"v_mul_hi_u32", k_mulhi},
      {"v_add_u32", k_add},       {"v_add/addc_co_u32", k_addc}, {"v_mul_u32_u24", k_mul24},
      {"v_mul_hi_u32_u24", k_mulhi24}, {"v_fma_f64", k_fma64}, {"v_xor_b32", k_xor}, {"v_lshl_add_u64", k_lshladd64}};
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    double lane_ops = 5.0 * blocks * threads * (double)ITERS * 8;
    double rate = lane_ops / (ms * 1e-3);
    // cycles per wave64 instruction per SIMD at 2.4 GHz nominal: (1024 SIMDs * clk) / (rate/64)
    double cyc = 1024.0 * 2.4e9 / (rate / 64.0);
    printf("{\"instr\": \"%s\", \"Tlane_ops_per_s\": %.3f, \"cyc_per_wave_instr_per_simd@2.4GHz\": %.2f}\n", k.name,
           rate / 1e12, cyc);
  }

  // Montgomery multiply throughput, 256-bit (N=8) and 384-bit (N=12), CIOS (compiler) and FIPS (asm)
  {
    ntt::Modulus<8> M8;
    const uint32_t bn[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                            0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
    for (int i = 0; i < 8; ++i) M8.p[i] = bn[i];
    uint32_t inv = 1;
    for (int i = 0; i < 5; ++i) inv *= 2 - bn[0] * inv;
    M8.pinv = 0u - inv;
    ntt::Modulus<12> M12;
    for (int i = 0; i < 12; ++i) M12.p[i] = i < 8 ? bn[i] : 0;
    M12.pinv = M8.pinv;
    double muls = 5.0 * blocks * threads * MM_ITERS * 2;
    auto run8 = [&](auto kern, const char* name) -> int {
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, M8);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, M8);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"montmul\": \"%s\", \"Gmul_per_s\": %.2f}\n", name, muls / (ms * 1e-3) / 1e9);
      return 0;
    };
    auto run12 = [&](auto kern, const char* name) -> int {
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, M12);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, M12);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"montmul\": \"%s\", \"Gmul_per_s\": %.2f}\n", name, muls / (ms * 1e-3) / 1e9);
      return 0;
    };
    if (run8(k_montmul<8, false>, "256-cios")) return 1;
    if (run8(k_montmul<8, true>, "256-fips")) return 1;
    if (run12(k_montmul<12, false>, "384-cios")) return 1;
    if (run12(k_montmul<12, true>, "384-fips")) return 1;
  }
  return 0;
}
