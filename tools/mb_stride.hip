// HBM microbenchmark: the pass kernels' access patterns without the arithmetic.
//
// A "column pass" over n 32-B elements: workgroup w owns T adjacent columns of a block of N
// elements (R rows of stride s = N / R); every thread moves EPT elements as 2 x dwordx4 each.
// Reports GB/s (read + write) for: contiguous copy, the pass-1 pattern (s = 2^16 elements = 2 MB),
// the pass-2 pattern (s = 256 = 8 KB), the final-pass pattern (contiguous read, 2-MB-strided
// write), and the same strided patterns with a padded row pitch (s + PAD elements) to tell DRAM
// bank / channel conflicts of power-of-two strides from plain small-run inefficiency.
//
//   hipcc -O3 --offload-arch=gfx950 tools/mb_stride.hip -o tools/mb_stride && tools/mb_stride
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// src index of the (col, row) element of block b: base(b) + col + row * pitch_r; dst likewise
__global__ __launch_bounds__(256) void k_cols(const uint4* __restrict__ src, uint4* __restrict__ dst, uint32_t log_r,
                                              uint32_t log_t, uint32_t log_cols, uint64_t pitch_rd, uint64_t pitch_wr,
                                              uint64_t blk_rd, uint64_t blk_wr) {
  // tile = 1024 elements = T columns x R rows; 256 threads x 4 elements
  const uint32_t T = 1u << log_t;
  const uint32_t groups = 1u << (log_cols - log_t);
  const uint64_t blk = blockIdx.x / groups;
  const uint32_t col0 = (blockIdx.x % groups) * T;
  uint4 v[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t lam = threadIdx.x + 256 * j;
    const uint32_t c = lam & (T - 1), row = lam >> log_t;
    const uint64_t e = blk * blk_rd + col0 + c + row * pitch_rd;
    v[j][0] = src[2 * e];
    v[j][1] = src[2 * e + 1];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t lam = threadIdx.x + 256 * j;
    const uint32_t c = lam & (T - 1), row = lam >> log_t;
    const uint64_t e = blk * blk_wr + col0 + c + row * pitch_wr;
    uint4 a = v[j][0], b = v[j][1];
    a.x ^= 1u;  // keep the loads live
    dst[2 * e] = a;
    dst[2 * e + 1] = b;
  }
}

struct Case {
  const char* name;
  uint32_t log_r, log_t, log_cols;  // rows per column (= R), columns per WG, columns per block
  uint64_t pitch_rd, pitch_wr;      // row pitch in elements (read, write)
  uint64_t blk_rd, blk_wr;          // block pitch in elements
};

int main() {
  const uint64_t n = 1ull << 24;  // elements of 32 B (512 MiB)
  const uint64_t pad = 64;        // padded pitch: + 64 elements (2 KiB) per row
  uint4 *a, *b;
  CHECK(hipMalloc(&a, (n + (n >> 8) * pad + (1 << 20)) * 32));
  CHECK(hipMalloc(&b, (n + (n >> 8) * pad + (1 << 20)) * 32));
  CHECK(hipMemset(a, 1, n * 32));
  CHECK(hipMemset(b, 0, n * 32));
  std::vector<Case> cs = {
      // contiguous: 1024 consecutive elements per WG (T = 1024 columns of 1 row)
      {"contiguous copy", 0, 10, 24, 0, 0, 0, 0},
      // pass 1: one block of 2^24, R = 256 rows at stride 2^16, T = 4
      {"pass1 2MB stride rd+wr", 8, 2, 16, 1ull << 16, 1ull << 16, 0, 0},
      {"pass1 2MB stride rd, padded wr", 8, 2, 16, 1ull << 16, (1ull << 16) + pad, 0, 0},
      {"pass1 padded rd+wr", 8, 2, 16, (1ull << 16) + pad, (1ull << 16) + pad, 0, 0},
      // pass 2: blocks of 2^16, R = 256 rows at stride 256, T = 4
      {"pass2 8KB stride rd+wr", 8, 2, 8, 256, 256, 1ull << 16, 1ull << 16},
      {"pass2 padded (256+8) rd+wr", 8, 2, 8, 256 + 8, 256 + 8, (1ull << 16) + 2048, (1ull << 16) + 2048},
      // T = 8 variants (256-B runs)
      {"pass1 2MB stride T=8", 7, 3, 17, 1ull << 17, 1ull << 17, 0, 0},
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (const Case& c : cs) {
    const uint64_t per_blk = (1ull << c.log_cols) << c.log_r;
    const uint64_t nblk = n / per_blk;
    const uint32_t grid = (uint32_t)(n / 1024);
    const uint64_t brd = c.blk_rd ? c.blk_rd : per_blk, bwr = c.blk_wr ? c.blk_wr : per_blk;
    const uint64_t prd = c.pitch_rd ? c.pitch_rd : 1, pwr = c.pitch_wr ? c.pitch_wr : 1;
    (void)nblk;
    for (int it = 0; it < 3; ++it)
      hipLaunchKernelGGL(k_cols, dim3(grid), dim3(256), 0, 0, a, b, c.log_r, c.log_t, c.log_cols, prd, pwr, brd, bwr);
    CHECK(hipEventRecord(e0));
    const int reps = 20;
    for (int it = 0; it < reps; ++it)
      hipLaunchKernelGGL(k_cols, dim3(grid), dim3(256), 0, 0, a, b, c.log_r, c.log_t, c.log_cols, prd, pwr, brd, bwr);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("{\"case\": \"%s\", \"ms\": %.4f, \"GBps_rd_wr\": %.1f}\n", c.name, ms, 2.0 * n * 32 / (ms * 1e-3) / 1e9);
  }
  return 0;
}
