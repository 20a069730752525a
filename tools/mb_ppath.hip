// HBM microbenchmark of the P469762049 path's access patterns (the SSIP field, 2^26 points), without
// the arithmetic: 8192-element tiles, 1024 threads x 8 elements, load phase -> LDS round trip +
// barrier (as the pass kernels' first exchange) -> store phase.  Elements are 8 B in the caller's
// buffer (long long) and 4 B in the plan scratch.
//
//   pass1   read 8 B at c + 2^18 r (R = 256 rows, T = 32 columns), write 4 B at the same positions
//   pass2   read/write 4 B in blocks of 2^18: c + 2^9 r (R = 512, T = 16: 64-B runs)
//   pass2t  the same with T = 32 (R = 256 per tile, 128-B runs; not a valid schedule, a ceiling)
//   final   read 4 B runs of 512 (T = 16 runs), write 8 B at k1 + 2^8 m + 2^17 k (16 adjacent k1)
//   copy8 / copy4   contiguous copies
//
//   hipcc -O3 --offload-arch=gfx950 tools/mb_ppath.hip -o tools/mb_ppath && tools/mb_ppath
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int NT = 1024, EPT = 8, TILE = NT * EPT;

// element i (< TILE) of tile w -> global index, per pattern
template <int PAT>
__device__ __forceinline__ uint64_t pos(uint32_t w, uint32_t i, bool write) {
  if constexpr (PAT == 0) {  // pass1: T = 32, R = 256, stride 2^18 (one block of 2^26)
    const uint32_t c = i & 31, r = i >> 5;
    return (uint64_t)w * 32 + c + ((uint64_t)r << 18);
  } else if constexpr (PAT == 1) {  // pass2: blocks of 2^18, T = 16, R = 512, stride 2^9
    const uint32_t groups = (1u << 9) / 16;  // column groups per block
    const uint64_t blk = w / groups, col0 = (w % groups) * 16;
    const uint32_t c = i & 15, r = i >> 4;
    return (blk << 18) + col0 + c + ((uint64_t)r << 9);
  } else if constexpr (PAT == 2) {  // pass2t: T = 32, R = 256 (ceiling)
    const uint32_t groups = (1u << 9) / 32;
    const uint64_t blk = w / groups, col0 = (w % groups) * 32;
    const uint32_t c = i & 31, r = i >> 5;
    return (blk << 18) + col0 + c + ((uint64_t)r << 9);
  } else if constexpr (PAT == 3) {  // final: 16 runs of 512 (k1 = k10 + c, mid m), natural write
    const uint32_t m = w & 511, k10 = (w >> 9) * 16;  // 2^9 mids x 16 k1 groups = 8192 tiles
    if (!write) {
      const uint32_t c = i >> 9, j = i & 511;
      return ((uint64_t)(k10 + c) << 18) + ((uint64_t)m << 9) + j;
    }
    const uint32_t c = i & 15, k = i >> 4;  // writes with the 16 adjacent k1 fastest
    return (uint64_t)(k10 + c) + ((uint64_t)m << 8) + ((uint64_t)k << 17);
  } else {  // contiguous
    return (uint64_t)w * TILE + i;
  }
}

template <int PAT, int RB, int WB>
__global__ __launch_bounds__(NT) void k_pat(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst) {
  __shared__ uint32_t lds[TILE];
  const uint32_t w = blockIdx.x, t = threadIdx.x;
  uint32_t v[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const uint64_t p = pos<PAT>(w, t + NT * j, false);
    v[j] = RB == 8 ? reinterpret_cast<const uint2*>(src)[p].x : src[p];
  }
#pragma unroll
  for (int j = 0; j < EPT; ++j) lds[t + NT * j] = v[j] ^ 1u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < EPT; ++j) v[j] = lds[(t * 8 + j) & (TILE - 1)];
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const uint64_t p = pos<PAT>(w, t + NT * j, true);
    if (WB == 8)
      reinterpret_cast<uint2*>(dst)[p] = make_uint2(v[j], 0u);
    else
      dst[p] = v[j];
  }
}

template <int PAT, int RB, int WB>
int run(const char* name, const uint32_t* a, uint32_t* b) {
  const uint64_t n = 1ull << 26;
  const uint32_t grid = (uint32_t)(n / TILE);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int it = 0; it < 5; ++it) hipLaunchKernelGGL((k_pat<PAT, RB, WB>), dim3(grid), dim3(NT), 0, 0, a, b);
  CHECK(hipEventRecord(e0));
  const int reps = 30;
  for (int it = 0; it < reps; ++it) hipLaunchKernelGGL((k_pat<PAT, RB, WB>), dim3(grid), dim3(NT), 0, 0, a, b);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = (double)n * (RB + WB);
  printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

int main() {
  const uint64_t n = 1ull << 26;
  uint32_t *a, *b;
  CHECK(hipMalloc(&a, n * 8));
  CHECK(hipMalloc(&b, n * 8));
  CHECK(hipMemset(a, 1, n * 8));
  CHECK(hipMemset(b, 0, n * 8));
  for (int round = 0; round < 2; ++round) {
    if (run<4, 8, 8>("copy8", a, b) || run<4, 4, 4>("copy4", a, b) || run<0, 8, 4>("pass1 8B->4B T=32 2MB stride", a, b) ||
        run<1, 4, 4>("pass2 4B T=16 (64-B runs)", a, b) || run<2, 4, 4>("pass2 4B T=32 (128-B runs)", a, b) ||
        run<3, 4, 8>("final 4B runs -> 8B natural", a, b))
      return 1;
  }
  return 0;
}
