// Kernel-facing argument structs and launcher declarations (host + device).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "ntt_device.hpp"

namespace ntt {

enum : int { KIND_COLUMN = 0, KIND_FINAL = 1, KIND_SINGLE = 2 };

// Elements per workgroup tile: 2048 x 32 B = 64 KiB of LDS (two workgroups per CU); the 384-bit
// template halves the tile to keep the same LDS footprint.
__host__ __device__ constexpr int tile_elems(int N) { return N >= 12 ? 1024 : 2048; }
__host__ __device__ constexpr int tile_log(int N) { return N >= 12 ? 10 : 11; }

template <int N>
struct PassArgs {
  FieldArgs<N> F;
  const uint32_t* tw_int;  // w_R^e, e < R (this pass's radix), Montgomery form
  const uint32_t* tw_lo;   // outer twiddles w_n^e = tw_lo[e mod 2^lo_bits] * tw_hi[e >> lo_bits]
  const uint32_t* tw_hi;
  uint32_t lo_bits;
  uint32_t log_n;
  uint32_t log_blk;  // column pass: log2 of the block length N_i
  uint32_t log_m;    // column pass: log2(n / N_i)
  uint32_t r1;       // final pass: log2 R_1
  uint32_t nmid;     // final pass: number of middle digits (p - 2)
  uint32_t mid_bits[4];  // final pass: middle digit widths, least significant (k_{p-1}) first
  uint32_t mid_off[4];   // final pass: output bit offset (relative to R_1) of those digits
  uint32_t flags;        // bit 0: multiply outputs by ninv (single-pass inverse)
  uint32_t ninv[N];      // n^-1 in Montgomery form
  size_t batch_stride;   // 32-bit words between batched transforms
};

template <int N, int MEMW>
hipError_t launch_pass(int kind, int logr, const uint32_t* src, uint32_t* dst, const PassArgs<N>& A, uint32_t grid,
                       uint32_t batch, hipStream_t st);
template <int N, int MEMW>
hipError_t launch_naive(const uint32_t* src, uint32_t* dst, const PassArgs<N>& A, uint32_t batch, hipStream_t st);
template <int N, int MEMW>
hipError_t launch_fill(int kind, uint32_t* dst, size_t n, uint64_t seed, uint32_t nrand, uint32_t top_bits,
                       hipStream_t st);
template <int N, int MEMW>
hipError_t launch_pointwise(const uint32_t* a, const uint32_t* b, uint32_t* c, size_t n, const FieldArgs<N>& F,
                            const Elem<N>& r2, hipStream_t st);

}  // namespace ntt
