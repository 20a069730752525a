// HIP kernels for the MI355X NTT (gfx950).  See DESIGN.md for the decomposition.
//
// A forward transform of n = 2^L elements is p passes of radix R_i = 2^r_i (sum r_i = L):
//   * passes 1..p-1 ("column passes", k_pass<KIND_COLUMN>): in a block of length N_i the element at
//     c + s_i*d (c < s_i = N_i/R_i, d < R_i) takes part in a length-R_i DFT over d; output k is
//     multiplied by w_{N_i}^{c*k} and stored back at c + s_i*k (four-step DIF, in place).  A workgroup
//     owns T = TILE/R_i adjacent columns, so every global access is a T*S-byte contiguous run.
//   * pass p ("final pass", k_pass<KIND_FINAL>): length-R_p DFTs over contiguous runs, written to the
//     digit-reversed (= natural) output position, src -> dst (out of place).  This replaces the
//     reference's SSIP stage-2 mirror-pair trick (GZKP-NTT.cu:1359-1449) with a plan-owned
//     ping-pong buffer: 288 GB of HBM makes an n*S scratch free, and both reads and writes stay
//     fully coalesced.
//   * n <= TILE: one workgroup per transform (k_pass<KIND_SINGLE>).
// Inside a workgroup the R-point DFT is sub-stages of radix 8 (last 2/4/8) in registers with
// LDS exchanges (16-B planes) in between: the wave64 replacement for the reference's shared-memory
// radix-2 rounds (SSIP_NTT_stage1 1297-1357) and its cub::WarpExchange / parallel-load staging.
#pragma once
#include "ntt_device.hpp"
#include "ntt_kernels.hpp"

namespace ntt {

template <int LOGR>
struct Sched {
  static constexpr int nsub = (LOGR + 2) / 3;
  static constexpr int qb(int s) { return (LOGR - 3 * s) >= 3 ? 3 : (LOGR - 3 * s); }
  static constexpr int logN(int s) { return LOGR - 3 * s; }         // log2 N_s
  static constexpr int logsig(int s) { return logN(s) - qb(s); }    // log2 sigma_s
};

// natural index of in-workgroup position pi after all sub-stages (digit reversal)
template <int LOGR>
__device__ __forceinline__ uint32_t natural_index(uint32_t pi) {
  using S = Sched<LOGR>;
  uint32_t k = 0;
#pragma unroll
  for (int s = 0; s < S::nsub; ++s) {
    const uint32_t ks = (pi >> S::logsig(s)) & ((1u << S::qb(s)) - 1);
    k |= ks << (3 * s);
  }
  return k;
}

template <int N>
__device__ __forceinline__ void twiddle_mul(uint32_t (&x)[N], const uint32_t* tab, uint32_t e, const Modulus<N>& M) {
  uint32_t w[N];
  tload<N>(w, tab, e);
  mont_mul<N>(x, x, w, M);
}

// One LDS exchange + in-register radix-Q sub-stage s (s >= 1).
template <int N, int LOGR, int T, int E, int NT, int s>
__device__ __forceinline__ void substage(uint32_t (&x)[8][N], uint32_t (&cl)[4], uint32_t (&pil)[4], uint32_t* lds,
                                         const PassArgs<N>& A, int t) {
  using S = Sched<LOGR>;
  constexpr int pqb = S::qb(s - 1), PQ = 1 << pqb, PG = 8 / PQ, psb = S::logsig(s - 1), plN = S::logN(s - 1);
  if constexpr (s > 1) __syncthreads();  // everyone finished reading the previous exchange
#pragma unroll
  for (int j = 0; j < PG; ++j) {
    const uint32_t g = pil[j];
    const uint32_t rho = g >> psb, cp = g & ((1u << psb) - 1);
#pragma unroll
    for (int k = 0; k < PQ; ++k) {
      const uint32_t pi = (rho << plN) + cp + (k << psb);
      lds_store<N, E>(lds, cl[j] + T * pi, x[j * PQ + brev_bits(k, pqb)]);
    }
  }
  __syncthreads();
  constexpr int qb = S::qb(s), Q = 1 << qb, G = 8 / Q, sb = S::logsig(s), lN = S::logN(s);
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const uint32_t lam = t + NT * j;
    const uint32_t c = lam % T, g = lam / T;
    const uint32_t rho = g >> sb, cp = g & ((1u << sb) - 1);
    cl[j] = c;
    pil[j] = g;
#pragma unroll
    for (int d = 0; d < Q; ++d) {
      const uint32_t pi = (rho << lN) + cp + (d << sb);
      lds_load<N, E>(x[j * Q + d], lds, c + T * pi);
    }
  }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    dft_q<N, Q>(x, j * Q, 1, A.F);
    if constexpr (s + 1 < S::nsub) {
      const uint32_t cp = pil[j] & ((1u << sb) - 1);
#pragma unroll
      for (int k = 1; k < Q; ++k)
        twiddle_mul<N>(x[j * Q + brev_bits(k, qb)], A.tw_int, (cp * k) << (LOGR - lN), A.F.M);
    }
  }
}

template <int N, int MEMW, int LOGR, int KIND>
__global__ __launch_bounds__(256) void k_pass(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                              const PassArgs<N> A) {
  using S = Sched<LOGR>;
  constexpr int E = (KIND == KIND_SINGLE) ? (1 << LOGR) : tile_elems(N);
  constexpr int T = E >> LOGR;  // columns (column pass) or blocks (final / single) per workgroup
  constexpr int NT = E / 8;     // threads
  static_assert(LOGR >= 3 && T >= 1, "radix");
  __shared__ __attribute__((aligned(16))) uint32_t lds[E * N];

  const int t = threadIdx.x;
  if (t >= NT) return;
  const size_t boff = (size_t)blockIdx.y * A.batch_stride;
  src += boff;
  dst += boff;

  // ------------------------------------------------------------------ workgroup geometry
  size_t colbase = 0;       // column pass: first element of this WG's column group
  uint32_t col0 = 0;        // column pass: column index (within block) of local column 0
  uint32_t mid = 0, k10 = 0, midrev = 0;  // final pass
  const uint32_t w = blockIdx.x;
  if constexpr (KIND == KIND_COLUMN) {
    const uint32_t log_s = A.log_blk - LOGR;            // column stride
    const uint32_t groups_log = log_s - __builtin_ctz(T);  // column groups per block (log)
    const size_t blk = w >> groups_log;
    col0 = (w & ((1u << groups_log) - 1)) * T;
    colbase = (blk << A.log_blk) + col0;
  } else if constexpr (KIND == KIND_FINAL) {
    const uint32_t w1_log = A.log_n - A.r1 - LOGR;     // W1 = n / (R_1 R_p)
    mid = w & ((1u << w1_log) - 1);
    k10 = (w >> w1_log) * T;
    uint32_t m = mid;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < (int)A.nmid) {
        const uint32_t d = m & ((1u << A.mid_bits[i]) - 1);
        m >>= A.mid_bits[i];
        midrev |= d << A.mid_off[i];
      }
    }
  }
  const uint32_t log_s = (KIND == KIND_COLUMN) ? (A.log_blk - LOGR) : 0u;

  uint32_t x[8][N];
  // per-slot bookkeeping for the last sub-stage
  uint32_t cl[4];   // local column/block of each group (<= 4 groups per thread)
  uint32_t pil[4];  // group index of each group

  // ------------------------------------------------------------------ sub-stage 0: global -> regs
  {
    constexpr int qb = S::qb(0), Q = 1 << qb, G = 8 / Q, sb = S::logsig(0);
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const uint32_t lam = t + NT * j;
      uint32_t c, g;
      if constexpr (KIND == KIND_COLUMN) {
        c = lam % T;
        g = lam / T;
      } else {
        g = lam & ((1u << sb) - 1);
        c = lam >> sb;
      }
      cl[j] = c;
      pil[j] = g;
#pragma unroll
      for (int d = 0; d < Q; ++d) {
        const uint32_t pi = g + (d << sb);
        size_t pos;
        if constexpr (KIND == KIND_COLUMN) {
          pos = colbase + c + ((size_t)pi << log_s);
        } else if constexpr (KIND == KIND_FINAL) {
          const size_t beta = ((size_t)(k10 + c) << (A.log_n - A.r1 - LOGR)) + mid;
          pos = (beta << LOGR) + pi;
        } else {
          pos = pi;
        }
        gload<N, MEMW>(x[j * Q + d], src, pos);
      }
      dft_q<N, Q>(x, j * Q, 1, A.F);
      if constexpr (S::nsub > 1) {
#pragma unroll
        for (int k = 1; k < Q; ++k) twiddle_mul<N>(x[j * Q + brev_bits(k, qb)], A.tw_int, g * k, A.F.M);
      }
    }
  }

  // ------------------------------------------------------------------ sub-stages 1..nsub-1 via LDS
  if constexpr (S::nsub > 1) substage<N, LOGR, T, E, NT, 1>(x, cl, pil, lds, A, t);
  if constexpr (S::nsub > 2) substage<N, LOGR, T, E, NT, 2>(x, cl, pil, lds, A, t);
  if constexpr (S::nsub > 3) substage<N, LOGR, T, E, NT, 3>(x, cl, pil, lds, A, t);

  // ------------------------------------------------------------------ output
  {
    constexpr int ls = S::nsub - 1;
    constexpr int qb = S::qb(ls), Q = 1 << qb, G = 8 / Q, sb = S::logsig(ls), lN = S::logN(ls);
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const uint32_t g = pil[j];
      const uint32_t rho = g >> sb, cp = g & ((1u << sb) - 1);
      const uint32_t c = cl[j];
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        uint32_t(&v)[N] = x[j * Q + brev_bits(k, qb)];
        const uint32_t pi = (rho << lN) + cp + (k << sb);
        const uint32_t kn = natural_index<LOGR>(pi);
        size_t pos;
        if constexpr (KIND == KIND_COLUMN) {
          // outer twiddle w_{N_i}^{col * kn} = w_n^{(col * kn) << log_m}, two-level table
          const size_t e = ((size_t)(col0 + c) * kn) << A.log_m;
          uint32_t tl[N], th[N];
          tload<N>(tl, A.tw_lo, (uint32_t)(e & ((1u << A.lo_bits) - 1)));
          tload<N>(th, A.tw_hi, (uint32_t)(e >> A.lo_bits));
          mont_mul<N>(tl, tl, th, A.F.M);
          mont_mul<N>(v, v, tl, A.F.M);
          pos = colbase + c + ((size_t)kn << log_s);
        } else if constexpr (KIND == KIND_FINAL) {
          pos = (size_t)(k10 + c) + ((size_t)midrev << A.r1) + ((size_t)kn << (A.log_n - LOGR));
        } else {
          if (A.flags & 1u) mont_mul<N>(v, v, A.ninv, A.F.M);
          pos = kn;
        }
        gstore<N, MEMW>(dst, pos, v);
      }
    }
  }
}

// O(n^2) transform for tiny n (n <= 4): X_k = sum_j x_j w^(jk); tw holds w^e, e < n (Montgomery).
template <int N, int MEMW>
__global__ void k_dft_naive(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, const PassArgs<N> A) {
  const uint32_t n = 1u << A.log_n;
  const uint32_t k = threadIdx.x;
  const size_t boff = (size_t)blockIdx.y * A.batch_stride;
  if (k >= n) return;
  uint32_t acc[N];
#pragma unroll
  for (int i = 0; i < N; ++i) acc[i] = 0;
  for (uint32_t j = 0; j < n; ++j) {
    uint32_t v[N], w[N];
    gload<N, MEMW>(v, src + boff, j);
    tload<N>(w, A.tw_int, (j * k) & (n - 1));
    mont_mul<N>(v, v, w, A.F.M);
    add_mod<N>(acc, acc, v, A.F.M);
  }
  if (A.flags & 1u) mont_mul<N>(acc, acc, A.ninv, A.F.M);
  __syncthreads();  // every thread has read src before anyone writes dst (in-place use)
  gstore<N, MEMW>(dst + boff, k, acc);
}

// ---------------------------------------------------------------------------- utility kernels
__device__ __forceinline__ uint64_t splitmix64(uint64_t c) {
  uint64_t z = c + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// SURVEY §8d vector B: limb_i = SplitMix64(seed*2^32 + 4j + i) (64-bit limbs), limbs at and above
// `nrand` zero, the top random limb masked to `top_bits` so that every value is < p.
template <int N, int MEMW>
__global__ void k_fill_random(uint32_t* __restrict__ dst, size_t n, uint64_t seed, uint32_t nrand, uint32_t top_bits) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  uint32_t v[N];
  if constexpr (N == 1) {
    v[0] = (uint32_t)(splitmix64((seed << 32) + 4 * j) & ((1ull << top_bits) - 1));
  } else {
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
      uint64_t limb = 0;
      if ((uint32_t)i < nrand) {
        limb = splitmix64((seed << 32) + 4 * j + i);
        if ((uint32_t)i + 1 == nrand && top_bits < 64) limb &= (1ull << top_bits) - 1;
      }
      v[2 * i] = (uint32_t)limb;
      v[2 * i + 1] = (uint32_t)(limb >> 32);
    }
  }
  gstore<N, MEMW>(dst, j, v);
}

template <int N, int MEMW>
__global__ void k_fill_iota(uint32_t* __restrict__ dst, size_t n) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  uint32_t v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = 0;
  v[0] = (uint32_t)j;
  if constexpr (N > 1) v[1] = (uint32_t)((uint64_t)j >> 32);
  gstore<N, MEMW>(dst, j, v);
}

// c = a * b mod p (canonical in/out): mont(mont(a, b), R^2).
template <int N, int MEMW>
__global__ void k_pointwise_mul(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, uint32_t* __restrict__ c,
                                size_t n, const FieldArgs<N> F, const Elem<N> r2) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  uint32_t x[N], y[N];
  gload<N, MEMW>(x, a, j);
  gload<N, MEMW>(y, b, j);
  mont_mul<N>(x, x, y, F.M);
  mont_mul<N>(x, x, r2.w, F.M);
  gstore<N, MEMW>(c, j, x);
}

// ---------------------------------------------------------------------------- launchers
template <int N, int MEMW, int KIND, int LOGR>
static hipError_t launch_pass_r(const uint32_t* src, uint32_t* dst, const PassArgs<N>& A, uint32_t grid, uint32_t batch,
                                hipStream_t st) {
  constexpr int E = (KIND == KIND_SINGLE) ? (1 << LOGR) : tile_elems(N);
  constexpr int NT = E / 8;
  hipLaunchKernelGGL((k_pass<N, MEMW, LOGR, KIND>), dim3(grid, batch), dim3(NT < 64 ? 64 : NT), 0, st, src, dst, A);
  return hipGetLastError();
}

template <int N, int MEMW, int KIND>
static hipError_t launch_pass_k(int logr, const uint32_t* src, uint32_t* dst, const PassArgs<N>& A, uint32_t grid,
                                uint32_t batch, hipStream_t st) {
  constexpr int MAXR = (tile_elems(N) == 2048) ? 11 : 10;
  switch (logr) {
    case 3: return launch_pass_r<N, MEMW, KIND, 3>(src, dst, A, grid, batch, st);
    case 4: return launch_pass_r<N, MEMW, KIND, 4>(src, dst, A, grid, batch, st);
    case 5: return launch_pass_r<N, MEMW, KIND, 5>(src, dst, A, grid, batch, st);
    case 6: return launch_pass_r<N, MEMW, KIND, 6>(src, dst, A, grid, batch, st);
    case 7: return launch_pass_r<N, MEMW, KIND, 7>(src, dst, A, grid, batch, st);
    case 8: return launch_pass_r<N, MEMW, KIND, 8>(src, dst, A, grid, batch, st);
    case 9: return launch_pass_r<N, MEMW, KIND, 9>(src, dst, A, grid, batch, st);
    case 10: return launch_pass_r<N, MEMW, KIND, 10>(src, dst, A, grid, batch, st);
    case 11:
      if constexpr (MAXR >= 11) return launch_pass_r<N, MEMW, KIND, 11>(src, dst, A, grid, batch, st);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

template <int N, int MEMW>
hipError_t launch_pass(int kind, int logr, const uint32_t* src, uint32_t* dst, const PassArgs<N>& A, uint32_t grid,
                       uint32_t batch, hipStream_t st) {
  if (kind == KIND_COLUMN) return launch_pass_k<N, MEMW, KIND_COLUMN>(logr, src, dst, A, grid, batch, st);
  if (kind == KIND_FINAL) return launch_pass_k<N, MEMW, KIND_FINAL>(logr, src, dst, A, grid, batch, st);
  return launch_pass_k<N, MEMW, KIND_SINGLE>(logr, src, dst, A, grid, batch, st);
}

template <int N, int MEMW>
hipError_t launch_naive(const uint32_t* src, uint32_t* dst, const PassArgs<N>& A, uint32_t batch, hipStream_t st) {
  hipLaunchKernelGGL((k_dft_naive<N, MEMW>), dim3(1, batch), dim3(64), 0, st, src, dst, A);
  return hipGetLastError();
}

template <int N, int MEMW>
hipError_t launch_fill(int kind, uint32_t* dst, size_t n, uint64_t seed, uint32_t nrand, uint32_t top_bits,
                       hipStream_t st) {
  const uint32_t blocks = (uint32_t)((n + 255) / 256);
  if (kind == 0)
    hipLaunchKernelGGL((k_fill_iota<N, MEMW>), dim3(blocks), dim3(256), 0, st, dst, n);
  else
    hipLaunchKernelGGL((k_fill_random<N, MEMW>), dim3(blocks), dim3(256), 0, st, dst, n, seed, nrand, top_bits);
  return hipGetLastError();
}

template <int N, int MEMW>
hipError_t launch_pointwise(const uint32_t* a, const uint32_t* b, uint32_t* c, size_t n, const FieldArgs<N>& F,
                            const Elem<N>& r2, hipStream_t st) {
  const uint32_t blocks = (uint32_t)((n + 255) / 256);
  hipLaunchKernelGGL((k_pointwise_mul<N, MEMW>), dim3(blocks), dim3(256), 0, st, a, b, c, n, F, r2);
  return hipGetLastError();
}

#define NTT_INSTANTIATE(N, MEMW)                                                                                  \
  template hipError_t launch_pass<N, MEMW>(int, int, const uint32_t*, uint32_t*, const PassArgs<N>&, uint32_t,    \
                                           uint32_t, hipStream_t);                                                \
  template hipError_t launch_naive<N, MEMW>(const uint32_t*, uint32_t*, const PassArgs<N>&, uint32_t, hipStream_t); \
  template hipError_t launch_fill<N, MEMW>(int, uint32_t*, size_t, uint64_t, uint32_t, uint32_t, hipStream_t);     \
  template hipError_t launch_pointwise<N, MEMW>(const uint32_t*, const uint32_t*, uint32_t*, size_t,               \
                                                const FieldArgs<N>&, const Elem<N>&, hipStream_t);

}  // namespace ntt
