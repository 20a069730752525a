// Field engines: how an element lives in registers, LDS, HBM and twiddle tables, and the lazy
// butterfly arithmetic on it.  The NTT kernels are generic over the engine.
//
//   Eng29<L, W32>: radix-2^29 limbs (field29.hpp); HBM holds W32 canonical 32-bit words
//                  (cgbn_mem_t<32*W32>, reference cgbn_cuda.h:51-55).  L = 9 / W32 = 8 is the 256-bit
//                  class (BN254 Fr, BLS12-381 Fr, zero-padded P), L = 14 / W32 = 12 the 384-bit
//                  (6 x 64-bit limb) template.
//   Eng32<1>:      one 32-bit limb, HBM holds the reference's `long long` (P469762049 path).
#pragma once
#include "field.hpp"
#include "field29.hpp"

namespace ntt {

// ------------------------------------------------------------------------------ 29-bit engine
template <int L, int W32>
struct Eng29 {
  static constexpr int W = L;               // registers per element
  static constexpr int MEMW = W32;          // 32-bit words per element in HBM
  static constexpr int TW = (L + 3) & ~3;   // words per twiddle-table entry (16-B aligned)
  static constexpr int LDSW = L;            // words per element in LDS
  struct Args {
    Mod29<L> M;
    uint32_t p4[L], p8[L];  // 4p, 8p (normalised) for the lazy butterflies
    uint32_t w8[3][L];  // w_8^1, w_8^2, w_8^3 (Montgomery, R = 2^(29L))
    uint32_t ninv[L];   // n^-1 (Montgomery)
  };

  __device__ static __forceinline__ void load(uint32_t (&x)[W], const uint32_t* __restrict__ base, size_t idx) {
    uint32_t w[W32];
    const uint4* p = reinterpret_cast<const uint4*>(base + idx * W32);
#pragma unroll
    for (int q = 0; q < W32 / 4; ++q) {
      const uint4 v = p[q];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
    pack29<L, W32>(x, w);
  }
  // x < 2p -> canonical -> HBM
  __device__ static __forceinline__ void store(uint32_t* __restrict__ base, size_t idx, uint32_t (&x)[W],
                                               const Args& A) {
    cond_sub<L>(x, A.M.p);
    uint32_t w[W32];
    unpack29<L, W32>(w, x);
    uint4* p = reinterpret_cast<uint4*>(base + idx * W32);
#pragma unroll
    for (int q = 0; q < W32 / 4; ++q) p[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
  __device__ static __forceinline__ void tload(uint32_t (&x)[W], const uint32_t* __restrict__ tab, uint32_t idx) {
    const uint4* p = reinterpret_cast<const uint4*>(tab + (size_t)idx * TW);
#pragma unroll
    for (int q = 0; q < TW / 4; ++q) {
      const uint4 v = p[q];
      if (4 * q + 0 < L) x[4 * q + 0] = v.x;
      if (4 * q + 1 < L) x[4 * q + 1] = v.y;
      if (4 * q + 2 < L) x[4 * q + 2] = v.z;
      if (4 * q + 3 < L) x[4 * q + 3] = v.w;
    }
  }
  __device__ static __forceinline__ void mul(uint32_t (&x)[W], const uint32_t (&w)[W], const Args& A) {
    uint32_t r[W];
    mont29<L>(r, x, w, A.M);
#pragma unroll
    for (int i = 0; i < W; ++i) x[i] = r[i];
  }
  // ---- lazy DIF butterflies for the in-register DFTs: stage s (1-based) takes inputs < 2^s p and
  // produces (a + b, a - b + K p) with K = 2^s, i.e. outputs < 2^(s+1) p.  Sums and differences are
  // only carry-normalised (no conditional subtraction); values stay far below R = 2^(29L) (16p <
  // 2^259), so every Montgomery product still returns < 2p.  reduce_to_2p() brings the outputs that
  // are not multiplied afterwards back under 2p.
  template <int K>
  __device__ static __forceinline__ const uint32_t (&kp(const Args& A))[L] {
    static_assert(K == 2 || K == 4 || K == 8, "lazy bound");
    if constexpr (K == 2) return A.M.p2;
    else if constexpr (K == 4) return A.p4;
    else return A.p8;
  }
  template <int K>
  __device__ static __forceinline__ void bfly_l(uint32_t (&a)[W], uint32_t (&b)[W], const Args& A) {
    const uint32_t(&q)[L] = kp<K>(A);
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const uint32_t x = a[i], y = b[i];
      a[i] = x + y;
      b[i] = x - y + q[i];
    }
    norm_u<L>(a);
    norm_s<L>(b);
  }
  template <int K>
  __device__ static __forceinline__ void bfly_w_l(uint32_t (&a)[W], uint32_t (&b)[W], const uint32_t (&w)[W],
                                                  const Args& A) {
    bfly_l<K>(a, b, A);
    uint32_t r[W];
    mont29<L>(r, b, w, A.M);
#pragma unroll
    for (int i = 0; i < W; ++i) b[i] = r[i];
  }
  // x < B p -> x < 2p (B a power of two <= 16)
  template <int B>
  __device__ static __forceinline__ void reduce_to_2p(uint32_t (&x)[W], const Args& A) {
    if constexpr (B > 8) cond_sub<L>(x, A.p8);
    if constexpr (B > 4) cond_sub<L>(x, A.p4);
    if constexpr (B > 2) cond_sub<L>(x, A.M.p2);
  }

  // DIF butterflies on lazy residues (< 2p in, < 2p out)
  __device__ static __forceinline__ void bfly(uint32_t (&a)[W], uint32_t (&b)[W], const Args& A) {
    uint32_t u[W], d[W];
    add29<L>(u, a, b, A.M);
    sub29<L>(d, a, b, A.M);
#pragma unroll
    for (int i = 0; i < W; ++i) { a[i] = u[i]; b[i] = d[i]; }
  }
  __device__ static __forceinline__ void bfly_w(uint32_t (&a)[W], uint32_t (&b)[W], const uint32_t (&w)[W],
                                                const Args& A) {
    uint32_t u[W], d[W];
    add29<L>(u, a, b, A.M);
    sub29_raw<L>(d, a, b, A.M);  // < 4p, fine as a Montgomery operand
    mont29<L>(b, d, w, A.M);
#pragma unroll
    for (int i = 0; i < W; ++i) a[i] = u[i];
  }
};

// ------------------------------------------------------------------------------ 32-bit engine
// N x 32-bit limbs, canonical residues, CIOS/FIPS Montgomery (field.hpp).  Used for the 1-limb
// P469762049 `long long` path (MEMW = 2).
template <int N, int MEMW_>
struct Eng32 {
  static constexpr int W = N;
  static constexpr int MEMW = MEMW_;
  static constexpr int TW = N;
  static constexpr int LDSW = N;
  struct Args {
    Modulus<N> M;
    uint32_t w8[3][N];
    uint32_t ninv[N];
  };
  __device__ static __forceinline__ void load(uint32_t (&x)[W], const uint32_t* __restrict__ base, size_t idx) {
    if constexpr (N == 1) {
      x[0] = reinterpret_cast<const uint2*>(base)[idx].x;
    } else {
      const uint4* p = reinterpret_cast<const uint4*>(base + idx * MEMW);
#pragma unroll
      for (int q = 0; q < N / 4; ++q) {
        const uint4 v = p[q];
        x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
      }
    }
  }
  __device__ static __forceinline__ void store(uint32_t* __restrict__ base, size_t idx, uint32_t (&x)[W],
                                               const Args&) {
    if constexpr (N == 1) {
      reinterpret_cast<uint2*>(base)[idx] = make_uint2(x[0], 0u);
    } else {
      uint4* p = reinterpret_cast<uint4*>(base + idx * MEMW);
#pragma unroll
      for (int q = 0; q < N / 4; ++q) p[q] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
    }
  }
  __device__ static __forceinline__ void tload(uint32_t (&x)[W], const uint32_t* __restrict__ tab, uint32_t idx) {
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = tab[(size_t)idx * N + i];
  }
  __device__ static __forceinline__ void mul(uint32_t (&x)[W], const uint32_t (&w)[W], const Args& A) {
    mont_mul<N>(x, x, w, A.M);
  }
  template <int K>
  __device__ static __forceinline__ void bfly_l(uint32_t (&a)[W], uint32_t (&b)[W], const Args& A) {
    bfly(a, b, A);
  }
  template <int K>
  __device__ static __forceinline__ void bfly_w_l(uint32_t (&a)[W], uint32_t (&b)[W], const uint32_t (&w)[W],
                                                  const Args& A) {
    bfly_w(a, b, w, A);
  }
  template <int B>
  __device__ static __forceinline__ void reduce_to_2p(uint32_t (&)[W], const Args&) {}
  __device__ static __forceinline__ void bfly(uint32_t (&a)[W], uint32_t (&b)[W], const Args& A) {
    uint32_t s[W], d[W];
    add_mod<N>(s, a, b, A.M);
    sub_mod<N>(d, a, b, A.M);
#pragma unroll
    for (int i = 0; i < W; ++i) { a[i] = s[i]; b[i] = d[i]; }
  }
  __device__ static __forceinline__ void bfly_w(uint32_t (&a)[W], uint32_t (&b)[W], const uint32_t (&w)[W],
                                                const Args& A) {
    uint32_t s[W], d[W];
    add_mod<N>(s, a, b, A.M);
    sub_mod<N>(d, a, b, A.M);
#pragma unroll
    for (int i = 0; i < W; ++i) a[i] = s[i];
    mont_mul<N>(b, d, w, A.M);
  }
};

// ------------------------------------------------------------------------------ LDS (any engine)
// An element of LDSW words is split into 16-byte planes ([plane][idx]) plus a 4-byte plane per
// leftover word, so lanes reading consecutive indices hit consecutive slots.
template <int LDSW, int E>
__device__ __forceinline__ void lds_put(uint32_t* lds, uint32_t idx, const uint32_t (&x)[LDSW]) {
  constexpr int Q = LDSW / 4;
  uint4* l4 = reinterpret_cast<uint4*>(lds);
#pragma unroll
  for (int q = 0; q < Q; ++q) l4[q * E + idx] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
  uint32_t* l1 = lds + 4 * Q * E;
#pragma unroll
  for (int r = 4 * Q; r < LDSW; ++r) l1[(r - 4 * Q) * E + idx] = x[r];
}
template <int LDSW, int E>
__device__ __forceinline__ void lds_get(uint32_t (&x)[LDSW], const uint32_t* lds, uint32_t idx) {
  constexpr int Q = LDSW / 4;
  const uint4* l4 = reinterpret_cast<const uint4*>(lds);
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const uint4 v = l4[q * E + idx];
    x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
  }
  const uint32_t* l1 = lds + 4 * Q * E;
#pragma unroll
  for (int r = 4 * Q; r < LDSW; ++r) x[r] = l1[(r - 4 * Q) * E + idx];
}

}  // namespace ntt
