// Device building blocks for the MI355X NTT: element load/store, LDS planes, radix-8/4/2 DIF
// butterflies in registers.
//
// Transform definition (reference GZKP-NTT.cu:30-48): X_k = sum_j x_j w^(jk), w = g^((p-1)/n),
// natural order in and out, canonical elements.  Everything here is exact integer arithmetic.
#pragma once
#include "field.hpp"

namespace ntt {

// Kernel-argument field constants (land in SGPRs).
template <int N>
struct FieldArgs {
  Modulus<N> M;
  uint32_t w8[3][N];   // w_8^1, w_8^2 (= w_4), w_8^3 in Montgomery form, w_8 = w_n^(n/8)
  uint32_t one[N];     // R mod p (Montgomery one)
};

// ------------------------------------------------------------------------------- memory
// MEMW = 32-bit words per element in global memory.  N = 8/12: MEMW = N (cgbn_mem_t layout).
// N = 1: MEMW = 2 (the reference's `long long` element, GZKP-NTT.cu:1452, value < 2^31).
template <int N, int MEMW>
__device__ __forceinline__ void gload(uint32_t (&x)[N], const uint32_t* __restrict__ base, size_t idx) {
  if constexpr (N % 4 == 0) {
    const uint4* p = reinterpret_cast<const uint4*>(base + idx * MEMW);
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      uint4 v = p[q];
      x[4 * q + 0] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
  } else {
    static_assert(N == 1 && MEMW == 2, "unsupported element layout");
    uint2 v = reinterpret_cast<const uint2*>(base)[idx];
    x[0] = v.x;
  }
}
template <int N, int MEMW>
__device__ __forceinline__ void gstore(uint32_t* __restrict__ base, size_t idx, const uint32_t (&x)[N]) {
  if constexpr (N % 4 == 0) {
    uint4* p = reinterpret_cast<uint4*>(base + idx * MEMW);
#pragma unroll
    for (int q = 0; q < N / 4; ++q) p[q] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
  } else {
    reinterpret_cast<uint2*>(base)[idx] = make_uint2(x[0], 0u);
  }
}
// Table entries (twiddles) are dense N-word Montgomery values.
template <int N>
__device__ __forceinline__ void tload(uint32_t (&x)[N], const uint32_t* __restrict__ tab, uint32_t idx) {
  if constexpr (N % 4 == 0) {
    const uint4* p = reinterpret_cast<const uint4*>(tab + (size_t)idx * N);
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      uint4 v = p[q];
      x[4 * q + 0] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
  } else {
    x[0] = tab[idx];
  }
}

// LDS: an element is split into 16-byte planes ([plane][idx]) so that lanes reading consecutive
// indices hit consecutive 16-B slots (conflict-free ds_read_b128 / ds_write_b128).
template <int N>
struct Planes {
  static constexpr int P = (N % 4 == 0) ? N / 4 : 1;
};
template <int N, int E>
__device__ __forceinline__ void lds_store(uint32_t* lds, uint32_t idx, const uint32_t (&x)[N]) {
  if constexpr (N % 4 == 0) {
    uint4* l = reinterpret_cast<uint4*>(lds);
#pragma unroll
    for (int q = 0; q < N / 4; ++q) l[q * E + idx] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
  } else {
    lds[idx] = x[0];
  }
}
template <int N, int E>
__device__ __forceinline__ void lds_load(uint32_t (&x)[N], const uint32_t* lds, uint32_t idx) {
  if constexpr (N % 4 == 0) {
    const uint4* l = reinterpret_cast<const uint4*>(lds);
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      uint4 v = l[q * E + idx];
      x[4 * q + 0] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
  } else {
    x[0] = lds[idx];
  }
}

// ------------------------------------------------------------------------------- butterflies
template <int N>
__device__ __forceinline__ void cpy(uint32_t (&d)[N], const uint32_t (&s)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) d[i] = s[i];
}

// DIF butterfly with twiddle: (a, b) -> (a + b, (a - b) * w), w in Montgomery form.
template <int N>
__device__ __forceinline__ void bfly_w(uint32_t (&a)[N], uint32_t (&b)[N], const uint32_t (&w)[N], const Modulus<N>& M) {
  uint32_t s[N], d[N];
  add_mod<N>(s, a, b, M);
  sub_mod<N>(d, a, b, M);
  cpy<N>(a, s);
  mont_mul<N>(b, d, w, M);
}
// DIF butterfly without twiddle.
template <int N>
__device__ __forceinline__ void bfly(uint32_t (&a)[N], uint32_t (&b)[N], const Modulus<N>& M) {
  uint32_t s[N], d[N];
  add_mod<N>(s, a, b, M);
  sub_mod<N>(d, a, b, M);
  cpy<N>(a, s);
  cpy<N>(b, d);
}

// In-register DFT of size Q in {2,4,8} over x[base + stride*d], d < Q.  DIF radix-2 network:
// output X_k lands in slot base + stride*brev(k).
template <int N, int Q>
__device__ __forceinline__ void dft_q(uint32_t (&x)[8][N], int base, int stride, const FieldArgs<N>& F) {
  if constexpr (Q == 2) {
    bfly<N>(x[base], x[base + stride], F.M);
  } else if constexpr (Q == 4) {
    bfly<N>(x[base], x[base + 2 * stride], F.M);
    bfly_w<N>(x[base + stride], x[base + 3 * stride], F.w8[1], F.M);
    bfly<N>(x[base], x[base + stride], F.M);
    bfly<N>(x[base + 2 * stride], x[base + 3 * stride], F.M);
  } else {
    static_assert(Q == 8, "radix");
    bfly<N>(x[base], x[base + 4 * stride], F.M);
    bfly_w<N>(x[base + stride], x[base + 5 * stride], F.w8[0], F.M);
    bfly_w<N>(x[base + 2 * stride], x[base + 6 * stride], F.w8[1], F.M);
    bfly_w<N>(x[base + 3 * stride], x[base + 7 * stride], F.w8[2], F.M);
    bfly<N>(x[base], x[base + 2 * stride], F.M);
    bfly_w<N>(x[base + stride], x[base + 3 * stride], F.w8[1], F.M);
    bfly<N>(x[base + 4 * stride], x[base + 6 * stride], F.M);
    bfly_w<N>(x[base + 5 * stride], x[base + 7 * stride], F.w8[1], F.M);
    bfly<N>(x[base], x[base + stride], F.M);
    bfly<N>(x[base + 2 * stride], x[base + 3 * stride], F.M);
    bfly<N>(x[base + 4 * stride], x[base + 5 * stride], F.M);
    bfly<N>(x[base + 6 * stride], x[base + 7 * stride], F.M);
  }
}

__host__ __device__ constexpr int brev_bits(int v, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1) << (bits - 1 - i);
  return r;
}

}  // namespace ntt
