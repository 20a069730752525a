// Radix-2^29 prime-field engine for the 256-bit (L = 9) and 384-bit (L = 14) element classes.
//
// Why 29-bit limbs on gfx950: the only wide multiplier is v_mad_u64_u32 (32x32+64 -> 64, measured
// 4.65 cycles per wave64 instruction, the same issue cost as a 32-bit carry add).  With 29-bit
// limbs a column of the Montgomery product sums at most 2L products of < 2^58 (2L <= 28), which
// never overflows the 64-bit accumulator: every partial product is exactly ONE v_mad_u64_u32 with
// no carry handling, no zero-extension moves and no asm (162 MADs for L = 9, versus 128 MAD + 128
// carry-add + moves for 8 x 32-bit limbs).  See DESIGN.md "Field arithmetic".
//
// Value invariant between operations: limbs normalised (< 2^29), value < 2p ("lazy" residues);
// canonical (< p) only in HBM.  R = 2^(29L) > 16p for every supported field (p < 2^255), so a
// Montgomery product of x < 8p by a canonical twiddle is < 2p.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define F29_HD __host__ __device__ __forceinline__
#else
#define F29_HD static inline
#endif

namespace ntt {

constexpr uint32_t kMask29 = (1u << 29) - 1;

template <int L>
struct Mod29 {
  uint32_t p[L];    // modulus, normalised 29-bit limbs
  uint32_t p2[L];   // 2p, normalised
  uint32_t pinv;    // -p^-1 mod 2^29
};

// unsigned carry normalisation: limbs may exceed 2^29 (non-negative); top limb keeps the excess
template <int L>
F29_HD void norm_u(uint32_t (&x)[L]) {
#pragma unroll
  for (int i = 0; i + 1 < L; ++i) {
    x[i + 1] += x[i] >> 29;
    x[i] &= kMask29;
  }
}
// signed carry normalisation: limbs hold int32 values; returns the (signed) top limb
template <int L>
F29_HD int32_t norm_s(uint32_t (&x)[L]) {
#pragma unroll
  for (int i = 0; i + 1 < L; ++i) {
    x[i + 1] = (uint32_t)((int32_t)x[i + 1] + ((int32_t)x[i] >> 29));
    x[i] &= kMask29;
  }
  return (int32_t)x[L - 1];
}

// x -= q if x >= q (x, q normalised, x < 2q)
template <int L>
F29_HD void cond_sub(uint32_t (&x)[L], const uint32_t (&q)[L]) {
  uint32_t t[L];
#pragma unroll
  for (int i = 0; i < L; ++i) t[i] = x[i] - q[i];
  const bool neg = norm_s<L>(t) < 0;
#pragma unroll
  for (int i = 0; i < L; ++i) x[i] = neg ? x[i] : t[i];
}

// u = a + b mod-lazy: < 2p for a, b < 2p
template <int L>
F29_HD void add29(uint32_t (&u)[L], const uint32_t (&a)[L], const uint32_t (&b)[L], const Mod29<L>& M) {
#pragma unroll
  for (int i = 0; i < L; ++i) u[i] = a[i] + b[i];
  norm_u<L>(u);
  cond_sub<L>(u, M.p2);
}
// d = a - b + 2p (normalised, < 4p) for a, b < 2p
template <int L>
F29_HD void sub29_raw(uint32_t (&d)[L], const uint32_t (&a)[L], const uint32_t (&b)[L], const Mod29<L>& M) {
#pragma unroll
  for (int i = 0; i < L; ++i) d[i] = a[i] - b[i] + M.p2[i];
  norm_s<L>(d);
}
// d = a - b lazily reduced: < 2p
template <int L>
F29_HD void sub29(uint32_t (&d)[L], const uint32_t (&a)[L], const uint32_t (&b)[L], const Mod29<L>& M) {
  sub29_raw<L>(d, a, b, M);
  cond_sub<L>(d, M.p2);
}

// Montgomery product r = a * b * 2^(-29L) mod p (finely-integrated product scanning).
// a: normalised limbs, value < 8p; b: normalised, < p (twiddle) or < 2p.  r: normalised, < 2p.
// Column bound: <= 2L products of < 2^58 plus the carried column (< 2^36): < 2^63 for L <= 14.
template <int L>
F29_HD void mont29(uint32_t (&r)[L], const uint32_t (&a)[L], const uint32_t (&b)[L], const Mod29<L>& M) {
  uint32_t m[L];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      acc += (uint64_t)a[j] * b[i - j];
      acc += (uint64_t)m[j] * M.p[i - j];
    }
    acc += (uint64_t)a[i] * b[0];
    m[i] = ((uint32_t)acc * M.pinv) & kMask29;
    acc += (uint64_t)m[i] * M.p[0];
    acc >>= 29;
  }
#pragma unroll
  for (int i = L; i < 2 * L; ++i) {
#pragma unroll
    for (int j = i - L + 1; j < L; ++j) {
      acc += (uint64_t)a[j] * b[i - j];
      acc += (uint64_t)m[j] * M.p[i - j];
    }
    r[i - L] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
}

// ---------------------------------------------------------------- single-chain MAD helpers
// v_mad_u64_u32 through inline asm: the compiler cannot split a column's accumulation into two
// chains re-joined by a 64-bit add (it does for the plain C++ form: +17 v_lshl_add_u64 per product).
// mad29v: both factors per-lane (VGPR); mad29s: b wave-uniform (an SGPR, e.g. the modulus).
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint64_t mad29v(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint64_t mad29s(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "s"(b), "v"(c));
  return r;
}
#else
static inline uint64_t mad29v(uint32_t a, uint32_t b, uint64_t c) { return c + (uint64_t)a * b; }
static inline uint64_t mad29s(uint32_t a, uint32_t b, uint64_t c) { return c + (uint64_t)a * b; }
#endif

// Chains of 4 / 2 MADs in ONE asm statement: the hazard recognizer pads every inline-asm VALU
// statement with an s_nop, so grouping cuts the pads 4x.  vv: both factors per-lane; vs: second
// factor wave-uniform.
#if defined(__HIP_DEVICE_COMPILE__)
#define NTT_MAD4(C1, C2)                                                                          \
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"                                                   \
      "v_mad_u64_u32 %0, %1, %4, %5, %0\n\t"                                                   \
      "v_mad_u64_u32 %0, %1, %6, %7, %0\n\t"                                                   \
      "v_mad_u64_u32 %0, %1, %8, %9, %0"                                                       \
      : "+v"(acc), "=&s"(cc)                                                                    \
      : "v"(a0), C2(b0), "v"(a1), C2(b1), "v"(a2), C2(b2), "v"(a3), C2(b3))
#define NTT_MAD2(C2)                                                                              \
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"                                                   \
      "v_mad_u64_u32 %0, %1, %4, %5, %0"                                                       \
      : "+v"(acc), "=&s"(cc)                                                                    \
      : "v"(a0), C2(b0), "v"(a1), C2(b1))
#define NTT_CV(x) "v"(x)
#define NTT_CS(x) "s"(x)
__device__ __forceinline__ uint64_t mad4vv(uint64_t acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1,
                                           uint32_t a2, uint32_t b2, uint32_t a3, uint32_t b3) {
  uint64_t cc;
  NTT_MAD4(NTT_CV, NTT_CV);
  return acc;
}
__device__ __forceinline__ uint64_t mad4vs(uint64_t acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1,
                                           uint32_t a2, uint32_t b2, uint32_t a3, uint32_t b3) {
  uint64_t cc;
  NTT_MAD4(NTT_CV, NTT_CS);
  return acc;
}
__device__ __forceinline__ uint64_t mad2vv(uint64_t acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1) {
  uint64_t cc;
  NTT_MAD2(NTT_CV);
  return acc;
}
__device__ __forceinline__ uint64_t mad2vs(uint64_t acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1) {
  uint64_t cc;
  NTT_MAD2(NTT_CS);
  return acc;
}
#undef NTT_MAD4
#undef NTT_MAD2
#undef NTT_CV
#undef NTT_CS
#else
static inline uint64_t mad4vv(uint64_t acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2,
                              uint32_t b2, uint32_t a3, uint32_t b3) {
  return acc + (uint64_t)a0 * b0 + (uint64_t)a1 * b1 + (uint64_t)a2 * b2 + (uint64_t)a3 * b3;
}
static inline uint64_t mad4vs(uint64_t acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2,
                              uint32_t b2, uint32_t a3, uint32_t b3) {
  return mad4vv(acc, a0, b0, a1, b1, a2, b2, a3, b3);
}
static inline uint64_t mad2vv(uint64_t acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1) {
  return acc + (uint64_t)a0 * b0 + (uint64_t)a1 * b1;
}
static inline uint64_t mad2vs(uint64_t acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1) {
  return mad2vv(acc, a0, b0, a1, b1);
}
#endif

// acc += sum_{i=lo}^{hi} a[i] * b[k - i] as one MAD chain, in asm groups of 4 / 2 / 1.
// US: b is wave-uniform (SGPR operands).
template <int L, bool US, int lo, int hi>
F29_HD uint64_t mad_span(uint64_t acc, const uint32_t (&a)[L], const uint32_t (&b)[L], int k) {
  if constexpr (hi - lo + 1 >= 4) {
    acc = US ? mad4vs(acc, a[lo], b[k - lo], a[lo + 1], b[k - lo - 1], a[lo + 2], b[k - lo - 2], a[lo + 3],
                      b[k - lo - 3])
             : mad4vv(acc, a[lo], b[k - lo], a[lo + 1], b[k - lo - 1], a[lo + 2], b[k - lo - 2], a[lo + 3],
                      b[k - lo - 3]);
    return mad_span<L, US, lo + 4, hi>(acc, a, b, k);
  } else if constexpr (hi - lo + 1 >= 2) {
    acc = US ? mad2vs(acc, a[lo], b[k - lo], a[lo + 1], b[k - lo - 1])
             : mad2vv(acc, a[lo], b[k - lo], a[lo + 1], b[k - lo - 1]);
    return mad_span<L, US, lo + 2, hi>(acc, a, b, k);
  } else if constexpr (hi - lo + 1 == 1) {
    return US ? mad29s(a[lo], b[k - lo], acc) : mad29v(a[lo], b[k - lo], acc);
  } else {
    return acc;
  }
}

// mulc29 with grouped asm MAD chains (same result as mulc29).
template <int L, int K = L - 2>
F29_HD void mulc29_hi(uint32_t (&q)[L], uint64_t& acc, const uint32_t (&x)[L], const uint32_t (&ws)[L]) {
  if constexpr (K < 2 * L - 1) {
    constexpr int lo = (K - (L - 1) > 0) ? K - (L - 1) : 0, hi = (K < L - 1) ? K : L - 1;
    acc = mad_span<L, false, lo, hi>(acc, x, ws, K);
    if constexpr (K >= L) q[K - L] = (uint32_t)acc & kMask29;
    acc >>= 29;
    mulc29_hi<L, K + 1>(q, acc, x, ws);
  }
}
template <int L, int K = 0>
F29_HD void mulc29_lo(uint32_t (&r)[L], uint64_t& acc, const uint32_t (&x)[L], const uint32_t (&w)[L],
                      const uint32_t (&q)[L], const uint32_t (&pbar)[L]) {
  if constexpr (K < L) {
    acc = mad_span<L, false, 0, K>(acc, x, w, K);
    acc = mad_span<L, true, 0, K>(acc, q, pbar, K);
    r[K] = (uint32_t)acc & kMask29;
    acc >>= 29;
    mulc29_lo<L, K + 1>(r, acc, x, w, q, pbar);
  }
}
template <int L>
F29_HD void mulc29_blk(uint32_t (&r)[L], const uint32_t (&x)[L], const uint32_t (&w)[L], const uint32_t (&ws)[L],
                       const uint32_t (&pbar)[L]) {
  uint32_t q[L];
  uint64_t acc = 0;
  mulc29_hi<L>(q, acc, x, ws);
  q[L - 1] = (uint32_t)acc;
  acc = 0;
  mulc29_lo<L>(r, acc, x, w, q, pbar);
}

// mont29 with every column accumulated in ONE dependent chain (same result as mont29).
template <int L>
F29_HD void mont29_chain(uint32_t (&r)[L], const uint32_t (&a)[L], const uint32_t (&b)[L], const Mod29<L>& M) {
  uint32_t m[L];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int j = 0; j <= i; ++j) acc = mad29v(a[j], b[i - j], acc);
#pragma unroll
    for (int j = 0; j < i; ++j) acc = mad29s(m[j], M.p[i - j], acc);
    m[i] = ((uint32_t)acc * M.pinv) & kMask29;
    acc = mad29s(m[i], M.p[0], acc);
    acc >>= 29;
  }
#pragma unroll
  for (int i = L; i < 2 * L; ++i) {
#pragma unroll
    for (int j = i - L + 1; j < L; ++j) acc = mad29v(a[j], b[i - j], acc);
#pragma unroll
    for (int j = i - L + 1; j < L; ++j) acc = mad29s(m[j], M.p[i - j], acc);
    r[i - L] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
}

// Multiplication by a precomputed constant (Shoup): w < p, ws = floor(w * B / p), B = 2^(29L),
// pbar = B - p (normalised limbs).  q = floor(x * ws / B) is formed from columns >= L-2 of x*ws
// only (the dropped columns sum to < B for x limbs < 2^31, so q is short by at most 1), and
// r = x*w - q*p = (x*w + q*pbar) mod B lies in [0, 3p) for ANY x < B.  143 MADs for L = 9
// (53 + 90) versus 162 for the Montgomery product, and no m = t * pinv multiplies.
template <int L>
F29_HD void mulc29(uint32_t (&r)[L], const uint32_t (&x)[L], const uint32_t (&w)[L], const uint32_t (&ws)[L],
                   const uint32_t (&pbar)[L]) {
  uint32_t q[L];
  uint64_t acc = 0;
#pragma unroll
  for (int k = L - 2; k < 2 * L - 1; ++k) {
#pragma unroll
    for (int i = (k - (L - 1) > 0 ? k - (L - 1) : 0); i <= (k < L - 1 ? k : L - 1); ++i)
      acc = mad29v(x[i], ws[k - i], acc);
    if (k >= L) q[k - L] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
  q[L - 1] = (uint32_t)acc;
  acc = 0;
#pragma unroll
  for (int k = 0; k < L; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) acc = mad29v(x[i], w[k - i], acc);
#pragma unroll
    for (int i = 0; i <= k; ++i) acc = mad29s(q[i], pbar[k - i], acc);
    r[k] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
}

// mulc29 in plain C++ (the compiler schedules the MAD chains; no inline asm)
template <int L>
F29_HD void mulc29_cc(uint32_t (&r)[L], const uint32_t (&x)[L], const uint32_t (&w)[L], const uint32_t (&ws)[L],
                   const uint32_t (&pbar)[L]) {
  uint32_t q[L];
  uint64_t acc = 0;
#pragma unroll
  for (int k = L - 2; k < 2 * L - 1; ++k) {
#pragma unroll
    for (int i = (k - (L - 1) > 0 ? k - (L - 1) : 0); i <= (k < L - 1 ? k : L - 1); ++i)
      acc += (uint64_t)x[i] * ws[k - i];
    if (k >= L) q[k - L] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
  q[L - 1] = (uint32_t)acc;
  acc = 0;
#pragma unroll
  for (int k = 0; k < L; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) acc += (uint64_t)x[i] * w[k - i];
#pragma unroll
    for (int i = 0; i <= k; ++i) acc += (uint64_t)q[i] * pbar[k - i];
    r[k] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
}

// r = a * b mod B (the low L limbs of the product), normalised.  45 MADs for L = 9.
template <int L>
F29_HD void mullo29(uint32_t (&r)[L], const uint32_t (&a)[L], const uint32_t (&b)[L]) {
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < L; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) acc = mad29v(a[i], b[k - i], acc);
    r[k] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
}
// r = (B - a) mod B for normalised a
template <int L>
F29_HD void neg29(uint32_t (&r)[L], const uint32_t (&a)[L]) {
  uint32_t c = 1;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint32_t v = (kMask29 - a[i]) + c;
    r[i] = v & kMask29;
    c = v >> 29;
  }
}
// Shoup companion of a canonical w: ws = floor(w * B / p), from wR = w * B mod p (canonical).
// w * B = ws * p + wR exactly, so ws = (w * B - wR) / p = (-wR) * p^-1 mod B (pinvB = p^-1 mod B).
template <int L>
F29_HD void shoup_ws29(uint32_t (&ws)[L], const uint32_t (&wR)[L], const uint32_t (&pinvB)[L]) {
  uint32_t t[L];
  neg29<L>(t, wR);
  mullo29<L>(ws, t, pinvB);
}
// p^-1 mod B by Newton iteration (host side, plan creation)
template <int L>
F29_HD void inv_mod_B29(uint32_t (&inv)[L], const uint32_t (&p)[L]) {
  uint32_t i0 = 1;
  for (int k = 0; k < 5; ++k) i0 *= 2 - p[0] * i0;  // p^-1 mod 2^32
#pragma unroll
  for (int i = 0; i < L; ++i) inv[i] = 0;
  inv[0] = i0 & kMask29;
  for (int bits = 29; bits < 29 * L; bits *= 2) {  // inv <- inv * (2 - p * inv) mod B
    uint32_t t[L], u[L];
    mullo29<L>(t, p, inv);
    neg29<L>(u, t);
    uint32_t c = 2;  // u += 2
    for (int i = 0; i < L; ++i) {
      const uint32_t v = u[i] + c;
      u[i] = v & kMask29;
      c = v >> 29;
    }
    mullo29<L>(t, inv, u);
    for (int i = 0; i < L; ++i) inv[i] = t[i];
  }
}

// ---------------------------------------------------------------- 32-bit <-> 29-bit limb packing
// canonical little-endian 32-bit words (W32 of them) -> L normalised 29-bit limbs
template <int L, int W32>
F29_HD void pack29(uint32_t (&x)[L], const uint32_t (&w)[W32]) {
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int bit = 29 * i, k = bit / 32, s = bit % 32;
    const uint32_t lo = (k < W32) ? w[k] : 0u;
    const uint32_t hi = (k + 1 < W32) ? w[k + 1] : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
    // one v_alignbit per limb: the 64-bit form let the vectoriser read the words back through a
    // stack copy at a one-word offset (48 B of scratch per thread in the 48-B layout's pass 1)
    x[i] = __builtin_amdgcn_alignbit(hi, lo, (uint32_t)s) & kMask29;
#else
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    x[i] = (uint32_t)(v >> s) & kMask29;
#endif
  }
}
// L normalised 29-bit limbs -> W32 little-endian 32-bit words (value must fit 32*W32 bits)
template <int L, int W32>
F29_HD void unpack29(uint32_t (&w)[W32], const uint32_t (&x)[L]) {
#pragma unroll
  for (int k = 0; k < W32; ++k) {
    const int bit = 32 * k, i = bit / 29, s = bit % 29;
    uint32_t v = (i < L) ? (x[i] >> s) : 0u;
    if (i + 1 < L) v |= x[i + 1] << (29 - s);
    if (i + 2 < L && 58 - s < 32) v |= x[i + 2] << (58 - s);
    w[k] = v;
  }
}

}  // namespace ntt
