// Prime-field arithmetic for the MI355X NTT: N x 32-bit little-endian limbs.
//
// Storage contract (matches the reference's cgbn_mem_t<bits>, cgbn_cuda.h:51-55, loaded with
// mpz_import(order=-1) impl_mpz.cc:1336): limb 0 is least significant, elements are canonical
// (in [0,p)) and NOT in Montgomery form in memory.  N = 8 is the reference's 256-bit element
// (= 4 x 64-bit limbs, byte-identical), N = 12 is the 384-bit (6 x 64-bit limb) template.
//
// The reference multiplies with CGBN: bn2mont(b), bn2mont(w), mont_mul, mont2bn per butterfly
// (big-num.cu:84-88, impl_cuda.cu:980-1024, core_mont.cu:29-77).  Here data stays canonical and
// twiddles are stored pre-multiplied by R = 2^(32N) mod p, so mont_mul(x, w*R) = x*w mod p with a
// single Montgomery product and no per-butterfly conversion.
//
// The product is a coarsely-integrated operand-scanning (CIOS) Montgomery multiply in the
// "no final carry word" form, valid when the top 32-bit limb of p is < 2^31 - 1 (true for
// BN254 Fr, BLS12-381 Fr and the zero-padded P = 469762049).  On gfx950 each 32x32+64 step is one
// v_mad_u64_u32; the carry chains lower to v_add_co_u32 / v_addc_co_u32.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define NTT_HD __host__ __device__ __forceinline__
#else
#define NTT_HD static inline
#endif

namespace ntt {

template <int N>
struct Modulus {
  uint32_t p[N];
  uint32_t pinv;  // -p^{-1} mod 2^32
};

template <int N>
struct alignas(16) Elem {
  uint32_t w[N];
};

// ---------------------------------------------------------------- carry helpers
NTT_HD uint32_t add_cc(uint32_t a, uint32_t b, uint32_t& carry) {
  uint64_t s = (uint64_t)a + b + carry;
  carry = (uint32_t)(s >> 32);
  return (uint32_t)s;
}
NTT_HD uint32_t sub_bb(uint32_t a, uint32_t b, uint32_t& borrow) {
  uint64_t d = (uint64_t)a - b - borrow;
  borrow = (uint32_t)(d >> 63);
  return (uint32_t)d;
}

// r = a + b (no reduction), returns carry out
template <int N>
NTT_HD uint32_t add_raw(uint32_t r[N], const uint32_t a[N], const uint32_t b[N]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = add_cc(a[i], b[i], c);
  return c;
}
// r = a - b (no reduction), returns borrow out
template <int N>
NTT_HD uint32_t sub_raw(uint32_t r[N], const uint32_t a[N], const uint32_t b[N]) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = sub_bb(a[i], b[i], br);
  return br;
}

// a in [0, 2p) -> [0, p)
template <int N>
NTT_HD void reduce_once(uint32_t a[N], const Modulus<N>& M) {
  uint32_t t[N];
  uint32_t br = sub_raw<N>(t, a, M.p);
#pragma unroll
  for (int i = 0; i < N; ++i) a[i] = br ? a[i] : t[i];
}

// r = a + b mod p, inputs canonical, output canonical.  a + b < 2p < 2^(32N) since p's top limb
// is < 2^31.
template <int N>
NTT_HD void add_mod(uint32_t r[N], const uint32_t a[N], const uint32_t b[N], const Modulus<N>& M) {
  uint32_t s[N], t[N];
  add_raw<N>(s, a, b);
  uint32_t br = sub_raw<N>(t, s, M.p);
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = br ? s[i] : t[i];
}

// r = a - b mod p, inputs canonical, output canonical.
template <int N>
NTT_HD void sub_mod(uint32_t r[N], const uint32_t a[N], const uint32_t b[N], const Modulus<N>& M) {
  uint32_t d[N];
  uint32_t br = sub_raw<N>(d, a, b);
  // add p masked by the borrow
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = add_cc(d[i], br ? M.p[i] : 0u, c);
}

// r = a * b * 2^(-32N) mod p.  Inputs canonical (< p); output canonical.
// CIOS, no-carry form (needs p[N-1] < 2^31 - 1).  Portable (host + device) form.
template <int N>
NTT_HD void mont_mul_cios(uint32_t r[N], const uint32_t a[N], const uint32_t b[N], const Modulus<N>& M) {
  uint32_t t[N];
#pragma unroll
  for (int j = 0; j < N; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t bi = b[i];
    uint64_t acc = (uint64_t)a[0] * bi + t[0];
    uint32_t A = (uint32_t)(acc >> 32);
    const uint32_t t0 = (uint32_t)acc;
    const uint32_t m = t0 * M.pinv;
    uint64_t acc2 = (uint64_t)m * M.p[0] + t0;
    uint32_t C = (uint32_t)(acc2 >> 32);
#pragma unroll
    for (int j = 1; j < N; ++j) {
      acc = (uint64_t)a[j] * bi + t[j] + A;
      A = (uint32_t)(acc >> 32);
      acc2 = (uint64_t)m * M.p[j] + (uint32_t)acc + C;
      C = (uint32_t)(acc2 >> 32);
      t[j - 1] = (uint32_t)acc2;
    }
    t[N - 1] = A + C;
  }
  reduce_once<N>(t, M);
#pragma unroll
  for (int j = 0; j < N; ++j) r[j] = t[j];
}

// ---------------------------------------------------------------- gfx950 product scanning
// Column-wise (finely integrated product scanning, FIPS) Montgomery product.  Every 32x32
// partial product is ONE v_mad_u64_u32 into a 64-bit column accumulator whose carry-out (the
// VOP3b sdst) feeds ONE v_addc_co_u32 into a third accumulator word: 2 VALU ops per partial
// product instead of the mad + 64-bit add + zero-extension moves the compiler emits for the
// CIOS form.  2N^2 products + N m-digit multiplies.
struct Acc96 {
  uint64_t lo;   // bits 0..63 of the running column sum
  uint32_t top;  // bits 64..95
};
NTT_HD void mac_vv(Acc96& c, uint32_t x, uint32_t y) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
      : "+v"(c.lo), "=&s"(cc), "+v"(c.top)
      : "v"(x), "v"(y));
#else
  uint64_t p = (uint64_t)x * y;
  uint64_t s = c.lo + p;
  c.top += (s < p);
  c.lo = s;
#endif
}
NTT_HD void mac_vs(Acc96& c, uint32_t x, uint32_t y_sgpr) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
      : "+v"(c.lo), "=&s"(cc), "+v"(c.top)
      : "v"(x), "s"(y_sgpr));
#else
  mac_vv(c, x, y_sgpr);
#endif
}
NTT_HD void acc_shift(Acc96& c) {
  c.lo = (c.lo >> 32) | ((uint64_t)c.top << 32);
  c.top = 0;
}

template <int N>
NTT_HD void mont_mul_fips(uint32_t r[N], const uint32_t a[N], const uint32_t b[N],
                                              const Modulus<N>& M) {
  uint32_t m[N];
  Acc96 c{0, 0};
#pragma unroll
  for (int i = 0; i < N; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      mac_vv(c, a[j], b[i - j]);
      mac_vs(c, m[j], M.p[i - j]);
    }
    mac_vv(c, a[i], b[0]);
    m[i] = (uint32_t)c.lo * M.pinv;
    mac_vs(c, m[i], M.p[0]);
    acc_shift(c);
  }
#pragma unroll
  for (int i = N; i < 2 * N; ++i) {
#pragma unroll
    for (int j = i - N + 1; j < N; ++j) {
      mac_vv(c, a[j], b[i - j]);
      mac_vs(c, m[j], M.p[i - j]);
    }
    r[i - N] = (uint32_t)c.lo;
    acc_shift(c);
  }
  reduce_once<N>(r, M);
}

// Dispatch: the asm product-scanning form on the device, CIOS on the host.
template <int N>
NTT_HD void mont_mul(uint32_t r[N], const uint32_t a[N], const uint32_t b[N], const Modulus<N>& M) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(NTT_FORCE_CIOS)
  mont_mul_fips<N>(r, a, b, M);
#else
  mont_mul_cios<N>(r, a, b, M);
#endif
}

template <int N>
NTT_HD bool is_zero(const uint32_t a[N]) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) o |= a[i];
  return o == 0;
}

}  // namespace ntt
