// Field engines: how an element lives in registers, LDS, HBM and twiddle tables, and the lazy
// butterfly arithmetic on it.  The NTT kernels are generic over the engine.
//
//   Eng29<L, W32[, SCR]>: radix-2^29 limbs (field29.hpp); HBM holds W32 canonical 32-bit words
//                  (cgbn_mem_t<32*W32>, reference cgbn_cuda.h:51-55).  L = 9 / W32 = 8 is the 256-bit
//                  class (BN254 Fr, BLS12-381 Fr, zero-padded P), L = 14 / W32 = 12 the 384-bit
//                  (6 x 64-bit limb) template.
//   Eng32<1>:      one 32-bit limb, HBM holds the reference's `long long` (P469762049 path).
#pragma once
#include "field.hpp"
#include "field29.hpp"
#include "field29_asm9.hpp"

// Debug build (ntt_amd/libntt_debug.so, NTT_DEBUG_CHECKS=1): the pass kernels check every HBM index
// against its buffer, the caller's inputs for canonical form, the lazy bound (< 2p) of every
// intermediate and the canonical form of every output, and record violations in a per-plan status
// word that ntt_plan_device_status reports (bits below).  The product build compiles none of it.
#ifndef NTT_DEBUG_CHECKS
#define NTT_DEBUG_CHECKS 0
#endif
enum : uint32_t {
  NTT_DBG_BOUNDS = 1u << 8,  // an element index outside its buffer (the access is redirected to element 0)
  NTT_DBG_INPUT = 1u << 9,   // a caller input element >= p
  NTT_DBG_LAZY = 1u << 10,   // an intermediate (plan scratch) >= 2p
  NTT_DBG_OUTPUT = 1u << 11  // an output element >= p
};
__device__ __forceinline__ void ntt_dbg_flag(uint32_t* status, uint32_t bit) {
  if (status) __hip_atomic_fetch_or(status, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#ifndef NTT_WAVES_256
#define NTT_WAVES_256 4
#endif
// elements per thread in the pass kernels for the 256-bit class (4: radix-4 register sub-stages, 4
// waves/SIMD; 8: radix-8 sub-stages, 2 waves/SIMD)
#ifndef NTT_EPT_256
#define NTT_EPT_256 4
#endif
#ifndef NTT_256_PASS1_TABLE
#define NTT_256_PASS1_TABLE 1
#endif
#ifndef NTT_P_SCRATCH32
#define NTT_P_SCRATCH32 1
#endif
#ifndef NTT_P_NARROW_FIRST
#define NTT_P_NARROW_FIRST 1
#endif
#ifndef NTT_P_PASS1_TABLE
#define NTT_P_PASS1_TABLE 1
#endif
#ifndef NTT_P_LDS_TW
#define NTT_P_LDS_TW 1
#endif
#ifndef NTT_EPT_P
#define NTT_EPT_P 8  // elements per thread of the P path (16: two radix-8 register groups per thread)
#endif
#ifndef NTT_TILE_LOG_P
#define NTT_TILE_LOG_P 13
#endif
#ifndef NTT_MIN_COLS_LOG_P
#define NTT_MIN_COLS_LOG_P 4
#endif
#ifndef NTT_TILE_LOG_256
#define NTT_TILE_LOG_256 10
#endif

namespace ntt {

// 16-B write-through vector store (sc1: the line leaves this XCD's L2 at once, so a workgroup on any
// XCD that acquires after the publishing counter reads it fresh; MI355X_MICROARCH.md § visibility,
// the R1 publish form).  The compiler does not count inline-asm stores: the publisher drains them
// with an explicit s_waitcnt vmcnt(0) before it signals.  s_nop 1: the store-data VGPR hazard.
__device__ __forceinline__ void store_wt16(uint4* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u v = {a, b, c, d};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// ------------------------------------------------------------------------------ 29-bit engine
// Twiddles are multiplied with Shoup's precomputed-quotient product (mulc29): a table entry holds
// the canonical w and ws = floor(w * B / p), B = 2^(29L).  143 MADs per product for L = 9 instead
// of the Montgomery product's 162, measured 14-18 % faster per product on MI355X
// (profiles/r01_mb_mont29_v2.txt).  Element x twiddle products are < 3p for any input < B.
//
// Lazy bounds (units of p): the in-register DFTs take inputs < IN p (IN = 4: products < 3p,
// reduced k = 0 outputs < 4p, HBM loads < p) and radix-2 stage s adds/subtracts with offset
// IN 2^(s-1) p, so a Q-point DFT returns values < IN Q p <= 32p < B for every supported field.
template <int L, int W32, int SCR_ = 0, int TL_ = 0>
struct Eng29 {
  static constexpr int W = L;                   // registers per element
  static constexpr int MEMW = W32;              // 32-bit words per element in HBM (canonical)
  // words per element of the plan's own scratch: 256-bit values (< 2p, p < 2^255) need 8 even in the
  // 48-B caller layout, so only the first read and the last write of a transform move 48 B per
  // element.  SCR_ != 0 forces it (Eng256wI: the caller's 48-B element, for NTT_PLAN_IN_PLACE plans,
  // whose intermediates live in the caller's buffer)
  static constexpr int SCRW = SCR_ ? SCR_ : ((L <= 9 && W32 > 8) ? 8 : W32);
  // words per entry of the element-format twiddle tables (values < p: 8 words for the 256-bit class)
  static constexpr int TABW = (L <= 9) ? 8 : W32;
  static constexpr int TW = (2 * L + 3) & ~3;   // words per twiddle-table entry: w, ws (16-B aligned)
  static constexpr int LDSW = L;                // words per element in LDS
  static constexpr int IN = 4;                  // DFT input bound (units of p)
  static constexpr int MUL_OUT = 4;             // bound used for twiddle products (they are < 3p)
  // Pass-kernel shape.  The products are long dependent v_mad_u64_u32 chains, so a SIMD needs 3-4
  // resident waves to keep its VALU busy (Shoup product: 851 SIMD cycles at 2 waves, 785 at 3-4;
  // profiles/r01_mb_mont29_v2.txt).  256-bit class: 4 elements per thread (radix-4 register
  // sub-stages), 1024-element tiles (36 KiB LDS), 4 workgroups = 4 waves per SIMD.  384-bit class:
  // 8 elements per thread, 1024-element tiles, 2 waves per SIMD.
  static constexpr int EPT = (L <= 9) ? NTT_EPT_256 : 8;
  // TL_ != 0 forces the tile: Eng256T's 4096-element tiles (one 1024-thread workgroup, 144 KiB of
  // LDS, per CU), which run 2^20 in two passes (10 + 10) instead of three (7 + 7 + 6)
  static constexpr int TILE_LOG = TL_ ? TL_ : ((L <= 9) ? (EPT == 8 ? 11 : NTT_TILE_LOG_256) : 10);
  static constexpr int WAVES_PER_EU = (L <= 9) ? (EPT == 4 ? NTT_WAVES_256 : 2) : 2;
  static constexpr bool LDS_SPLIT = false;
  // column passes own >= 4 adjacent columns: >= 128-B runs.  The 4096-element tiles also take one
  // column per tile (radix 4096: 2^24 in two passes, 12 + 12, whose 32-B runs meet their three
  // neighbours on one XCD through the XCD-grouped tile order; ntt_plan.cpp make_wide_plan)
  static constexpr int MIN_COLS_LOG = TL_ == 12 ? 0 : 2;
  static constexpr bool PASS1_FULL_TABLE = NTT_256_PASS1_TABLE;  // VALU-bound: a table read beats a second product
  static constexpr bool NARROW_FIRST = false;  // near-equal radices
  // column passes after the first take their outer twiddles as Shoup pairs (w, ws) from L2-resident
  // tables (E::TW words per entry): 143 MADs per product instead of the Montgomery product's 162
  static constexpr bool SHOUP_OUTER = (L == 9);
  // no LDS twiddle staging: a radix-256 table of Shoup pairs (20 KiB) beside the 36-KiB tile would
  // halve the workgroups per CU
  static constexpr bool LDS_TW = false;
  // quotient-estimate reduction needs p's top limb >= 2^18: possible only when 29L - 18 <= 255
  static constexpr bool FASTRED = 29 * L - 18 <= 255;
  struct Tw {
    uint32_t w[L];   // canonical twiddle
    uint32_t ws[L];  // floor(w * B / p)
  };
  struct Args {
    Mod29<L> M;           // p, 2p, -p^-1 mod 2^29 (Montgomery products of two variables)
    uint32_t kp[5][L];    // 2^j p, j = 0..4, normalised: lazy offsets and reductions
    uint32_t pbar[L];     // B - p (Shoup)
    Tw w8[3];             // w_8^1, w_8^2, w_8^3
    Tw ninv;              // n^-1
    float red_inv;        // 1 / (p_top + 1) rounded down (quotient-estimate reduction)
    uint32_t red_ok;      // p_top >= 2^18: the top-limb quotient estimate is within 1
    uint32_t pc[5][L];    // padded offsets K p for the unnormalised butterflies (PC_* below)
    uint32_t* dbg;        // debug builds: the plan's status word (NTT_DBG_*); null otherwise
  };
  // debug builds: x < q (x any limb representation of a non-negative value, q normalised)
  __device__ static bool dbg_below(const uint32_t (&x)[W], const uint32_t (&q)[L]) {
    uint32_t y[W];
#pragma unroll
    for (int i = 0; i < W; ++i) y[i] = x[i];
    norm_u<L>(y);
    for (int i = L - 1; i >= 0; --i)
      if (y[i] != q[i]) return y[i] < q[i];
    return false;
  }
  __device__ static bool dbg_canonical(const uint32_t (&x)[W], const Args& A) { return dbg_below(x, A.kp[0]); }
  // Padded offsets: value K p, limbs c_0 = kp_0 + P, c_i = kp_i + P - P/2^29 (0 < i < 8),
  // c_8 = kp_8 - P/2^29, so that c_i >= P > b_i for limb bound P and a - b + C never goes negative
  // limb-wise; K = (value bound of b) + 1 keeps the top limb non-negative when p_top >= 3.
  enum : int { PC_5_29 = 0, PC_9_30 = 1, PC_4_29 = 2, PC_17_29 = 3, PC_7_30 = 4 };

  // The 256-bit class in the 48-B layout (W32 = 12) reads only the first 32 B of an element: its
  // values (canonical inputs < p < 2^255, lazy intermediates < 2p) leave words 8..11 zero.  Holding
  // 12 words per element in flight spilled 48 B per thread in pass 1 (12 B with 8 words).  The
  // checked build reads all 48 B, so a non-canonical input still raises its flag.
  template <int MW = W32>
  __device__ static __forceinline__ void load(uint32_t (&x)[W], const uint32_t* __restrict__ base, size_t idx) {
    constexpr int MR = (L <= 9 && MW > 8 && !NTT_DEBUG_CHECKS) ? 8 : MW;
    uint32_t w[MW];
    const uint4* p = reinterpret_cast<const uint4*>(base + idx * MW);
#pragma unroll
    for (int q = 0; q < MW / 4; ++q) {
      if (4 * q < MR) {
        const uint4 v = p[q];
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
      } else {
        w[4 * q] = w[4 * q + 1] = w[4 * q + 2] = w[4 * q + 3] = 0u;
      }
    }
    pack29<L, MW>(x, w);
  }
  // x < FROM p (power of two) -> x < TO p by conditional subtractions of FROM/2 p, ..., TO p
  template <int FROM, int TO>
  __device__ static __forceinline__ void reduce_chain(uint32_t (&x)[W], const Args& A) {
    static_assert(FROM <= 32 && TO >= 1, "lazy bound");
    if constexpr (FROM > TO) {
      constexpr int j = __builtin_ctz(FROM / 2);
      cond_sub<L>(x, A.kp[j]);
      reduce_chain<FROM / 2, TO>(x, A);
    }
  }
  // x < 64p -> [0, 2p): x - q p with q = floor(x_top / (p_top + 1)) (float estimate biased low by
  // 2^-15, more than its worst rounding overshoot 2^-17.9), which is floor(x / p) or one less when
  // p_top >= 2^18; it is one less only when x / p is within ~2^-14 below an integer, so the result
  // is < p for all but ~2^-14 of inputs.  x - q p = (x + q pbar) mod B.  9 MADs + ~30 simple ops
  // instead of up to four conditional subtractions.
  // The carry stays 32-bit: q <= 64 and pbar_i < 2^29, so every column is < 2^35.2 and its carry
  // c < 2^6.2; x_i + c < 2^32 for the input limbs (< 2^31.6).  Per limb one 32-bit add, one MAD
  // (q pbar_i + (x_i + c)), a mask and one v_alignbit (the carry) -- instead of a 64-bit shift and a
  // 64-bit add of the zero-extended limb, whose register pairs cost the compiler extra moves.
  // R32 = false: the 64-bit-carry form, which needs fewer registers (the column passes run at the
  // 128-VGPR cap, where the 32-bit form spills and measured 3.6 % slower in pass 1).
  template <bool R32 = true>
  __device__ static __forceinline__ void reduce_top(uint32_t (&x)[W], const Args& A) {
    const float qf = __builtin_fmaf((float)x[L - 1], A.red_inv, -0x1p-15f);
    const uint32_t q = qf > 0.f ? (uint32_t)qf : 0u;
    if constexpr (R32) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const uint64_t acc = (uint64_t)q * A.pbar[i] + (uint32_t)(x[i] + c);
      x[i] = (uint32_t)acc & kMask29;
      c = (uint32_t)(acc >> 29);
    }
    } else {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      acc = (acc >> 29) + x[i] + (uint64_t)q * A.pbar[i];
      x[i] = (uint32_t)acc & kMask29;
    }
    }
  }
  // FAST (a kernel template flag, chosen per plan from Args::red_ok): quotient-estimate reduction
  // for the large drops.  A runtime branch here makes the compiler sink the two paths' kp[] uses into
  // one dynamically indexed access and copy the kernel arguments to scratch, hence the template.
  // x < 2q (normalised) -> x < q, skipping the subtraction when no lane of the wave can need it
  // (top limb below q's: x < q for sure).  Wave-uniform branch.
  __device__ static __forceinline__ void cond_sub_rare(uint32_t (&x)[W], const uint32_t (&q)[L]) {
    if (__any(x[L - 1] >= q[L - 1])) cond_sub<L>(x, q);
  }
  template <int FROM, int TO, bool FAST = false, bool R32 = true>
  __device__ static __forceinline__ void reduce(uint32_t (&x)[W], const Args& A) {
    if constexpr (FAST && FROM > 4 && TO <= 4) {
      reduce_top<R32>(x, A);
      if constexpr (TO == 1) cond_sub_rare(x, A.kp[0]);
    } else if constexpr (FAST && FROM == 4 && TO == 2) {
      cond_sub_rare(x, A.kp[1]);  // products: < 1.6p for BN254 Fr, < 2.4p for BLS12-381 Fr
    } else {
      reduce_chain<FROM, TO>(x, A);
    }
  }
  // x < BOUND p -> x < 2p (fits the HBM words: p < 2^255) -> HBM.  Between passes only.
  // WT: write-through stores (the fused single-launch schedule hands the tile to other workgroups)
  template <int BOUND, bool FAST = false, int MW = W32, bool WT = false>
  __device__ static __forceinline__ void store_lazy(uint32_t* __restrict__ base, size_t idx, uint32_t (&x)[W],
                                                    const Args& A) {
    reduce<BOUND, 2, FAST>(x, A);
#if NTT_DEBUG_CHECKS
    if (!dbg_below(x, A.kp[1])) ntt_dbg_flag(A.dbg, NTT_DBG_LAZY);
#endif
    put<MW, WT>(base, idx, x);
  }
  // x < BOUND p -> canonical -> HBM
  template <int BOUND, bool FAST = false, int MW = W32>
  __device__ static __forceinline__ void store(uint32_t* __restrict__ base, size_t idx, uint32_t (&x)[W],
                                               const Args& A) {
    reduce<BOUND, 1, FAST>(x, A);
#if NTT_DEBUG_CHECKS
    if (!dbg_below(x, A.kp[0])) ntt_dbg_flag(A.dbg, NTT_DBG_OUTPUT);
#endif
    put<MW>(base, idx, x);
  }
  template <int MW = W32, bool WT = false>
  __device__ static __forceinline__ void put(uint32_t* __restrict__ base, size_t idx, const uint32_t (&x)[W]) {
    uint32_t w[MW];
    unpack29<L, MW>(w, x);
    uint4* p = reinterpret_cast<uint4*>(base + idx * MW);
#pragma unroll
    for (int q = 0; q < MW / 4; ++q) {
      if constexpr (WT)
        store_wt16(p + q, w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
      else
        p[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    }
  }
  __device__ static __forceinline__ void tload(Tw& t, const uint32_t* __restrict__ tab, size_t idx) {
    const uint4* p = reinterpret_cast<const uint4*>(tab + idx * TW);
#pragma unroll
    for (int q = 0; q < TW / 4; ++q) {
      const uint4 v = p[q];
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * q + r;
        if (i < L) t.w[i] = vv[r];
        else if (i < 2 * L) t.ws[i - L] = vv[r];
      }
    }
  }
  // x <- x * w mod p, x any value < B (limbs < 2^31): result < 3p
  __device__ static __forceinline__ void mul(uint32_t (&x)[W], const Tw& t, const Args& A) {
    uint32_t r[W];
    if constexpr (L == 9)
      mulc29_a9(r, x, t.w, t.ws, A.pbar);
    else
      mulc29_blk<L>(r, x, t.w, t.ws, A.pbar);
#pragma unroll
    for (int i = 0; i < W; ++i) x[i] = r[i];
  }
  // the same product by a wave-uniform twiddle (the w_8^k constants of the in-register DFTs): its
  // words stay in SGPRs instead of being copied to VGPRs before every product
  __device__ static __forceinline__ void mul_u(uint32_t (&x)[W], const Tw& t, const Args& A) {
    uint32_t r[W];
    if constexpr (L == 9)
      mulc29_a9u(r, x, t.w, t.ws, A.pbar);
    else
      mulc29_blk<L>(r, x, t.w, t.ws, A.pbar);
#pragma unroll
    for (int i = 0; i < W; ++i) x[i] = r[i];
  }
  // x <- x * y / B mod p (Montgomery product of two variables), x < 32p, y < 4p: result < 3p
  __device__ static __forceinline__ void mulv(uint32_t (&x)[W], const uint32_t (&y)[W], const Args& A) {
    uint32_t r[W];
    if constexpr (L == 9)
      mont29_a9(r, x, y, A.M);
    else
      mont29<L>(r, x, y, A.M);
#pragma unroll
    for (int i = 0; i < W; ++i) x[i] = r[i];
  }
  // ---- lazy DIF butterflies: a, b < K p  ->  (a + b, a - b + K p), both < 2K p, normalised.
  __device__ static __forceinline__ void bfly_lk(uint32_t (&a)[W], uint32_t (&b)[W], const uint32_t (&q)[L]) {
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
  __device__ static __forceinline__ void bfly_l(uint32_t (&a)[W], uint32_t (&b)[W], const Args& A) {
    static_assert(K == 4 || K == 8 || K == 16, "lazy bound");
    bfly_lk(a, b, A.kp[__builtin_ctz(K)]);
  }
  template <int K>
  __device__ static __forceinline__ void bfly_w_l(uint32_t (&a)[W], uint32_t (&b)[W], const Tw& t,
                                                  const Args& A) {
    bfly_l<K>(a, b, A);
    mul_u(b, t, A);  // t: one of the w_8^k kernel arguments
  }
  // ---- unnormalised butterflies (FAST engines; limb/value bounds tracked in dft_q_fast)
  template <int CI>
  __device__ static __forceinline__ void bfly_raw(uint32_t (&a)[W], uint32_t (&b)[W], const Args& A) {
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const uint32_t x = a[i], y = b[i];
      a[i] = x + y;
      b[i] = x - y + A.pc[CI][i];
    }
  }
  template <int CI>
  __device__ static __forceinline__ void bfly_raw_w(uint32_t (&a)[W], uint32_t (&b)[W], const Tw& t,
                                                    const Args& A) {
    bfly_raw<CI>(a, b, A);
    mul_u(b, t, A);  // t: one of the w_8^k kernel arguments
  }
  __device__ static __forceinline__ void norm(uint32_t (&x)[W]) {
    norm_u<L>(x);
  }
};

// ------------------------------------------------------------------------------ 32-bit engine
// One 32-bit limb: the P469762049 `long long` path (MEMW = 2), the reference's own field
// (GZKP-NTT.cu:7-8) and any odd modulus p < 2^30.  Values live in [0, 2p) between operations
// (Harvey's lazy butterflies: 4p < 2^32, so a + b and a - b + 2p never wrap) and are canonical in
// the caller's HBM buffers; the plan scratch holds the lazy value.
//   * twiddle x element: Shoup's product with a table entry (w, floor(w 2^32 / p)):
//     q = mulhi(x, w'), r = x w - q p (mod 2^32) in [0, 2p) for any 32-bit x -- 4 VALU ops
//     (v_mul_hi_u32, 2 x v_mul_lo_u32, v_sub_u32);
//   * variable x variable (outer-twiddle tables in the element format, pointwise products):
//     Montgomery with R = 2^32, r = hi(x y) - hi(m p) + p in (0, 2p) for x y < 2^32 p -- 6 ops;
//   * reduction 2p -> p (and 4p -> 2p): min(x, x - p) as unsigned -- 2 ops, no compare.
// The former CIOS / 64-bit-carry form took 127 VALU ops per element in a radix-256 column pass.
template <int N, int MEMW_, int SCR_ = 0>
struct Eng32 {
  static_assert(N == 1, "the 32-bit engine is the 1-limb path (p < 2^30)");
  static constexpr int W = 1;
  static constexpr int MEMW = MEMW_;
  // 1-limb P path: values < 2^31, so the plan's scratch and tables hold 4 B per element where the
  // caller's `long long` layout holds 8 (HBM-bound path: a third less traffic per transform).
  // SCR_ != 0 forces the scratch width (EngPI: the caller's 8 B, for NTT_PLAN_IN_PLACE)
  static constexpr int SCRW = SCR_ ? SCR_ : (NTT_P_SCRATCH32 ? 1 : MEMW_);
  // element-format twiddle tables (w R mod p < 2^31) take 4 B per entry whatever the scratch width:
  // the in-place plan's pass 1 streams a 2^26-entry table at the SSIP size
  static constexpr int TABW = 1;
  static constexpr int TW = 2;  // Shoup pair (w, floor(w 2^32 / p))
  static constexpr int LDSW = 1;
  static constexpr int IN = 4;       // bound hints of the generic kernels (every value here is < 2p)
  static constexpr int MUL_OUT = 4;
  static constexpr int EPT = NTT_EPT_P;
  // 8192-element tiles (32 KiB LDS, 1024 threads) and >= 16 columns per column-pass workgroup, so
  // every HBM run is >= 128 B; 2048-element tiles left 64-B runs at radix 256 and 32-B runs at
  // radix 512 (2.0-3.3 TB/s).
  static constexpr int TILE_LOG = NTT_TILE_LOG_P;
  static constexpr int MIN_COLS_LOG = NTT_MIN_COLS_LOG_P;
  // pass 1 streams its n-entry outer-twiddle table (4 B per entry: +33 % pass-1 bytes) instead of
  // forming the twiddle from the two-level tables: those are 64 KiB + 64 KiB of Shoup pairs gathered
  // per element, and the shorter arithmetic of this engine made pass 1 wait on them (2^26: 307 ->
  // 237 us with the table, profiles/r03_pab/)
  static constexpr bool PASS1_FULL_TABLE = NTT_P_PASS1_TABLE;
  // pass 1 (columns n / R_1 apart) takes a radix one below the rest: twice as wide runs (2^26: 8+9+9)
  static constexpr bool NARROW_FIRST = NTT_P_NARROW_FIRST;
  static constexpr bool SHOUP_OUTER = false;
  // the parallel-load stage (parallel-load.cu:114-193, re-derived): the pass's w_R^e table (R <= 512
  // Shoup pairs) is staged into LDS while the tile's HBM loads are in flight; sub-stages read their
  // twiddles from LDS instead of issuing L1/L2 loads beside the data stream
  static constexpr bool LDS_TW = NTT_P_LDS_TW;
  static constexpr int WAVES_PER_EU = 4;
  static constexpr bool LDS_SPLIT = false;
  static constexpr bool FASTRED = false;
  struct Tw {
    uint32_t w[1];  // canonical w
    uint32_t ws;    // floor(w 2^32 / p)
  };
  struct Args {
    uint32_t p, p2;  // p, 2p
    uint32_t pinv;   // p^-1 mod 2^32 (Montgomery products)
    Tw w8[3];        // w_8^1, w_8^2, w_8^3
    Tw ninv;         // n^-1
    uint32_t* dbg;   // debug builds: the plan's status word (NTT_DBG_*); null otherwise
  };
  __device__ static __forceinline__ uint32_t red(uint32_t x, uint32_t m) {  // x < 2m -> x < m
    return min(x, x - m);
  }
  __device__ static bool dbg_canonical(const uint32_t (&x)[W], const Args& A) { return x[0] < A.p; }
  __device__ static __forceinline__ uint32_t shoup(uint32_t x, uint32_t w, uint32_t ws, uint32_t p) {
    const uint32_t q = __umulhi(x, ws);
    return x * w - q * p;  // [0, 2p)
  }
  template <int MW = MEMW_>
  __device__ static __forceinline__ void load(uint32_t (&x)[W], const uint32_t* __restrict__ base, size_t idx) {
    static_assert(MW == MEMW_ || MW == SCRW || MW == TABW, "HBM width");
    if constexpr (MW == 1)
      x[0] = base[idx];
    else
      x[0] = reinterpret_cast<const uint2*>(base)[idx].x;
  }
  template <int FROM, int TO, bool FAST = false, bool R32 = true>
  __device__ static __forceinline__ void reduce(uint32_t (&)[W], const Args&) {}  // always < 2p
  template <int MW = MEMW_>
  __device__ static __forceinline__ void put(uint32_t* __restrict__ base, size_t idx, uint32_t v) {
    static_assert(MW == MEMW_ || MW == SCRW || MW == TABW, "HBM width");
    if constexpr (MW == 1)
      base[idx] = v;
    else
      reinterpret_cast<uint2*>(base)[idx] = make_uint2(v, 0u);
  }
  // scratch between passes: the lazy value (< 2p < 2^31)
  template <int BOUND, bool FAST = false, int MW = MEMW_, bool WT = false>
  __device__ static __forceinline__ void store_lazy(uint32_t* __restrict__ base, size_t idx, uint32_t (&x)[W],
                                                    [[maybe_unused]] const Args& A) {
    static_assert(!WT, "write-through scratch stores: Eng29 engines only (fused schedule)");
#if NTT_DEBUG_CHECKS
    if (x[0] >= A.p2) ntt_dbg_flag(A.dbg, NTT_DBG_LAZY);
#endif
    put<MW>(base, idx, x[0]);
  }
  // canonical (< p)
  template <int BOUND, bool FAST = false, int MW = MEMW_>
  __device__ static __forceinline__ void store(uint32_t* __restrict__ base, size_t idx, uint32_t (&x)[W],
                                               const Args& A) {
    const uint32_t v = red(x[0], A.p);
#if NTT_DEBUG_CHECKS
    if (v >= A.p) ntt_dbg_flag(A.dbg, NTT_DBG_OUTPUT);
#endif
    put<MW>(base, idx, v);
  }
  __device__ static __forceinline__ void tload(Tw& t, const uint32_t* __restrict__ tab, size_t idx) {
    const uint2 v = reinterpret_cast<const uint2*>(tab)[idx];
    t.w[0] = v.x;
    t.ws = v.y;
  }
  __device__ static __forceinline__ void tload_lds(Tw& t, const uint32_t* lds_tw, uint32_t idx) {
    const uint2 v = reinterpret_cast<const uint2*>(lds_tw)[idx];
    t.w[0] = v.x;
    t.ws = v.y;
  }
  __device__ static __forceinline__ void mul(uint32_t (&x)[W], const Tw& t, const Args& A) {
    x[0] = shoup(x[0], t.w[0], t.ws, A.p);
  }
  __device__ static __forceinline__ void mul_u(uint32_t (&x)[W], const Tw& t, const Args& A) { mul(x, t, A); }
  // x y / 2^32 mod p in (0, 2p) for x y < 2^32 p (x, y < 2p: 4p^2 < 2^32 p)
  __device__ static __forceinline__ void mulv(uint32_t (&x)[W], const uint32_t (&y)[W], const Args& A) {
    const uint32_t lo = x[0] * y[0], hi = __umulhi(x[0], y[0]);
    const uint32_t m = lo * A.pinv;
    x[0] = hi - __umulhi(m, A.p) + A.p;
  }
  // lazy DIF butterfly: a, b < 2p -> (a + b, a - b), both reduced to < 2p
  template <int K>
  __device__ static __forceinline__ void bfly_l(uint32_t (&a)[W], uint32_t (&b)[W], const Args& A) {
    const uint32_t s = a[0] + b[0], d = a[0] - b[0] + A.p2;
    a[0] = red(s, A.p2);
    b[0] = red(d, A.p2);
  }
  template <int K>
  __device__ static __forceinline__ void bfly_w_l(uint32_t (&a)[W], uint32_t (&b)[W], const Tw& t, const Args& A) {
    const uint32_t s = a[0] + b[0], d = a[0] - b[0] + A.p2;  // d < 4p: any 32-bit x is fine for Shoup
    a[0] = red(s, A.p2);
    b[0] = shoup(d, t.w[0], t.ws, A.p);
  }
};

// ------------------------------------------------------------------------------ LDS (any engine)
// An element of LDSW words is split into 16-byte planes ([plane][idx]) plus a 4-byte plane per
// leftover word, so lanes reading consecutive indices hit consecutive slots.
//
// With SPLIT (engines that target 3 waves/SIMD) exchanges run in two rounds over the same buffer:
// part 0 moves planes [0, Q/2) and the leftover words, part 1 planes [Q/2, Q).  Halving the words
// resident at once halves the tile's LDS (40 KiB instead of 72 KiB for a 2048-element 256-bit
// tile), which lets 3 workgroups (3 waves per SIMD) share a CU instead of 2.
template <int LDSW, bool SPLIT>
struct LdsParts {
  static constexpr int Q = LDSW / 4, REM = LDSW - 4 * Q;
  static constexpr int PARTS = (SPLIT && Q >= 2) ? 2 : 1;
  static constexpr int q_lo(int part) { return PARTS == 1 ? 0 : (part == 0 ? 0 : Q / 2); }
  static constexpr int q_hi(int part) { return PARTS == 1 ? Q : (part == 0 ? Q / 2 : Q); }
  static constexpr bool has_rem(int part) { return part == 0; }
  static constexpr int words(int part) { return 4 * (q_hi(part) - q_lo(part)) + (has_rem(part) ? REM : 0); }
  static constexpr int max_words() { return words(0) > words(PARTS - 1) ? words(0) : words(PARTS - 1); }
};

template <int LDSW, bool SPLIT, int E, int PART>
__device__ __forceinline__ void lds_put_part(uint32_t* lds, uint32_t idx, const uint32_t (&x)[LDSW]) {
  using P = LdsParts<LDSW, SPLIT>;
  uint4* l4 = reinterpret_cast<uint4*>(lds);
#pragma unroll
  for (int q = P::q_lo(PART); q < P::q_hi(PART); ++q)
    l4[(q - P::q_lo(PART)) * E + idx] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
  if constexpr (P::has_rem(PART)) {
    uint32_t* l1 = lds + 4 * (P::q_hi(PART) - P::q_lo(PART)) * E;
#pragma unroll
    for (int r = 4 * P::Q; r < LDSW; ++r) l1[(r - 4 * P::Q) * E + idx] = x[r];
  }
}
template <int LDSW, bool SPLIT, int E, int PART>
__device__ __forceinline__ void lds_get_part(uint32_t (&x)[LDSW], const uint32_t* lds, uint32_t idx) {
  using P = LdsParts<LDSW, SPLIT>;
  const uint4* l4 = reinterpret_cast<const uint4*>(lds);
#pragma unroll
  for (int q = P::q_lo(PART); q < P::q_hi(PART); ++q) {
    const uint4 v = l4[(q - P::q_lo(PART)) * E + idx];
    x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
  }
  if constexpr (P::has_rem(PART)) {
    const uint32_t* l1 = lds + 4 * (P::q_hi(PART) - P::q_lo(PART)) * E;
#pragma unroll
    for (int r = 4 * P::Q; r < LDSW; ++r) x[r] = l1[(r - 4 * P::Q) * E + idx];
  }
}

}  // namespace ntt
