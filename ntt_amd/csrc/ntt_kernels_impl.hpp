// HIP kernels for the MI355X NTT (gfx950), generic over the field engine (engines.hpp).
// See DESIGN.md for the decomposition.
//
// A forward transform of n = 2^L elements is p passes of radix R_i = 2^r_i (sum r_i = L):
//   * passes 1..p-1 ("column passes", KIND_COLUMN): in a block of length N_i the element at
//     c + s_i*d (c < s_i = N_i/R_i, d < R_i) takes part in a length-R_i DFT over d; output k is
//     multiplied by w_{N_i}^{c*k} and stored at c + s_i*k (four-step DIF, in place).  A workgroup
//     owns T = TILE/R_i adjacent columns, so every global access is a T*S-byte contiguous run.
//   * pass p ("final pass", KIND_FINAL): length-R_p DFTs over contiguous runs, written to the
//     digit-reversed (= natural) output position, src -> dst (out of place).  This replaces the
//     reference's SSIP stage-2 mirror-pair trick (GZKP-NTT.cu:1359-1449) with a plan-owned
//     ping-pong buffer: 288 GB of HBM makes an n*S scratch free, and both reads and writes stay
//     fully coalesced.
//   * n <= TILE: one workgroup per transform (KIND_SINGLE).
// Inside a workgroup the R-point DFT is sub-stages of radix 8 (last 2/4/8) in registers with
// LDS exchanges (16-B planes) in between: the wave64 replacement for the reference's shared-memory
// radix-2 rounds (SSIP_NTT_stage1 GZKP-NTT.cu:1297-1357) and its cub::WarpExchange /
// parallel-load staging (test-cub-WarpExchange.cu:6-64, parallel-load.cu:114-193).
#pragma once
#include <cstdlib>
#include <utility>

#include "ntt_kernels.hpp"

namespace ntt {


// Compile-time loop: f(std::integral_constant<int, I>{}) for I in [0, N).  Register arrays indexed
// by I stay in VGPRs (a loop the unroller gives up on would send x[][] to scratch).
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__host__ __device__ constexpr int brev_bits(int v, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1) << (bits - 1 - i);
  return r;
}

// Sub-stage schedule of one radix-2^LOGR pass: register DFTs of radix 2^QB (QB = log2 of the
// elements per thread), the last one smaller when QB does not divide LOGR.
template <int LOGR, int QB>
struct Sched {
  static constexpr int nsub = (LOGR + QB - 1) / QB;
  static constexpr int qb(int s) { return (LOGR - QB * s) >= QB ? QB : (LOGR - QB * s); }
  static constexpr int logN(int s) { return LOGR - QB * s; }      // log2 N_s
  static constexpr int logsig(int s) { return logN(s) - qb(s); }  // log2 sigma_s
};
template <class E>
constexpr int ept_log() { return E::EPT >= 8 ? 3 : (E::EPT == 4 ? 2 : 1); }  // register DFTs of <= 8 points

// natural index of in-workgroup position pi after all sub-stages (digit reversal)
template <int LOGR, int QB>
__device__ __forceinline__ uint32_t natural_index(uint32_t pi) {
  using S = Sched<LOGR, QB>;
  uint32_t k = 0;
#pragma unroll
  for (int s = 0; s < S::nsub; ++s) {
    const uint32_t ks = (pi >> S::logsig(s)) & ((1u << S::qb(s)) - 1);
    k |= ks << (QB * s);
  }
  return k;
}

// In-register DFT of size Q in {2,4,8} over x[base + d], d < Q (DIF radix-2 network): output X_k
// lands in slot base + brev(k).  Lazy bounds (engines.hpp): inputs < IN p, stage s offsets by
// IN 2^(s-1) p, outputs < IN Q p.
template <class E, int Q, int base, int N>
__device__ __forceinline__ void dft_q(uint32_t (&x)[N][E::W], const typename E::Args& F) {
  constexpr int K1 = E::IN, K2 = 2 * E::IN, K3 = 4 * E::IN;
  if constexpr (Q == 2) {
    E::template bfly_l<K1>(x[base], x[base + 1], F);
  } else if constexpr (Q == 4) {
    E::template bfly_l<K1>(x[base], x[base + 2], F);
    E::template bfly_w_l<K1>(x[base + 1], x[base + 3], F.w8[1], F);
    E::template bfly_l<K2>(x[base], x[base + 1], F);
    E::template bfly_l<K2>(x[base + 2], x[base + 3], F);
  } else {
    static_assert(Q == 8, "radix");
    E::template bfly_l<K1>(x[base], x[base + 4], F);
    E::template bfly_w_l<K1>(x[base + 1], x[base + 5], F.w8[0], F);
    E::template bfly_w_l<K1>(x[base + 2], x[base + 6], F.w8[1], F);
    E::template bfly_w_l<K1>(x[base + 3], x[base + 7], F.w8[2], F);
    E::template bfly_l<K2>(x[base], x[base + 2], F);
    E::template bfly_w_l<K2>(x[base + 1], x[base + 3], F.w8[1], F);
    E::template bfly_l<K2>(x[base + 4], x[base + 6], F);
    E::template bfly_w_l<K2>(x[base + 5], x[base + 7], F.w8[1], F);
    E::template bfly_l<K3>(x[base], x[base + 1], F);
    E::template bfly_l<K3>(x[base + 2], x[base + 3], F);
    E::template bfly_l<K3>(x[base + 4], x[base + 5], F);
    E::template bfly_l<K3>(x[base + 6], x[base + 7], F);
  }
}

// The same DFTs with unnormalised butterflies (FAST Eng29 engines): limbs grow past 29 bits and are
// carry-normalised only where a later stage could overflow 32 bits.  (limb bound, value bound / p)
// per slot, inputs (2^29, 4):
//   Q = 8  stage 1: s (2^30, 8), d (1.5 2^30, 9), d * w -> (2^29, 3)
//          stage 2: x0,x1 (2^31, 16)  x2 (2.5 2^30, 17)  x4 (2^31, 12)  x5 (2^30, 6)  x6 (2.5 2^30, 13)
//          normalise x0 x1 x2 x4 x6; stage 3 outputs <= (2^31, 33)
//   Q = 4  stage 2 outputs <= (2.5 2^30, 17); Q = 2: (1.5 2^30, 9)
// Products accept limbs < 2^31.6 (64-bit column sums) and values < B = 2^261 (33p < 2^260).
template <class E, int Q, int base, int N>
__device__ __forceinline__ void dft_q_fast(uint32_t (&x)[N][E::W], const typename E::Args& F) {
  if constexpr (Q == 2) {
    E::template bfly_raw<E::PC_5_29>(x[base], x[base + 1], F);
  } else if constexpr (Q == 4) {
    E::template bfly_raw<E::PC_5_29>(x[base], x[base + 2], F);
    E::template bfly_raw_w<E::PC_5_29>(x[base + 1], x[base + 3], F.w8[1], F);
    E::template bfly_raw<E::PC_9_30>(x[base], x[base + 1], F);
    E::template bfly_raw<E::PC_4_29>(x[base + 2], x[base + 3], F);
  } else {
    static_assert(Q == 8, "radix");
    E::template bfly_raw<E::PC_5_29>(x[base], x[base + 4], F);
    E::template bfly_raw_w<E::PC_5_29>(x[base + 1], x[base + 5], F.w8[0], F);
    E::template bfly_raw_w<E::PC_5_29>(x[base + 2], x[base + 6], F.w8[1], F);
    E::template bfly_raw_w<E::PC_5_29>(x[base + 3], x[base + 7], F.w8[2], F);
    E::template bfly_raw<E::PC_9_30>(x[base], x[base + 2], F);
    E::template bfly_raw_w<E::PC_9_30>(x[base + 1], x[base + 3], F.w8[1], F);
    E::template bfly_raw<E::PC_4_29>(x[base + 4], x[base + 6], F);
    E::template bfly_raw_w<E::PC_4_29>(x[base + 5], x[base + 7], F.w8[1], F);
    E::norm(x[base]);
    E::norm(x[base + 1]);
    E::norm(x[base + 2]);
    E::norm(x[base + 4]);
    E::norm(x[base + 6]);
    E::template bfly_raw<E::PC_17_29>(x[base], x[base + 1], F);
    E::template bfly_raw<E::PC_4_29>(x[base + 2], x[base + 3], F);
    E::template bfly_raw<E::PC_7_30>(x[base + 4], x[base + 5], F);
    E::template bfly_raw<E::PC_4_29>(x[base + 6], x[base + 7], F);
  }
}
template <class E, int Q, int base, bool FAST, int N>
__device__ __forceinline__ void dft(uint32_t (&x)[N][E::W], const typename E::Args& F) {
  if constexpr (FAST)
    dft_q_fast<E, Q, base>(x, F);
  else
    dft_q<E, Q, base>(x, F);
}

template <class E>
__device__ __forceinline__ void twiddle_mul(uint32_t (&x)[E::W], const uint32_t* tab, uint32_t e,
                                            const typename E::Args& F) {
  typename E::Tw w;
  E::tload(w, tab, e);
  E::mul(x, w, F);
}
// the same from the LDS copy of the table (E::LDS_TW engines: E::TW words per entry)
template <class E>
__device__ __forceinline__ void twiddle_mul_lds(uint32_t (&x)[E::W], const uint32_t* lds_tw, uint32_t e,
                                                const typename E::Args& F) {
  typename E::Tw w;
  E::tload_lds(w, lds_tw, e);
  E::mul(x, w, F);
}

// LDS slot of (local column/block c, in-column position pi): column-minor like HBM, with c XOR-ed
// by the low bits of pi so that both lane orders used (c fastest, or pi fastest) hit distinct
// 16-byte slots (the final pass writes with pi fastest: 8-way conflicts without the swizzle).  A
// swizzle that also removed the wave-uniform sub-stage's read conflicts cost more address VALU than
// the conflicts (+0.8 %).
// One column per tile (T = 1, radix 4096 on 4096-element tiles): consecutive lanes step pi by 1, 4, 16
// or 64, so pi's 16-B slot is XOR-ed by bits 4..7 and 8..11 of pi (tools/lds_t1_sim.py: 0 extra
// cycles per ds_read_b128 and 1.6 per ds_write_b128 against 26 / 22 unswizzled, measured 23).
template <int T>
__device__ __forceinline__ uint32_t lds_slot(uint32_t c, uint32_t pi) {
  if constexpr (T == 1)
    return pi ^ (((pi >> 4) ^ (pi >> 8)) & 15u);
  else
    return (c ^ (pi & (T - 1))) + T * pi;
}

// Wave-uniform trivial twiddles.  Sub-stage s multiplies its outputs k = 1..Q-1 by w^(cp k) with
// cp = g mod sigma_s.  When sigma_s divides the wave count, every cp class is whole waves: wave w
// takes cp = (w + rot) mod sigma_s (rot = the tile index, so that each SIMD -- which holds the same wave
// slot of several workgroups -- gets its share of the cp = 0 waves), and the cp = 0 waves skip their
// products (w^0 = 1) with a scalar branch.  NTT_UNIFORM_CP=0 keeps the lane-order mapping.
#ifndef NTT_UNIFORM_CP
#define NTT_UNIFORM_CP 1
#endif
template <int LOGR, int QB, int NT, int s>
struct Uniform {
  using S = Sched<LOGR, QB>;
  static constexpr int sb = S::logsig(s);
  static constexpr bool on = NTT_UNIFORM_CP && s > 0 && s + 1 < S::nsub && sb >= 1 && (1 << sb) <= NT / 64;
};
// (local column c, group g) of thread t's j-th group in sub-stage s
template <int LOGR, int QB, int T, int NT, int EPT, int s>
__device__ __forceinline__ void sub_map(uint32_t t, int j, uint32_t rot, uint32_t& c, uint32_t& g) {
  using U = Uniform<LOGR, QB, NT, s>;
  if constexpr (U::on) {
    constexpr int sb = U::sb, G = EPT >> Sched<LOGR, QB>::qb(s);
    const uint32_t wave = t >> 6, lane = t & 63;
    const uint32_t cp = (wave + rot) & ((1u << sb) - 1);
    const uint32_t u = ((((wave >> sb) << 6) | lane)) + (uint32_t)(NT >> sb) * (uint32_t)j;
    (void)G;
    c = u % T;
    g = ((u / T) << sb) | cp;
  } else {
    const uint32_t lam = t + NT * j;
    c = lam % T;
    g = lam / T;
  }
}

// One LDS exchange + in-register radix-Q sub-stage s (s >= 1).
template <class E, int LOGR, int T, int TE, int NT, int s, bool FAST, bool R32, bool LTW>
__device__ __forceinline__ void substage(uint32_t (&x)[E::EPT][E::W], uint32_t (&cl)[E::EPT / 2],
                                         uint32_t (&pil)[E::EPT / 2], uint32_t* lds, const PassArgs<E>& A, int t,
                                         const uint32_t* lds_tw, uint32_t rot) {
  using S = Sched<LOGR, ept_log<E>()>;
  constexpr int EPT = E::EPT;
  constexpr int pqb = S::qb(s - 1), PQ = 1 << pqb, PG = EPT / PQ, psb = S::logsig(s - 1), plN = S::logN(s - 1);
  constexpr int qb = S::qb(s), Q = 1 << qb, G = EPT / Q, sb = S::logsig(s), lN = S::logN(s);
  using P = LdsParts<E::LDSW, E::LDS_SPLIT>;
  static_for<P::PARTS>([&](auto PT) {
    constexpr int part = PT;
    if constexpr (s > 1 || part > 0) __syncthreads();  // everyone finished reading the previous round
    static_for<PG>([&](auto J) {
      constexpr int j = J;
      const uint32_t g = pil[j];
      const uint32_t rho = g >> psb, cp = g & ((1u << psb) - 1);
      static_for<PQ>([&](auto K) {
        constexpr int k = K;
        const uint32_t pi = (rho << plN) + cp + (k << psb);
        lds_put_part<E::LDSW, E::LDS_SPLIT, TE, part>(lds, lds_slot<T>(cl[j], pi), x[j * PQ + brev_bits(k, pqb)]);
      });
    });
    __syncthreads();
    static_for<G>([&](auto J) {
      constexpr int j = J;
      uint32_t c, g;
      sub_map<LOGR, ept_log<E>(), T, NT, EPT, s>(t, j, rot, c, g);
      const uint32_t rho = g >> sb, cp = g & ((1u << sb) - 1);
      static_for<Q>([&](auto D) {
        constexpr int d = D;
        const uint32_t pi = (rho << lN) + cp + (d << sb);
        lds_get_part<E::LDSW, E::LDS_SPLIT, TE, part>(x[j * Q + d], lds, lds_slot<T>(c, pi));
      });
    });
  });
  static_for<G>([&](auto J) {
    constexpr int j = J;
    uint32_t c, g;
    sub_map<LOGR, ept_log<E>(), T, NT, EPT, s>(t, j, rot, c, g);
    cl[j] = c;
    pil[j] = g;
  });
  static_for<G>([&](auto J) {
    constexpr int j = J;
    dft<E, Q, j * Q, FAST>(x, A.F);
    if constexpr (s + 1 < S::nsub) {
      E::template reduce<E::IN * Q, E::IN, FAST, R32>(x[j * Q], A.F);  // k = 0: the only output not multiplied
      const uint32_t cp = pil[j] & ((1u << sb) - 1);
      auto twiddles = [&]() {
        static_for<Q - 1>([&](auto K1) {
          constexpr int k = K1 + 1;
          if constexpr (LTW)
            twiddle_mul_lds<E>(x[j * Q + brev_bits(k, qb)], lds_tw, (cp * k) << (LOGR - lN), A.F);
          else
            twiddle_mul<E>(x[j * Q + brev_bits(k, qb)], A.tw_int, (cp * k) << (LOGR - lN), A.F);
        });
      };
      if constexpr (Uniform<LOGR, ept_log<E>(), NT, s>::on) {
        if (__builtin_amdgcn_readfirstlane(cp) == 0) {  // wave-uniform: w^0 = 1, only bring the bounds down
          static_for<Q - 1>([&](auto K1) {
            E::template reduce<E::IN * Q, E::IN, FAST, R32>(x[j * Q + brev_bits(K1 + 1, qb)], A.F);
          });
        } else {
          twiddles();
        }
      } else {
        twiddles();
      }
    }
  });
}

// PRO: load prologue of a fused first column pass (FAST engines with full tables only).
//   PRO_PW:    polynomial multiply.  The pass reads the two forward transforms src and A.src2 and
//              starts from their Montgomery product a b / R_e; R_e is folded into the pass's
//              outer-twiddle table together with n^-1 (PlanImpl::ensure_polymul_table).
//   PRO_COSET: coset forward, x_j <- x_j c^j with j = col + s d: x_j u^d (u = c^s, Shoup table
//              A.tw_in over the in-column index d) and c^col folded into the outer-twiddle table
//              (PlanImpl::coset).
enum : int { PRO_NONE = 0, PRO_PW = 1, PRO_COSET = 2 };
// FSM: four-step addressing (PassArgs::fs) compiled in: 0 = plain batched transforms (every
// product path), 1 = chunk maps / interleave, 2 = the same plus the output twiddle epilogue.
// SHTW: the column pass's full outer-twiddle table holds Shoup pairs (PassArgs::tw_sh).
// Column passes of radix < 2^NTT_COL_R32_BELOW also take the 32-bit-carry reduce_top: below radix
// 256 they fit 122-123 VGPRs with it and no spills (radix 256 spills 28 B), -1.0 % on 2^28's four
// radix-128 passes (profiles/r02_uni/col_r32_ab_*.txt).
#ifndef NTT_COL_R32_BELOW
#define NTT_COL_R32_BELOW 8
#endif
// ---- in-place final pass with the digit reversal fused (NTT_PLAN_IN_PLACE; k_final_ipn below).
// The final pass's outputs of slab `mid` belong in slab `midrev` (the palindromic schedule makes the
// digit reversal an involution), so a tile may store only after every tile of slab midrev has READ
// its elements (an anti-dependency: nothing handed-off is loaded, so no acquire is needed).  Reads
// are counted per slab; the slab's last reader raises the slab's ready word.  Slab m's two words live
// on a 128-B line of their own (ipn_sync[32 (1 + m)]), the ticket / exit / watchdog words on line 0.
template <class E>
__device__ __forceinline__ void ipn_signal_read(const PassArgs<E>& A, uint32_t mid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's loads have returned
  __syncthreads();
  uint32_t* line = A.ipn_sync + 32 * (1 + mid);  // [0] reads done, [1] ready
  if (threadIdx.x == 0 && __hip_atomic_fetch_add(line, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == A.ipn_strips - 1)
    __hip_atomic_store(line + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A wait gave up (Watchdog, ntt_kernels.hpp): the launch's abort word, then the plan's host-mapped
// report word (system scope: the host reads it at the plan's next call without a device query).
__device__ __forceinline__ void watchdog_trip(const Watchdog& wd) {
  if (wd.abort) __hip_atomic_store(wd.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (wd.report) __hip_atomic_store(wd.report, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// One lane's bounded poll of `word` with relaxed agent-scope global loads (no read-modify-write
// polls: DESIGN §4), sleeping S0 below N0 polls, S1 below N1, S2 after.  True once the word is
// non-zero; false when the wait gave up: wd.spins polls without it (this lane trips the watchdog) or
// another workgroup of the launch gave up first (its abort word, checked every 256 polls, is set).
template <int S0, uint32_t N0, int S1, uint32_t N1, int S2>
__device__ __forceinline__ bool poll_bounded(uint32_t* word, const Watchdog& wd) {
  typedef __attribute__((address_space(1))) uint32_t gu32;  // a global (not flat) access
  gu32* const g = (gu32*)word;
  gu32* const ab = (gu32*)wd.abort;
  for (uint32_t spins = 0;; ++spins) {
    if (__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return true;
    if (spins >= wd.spins) {
      watchdog_trip(wd);
      return false;
    }
    if ((spins & 255u) == 255u && ab && __hip_atomic_load(ab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    if (spins < N0) __builtin_amdgcn_s_sleep(S0);
    else if (spins < N1) __builtin_amdgcn_s_sleep(S1);
    else __builtin_amdgcn_s_sleep(S2);
  }
}
// True (workgroup-uniform) once slab midrev has been read; false when the wait gave up, and the tile
// must then not store: its outputs would overwrite elements of midrev that are still unread.
template <class E>
__device__ __forceinline__ bool ipn_wait_mirror(const PassArgs<E>& A, uint32_t midrev) {
  __shared__ uint32_t s_ok;
  if (threadIdx.x == 0)
    s_ok = poll_bounded<4, 8, 32, 8, 32>(A.ipn_sync + 32 * (1 + midrev) + 1, A.wd) ? 1u : 0u;
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(s_ok) != 0u;  // wave-uniform: scalar branches around it
}

// Grid-wide barrier k of a launch (k = 1, 2, ...), the guide's R1 publish (MI355X_MICROARCH.md
// § visibility): every wave drains its (write-through) stores, a workgroup barrier, then one lane's
// agent-scope add.  The arrivals are sharded: workgroup b adds to shard b mod 8 (8 counters, each on a
// 128-B line of its own, cumulative: shard s completes barrier k at k n_s arrivals, n_s = its
// workgroups), and the last arrival of each shard adds to the top counter, whose last arrival (k S,
// S = non-empty shards) raises the barrier's go word.  One counter taking all G arrivals serialises
// them (the guide's fan-in: ~12 ns per atomic, ~12 us at G = 1024); eight shards take them in
// parallel.  The sharding is by block index, so it is correct under any placement; under the observed
// round-robin dealing a shard is one XCD.  Then one lane polls the go word (bounded, Watchdog), ONE
// agent-scope acquire, and the workgroup barrier releases every wave.  False (workgroup-uniform) when
// the wait gave up: the workgroup then skips what is left of the launch.
__device__ __forceinline__ bool grid_barrier_words(uint32_t* top, uint32_t* shards, uint32_t* go, uint32_t k,
                                                   const Watchdog& wd) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores (and loads) are done
  __syncthreads();
  __shared__ uint32_t s_ok;
  if (threadIdx.x == 0) {
    const uint32_t G = gridDim.x, sh = blockIdx.x & 7u;
    const uint32_t ns = (G + 7u - sh) >> 3, nsh = G < 8u ? G : 8u;
    if (__hip_atomic_fetch_add(shards + 32 * sh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k * ns - 1 &&
        __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k * nsh - 1)
      __hip_atomic_store(go, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_ok = poll_bounded<4, 16, 32, 16, 32>(go, wd) ? 1u : 0u;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(s_ok) != 0u;
}
// The in-place single launch's last barrier (the K-th of the launch: 4 in k_fused3bi, 3 in
// k_fused2bi), between every final tile's loads and any store (PassArgs: ipn_sync = the top counter,
// ipn_shards = the shard lines, ipn_go = the go word)
template <uint32_t K, class E>
__device__ __forceinline__ bool ipn_grid_barrier(const PassArgs<E>& A) {
  return grid_barrier_words(A.ipn_sync, A.ipn_shards, A.ipn_go, K, A.wd);
}

// Residency of an in-place single launch (k_fused2bi, k_fused3bi).  Their grid barriers need every
// workgroup resident at once, which a plain launch promises only on a device nobody else holds CUs of
// (another process, or a persistent kernel of the caller's on another stream).  Were a workgroup left
// waiting for a CU, the resident ones would trip the watchdog after pass 1 had already overwritten the
// caller's buffer.  So every workgroup arrives at kernel start (grid barrier 1 of the launch, no wait),
// and before its FIRST store waits until all G have arrived.  The go word is decided once, by
// compare-exchange: the last arrival sets it 0 -> 1 (go), a waiter whose bounded poll ran out sets it
// 0 -> 2 (abandon: no workgroup of the launch stores anything, the caller's buffer is unchanged, and
// the call is reported through the watchdog as NTT_ERR_DEVICE).  Arriving costs one atomic per
// workgroup; the wait is normally satisfied at its first poll, a whole pass-1 tile after the last
// workgroup started.
__device__ __forceinline__ void residency_arrive(uint32_t* top, uint32_t* shards, uint32_t* go) {
  if (threadIdx.x == 0) {
    const uint32_t G = gridDim.x, sh = blockIdx.x & 7u;
    const uint32_t ns = (G + 7u - sh) >> 3, nsh = G < 8u ? G : 8u;
    if (__hip_atomic_fetch_add(shards + 32 * sh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ns - 1 &&
        __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1) {
      uint32_t zero = 0u;
      __hip_atomic_compare_exchange_strong(go, &zero, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
// True (workgroup-uniform) when the launch's go word says go; false when it was abandoned.
__device__ __forceinline__ bool residency_wait(uint32_t* go, const Watchdog& wd) {
  __shared__ uint32_t s_go;
  if (threadIdx.x == 0) {
    typedef __attribute__((address_space(1))) uint32_t gu32;
    uint32_t v = 0;
    for (uint32_t spins = 0;; ++spins) {
      v = __hip_atomic_load((gu32*)go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v) break;
      if (spins >= wd.spins) {
        uint32_t cur = 0u;
        if (__hip_atomic_compare_exchange_strong(go, &cur, 2u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          watchdog_trip(wd);
          v = 2u;
        } else {
          v = cur;  // decided meanwhile
        }
        break;
      }
      if (spins < 16) __builtin_amdgcn_s_sleep(4);
      else __builtin_amdgcn_s_sleep(32);
    }
    s_go = v;
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(s_go) == 1u;
}
// Once a workgroup has passed its residency_wait the go word is final (1 or 2) until the launch's
// last workgroup out clears it: the kernel reads the decision there.
__device__ __forceinline__ bool residency_went(uint32_t* go) {
  __shared__ uint32_t s_go;
  if (threadIdx.x == 0) s_go = __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(s_go) == 1u;
}

// LDS of one pass tile (words), and whether the pass stages its w_R^e table in LDS: E::LDS_TW
// (parallel-load stage), not in a first pass with two-level outer twiddles (the P path's pass 1),
// where it measured slower (profiles/r02_ldstw/)
template <class E, int LOGR, int KIND>
__host__ __device__ constexpr int pass_tile_te() {
  return (KIND == KIND_SINGLE) ? (1 << LOGR) : (1 << tile_log_of<E>());  // KIND_ROWS: TILE / 2^LOGR transforms
}
template <class E, int LOGR, int KIND>
__host__ __device__ constexpr int pass_lds_words() {
  return pass_tile_te<E, LOGR, KIND>() * LdsParts<E::LDSW, E::LDS_SPLIT>::max_words();
}
template <class E, int KIND, bool FULLTW>
__host__ __device__ constexpr bool pass_ltw() {
  return E::LDS_TW && !(KIND == KIND_COLUMN && !FULLTW);
}

// One workgroup tile of one pass: tile w (the workgroup index of a k_pass launch) of transform bq
// (its blockIdx.y).  lds: pass_lds_words() words, lds_tw: 2^LOGR E::TW words when pass_ltw().  k_pass runs
// one tile per workgroup; the fused single-launch schedule (k_fused3) runs several passes' tiles
// in one persistent workgroup.
// LOOPED (persistent workgroups, k_fused3): the thread index is re-read per tile through an opaque
// copy, so that the compiler does not hoist every lane-dependent address out of the tile loop (held in
// VGPRs across the whole loop, they spilled 200-380 B per thread; per tile they cost a few VALU ops).
// IPN (final pass of an in-place plan): outputs go to their natural positions in the same buffer.
// 1 (k_final_ipn): a tile's loads are counted in per slab, and its stores wait until the mirror slab
// has been read.  2 / 3 (k_fused3bi / k_fused2bi, every final tile resident): a grid barrier between
// all loads and all stores.  4 (pass 1 of k_fused3bi / k_fused2bi): the stores wait for the launch's
// residency decision (residency_wait) and are skipped when it was abandoned.
template <class E, int LOGR, int KIND, bool FULLTW, bool FAST, int PRO = PRO_NONE, bool SRC_USER = true,
          int FSM = 0, bool SHTW = false, bool WT = false, bool LOOPED = false, int IPN = 0>
__device__ __forceinline__ void pass_tile(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                          const PassArgs<E>& A, const uint32_t w, const uint32_t bq,
                                          uint32_t* __restrict__ lds, uint32_t* __restrict__ lds_tw) {
  constexpr int QB = ept_log<E>(), EPT = E::EPT;
  using S = Sched<LOGR, QB>;
  constexpr bool COLLIKE = KIND == KIND_COLUMN || KIND == KIND_STOCKHAM || KIND == KIND_DIT;  // column groups
  constexpr bool ROWS = KIND == KIND_ROWS;  // T whole transforms per workgroup: transform w T + c
  constexpr int TE = pass_tile_te<E, LOGR, KIND>();
  constexpr int T = TE >> LOGR;  // columns (column pass) or blocks (final / single) per workgroup
  // reduce_top form (engines.hpp): radix-256 column passes are at the VGPR cap and keep the 64-bit one
  constexpr bool R32 = KIND != KIND_COLUMN || LOGR < NTT_COL_R32_BELOW;
  constexpr int NT = TE / EPT;   // threads
  static_assert(LOGR >= QB && T >= 1, "radix");
  constexpr bool LTW = pass_ltw<E, KIND, FULLTW>();

  // HBM words per element: the caller's buffers hold E::MEMW, the plan's scratch and outer-twiddle
  // tables E::SCRW (8 for 256-bit values in the 48-B layout).  Column passes read the caller's
  // buffer (pass 1, SRC_USER) or scratch and write scratch; the final pass reads scratch.
  // (Stockham passes ping-pong between caller-format buffers: E::MEMW words both ways)
  constexpr int SW = (KIND == KIND_COLUMN) ? (SRC_USER ? E::MEMW : E::SCRW) : (KIND == KIND_FINAL ? E::SCRW : E::MEMW);
  constexpr int DW = (KIND == KIND_COLUMN) ? E::SCRW : E::MEMW;

  int t = threadIdx.x;
  if constexpr (LOOPED) asm volatile("" : "+v"(t));
  if (t >= NT) return;
  // Four-step addressing (PassArgs::fs, ntt_rplan_*): the first pass may read and the last pass may
  // write through the per-peer chunk maps, and Mode I runs 2^il interleaved transforms.  All flags
  // are kernel arguments (wave-uniform branches); fs == 0 is the plain batched transform.
  constexpr bool IN_USER = (KIND == KIND_COLUMN && SRC_USER) || KIND == KIND_SINGLE || ROWS;
  constexpr bool EPI = FSM == 2 && KIND != KIND_COLUMN;
  const bool fs_il = FSM > 0 && (A.fs & FS_IL) != 0;
  const bool map_in = FSM > 0 && IN_USER && (A.fs & FS_MAP_IN);
  const bool map_out = FSM > 0 && KIND != KIND_COLUMN && (A.fs & FS_MAP_OUT);
  // one interleaved transform per workgroup (KIND_ROWS: T adjacent ones, runs of T elements)
  const bool single_il = (KIND == KIND_SINGLE || ROWS) && fs_il;
  const size_t tstride = A.batch_stride / E::MEMW;  // elements between batched transforms
  const size_t bidx = (size_t)bq * tstride;         // first element of this transform (KIND_ROWS: bq = 0)
  if (!map_in && !single_il) src += bidx * SW;
  if (!map_out && !single_il) dst += bidx * DW;
  const size_t boff = bidx * E::MEMW;  // caller-buffer words (src2)
  // input element `pos` of transform b (= bq, or w T + c in KIND_ROWS; Mode I column passes: the
  // interleaved linear index)
  auto in_pos = [&](size_t pos, size_t b) -> size_t {
    if (single_il) pos = (pos << A.il) + b;
    else if (ROWS && !map_in) pos += b * tstride;
    if (!map_in) return pos;
    return A.min(pos, fs_il ? 0 : b);
  };
  // output element (pre-map position as above) -> address; epilogue-table index of the same element
  auto out_pos = [&](size_t pos, size_t b) -> size_t {
    if (single_il) pos = (pos << A.il) + b;
    else if (ROWS && !map_out) pos += b * tstride;
    if (!map_out) return pos;
    return A.mout(pos, fs_il ? 0 : b);
  };
  auto epi_idx = [&](size_t pos, size_t b) -> size_t {
    if (!fs_il) return (b << A.log_n) + pos;
    if (single_il) pos = (pos << A.il) + b;
    return (A.fs & FS_MAP_EPI) ? A.mepi(pos, 0) : pos;
  };
  // debug builds: an index outside its buffer is recorded and redirected to element 0
  auto ck = [&](size_t i, [[maybe_unused]] size_t lim) -> size_t {
#if NTT_DEBUG_CHECKS
    if (i >= lim) {
      ntt_dbg_flag(A.F.dbg, NTT_DBG_BOUNDS);
      return 0;
    }
#endif
    return i;
  };

  // ------------------------------------------------------------------ workgroup geometry
  size_t colbase = 0;  // column pass: first element of this WG's column group
  uint32_t col0 = 0;   // column pass: column index (within block) of local column 0
  uint32_t mid = 0, k10 = 0, midrev = 0;  // final pass
  uint32_t b0 = 0, tb_log = 0;            // final pass, Mode I: first transform, log2 transforms per WG
  if constexpr (COLLIKE) {
    const uint32_t log_s = A.log_blk - LOGR;
    const uint32_t groups_log = log_s - __builtin_ctz(T);  // column groups per block (log)
    const size_t blk = w >> groups_log;
    col0 = (w & ((1u << groups_log) - 1)) * T;
    colbase = (blk << A.log_blk) + col0;
  } else if constexpr (KIND == KIND_FINAL) {
    const uint32_t w1_log = A.log_n - A.r1 - LOGR;  // W1 = n / (R_1 R_p)
    mid = w & ((1u << w1_log) - 1);
    if (fs_il) {
      // T = (adjacent transforms) x (adjacent k_1 values): as many transforms as the interleave has
      constexpr uint32_t tl = __builtin_ctz(T);
      tb_log = tl < A.il ? tl : A.il;
      const uint32_t tk_log = tl - tb_log;
      const uint32_t rest = w >> w1_log;
      k10 = (rest & ((1u << (A.r1 - tk_log)) - 1)) << tk_log;
      b0 = (rest >> (A.r1 - tk_log)) << tb_log;
    } else {
      k10 = (w >> w1_log) * T;
    }
    uint32_t m = mid;
    for (uint32_t i = 0; i < A.nmid; ++i) {
      const uint32_t d = m & ((1u << A.mid_bits[i]) - 1);
      m >>= A.mid_bits[i];
      midrev |= d << A.mid_off[i];
    }
  }
  const uint32_t log_s = COLLIKE ? (A.log_blk - LOGR) : 0u;

  uint32_t x[EPT][E::W];
  uint32_t cl[EPT / 2];   // local column/block of each group (<= EPT/2 groups per thread)
  uint32_t pil[EPT / 2];  // group index of each group

  // ------------------------------------------------------------------ sub-stage 0: global -> regs
  // E::LDS_TW: this pass's w_R^e words, loaded ahead of the tile (L2 hits) and stored to LDS after
  // sub-stage 0 (which still multiplies from the global table)
  constexpr int TWWORDS = LTW ? (1 << LOGR) * E::TW : 1;  // the staged table, E::TW words per entry
  uint32_t stw[LTW ? (TWWORDS + NT - 1) / NT : 1];
  if constexpr (LTW && S::nsub > 1) {
    static_for<(TWWORDS + NT - 1) / NT>([&](auto I) {
      constexpr int i = I;
      stw[i] = (t + NT * i < TWWORDS) ? A.tw_int[t + NT * i] : 0u;
    });
  }
  {
    constexpr int qb = S::qb(0), Q = 1 << qb, G = EPT / Q, sb = S::logsig(0);
    static_for<G>([&](auto J) {
      constexpr int j = J;
      const uint32_t lam = t + NT * j;
      uint32_t c, g;
      if constexpr (COLLIKE) {
        c = lam % T;
        g = lam / T;
      } else {
        g = lam & ((1u << sb) - 1);
        c = lam >> sb;
      }
      cl[j] = c;
      pil[j] = g;
      static_for<Q>([&](auto D) {
        constexpr int d = D;
        const uint32_t pi = g + (d << sb);
        size_t pos;
        if constexpr (COLLIKE) {
          pos = colbase + c + ((size_t)pi << log_s);
        } else if constexpr (KIND == KIND_FINAL) {
          if (fs_il) {
            const uint32_t k1 = k10 + (c >> tb_log), b = b0 + (c & ((1u << tb_log) - 1));
            const size_t beta = ((size_t)k1 << (A.log_n - A.r1 - LOGR)) + mid;
            pos = (((beta << LOGR) + pi) << A.il) + b;
          } else {
            const size_t beta = ((size_t)(k10 + c) << (A.log_n - A.r1 - LOGR)) + mid;
            pos = (beta << LOGR) + pi;
          }
        } else {
          pos = pi;
        }
        const size_t b = ROWS ? (size_t)w * T + c : (size_t)bq;  // this element's transform
        E::template load<SW>(x[j * Q + d], src, ck(IN_USER ? in_pos(pos, b) : pos, A.dbg_src_n));
#if NTT_DEBUG_CHECKS
        // the caller's elements must be canonical (the reference's BAD LIMB trap); a column pass reads
        // them only when A.src_user (one SRC_USER instance also serves later passes when the scratch
        // and caller layouts agree)
        if (KIND == KIND_SINGLE || ROWS || (KIND == KIND_COLUMN && A.src_user))
          if (!E::dbg_canonical(x[j * Q + d], A.F)) ntt_dbg_flag(A.F.dbg, NTT_DBG_INPUT);
#endif
        if constexpr ((KIND == KIND_STOCKHAM || KIND == KIND_DIT) && FULLTW) {
          // bellperson's input twiddle (GZKP-NTT.cu:348-354): element pi of group k = index mod p is
          // multiplied by w_n^((n >> lgp >> deg) k pi), from a [k / T][pi][k mod T] table (p >= T).
          // KIND_DIT (GZKP(B, G), in place after the bit reversal): column c < s = 2^lgp of a block of
          // N = s R, input d multiplied by w_N^(c d) -- the same table shape with k = c
          uint32_t tw[E::W];
          const uint32_t k0 = col0 & ((1u << A.lgp) - 1);
          E::template load<E::TABW>(tw, A.tw_full, ((size_t)k0 << LOGR) + pi * T + c);
          E::mulv(x[j * Q + d], tw, A.F);
        }
        if constexpr (PRO == PRO_PW) {
          uint32_t y[E::W];
          E::load(y, A.src2 + boff, in_pos(pos, b));  // src2 has src's layout (a four-step piece: mapped)
          E::mulv(x[j * Q + d], y, A.F);  // canonical inputs: < 3p, normalised
        } else if constexpr (PRO == PRO_COSET) {
          typename E::Tw u;
          E::tload(u, A.tw_in, pi);
          E::mul(x[j * Q + d], u, A.F);  // < 3p, normalised
        }
      });
    });
    static_for<G>([&](auto J) {
      constexpr int j = J;
      dft<E, Q, j * Q, FAST>(x, A.F);
      if constexpr (S::nsub > 1) {
        E::template reduce<E::IN * Q, E::IN, FAST, R32>(x[j * Q], A.F);  // k = 0: the only output not multiplied
        static_for<Q - 1>([&](auto K1) {
          constexpr int k = K1 + 1;
          twiddle_mul<E>(x[j * Q + brev_bits(k, qb)], A.tw_int, pil[j] * k, A.F);
        });
      }
    });
    if constexpr (LTW && S::nsub > 1) {
      // parallel-load stage: the table words loaded with the tile (above) go to LDS now; the first
      // exchange's barrier publishes them to sub-stages 1.. (no barrier of its own)
      static_for<(TWWORDS + NT - 1) / NT>([&](auto I) {
        constexpr int i = I;
        if (t + NT * i < TWWORDS) lds_tw[t + NT * i] = stw[i];
      });
    }
  }

  if constexpr (IPN == 1) ipn_signal_read(A, mid);  // this tile's elements are in registers now

  // ------------------------------------------------------------------ sub-stages 1..nsub-1 via LDS
  if constexpr (S::nsub > 1) substage<E, LOGR, T, TE, NT, 1, FAST, R32, LTW>(x, cl, pil, lds, A, t, lds_tw, w);
  if constexpr (S::nsub > 2) substage<E, LOGR, T, TE, NT, 2, FAST, R32, LTW>(x, cl, pil, lds, A, t, lds_tw, w);
  if constexpr (S::nsub > 3) substage<E, LOGR, T, TE, NT, 3, FAST, R32, LTW>(x, cl, pil, lds, A, t, lds_tw, w);
  if constexpr (S::nsub > 4) substage<E, LOGR, T, TE, NT, 4, FAST, R32, LTW>(x, cl, pil, lds, A, t, lds_tw, w);
  if constexpr (S::nsub > 5) substage<E, LOGR, T, TE, NT, 5, FAST, R32, LTW>(x, cl, pil, lds, A, t, lds_tw, w);
  static_assert(S::nsub <= 6, "sub-stages");

  // ------------------------------------------------------------------ output
  if constexpr (IPN == 1) {  // the slab this tile writes into has been read (or the wait gave up: no stores)
    if (!ipn_wait_mirror(A, midrev)) return;
  } else if constexpr (IPN == 2 || IPN == 3) {  // in-place single launch: every final tile has read (grid barrier)
    if (!ipn_grid_barrier<IPN == 2 ? 4u : 3u>(A)) return;
  } else if constexpr (IPN == 4) {  // in-place single launch, pass 1: every workgroup is resident (A.ipn_go)
    if (!residency_wait(A.ipn_go, A.wd)) return;
  }
  {
    constexpr int ls = S::nsub - 1;
    constexpr int qb = S::qb(ls), Q = 1 << qb, G = EPT / Q, sb = S::logsig(ls), lN = S::logN(ls);
    static_for<G>([&](auto J) {
      constexpr int j = J;
      const uint32_t g = pil[j];
      const uint32_t rho = g >> sb, cp = g & ((1u << sb) - 1);
      const uint32_t c = cl[j];
      static_for<Q>([&](auto K) {
        constexpr int k = K;
        uint32_t(&v)[E::W] = x[j * Q + brev_bits(k, qb)];
        const uint32_t pi = (rho << lN) + cp + (k << sb);
        const uint32_t kn = natural_index<LOGR, QB>(pi);
        size_t pos;
        if constexpr (KIND == KIND_DIT) {
          // in place (GZKP-NTT.cu:157-158): output k of column c back to c + s k of its block
          pos = colbase + c + ((size_t)kn << log_s);
          E::template store<E::IN * Q, FAST, DW>(dst, ck(pos, A.dbg_dst_n), v, A.F);
        } else if constexpr (KIND == KIND_STOCKHAM) {
          // autosort store (GZKP-NTT.cu:378-384): y[((index - k) << deg) + k + kn p], k = index mod p
          const uint32_t idx = col0 + c, kk = idx & ((1u << A.lgp) - 1);
          pos = ((size_t)(idx - kk) << LOGR) + kk + ((size_t)kn << A.lgp);
          E::template store<E::IN * Q, FAST, DW>(dst, ck(pos, A.dbg_dst_n), v, A.F);
        } else if constexpr (KIND == KIND_COLUMN) {
          if constexpr (FULLTW) {
            // outer twiddle w_{N_i}^{col * kn} R_e from the per-pass table (HBM element format,
            // column-group-major [col / T][kn][col mod T], so one workgroup's entries are one
            // contiguous T * R run: HBM-streamed for pass 1, L2-resident later); the Montgomery
            // product removes R_e.  32 B per entry instead of a 80-B Shoup pair.
            uint32_t tw[E::W];
            size_t ti = ((size_t)col0 << LOGR) + (kn * T + c);
            if (fs_il) {  // Mode I: transform columns (col0 + c) >> il, in the table's column-group-major layout
              const uint32_t tc = (col0 + c) >> A.il;
              ti = ((size_t)(tc & ~(uint32_t)(T - 1)) << LOGR) + kn * T + (tc & (T - 1));
            }
            if constexpr (SHTW) {  // Shoup pair (w, floor(w B / p)), E::TW words: 143 MADs, no R_e
              typename E::Tw tws;
              E::tload(tws, A.tw_full, ti);
              E::mul(v, tws, A.F);
            } else {
              E::template load<E::TABW>(tw, A.tw_full, ti);
              E::mulv(v, tw, A.F);
            }
          } else {
            // outer twiddle w_{N_i}^{col * kn} = w_n^{(col * kn) << log_m} from the two-level
            // tables: t = (lo R_e) * hi, then the Montgomery product v * t / R_e = v * lo * hi
            const size_t e = ((size_t)((col0 + c) >> A.il) * kn) << A.log_m;  // il = 0 unless Mode I
            typename E::Tw tl, th;
            E::tload(tl, A.tw_lo, (uint32_t)(e & ((1u << A.lo_bits) - 1)));
            E::tload(th, A.tw_hi, (uint32_t)(e >> A.lo_bits));
            E::mul(tl.w, th, A.F);
            E::mulv(v, tl.w, A.F);
          }
          pos = colbase + c + ((size_t)kn << log_s);
          E::template store_lazy<E::MUL_OUT, FAST, DW, WT>(dst, ck(pos, A.dbg_dst_n), v, A.F);  // scratch: < 2p, read by the next pass
        } else if constexpr (KIND == KIND_FINAL) {
          if (fs_il) {
            const uint32_t k1 = k10 + (c >> tb_log), b = b0 + (c & ((1u << tb_log) - 1));
            pos = (((size_t)k1 + ((size_t)midrev << A.r1) + ((size_t)kn << (A.log_n - LOGR))) << A.il) + b;
          } else if (!IPN && (A.flags & 2u)) {  // NTT_PLAN_IN_PLACE: the input's own position; k_digitrev_swap follows
            pos = ((size_t)(k10 + c) << (A.log_n - A.r1)) + ((size_t)mid << LOGR) + kn;
          } else {
            pos = (size_t)(k10 + c) + ((size_t)midrev << A.r1) + ((size_t)kn << (A.log_n - LOGR));
          }
          if constexpr (EPI) {  // four-step twiddle w_n^(j1 k2) of this output (ntt_rplan), then the pack map
            uint32_t tw[E::W];
            E::template load<E::TABW>(tw, A.tw_epi, epi_idx(pos, bq));
            E::mulv(v, tw, A.F);
            E::template store<E::MUL_OUT, FAST, DW>(dst, ck(out_pos(pos, bq), A.dbg_dst_n), v, A.F);
          } else {
            E::template store<E::IN * Q, FAST, DW>(dst, ck(out_pos(pos, bq), A.dbg_dst_n), v, A.F);
          }
        } else {  // KIND_SINGLE, KIND_ROWS
          pos = kn;
          const size_t b = ROWS ? (size_t)w * T + c : (size_t)bq;
          if constexpr (EPI) {
            if (A.flags & 1u) E::mul(v, A.F.ninv, A.F);
            uint32_t tw[E::W];
            E::template load<E::TABW>(tw, A.tw_epi, epi_idx(pos, b));
            E::mulv(v, tw, A.F);
            E::template store<E::MUL_OUT, FAST>(dst, ck(out_pos(pos, b), A.dbg_dst_n), v, A.F);
          } else if (A.flags & 1u) {
            E::mul(v, A.F.ninv, A.F);
            E::template store<E::MUL_OUT, FAST>(dst, ck(out_pos(pos, b), A.dbg_dst_n), v, A.F);
          } else {
            E::template store<E::IN * Q, FAST>(dst, ck(out_pos(pos, b), A.dbg_dst_n), v, A.F);
          }
        }
      });
    });
  }
}

template <class E, int LOGR, int KIND, bool FULLTW, bool FAST, int PRO = PRO_NONE, bool SRC_USER = true,
          int FSM = 0, bool SHTW = false>
__global__ __launch_bounds__((1 << E::TILE_LOG) / E::EPT) __attribute__((amdgpu_waves_per_eu(E::WAVES_PER_EU)))
void k_pass(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, const PassArgs<E> A) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[pass_lds_words<E, LOGR, KIND>()];
  __shared__ __attribute__((aligned(16))) uint32_t lds_tw[pass_ltw<E, KIND, FULLTW>() ? (1 << LOGR) * E::TW : 1];
  // flags bit 2: workgroups are dealt round-robin over the 8 XCDs (b and b + 8 share one, for speed
  // only), so tile (b mod 8) G/8 + b / 8 puts neighbouring tiles -- which share 128-B lines when a
  // pass's runs are 64 B -- on one XCD's L2 at about the same time
  uint32_t w = blockIdx.x;
  if (A.flags & 4u) {
    const uint32_t G = gridDim.x;
    if ((G & 7u) == 0) w = (w & 7u) * (G >> 3) + (w >> 3);
  }
  pass_tile<E, LOGR, KIND, FULLTW, FAST, PRO, SRC_USER, FSM, SHTW>(src, dst, A, w, blockIdx.y, lds, lds_tw);
}

// In-place final pass with the fused digit reversal: one tile per workgroup, tiles taken from a
// ticket counter in slab-pair order (slab m's tiles, then slab rev(m)'s), so that a tile waits only
// for tiles of its own pair.  Deadlock-free at any residency: every ticket below the newest pair's
// was taken by a running workgroup, those pairs complete, and a pair has 2 R_1 / T <= 128 tiles.
// The last workgroup out re-zeroes the counters for the next launch.
template <class E, int LOGR>
__global__ __launch_bounds__((1 << E::TILE_LOG) / E::EPT) __attribute__((amdgpu_waves_per_eu(E::WAVES_PER_EU)))
void k_final_ipn(uint32_t* data, const PassArgs<E> A) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[pass_lds_words<E, LOGR, KIND_FINAL>()];
  __shared__ __attribute__((aligned(16))) uint32_t lds_tw[pass_ltw<E, KIND_FINAL, false>() ? (1 << LOGR) * E::TW : 1];
  __shared__ uint32_t s_w, s_last;
  const uint32_t t = threadIdx.x;
  if (t == 0) {
    const uint32_t tk = __hip_atomic_fetch_add(A.ipn_sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t slab = A.ipn_order[tk / A.ipn_strips], strip = tk % A.ipn_strips;
    s_w = (strip << (A.log_n - A.r1 - LOGR)) | slab;  // the final pass's tile index: (k1 group, mid)
  }
  __syncthreads();
  const uint32_t w = s_w;
  if constexpr (E::FASTRED) {
    if (A.F.red_ok)
      pass_tile<E, LOGR, KIND_FINAL, false, true, PRO_NONE, true, 0, false, false, false, 1>(data, data, A, w, 0, lds,
                                                                                           lds_tw);
    else
      pass_tile<E, LOGR, KIND_FINAL, false, false, PRO_NONE, true, 0, false, false, false, 1>(data, data, A, w, 0,
                                                                                            lds, lds_tw);
  } else {
    pass_tile<E, LOGR, KIND_FINAL, false, false, PRO_NONE, true, 0, false, false, false, 1>(data, data, A, w, 0, lds,
                                                                                          lds_tw);
  }
  if (t == 0)
    s_last = __hip_atomic_fetch_add(A.ipn_sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (s_last) {  // nobody touches the counters again in this launch
    const uint32_t slabs = (uint32_t)(gridDim.x / A.ipn_strips);
    for (uint32_t m = t; m < slabs; m += blockDim.x) {
      A.ipn_sync[32 * (1 + m)] = 0u;
      A.ipn_sync[32 * (1 + m) + 1] = 0u;
    }
    if (t == 0) {
      A.ipn_sync[0] = A.ipn_sync[1] = 0u;
      if (A.wd.abort) *A.wd.abort = 0u;
    }
  }
}

template <class E>
hipError_t launch_final_ipn(int logr, uint32_t* data, const PassArgs<E>& A, uint32_t grid, hipStream_t st) {
  constexpr int TL = tile_log_of<E>();
  constexpr int NT = (1 << TL) / E::EPT;
  switch (logr) {
#define NTT_IPN_CASE(R)                                                                          \
  case R:                                                                                        \
    if constexpr (R <= TL - E::MIN_COLS_LOG) {                                                   \
      hipLaunchKernelGGL((k_final_ipn<E, R>), dim3(grid), dim3(NT), 0, st, data, A);             \
      return hipGetLastError();                                                                  \
    }                                                                                            \
    return hipErrorInvalidValue;
    NTT_IPN_CASE(3)
    NTT_IPN_CASE(4)
    NTT_IPN_CASE(5)
    NTT_IPN_CASE(6)
    NTT_IPN_CASE(7)
    NTT_IPN_CASE(8)
    NTT_IPN_CASE(9)
#undef NTT_IPN_CASE
    default: return hipErrorInvalidValue;
  }
}

// Workgroups of k_final_ipn<E, logr> the device keeps resident at once (occupancy x CUs; 0 if the
// query fails or the radix has no instance)
template <class E>
uint32_t launch_final_ipn_capacity(int logr, int device) {
  constexpr int TL = tile_log_of<E>();
  constexpr int NT = (1 << TL) / E::EPT;
  int cus = 0, per = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
  hipError_t e = hipErrorInvalidValue;
  switch (logr) {
#define NTT_IPN_OCC(R)                                                                                   \
  case R:                                                                                                \
    if constexpr (R <= TL - E::MIN_COLS_LOG)                                                             \
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&k_final_ipn<E, R>), NT, 0); \
    break;
    NTT_IPN_OCC(3)
    NTT_IPN_OCC(4)
    NTT_IPN_OCC(5)
    NTT_IPN_OCC(6)
    NTT_IPN_OCC(7)
    NTT_IPN_OCC(8)
    NTT_IPN_OCC(9)
#undef NTT_IPN_OCC
    default: break;
  }
  return (e == hipSuccess && per > 0 && cus > 0) ? (uint32_t)per * (uint32_t)cus : 0u;
}

// ---------------------------------------------------------------------------- fused 3-pass launch
// BASELINE config 2 asks for the 2^20 transform as a single kernel (the reference's SSIP schedule is
// 4 launches at 2^20, GZKP-NTT.cu:1509-1545).  k_fused3 runs the three passes of a 3-pass schedule in
// ONE persistent launch.  Workgroups take tiles from one ticket counter in pass-major order (pass 1's
// tiles, then pass 2's, then the final pass's); a tile waits only for the tiles it reads, through
// counters keyed by the dependency structure of the four-step passes:
//   * pass-2 tile (block k1, column group g) reads columns g T2 + [0, T2) + s2 j2 of every j2 < R2,
//     written by the pass-1 tiles whose columns mod s2 (= 2^r3) fall in the same U-column unit
//     (U = max(T1, T2)): s2 / U counters, each reached by (U / T1) R2 pass-1 tiles;
//   * a final tile (T3 adjacent k1, one k2) reads every column of those k1 blocks: counters keyed by
//     k1 >> log T3 (R1 / T3 of them), each reached by T3 (s2 / T2) pass-2 tiles.
// Deadlock-free at any residency: a tile waits only for tiles with smaller tickets, which are held
// by running workgroups whose own waits are on smaller tickets still (pass 1 waits on nothing).
// Hand-off (MI355X_MICROARCH.md § visibility, publish form R1): scratch stores are write-through
// (sc1), every wave drains them (s_waitcnt vmcnt(0)), a workgroup barrier, then one lane's agent-scope
// counter add; the group's last arrival raises a ready word; the consumer polls it, takes ONE
// agent-scope acquire, waits, barrier, plain loads.
// Every dependency wait is bounded (Watchdog: a workgroup whose wait gives up runs no further tile,
// the launch's other waits give up at once, and the plan's next call returns NTT_ERR_DEVICE), so every
// wave reaches the exit; the last workgroup out re-zeroes the counters for the next launch.
// Producer: every wave drains its write-through stores, a barrier, then one lane counts the tile in;
// the group's last arrival (told by the value its add returns) raises the group's ready word, which
// lies on a 128-B line of its own.  Consumers poll only that word: 128 pollers on the counter itself
// queued the producers' adds behind their polls (2^20: 350-450 us per transform instead of 160).
__device__ __forceinline__ void fused_publish(uint32_t* cnt, uint32_t* ready, uint32_t need) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its write-through stores are done
  __syncthreads();
  if (threadIdx.x == 0 && __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == need - 1)
    __hip_atomic_store(ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Consumer: one lane polls the ready word with relaxed agent-scope loads (compare-exchange polls,
// read-modify-writes at the memory side, queued the producers' updates behind them: 2^20 single
// launch 0.162 -> see DESIGN §4), sleeping 60 ns .. 1 us between polls; then ONE agent-scope acquire, its wait, and
// the workgroup barrier before any load of the handed-off tile.  Bounded (Watchdog): false
// (workgroup-uniform) when the wait gave up; the workgroup then runs no further tile.
__device__ __forceinline__ bool fused_wait(uint32_t* ready, const FusedArgs& F) {
  if (F.dbg & 1u) return true;  // diagnostics only: no dependency waits (wrong output)
  __shared__ uint32_t s_ok;
  if (threadIdx.x == 0) {
    s_ok = poll_bounded<2, 4, 8, 16, 32>(ready, F.wd) ? 1u : 0u;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(s_ok) != 0u;
}

template <class E>
struct FusedKArgs {
  const uint32_t* src;
  uint32_t* scratch;
  uint32_t* dst;
  PassArgs<E> A1, A2, A3;
  FusedArgs F;
};
static_assert(sizeof(FusedKArgs<Eng256>) <= 4096, "kernel argument segment");
// The kernel arguments re-addressed per tile through an opaque copy of the kernarg pointer, so that
// the persistent loops do not keep every pass's uniform arguments live across the loop (with the
// LOOPED thread index above: 0-16 B of spills instead of 200-380 B).
template <class E>
__device__ __forceinline__ const FusedKArgs<E>& fused_kargs() {
  typedef const __attribute__((address_space(4))) FusedKArgs<E>* KP;
  KP p = (KP)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const FusedKArgs<E>*)p;
}

template <class E, int R1, int R2, int R3>
__global__ __launch_bounds__((1 << E::TILE_LOG) / E::EPT) __attribute__((amdgpu_waves_per_eu(E::WAVES_PER_EU)))
void k_fused3(const FusedKArgs<E> K) {
  static_assert(E::FASTRED && E::SHOUP_OUTER && !E::LDS_TW, "fused schedule: FAST 256-bit engines");
  constexpr int LW = pass_lds_words<E, R1, KIND_COLUMN>();
  static_assert(LW == pass_lds_words<E, R3, KIND_FINAL>(), "one tile size");
  __shared__ __attribute__((aligned(16))) uint32_t lds[LW];
  __shared__ uint32_t lds_tw[1];
  __shared__ uint32_t s_ticket;
  const FusedArgs& F = K.F;
  uint32_t* const cnt12 = F.sync + 4;
  uint32_t* const cnt23 = F.sync + 4 + F.n12;
  const uint32_t t = threadIdx.x, total = 3 * F.tiles;
  // Tile order: every tile is a ticket sync[0]++, the first taken at start, each later one while the
  // previous tile's stores drain, i.e. in completion order.  (A ticket prefetched at tile START let
  // the first workgroups to start take two or three pass-1 tiles each while later ones idled on
  // pass-2 tiles: 4x slower at 2^20.)
  uint32_t stat = blockIdx.x;  // dbg bit 2: static order b, b + nwg, ...
  auto ticket = [&]() -> uint32_t {
    if (F.dbg & 4u) return stat += F.nwg;
    return t == 0 ? __hip_atomic_fetch_add(F.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  };
  if (t == 0) s_ticket = (F.dbg & 4u) ? blockIdx.x : ticket();
  __syncthreads();
  uint32_t tk = s_ticket;
  auto advance = [&](uint32_t next) {
    __syncthreads();  // every wave is done with this tile's LDS and s_ticket
    if (t == 0) s_ticket = next;
    __syncthreads();
    tk = s_ticket;
  };
  // tickets only grow per workgroup and are handed out pass-major: one loop per pass
  while (tk < F.tiles) {  // pass 1: the caller's buffer -> scratch
    const uint32_t w = tk;
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R1, KIND_COLUMN, true, true, PRO_NONE, true, 0, false, true, true>(L.src, L.scratch, L.A1, w, 0,
                                                                                      lds, lds_tw);
    const uint32_t next = ticket();  // issued before the drain of this tile's stores
    const uint32_t key = (w & F.k1_mask) >> F.k1_shift;
    fused_publish(cnt12 + key, F.sync + F.rbase + 32 * key, F.need12);
    advance(next);
  }
  while (tk < 2 * F.tiles) {  // pass 2: scratch in place (Shoup-pair outer twiddles)
    const uint32_t w = tk - F.tiles, g = w & ((1u << F.cg_log) - 1);
    if (!fused_wait(F.sync + F.rbase + 32 * (g >> F.k2_shift), F)) {
      tk = total;  // gave up (watchdog): no further tile, straight to the exit
      break;
    }
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R2, KIND_COLUMN, true, true, PRO_NONE, true, 0, true, true, true>(L.scratch, L.scratch, L.A2, w, 0,
                                                                                     lds, lds_tw);
    const uint32_t next = ticket();
    const uint32_t key = (w >> F.cg_log) >> F.t3_log;
    fused_publish(cnt23 + key, F.sync + F.rbase + 32 * (F.n12 + key), F.need23);
    advance(next);
  }
  while (tk < total) {  // final pass: scratch -> the caller's buffer, natural order
    const uint32_t w = tk - 2 * F.tiles;
    if (!fused_wait(F.sync + F.rbase + 32 * (F.n12 + (w >> F.r2)), F)) break;
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R3, KIND_FINAL, false, true, PRO_NONE, true, 0, false, false, true>(L.scratch, L.dst, L.A3, w, 0,
                                                                                       lds, lds_tw);
    advance(ticket());
  }
  if (t == 0 && __hip_atomic_fetch_add(F.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == F.nwg - 1) {
    // the last workgroup out: nobody touches the counters again in this launch
    const uint32_t words = F.rbase + 32 * (F.n12 + F.n23);
    for (uint32_t i = 0; i < words; ++i) __hip_atomic_store(F.sync + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (F.wd.abort) __hip_atomic_store(F.wd.abort, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The same three passes with two grid-wide barriers instead of per-tile hand-offs (FusedArgs::mode 1,
// a plain launch of at most the workgroups the device holds at once).  Each workgroup runs tiles b, b + G, ... of a
// pass, then the barrier.  The barrier (the guide's R1 publish, MI355X_MICROARCH.md § visibility):
// * scratch stores are write-through (sc1), so no release fence: every wave drains them, then a
//   workgroup barrier, then one lane counts the workgroup in;
// * the last of the G arrivals raises the barrier's go word (its own 128-B line);
// * one lane per workgroup polls that word with relaxed global loads (bounded: then the watchdog
//   word), takes ONE agent-scope acquire, and the workgroup barrier releases every wave.
// A/B: plain stores with an agent-scope release per workgroup were slower at 2^20
// (every release writes back its XCD's L2), and compare-exchange polls of one word by 1024
// workgroups made each barrier cost ~0.15 ms.
// The arrival counter is cumulative (barrier k completes at k G arrivals); the last workgroup out
// re-zeroes the words for the next launch.
// False (workgroup-uniform) when the wait gave up (Watchdog): the workgroup then skips the passes left.
__device__ __forceinline__ bool fused_grid_barrier(const FusedArgs& F, uint32_t k) {
  return grid_barrier_words(F.sync, F.shards, F.sync + F.rbase + 32 * (k - 1), k, F.wd);
}

template <class E, int R1, int R2, int R3>
__global__ __launch_bounds__((1 << E::TILE_LOG) / E::EPT) __attribute__((amdgpu_waves_per_eu(E::WAVES_PER_EU)))
void k_fused3b(const FusedKArgs<E> K) {
  static_assert(E::FASTRED && E::SHOUP_OUTER && !E::LDS_TW, "fused schedule: FAST 256-bit engines");
  constexpr int LW = pass_lds_words<E, R1, KIND_COLUMN>();
  static_assert(LW == pass_lds_words<E, R3, KIND_FINAL>(), "one tile size");
  __shared__ __attribute__((aligned(16))) uint32_t lds[LW];
  __shared__ uint32_t lds_tw[1];
  const FusedArgs& F = K.F;
  const uint32_t G = gridDim.x;
  for (uint32_t w = blockIdx.x; w < F.tiles; w += G) {  // pass 1: the caller's buffer -> scratch
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R1, KIND_COLUMN, true, true, PRO_NONE, true, 0, false, true, true>(L.src, L.scratch, L.A1,
                                                                                                w, 0, lds, lds_tw);
    __syncthreads();  // every wave is done with this tile's LDS
  }
  bool ok = fused_grid_barrier(F, 1);
  for (uint32_t w = blockIdx.x; ok && w < F.tiles; w += G) {  // pass 2: scratch in place
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R2, KIND_COLUMN, true, true, PRO_NONE, true, 0, true, true, true>(L.scratch, L.scratch, L.A2,
                                                                                               w, 0, lds, lds_tw);
    __syncthreads();
  }
  ok = ok && fused_grid_barrier(F, 2);  // a workgroup that gave up does not arrive: the others give up too
  for (uint32_t w = blockIdx.x; ok && w < F.tiles; w += G) {  // final pass: scratch -> the caller's buffer
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R3, KIND_FINAL, false, true, PRO_NONE, true, 0, false, false, true>(L.scratch, L.dst, L.A3, w, 0,
                                                                                       lds, lds_tw);
    __syncthreads();
  }
  if (threadIdx.x == 0 && __hip_atomic_fetch_add(F.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
    // the last workgroup out: every other one has passed both barriers
    __hip_atomic_store(F.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(F.sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (F.wd.abort) __hip_atomic_store(F.wd.abort, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(F.sync + F.rbase, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(F.sync + F.rbase + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t sh = 0; sh < 8; ++sh) __hip_atomic_store(F.shards + 32 * sh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The single-launch schedule of an NTT_PLAN_IN_PLACE plan (FusedArgs::mode 2; BASELINE config 2's
// "single-kernel self-sort-in-place"): no scratch, every pass in the caller's buffer.  Passes 1 and 2
// write the positions they read (write-through, as k_fused3b); the final pass of the palindromic
// schedule writes its outputs to their natural positions, which lie in the mirror slab, so every final
// tile loads and transforms, a third grid barrier makes sure every tile has read, and only then do the
// tiles store (IPN = 2 in pass_tile).  That needs every final tile resident at once: one tile per
// workgroup, nwg == tiles (n <= 2^20 at 4 workgroups per CU), and a residency check before the first
// store (residency_arrive / residency_wait: barrier 1), so that a launch whose workgroups are not all
// resident stores nothing.
template <class E, int R1, int R2, int R3>
__global__ __launch_bounds__((1 << E::TILE_LOG) / E::EPT) __attribute__((amdgpu_waves_per_eu(E::WAVES_PER_EU)))
void k_fused3bi(const FusedKArgs<E> K) {
  static_assert(E::FASTRED && E::SHOUP_OUTER && !E::LDS_TW && E::SCRW == E::MEMW, "fused in place: 256-bit engines");
  constexpr int LW = pass_lds_words<E, R1, KIND_COLUMN>();
  static_assert(LW == pass_lds_words<E, R3, KIND_FINAL>(), "one tile size");
  __shared__ __attribute__((aligned(16))) uint32_t lds[LW];
  __shared__ uint32_t lds_tw[1];
  const FusedArgs& F = K.F;
  const uint32_t G = gridDim.x;
  uint32_t* const go1 = F.sync + F.rbase;  // residency: grid barrier 1 (residency_arrive)
  residency_arrive(F.sync, F.shards, go1);
  for (uint32_t w = blockIdx.x; w < F.tiles; w += G) {  // pass 1, in place; its stores wait for residency
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R1, KIND_COLUMN, true, true, PRO_NONE, true, 0, false, true, true, 4>(L.dst, L.dst, L.A1, w, 0, lds,
                                                                                         lds_tw);
    __syncthreads();
  }
  bool ok = residency_went(go1) && fused_grid_barrier(F, 2);
  for (uint32_t w = blockIdx.x; ok && w < F.tiles; w += G) {  // pass 2, in place
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R2, KIND_COLUMN, true, true, PRO_NONE, true, 0, true, true, true>(L.dst, L.dst, L.A2, w, 0, lds,
                                                                                     lds_tw);
    __syncthreads();
  }
  ok = ok && fused_grid_barrier(F, 3);
  if (ok && blockIdx.x < F.tiles) {  // final pass: load, transform, barrier 4 (inside), natural-order stores
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R3, KIND_FINAL, false, true, PRO_NONE, true, 0, false, false, true, 2>(L.dst, L.dst, L.A3,
                                                                                         blockIdx.x, 0, lds, lds_tw);
  }
  if (threadIdx.x == 0 && __hip_atomic_fetch_add(F.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
    // the last workgroup out: every other one has passed (or given up at) all four barriers
    __hip_atomic_store(F.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(F.sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (F.wd.abort) __hip_atomic_store(F.wd.abort, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t k = 0; k < 4; ++k)
      __hip_atomic_store(F.sync + F.rbase + 32 * k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t sh = 0; sh < 8; ++sh) __hip_atomic_store(F.shards + 32 * sh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// BASELINE config 2 as ONE kernel on 4096-element tiles (the reference's 2^20
// schedule is 4 launches, GZKP-NTT.cu:1509-1545): the two passes (10 + 10) of Eng256T with ONE grid
// barrier between them.  2^20 is 256 tiles per pass, one 1024-thread workgroup per CU, so each
// workgroup runs one tile of each pass.  A plain launch (no cooperative launch: its ~20 us per call
// was most of the 3-pass single launch's deficit) of at most the occupancy query's
// workgroups; the barrier is bounded (Watchdog), so a device shared with another persistent kernel
// ends in NTT_ERR_DEVICE, never a hang.
//   k_fused2b  (FusedArgs::mode 3): pass 1 caller -> scratch (write-through), barrier, final pass
//              scratch -> caller, natural order.
//   k_fused2bi (FusedArgs::mode 4): NTT_PLAN_IN_PLACE, the palindromic 10 + 10: pass 1 in place (its
//              stores wait for the residency decision, barrier 1), barrier 2, the final pass loads and
//              transforms every tile, barrier 3 (every tile has read: all 256 final tiles are
//              resident), then the stores to the natural positions in the mirror slab (pass_tile
//              IPN = 3).  No scratch.
// FusedArgs::trace (diagnostics, NTT_FUSED_TRACE): per workgroup the wall clock (100 MHz) at start,
// after pass 1, after the pass barrier and at the end.
__device__ __forceinline__ void fused_trace(const FusedArgs& F, uint32_t at) {
  if (F.trace && threadIdx.x == 0) F.trace[4 * blockIdx.x + at] = (unsigned long long)wall_clock64();
}
template <class E, int R1, int R2>
__global__ __launch_bounds__((1 << E::TILE_LOG) / E::EPT) __attribute__((amdgpu_waves_per_eu(E::WAVES_PER_EU)))
void k_fused2b(const FusedKArgs<E> K) {
  static_assert(E::FASTRED && !E::LDS_TW, "fused schedule: FAST 256-bit engines");
  constexpr int LW = pass_lds_words<E, R1, KIND_COLUMN>();
  static_assert(LW == pass_lds_words<E, R2, KIND_FINAL>(), "one tile size");
  __shared__ __attribute__((aligned(16))) uint32_t lds[LW];
  __shared__ uint32_t lds_tw[1];
  const FusedArgs& F = K.F;
  const uint32_t G = gridDim.x;
  fused_trace(F, 0);
  for (uint32_t w = blockIdx.x; w < F.tiles; w += G) {  // pass 1: the caller's buffer -> scratch
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R1, KIND_COLUMN, true, true, PRO_NONE, true, 0, false, true, true>(L.src, L.scratch, L.A1, w, 0, lds,
                                                                                      lds_tw);
    __syncthreads();
  }
  fused_trace(F, 1);
  const bool ok = fused_grid_barrier(F, 1);
  fused_trace(F, 2);
  for (uint32_t w = blockIdx.x; ok && w < F.tiles; w += G) {  // final pass: scratch -> the caller's buffer
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R2, KIND_FINAL, false, true, PRO_NONE, true, 0, false, false, true>(L.scratch, L.dst, L.A3, w, 0, lds,
                                                                                      lds_tw);
    __syncthreads();
  }
  fused_trace(F, 3);
  if (threadIdx.x == 0 && __hip_atomic_fetch_add(F.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
    // the last workgroup out: every other one has passed (or given up at) the barrier
    __hip_atomic_store(F.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(F.sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (F.wd.abort) __hip_atomic_store(F.wd.abort, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(F.sync + F.rbase, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t sh = 0; sh < 8; ++sh) __hip_atomic_store(F.shards + 32 * sh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <class E, int R>
__global__ __launch_bounds__((1 << E::TILE_LOG) / E::EPT) __attribute__((amdgpu_waves_per_eu(E::WAVES_PER_EU)))
void k_fused2bi(const FusedKArgs<E> K) {
  static_assert(E::FASTRED && !E::LDS_TW && E::SCRW == E::MEMW, "fused in place: 256-bit engines");
  constexpr int LW = pass_lds_words<E, R, KIND_COLUMN>();
  static_assert(LW == pass_lds_words<E, R, KIND_FINAL>(), "one tile size");
  __shared__ __attribute__((aligned(16))) uint32_t lds[LW];
  __shared__ uint32_t lds_tw[1];
  const FusedArgs& F = K.F;
  const uint32_t G = gridDim.x;
  uint32_t* const go1 = F.sync + F.rbase;  // residency: grid barrier 1 (residency_arrive)
  fused_trace(F, 0);
  residency_arrive(F.sync, F.shards, go1);
  for (uint32_t w = blockIdx.x; w < F.tiles; w += G) {  // pass 1, in place; its stores wait for residency
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R, KIND_COLUMN, true, true, PRO_NONE, true, 0, false, true, true, 4>(L.dst, L.dst, L.A1, w, 0, lds,
                                                                                        lds_tw);
    __syncthreads();
  }
  fused_trace(F, 1);
  const bool ok = residency_went(go1) && fused_grid_barrier(F, 2);
  fused_trace(F, 2);
  if (ok && blockIdx.x < F.tiles) {  // final pass: load, transform, barrier 3 (inside), natural-order stores
    const FusedKArgs<E>& L = fused_kargs<E>();
    pass_tile<E, R, KIND_FINAL, false, true, PRO_NONE, true, 0, false, false, true, 3>(L.dst, L.dst, L.A3, blockIdx.x, 0,
                                                                                        lds, lds_tw);
  }
  fused_trace(F, 3);
  if (threadIdx.x == 0 && __hip_atomic_fetch_add(F.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
    __hip_atomic_store(F.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(F.sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (F.wd.abort) __hip_atomic_store(F.wd.abort, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t k = 0; k < 3; ++k)
      __hip_atomic_store(F.sync + F.rbase + 32 * k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t sh = 0; sh < 8; ++sh) __hip_atomic_store(F.shards + 32 * sh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <class E>
hipError_t launch_fused2(int r1, int r2, const uint32_t* src, uint32_t* scratch, uint32_t* dst, const PassArgs<E>& A1,
                         const PassArgs<E>& A2, const FusedArgs& F, hipStream_t st) {
  if constexpr (!fused2_engine<E>()) {
    return hipErrorInvalidValue;
  } else {
    if (r1 != 10 || r2 != 10 || (F.mode != 3 && F.mode != 4)) return hipErrorInvalidValue;
    const dim3 g(F.nwg), b((1 << E::TILE_LOG) / E::EPT);
    FusedKArgs<E> K{src, scratch, dst, A1, A1, A2, F};
    if (F.mode == 4)
      hipLaunchKernelGGL((k_fused2bi<E, 10>), g, b, 0, st, K);
    else
      hipLaunchKernelGGL((k_fused2b<E, 10, 10>), g, b, 0, st, K);
    return hipGetLastError();
  }
}
// workgroups of k_fused2b (mode 3) / k_fused2bi (mode 4) resident at once on `device`
template <class E>
hipError_t fused2_capacity(int r1, int r2, int device, uint32_t* wgs, uint32_t mode) {
  if constexpr (!fused2_engine<E>()) {
    return hipErrorInvalidValue;
  } else {
    if (r1 != 10 || r2 != 10) return hipErrorInvalidValue;
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return hipErrorInvalidValue;
    const int threads = (1 << E::TILE_LOG) / E::EPT;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per, mode == 4 ? reinterpret_cast<const void*>(&k_fused2bi<E, 10>) : reinterpret_cast<const void*>(&k_fused2b<E, 10, 10>),
        threads, 0);
    if (e != hipSuccess) return e;
    *wgs = (uint32_t)(cus * per);
    return hipSuccess;
  }
}

template <class E>
hipError_t launch_fused3(int r1, int r2, int r3, const uint32_t* src, uint32_t* scratch, uint32_t* dst,
                         const PassArgs<E>& A1, const PassArgs<E>& A2, const PassArgs<E>& A3, const FusedArgs& F,
                         hipStream_t st) {
  if constexpr (!(E::FASTRED && E::SHOUP_OUTER && !E::LDS_TW && E::TILE_LOG == 10 && E::EPT == 4)) {
    return hipErrorInvalidValue;
  } else {
    const dim3 g(F.nwg), b((1 << E::TILE_LOG) / E::EPT);
    FusedKArgs<E> K{src, scratch, dst, A1, A2, A3, F};
    // The grid-barrier forms are plain launches of at most the occupancy query's workgroups (the plan
    // checks that the grid fits the device, fused3_capacity); the plan serialises its single launches
    // per device (ntt_plan.cpp FusedSerial), and the in-place form checks residency before its first
    // store.  Round 6 retired the cooperative launch: ~20 us more per call, and every
    // rocprofv3-traced process that had made one crashed in the runtime's exit handlers.
    if (F.mode == 2) {  // in place: one workgroup per tile
#define NTT_FUSED_IP_CASE(a, c, d)                                                                \
  if (r1 == a && r2 == c && r3 == d) {                                                            \
    hipLaunchKernelGGL((k_fused3bi<E, a, c, d>), g, b, 0, st, K);                                 \
    return hipGetLastError();                                                                     \
  }
      NTT_FUSED_IP_CASE(6, 6, 6)
      NTT_FUSED_IP_CASE(6, 7, 6)
      NTT_FUSED_IP_CASE(7, 6, 7)
#undef NTT_FUSED_IP_CASE
      return hipErrorInvalidValue;
    }
#define NTT_FUSED_CASE(a, c, d)                                                                   \
  if (r1 == a && r2 == c && r3 == d) {                                                            \
    if (F.mode == 1) {                                                                            \
      hipLaunchKernelGGL((k_fused3b<E, a, c, d>), g, b, 0, st, K);                                \
      return hipGetLastError();                                                                   \
    }                                                                                             \
    hipLaunchKernelGGL((k_fused3<E, a, c, d>), g, b, 0, st, K);                                   \
    return hipGetLastError();                                                                     \
  }
    NTT_FUSED_CASE(6, 6, 6)
    NTT_FUSED_CASE(7, 6, 6)
    NTT_FUSED_CASE(7, 7, 6)
    NTT_FUSED_CASE(7, 7, 7)
    NTT_FUSED_CASE(8, 7, 7)
    NTT_FUSED_CASE(8, 8, 7)
    NTT_FUSED_CASE(8, 8, 8)
#undef NTT_FUSED_CASE
    return hipErrorInvalidValue;
  }
}

template <class E>
hipError_t fused3_capacity(int r1, int r2, int r3, int device, uint32_t* wgs, uint32_t mode) {
  if constexpr (!(E::FASTRED && E::SHOUP_OUTER && !E::LDS_TW && E::TILE_LOG == 10 && E::EPT == 4)) {
    return hipErrorInvalidValue;
  } else {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return hipErrorInvalidValue;
    const int threads = (1 << E::TILE_LOG) / E::EPT;
    hipError_t e = hipErrorInvalidValue;
#define NTT_FUSED_OCC(a, c, d)                                                                         \
  if (r1 == a && r2 == c && r3 == d)                                                                   \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(                                                   \
        &per, mode == 1 ? reinterpret_cast<const void*>(&k_fused3b<E, a, c, d>)                        \
                        : reinterpret_cast<const void*>(&k_fused3<E, a, c, d>),                        \
        threads, 0);
#define NTT_FUSED_IP_OCC(a, c, d)                                                                      \
  if (mode == 2 && r1 == a && r2 == c && r3 == d)                                                      \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&k_fused3bi<E, a, c, d>), \
                                                     threads, 0);
    NTT_FUSED_IP_OCC(6, 6, 6)
    NTT_FUSED_IP_OCC(6, 7, 6)
    NTT_FUSED_IP_OCC(7, 6, 7)
#undef NTT_FUSED_IP_OCC
    if (mode != 2) {
    NTT_FUSED_OCC(6, 6, 6)
    NTT_FUSED_OCC(7, 6, 6)
    NTT_FUSED_OCC(7, 7, 6)
    NTT_FUSED_OCC(7, 7, 7)
    NTT_FUSED_OCC(8, 7, 7)
    NTT_FUSED_OCC(8, 8, 7)
    NTT_FUSED_OCC(8, 8, 8)
    }
#undef NTT_FUSED_OCC
    if (e != hipSuccess) return e;
    *wgs = (uint32_t)(cus * per);
    return hipSuccess;
  }
}

// Element-wise kernels run as grid-stride loops over at most 2^20 workgroups of 256 threads:
// grid.x * blockDim.x stays far below HIP's 2^32-thread launch limit at every supported size
// (2^32-element BLS12-381 vectors included).
__host__ __device__ constexpr uint32_t grid_1d(size_t count) {
  return (uint32_t)((count + 255) / 256 < (size_t(1) << 20) ? (count + 255) / 256 : (size_t(1) << 20));
}
#define NTT_GRID_STRIDE(idx, count) \
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < (count); idx += (size_t)gridDim.x * blockDim.x)

// O(n^2) transform for tiny n (n <= 4): X_k = sum_j x_j w^(jk); tw_int holds w^e, e < n.
template <class E>
__global__ void k_dft_naive(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, const PassArgs<E> A) {
  const uint32_t n = 1u << A.log_n;
  const uint32_t k = threadIdx.x;
  const size_t boff = (size_t)blockIdx.y * A.batch_stride;
  uint32_t acc[E::W];
  if (k < n) {
    // acc = x_0 * w^0 (Montgomery by w^0 = R brings it to the engine's residue form)
    uint32_t v[E::W];
    typename E::Tw w;
    E::load(acc, src + boff, 0);
    E::tload(w, A.tw_int, 0);
    E::mul(acc, w, A.F);
#pragma unroll 1
    for (uint32_t j = 1; j < n; ++j) {
      E::load(v, src + boff, j);
      E::tload(w, A.tw_int, (j * k) & (n - 1));
      E::mul(v, w, A.F);
      E::template bfly_l<E::IN>(acc, v, A.F);  // acc <- acc + v (the difference is discarded)
      E::template reduce<2 * E::IN, E::IN>(acc, A.F);
    }
    if (A.flags & 1u) E::mul(acc, A.F.ninv, A.F);
  }
  __syncthreads();  // every thread has read src before anyone writes dst (in-place use)
  if (k < n) E::template store<E::IN>(dst + boff, k, acc, A.F);
}

// Per-pass outer-twiddle table of a column pass with radix 2^log_r and T = 2^log_t columns per
// workgroup: entry (c, k) = w_n^((c*k) << log_m) R_e mod p (R_e the engine's Montgomery radix) at
// [c >> log_t][k][c mod T], canonical in the HBM element format, built on the device from the
// two-level tables (lo_s = lo R_e, so lo_s * hi = w R_e).  With clo/chi (two-level tables of a coset
// shift c in the same format) the entry is also multiplied by c^col.
template <class E>
__global__ void k_build_tw(uint32_t* __restrict__ out, size_t count, uint32_t log_r, uint32_t log_t, uint32_t log_m,
                           const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hi, uint32_t lo_bits,
                           const typename E::Args F, const uint32_t* __restrict__ clo,
                           const uint32_t* __restrict__ chi) {
  NTT_GRID_STRIDE(idx, count) {
    const size_t k = (idx >> log_t) & ((1ull << log_r) - 1);
    const size_t c = ((idx >> (log_t + log_r)) << log_t) + (idx & ((1ull << log_t) - 1));
    const size_t e = (c * k) << log_m;
    typename E::Tw a, b;
    E::tload(a, lo, (uint32_t)(e & ((1ull << lo_bits) - 1)));
    E::tload(b, hi, (uint32_t)(e >> lo_bits));
    E::mul(a.w, b, F);
    if (clo) {  // c^col R_e = clo[col & mask] * chi[col >> lo_bits]; mulv removes one R_e
      typename E::Tw u, v;
      E::tload(u, clo, (uint32_t)(c & ((1ull << lo_bits) - 1)));
      E::tload(v, chi, (uint32_t)(c >> lo_bits));
      E::mul(u.w, v, F);
      E::mulv(a.w, u.w, F);
    }
    E::template store<E::MUL_OUT, false, E::TABW>(out, idx, a.w, F);  // outer-twiddle tables: E::TABW words
  }
}

template <class E>
hipError_t launch_build_tw(uint32_t* out, size_t count, uint32_t log_r, uint32_t log_t, uint32_t log_m,
                           const uint32_t* lo, const uint32_t* hi, uint32_t lo_bits, const typename E::Args& F,
                           hipStream_t st, const uint32_t* clo, const uint32_t* chi) {
  hipLaunchKernelGGL((k_build_tw<E>), dim3(grid_1d(count)), dim3(256), 0, st, out, count, log_r,
                     log_t, log_m, lo, hi, lo_bits, F, clo, chi);
  return hipGetLastError();
}

// NTT_PLAN_NAIVE (the reference's `naive` rival, GZKP-NTT.cu:59-71 / big-num.cu:67-104): the power
// table entry i = w_n^i R_e mod p, i < count, canonical in the element format (E::TABW words) -- the
// reference's `roots` table (GZKP-NTT.cu:81-83), built on the device from the two-level tables.
template <class E>
__global__ void k_build_pow(uint32_t* __restrict__ out, size_t count, const uint32_t* __restrict__ lo,
                            const uint32_t* __restrict__ hi, uint32_t lo_bits, const typename E::Args F) {
  NTT_GRID_STRIDE(i, count) {
    typename E::Tw a, b;
    E::tload(a, lo, i & ((size_t(1) << lo_bits) - 1));
    E::tload(b, hi, i >> lo_bits);
    E::mul(a.w, b, F);
    E::template store<E::MUL_OUT, false, E::TABW>(out, i, a.w, F);
  }
}

template <class E>
hipError_t launch_build_pow(uint32_t* out, size_t count, const uint32_t* lo, const uint32_t* hi, uint32_t lo_bits,
                            const typename E::Args& F, hipStream_t st) {
  hipLaunchKernelGGL((k_build_pow<E>), dim3(grid_1d(count)), dim3(256), 0, st, out, count, lo, hi, lo_bits, F);
  return hipGetLastError();
}

// One radix-2 DIT round of the `naive` rival over a bit-reversed vector: butterfly id < n/2 pairs
// pos = 2 (id - off) + off and pos + s (s = 2^log_s, off = id mod s) as (a + w b, a - w b) with
// w = w_n^(off n / 2s) -- the reference kernel's indexing (GZKP-NTT.cu:59-71), one thread per
// butterfly, canonical in and out (the product through the element-format power table: mulv).
// HBM-bound by construction: every round reads and writes the whole vector.  src and dst alias (every
// round but the last runs in place), so neither is __restrict__: each thread reads its two
// elements before it writes them, and no other thread touches them in the round.
template <class E>
__global__ void k_naive_round(const uint32_t* src, uint32_t* dst, uint32_t log_n,
                              uint32_t log_s, const uint32_t* __restrict__ pw, const typename E::Args F) {
  const size_t half = size_t(1) << (log_n - 1), s = size_t(1) << log_s;
  NTT_GRID_STRIDE(id, half) {
    const size_t off = id & (s - 1), pos = ((id - off) << 1) + off;
    uint32_t a[E::W], b[E::W], w[E::W];
    E::load(a, src, pos);
    E::load(b, src, pos + s);
    E::template load<E::TABW>(w, pw, off << (log_n - 1 - log_s));
    E::mulv(b, w, F);  // w R_e: the Montgomery product leaves w b, < 3p (Eng29) / < 2p (Eng32)
    E::template bfly_l<E::IN>(a, b, F);
    E::template store<2 * E::IN>(dst, pos, a, F);
    E::template store<2 * E::IN>(dst, pos + s, b, F);
  }
}

// One radix-2 round of the `naive_no_swap` rival (GZKP-NTT.cu:237-258): butterfly i < n/2 reads
// x[i] and x[i + n/2], multiplies the second by w = w_n^(k n / 2s) (k = i mod s, s = 2^log_s: the
// reference's roots[k * (len / (stride << 1))]) and writes a + w b to y[2i - k], a - w b to
// y[2i - k + s] -- a radix-2 Stockham autosort: natural order in and out after log2 n rounds.
// src != dst (ping-pong).  HBM-bound by construction, like k_naive_round.
template <class E>
__global__ void k_noswap_round(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t log_n,
                               uint32_t log_s, const uint32_t* __restrict__ pw, const typename E::Args F) {
  const size_t half = size_t(1) << (log_n - 1), s = size_t(1) << log_s;
  NTT_GRID_STRIDE(i, half) {
    const size_t k = i & (s - 1), j = (i << 1) - k;
    uint32_t a[E::W], b[E::W], w[E::W];
    E::load(a, src, i);
    E::load(b, src, i + half);
    E::template load<E::TABW>(w, pw, k << (log_n - 1 - log_s));
    E::mulv(b, w, F);  // w R_e: the Montgomery product leaves w b
    E::template bfly_l<E::IN>(a, b, F);
    E::template store<2 * E::IN>(dst, j, a, F);
    E::template store<2 * E::IN>(dst, j + s, b, F);
  }
}

template <class E>
hipError_t launch_noswap_round(const uint32_t* src, uint32_t* dst, uint32_t log_n, uint32_t log_s, const uint32_t* pw,
                               const typename E::Args& F, hipStream_t st) {
  if (log_n == 0 || log_s >= log_n || src == dst) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_noswap_round<E>), dim3(grid_1d(size_t(1) << (log_n - 1))), dim3(256), 0, st, src, dst, log_n,
                     log_s, pw, F);
  return hipGetLastError();
}

template <class E>
hipError_t launch_naive_round(const uint32_t* src, uint32_t* dst, uint32_t log_n, uint32_t log_s, const uint32_t* pw,
                              const typename E::Args& F, hipStream_t st) {
  if (log_n == 0 || log_s >= log_n) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_naive_round<E>), dim3(grid_1d(size_t(1) << (log_n - 1))), dim3(256), 0, st, src, dst, log_n,
                     log_s, pw, F);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- bealto / bellperson rivals
// The reference's radix-2^deg Stockham family (bealto.com's group FFT as bellperson ships it,
// FIELD_radix_fft_revised, GZKP-NTT.cu:391-464, and the four "improved" kernels, GZKP-NTT.cu:556-630,
// 632-719, 892-989, 1077-1210; ntt.h NTT_PLAN_BELLPERSON / NTT_PLAN_IMPROVED_V1..V4) as ONE kernel
// with the variant as a template argument: they compute the same round and differ only in how
// threads, groups and LDS rows are mapped, which is what they are kept for (comparison).  A round
// takes groups `index` of 2^deg elements x[index + i t] (t = n >> deg), multiplies element i by
// w_n^(e i), e = (n >> lgp >> deg) (index mod 2^lgp) (from the two-level tables: the reference raises
// FIELD_pow_lookup's twiddle per thread), runs deg radix-2 rounds in LDS with the pq table and writes
// y[((index - k) << deg) + k + i 2^lgp].  lsize = 2^(deg-1) threads per group, two elements each.
//   bellperson: inputs land bit-reversed in LDS, DIT rounds (twiddle, then butterfly), natural out;
//   v1:         DIF rounds (butterfly, then twiddle), bit-reversed out; 2^log_g groups per workgroup;
//   v2:         loads on the transposed map (thread -> group tid mod G: coalesced x[index + i t]);
//   v3:         and stores on it too when lgp > 0 (consecutive k: coalesced y);
//   v4:         and LDS rows of 2 lsize + 1 elements (the reference's bank-conflict padding).
// Lazy bounds (Eng29): loads < p, input products < 3p, every butterfly's outputs brought back < 4p.
__device__ __forceinline__ uint32_t brev_rt(uint32_t v, uint32_t bits) {
  return bits ? __builtin_bitreverse32(v) >> (32u - bits) : 0u;
}
template <class E>
__device__ __forceinline__ void lds_put_el(uint32_t* u, uint32_t slot, const uint32_t (&v)[E::W]) {
#pragma unroll
  for (int w = 0; w < E::W; ++w) u[(size_t)slot * E::W + w] = v[w];
}
template <class E>
__device__ __forceinline__ void lds_get_el(uint32_t (&v)[E::W], const uint32_t* u, uint32_t slot) {
#pragma unroll
  for (int w = 0; w < E::W; ++w) v[w] = u[(size_t)slot * E::W + w];
}
template <class E, int V>
__global__ __launch_bounds__(1024) void k_bealto(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                 const PassArgs<E> A, const BealtoArgs B) {
  extern __shared__ __attribute__((aligned(16))) uint32_t u_g[];
  const uint32_t deg = B.deg, lsz = 1u << (deg - 1), G = 1u << B.log_g, tid = threadIdx.x;
  const size_t t = (size_t)1 << (B.log_n - deg), p = (size_t)1 << B.lgp;
  const uint32_t rl = 2 * lsz + (V == BEALTO_V4 ? 1u : 0u);  // one group's LDS row, elements
  // compute map: group gid, lane lid; load map: transposed from v2 on
  const uint32_t lid = tid & (lsz - 1), gid = tid >> (deg - 1);
  const uint32_t gid_r = V >= BEALTO_V2 ? (tid & (G - 1)) : gid, lid_r = V >= BEALTO_V2 ? (tid >> B.log_g) : lid;
  const size_t index = (size_t)blockIdx.x * G + gid, index_r = (size_t)blockIdx.x * G + gid_r;
  const size_t k = index & (p - 1), k_r = index_r & (p - 1);
  {
    const size_t e = (t >> B.lgp) * k_r;  // w_n^(e i): < n for i < 2^deg
    uint32_t* u = u_g + (size_t)gid_r * rl * E::W;
#pragma unroll
    for (uint32_t j = 0; j < 2; ++j) {
      const uint32_t i = 2 * lid_r + j;
      uint32_t v[E::W];
      E::load(v, src, index_r + i * t);
      const size_t ei = e * i;
      typename E::Tw tl, th;
      E::tload(tl, A.tw_lo, (uint32_t)(ei & ((1u << A.lo_bits) - 1)));
      E::tload(th, A.tw_hi, (uint32_t)(ei >> A.lo_bits));
      E::mul(tl.w, th, A.F);  // (lo R_e) hi
      E::mulv(v, tl.w, A.F);  // v w_n^(e i), < 3p
      lds_put_el<E>(u, V == BEALTO_BELLPERSON ? brev_rt(i, deg) : i, v);
    }
  }
  __syncthreads();
  {
    uint32_t* u = u_g + (size_t)gid * rl * E::W;
    const uint32_t pqshift = B.max_deg - deg;
    for (uint32_t s = 0; s < deg; ++s) {
      const uint32_t rnd = V == BEALTO_BELLPERSON ? deg - 1 - s : s;
      const uint32_t bit = lsz >> rnd, di = lid & (bit - 1), i0 = (lid << 1) - di, i1 = i0 + bit;
      uint32_t a[E::W], b[E::W];
      lds_get_el<E>(a, u, i0);
      lds_get_el<E>(b, u, i1);
      typename E::Tw w;
      if (di) E::tload(w, A.tw_int, di << rnd << pqshift);  // w_{2^(deg - rnd)}^di
      if constexpr (V == BEALTO_BELLPERSON) {  // DIT: twiddle, then butterfly
        if (di) E::mul(b, w, A.F);
        E::template bfly_l<E::IN>(a, b, A.F);
        E::template reduce<2 * E::IN, E::IN>(b, A.F);
      } else {  // DIF: butterfly, then twiddle
        E::template bfly_l<E::IN>(a, b, A.F);
        if (di) E::mul(b, w, A.F);
        else E::template reduce<2 * E::IN, E::IN>(b, A.F);
      }
      E::template reduce<2 * E::IN, E::IN>(a, A.F);
      lds_put_el<E>(u, i0, a);
      lds_put_el<E>(u, i1, b);
      __syncthreads();
    }
  }
  // stores: the load map for v3 / v4 after the first round (consecutive k: coalesced), else the compute map
  const bool rmap = V >= BEALTO_V3 && B.lgp != 0;
  const size_t gi = rmap ? index_r : index, kk = rmap ? k_r : k;
  const uint32_t li = rmap ? lid_r : lid;
  const uint32_t* u = u_g + (size_t)(rmap ? gid_r : gid) * rl * E::W;
  const size_t base = ((gi - kk) << deg) + kk;
#pragma unroll
  for (uint32_t j = 0; j < 2; ++j) {
    const uint32_t i = li + j * lsz;
    uint32_t v[E::W];
    lds_get_el<E>(v, u, V == BEALTO_BELLPERSON ? i : brev_rt(i, deg));
    E::template store<E::IN>(dst, base + i * p, v, A.F);
  }
}

template <class E>
hipError_t launch_bealto(int variant, const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, const BealtoArgs& B,
                         hipStream_t st) {
  if constexpr (!HasStockham<E>::value) {
    return hipErrorInvalidValue;
  } else {
    if (B.deg < 1 || B.deg > B.max_deg || B.deg > B.log_n || B.log_n - B.deg < B.log_g || src == dst)
      return hipErrorInvalidValue;
    const uint32_t threads = (1u << (B.deg - 1)) << B.log_g;
    const size_t grid = ((size_t)1 << (B.log_n - B.deg)) >> B.log_g;
    const size_t lds = ((size_t)((2u << (B.deg - 1)) + (variant == BEALTO_V4 ? 1u : 0u)) << B.log_g) * E::W * 4;
    if (threads > 1024 || grid > 0x7fffffffull || lds > 64 * 1024) return hipErrorInvalidValue;
    const dim3 g((uint32_t)grid), b(threads);
    switch (variant) {
      case BEALTO_BELLPERSON: hipLaunchKernelGGL((k_bealto<E, BEALTO_BELLPERSON>), g, b, lds, st, src, dst, A, B); break;
      case BEALTO_V1: hipLaunchKernelGGL((k_bealto<E, BEALTO_V1>), g, b, lds, st, src, dst, A, B); break;
      case BEALTO_V2: hipLaunchKernelGGL((k_bealto<E, BEALTO_V2>), g, b, lds, st, src, dst, A, B); break;
      case BEALTO_V3: hipLaunchKernelGGL((k_bealto<E, BEALTO_V3>), g, b, lds, st, src, dst, A, B); break;
      case BEALTO_V4: hipLaunchKernelGGL((k_bealto<E, BEALTO_V4>), g, b, lds, st, src, dst, A, B); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
}

// k_build_tw's table as Shoup pairs: entry (c, k) = (w, floor(w B / p)) with w = w_n^((c*k) << log_m)
// canonical, in the engine's twiddle format (E::TW words).  t = lo_s * hi = w B mod p; w = t / B
// (Montgomery product by 1); floor(w B / p) = (-(w B mod p)) p^-1 mod B (shoup_ws29).
template <class E>
__global__ void k_build_tw_sh(uint32_t* __restrict__ out, size_t count, uint32_t log_r, uint32_t log_t,
                              uint32_t log_m, const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hi,
                              uint32_t lo_bits, const typename E::Args F, const uint32_t* __restrict__ pinvB) {
  constexpr int L = E::W;
  NTT_GRID_STRIDE(idx, count) {
    const size_t k = (idx >> log_t) & ((1ull << log_r) - 1);
    const size_t c = ((idx >> (log_t + log_r)) << log_t) + (idx & ((1ull << log_t) - 1));
    const size_t e = (c * k) << log_m;
    typename E::Tw a, b;
    E::tload(a, lo, (uint32_t)(e & ((1ull << lo_bits) - 1)));
    E::tload(b, hi, (uint32_t)(e >> lo_bits));
    E::mul(a.w, b, F);  // w B mod p, < 3p
    uint32_t wr[L], w[L], one[L], t[L], ws[L], pib[L];
#pragma unroll
    for (int i = 0; i < L; ++i) {
      wr[i] = a.w[i];
      one[i] = i == 0 ? 1u : 0u;
      pib[i] = pinvB[i];
    }
    E::template reduce<4, 1, false>(wr, F);  // canonical w B mod p
#pragma unroll
    for (int i = 0; i < L; ++i) w[i] = wr[i];
    E::mulv(w, one, F);  // w, < 3p
    E::template reduce<4, 1, false>(w, F);
    neg29<L>(t, wr);
    mullo29<L>(ws, t, pib);
    uint32_t o[E::TW];
#pragma unroll
    for (int i = 0; i < E::TW; ++i) o[i] = i < L ? w[i] : (i < 2 * L ? ws[i - L] : 0u);
    uint4* p = reinterpret_cast<uint4*>(out + idx * E::TW);
#pragma unroll
    for (int q = 0; q < E::TW / 4; ++q) p[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  }
}

template <class E>
hipError_t launch_build_tw_sh(uint32_t* out, size_t count, uint32_t log_r, uint32_t log_t, uint32_t log_m,
                              const uint32_t* lo, const uint32_t* hi, uint32_t lo_bits, const typename E::Args& F,
                              const uint32_t* pinvB, hipStream_t st) {
  if constexpr (!E::SHOUP_OUTER) {
    return hipErrorInvalidValue;
  } else {
    hipLaunchKernelGGL((k_build_tw_sh<E>), dim3(grid_1d(count)), dim3(256), 0, st, out, count,
                       log_r, log_t, log_m, lo, hi, lo_bits, F, pinvB);
    return hipGetLastError();
  }
}

// GZKP rival's `rearrange` (GZKP-NTT.cu:167-233 via reverse pairs), out of place: dst[i] = src[drev(i)].
// The reference's rounds are radix 2, so its permutation is the bit reversal; here every pass is a
// natural-order radix-2^r_q DFT, so the permutation that gives natural-order output is the mixed-radix
// digit reversal: digit q of i (r_q bits, from the low end, in pass order) becomes digit q of the
// source index counted from the HIGH end.  (All r_q = 1 gives the bit reversal.)
struct DigitRev {
  uint32_t nd;
  uint32_t r[8];
};
template <int MEMW>
__global__ void k_digitrev(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t log_n,
                           DigitRev D) {
  NTT_GRID_STRIDE(i, (size_t(1) << log_n)) {
    size_t j = 0, rem = i;
    uint32_t top = log_n;
    for (uint32_t q = 0; q < D.nd; ++q) {
      top -= D.r[q];
      j |= (rem & ((1ull << D.r[q]) - 1)) << top;
      rem >>= D.r[q];
    }
    if (D.nd == 0) j = (size_t)(__brevll((unsigned long long)i) >> (64 - log_n));  // log_n 1-bit digits
    if constexpr (MEMW % 4 == 0) {
#pragma unroll
      for (int q = 0; q < MEMW / 4; ++q)
        reinterpret_cast<uint4*>(dst + i * MEMW)[q] = reinterpret_cast<const uint4*>(src + j * MEMW)[q];
    } else {
#pragma unroll
      for (int q = 0; q < MEMW; ++q) dst[i * MEMW + q] = src[j * MEMW + q];
    }
  }
}

template <class E>
hipError_t launch_bitrev(const uint32_t* src, uint32_t* dst, uint32_t log_n, const uint32_t* digits, uint32_t nd,
                         hipStream_t st) {
  DigitRev D{};
  uint32_t sum = 0;
  if (nd > 8 || log_n == 0 || log_n > 40) return hipErrorInvalidValue;
  D.nd = nd;
  for (uint32_t q = 0; q < nd; ++q) sum += (D.r[q] = digits[q]);
  if (nd > 0 && sum != log_n) return hipErrorInvalidValue;  // nd = 0: the bit reversal (digits unused)
  const size_t n = 1ull << log_n;
  hipLaunchKernelGGL((k_digitrev<E::MEMW>), dim3(grid_1d(n)), dim3(256), 0, st, src, dst, log_n,
                     D);
  return hipGetLastError();
}

// Four-step twiddle table of one rank (ntt_rplan): entry (a, b) at a 2^log_cols + b holds
// w_n^((row0 + a)(col0 + b) mod n) R_e (the epilogue of the final pass multiplies by it with mulv),
// from the two-level tables (lo_s = lo R_e, so lo_s * hi = w R_e).
template <class E>
__global__ void k_build_fs_tw(uint32_t* __restrict__ out, uint32_t log_rows, uint32_t log_cols, uint64_t row0,
                              uint64_t col0, uint32_t log_n, const uint32_t* __restrict__ lo,
                              const uint32_t* __restrict__ hi, uint32_t lo_bits, const typename E::Args F,
                              const uint32_t* __restrict__ scale) {
  NTT_GRID_STRIDE(idx, (size_t(1) << (log_rows + log_cols))) {
    const uint64_t a = idx >> log_cols, b = idx & ((1ull << log_cols) - 1);
    const uint64_t e = ((row0 + a) * (col0 + b)) & ((1ull << log_n) - 1);
    typename E::Tw x, y;
    E::tload(x, lo, (uint32_t)(e & ((1ull << lo_bits) - 1)));
    E::tload(y, hi, (uint32_t)(e >> lo_bits));
    E::mul(x.w, y, F);
    if (scale) {  // a constant folded into every entry (the four-step's row n2^-1); mul takes any x < B
      E::tload(y, scale, 0);
      E::mul(x.w, y, F);
    }
    E::template store<E::MUL_OUT, false, E::TABW>(out, idx, x.w, F);
  }
}

template <class E>
hipError_t launch_build_fs_tw(uint32_t* out, uint32_t log_rows, uint32_t log_cols, uint64_t row0, uint64_t col0,
                              uint32_t log_n, const uint32_t* lo, const uint32_t* hi, uint32_t lo_bits,
                              const typename E::Args& F, hipStream_t st, const uint32_t* scale) {
  const size_t count = 1ull << (log_rows + log_cols);
  hipLaunchKernelGGL((k_build_fs_tw<E>), dim3(grid_1d(count)), dim3(256), 0, st, out, log_rows,
                     log_cols, row0, col0, log_n, lo, hi, lo_bits, F, scale);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- four-step helpers
// Multi-GPU four-step, local steps.  twiddle_pack: src is [rows][row_len] (row-major);
// element (a, b) is multiplied by w_n^((row0 + a) * b) and written to dst block b / bw (bw =
// row_len / G) at blk * peer_stride + a * bw + b % bw, i.e. dst = [G][rows][bw] (peer_stride =
// rows * bw): one contiguous chunk per peer for the all-to-all.  A larger peer_stride interleaves
// several vectors' chunks per peer (the distributed polymul exchanges a and b in one all-to-all).  Twiddles from the plan's two-level tables: lo_s holds lo * R_e (R_e the engine's
// Montgomery radix), so t = lo_s[e & mask] * hi[e >> lo_bits] = w_n^e R_e and mulv(x, t) = x w_n^e.
template <class E>
__global__ void k_twiddle_pack(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t log_rows,
                               uint32_t log_len, uint32_t log_bw, uint64_t row0, uint32_t log_n,
                               const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hi, uint32_t lo_bits,
                               const typename E::Args F, uint64_t peer_stride) {
  NTT_GRID_STRIDE(i, (1ull << (log_rows + log_len))) {
    const uint64_t a = i >> log_len, b = i & ((1ull << log_len) - 1);
    const uint64_t e = ((row0 + a) * b) & ((1ull << log_n) - 1);
    uint32_t x[E::W];
    typename E::Tw w, h;
    E::load(x, src, i);
    E::tload(w, lo, (uint32_t)(e & ((1ull << lo_bits) - 1)));
    E::tload(h, hi, (uint32_t)(e >> lo_bits));
    E::mul(w.w, h, F);
    E::mulv(x, w.w, F);
    const size_t blk = b >> log_bw, off = b & ((1ull << log_bw) - 1);
    E::template store<E::MUL_OUT>(dst, blk * peer_stride + (a << log_bw) + off, x, F);
  }
}

// Coset scale (low-degree-extension step): data[j] *= c^j over `batch` vectors of 2^log_n elements,
// c^j from two-level tables (lo_s[j & mask] = c^lo R_e, hi[j >> lo_bits] = Shoup entries), so
// t = lo_s * hi = c^j R_e and mulv(x, t) = x c^j.  One HBM read + write, two products per element.
template <class E>
__global__ void k_scale_pow(uint32_t* __restrict__ data, uint32_t log_n, const uint32_t* __restrict__ lo_s,
                            const uint32_t* __restrict__ hi, uint32_t lo_bits, const typename E::Args F,
                            size_t batch_stride) {
  NTT_GRID_STRIDE(j, (size_t(1) << log_n)) {
    uint32_t* d = data + (size_t)blockIdx.y * batch_stride;
    uint32_t x[E::W];
    typename E::Tw w, h;
    E::load(x, d, j);
    E::tload(w, lo_s, (uint32_t)(j & ((1ull << lo_bits) - 1)));
    E::tload(h, hi, (uint32_t)(j >> lo_bits));
    E::mul(w.w, h, F);
    E::mulv(x, w.w, F);
    E::template store<E::MUL_OUT>(d, j, x, F);
  }
}

template <class E>
hipError_t launch_scale_pow(uint32_t* data, uint32_t log_n, uint32_t batch, const uint32_t* lo_s, const uint32_t* hi,
                            uint32_t lo_bits, const typename E::Args& F, hipStream_t st) {
  const size_t n = 1ull << log_n;
  const dim3 grid(grid_1d(n), batch);
  hipLaunchKernelGGL((k_scale_pow<E>), grid, dim3(256), 0, st, data, log_n, lo_s, hi, lo_bits, F,
                     n * (size_t)E::MEMW);
  return hipGetLastError();
}

// dst[c][r] = src[r][c] for a rows x cols matrix of MEMW-word elements (32x32 tiles through LDS,
// 16-B vector accesses).  Source rows come in blocks of 2^log_blk_rows rows, block b starting at
// element b * blk_stride (blk_stride = 2^(log_blk_rows + log_cols): one dense matrix; larger: the
// per-peer chunks of an all-to-all that carried several vectors).
template <int MEMW>
__global__ void k_transpose(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t log_rows,
                            uint32_t log_cols, uint32_t log_blk_rows, uint64_t blk_stride) {
  constexpr int TILE = 32;
  constexpr bool VEC = (MEMW % 4) == 0;
  __shared__ uint32_t tile[TILE][TILE + 1][MEMW];
  const uint64_t rows = 1ull << log_rows, cols = 1ull << log_cols;
  const uint64_t bx = (uint64_t)blockIdx.x * TILE, by = (uint64_t)blockIdx.y * TILE;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int k = ty; k < TILE; k += 8) {
    const uint64_t r = by + k, c = bx + tx;
    if (r < rows && c < cols) {
      const uint64_t rin = r & ((1ull << log_blk_rows) - 1);
      const uint32_t* s = src + ((r >> log_blk_rows) * blk_stride + (rin << log_cols) + c) * MEMW;
      if constexpr (VEC) {
#pragma unroll
        for (int w = 0; w < MEMW / 4; ++w) {
          const uint4 v = reinterpret_cast<const uint4*>(s)[w];
          tile[k][tx][4 * w] = v.x;
          tile[k][tx][4 * w + 1] = v.y;
          tile[k][tx][4 * w + 2] = v.z;
          tile[k][tx][4 * w + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int w = 0; w < MEMW; ++w) tile[k][tx][w] = s[w];
      }
    }
  }
  __syncthreads();
  for (int k = ty; k < TILE; k += 8) {
    const uint64_t c = bx + k, r = by + tx;
    if (r < rows && c < cols) {
      uint32_t* d = dst + (c * rows + r) * MEMW;
      if constexpr (VEC) {
#pragma unroll
        for (int w = 0; w < MEMW / 4; ++w)
          reinterpret_cast<uint4*>(d)[w] =
              make_uint4(tile[tx][k][4 * w], tile[tx][k][4 * w + 1], tile[tx][k][4 * w + 2], tile[tx][k][4 * w + 3]);
      } else {
#pragma unroll
        for (int w = 0; w < MEMW; ++w) d[w] = tile[tx][k][w];
      }
    }
  }
}

template <class E>
hipError_t launch_twiddle_pack(const uint32_t* src, uint32_t* dst, uint32_t log_rows, uint32_t log_len,
                               uint32_t log_bw, uint64_t row0, uint32_t log_n, const uint32_t* lo, const uint32_t* hi,
                               uint32_t lo_bits, const typename E::Args& F, uint64_t peer_stride, hipStream_t st) {
  const size_t total = 1ull << (log_rows + log_len);
  hipLaunchKernelGGL((k_twiddle_pack<E>), dim3(grid_1d(total)), dim3(256), 0, st, src, dst, log_rows,
                     log_len, log_bw, row0, log_n, lo, hi, lo_bits, F, peer_stride);
  return hipGetLastError();
}

template <class E>
hipError_t launch_transpose(const uint32_t* src, uint32_t* dst, uint32_t log_rows, uint32_t log_cols,
                            uint32_t log_blk_rows, uint64_t blk_stride, hipStream_t st) {
  const uint64_t rows = 1ull << log_rows, cols = 1ull << log_cols;
  const dim3 grid((uint32_t)((cols + 31) / 32), (uint32_t)((rows + 31) / 32));
  hipLaunchKernelGGL((k_transpose<E::MEMW>), grid, dim3(256), 0, st, src, dst, log_rows, log_cols, log_blk_rows,
                     blk_stride);
  return hipGetLastError();
}

// In-place digit reversal after an in-place final pass (NTT_PLAN_IN_PLACE; the replacement for the
// reference's SSIP stage-2 mirror pairs, GZKP-NTT.cu:1359-1449).  With a palindromic radix sequence
// (R_1 = R_p = 2^R, middle widths symmetric) the element at position (k1, mid, kn) =
// k1 2^(L-R) + mid 2^R + kn belongs at (kn, midrev, k1): an involution, so the permutation is a set of
// disjoint swaps.  A workgroup owns the tile pair {(I tb + a, mid, J tb + b)} and its image
// {(J tb + a, midrev, I tb + b)} (a, b < tb): both tiles are read as tb-element contiguous rows, swapped
// through LDS and written back transposed.  Of the two workgroups of a pair the one with the larger
// index exits; a tile that is its own image (mid = midrev, I = J) is transposed in place.
template <int MW>
__global__ __launch_bounds__(256) void k_digitrev_swap(uint32_t* data, DrevArgs A) {
  constexpr int SL = MW + 1;  // LDS slot stride (words): odd, so transposed reads spread over banks
  __shared__ uint32_t tile[2][256 * SL];
  const uint32_t tl = A.tb_log, ntl = A.R - tl;
  const uint64_t u = A.unit0 + blockIdx.x;
  const uint32_t nm = (1u << ntl) - 1;
  const uint32_t lo = (uint32_t)(u & nm), hi = (uint32_t)((u >> ntl) & nm);
  // diagonal order (A.diag): I = lo, J = lo + hi, so that neighbouring workgroups differ in both tile
  // coordinates and neither tile of a pair walks down one column of 2^(log_n - R)-element rows
  // (power-of-two strides that land on the same HBM channels); else row-major (I = hi, J = lo)
  const uint32_t I = A.diag ? lo : hi, J = A.diag ? ((lo + hi) & nm) : lo;
  const uint64_t mid = u >> (2 * ntl);
  uint64_t m = mid, midrev = 0;
  for (uint32_t i = 0; i < A.nmid; ++i) {
    midrev |= (m & ((1ull << A.mid_bits[i]) - 1)) << A.mid_off[i];
    m >>= A.mid_bits[i];
  }
  // the image tile (midrev, J, I) in the same order
  const uint64_t partner = (midrev << (2 * ntl)) |
                           (A.diag ? (((uint64_t)((I - J) & nm) << ntl) | J) : (((uint64_t)J << ntl) | I));
  if (partner < u) return;  // the pair is handled by the partner's workgroup (uniform exit)
  uint32_t* d = data + (size_t)blockIdx.y * A.batch_stride;
  const uint32_t t = threadIdx.x, tb = 1u << tl;
  const bool act = t < (tb << tl);
  const uint32_t a = t >> tl, b = t & (tb - 1);
  const uint32_t sh = A.log_n - A.R;
  const size_t posA = ((size_t)(I * tb + a) << sh) + (mid << A.R) + J * tb + b;
  const size_t posB = ((size_t)(J * tb + a) << sh) + (midrev << A.R) + I * tb + b;
  uint32_t va[MW], vb[MW];
  if (act) {
    if constexpr (MW % 4 == 0) {
#pragma unroll
      for (int w = 0; w < MW / 4; ++w) {
        const uint4 x = reinterpret_cast<const uint4*>(d + posA * MW)[w];
        const uint4 y = reinterpret_cast<const uint4*>(d + posB * MW)[w];
        va[4 * w] = x.x, va[4 * w + 1] = x.y, va[4 * w + 2] = x.z, va[4 * w + 3] = x.w;
        vb[4 * w] = y.x, vb[4 * w + 1] = y.y, vb[4 * w + 2] = y.z, vb[4 * w + 3] = y.w;
      }
    } else {
#pragma unroll
      for (int w = 0; w < MW; ++w) va[w] = d[posA * MW + w], vb[w] = d[posB * MW + w];
    }
#pragma unroll
    for (int w = 0; w < MW; ++w) tile[0][t * SL + w] = va[w], tile[1][t * SL + w] = vb[w];
  }
  __syncthreads();
  if (!act) return;
  const uint32_t tt = (b << tl) + a;  // the transposed slot
#pragma unroll
  for (int w = 0; w < MW; ++w) va[w] = tile[1][tt * SL + w], vb[w] = tile[0][tt * SL + w];
  const bool self = partner == u;
  if constexpr (MW % 4 == 0) {
#pragma unroll
    for (int w = 0; w < MW / 4; ++w) {
      reinterpret_cast<uint4*>(d + posA * MW)[w] = make_uint4(va[4 * w], va[4 * w + 1], va[4 * w + 2], va[4 * w + 3]);
      if (!self)
        reinterpret_cast<uint4*>(d + posB * MW)[w] = make_uint4(vb[4 * w], vb[4 * w + 1], vb[4 * w + 2], vb[4 * w + 3]);
    }
  } else {
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      d[posA * MW + w] = va[w];
      if (!self) d[posB * MW + w] = vb[w];
    }
  }
}

template <class E>
hipError_t launch_digitrev_swap(uint32_t* data, const DrevArgs& A, uint32_t batch, hipStream_t st) {
  if (A.R < A.tb_log || 2 * A.R > A.log_n || A.tb_log > 4) return hipErrorInvalidValue;
  // grid.x * blockDim.x must stay below 2^32 threads: 2^(log_n - 2 tb_log) tile pairs go as launches
  // of at most 2^23 workgroups (A.unit0 = the first pair of the launch)
  const uint64_t units = 1ull << (A.log_n - 2 * A.tb_log), chunk = 1ull << 23;
  for (uint64_t u0 = 0; u0 < units; u0 += chunk) {
    DrevArgs B = A;
    B.unit0 = u0;
    const uint64_t cnt = units - u0 < chunk ? units - u0 : chunk;
    hipLaunchKernelGGL((k_digitrev_swap<E::MEMW>), dim3((uint32_t)cnt, batch), dim3(256), 0, st, data, B);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  }
  return hipSuccess;
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
struct FillMap {
  uint64_t row0;       // global index of local row 0
  uint32_t log_inner;  // local row length (log2); 64 = identity map
  uint32_t log_stride; // global stride of the inner index (log2)
};
__device__ __forceinline__ uint64_t fill_index(size_t i, const FillMap& m) {
  if (m.log_inner >= 64) return i;
  return m.row0 + (i >> m.log_inner) + ((uint64_t)(i & ((1ull << m.log_inner) - 1)) << m.log_stride);
}

template <int MEMW>
__global__ void k_fill_random(uint32_t* __restrict__ dst, size_t n, uint64_t seed, uint32_t nrand, uint32_t top_bits,
                              FillMap fm) {
  NTT_GRID_STRIDE(i, n) {
    const uint64_t j = fill_index(i, fm);
    if constexpr (MEMW == 2) {
      const uint64_t v = splitmix64((seed << 32) + 4 * j) & ((1ull << top_bits) - 1);
      reinterpret_cast<uint2*>(dst)[i] = make_uint2((uint32_t)v, 0u);
    } else {
      uint32_t v[MEMW];
#pragma unroll
      for (int l = 0; l < MEMW / 2; ++l) {
        uint64_t limb = 0;
        if ((uint32_t)l < nrand) {
          limb = splitmix64((seed << 32) + 4 * j + l);
          if ((uint32_t)l + 1 == nrand && top_bits < 64) limb &= (1ull << top_bits) - 1;
        }
        v[2 * l] = (uint32_t)limb;
        v[2 * l + 1] = (uint32_t)(limb >> 32);
      }
      uint4* p = reinterpret_cast<uint4*>(dst + i * MEMW);
#pragma unroll
      for (int q = 0; q < MEMW / 4; ++q) p[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
  }
}

template <int MEMW>
__global__ void k_fill_iota(uint32_t* __restrict__ dst, size_t n, FillMap fm) {
  NTT_GRID_STRIDE(i, n) {
    const uint64_t j = fill_index(i, fm);
    if constexpr (MEMW == 2) {
      reinterpret_cast<uint2*>(dst)[i] = make_uint2((uint32_t)j, (uint32_t)((uint64_t)j >> 32));
    } else {
      uint4* p = reinterpret_cast<uint4*>(dst + i * MEMW);
      p[0] = make_uint4((uint32_t)j, (uint32_t)((uint64_t)j >> 32), 0u, 0u);
#pragma unroll
      for (int q = 1; q < MEMW / 4; ++q) p[q] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
}

template <class E>
__global__ void k_pointwise_mul(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, uint32_t* __restrict__ c,
                                size_t n, const typename E::Args F, const uint32_t* __restrict__ r2, const FsMap m,
                                const uint32_t mapped) {
  NTT_GRID_STRIDE(j, n) {
    uint32_t x[E::W], y[E::W];
    typename E::Tw z;  // R_e mod p as a twiddle: mulv leaves x y / R_e
    const size_t src = mapped ? m(j, 0) : j;  // a four-step piece gathered from the column layout
    E::load(x, a, src);
    E::load(y, b, src);
    E::tload(z, r2, 0);
    E::mulv(x, y, F);
    E::mul(x, z, F);
    E::template store<E::MUL_OUT>(c, j, x, F);
  }
}

// Canonical-range check (the reference's padded-store `BAD LIMB` trap, impl_cuda.cu:1402-1408, as a
// query): counts elements that are not < p in a caller buffer of E::MEMW-word elements.  p holds
// the modulus in MEMW little-endian 32-bit words (zero above its top word).
template <int MEMW>
__global__ void k_count_noncanonical(const uint32_t* __restrict__ d, size_t n, ModWords<MEMW> p,
                                     unsigned long long* __restrict__ bad) {
  NTT_GRID_STRIDE(i, n) {
    const uint32_t* e = d + i * MEMW;
    int cmp = 0;  // sign of e - p, decided by the most significant differing word
#pragma unroll
    for (int k = MEMW - 1; k >= 0; --k)
      if (cmp == 0 && e[k] != p.w[k]) cmp = e[k] < p.w[k] ? -1 : 1;
    if (cmp >= 0) atomicAdd(bad, 1ull);
  }
}

template <class E>
hipError_t launch_count_noncanonical(const uint32_t* d, size_t n, const ModWords<E::MEMW>& p,
                                     unsigned long long* bad, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL((k_count_noncanonical<E::MEMW>), dim3(grid_1d(n)), dim3(256), 0, st, d, n, p,
                     bad);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- launchers
// Radices the planner can emit: column/final passes use 3 <= r <= tile_log - MIN_COLS_LOG, single-workgroup
// transforms 3 <= r <= tile_log.  Only those are instantiated.
// Plain (no prologue) pass launch; later column passes of engines whose scratch is narrower than the
// caller's layout read scratch (SRC_USER = false).
template <class E, int LOGR, int KIND, bool FULLTW, bool FAST, int FSM>
static hipError_t launch_plain(const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, dim3 g, dim3 b,
                               hipStream_t st) {
  if constexpr (KIND == KIND_COLUMN && FULLTW && FAST && E::SHOUP_OUTER) {
    if (A.tw_sh) {  // Shoup-pair outer twiddles: later column passes, or pass 1 of a small plan
      constexpr bool SU = E::SCRW == E::MEMW;  // one instance when scratch and caller layouts agree
      if (A.src_user && !SU) return hipErrorInvalidValue;
      hipLaunchKernelGGL((k_pass<E, LOGR, KIND, true, true, PRO_NONE, SU, FSM, true>), g, b, 0, st, src, dst, A);
      return hipGetLastError();
    }
  }
  if (A.tw_sh) return hipErrorInvalidValue;
  if constexpr (KIND == KIND_COLUMN && E::SCRW != E::MEMW) {
    if (!A.src_user) {
      hipLaunchKernelGGL((k_pass<E, LOGR, KIND, FULLTW, FAST, PRO_NONE, false, FSM>), g, b, 0, st, src, dst, A);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((k_pass<E, LOGR, KIND, FULLTW, FAST, PRO_NONE, true, FSM>), g, b, 0, st, src, dst, A);
  return hipGetLastError();
}

// FSM (four-step addressing) instance for this pass: column passes need it only for a mapped input
// (first pass) or Mode I twiddles; final / single passes for a mapped output, Mode I or the epilogue.
template <class E, int KIND, int LOGR, bool FULLTW, bool FAST>
static hipError_t launch_fsm(const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, dim3 g, dim3 b,
                             hipStream_t st) {
  if constexpr (KIND == KIND_STOCKHAM || KIND == KIND_DIT) {
    if (A.fs || A.tw_epi) return hipErrorInvalidValue;
    return launch_plain<E, LOGR, KIND, FULLTW, FAST, 0>(src, dst, A, g, b, st);
  }
  if (A.fs == 0 && !A.tw_epi) return launch_plain<E, LOGR, KIND, FULLTW, FAST, 0>(src, dst, A, g, b, st);
  if constexpr (KIND != KIND_COLUMN) {
    if (A.tw_epi) return launch_plain<E, LOGR, KIND, FULLTW, FAST, 2>(src, dst, A, g, b, st);
  }
  return launch_plain<E, LOGR, KIND, FULLTW, FAST, 1>(src, dst, A, g, b, st);
}

template <class E, int KIND, int LOGR>
static hipError_t launch_pass_r(const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, uint32_t grid,
                                uint32_t batch, hipStream_t st) {
  constexpr int TL = tile_log_of<E>();
  constexpr int MAXR = (KIND == KIND_SINGLE || KIND == KIND_ROWS) ? TL : TL - E::MIN_COLS_LOG;
  // KIND_ROWS: the engines and radices the ntt_*_rows.hip units instantiate (>= 2 transforms per tile);
  // the quotient-estimate engines only in their FAST form
  constexpr bool ROWS_OFF = KIND == KIND_ROWS && (!HasRows<E>::value || LOGR < kRowsMinLog ||
                                                  LOGR > rows_max_log<E>() || LOGR >= TL);
  if constexpr (LOGR > MAXR || ROWS_OFF || ((KIND == KIND_STOCKHAM || KIND == KIND_DIT) && !HasStockham<E>::value)) {
    return hipErrorInvalidValue;
  } else {
    constexpr int TE = (KIND == KIND_SINGLE) ? (1 << LOGR) : (1 << TL);
    constexpr int NT = TE / E::EPT;
    const dim3 g(grid, batch), b(NT < 64 ? 64 : NT);
    if constexpr (E::FASTRED) {
      if (A.F.red_ok) {
        if constexpr (KIND == KIND_STOCKHAM || KIND == KIND_DIT) {
          return A.tw_full ? launch_fsm<E, KIND, LOGR, true, true>(src, dst, A, g, b, st)
                           : launch_fsm<E, KIND, LOGR, false, true>(src, dst, A, g, b, st);
        }
        if constexpr (KIND == KIND_COLUMN) {
          if (A.tw_full && A.src2) {
            if (A.fs)  // Mode I polymul inverse (ntt_rplan)
              hipLaunchKernelGGL((k_pass<E, LOGR, KIND, true, true, PRO_PW, true, 1>), g, b, 0, st, src, dst, A);
            else
              hipLaunchKernelGGL((k_pass<E, LOGR, KIND, true, true, PRO_PW>), g, b, 0, st, src, dst, A);
            return hipGetLastError();
          }
          if (A.tw_full && A.tw_in) {
            if (A.fs) return hipErrorInvalidValue;
            hipLaunchKernelGGL((k_pass<E, LOGR, KIND, true, true, PRO_COSET>), g, b, 0, st, src, dst, A);
            return hipGetLastError();
          }
          if (A.tw_full) return launch_fsm<E, KIND, LOGR, true, true>(src, dst, A, g, b, st);
        }
        if (A.src2 || A.tw_in) return hipErrorInvalidValue;  // fused prologues: FAST column + full tables
        return launch_fsm<E, KIND, LOGR, false, true>(src, dst, A, g, b, st);
      }
    }
    if (A.src2 || A.tw_in) return hipErrorInvalidValue;
    if constexpr (KIND == KIND_ROWS && E::FASTRED) {
      return hipErrorInvalidValue;  // fast reductions only (the caller runs KIND_SINGLE otherwise)
    } else {
      if constexpr (KIND == KIND_COLUMN || KIND == KIND_STOCKHAM || KIND == KIND_DIT) {
        if (A.tw_full) return launch_fsm<E, KIND, LOGR, true, false>(src, dst, A, g, b, st);
      }
      return launch_fsm<E, KIND, LOGR, false, false>(src, dst, A, g, b, st);
    }
  }
}

template <class E, int KIND>
hipError_t launch_pass_kind(int logr, const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, uint32_t grid,
                                uint32_t batch, hipStream_t st) {
  switch (logr) {
    case 3: return launch_pass_r<E, KIND, 3>(src, dst, A, grid, batch, st);
    case 4: return launch_pass_r<E, KIND, 4>(src, dst, A, grid, batch, st);
    case 5: return launch_pass_r<E, KIND, 5>(src, dst, A, grid, batch, st);
    case 6: return launch_pass_r<E, KIND, 6>(src, dst, A, grid, batch, st);
    case 7: return launch_pass_r<E, KIND, 7>(src, dst, A, grid, batch, st);
    case 8: return launch_pass_r<E, KIND, 8>(src, dst, A, grid, batch, st);
    case 9: return launch_pass_r<E, KIND, 9>(src, dst, A, grid, batch, st);
    case 10: return launch_pass_r<E, KIND, 10>(src, dst, A, grid, batch, st);
    case 11: return launch_pass_r<E, KIND, 11>(src, dst, A, grid, batch, st);
    case 12: return launch_pass_r<E, KIND, 12>(src, dst, A, grid, batch, st);
    case 13: return launch_pass_r<E, KIND, 13>(src, dst, A, grid, batch, st);
    default: return hipErrorInvalidValue;
  }
}

template <class E>
hipError_t launch_pass(int kind, int logr, const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, uint32_t grid,
                       uint32_t batch, hipStream_t st) {
  if (kind == KIND_COLUMN) return launch_pass_kind<E, KIND_COLUMN>(logr, src, dst, A, grid, batch, st);
  if (kind == KIND_FINAL) return launch_pass_kind<E, KIND_FINAL>(logr, src, dst, A, grid, batch, st);
  if (kind == KIND_STOCKHAM || kind == KIND_DIT) {
    if constexpr (HasStockham<E>::value) {
      if (kind == KIND_DIT) return launch_pass_kind<E, KIND_DIT>(logr, src, dst, A, grid, batch, st);
      return launch_pass_kind<E, KIND_STOCKHAM>(logr, src, dst, A, grid, batch, st);
    }
    return hipErrorInvalidValue;
  }
  if (kind == KIND_ROWS) {  // grid = batch / (TILE / 2^logr) workgroups, batch argument 1
    if constexpr (HasRows<E>::value) return launch_pass_kind<E, KIND_ROWS>(logr, src, dst, A, grid, batch, st);
    return hipErrorInvalidValue;
  }
  return launch_pass_kind<E, KIND_SINGLE>(logr, src, dst, A, grid, batch, st);
}

template <class E>
hipError_t launch_naive(const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, uint32_t batch, hipStream_t st) {
  hipLaunchKernelGGL((k_dft_naive<E>), dim3(1, batch), dim3(64), 0, st, src, dst, A);
  return hipGetLastError();
}

template <class E>
hipError_t launch_fill(int kind, uint32_t* dst, size_t n, uint64_t seed, uint32_t nrand, uint32_t top_bits,
                       uint64_t row0, uint32_t log_inner, uint32_t log_stride, hipStream_t st) {
  const uint32_t blocks = grid_1d(n);
  const FillMap fm{row0, log_inner, log_stride};
  if (kind == 0)
    hipLaunchKernelGGL((k_fill_iota<E::MEMW>), dim3(blocks), dim3(256), 0, st, dst, n, fm);
  else
    hipLaunchKernelGGL((k_fill_random<E::MEMW>), dim3(blocks), dim3(256), 0, st, dst, n, seed, nrand, top_bits, fm);
  return hipGetLastError();
}

template <class E>
hipError_t launch_pointwise(const uint32_t* a, const uint32_t* b, uint32_t* c, size_t n, const typename E::Args& F,
                            const uint32_t* d_r2, hipStream_t st, const FsMap* in_map) {
  const uint32_t blocks = grid_1d(n);
  const FsMap m = in_map ? *in_map : FsMap{};
  hipLaunchKernelGGL((k_pointwise_mul<E>), dim3(blocks), dim3(256), 0, st, a, b, c, n, F, d_r2, m, in_map ? 1u : 0u);
  return hipGetLastError();
}

// One pass kind of one engine per translation unit (the kernels dominate compile time).
#define NTT_INSTANTIATE_KIND(E, KIND)                                                                          \
  template hipError_t launch_pass_kind<E, KIND>(int, const uint32_t*, uint32_t*, const PassArgs<E>&, uint32_t, \
                                                uint32_t, hipStream_t);

#define NTT_EXTERN_KIND(E, KIND)                                                                                     \
  extern template hipError_t launch_pass_kind<E, KIND>(int, const uint32_t*, uint32_t*, const PassArgs<E>&, uint32_t, \
                                                       uint32_t, hipStream_t);

#define NTT_INSTANTIATE_FUSED(E)                                                                                  \
  template hipError_t launch_fused3<E>(int, int, int, const uint32_t*, uint32_t*, uint32_t*, const PassArgs<E>&,     \
                                       const PassArgs<E>&, const PassArgs<E>&, const FusedArgs&, hipStream_t);      \
  template hipError_t fused3_capacity<E>(int, int, int, int, uint32_t*, uint32_t);

#define NTT_INSTANTIATE_FUSED2(E)                                                                                 \
  template hipError_t launch_fused2<E>(int, int, const uint32_t*, uint32_t*, uint32_t*, const PassArgs<E>&,           \
                                       const PassArgs<E>&, const FusedArgs&, hipStream_t);                          \
  template hipError_t fused2_capacity<E>(int, int, int, uint32_t*, uint32_t);

#define NTT_INSTANTIATE(E)                                                                                         \
  NTT_EXTERN_KIND(E, KIND_COLUMN)                                                                                  \
  NTT_EXTERN_KIND(E, KIND_FINAL)                                                                                   \
  NTT_EXTERN_KIND(E, KIND_SINGLE)                                                                                  \
  NTT_EXTERN_KIND(E, KIND_STOCKHAM)                                                                                \
  NTT_EXTERN_KIND(E, KIND_DIT)                                                                                     \
  template hipError_t launch_pass<E>(int, int, const uint32_t*, uint32_t*, const PassArgs<E>&, uint32_t, uint32_t, \
                                     hipStream_t);                                                                 \
  template hipError_t launch_naive<E>(const uint32_t*, uint32_t*, const PassArgs<E>&, uint32_t, hipStream_t);       \
  template hipError_t launch_fill<E>(int, uint32_t*, size_t, uint64_t, uint32_t, uint32_t, uint64_t, uint32_t,     \
                                     uint32_t, hipStream_t);                                                       \
  template hipError_t launch_twiddle_pack<E>(const uint32_t*, uint32_t*, uint32_t, uint32_t, uint32_t, uint64_t,   \
                                             uint32_t, const uint32_t*, const uint32_t*, uint32_t,                 \
                                             const typename E::Args&, uint64_t, hipStream_t);                      \
  template hipError_t launch_transpose<E>(const uint32_t*, uint32_t*, uint32_t, uint32_t, uint32_t, uint64_t,     \
                                          hipStream_t);                                                            \
  template hipError_t launch_digitrev_swap<E>(uint32_t*, const DrevArgs&, uint32_t, hipStream_t);                  \
  template hipError_t launch_final_ipn<E>(int, uint32_t*, const PassArgs<E>&, uint32_t, hipStream_t);              \
  template uint32_t launch_final_ipn_capacity<E>(int, int);                                                        \
  template hipError_t launch_pointwise<E>(const uint32_t*, const uint32_t*, uint32_t*, size_t,                     \
                                          const typename E::Args&, const uint32_t*, hipStream_t, const FsMap*);    \
  template hipError_t launch_build_tw<E>(uint32_t*, size_t, uint32_t, uint32_t, uint32_t, const uint32_t*,        \
                                         const uint32_t*, uint32_t, const typename E::Args&, hipStream_t,          \
                                         const uint32_t*, const uint32_t*);                                        \
  template hipError_t launch_bitrev<E>(const uint32_t*, uint32_t*, uint32_t, const uint32_t*, uint32_t,           \
                                       hipStream_t);                                                              \
  template hipError_t launch_build_tw_sh<E>(uint32_t*, size_t, uint32_t, uint32_t, uint32_t, const uint32_t*,     \
                                            const uint32_t*, uint32_t, const typename E::Args&, const uint32_t*,  \
                                            hipStream_t);                                                         \
  template hipError_t launch_build_fs_tw<E>(uint32_t*, uint32_t, uint32_t, uint64_t, uint64_t, uint32_t,           \
                                            const uint32_t*, const uint32_t*, uint32_t, const typename E::Args&,    \
                                            hipStream_t, const uint32_t*);                                                           \
  template hipError_t launch_scale_pow<E>(uint32_t*, uint32_t, uint32_t, const uint32_t*, const uint32_t*, uint32_t, \
                                          const typename E::Args&, hipStream_t);                                   \
  template hipError_t launch_count_noncanonical<E>(const uint32_t*, size_t, const ModWords<E::MEMW>&,              \
                                                   unsigned long long*, hipStream_t);                              \
  template hipError_t launch_build_pow<E>(uint32_t*, size_t, const uint32_t*, const uint32_t*, uint32_t,           \
                                          const typename E::Args&, hipStream_t);                                   \
  template hipError_t launch_naive_round<E>(const uint32_t*, uint32_t*, uint32_t, uint32_t, const uint32_t*,       \
                                            const typename E::Args&, hipStream_t);                                 \
  template hipError_t launch_noswap_round<E>(const uint32_t*, uint32_t*, uint32_t, uint32_t, const uint32_t*,      \
                                             const typename E::Args&, hipStream_t);                                 \
  template hipError_t launch_bealto<E>(int, const uint32_t*, uint32_t*, const PassArgs<E>&, const BealtoArgs&,     \
                                       hipStream_t);

}  // namespace ntt
