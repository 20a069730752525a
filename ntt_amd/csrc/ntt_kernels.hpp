// Kernel-facing argument structs and launcher declarations (host + device).
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "engines.hpp"

namespace ntt {

// KIND_STOCKHAM: the rival schedule of the reference's bellperson / improved_NTT_v1..v4 family
// (GZKP-NTT.cu:324-386, 556-1296): Stockham autosort passes, input-side twiddles, no final
// permutation (ntt_plan_create_ex flag NTT_PLAN_STOCKHAM).
// KIND_DIT: the GZKP(B, G) rival (GZKP-NTT.cu:115-165): in-place DIT column passes with input-side
// twiddles w_N^(c d) over bit-reversed data (ntt_plan_create_ex flag NTT_PLAN_GZKP).
// KIND_ROWS: a batch of short single-tile transforms (below one wave each: n <= 2^7 on the 256-bit
// engines, 2^6 on P), TILE / n of them per workgroup (the final pass's block layout), instead of one
// per workgroup (KIND_SINGLE): batched short transforms and the four-step's row transforms
// (ntt_rplan) of such n.  At n = 2^8 / 2^9 on the 256-bit engines one transform per one- / two-wave
// workgroup is as fast or faster.
enum : int { KIND_COLUMN = 0, KIND_FINAL = 1, KIND_SINGLE = 2, KIND_STOCKHAM = 3, KIND_DIT = 4, KIND_ROWS = 5 };
// engines with KIND_STOCKHAM instances (ntt_e256_stk.hip, ntt_ep_stk.hip)
template <class E>
struct HasStockham {
  static constexpr bool value = false;
};
// engines with KIND_ROWS instances (ntt_e256_rows.hip, ntt_e256w_rows.hip, ntt_ep_rows.hip) and the radices they cover
template <class E>
struct HasRows {
  static constexpr bool value = false;
};
constexpr int kRowsMinLog = 3;
// the largest KIND_ROWS radix of an engine, measured (profiles/r05_rows/): 2^7 on the
// 256-bit engines (1024-element tiles, 256-thread workgroups); 2^6 on P, whose 8192-element tiles
// make 1024-thread workgroups that lose to one transform per workgroup from 2^7 up (+20 %, 2^8 +180 %)
template <class E>
constexpr int rows_max_log() {
  return E::W == 1 ? 6 : 7;
}

// Elements per workgroup tile of the multi-pass kernels (engines.hpp: E::TILE_LOG, E::EPT per thread).
template <class E>
__host__ __device__ constexpr int tile_log_of() { return E::TILE_LOG; }

using Eng256 = Eng29<9, 8>;    // 4 x 64-bit limbs in HBM
using Eng384 = Eng29<14, 12>;  // 6 x 64-bit limbs in HBM, moduli up to 2^383
using Eng256w = Eng29<9, 12>;  // 6 x 64-bit limbs in HBM, moduli < 2^255 (256-bit arithmetic)
using Eng256wI = Eng29<9, 12, 12>;  // the same with 48-B intermediates: NTT_PLAN_IN_PLACE plans (C3 in place)
using Eng256T = Eng29<9, 8, 0, 12>;  // 4 x 64-bit limbs, 4096-element tiles: single 2^20 transforms (C2)
using EngP = Eng32<1, 2>;      // P469762049, `long long` in HBM
using EngPI = Eng32<1, 2, 2>;  // the same with 8-B scratch elements: NTT_PLAN_IN_PLACE plans of P
template <class E>
struct IsEng32 : std::false_type {};
template <int N, int M, int S>
struct IsEng32<Eng32<N, M, S>> : std::true_type {};
template <>
struct HasStockham<Eng256> {
  static constexpr bool value = true;
};
template <>
struct HasStockham<EngP> {
  static constexpr bool value = true;
};
template <>
struct HasRows<Eng256> {
  static constexpr bool value = true;
};
template <>
struct HasRows<Eng256w> {  // the 6 x 64-bit layout of 256-bit moduli (BLS12-381 C3), ntt_e256w_rows.hip
  static constexpr bool value = true;
};
template <>
struct HasRows<EngP> {  // P469762049 (the reference's own field), ntt_ep_rows.hip
  static constexpr bool value = true;
};

// a modulus as W little-endian 32-bit words (canonical-range checks)
template <int W>
struct ModWords {
  uint32_t w[W];
};
template <class E>
hipError_t launch_count_noncanonical(const uint32_t* d, size_t n, const ModWords<E::MEMW>& p,
                                     unsigned long long* bad, hipStream_t st);

// Four-step position map (PassArgs::min / mout / mepi): p -> (p >> lc) ps + ((p mod 2^lc) >> lc2) ps2
// + (b << lc2) + (p mod 2^lc2); lc2 = lc (and ps2 = 0) is the one-level map of round 2.
struct FsMap {
  uint32_t lc, lc2;
  uint64_t ps, ps2;
  __host__ __device__ size_t operator()(size_t p, size_t b) const {
    const size_t m = ((size_t)1 << lc) - 1, m2 = ((size_t)1 << lc2) - 1;
    return (p >> lc) * ps + ((p & m) >> lc2) * ps2 + (b << lc2) + (p & m2);
  }
};

// Every inter-workgroup wait (k_final_ipn, k_fused3, k_fused3b, k_fused3bi) is bounded.  A wait that
// reaches `spins` polls gives up: it raises the launch's own abort word (which the launch's other
// waits check every 256 polls, so they give up too and every wave reaches the exit), the workgroup
// skips its remaining stores, and the plan's
// host-mapped report word `report` is set (system scope).  The next call on the plan returns
// NTT_ERR_DEVICE without any device query (ntt_plan_device_status reads and clears the report).
// spins = 0 gives up at once (ntt_plan_set_watchdog: a test hook).
struct Watchdog {
  uint32_t* report;  // host-mapped word of the plan (null: none)
  uint32_t* abort;   // the launch's abort word, on a 128-B line of its own (pollers of a line that also
                     // holds a counter queue the counter's atomic adds: DESIGN §4); zeroed by the last
                     // workgroup out
  uint32_t spins;    // poll limit, ~1 us per poll after the first few (default 2^21, ~2 s)
};

template <class E>
struct PassArgs {
  typename E::Args F;
  const uint32_t* tw_int;  // w_R^e, e < R (this pass's radix), engine table format
  const uint32_t* tw_lo;   // outer twiddles w_n^e = tw_lo[e mod 2^lo_bits] * tw_hi[e >> lo_bits]
  const uint32_t* tw_hi;
  const uint32_t* tw_full;  // column pass: per-pass outer twiddle table (HBM element format) or null
  const uint32_t* src2;     // first column pass of a fused polymul inverse: x <- mont(src, src2) at load
  const uint32_t* tw_in;    // first column pass of a fused coset forward: x_d <- x_d u^d (Shoup table, d < R)
  uint32_t lo_bits;
  uint32_t log_n;
  uint32_t log_blk;  // column pass: log2 of the block length N_i
  uint32_t log_m;    // column pass: log2(n / N_i)
  uint32_t r1;       // final pass: log2 R_1
  uint32_t nmid;     // final pass: number of middle digits (p - 2)
  uint32_t mid_bits[4];  // final pass: middle digit widths, least significant (k_{p-1}) first
  uint32_t mid_off[4];   // final pass: output bit offset (relative to R_1) of those digits
  uint32_t flags;        // bit 0: multiply outputs by ninv (single-pass inverse); bit 1: final pass
                         // writes each output to its input's position (NTT_PLAN_IN_PLACE); bit 2:
                         // XCD-grouped tile order (tiles t and t + 1 on one XCD, k_pass)
  uint32_t src_user;     // column pass: src is the caller's buffer (E::MEMW words/element), not scratch (E::SCRW)
  size_t batch_stride;   // 32-bit words between batched transforms in the caller's buffers (n * E::MEMW)
  // ---- distributed four-step addressing (ntt_rplan_*); fs == 0: plain batched transforms.
  // Mode B (fs & FS_IL == 0): transform b (= blockIdx.y) of a batch, position p (the row transforms:
  //   packed output of the forward, exchanged input of the inverse).
  // Mode I (fs & FS_IL): 2^il transforms interleaved, element j of transform b at P = j 2^il + b (the
  //   [n1][c] column layout and the exchanged blocks); every pass groups T adjacent transforms, so
  //   runs stay contiguous.  b = 0 in the maps below (P carries it).
  // A map (FsMap) sends p to (p >> lc) ps + ((p mod 2^lc) >> lc2) ps2 + (b << lc2) + (p mod 2^lc2):
  //   peer blocks of ps elements, within them column pieces of ps2 elements (lc2 = lc: no pieces).
  //   min: the first pass's input (FS_MAP_IN, src and src2), mout: the last pass's output
  //   (FS_MAP_OUT), mepi: the Mode I epilogue-table index (FS_MAP_EPI).
  uint32_t lgp;          // KIND_STOCKHAM: log2 of the number of groups p already combined (bellperson `lgp`)
  uint32_t fs;           // FS_* bits
  uint32_t il;           // Mode I: log2 of the interleave
  FsMap min, mout, mepi;
  const uint32_t* tw_epi;  // final pass: multiply output k of transform b by this table's entry (w R_e,
                           // E::SCRW words; index b N + k in Mode B, k 2^il + b in Mode I) or null
  uint32_t tw_sh;          // column pass: tw_full holds Shoup pairs (canonical w, floor(w B / p); E::TW words
                           // per entry, E::SHOUP_OUTER engines) instead of w R_e in the element format
  // ---- in-place final pass with the digit reversal fused (k_final_ipn, NTT_PLAN_IN_PLACE):
  uint32_t* ipn_sync;        // [0] tile ticket, [1] workgroups exited; slab m: reads done at [32 (1 + m)],
                             // ready at [32 (1 + m) + 1] (one 128-B line per slab)
  const uint32_t* ipn_order; // slab (middle-digit value) of the i-th slab in ticket order (pairs adjacent)
  uint32_t ipn_strips;       // workgroups per slab (R_1 / T)
  uint32_t* ipn_go;          // k_fused3bi (the in-place single launch): the final pass's barrier go word
  uint32_t* ipn_shards;      //   and its arrival shard lines (ipn_sync: the top counter)
  Watchdog wd;               // bounded waits (k_final_ipn, k_fused3bi)
  // debug builds (NTT_DEBUG_CHECKS): element extents of src / dst from this transform's first element
  // (~0: not checked, e.g. four-step maps into the caller's exchange blocks)
  size_t dbg_src_n, dbg_dst_n;
};
enum : uint32_t { FS_MAP_IN = 1u, FS_MAP_OUT = 2u, FS_IL = 4u, FS_MAP_EPI = 8u };

// Fused single-launch schedule of a 3-pass transform (k_fused3, BASELINE config 2's "single-kernel"):
// one persistent launch runs pass 1's, pass 2's and the final pass's tiles, handed between
// workgroups through counters instead of kernel boundaries.  Word layout of `sync` (zero before the
// first launch; the last workgroup to leave re-zeroes it): [0] tile ticket, [1] workgroups exited,
// [2], [3] spare, [4, 4 + n12) pass 1 -> 2 counters,
// [4 + n12, 4 + n12 + n23) pass 2 -> final counters, then one ready word per counter (rbase).
struct FusedArgs {
  uint32_t* sync;
  uint32_t tiles;      // tiles per pass (n / TILE)
  uint32_t nwg;        // workgroups launched
  uint32_t k1_mask, k1_shift;  // pass-1 tile w: counter (w & k1_mask) >> k1_shift
  uint32_t cg_log;             // pass-2 tile w: column group w mod 2^cg_log, block k1 = w >> cg_log
  uint32_t k2_shift;           //   waits on counter (w mod 2^cg_log) >> k2_shift
  uint32_t t3_log;             //   signals counter n12 + (k1 >> t3_log)
  uint32_t r2;                 // final tile w: waits on counter n12 + (w >> r2)
  uint32_t n12, n23;
  uint32_t need12, need23;     // arrivals per counter
  uint32_t rbase;              // ready word of counter i at sync[rbase + 32 i] (one 128-B line each)
  uint32_t dbg;                // diagnostics only (NTT_FUSED_DBG): bit 0 no dependency waits (wrong
                               // output), bit 2 static tile order (needs every workgroup resident)
  uint32_t mode;               // 0: dataflow hand-offs between tiles (k_fused3); 1: two grid barriers
                               // (k_fused3b); 2: the NTT_PLAN_IN_PLACE form, residency + three grid
                               // barriers, one workgroup per tile (k_fused3bi); 3: two passes on
                               // 4096-element tiles, one barrier (k_fused2b); 4: the same in place,
                               // residency + two barriers (k_fused2bi)
  Watchdog wd;                 // bounded waits
  uint32_t* shards;            // grid barriers (modes 1..4): 8 arrival shards, one 128-B line each
  unsigned long long* trace;   // diagnostics (NTT_FUSED_TRACE, modes 3 and 4): 4 timestamps per workgroup
};
template <class E>
hipError_t launch_fused3(int r1, int r2, int r3, const uint32_t* src, uint32_t* scratch, uint32_t* dst,
                         const PassArgs<E>& A1, const PassArgs<E>& A2, const PassArgs<E>& A3, const FusedArgs& F,
                         hipStream_t st);
// workgroups one launch of k_fused3<E, r1, r2, r3> (mode 0) or k_fused3b (mode 1) keeps resident on
// `device` (occupancy query x CUs)
template <class E>
hipError_t fused3_capacity(int r1, int r2, int r3, int device, uint32_t* wgs, uint32_t mode = 0);

// The two-pass single launch on 4096-element tiles (k_fused2b, FusedArgs::mode 3; in place:
// k_fused2bi, mode 4): 2^20 = 10 + 10 on Eng256T with one grid barrier, a plain launch
// the engines k_fused2b / k_fused2bi are instantiated for (radices 10 + 10: 2^20 on 4096-element tiles)
template <class E>
__host__ __device__ constexpr bool fused2_engine() {
  return E::FASTRED && !E::LDS_TW && E::TILE_LOG == 12 && E::EPT == 4 && E::W == 9 && E::MEMW == 8;
}
template <class E>
hipError_t launch_fused2(int r1, int r2, const uint32_t* src, uint32_t* scratch, uint32_t* dst, const PassArgs<E>& A1,
                         const PassArgs<E>& A2, const FusedArgs& F, hipStream_t st);
template <class E>
hipError_t fused2_capacity(int r1, int r2, int device, uint32_t* wgs, uint32_t mode);

// The in-place final pass with the digit reversal fused (NTT_PLAN_IN_PLACE, batch 1): A.ipn_* set,
// grid = n / TILE workgroups, src == dst.  See k_final_ipn.
template <class E>
hipError_t launch_final_ipn(int logr, uint32_t* data, const PassArgs<E>& A, uint32_t grid, hipStream_t st);
// workgroups of k_final_ipn<E, logr> resident at once on `device` (0: unknown)
template <class E>
uint32_t launch_final_ipn_capacity(int logr, int device);

template <class E, int KIND>
hipError_t launch_pass_kind(int logr, const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, uint32_t grid,
                            uint32_t batch, hipStream_t st);
template <class E>
hipError_t launch_pass(int kind, int logr, const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, uint32_t grid,
                       uint32_t batch, hipStream_t st);
template <class E>
hipError_t launch_build_tw(uint32_t* out, size_t count, uint32_t log_r, uint32_t log_t, uint32_t log_m,
                           const uint32_t* lo, const uint32_t* hi, uint32_t lo_bits, const typename E::Args& F,
                           hipStream_t st, const uint32_t* clo = nullptr, const uint32_t* chi = nullptr);
// The same table as Shoup pairs (w, floor(w B / p)) in the engine's twiddle format (E::TW words per
// entry); pinvB = p^-1 mod B (E::W limbs, device memory).  E::SHOUP_OUTER engines only.
template <class E>
hipError_t launch_build_tw_sh(uint32_t* out, size_t count, uint32_t log_r, uint32_t log_t, uint32_t log_m,
                              const uint32_t* lo, const uint32_t* hi, uint32_t lo_bits, const typename E::Args& F,
                              const uint32_t* pinvB, hipStream_t st);
// NTT_PLAN_NAIVE: the power table w_n^i R_e (i < count, E::TABW words per entry) and one radix-2
// DIT round (stride 2^log_s) of the reference's `naive` rival over a bit-reversed vector
template <class E>
hipError_t launch_build_pow(uint32_t* out, size_t count, const uint32_t* lo, const uint32_t* hi, uint32_t lo_bits,
                            const typename E::Args& F, hipStream_t st);
// NTT_PLAN_NO_SWAP: one radix-2 Stockham round (stride 2^log_s) of the reference's `naive_no_swap`
template <class E>
hipError_t launch_noswap_round(const uint32_t* src, uint32_t* dst, uint32_t log_n, uint32_t log_s, const uint32_t* pw,
                               const typename E::Args& F, hipStream_t st);
// The reference's bealto.com radix-2^deg Stockham family (ntt.h NTT_PLAN_BELLPERSON,
// NTT_PLAN_IMPROVED_V1..V4): one round of 2^deg-point groups, 2^log_g groups per workgroup
// (A: tw_lo / tw_hi / lo_bits two-level tables for the input twiddles, tw_int the pq table of
// w_{2^max_deg}^j Shoup pairs, j < 2^(max_deg - 1)).  Engines with HasStockham only.
enum : int { BEALTO_BELLPERSON = 0, BEALTO_V1 = 1, BEALTO_V2 = 2, BEALTO_V3 = 3, BEALTO_V4 = 4 };
struct BealtoArgs {
  uint32_t log_n, lgp, deg, log_g, max_deg;
};
template <class E>
hipError_t launch_bealto(int variant, const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, const BealtoArgs& B,
                         hipStream_t st);
template <class E>
hipError_t launch_naive_round(const uint32_t* src, uint32_t* dst, uint32_t log_n, uint32_t log_s, const uint32_t* pw,
                              const typename E::Args& F, hipStream_t st);
// dst[i] = src[digit reversal of i] over 2^log_n elements of E::MEMW words, digits of digits[q] bits
// in pass order (the GZKP rival's `rearrange`); nd = 0: the bit reversal (the naive rival's)
template <class E>
hipError_t launch_bitrev(const uint32_t* src, uint32_t* dst, uint32_t log_n, const uint32_t* digits, uint32_t nd,
                         hipStream_t st);
// scale (E::TW words, a twiddle) or null: every entry is also multiplied by it
template <class E>
hipError_t launch_build_fs_tw(uint32_t* out, uint32_t log_rows, uint32_t log_cols, uint64_t row0, uint64_t col0,
                              uint32_t log_n, const uint32_t* lo, const uint32_t* hi, uint32_t lo_bits,
                              const typename E::Args& F, hipStream_t st, const uint32_t* scale = nullptr);
template <class E>
hipError_t launch_naive(const uint32_t* src, uint32_t* dst, const PassArgs<E>& A, uint32_t batch, hipStream_t st);
// Fill local element i with the synthetic value of global index
// j = row0 + (i >> log_inner) + ((i mod 2^log_inner) << log_stride)   (log_inner = 64: j = i).
template <class E>
hipError_t launch_fill(int kind, uint32_t* dst, size_t n, uint64_t seed, uint32_t nrand, uint32_t top_bits,
                       uint64_t row0, uint32_t log_inner, uint32_t log_stride, hipStream_t st);
template <class E>
hipError_t launch_twiddle_pack(const uint32_t* src, uint32_t* dst, uint32_t log_rows, uint32_t log_len,
                               uint32_t log_bw, uint64_t row0, uint32_t log_n, const uint32_t* lo, const uint32_t* hi,
                               uint32_t lo_bits, const typename E::Args& F, uint64_t peer_stride, hipStream_t st);
template <class E>
hipError_t launch_transpose(const uint32_t* src, uint32_t* dst, uint32_t log_rows, uint32_t log_cols,
                            uint32_t log_blk_rows, uint64_t blk_stride, hipStream_t st);
// In-place digit reversal of a palindromic schedule (NTT_PLAN_IN_PLACE): position
// (k1, mid, kn) = k1 2^(log_n - R) + mid 2^R + kn  <->  (kn, midrev, k1), tiles of 2^tb_log x 2^tb_log.
struct DrevArgs {
  uint32_t log_n, R, tb_log, nmid;
  uint32_t diag;         // workgroup -> tile-pair order: 1 diagonal, 0 row-major
  uint32_t mid_bits[4];  // middle digit widths of `mid`, least significant first (PassArgs::mid_bits)
  uint32_t mid_off[4];   // their bit offsets in midrev (PassArgs::mid_off)
  size_t batch_stride;   // 32-bit words between batched transforms
  uint64_t unit0;        // first tile pair of this launch (launch_digitrev_swap chunks the grid)
};
template <class E>
hipError_t launch_digitrev_swap(uint32_t* data, const DrevArgs& A, uint32_t batch, hipStream_t st);
// data[j] *= c^j (coset / low-degree-extension scale), c^j = lo_s[j & mask] * hi[j >> lo_bits]
template <class E>
hipError_t launch_scale_pow(uint32_t* data, uint32_t log_n, uint32_t batch, const uint32_t* lo_s, const uint32_t* hi,
                            uint32_t lo_bits, const typename E::Args& F, hipStream_t st);
// c = a * b (canonical in/out): mont(mont(a, b), R^2) with r2 in the engine table format; in_map:
// element j of a and b is read at (*in_map)(j, 0) (a four-step piece of the column layout)
template <class E>
hipError_t launch_pointwise(const uint32_t* a, const uint32_t* b, uint32_t* c, size_t n, const typename E::Args& F,
                            const uint32_t* d_r2, hipStream_t st, const FsMap* in_map = nullptr);

}  // namespace ntt
