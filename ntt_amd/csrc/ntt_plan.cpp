// Host side of libntt.so: plans (twiddle tables + scratch cached per device), pass scheduling, the
// C ABI of include/ntt.h and the reference-shaped shims (SSIP, NTT_GZKP_256, NTT_GZKP_64).
//
// Reference behaviour mirrored (file:line in tie-pilot-qxw/NTT):
//   * w_n = g^((p-1)/n) from the generator argument        GZKP-NTT.cu:1462, big-num.cu:292-296
//   * forward = natural -> natural, in place               SSIP GZKP-NTT.cu:1452-1558
//   * inverse = forward with g^-1, then * n^-1             GZKP-NTT.cu:1725-1732
//   * modulus-generic 256-bit path (prime argument)        big-num.cu:68,173,260
// Differences: tables are built once per plan (the reference rebuilt pq/omegas on every call and
// freed them with a new[]/free mismatch, GZKP-NTT.cu:1554-1555); errors are returned as status
// codes instead of asserts; nothing is printed.
#include <algorithm>
#include <hip/hip_runtime.h>

#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "../../include/ntt.h"
#include "ntt_internal.hpp"
#include "ntt_kernels.hpp"

using namespace ntt;

namespace {

thread_local int g_last_error = NTT_OK;

// the bealto-family rival schedules (ntt.h): one k_bealto variant each
constexpr unsigned kBealtoFlags = NTT_PLAN_BELLPERSON | NTT_PLAN_IMPROVED_V1 | NTT_PLAN_IMPROVED_V2 |
                                  NTT_PLAN_IMPROVED_V3 | NTT_PLAN_IMPROVED_V4;

// ------------------------------------------------------------------------------ single-launch order
// The single launches (k_fused3 / k_fused3b / k_fused3bi / k_fused2b / k_fused2bi) wait across
// workgroups, so each assumes its workgroups own the device: two of them enqueued on two streams could
// have their workgroups dispatched interleaved, each holding part of the CUs, and both would wait for
// the other's workgroups until the watchdog gave up (NTT_ERR_DEVICE).  The library therefore orders
// them per device, under one lock: a single launch on another stream than the device's previous one
// first makes its stream wait for everything enqueued so far on that previous stream (an event
// recorded there at this moment), which includes the previous single launch.  Launches on one stream
// are in order already and pay nothing: an event recorded after every launch cost 4.5 us of device time
// per call (a marker packet behind the kernel; profiles/r06_c2/).  A previous stream that has been
// destroyed (hipStreamGetFlags fails) has finished its work.  Work of other kinds is not ordered.
// (The in-place forms also check residency before their first store, for CUs held by anything else:
// ntt_kernels_impl.hpp residency_wait.)
class FusedSerial {
 public:
  FusedSerial(int device, hipStream_t st) : lk_(mu()), s_(enabled() ? slot(device) : nullptr), st_(st) {
    if (!s_ || !s_->used || s_->last == st) return;
    unsigned fl = 0;
    if (hipStreamGetFlags(s_->last, &fl) != hipSuccess) {  // gone: its work is done
      (void)hipGetLastError();
      return;
    }
    if (!s_->ev && hipEventCreateWithFlags(&s_->ev, hipEventDisableTiming) != hipSuccess) {
      s_->ev = nullptr;
      (void)hipGetLastError();
      return;
    }
    if (hipEventRecord(s_->ev, s_->last) == hipSuccess) (void)hipStreamWaitEvent(st, s_->ev, 0);
  }
  void done(hipError_t launched) {
    if (!s_ || launched != hipSuccess) return;
    s_->last = st_;
    s_->used = true;
  }

 private:
  struct Slot {
    hipStream_t last = nullptr;  // the stream of the device's latest single launch
    bool used = false;
    hipEvent_t ev = nullptr;     // process-lifetime, like the plan cache
  };
  static bool enabled() {  // NTT_FUSED_ORDER=0: no ordering (A/B only)
    static const bool on = [] {
      const char* v = getenv("NTT_FUSED_ORDER");
      return !(v && *v == '0');
    }();
    return on;
  }
  static std::mutex& mu() {
    static std::mutex* m = new std::mutex;
    return *m;
  }
  static Slot* slot(int device) {
    static Slot* slots = new Slot[64];
    return (device >= 0 && device < 64) ? &slots[device] : nullptr;
  }
  std::lock_guard<std::mutex> lk_;
  Slot* s_;
  hipStream_t st_;
};

// Diagnostics (NTT_FUSED_TRACE=<file>): the two-pass single launch writes per-workgroup wall-clock
// stamps (start, after pass 1, after the barrier, end; 100 MHz), appended to <file> after each call,
// which then synchronises its stream.  Never on in measured runs.
static const char* fused_trace_path() {
  static const char* p = getenv("NTT_FUSED_TRACE");
  return (p && *p) ? p : nullptr;
}

// ------------------------------------------------------------------------------ host field math
template <int N>
using Vec = std::array<uint32_t, N>;

template <int N>
struct HostField {
  Modulus<N> M;
  Vec<N> r1{}, r2{};  // R mod p, R^2 mod p

  Vec<N> mul(const Vec<N>& a, const Vec<N>& b) const {
    Vec<N> r;
    mont_mul_cios<N>(r.data(), a.data(), b.data(), M);
    return r;
  }
  Vec<N> add(const Vec<N>& a, const Vec<N>& b) const {
    Vec<N> r;
    add_mod<N>(r.data(), a.data(), b.data(), M);
    return r;
  }
  Vec<N> to_mont(const Vec<N>& a) const { return mul(a, r2); }
  Vec<N> from_mont(const Vec<N>& a) const {
    Vec<N> one{};
    one[0] = 1;
    return mul(a, one);
  }
  // base (Montgomery) ^ e, e given as 32-bit little-endian words
  Vec<N> pow(const Vec<N>& base, const std::vector<uint32_t>& e) const {
    Vec<N> acc = r1, b = base;
    for (size_t i = 0; i < e.size() * 32; ++i) {
      if ((e[i / 32] >> (i % 32)) & 1) acc = mul(acc, b);
      b = mul(b, b);
    }
    return acc;
  }
  Vec<N> pow_u64(const Vec<N>& base, uint64_t e) const {
    return pow(base, std::vector<uint32_t>{(uint32_t)e, (uint32_t)(e >> 32)});
  }
};

template <int N>
static bool vec_lt(const Vec<N>& a, const Vec<N>& b) {
  for (int i = N - 1; i >= 0; --i)
    if (a[i] != b[i]) return a[i] < b[i];
  return false;
}

// ------------------------------------------------------------------------------ watchdog words
// One 4-KiB mapped, coherent pinned page per 1024 plans that use inter-workgroup waits; a plan takes
// a 4-byte slot when it first builds such a schedule and returns it when destroyed.  The pages are
// never freed: nothing is released during process teardown, where the HIP runtime (and a profiler
// such as rocprofv3) may already be gone.
static std::mutex g_watch_mu;
static std::vector<uint32_t*> g_watch_free;
static uint32_t* watch_slot_acquire() {
  std::lock_guard<std::mutex> lk(g_watch_mu);
  if (g_watch_free.empty()) {
    void* page = nullptr;
    if (hipHostMalloc(&page, 4096, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess)
      return nullptr;
    auto* w = static_cast<uint32_t*>(page);
    for (int i = 1023; i >= 0; --i) {
      w[i] = 0u;
      g_watch_free.push_back(w + i);
    }
  }
  uint32_t* s = g_watch_free.back();
  g_watch_free.pop_back();
  *s = 0u;
  return s;
}
static void watch_slot_release(uint32_t* s) {
  if (!s) return;
  std::lock_guard<std::mutex> lk(g_watch_mu);
  g_watch_free.push_back(s);
}

// ------------------------------------------------------------------------------ plan
struct PlanBase {
  virtual ~PlanBase() = default;
  virtual int run(void* d, unsigned batch, bool inverse, hipStream_t st) = 0;
  virtual int pointwise(const void* a, const void* b, void* c, hipStream_t st) = 0;
  virtual int polymul(void* a, void* b, void* c, hipStream_t st) = 0;
  virtual int fill(void* d, uint64_t count, int kind, uint64_t seed, uint64_t row0, unsigned log_inner,
                   unsigned log_stride, hipStream_t st) = 0;
  virtual int twiddle_pack(const void* src, void* dst, unsigned log_rows, unsigned log_len, unsigned log_bw,
                           uint64_t row0, bool inverse, uint64_t peer_stride, hipStream_t st) = 0;
  virtual int transpose(const void* src, void* dst, unsigned log_rows, unsigned log_cols, unsigned log_blk_rows,
                        uint64_t blk_stride, hipStream_t st) = 0;
  virtual int inverse_pointwise(const void* a, const void* b, void* c, unsigned batch, hipStream_t st) = 0;
  virtual int run_fs(const void* in, const void* in2, void* out, unsigned batch, bool inverse, const ntt::FsIO& io,
                     hipStream_t st) = 0;
  virtual int build_fs_table(void* table, unsigned log_rows, unsigned log_cols, uint64_t row0, uint64_t col0,
                             bool inverse, unsigned scale_log, hipStream_t st) = 0;
  virtual size_t table_entry_bytes() const = 0;
  // pass kernels a transform of 2^log_x points takes with this plan's engine (its schedule()), and
  // the largest radix (log2) among them
  virtual unsigned passes_for(unsigned log_x) const = 0;
  virtual unsigned max_radix_for(unsigned log_x) const = 0;
  virtual int coset(void* d, const uint64_t* shift, unsigned limbs64, bool inverse, hipStream_t st) = 0;
  virtual int count_noncanonical(const void* d, uint64_t count, uint64_t* bad, hipStream_t st) = 0;
  virtual int device_status(unsigned* bad) = 0;
  // the plan's batch-1 forward / inverse run as ONE launch (NTT_PLAN_SINGLE_LAUNCH): its single-launch
  // state is built now (a second plan of 4096-element tiles is kept only when this holds)
  virtual bool single_launch_ready() { return false; }
  uint64_t n = 0;
  unsigned flags = 0;
  unsigned log_n = 0, elem_bytes = 0, npass = 0;
  unsigned r[8] = {0};
  int device = 0;
  // optional per-launch timing: events recorded on the caller's stream between launches, one
  // slot per transform in a ring of kSlots transforms (no host synchronisation per transform).
  // Each interval between two events carries a label naming the launch it timed (kind letter +
  // log2 radix, "s" for a Shoup-pair outer table: c8, c8s, f8, r8, s12, i8, d, b; tools/pmc_to_traffic.py
  // derives the same labels from the rocprofv3 kernel names), "" when unlabelled.
  // Grouping (ntt_plan_profile_group, the rank plan's four-step transforms): once a plan has been put
  // in group mode, a transform continues the current slot until the next group call, so the slot holds
  // every launch of one caller-level operation (e.g. a row transform run as two launches of 2^15 rows);
  // the time between two transforms of a group is an interval labelled "-" and is not a launch.
  static constexpr unsigned kSlots = 64, kEv = 17;
  bool profiling = false;
  hipEvent_t ev[kSlots][kEv] = {};
  char lab[kSlots][kEv][6] = {};  // label of the interval that ends at event k
  unsigned ev_used = 0, slot = 0, nrec = 0;
  bool grouped = false, group_new = false;
  // Watchdog report (ntt_kernels.hpp): a host-mapped word that a kernel sets when one of its bounded
  // inter-workgroup waits gives up.  Every later call on the plan returns NTT_ERR_DEVICE (a plain host
  // read, no device query) until ntt_plan_device_status reads and clears it.
  // The word is a slot of a process-wide pinned page (watch_slot_acquire below), taken when the plan
  // first builds a schedule with such waits; plans that never do hold none.
  uint32_t* h_watch = nullptr;  // host pointer (a slot of the mapped, coherent page)
  uint32_t* d_watch = nullptr;  // its device alias (the kernels' Watchdog::report)
  uint32_t wd_spins = 1u << 21; // poll limit of a wait (~2 s); ntt_plan_set_watchdog
  bool tripped() const { return h_watch && __atomic_load_n(h_watch, __ATOMIC_ACQUIRE) != 0u; }
  void clear_trip() {
    if (h_watch) __atomic_store_n(h_watch, 0u, __ATOMIC_RELEASE);
  }
  ntt::Watchdog watchdog(uint32_t* abort_w) const { return ntt::Watchdog{d_watch, abort_w, wd_spins}; }
  bool alloc_watch();  // true once the plan holds a report word (defined after the slot pool)
  void begin(hipStream_t st) {
    if (!profiling) return;
    if (grouped && !group_new && nrec > 0 && ev_used > 0 && ev_used + 1 < kEv) {
      mark(st, "-");  // the same group: the time since its previous transform is a gap
      return;
    }
    group_new = false;
    slot = nrec % kSlots;
    ev_used = 0;
    ++nrec;
    mark(st);
  }
  void mark(hipStream_t st, const char* kind = "", unsigned log_radix = 0, bool shoup = false) {
    if (!profiling || ev_used >= kEv) return;
    char* l = lab[slot][ev_used];
    if (log_radix)
      snprintf(l, sizeof lab[0][0], "%s%u%s", kind, log_radix, shoup ? "s" : "");
    else
      snprintf(l, sizeof lab[0][0], "%s", kind);
    (void)hipEventRecord(ev[slot][ev_used++], st);
  }
};

bool PlanBase::alloc_watch() {
  if (h_watch) return true;
  h_watch = watch_slot_acquire();
  if (!h_watch) return false;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h_watch, 0) != hipSuccess) {
    watch_slot_release(h_watch);
    h_watch = nullptr;
    return false;
  }
  d_watch = static_cast<uint32_t*>(d);
  return true;
}

// radices for log_n: near-equal split with each radix <= tile_log - min_cols_log so that every
// global access is a contiguous run of T = TILE / R >= 2^min_cols_log elements (>= 128 B).
// The pass kernels also need every column pass's block to span a whole tile (N_i = R_i ... R_p >=
// TILE, so a workgroup's T columns lie in one block) and the final pass's T blocks to fit in R_1
// (r_1 + r_p >= tile_log).  The near-equal split violates that only for short 3-pass schedules of
// big tiles (2^19 on the 8192-element P tiles: 7+6+6); ascending order fixes every such case.
static bool schedule_ok(const unsigned* r, unsigned p, unsigned tile_log) {
  if (p < 2) return true;
  if (r[0] + r[p - 1] < tile_log) return false;
  unsigned tail = r[p - 1];
  for (int i = (int)p - 2; i >= 0; --i) {
    tail += r[i];
    if (tail < tile_log) return false;
  }
  return true;
}
// narrow_first (HBM-bound engines): pass 1, whose columns are n / R_1 elements apart, takes a radix
// one below the rest so that its workgroups read twice as wide runs (2^24 P: 7+8+9 instead of 8+8+8).
// NTT_SCHEDULE="r1,r2,..." (experiments only): that radix sequence for the sizes it sums to, when the
// pass kernels accept it.
static bool schedule_env(unsigned log_n, unsigned tile_log, unsigned rmax, unsigned* r, unsigned& p) {
  const char* v = getenv("NTT_SCHEDULE");
  if (!v || !*v) return false;
  unsigned rr[8], pp = 0, sum = 0;
  for (const char* c = v; *c && pp < 8;) {
    const unsigned x = (unsigned)strtoul(c, const_cast<char**>(&c), 10);
    if (x < 3 || x > rmax) return false;
    rr[pp++] = x;
    sum += x;
    if (*c == ',') ++c;
    else if (*c) return false;
  }
  if (sum != log_n || pp < 2 || !schedule_ok(rr, pp, tile_log)) return false;
  for (unsigned i = 0; i < pp; ++i) r[i] = rr[i];
  p = pp;
  return true;
}
static bool schedule(unsigned log_n, unsigned tile_log, unsigned min_cols_log, bool narrow_first, unsigned* r,
                     unsigned& p) {
  if (log_n <= 2) { p = 0; return true; }
  if (log_n <= tile_log) { p = 1; r[0] = log_n; return true; }
  if (schedule_env(log_n, tile_log, tile_log - min_cols_log, r, p)) return true;
  const unsigned rmax = tile_log - min_cols_log;
  p = (log_n + rmax - 1) / rmax;
  if (p < 2) p = 2;
  const unsigned base = log_n / p, rem = log_n % p;
  for (unsigned i = 0; i < p; ++i) r[i] = base + (i < rem ? 1 : 0);
  if (narrow_first) {
    std::sort(r, r + p);
    if (r[p - 1] < rmax && r[0] > 3) {
      r[0] -= 1;
      r[p - 1] += 1;
      std::sort(r + 1, r + p);
      if (!schedule_ok(r, p, tile_log)) { r[0] += 1; r[p - 1] -= 1; std::sort(r, r + p); }
    }
  }
  if (!schedule_ok(r, p, tile_log)) std::sort(r, r + p);
  return schedule_ok(r, p, tile_log);
}

// NTT_PLAN_IN_PLACE: a palindromic sequence (r_i = r_{p-1-i}, 3 <= r_i <= rmax, schedule_ok) with the
// fewest passes (>= p0), then the smallest largest radix, then the largest smallest one.  The digit
// reversal of a palindromic sequence is an involution (k_digitrev_swap).
static bool schedule_palindrome(unsigned log_n, unsigned tile_log, unsigned rmax, unsigned p0, unsigned* r,
                                unsigned& p) {
  if (rmax < 3) return false;
  const unsigned span = rmax - 2;  // radices 3..rmax
  for (unsigned pp = (p0 < 2 ? 2 : p0); pp <= 8; ++pp) {
    const unsigned h = (pp + 1) / 2;
    unsigned combos = 1;
    for (unsigned i = 0; i < h; ++i) combos *= span;
    unsigned best[8] = {0}, bmax = 99, bmin = 0;
    for (unsigned code = 0; code < combos; ++code) {
      unsigned v[8], c = code, sum = 0, mx = 0, mn = 99;
      for (unsigned i = 0; i < h; ++i) {
        v[i] = 3 + c % span;
        c /= span;
      }
      for (unsigned i = 0; i < pp; ++i) {
        v[i] = v[i < h ? i : pp - 1 - i];
        sum += v[i];
        mx = v[i] > mx ? v[i] : mx;
        mn = v[i] < mn ? v[i] : mn;
      }
      if (sum != log_n || !schedule_ok(v, pp, tile_log)) continue;
      if (mx < bmax || (mx == bmax && mn > bmin)) {
        bmax = mx;
        bmin = mn;
        for (unsigned i = 0; i < pp; ++i) best[i] = v[i];
      }
    }
    if (bmax != 99) {
      p = pp;
      for (unsigned i = 0; i < pp; ++i) r[i] = best[i];
      return true;
    }
  }
  return false;
}

// ------------------------------------------------------------------------------ engine encodings
// The host does all table arithmetic in 32-bit Montgomery form (HostField<NH>), produces canonical
// values, then encodes them in the engine's own Montgomery domain / limb layout.
template <class E>
struct EngHost;

template <int L, int W32, int S, int T>
struct EngHost<Eng29<L, W32, S, T>> {
  using E29 = Eng29<L, W32, S, T>;
  static constexpr int NH = W32;
  static constexpr int TW = E29::TW;
  using EA = typename E29::Args;
  HostField<NH> const* H = nullptr;
  Vec<NH> kR{};          // B = 2^(29L) mod p, canonical
  uint32_t pinvB[L] = {};  // p^-1 mod B
  void init(const HostField<NH>& h) {
    H = &h;
    Vec<NH> x{};
    x[0] = 1;
    for (int k = 0; k < 29 * L; ++k) x = h.add(x, x);
    kR = x;
    uint32_t pw[NH], pl[L];
    for (int i = 0; i < NH; ++i) pw[i] = h.M.p[i];
    pack29<L, NH>(pl, pw);
    inv_mod_B29<L>(pinvB, pl);
  }
  static void limbs(const Vec<NH>& c, uint32_t (&x)[L]) {
    uint32_t w[NH];
    for (int i = 0; i < NH; ++i) w[i] = c[i];
    pack29<L, NH>(x, w);
  }
  Vec<NH> times_B(const Vec<NH>& c) const { return H->mul(c, H->to_mont(kR)); }  // c B mod p
  // canonical c -> Shoup table entry (c, floor(c B / p)) as TW words
  void encode(const Vec<NH>& c, uint32_t* out) const {
    uint32_t w[L], wr[L], ws[L];
    limbs(c, w);
    limbs(times_B(c), wr);
    shoup_ws29<L>(ws, wr, pinvB);
    for (int i = 0; i < TW; ++i) out[i] = i < L ? w[i] : (i < 2 * L ? ws[i - L] : 0u);
  }
  // entry whose value is c R_e (R_e = B): the left factor of the two-level twiddle products
  void encode_scaled(const Vec<NH>& c, uint32_t* out) const { encode(times_B(c), out); }
  bool check_modulus(const uint32_t* p) const {
    // 2p fits the HBM words (p < 2^(32 W32 - 1)) and 64p <= B = 2^(29L) (lazy bounds up to 33p)
    int bits = 0;
    for (int i = NH - 1; i >= 0; --i)
      if (p[i]) { bits = 32 * i + 32 - __builtin_clz(p[i]); break; }
    return bits <= 32 * NH - 1 && bits <= 29 * L - 6;
  }
  void fill_args(EA& A, const uint32_t* p, const Vec<NH>* w8, const Vec<NH>& ninv) const {
    uint32_t pw[NH];
    for (int i = 0; i < NH; ++i) pw[i] = p[i];
    pack29<L, NH>(A.M.p, pw);
    for (int i = 0; i < L; ++i) A.kp[0][i] = A.M.p[i];
    for (int j = 1; j < 5; ++j) {  // 2^j p: double the normalised limbs and renormalise
      for (int i = 0; i < L; ++i) A.kp[j][i] = A.kp[j - 1][i] << 1;
      norm_u<L>(A.kp[j]);
    }
    for (int i = 0; i < L; ++i) A.M.p2[i] = A.kp[1][i];
    neg29<L>(A.pbar, A.M.p);
    uint32_t inv = 1;
    for (int i = 0; i < 5; ++i) inv *= 2 - p[0] * inv;
    A.M.pinv = (0u - inv) & kMask29;
    uint32_t tmp[TW];
    auto to_tw = [&](const Vec<NH>& c, typename E29::Tw& t) {
      encode(c, tmp);
      for (int i = 0; i < L; ++i) {
        t.w[i] = tmp[i];
        t.ws[i] = tmp[L + i];
      }
    };
    for (int k = 0; k < 3; ++k) to_tw(w8[k], A.w8[k]);
    to_tw(ninv, A.ninv);
    const uint32_t ptop = A.M.p[L - 1];
    A.red_ok = ptop >= (1u << 18) ? 1u : 0u;
    A.red_inv = std::nextafter(1.0f / (float)(ptop + 1u), 0.0f);
    // padded offsets for the unnormalised butterflies (used only when red_ok: p_top >= 3)
    auto padded = [&](uint32_t K, uint32_t pad, uint32_t* c) {
      uint32_t kp[L];
      uint64_t carry = 0;
      for (int i = 0; i < L; ++i) {
        const uint64_t v = (uint64_t)A.M.p[i] * K + carry;
        kp[i] = (uint32_t)v & kMask29;
        carry = v >> 29;
      }
      kp[L - 1] += (uint32_t)(carry << 29);  // K p < 2^(29L): carry is 0 for the supported fields
      const uint32_t b = pad >> 29;
      c[0] = kp[0] + pad;
      for (int i = 1; i + 1 < L; ++i) c[i] = kp[i] + pad - b;
      c[L - 1] = kp[L - 1] - b;
    };
    padded(5, 1u << 29, A.pc[E29::PC_5_29]);
    padded(9, 1u << 30, A.pc[E29::PC_9_30]);
    padded(4, 1u << 29, A.pc[E29::PC_4_29]);
    padded(17, 1u << 29, A.pc[E29::PC_17_29]);
    padded(7, 1u << 30, A.pc[E29::PC_7_30]);
  }
};

template <int N, int MEMW_, int SCR_>
struct EngHost<Eng32<N, MEMW_, SCR_>> {
  static constexpr int NH = N;
  using EA = typename Eng32<N, MEMW_, SCR_>::Args;
  using ET = typename Eng32<N, MEMW_, SCR_>::Tw;
  HostField<NH> const* H = nullptr;
  void init(const HostField<NH>& h) { H = &h; }
  // canonical c -> Shoup pair (c, floor(c 2^32 / p))
  void encode(const Vec<NH>& c, uint32_t* out) const {
    out[0] = c[0];
    out[1] = (uint32_t)(((uint64_t)c[0] << 32) / H->M.p[0]);
  }
  // entry whose value is c R_e (R_e = 2^32, the Montgomery radix of Eng32::mulv): c's Montgomery form
  void encode_scaled(const Vec<NH>& c, uint32_t* out) const { encode(H->to_mont(c), out); }
  // lazy values up to 4p must fit 32 bits
  bool check_modulus(const uint32_t* p) const { return p[0] < (1u << 30); }
  void fill_args(EA& A, const uint32_t* p, const Vec<NH>* w8, const Vec<NH>& ninv) const {
    A.p = p[0];
    A.p2 = 2 * p[0];
    uint32_t inv = 1;
    for (int i = 0; i < 5; ++i) inv *= 2 - p[0] * inv;  // p^-1 mod 2^32 (Newton)
    A.pinv = inv;
    uint32_t t[2];
    auto tw = [&](const Vec<NH>& c, ET& e) {
      encode(c, t);
      e.w[0] = t[0];
      e.ws = t[1];
    };
    for (int k = 0; k < 3; ++k) tw(w8[k], A.w8[k]);
    tw(ninv, A.ninv);
  }
};

template <class E>
struct PlanImpl final : PlanBase {
  static constexpr int NH = EngHost<E>::NH;
  static constexpr int TW = E::TW;
  static constexpr int MEMW = E::MEMW;
  static constexpr int SCRW = E::SCRW;  // scratch (engines.hpp)
  static constexpr int TABW = E::TABW;  // element-format twiddle tables (engines.hpp)
  HostField<NH> H;
  EngHost<E> EH;
  typename E::Args Ff{}, Fi{};
  uint32_t* d_tab = nullptr;
  uint32_t* d_scratch = nullptr;
  // per-pass outer twiddle tables (w R_e, HBM element format), one allocation per direction: the
  // forward's at plan creation, the inverse's at the first inverse call (a forward-only user pays for
  // one direction: 2^24 BN254 plan 1.55 -> 1.03 GB)
  uint32_t* d_fulls[2] = {nullptr, nullptr};
  size_t full_off[8] = {};  // element offsets of pass i's table in d_fulls[dir]
  size_t full_elems = 0;    // entries per direction
  bool use_full = false;
  uint32_t* d_full_sh = nullptr;  // passes >= 2: the same tables as Shoup pairs (E::TW words per entry)
  size_t full_sh_off[2][8] = {};  // entry offsets into d_full_sh, [dir][pass]
  bool full_sh_ok[8] = {};         // pass i takes its outer twiddles from d_full_sh
  size_t off_pinvB = 0;           // p^-1 mod B (E::W limbs) in d_tab (Shoup-pair table build)
  size_t scratch_elems = 0;
  // table word offsets
  size_t off_int_f[8] = {0}, off_int_i[8] = {0};
  size_t off_lo_f = 0, off_hi_f = 0, off_lo_i = 0, off_hi_i = 0, off_hi_is = 0, off_r2 = 0;
  size_t off_los_f = 0, off_los_i = 0;  // lo tables scaled by R_e (left factor of on-the-fly twiddles)
  size_t off_rm = 0;                    // R_e R^-1 (Montgomery-form pointwise product)
  size_t off_pow2inv = 0;               // 2^-k, k = 0..log_n, E::TW words each (build_fs_table's scale)
  size_t off_hi_ipm = 0;                // inverse hi table scaled by n^-1 R_e (fused polymul, pass 1)
  uint32_t* d_full_pm = nullptr;        // inverse pass-1 outer twiddles x n^-1 R_e (fused polymul)
  uint32_t* d_stk_tab = nullptr;        // NTT_PLAN_STOCKHAM: per-pass input-twiddle tables
  uint32_t* d_naive_pw = nullptr;       // NTT_PLAN_NAIVE: w_n^i R_e, i < n/2 (the reference's `roots`)
  uint32_t* d_naive_buf = nullptr;      // NTT_PLAN_NAIVE: the bit-reversed copy the rounds work on
                                        // (NO_SWAP, bealto family: the ping-pong partner of the caller's buffer)
  size_t off_bealto_pq = 0;             // bealto family: w_{2^max_deg}^j, j < 2^(max_deg - 1), Shoup pairs
  unsigned bealto_max_deg = 0, bealto_log_g = 0;
  size_t stk_off[8] = {};               // element offsets into d_stk_tab (pass >= 1)
  unsigned stk_ord[8] = {};             // Stockham pass i runs radix r[stk_ord[i]] (widest first)
  uint32_t* d_stk_buf[2] = {nullptr, nullptr};  // NTT_PLAN_STOCKHAM ping-pong buffers (E::MEMW words)
  unsigned lo_bits = 0;
  uint32_t nrand = 1, top_bits = 28;

  ~PlanImpl() override {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    if (d_tab) (void)hipFree(d_tab);
    if (d_scratch) (void)hipFree(d_scratch);
    for (auto* p : d_fulls)
      if (p) (void)hipFree(p);
    if (d_full_sh) (void)hipFree(d_full_sh);
    if (d_full_pm) (void)hipFree(d_full_pm);
    if (d_stk_tab) (void)hipFree(d_stk_tab);
    if (d_naive_pw) (void)hipFree(d_naive_pw);
    if (d_naive_buf) (void)hipFree(d_naive_buf);
    for (auto* p : d_stk_buf)
      if (p) (void)hipFree(p);
    if (d_bad) (void)hipFree(d_bad);
    if (d_coset) (void)hipFree(d_coset);
    if (d_coset_full) (void)hipFree(d_coset_full);
    if (d_sync) (void)hipFree(d_sync);
    if (d_sync_ip) (void)hipFree(d_sync_ip);
    if (d_sync2) (void)hipFree(d_sync2);
    if (d_trace) (void)hipFree(d_trace);
    if (d_ipn) (void)hipFree(d_ipn);
    if (d_pw) (void)hipFree(d_pw);
    if (d_dbg) (void)hipFree(d_dbg);
    watch_slot_release(h_watch);
    for (auto& row : ev)
      for (auto& e : row)
        if (e) (void)hipEventDestroy(e);
    (void)hipSetDevice(cur);
  }

  // modulus / generator as NH 32-bit words
  int init(const uint32_t* p, const uint32_t* g, unsigned log_n_, int dev, unsigned flags_) {
    device = dev;
    flags = flags_;
    log_n = log_n_;
    n = 1ull << log_n;
    elem_bytes = 4 * MEMW;
    // ---- modulus checks: odd, top word < 2^31 - 1 (no-carry host Montgomery)
    for (int i = 0; i < NH; ++i) H.M.p[i] = p[i];
    if (!(p[0] & 1)) return NTT_ERR_FIELD;
    if (p[NH - 1] >= 0x7fffffffu) return NTT_ERR_FIELD;
    EH.init(H);
    if (!EH.check_modulus(p)) return NTT_ERR_FIELD;
    uint32_t inv = 1;
    for (int i = 0; i < 5; ++i) inv *= 2 - p[0] * inv;
    H.M.pinv = 0u - inv;
    // R mod p, R^2 mod p by doubling (R = 2^(32 NH))
    {
      Vec<NH> x{};
      x[0] = 1;
      for (int k = 0; k < 32 * NH; ++k) x = H.add(x, x);
      H.r1 = x;
      for (int k = 0; k < 32 * NH; ++k) x = H.add(x, x);
      H.r2 = x;
    }
    EH.init(H);  // needs r2 for to_mont
    Vec<NH> pv, gv;
    for (int i = 0; i < NH; ++i) {
      pv[i] = p[i];
      gv[i] = g[i];
    }
    if (!vec_lt<NH>(gv, pv)) return NTT_ERR_FIELD;
    // (p - 1) >> log_n, and n | p - 1
    std::vector<uint32_t> pm1(p, p + NH);
    pm1[0] -= 1;  // p odd: no borrow
    for (unsigned b = 0; b < log_n; ++b)
      if ((pm1[b / 32] >> (b % 32)) & 1) return NTT_ERR_FIELD;
    std::vector<uint32_t> e(NH, 0);
    for (int i = 0; i < NH; ++i) {
      const unsigned wsh = log_n / 32, bsh = log_n % 32;
      uint64_t lo = (i + wsh < (unsigned)NH) ? pm1[i + wsh] : 0;
      uint64_t hi = (i + wsh + 1 < (unsigned)NH) ? pm1[i + wsh + 1] : 0;
      e[i] = (uint32_t)(((hi << 32) | lo) >> bsh);
    }
    const Vec<NH> gm = H.to_mont(gv);
    const Vec<NH> w = H.pow(gm, e);  // w_n (32-bit Montgomery form)
    if (log_n >= 1) {                // primitive: w^(n/2) == -1
      Vec<NH> pm1v;
      for (int i = 0; i < NH; ++i) pm1v[i] = pm1[i];
      if (H.from_mont(H.pow_u64(w, n / 2)) != pm1v) return NTT_ERR_FIELD;
    }
    std::vector<uint32_t> pm2(p, p + NH);  // p - 2 with borrow (BLS12-381 Fr has p[0] = 1)
    {
      uint64_t br = 2;
      for (int i = 0; i < NH && br; ++i) {
        const uint64_t d = (uint64_t)pm2[i] - br;
        pm2[i] = (uint32_t)d;
        br = (d >> 63) & 1;
      }
    }
    const Vec<NH> winv = H.pow(w, pm2);
    Vec<NH> nv{};
    nv[0] = (uint32_t)n;
    if (NH > 1) nv[1] = (uint32_t)(n >> 32);
    const Vec<NH> ninv_c = H.from_mont(H.pow(H.to_mont(nv), pm2));
    // field args per direction: w_8^k canonical
    auto fill_args = [&](typename E::Args& F, const Vec<NH>& wn) {
      const Vec<NH> w8m = (log_n >= 3) ? H.pow_u64(wn, n / 8) : H.r1;
      Vec<NH> acc = w8m, w8c[3];
      for (int k = 0; k < 3; ++k) {
        w8c[k] = H.from_mont(acc);
        acc = H.mul(acc, w8m);
      }
      EH.fill_args(F, p, w8c, ninv_c);
    };
    fill_args(Ff, w);
    fill_args(Fi, winv);

    // random-fill parameters: top nonzero 64-bit limb of p, masked to bitlen-1 bits
    {
      const int L64 = (NH + 1) / 2;
      int top = 0;
      for (int i = L64 - 1; i >= 0; --i) {
        const uint64_t limb = (uint64_t)p[2 * i] | ((2 * i + 1 < NH) ? (uint64_t)p[2 * i + 1] << 32 : 0);
        if (limb) { top = i; break; }
      }
      const uint64_t tl = (uint64_t)p[2 * top] | ((2 * top + 1 < NH) ? (uint64_t)p[2 * top + 1] << 32 : 0);
      nrand = top + 1;
      top_bits = 63 - __builtin_clzll(tl);  // bitlen - 1
    }

    // ---- schedule + tables (engine-encoded)
    if (!schedule(log_n, tile_log_of<E>(), E::MIN_COLS_LOG, E::NARROW_FIRST, r, npass))
      return NTT_ERR_ARG;
    if (flags & NTT_PLAN_IN_PLACE) {
      // passes store their lazily reduced values where they read them: the scratch element must be
      // the caller's element
      if (E::SCRW != E::MEMW) return NTT_ERR_ARG;
      if (npass >= 2 &&
          !schedule_palindrome(log_n, tile_log_of<E>(), tile_log_of<E>() - E::MIN_COLS_LOG, npass, r, npass))
        return NTT_ERR_ARG;
    }
    const bool twiddle_only = (flags & NTT_PLAN_TWIDDLE_ONLY) != 0;
    std::vector<uint32_t> host;
    auto push_powers = [&](const Vec<NH>& base_m, uint64_t count, const Vec<NH>* scale_m,
                           bool scaled = false) -> size_t {
      return push_powers_to(host, base_m, count, scale_m, scaled);
    };
    const Vec<NH> ninv_m = H.to_mont(ninv_c);
    for (int dir = 0; dir < 2; ++dir) {
      const Vec<NH>& wn = dir ? winv : w;
      size_t* off_int = dir ? off_int_i : off_int_f;
      if (twiddle_only) {
        // no transform tables
      } else if (npass == 0) {
        off_int[0] = push_powers(wn, n, nullptr);
      } else {
        for (unsigned i = 0; i < npass; ++i) off_int[i] = push_powers(H.pow_u64(wn, n >> r[i]), 1ull << r[i], nullptr);
      }
      {  // two-level tables of w_n^e (outer twiddles, four-step twiddle_pack)
        lo_bits = (log_n + 1) / 2;
        const size_t lo = push_powers(wn, 1ull << lo_bits, nullptr);
        const size_t los = push_powers(wn, 1ull << lo_bits, nullptr, true);
        const Vec<NH> step = H.pow_u64(wn, 1ull << lo_bits);
        const size_t hi = push_powers(step, 1ull << (log_n - lo_bits), nullptr);
        if (dir == 0) {
          off_lo_f = lo;
          off_los_f = los;
          off_hi_f = hi;
        } else {
          off_lo_i = lo;
          off_los_i = los;
          off_hi_i = hi;
          off_hi_is = push_powers(step, 1ull << (log_n - lo_bits), &ninv_m);
          // fused polymul: the pointwise Montgomery product leaves a b / R_e; fold R_e in here
          const Vec<NH> ninv_re_m = H.mul(ninv_m, H.to_mont(engine_radix_mod_p()));
          off_hi_ipm = push_powers(step, 1ull << (log_n - lo_bits), &ninv_re_m);
        }
      }
    }
    if ((flags & kBealtoFlags) && !twiddle_only) {
      // the reference's pq table (GZKP-NTT.cu:489-499, 740-750): max_deg = min(8 - log_g, log_n), one
      // group per workgroup for bellperson, 2^5 for the improved kernels (GZKP-NTT.cu:1674-1704)
      if (log_n < 1) return NTT_ERR_ARG;
      bealto_log_g = (flags & NTT_PLAN_BELLPERSON) ? 0u : 5u;
      bealto_max_deg = std::min(8u - bealto_log_g, log_n);
      off_bealto_pq = push_powers(H.pow_u64(w, n >> bealto_max_deg), 1ull << (bealto_max_deg - 1), nullptr);
    }
    {  // pointwise product constants: mulv leaves a b / R_e (R_e the engine's Montgomery radix);
       // multiplying by R_e gives a b, by R_e R^-1 the Montgomery product a b R^-1 (R = 2^(64 limbs64))
      off_r2 = host.size();
      uint32_t enc[TW];
      EH.encode(engine_radix_mod_p(), enc);
      host.insert(host.end(), enc, enc + TW);
      while (host.size() % 4) host.push_back(0);
      Vec<NH> rio{};  // R = 2^(64 limbs64) mod p by doubling
      rio[0] = 1;
      for (int k = 0; k < 64 * ((NH + 1) / 2); ++k) rio = H.add(rio, rio);
      const Vec<NH> rio_inv = H.from_mont(H.pow(H.to_mont(rio), pm2));
      off_rm = host.size();
      EH.encode(H.from_mont(H.mul(H.to_mont(engine_radix_mod_p()), H.to_mont(rio_inv))), enc);
      host.insert(host.end(), enc, enc + TW);
      while (host.size() % 4) host.push_back(0);
    }
    {  // 2^-k mod p for k = 0..log_n as twiddles (Tw encoding): the four-step folds a row transform's
       // n2^-1 into its inverse epilogue table (build_fs_table's scale_log, ntt_rplan.cpp)
      off_pow2inv = host.size();
      uint32_t enc[TW];
      std::vector<std::vector<uint32_t>> ent(log_n + 1);
      Vec<NH> x = ninv_m;  // 2^-log_n (Montgomery form); doubling walks k down to 0
      for (int k = (int)log_n; k >= 0; --k) {
        EH.encode(H.from_mont(x), enc);
        ent[k].assign(enc, enc + TW);
        x = H.add(x, x);
      }
      for (unsigned k = 0; k <= log_n; ++k) host.insert(host.end(), ent[k].begin(), ent[k].end());
      while (host.size() % 4) host.push_back(0);
    }
    if constexpr (E::SHOUP_OUTER) {
      off_pinvB = host.size();
      host.insert(host.end(), EH.pinvB, EH.pinvB + E::W);
      while (host.size() % 4) host.push_back(0);
    }
    pm2_ = pm2;
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (hipSetDevice(device) != hipSuccess) return NTT_ERR_HIP;
    int rc = NTT_OK;
    if (hipMalloc(&d_tab, host.size() * 4) != hipSuccess ||
        hipMemcpy(d_tab, host.data(), host.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
      rc = NTT_ERR_HIP;
#if NTT_DEBUG_CHECKS
    // debug builds: the status word every kernel of this plan records check failures in
    if (rc == NTT_OK && (hipMalloc(&d_dbg, 4) != hipSuccess || hipMemset(d_dbg, 0, 4) != hipSuccess)) rc = NTT_ERR_HIP;
    Ff.dbg = Fi.dbg = d_dbg;
#endif
    if (rc == NTT_OK && npass >= 2 && !twiddle_only && !(flags & NTT_PLAN_IN_PLACE)) rc = ensure_scratch(1);
    if (rc == NTT_OK && npass >= 2 && !twiddle_only) rc = build_full_tables();
    // NTT_PLAN_GZKP runs on the same per-pass tables: Stockham pass i's w_n^((k pi) << (log_n - lgp_i - r_i))
    // for k < 2^lgp_i is the GZKP DIT pass's w_N^(c d), N = 2^(lgp_i + r_i)
    if (rc == NTT_OK && (flags & (NTT_PLAN_STOCKHAM | NTT_PLAN_GZKP))) rc = build_stockham();
    if (rc == NTT_OK && (flags & (NTT_PLAN_NAIVE | NTT_PLAN_NO_SWAP))) rc = build_naive();
    if (rc == NTT_OK && (flags & kBealtoFlags)) rc = build_bealto();
    (void)hipSetDevice(cur);
    return rc;
  }

  // NTT_PLAN_STOCKHAM (rival schedule, bellperson family): pass i (i >= 1) multiplies element pi of
  // group k < p_i = 2^(r_0 + ... + r_{i-1}) by w_n^((k pi) << (log_n - lgp_i - r_i)) from a table in
  // the column-group-major layout of the pass kernels (k_build_tw with c := k); two ping-pong buffers.
  int build_stockham() {
    if constexpr (!HasStockham<E>::value) {
      return NTT_ERR_ARG;
    } else {
      if (npass < 2) return NTT_ERR_ARG;
      // widest radix first: pass i >= 1 needs p_i = 2^(r_0 + ... + r_{i-1}) >= T_i = TILE / R_i
      for (unsigned i = 0; i < npass; ++i) stk_ord[i] = i;
      std::stable_sort(stk_ord, stk_ord + npass, [&](unsigned a, unsigned b) { return r[a] > r[b]; });
      size_t elems = 0;
      unsigned lgp = 0;
      const unsigned tl = tile_log_of<E>();
      for (unsigned i = 0; i < npass; ++i) {
        const unsigned ri = r[stk_ord[i]];
        if (i > 0) {
          if (lgp + ri < tl) return NTT_ERR_ARG;
          stk_off[i] = elems;
          elems += 1ull << (lgp + ri);
        }
        lgp += ri;
      }
      if (hipMalloc(&d_stk_tab, elems * TABW * 4) != hipSuccess) return NTT_ERR_HIP;
      for (auto*& p : d_stk_buf)
        if (hipMalloc(&p, (size_t)n * MEMW * 4) != hipSuccess) return NTT_ERR_HIP;
      lgp = r[stk_ord[0]];
      for (unsigned i = 1; i < npass; ++i) {
        const unsigned ri = r[stk_ord[i]];
        if (launch_build_tw<E>(d_stk_tab + stk_off[i] * TABW, 1ull << (lgp + ri), ri, tl - ri, log_n - lgp - ri,
                               d_tab + off_los_f, d_tab + off_hi_f, lo_bits, Ff, nullptr) != hipSuccess)
          return NTT_ERR_HIP;
        lgp += ri;
      }
      return hipDeviceSynchronize() == hipSuccess ? NTT_OK : NTT_ERR_HIP;
    }
  }

  // NTT_PLAN_GZKP (rival schedule, GZKP(B, G), GZKP-NTT.cu:115-233): digit reversal into a plan buffer
  // (`rearrange`; the bit reversal of the reference's radix-2 rounds), contiguous radix-2^r_0 DFTs (the reference's first rounds, `naive` / a GZKP launch
  // at stride 1), then in-place DIT passes over stride-2^lgp columns with input twiddles; the last
  // pass writes the caller's buffer.  Widest radix first, as for Stockham (lgp_i >= T_i).
  int run_gzkp(const uint32_t* in, uint32_t* out, hipStream_t st) {
    if constexpr (!HasStockham<E>::value) {
      return NTT_ERR_ARG;
    } else {
      const unsigned tl = tile_log_of<E>();
      uint32_t* buf = d_stk_buf[0];
      uint32_t digits[8];
      for (unsigned i = 0; i < npass; ++i) digits[i] = r[stk_ord[i]];
      begin(st);
      hipError_t e = launch_bitrev<E>(in, buf, log_n, digits, npass, st);
      mark(st);
      unsigned lgp = 0;
      for (unsigned i = 0; i < npass && e == hipSuccess; ++i) {
        const unsigned ri = r[stk_ord[i]];
        PassArgs<E> A = base_args(false);
        A.tw_int = d_tab + off_int_f[stk_ord[i]];  // w_R^e for this pass's radix
        uint32_t* dst = i + 1 == npass ? out : buf;
        if (i == 0) {  // s = 1: contiguous 2^r_0-point DFTs, batched (grid.y chunks of <= 2^15 blocks)
          A.batch_stride = ((size_t)1 << ri) * MEMW;
          const size_t blocks = n >> ri, chunk = size_t(1) << 15;
          for (size_t b0 = 0; b0 < blocks && e == hipSuccess; b0 += chunk) {
            const size_t off = (b0 << ri) * MEMW;
            e = launch_pass<E>(KIND_SINGLE, (int)ri, buf + off, buf + off, A, 1,
                               (uint32_t)(blocks - b0 < chunk ? blocks - b0 : chunk), st);
          }
        } else {
          A.tw_full = d_stk_tab + stk_off[i] * TABW;  // w_N^(c d), N = 2^(lgp + r_i)
          A.log_blk = lgp + ri;
          A.lgp = lgp;
          A.src_user = 1;
          e = launch_pass<E>(KIND_DIT, (int)ri, buf, dst, A, (uint32_t)(n >> tl), 1, st);
        }
        mark(st);
        lgp += ri;
      }
      return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
    }
  }

  // NTT_PLAN_NAIVE (rival schedule, the reference's `naive`, GZKP-NTT.cu:59-95 / big-num.cu:67-170):
  // the bit reversal (`rearrange`), then log2 n radix-2 DIT rounds of one launch each, every round
  // a full read and write of the vector (HBM-bound; the measure of what the pass kernels' fusion
  // buys).  The reference's n-entry `roots` table is the n/2 entries its rounds read.
  int build_naive() {
    if constexpr (!HasStockham<E>::value) {
      return NTT_ERR_ARG;  // the rival schedules: P and 4 x 64-bit plans
    } else {
      if (log_n < 1 || log_n > 32) return NTT_ERR_ARG;
      const size_t half = n / 2;
      if (hipMalloc(&d_naive_pw, half * TABW * 4) != hipSuccess) return NTT_ERR_HIP;
      if (hipMalloc(&d_naive_buf, (size_t)n * MEMW * 4) != hipSuccess) return NTT_ERR_HIP;
      if (launch_build_pow<E>(d_naive_pw, half, d_tab + off_los_f, d_tab + off_hi_f, lo_bits, Ff, nullptr) !=
          hipSuccess)
        return NTT_ERR_HIP;
      return hipDeviceSynchronize() == hipSuccess ? NTT_OK : NTT_ERR_HIP;
    }
  }

  int run_naive(const uint32_t* in, uint32_t* out, hipStream_t st) {
    begin(st);
    hipError_t e = launch_bitrev<E>(in, d_naive_buf, log_n, nullptr, 0, st);  // radix-2 rounds: the bit reversal
    mark(st);
    for (unsigned s = 0; s < log_n && e == hipSuccess; ++s)
      e = launch_naive_round<E>(d_naive_buf, s + 1 == log_n ? out : d_naive_buf, log_n, s, d_naive_pw, Ff, st);
    mark(st);  // last_launch_ms: [bit reversal, all rounds]
    return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
  }

  // NTT_PLAN_NO_SWAP (rival schedule, the reference's `naive_no_swap`, GZKP-NTT.cu:237-296): a radix-2
  // Stockham autosort, one launch per round, ping-pong between the caller's buffer and the plan
  // buffer (natural order in and out, no bit reversal); an odd round count ends in the plan buffer
  // and one device copy brings it back.  The same n/2-entry power table as NTT_PLAN_NAIVE.
  int run_noswap(uint32_t* data, hipStream_t st) {
    begin(st);
    hipError_t e = hipSuccess;
    uint32_t* buf[2] = {data, d_naive_buf};
    for (unsigned s = 0; s < log_n && e == hipSuccess; ++s)
      e = launch_noswap_round<E>(buf[s & 1], buf[(s + 1) & 1], log_n, s, d_naive_pw, Ff, st);
    if (e == hipSuccess && (log_n & 1))
      e = hipMemcpyAsync(data, d_naive_buf, (size_t)n * MEMW * 4, hipMemcpyDeviceToDevice, st);
    mark(st);  // last_launch_ms: [all rounds (and the copy)]
    return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
  }

  // NTT_PLAN_BELLPERSON / NTT_PLAN_IMPROVED_V1..V4 (rival schedules, the reference's bealto.com group
  // FFT and its four refinements, GZKP-NTT.cu:391-464, 556-1296): rounds of 2^deg-point groups,
  // deg = min(max_deg, log_n - lgp), one launch each (k_bealto), ping-pong between the caller's buffer
  // and the plan buffer; an odd round count ends in the plan buffer and one device copy brings it back.
  int build_bealto() {
    if constexpr (!HasStockham<E>::value) {
      return NTT_ERR_ARG;  // the rival schedules: P and 4 x 64-bit plans
    } else {
      if (log_n < 1 || log_n > 32 || bealto_max_deg < 1) return NTT_ERR_ARG;
      if (hipMalloc(&d_naive_buf, (size_t)n * MEMW * 4) != hipSuccess) return NTT_ERR_HIP;
      return NTT_OK;
    }
  }
  int bealto_variant() const {
    if (flags & NTT_PLAN_BELLPERSON) return BEALTO_BELLPERSON;
    if (flags & NTT_PLAN_IMPROVED_V1) return BEALTO_V1;
    if (flags & NTT_PLAN_IMPROVED_V2) return BEALTO_V2;
    if (flags & NTT_PLAN_IMPROVED_V3) return BEALTO_V3;
    return BEALTO_V4;
  }
  int run_bealto(uint32_t* data, hipStream_t st) {
    if constexpr (!HasStockham<E>::value) {
      return NTT_ERR_ARG;
    } else {
      const int variant = bealto_variant();
      PassArgs<E> A = base_args(false);
      A.tw_int = d_tab + off_bealto_pq;
      A.tw_lo = d_tab + off_los_f;  // lo R_e: (lo R_e) hi, then the Montgomery product leaves x w
      A.tw_hi = d_tab + off_hi_f;
      BealtoArgs B{log_n, 0u, 0u, 0u, bealto_max_deg};
      uint32_t* buf[2] = {data, d_naive_buf};
      const unsigned nr = (log_n + bealto_max_deg - 1) / bealto_max_deg;
      const bool per_round = nr + 2 < kEv;  // one profiling interval per round while they fit
      const char* lab = variant == BEALTO_BELLPERSON ? "g" : "v";
      begin(st);
      hipError_t e = hipSuccess;
      unsigned rounds = 0;
      while (B.lgp < log_n && e == hipSuccess) {
        B.deg = std::min(bealto_max_deg, log_n - B.lgp);
        B.log_g = std::min(bealto_log_g, log_n - B.deg);
        e = launch_bealto<E>(variant, buf[rounds & 1], buf[(rounds + 1) & 1], A, B, st);
        if (per_round) mark(st, lab, B.deg);
        B.lgp += B.deg;
        ++rounds;
      }
      if (e == hipSuccess && (rounds & 1))
        e = hipMemcpyAsync(data, d_naive_buf, (size_t)n * MEMW * 4, hipMemcpyDeviceToDevice, st);
      if (!per_round || (rounds & 1)) mark(st, per_round ? "cp" : lab);
      return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
    }
  }

  int run_stockham(const uint32_t* in, uint32_t* out, hipStream_t st) {
    const uint32_t grid = (uint32_t)(n >> tile_log_of<E>());
    hipError_t e = hipSuccess;
    unsigned lgp = 0;
    begin(st);
    for (unsigned i = 0; i < npass && e == hipSuccess; ++i) {
      const unsigned ri = r[stk_ord[i]];
      PassArgs<E> A = base_args(false);
      A.tw_int = d_tab + off_int_f[stk_ord[i]];  // w_R^e for this pass's radix
      A.tw_full = i ? d_stk_tab + stk_off[i] * TABW : nullptr;
      A.log_blk = log_n;
      A.lgp = lgp;
      A.src_user = 1;
      const uint32_t* src = i == 0 ? in : d_stk_buf[(i - 1) & 1];
      uint32_t* dst = i + 1 == npass ? out : d_stk_buf[i & 1];
      e = launch_pass<E>(KIND_STOCKHAM, (int)ri, src, dst, A, grid, 1, st);
      mark(st);
      lgp += ri;
    }
    return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
  }

  // Full per-pass outer-twiddle tables: pass i needs N_i entries (N_1 = n, N_2 = n / R_1, ...),
  // streamed from HBM like the data in pass 1 and L2-resident afterwards.  They replace the
  // two-level lookup's extra Montgomery product per element.  Skipped when a direction's tables
  // would not fit (the two-level tables are then used).
  // Cap: both directions together within a quarter of the free HBM at plan creation.
  int build_full_tables() {
    size_t elems = 0;
    unsigned blk = log_n;
    for (unsigned i = 0; i + 1 < npass; ++i) {
      full_off[i] = elems;
      elems += 1ull << blk;
      blk -= r[i];
    }
    full_elems = elems;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return NTT_OK;
    if (2 * elems * TABW * 4 > free_b / 4) return NTT_OK;  // both directions within a quarter of free HBM
    if (int rc = ensure_full(0, nullptr)) return rc;
    if (hipDeviceSynchronize() != hipSuccess) return NTT_ERR_HIP;  // plan creation is synchronous
    use_full = true;
    return build_shoup_tables();
  }
  // The per-pass tables of one direction (the inverse's pass-1 table carries n^-1), built on `st`.
  // The forward's are built at plan creation, the inverse's at the first inverse call (a forward-only
  // plan never holds them): that build is enqueued on the call's stream ahead of its passes, with no
  // device-wide synchronisation.  If the allocation fails then, the direction keeps its two-level
  // tables (one more product per element in pass 1) instead of failing the call.
  bool full_failed[2] = {false, false};
  int ensure_full(int dir, hipStream_t st) {
    if (d_fulls[dir] || full_failed[dir]) return NTT_OK;
    if (hipMalloc(&d_fulls[dir], full_elems * TABW * 4) != hipSuccess) {
      d_fulls[dir] = nullptr;
      (void)hipGetLastError();  // clear the sticky allocation error
      if (dir == 0) return NTT_ERR_HIP;  // at creation: the plan reports it
      full_failed[dir] = true;
      return NTT_OK;
    }
    unsigned blk = log_n;
    for (unsigned i = 0; i + 1 < npass; ++i) {
      const uint32_t* lo = d_tab + (dir ? off_los_i : off_los_f);
      const uint32_t* hi = d_tab + (dir ? (i == 0 ? off_hi_is : off_hi_i) : off_hi_f);
      // column-group-major layout of the pass kernel's tiles (T = TILE / R columns per workgroup)
      if (launch_build_tw<E>(d_fulls[dir] + full_off[i] * TABW, 1ull << blk, r[i], tile_log_of<E>() - r[i], log_n - blk,
                             lo, hi, lo_bits, dir ? Fi : Ff, st) != hipSuccess) {
        // a partly built table must never be read as a built one: drop it; the
        // direction falls back to the two-level tables (the inverse) or the plan fails (creation)
        (void)hipFree(d_fulls[dir]);
        d_fulls[dir] = nullptr;
        (void)hipGetLastError();
        if (dir == 0) return NTT_ERR_HIP;
        full_failed[dir] = true;
        return NTT_OK;
      }
      blk -= r[i];
    }
    return NTT_OK;
  }

  // Column passes whose table is small enough to stay in L2 (N_i entries of E::TW words <= 8 MiB):
  // Shoup pairs instead of w R_e, so their outer-twiddle product is a Shoup product (143 MADs)
  // instead of a Montgomery one (162).  Measured (profiles/r02_sh/): 2^24 pass 2 (5 MiB table)
  // -0.5 %, 2^28 pass 3 (1.3 MiB) -1.2 %, 2^28 pass 2 (168 MiB, not L2-resident) +6 % -- hence the cap.
  // Round 5: pass 1 too when its table fits (plans of <= 2^16 points: the four-step's 2^16-point
  // column transforms of 2^24, C4's 2^14-point rows and columns), on engines whose scratch and caller
  // layouts agree (one kernel instance reads both); the inverse's pass-1 table carries n^-1 as its
  // Montgomery twin does.  NTT_SHOUP_OUTER=0 in the environment keeps the Montgomery tables (A/B
  // switch); =1 keeps pass 1 on its Montgomery table (round-4 behaviour).
  static int shoup_outer_env() {
    static const int v = [] {
      const char* e = getenv("NTT_SHOUP_OUTER");
      return e && *e ? atoi(e) : 2;
    }();
    return v;
  }
  int build_shoup_tables() {
    if constexpr (!E::SHOUP_OUTER) {
      return NTT_OK;
    } else {
      if (shoup_outer_env() == 0) return NTT_OK;
      if (npass < 2 || !Ff.red_ok) return NTT_OK;  // the Shoup-pair column kernels are FAST instances
      constexpr size_t kMaxTableBytes = 8ull << 20;
      constexpr bool pass1_ok = E::SCRW == E::MEMW;  // pass 1 reads the caller's layout
      const unsigned i0 = (pass1_ok && shoup_outer_env() >= 2) ? 0u : 1u;
      size_t elems = 0;
      unsigned blk = log_n;
      for (unsigned i = 0; i + 1 < npass; ++i) {
        full_sh_off[0][i] = elems;
        full_sh_ok[i] = i >= i0 && ((1ull << blk) * TW * 4) <= kMaxTableBytes;
        if (full_sh_ok[i]) elems += 1ull << blk;
        blk -= r[i];
      }
      if (elems == 0) return NTT_OK;
      size_t free_b = 0, total_b = 0;
      if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return NTT_OK;
      if (2 * elems * TW * 4 > free_b / 8) {
        for (auto& ok : full_sh_ok) ok = false;
        return NTT_OK;
      }
      if (hipMalloc(&d_full_sh, 2 * elems * TW * 4) != hipSuccess) return NTT_ERR_HIP;
      for (int dir = 0; dir < 2; ++dir) {
        blk = log_n;
        for (unsigned i = 0; i + 1 < npass; ++i) {
          full_sh_off[dir][i] = dir * elems + full_sh_off[0][i];
          if (!full_sh_ok[i]) {
            blk -= r[i];
            continue;
          }
          const uint32_t* lo = d_tab + (dir ? off_los_i : off_los_f);
          const uint32_t* hi = d_tab + (dir ? (i == 0 ? off_hi_is : off_hi_i) : off_hi_f);
          if (launch_build_tw_sh<E>(d_full_sh + full_sh_off[dir][i] * TW, 1ull << blk, r[i], tile_log_of<E>() - r[i],
                                    log_n - blk, lo, hi, lo_bits, dir ? Fi : Ff, d_tab + off_pinvB,
                                    nullptr) != hipSuccess)
            return NTT_ERR_HIP;
          blk -= r[i];
        }
      }
      return hipDeviceSynchronize() == hipSuccess ? NTT_OK : NTT_ERR_HIP;
    }
  }

  // Append count entries base^k * scale (engine table format) to host; returns their word offset.
  // scaled: entries hold value * R_e (the left factor of two-level products, see encode_scaled).
  size_t push_powers_to(std::vector<uint32_t>& host, const Vec<NH>& base_m, uint64_t count, const Vec<NH>* scale_m,
                        bool scaled) const {
    const size_t off = host.size();
    Vec<NH> cur = scale_m ? *scale_m : H.r1;
    uint32_t enc[TW];
    for (uint64_t k = 0; k < count; ++k) {
      if (scaled)
        EH.encode_scaled(H.from_mont(cur), enc);
      else
        EH.encode(H.from_mont(cur), enc);
      host.insert(host.end(), enc, enc + TW);
      cur = H.mul(cur, base_m);
    }
    while (host.size() % 4) host.push_back(0);
    return off;
  }

  // ---- coset (low-degree extension): data[j] *= c^j before the forward, c^-j after the inverse
  std::vector<uint32_t> coset_key;  // shift c (NH words) of the cached tables
  uint32_t* d_coset = nullptr;
  uint32_t* d_coset_full = nullptr;  // fused coset forward: pass-1 outer twiddles x c^col (n entries)
  bool coset_full_ok = false;
  size_t coset_off[2][3] = {};  // [dir][lo_s, hi, u^d (forward only)] word offsets into d_coset
  std::vector<uint32_t> pm2_;    // p - 2 (inversion exponent)

  unsigned long long* d_bad = nullptr;  // canonical-range check counter
  int count_noncanonical(const void* d, uint64_t count, uint64_t* bad, hipStream_t st) override {
    if (!d || !bad) return NTT_ERR_ARG;
    if (!d_bad && hipMalloc(&d_bad, sizeof(*d_bad)) != hipSuccess) {
      d_bad = nullptr;
      return NTT_ERR_HIP;
    }
    ModWords<MEMW> pw{};
    for (int i = 0; i < NH && i < MEMW; ++i) pw.w[i] = H.M.p[i];
    unsigned long long h = 0;
    if (hipMemsetAsync(d_bad, 0, sizeof(*d_bad), st) != hipSuccess ||
        launch_count_noncanonical<E>(static_cast<const uint32_t*>(d), count, pw, d_bad, st) != hipSuccess ||
        hipMemcpyAsync(&h, d_bad, sizeof(h), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return NTT_ERR_HIP;
    *bad = h;
    return NTT_OK;
  }

  int coset(void* d, const uint64_t* shift, unsigned limbs64, bool inverse, hipStream_t st) override {
    if (!d || !shift || (flags & NTT_PLAN_TWIDDLE_ONLY)) return NTT_ERR_ARG;
    Vec<NH> c{};
    for (int i = 0; i < NH; ++i) c[i] = (uint32_t)(shift[i / 2] >> (32 * (i % 2)));
    for (unsigned i = (NH + 1) / 2; i < limbs64; ++i)
      if (shift[i]) return NTT_ERR_ARG;
    if ((NH & 1) && (shift[NH / 2] >> 32)) return NTT_ERR_ARG;
    Vec<NH> pv;
    for (int i = 0; i < NH; ++i) pv[i] = H.M.p[i];
    if (!vec_lt<NH>(c, pv) || c == Vec<NH>{}) return NTT_ERR_ARG;
    const std::vector<uint32_t> key(c.begin(), c.end());
    if (key != coset_key) {
      if (d_coset) (void)hipFree(d_coset);
      d_coset = nullptr;
      coset_key.clear();
      std::vector<uint32_t> host;
      const Vec<NH> cm = H.to_mont(c);
      const Vec<NH> cim = H.pow(cm, pm2_);
      for (int dir = 0; dir < 2; ++dir) {
        const Vec<NH>& b = dir ? cim : cm;
        coset_off[dir][0] = push_powers_to(host, b, 1ull << lo_bits, nullptr, true);
        const Vec<NH> step = H.pow_u64(b, 1ull << lo_bits);
        coset_off[dir][1] = push_powers_to(host, step, 1ull << (log_n - lo_bits), nullptr, false);
      }
      // fused forward: u^d, u = c^s (s = n / R_1 columns of pass 1), d < R_1, Shoup entries
      if (npass >= 2) coset_off[0][2] = push_powers_to(host, H.pow_u64(cm, n >> r[0]), 1ull << r[0], nullptr, false);
      coset_full_ok = false;
      if (hipMalloc(&d_coset, host.size() * 4) != hipSuccess) return NTT_ERR_HIP;
      if (hipMemcpy(d_coset, host.data(), host.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return NTT_ERR_HIP;
      coset_key = key;
    }
    const int dir = inverse ? 1 : 0;
    auto scale = [&]() {
      return launch_scale_pow<E>(static_cast<uint32_t*>(d), log_n, 1, d_coset + coset_off[dir][0],
                                 d_coset + coset_off[dir][1], lo_bits, Ff, st) == hipSuccess
                 ? NTT_OK
                 : NTT_ERR_HIP;
    };
    if (!inverse) {
      if (coset_fusable()) {  // the scale rides in pass 1: u^d at load, c^col in the outer twiddles
        if (int rc = ensure_coset_full()) return rc;
        uint32_t* x = static_cast<uint32_t*>(d);
        return run_io(x, nullptr, x, 1, false, st, d_coset_full, d_coset + coset_off[0][2]);
      }
      if (int rc = scale()) return rc;
      return run(d, 1, false, st);
    }
    if (int rc = run(d, 1, true, st)) return rc;
    return scale();
  }

  bool coset_fusable() const {
    if constexpr (!E::FASTRED) {
      return false;
    } else {
      return use_full && npass >= 2 && Ff.red_ok;
    }
  }
  // Pass-1 outer-twiddle table of the fused coset forward for the cached shift c: entry (col, k) =
  // w_n^(col k) c^col R_e, layout of d_full (built on the device once per shift).
  int ensure_coset_full() {
    if (coset_full_ok) return NTT_OK;
    if (!d_coset_full && hipMalloc(&d_coset_full, (size_t)n * TABW * 4) != hipSuccess) {
      d_coset_full = nullptr;
      return NTT_ERR_HIP;
    }
    if (launch_build_tw<E>(d_coset_full, n, r[0], tile_log_of<E>() - r[0], 0, d_tab + off_los_f, d_tab + off_hi_f,
                           lo_bits, Ff, nullptr, d_coset + coset_off[0][0], d_coset + coset_off[0][1]) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess)
      return NTT_ERR_HIP;
    coset_full_ok = true;
    return NTT_OK;
  }

  // canonical value of the engine's Montgomery radix R_e mod p
  Vec<NH> engine_radix_mod_p() const {
    if constexpr (IsEng32<E>::value) {
      return H.r1;  // 2^(32N) mod p
    } else {
      return EH.kR;  // 2^(29L) mod p
    }
  }

  int ensure_scratch(unsigned batch) {
    const size_t need = (size_t)n * batch;
    if (need <= scratch_elems) return NTT_OK;
    if (d_scratch) (void)hipFree(d_scratch);
    d_scratch = nullptr;
    scratch_elems = 0;
    if (hipMalloc(&d_scratch, need * SCRW * 4) != hipSuccess) return NTT_ERR_HIP;
    scratch_elems = need;
    return NTT_OK;
  }

  // debug builds: element extents of a pass's src / dst from the transform's first element (n per
  // transform, n 2^il in Mode I); the four-step maps into the caller's exchange blocks stay unchecked
  void set_extents(PassArgs<E>& A, const FsIO* io, uint32_t il) const {
    const size_t ext = (size_t)n << il;
    A.dbg_src_n = (io && (A.fs & FS_MAP_IN)) ? ~(size_t)0 : ext;
    A.dbg_dst_n = (io && (A.fs & FS_MAP_OUT)) ? ~(size_t)0 : ext;
  }
  PassArgs<E> base_args(bool inverse) const {
    PassArgs<E> A;
    memset(&A, 0, sizeof(A));
    A.F = inverse ? Fi : Ff;
    A.log_n = log_n;
    A.lo_bits = lo_bits;
    A.batch_stride = (size_t)n * MEMW;
    A.dbg_src_n = A.dbg_dst_n = ~(size_t)0;  // debug builds: unchecked unless run_io knows the extents
    return A;
  }

  unsigned passes_for(unsigned log_x) const override {
    unsigned rr[8] = {0}, p = 0;
    if (!schedule(log_x, tile_log_of<E>(), E::MIN_COLS_LOG, E::NARROW_FIRST, rr, p))
      return 99;
    return p == 0 ? 1 : p;
  }
  unsigned max_radix_for(unsigned log_x) const override {
    unsigned rr[8] = {0}, p = 0;
    if (!schedule(log_x, tile_log_of<E>(), E::MIN_COLS_LOG, E::NARROW_FIRST, rr, p)) return 99;
    unsigned m = p == 0 ? log_x : 0;
    for (unsigned i = 0; i < p; ++i) m = rr[i] > m ? rr[i] : m;
    return m;
  }

  int run(void* d, unsigned batch, bool inverse, hipStream_t st) override {
    if (!d || batch == 0 || (flags & NTT_PLAN_TWIDDLE_ONLY)) return NTT_ERR_ARG;
    if ((flags & NTT_PLAN_STOCKHAM) && !inverse && batch == 1 && d_stk_tab)
      return run_stockham(static_cast<uint32_t*>(d), static_cast<uint32_t*>(d), st);
    if ((flags & NTT_PLAN_GZKP) && !inverse && batch == 1 && d_stk_tab)
      return run_gzkp(static_cast<uint32_t*>(d), static_cast<uint32_t*>(d), st);
    if ((flags & NTT_PLAN_NAIVE) && !inverse && batch == 1 && d_naive_pw)
      return run_naive(static_cast<uint32_t*>(d), static_cast<uint32_t*>(d), st);
    if ((flags & NTT_PLAN_NO_SWAP) && !inverse && batch == 1 && d_naive_pw)
      return run_noswap(static_cast<uint32_t*>(d), st);
    if ((flags & kBealtoFlags) && !inverse && batch == 1 && d_naive_buf)
      return run_bealto(static_cast<uint32_t*>(d), st);
    return run_io(static_cast<uint32_t*>(d), nullptr, static_cast<uint32_t*>(d), batch, inverse, st);
  }

  // One transform (or a batch): reads `in` (and, for a fused polymul inverse, `in2`: the first pass
  // starts from the pointwise product in * in2), writes `out` (may equal `in`).
  // Fused coset forward: full0 replaces the first pass's outer-twiddle table and tw_in scales its
  // inputs (PRO_COSET in ntt_kernels_impl.hpp).
  int run_io(const uint32_t* in, const uint32_t* in2, uint32_t* out, unsigned batch, bool inverse, hipStream_t st,
             const uint32_t* full0 = nullptr, const uint32_t* tw_in = nullptr, const FsIO* io = nullptr) {
    const uint32_t il = (io && (io->fs & FS_IL)) ? io->il : 0u;
    auto set_fs = [&](PassArgs<E>& A, uint32_t bits) {
      if (!io) return;
      A.fs = io->fs & (bits | FS_IL | FS_MAP_EPI);
      A.il = il;
      A.min = io->min;
      A.mout = io->mout;
      A.mepi = io->mepi;
    };
    if (io && (log_n == 0 || npass == 0)) return NTT_ERR_ARG;  // four-step pieces are >= 8 points
    if (log_n == 0) {
      if (out != in && hipMemcpyAsync(out, in, (size_t)batch * MEMW * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return NTT_ERR_HIP;
      return NTT_OK;
    }
    const size_t* off_int = inverse ? off_int_i : off_int_f;
    hipError_t e = hipSuccess;
    begin(st);
    if (npass == 0) {
      PassArgs<E> A = base_args(inverse);
      A.tw_int = d_tab + off_int[0];
      A.flags = inverse ? 1u : 0u;
      e = launch_naive<E>(in, out, A, batch, st);
      mark(st, "n");
    } else if (npass == 1) {
      PassArgs<E> A = base_args(inverse);
      A.tw_int = d_tab + off_int[0];
      A.flags = (inverse && !(io && io->no_scale)) ? 1u : 0u;  // no_scale: n^-1 folded in by the caller
      set_fs(A, FS_MAP_IN | FS_MAP_OUT);
      if (io) A.tw_epi = static_cast<const uint32_t*>(io->tw_epi);
      set_extents(A, io, il);
      const uint32_t nt = il ? (1u << il) : batch;  // transforms of this launch
      // KIND_ROWS: TILE / n transforms per workgroup (the final pass's block layout: wave-uniform trivial
      // twiddles, 4-wave workgroups) when the engine has it and the count divides; NTT_ROWS=0: one per
      // workgroup (KIND_SINGLE)
      const unsigned rows_log = (unsigned)tile_log_of<E>() - r[0];
      static const bool rows_env = [] {
        const char* v = getenv("NTT_ROWS");
        return !(v && *v == '0');
      }();
      bool rows = false;
      if constexpr (HasRows<E>::value) {
        bool fast_ok = true;  // the quotient-estimate engines run KIND_ROWS in their FAST form only
        if constexpr (E::FASTRED) fast_ok = Ff.red_ok != 0;
        rows = rows_env && fast_ok && r[0] >= (unsigned)kRowsMinLog && r[0] <= (unsigned)rows_max_log<E>() &&
               rows_log >= 1 && nt >= (1u << rows_log) && (nt & ((1u << rows_log) - 1)) == 0;
      }
      if (rows) {
        if (!il) {  // the transform index is part of every position: extents over the whole batch
          if (A.dbg_src_n != ~(size_t)0) A.dbg_src_n = (size_t)n * batch;
          if (A.dbg_dst_n != ~(size_t)0) A.dbg_dst_n = (size_t)n * batch;
        }
        e = launch_pass<E>(KIND_ROWS, (int)r[0], in, out, A, nt >> rows_log, 1, st);
      } else {
        e = launch_pass<E>(KIND_SINGLE, (int)r[0], in, out, A, 1, nt, st);
      }
      mark(st, rows ? "r" : "s", r[0]);
    } else {
      if (il) batch = 1;  // Mode I: the 2^il interleaved transforms are one long column sweep
      // NTT_PLAN_IN_PLACE (not for four-step pieces, whose passes map positions): every pass reads and
      // writes `out`'s positions, the final pass included; the digit reversal follows as tile swaps
      const bool inplace = (flags & NTT_PLAN_IN_PLACE) && !io;
      uint32_t* work = inplace ? out : d_scratch;
      if (!inplace) {
        if (int rc = ensure_scratch(il ? (1u << il) : batch)) return rc;
        work = d_scratch;
      }
      const uint32_t grid = (uint32_t)((n << il) >> tile_log_of<E>());
      if (use_full)
        if (int rc = ensure_full(inverse ? 1 : 0, st)) return rc;
      const bool full_dir = use_full && d_fulls[inverse ? 1 : 0];  // else: the two-level tables
      // the passes' arguments: column passes 0..npass-2, then the final pass
      PassArgs<E> PA[8];
      unsigned blk = log_n;
      for (unsigned i = 0; i + 1 < npass; ++i) {
        PassArgs<E>& A = PA[i];
        A = base_args(inverse);
        A.tw_int = d_tab + off_int[i];
        A.tw_lo = d_tab + (inverse ? off_los_i : off_los_f);
        A.tw_hi = d_tab + (inverse ? (i == 0 ? off_hi_is : off_hi_i) : off_hi_f);
        // pass 1 of a memory-bound engine (8-B P path) computes its outer twiddles from the
        // L2-resident two-level tables: two 32-bit products are cheaper than streaming an n-entry table
        static const bool p1_full = [] {  // NTT_PASS1_FULL=1: pass 1 streams its table on every engine (A/B)
          const char* v = getenv("NTT_PASS1_FULL");
          return v && atoi(v) > 0;
        }();
        A.tw_full = (full_dir && (i > 0 || E::PASS1_FULL_TABLE || p1_full)) ? d_fulls[inverse ? 1 : 0] + full_off[i] * TABW
                                                                             : nullptr;
        if (d_full_sh && full_sh_ok[i] && (i > 0 || full_dir)) {
          A.tw_full = d_full_sh + full_sh_off[inverse ? 1 : 0][i] * TW;
          A.tw_sh = 1;
        }
        if (i == 0 && in2) {  // the fused prologues bring their own pass-1 tables (w R_e)
          A.src2 = in2;
          A.tw_full = d_full_pm;
          A.tw_sh = 0;
        }
        if (i == 0 && tw_in) {
          A.tw_in = tw_in;
          A.tw_full = full0;
          A.tw_sh = 0;
        }
        A.log_blk = blk + il;
        A.log_m = log_n - blk;
        A.src_user = (i == 0) ? 1u : 0u;
        set_fs(A, i == 0 ? FS_MAP_IN : 0u);
        blk -= r[i];
      }
      PassArgs<E>& A = PA[npass - 1];
      A = base_args(inverse);
      A.tw_int = d_tab + off_int[npass - 1];
      A.r1 = r[0];
      A.nmid = npass - 2;
      // middle digits k_2..k_{p-1}, least significant (k_{p-1}) first
      for (unsigned m = 0; m < A.nmid; ++m) {
        const unsigned idx = npass - 2 - m;  // pass index (0-based) of digit k_{idx+1}
        A.mid_bits[m] = r[idx];
        unsigned off = 0;
        for (unsigned j = 1; j < idx; ++j) off += r[j];
        A.mid_off[m] = off;
      }
      set_fs(A, FS_MAP_OUT);
      if (io) A.tw_epi = static_cast<const uint32_t*>(io->tw_epi);
      if (inplace) A.flags |= 2u;
      for (unsigned i = 0; i < npass; ++i) set_extents(PA[i], io, il);
      // XCD-grouped tile order (k_pass flag bit 2) for the column passes after the first whose runs are
      // shorter than a 128-B line (the 8-B path's 4-B scratch at radix 512: 64-B runs), so that the
      // two tiles sharing each line meet on one XCD's L2.  Passes of one column per tile (radix 4096 on
      // the 4096-element tiles) read and write 32-B runs, their final pass's stores too: every such
      // pass takes the order, so the four tiles of each 128-B line run together.  NTT_XCD_ORDER=0 off,
      // =1 on every column pass, =3 not on the one-column passes (A/B).
      static const int xcd_order = [] {
        const char* v = getenv("NTT_XCD_ORDER");
        return v && *v ? atoi(v) : 2;
      }();
      if (!io && xcd_order > 0)
        for (unsigned i = 0; i < npass; ++i) {
          const unsigned cols = 1u << (tile_log_of<E>() - r[i]);
          const unsigned run_bytes = cols * SCRW * 4;
          const bool column = i + 1 < npass;
          if ((column && (xcd_order == 1 || (i > 0 && run_bytes < 128))) || (cols == 1 && xcd_order != 3))
            PA[i].flags |= 4u;
        }
      if constexpr (fused2_engine<E>()) {  // 2^20 on 4096-element tiles: the two-pass single launch
        if (!io && batch == 1 && npass == 2 && fused_enabled() && fused2_ready(PA, inplace)) {
          FusedArgs F = inplace ? fargs2_ip : fargs2;
          F.wd = watchdog(F.wd.abort);
          F.trace = fused_trace_buffer(F.nwg);
          {
            FusedSerial order(device, st);
            if (inplace) {  // k_fused2bi: residency (barrier 1), pass barrier 2, the final pass's barrier 3
              PassArgs<E> A1 = PA[0];
              A1.ipn_go = F.sync + F.rbase;  // pass 1's stores wait for the residency decision
              A1.wd = F.wd;
              PassArgs<E> B = A;
              B.flags &= ~2u;
              B.ipn_sync = F.sync;
              B.ipn_go = F.sync + F.rbase + 64;
              B.ipn_shards = F.shards;
              B.wd = F.wd;
              e = launch_fused2<E>((int)r[0], (int)r[1], out, nullptr, out, A1, B, F, st);
            } else {
              e = launch_fused2<E>((int)r[0], (int)r[1], in, work, out, PA[0], A, F, st);
            }
            order.done(e);
          }
          mark(st, "b");
          if (F.trace && e == hipSuccess) dump_fused_trace(F, inplace, st);
          return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
        }
      }
      if constexpr (std::is_same_v<E, Eng256>) {  // the engine k_fused3 is instantiated for
        if (!io && !inplace && batch == 1 && fused_enabled() && fused_ready(PA)) {
          // one persistent launch for the three passes (NTT_PLAN_SINGLE_LAUNCH, k_fused3)
          FusedArgs F = fused_args();
          F.wd = watchdog(F.wd.abort);
          {
            FusedSerial order(device, st);
            e = launch_fused3<E>((int)r[0], (int)r[1], (int)r[2], in, work, out, PA[0], PA[1], PA[2], F, st);
            order.done(e);
          }
          mark(st, "b");
          return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
        }
      }
      if constexpr (std::is_same_v<E, Eng256>) {
        if (!io && inplace && batch == 1 && fused_enabled() && fused_ip_ready(PA)) {
          // the in-place single launch (k_fused3bi): three passes in the caller's buffer, no scratch
          FusedArgs F = fargs_ip;
          F.wd = watchdog(F.wd.abort);
          PassArgs<E> A1 = PA[0];
          A1.ipn_go = F.sync + F.rbase;  // pass 1's stores wait for the residency decision (barrier 1)
          A1.wd = F.wd;
          PassArgs<E> B = A;
          B.flags &= ~2u;
          B.ipn_sync = F.sync;
          B.ipn_go = F.sync + F.rbase + 96;  // the fourth barrier's go word
          B.ipn_shards = F.shards;           // its arrival shards (cumulative, like the top counter)
          B.wd = F.wd;
          {
            FusedSerial order(device, st);
            e = launch_fused3<E>((int)r[0], (int)r[1], (int)r[2], out, nullptr, out, A1, PA[1], B, F, st);
            order.done(e);
          }
          mark(st, "b");
          return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
        }
      }
      for (unsigned i = 0; i + 1 < npass && e == hipSuccess; ++i) {
        const uint32_t* src = (i == 0) ? in : work;
        e = launch_pass<E>(KIND_COLUMN, (int)r[i], src, work, PA[i], grid, batch, st);
        mark(st, "c", r[i], PA[i].tw_sh != 0);
      }
      if (e == hipSuccess && inplace && batch == 1 && ipn_ready(A)) {
        // the final pass writes natural positions in place, the digit reversal fused (k_final_ipn)
        PassArgs<E> B = A;
        B.flags &= ~2u;
        B.ipn_sync = d_ipn;
        B.ipn_order = d_ipn + 32 * (2 + ipn_slabs);
        B.ipn_strips = ipn_strips;
        B.wd = watchdog(d_ipn + 32 * (1 + ipn_slabs));
        e = launch_final_ipn<E>((int)r[npass - 1], out, B, grid, st);
        mark(st, "i", r[npass - 1]);
      } else if (e == hipSuccess) {
        e = launch_pass<E>(KIND_FINAL, (int)r[npass - 1], work, out, A, grid, batch, st);
        mark(st, "f", r[npass - 1]);
        if (inplace && e == hipSuccess) {
          DrevArgs D{};
          D.log_n = log_n;
          D.R = r[0];
          D.tb_log = r[0] < 4 ? r[0] : 4;
          D.nmid = A.nmid;
          for (unsigned m = 0; m < A.nmid; ++m) D.mid_bits[m] = A.mid_bits[m], D.mid_off[m] = A.mid_off[m];
          D.batch_stride = (size_t)n * MEMW;
          static const int drev_diag = [] {
            const char* v = getenv("NTT_DREV_DIAG");
            return v ? atoi(v) : 1;
          }();
          D.diag = drev_diag ? 1u : 0u;
          e = launch_digitrev_swap<E>(out, D, batch, st);
          mark(st, "d");
        }
      }
    }
    return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
  }

  // ---- fused single-launch schedule (NTT_PLAN_SINGLE_LAUNCH, k_fused3 in ntt_kernels_impl.hpp)
  uint32_t* d_sync = nullptr;  // FusedArgs::sync words (zeroed at creation; each launch leaves them zeroed)
  FusedArgs fargs{};
  bool fused_built = false, fused_ok = false;
  // NTT_SINGLE_LAUNCH=1 / =0 in the environment forces the schedule on / off for every plan (A/B)
  bool fused_enabled() const {
    static const int env = [] {
      const char* v = getenv("NTT_SINGLE_LAUNCH");
      return v && *v ? atoi(v) : -1;
    }();
    return env >= 0 ? env > 0 : (flags & NTT_PLAN_SINGLE_LAUNCH) != 0;
  }
  // 3-pass FAST 256-bit plans whose passes 1 and 2 take full tables (pass 2: Shoup pairs), and whose
  // radices the fused kernel is instantiated for; built on first use
  bool fused_ready(const PassArgs<E>* PA) {
    if (!fused_built) {
      fused_built = true;
      fused_ok = build_fused();
    }
    return fused_ok && PA[0].tw_full && PA[1].tw_full && PA[1].tw_sh && !PA[0].src2 && !PA[0].tw_in;
  }
  bool build_fused() {
    if constexpr (!std::is_same_v<E, Eng256>) {
      return false;
    } else {
    if (npass != 3 || !use_full || !d_full_sh || !full_sh_ok[1] || !Ff.red_ok) return false;
    if (!alloc_watch()) return false;
    const unsigned tl = tile_log_of<E>();
    // NTT_FUSED_MODE=0: the dataflow form (per-tile hand-offs), =1: the grid-barrier form (default);
    // read when the plan builds its fused schedule (its first single-launch call)
    const char* mv = getenv("NTT_FUSED_MODE");
    const uint32_t mode = (mv && *mv == '0') ? 0u : 1u;
    uint32_t cap = 0;
    if (fused3_capacity<E>((int)r[0], (int)r[1], (int)r[2], device, &cap, mode) != hipSuccess || cap == 0) return false;
    const unsigned r1 = r[0], r2 = r[1], r3 = r[2];
    const unsigned lt1 = tl - r1, lt2 = tl - r2, lt3 = tl - r3, lu = lt1 > lt2 ? lt1 : lt2;
    if (r3 < lu || r1 < lt3) return false;  // schedule_ok guarantees both; kept as the kernel's contract
    FusedArgs F{};
    F.tiles = (uint32_t)(n >> tl);
    F.nwg = F.tiles < cap ? F.tiles : cap;
    F.k1_mask = (1u << (r3 - lt1)) - 1;
    F.k1_shift = lu - lt1;
    F.cg_log = r3 - lt2;
    F.k2_shift = lu - lt2;
    F.t3_log = lt3;
    F.r2 = r2;
    F.n12 = 1u << (r3 - lu);
    F.n23 = 1u << (r1 - lt3);
    F.need12 = 1u << (lu - lt1 + r2);
    F.need23 = 1u << r2;
    F.mode = mode;
    if (getenv("NTT_FUSED_VERBOSE"))
      fprintf(stderr, "libntt: fused schedule mode %u, %u tiles per pass, %u workgroups (capacity %u)\n", mode, F.tiles,
              F.nwg, cap);
    if (const char* v = getenv("NTT_FUSED_DBG")) F.dbg = (uint32_t)atoi(v);
    F.rbase = (4 + F.n12 + F.n23 + 31) & ~31u;
    const size_t words = F.rbase + 32 * (F.n12 + F.n23);  // then the abort word on a line of its own
    // then the abort word and the 8 barrier shards, each on a line of its own
    if (hipMalloc(&d_sync, (words + 32 * 9) * 4) != hipSuccess) {
      d_sync = nullptr;
      return false;
    }
    if (hipMemset(d_sync, 0, (words + 32 * 9) * 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return false;
    F.sync = d_sync;
    F.wd.abort = d_sync + words;
    F.shards = d_sync + words + 32;
    fargs = F;
    return true;
    }
  }
  const FusedArgs& fused_args() const { return fargs; }

  // ---- the two-pass single launch on 4096-element tiles (NTT_PLAN_SINGLE_LAUNCH, 2^20 4-limb plans:
  // k_fused2b, and k_fused2bi in place; ntt_kernels_impl.hpp).  Plain launches of at most the occupancy
  // query's workgroups; the in-place form needs every one of the 256 final tiles resident.
  // Sync words: [0] top arrivals, [1] exits; go words at 32, 64, 96 (in place: residency, pass barrier,
  // final barrier); abort at 128; shards at 160 + 32 s.
  uint32_t* d_sync2 = nullptr;
  FusedArgs fargs2{}, fargs2_ip{};
  int fused2_state[2] = {0, 0};  // [in place]: 0 not built, 1 ready, -1 unavailable
  bool fused2_ready(const PassArgs<E>* PA, bool inplace) {
    int& st = fused2_state[inplace ? 1 : 0];
    if (st == 0) st = build_fused2(inplace) ? 1 : -1;
    return st > 0 && PA[0].tw_full && !PA[0].tw_sh && !PA[0].src2 && !PA[0].tw_in;
  }
  bool build_fused2(bool inplace) {
    if constexpr (!fused2_engine<E>()) {
      return false;
    } else {
      if (npass != 2 || r[0] != 10 || r[1] != 10 || !use_full || !Ff.red_ok) return false;
      if (!alloc_watch()) return false;
      const uint32_t tiles = (uint32_t)(n >> tile_log_of<E>()), mode = inplace ? 4u : 3u;
      uint32_t cap = 0;
      if (fused2_capacity<E>((int)r[0], (int)r[1], device, &cap, mode) != hipSuccess || cap == 0) return false;
      if (inplace && cap < tiles) return false;
      if (!d_sync2) {
        if (hipMalloc(&d_sync2, 416 * 4) != hipSuccess) {
          d_sync2 = nullptr;
          (void)hipGetLastError();
          return false;
        }
        if (hipMemset(d_sync2, 0, 416 * 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return false;
      }
      FusedArgs F{};
      F.tiles = tiles;
      F.nwg = inplace ? tiles : (tiles < cap ? tiles : cap);
      F.mode = mode;
      F.rbase = 32;
      F.sync = d_sync2;
      F.wd.abort = d_sync2 + 128;
      F.shards = d_sync2 + 160;
      if (getenv("NTT_FUSED_VERBOSE"))
        fprintf(stderr, "libntt: two-pass single launch (mode %u), %u tiles per pass, %u workgroups (capacity %u)\n",
                mode, tiles, F.nwg, cap);
      (inplace ? fargs2_ip : fargs2) = F;
      return true;
    }
  }
  // NTT_FUSED_TRACE (diagnostics): the stamps buffer, and its dump after the call
  unsigned long long* d_trace = nullptr;
  unsigned long long* fused_trace_buffer(uint32_t nwg) {
    if (!fused_trace_path()) return nullptr;
    if (!d_trace && hipMalloc(&d_trace, (size_t)4 * 8 * 1024) != hipSuccess) {
      d_trace = nullptr;
      (void)hipGetLastError();
    }
    return (d_trace && nwg <= 1024) ? d_trace : nullptr;
  }
  void dump_fused_trace(const FusedArgs& F, bool inplace, hipStream_t st) {
    std::vector<unsigned long long> h((size_t)4 * F.nwg);
    if (hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(h.data(), F.trace, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
      return;
    if (FILE* f = fopen(fused_trace_path(), "a")) {
      fprintf(f, "{\"kernel\": \"%s\", \"log_n\": %u, \"nwg\": %u, \"stamps\": [", inplace ? "k_fused2bi" : "k_fused2b",
              log_n, F.nwg);
      for (size_t i = 0; i < h.size(); ++i) fprintf(f, "%s%llu", i ? ", " : "", h[i]);
      fprintf(f, "]}\n");
      fclose(f);
    }
  }
  bool single_launch_ready() override {
    if constexpr (!fused2_engine<E>()) {
      return false;
    } else {
      const bool inplace = (flags & NTT_PLAN_IN_PLACE) != 0;
      if (ensure_full(0, nullptr) != NTT_OK || !d_fulls[0]) return false;
      int& st = fused2_state[inplace ? 1 : 0];
      if (st == 0) st = build_fused2(inplace) ? 1 : -1;
      return st > 0;
    }
  }

  // ---- the in-place single launch (NTT_PLAN_SINGLE_LAUNCH on an NTT_PLAN_IN_PLACE plan, k_fused3bi):
  // 3-pass palindromic FAST 256-bit schedules whose tiles all fit the device at once (2^18 .. 2^20)
  uint32_t* d_sync_ip = nullptr;  // [0] top arrivals, [1] exits; go words at 32 (residency), 64, 96, 128; abort at 160; shards at 192
  FusedArgs fargs_ip{};
  bool fused_ip_built = false, fused_ip_ok = false;
  bool fused_ip_ready(const PassArgs<E>* PA) {
    if (!fused_ip_built) {
      fused_ip_built = true;
      fused_ip_ok = build_fused_ip();
    }
    return fused_ip_ok && PA[0].tw_full && PA[1].tw_full && PA[1].tw_sh && !PA[0].src2 && !PA[0].tw_in;
  }
  bool build_fused_ip() {
    if constexpr (!std::is_same_v<E, Eng256>) {
      return false;
    } else {
      if (npass != 3 || r[0] != r[2] || !use_full || !d_full_sh || !full_sh_ok[1] || !Ff.red_ok) return false;
      if (!alloc_watch()) return false;
      const uint32_t tiles = (uint32_t)(n >> tile_log_of<E>());
      uint32_t cap = 0;
      if (fused3_capacity<E>((int)r[0], (int)r[1], (int)r[2], device, &cap, 2) != hipSuccess || cap < tiles) return false;
      FusedArgs F{};
      F.tiles = F.nwg = tiles;
      F.mode = 2;
      F.rbase = 32;
      if (const char* v = getenv("NTT_FUSED_VERBOSE"))
        fprintf(stderr, "libntt: in-place single launch, %u tiles per pass, %u workgroups (capacity %u)\n", tiles,
                tiles, cap);
      // go words at 32 (residency), 64, 96, 128; abort at 160; barrier shards at 192 + 32 s
      if (hipMalloc(&d_sync_ip, 448 * 4) != hipSuccess) {
        d_sync_ip = nullptr;
        return false;
      }
      if (hipMemset(d_sync_ip, 0, 448 * 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return false;
      F.sync = d_sync_ip;
      F.wd.abort = d_sync_ip + 160;
      F.shards = d_sync_ip + 192;
      fargs_ip = F;
      return true;
    }
  }
  // bit 0: a bounded wait gave up (the watchdog report, PlanBase::h_watch); then cleared.  Blocking:
  // the device is synchronised first, so the report covers every call enqueued before.
  int device_status(unsigned* bad) override {
    *bad = 0;
    if (hipDeviceSynchronize() != hipSuccess) return NTT_ERR_HIP;
    if (tripped()) *bad |= 1u;
    clear_trip();
    if (d_dbg) {  // debug builds: NTT_DBG_* bits (engines.hpp)
      uint32_t w = 0;
      if (hipMemcpy(&w, d_dbg, 4, hipMemcpyDeviceToHost) != hipSuccess) return NTT_ERR_HIP;
      if (w && hipMemset(d_dbg, 0, 4) != hipSuccess) return NTT_ERR_HIP;
      *bad |= w;
    }
    return NTT_OK;
  }
  uint32_t* d_dbg = nullptr;  // debug builds (NTT_DEBUG_CHECKS): the kernels' check-failure bits

  // ---- in-place final pass with the fused digit reversal (NTT_PLAN_IN_PLACE, k_final_ipn)
  uint32_t* d_ipn = nullptr;  // 32 (1 + slabs) sync words, then the slab order table
  uint32_t ipn_slabs = 0, ipn_strips = 0;
  bool ipn_built = false, ipn_ok = false;
  // NTT_IPN=0 in the environment keeps the separate tile-swap pass (A/B)
  bool ipn_ready(const PassArgs<E>& A) {
    if (!ipn_built) {
      ipn_built = true;
      const char* v = getenv("NTT_IPN");
      ipn_ok = !(v && v[0] == '0') && build_ipn(A);
    }
    return ipn_ok;
  }
  bool build_ipn(const PassArgs<E>& A) {
    const unsigned tl = tile_log_of<E>(), rp = r[npass - 1];
    if (npass < 2 || r[0] != rp || rp > 9 || tl < rp) return false;
    if (!alloc_watch()) return false;
    const unsigned mid_log = log_n - r[0] - rp;
    ipn_slabs = 1u << mid_log;
    ipn_strips = 1u << (r[0] - (tl - rp));  // R_1 / T, T = TILE / R_p
    // the deadlock-freedom argument of k_final_ipn needs a slab pair's tiles resident together: at
    // most 128 per pair, and no more than the device keeps resident
    if (r[0] < tl - rp || 2 * ipn_strips > 128) return false;
    if (launch_final_ipn_capacity<E>((int)rp, device) < 2 * ipn_strips) return false;
    // slab order: m, then its mirror (the final pass's middle-digit reversal, as k_pass computes it)
    std::vector<uint32_t> order, seen(ipn_slabs, 0);
    auto rev = [&](uint32_t m) {
      uint32_t out = 0;
      for (unsigned i = 0; i < A.nmid; ++i) {
        out |= (m & ((1u << A.mid_bits[i]) - 1)) << A.mid_off[i];
        m >>= A.mid_bits[i];
      }
      return out;
    };
    for (uint32_t m = 0; m < ipn_slabs; ++m) {
      if (seen[m]) continue;
      const uint32_t q = rev(m);
      if (q >= ipn_slabs || rev(q) != m) return false;  // the schedule is not palindromic
      order.push_back(m);
      seen[m] = 1;
      if (q != m) {
        order.push_back(q);
        seen[q] = 1;
      }
    }
    const size_t sync_words = 32 * (2 + (size_t)ipn_slabs);  // line 0, one line per slab, the abort line
    if (hipMalloc(&d_ipn, (sync_words + order.size()) * 4) != hipSuccess) {
      d_ipn = nullptr;
      return false;
    }
    if (hipMemset(d_ipn, 0, sync_words * 4) != hipSuccess ||
        hipMemcpy(d_ipn + sync_words, order.data(), order.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess)
      return false;
    return true;
  }

  // ---- distributed four-step pieces (ntt_rplan, ntt_amd/csrc/ntt_rplan.cpp)
  int run_fs(const void* in, const void* in2, void* out, unsigned batch, bool inverse, const FsIO& io,
             hipStream_t st) override {
    if (!in || !out || batch == 0 || (flags & NTT_PLAN_TWIDDLE_ONLY)) return NTT_ERR_ARG;
    auto pin = static_cast<const uint32_t*>(in);
    auto pout = static_cast<uint32_t*>(out);
    if (!in2) return run_io(pin, nullptr, pout, batch, inverse, st, nullptr, nullptr, &io);
    if (!inverse) return NTT_ERR_ARG;  // the product is taken at the inverse's load
    const size_t count = (size_t)n * ((io.fs & FS_IL) ? (1ull << io.il) : batch);
    if (polymul_fusable() && npass >= 2) {  // in2 read through the input map like in
      if (int rc = ensure_polymul_table(st)) return rc;
      return run_io(pin, static_cast<const uint32_t*>(in2), pout, batch, true, st, nullptr, nullptr, &io);
    }
    if (!(io.fs & (FS_MAP_IN | FS_MAP_OUT))) {  // same layout in and out: the product in place in out
      if (int rc = pointwise_n(pin, static_cast<const uint32_t*>(in2), pout, count, st)) return rc;
      return run_io(pout, nullptr, pout, batch, true, st, nullptr, nullptr, &io);
    }
    // a mapped piece (the column pieces of ntt_rplan_inverse_cols_piece): the product gathered into a
    // plan-owned buffer first (out's other pieces may still be in flight)
    if (count > pw_elems) {
      if (d_pw) (void)hipFree(d_pw);
      d_pw = nullptr;
      pw_elems = 0;
      if (hipMalloc(&d_pw, count * MEMW * 4) != hipSuccess) return NTT_ERR_HIP;
      pw_elems = count;
    }
    const size_t off = (flags & NTT_PLAN_MONTGOMERY_IO) ? off_rm : off_r2;
    if (launch_pointwise<E>(pin, static_cast<const uint32_t*>(in2), d_pw, count, Ff, d_tab + off, st,
                            (io.fs & FS_MAP_IN) ? &io.min : nullptr) != hipSuccess)
      return NTT_ERR_HIP;
    FsIO io2 = io;
    io2.fs &= ~FS_MAP_IN;
    return run_io(d_pw, nullptr, pout, batch, true, st, nullptr, nullptr, &io2);
  }
  uint32_t* d_pw = nullptr;  // gathered pointwise products of mapped pieces (run_fs), on first use
  size_t pw_elems = 0;

  // scale_log k > 0: every entry also carries 2^-k (the four-step's row n2^-1, folded into the inverse
  // columns' epilogue so that the single-pass inverse rows need no scaling product)
  int build_fs_table(void* table, unsigned log_rows, unsigned log_cols, uint64_t row0, uint64_t col0, bool inverse,
                     unsigned scale_log, hipStream_t st) override {
    if (!table || log_rows + log_cols > 40 || scale_log > log_n) return NTT_ERR_ARG;
    const uint32_t* lo = d_tab + (inverse ? off_los_i : off_los_f);
    const uint32_t* hi = d_tab + (inverse ? off_hi_i : off_hi_f);
    const uint32_t* scale = scale_log ? d_tab + off_pow2inv + (size_t)scale_log * TW : nullptr;
    return launch_build_fs_tw<E>(static_cast<uint32_t*>(table), log_rows, log_cols, row0, col0, log_n, lo, hi,
                                 lo_bits, inverse ? Fi : Ff, st, scale) == hipSuccess
               ? NTT_OK
               : NTT_ERR_HIP;
  }

  size_t table_entry_bytes() const override { return (size_t)TABW * 4; }

  // Fused polymul is available for multi-pass FAST plans with full outer-twiddle tables.
  bool polymul_fusable() const {
    if constexpr (!E::FASTRED) {
      return false;
    } else {
      return use_full && npass >= 2 && Fi.red_ok && !(flags & NTT_PLAN_MONTGOMERY_IO);
    }
  }
  // Inverse pass-1 outer-twiddle table scaled by n^-1 R_e (built on first use, same layout as d_full).
  // Built on the call's stream ahead of the passes that read it (no device-wide synchronisation).
  int ensure_polymul_table(hipStream_t st) {
    if (d_full_pm) return NTT_OK;
    const size_t elems = 1ull << log_n;
    if (hipMalloc(&d_full_pm, elems * TABW * 4) != hipSuccess) {
      d_full_pm = nullptr;
      return NTT_ERR_HIP;
    }
    if (launch_build_tw<E>(d_full_pm, elems, r[0], tile_log_of<E>() - r[0], 0, d_tab + off_los_i,
                           d_tab + off_hi_ipm, lo_bits, Fi, st) != hipSuccess) {
      (void)hipFree(d_full_pm);  // never leave a partly built table behind as if it were built
      d_full_pm = nullptr;
      return NTT_ERR_HIP;
    }
    return NTT_OK;
  }

  // c = a * b (cyclic convolution of length n): forward(a), forward(b) in place, then the inverse of
  // their pointwise product into c.  Fused: the inverse's first pass reads both transforms and
  // multiplies at load (one HBM pass and one kernel fewer than forward / pointwise / inverse).
  int polymul(void* a, void* b, void* c, hipStream_t st) override {
    if (!a || !b || !c || (flags & NTT_PLAN_TWIDDLE_ONLY)) return NTT_ERR_ARG;
    uint32_t *pa = static_cast<uint32_t*>(a), *pb = static_cast<uint32_t*>(b);
    if (int rc = run_io(pa, nullptr, pa, 1, false, st)) return rc;
    if (pb != pa)  // squaring (a == b): one forward transform, then the product of it with itself
      if (int rc = run_io(pb, nullptr, pb, 1, false, st)) return rc;
    return inverse_pointwise(pa, pb, c, 1, st);
  }

  // c = INTT(a * b) over `batch` transforms (the polymul's second half; a, b forward transforms).
  // Fused: the inverse's first pass reads both transforms and multiplies at load (one HBM pass and
  // one kernel fewer than pointwise + inverse).  c may alias a or b.
  int inverse_pointwise(const void* a, const void* b, void* c, unsigned batch, hipStream_t st) override {
    if (!a || !b || !c || batch == 0 || (flags & NTT_PLAN_TWIDDLE_ONLY)) return NTT_ERR_ARG;
    auto pa = static_cast<const uint32_t*>(a), pb = static_cast<const uint32_t*>(b);
    auto pc = static_cast<uint32_t*>(c);
    if (polymul_fusable()) {
      if (int rc = ensure_polymul_table(st)) return rc;
      return run_io(pa, pb, pc, batch, true, st);
    }
    if (int rc = pointwise_n(pa, pb, pc, (size_t)n * batch, st)) return rc;
    return run_io(pc, nullptr, pc, batch, true, st);
  }

  int pointwise_n(const uint32_t* a, const uint32_t* b, uint32_t* c, size_t count, hipStream_t st) {
    const size_t off = (flags & NTT_PLAN_MONTGOMERY_IO) ? off_rm : off_r2;
    return launch_pointwise<E>(a, b, c, count, Ff, d_tab + off, st) == hipSuccess ? NTT_OK : NTT_ERR_HIP;
  }

  int pointwise(const void* a, const void* b, void* c, hipStream_t st) override {
    if (!a || !b || !c) return NTT_ERR_ARG;
    return pointwise_n(static_cast<const uint32_t*>(a), static_cast<const uint32_t*>(b), static_cast<uint32_t*>(c), n,
                       st);
  }

  int fill(void* d, uint64_t count, int kind, uint64_t seed, uint64_t row0, unsigned log_inner, unsigned log_stride,
           hipStream_t st) override {
    if (!d || (kind != 0 && kind != 1)) return NTT_ERR_ARG;
    hipError_t e = launch_fill<E>(kind, static_cast<uint32_t*>(d), count, seed, nrand, top_bits, row0, log_inner,
                                  log_stride, st);
    return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
  }

  int twiddle_pack(const void* src, void* dst, unsigned log_rows, unsigned log_len, unsigned log_bw, uint64_t row0,
                   bool inverse, uint64_t peer_stride, hipStream_t st) override {
    if (!src || !dst || src == dst || log_bw > log_len || log_rows + log_len > 40) return NTT_ERR_ARG;
    if (peer_stride < (1ull << (log_rows + log_bw))) return NTT_ERR_ARG;  // peer chunks must not overlap
    const uint32_t* lo = d_tab + (inverse ? off_los_i : off_los_f);
    const uint32_t* hi = d_tab + (inverse ? off_hi_i : off_hi_f);
    hipError_t e = launch_twiddle_pack<E>(static_cast<const uint32_t*>(src), static_cast<uint32_t*>(dst), log_rows,
                                          log_len, log_bw, row0, log_n, lo, hi, lo_bits, inverse ? Fi : Ff,
                                          peer_stride, st);
    return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
  }

  int transpose(const void* src, void* dst, unsigned log_rows, unsigned log_cols, unsigned log_blk_rows,
                uint64_t blk_stride, hipStream_t st) override {
    if (!src || !dst || src == dst || log_rows + log_cols > 40 || log_blk_rows > log_rows) return NTT_ERR_ARG;
    if (blk_stride < (1ull << (log_blk_rows + log_cols))) return NTT_ERR_ARG;
    hipError_t e = launch_transpose<E>(static_cast<const uint32_t*>(src), static_cast<uint32_t*>(dst), log_rows,
                                       log_cols, log_blk_rows, blk_stride, st);
    return e == hipSuccess ? NTT_OK : NTT_ERR_HIP;
  }
};

// ------------------------------------------------------------------------------ built-in fields
struct FieldDef {
  uint64_t p[4];
  uint64_t g;
};
static const FieldDef kFields[3] = {
    {{469762049ull, 0, 0, 0}, 3},
    {{0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull}, 5},
    {{0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull, 0x73eda753299d7d48ull}, 7},
};

static int make_plan(std::unique_ptr<PlanBase>& out, const uint64_t* p64, const uint64_t* g64, unsigned limbs64,
                     unsigned log_n, int device, unsigned flags) {
  if (log_n > 40) return NTT_ERR_ARG;
  if (limbs64 != 1 && limbs64 != 4 && limbs64 != 6) return NTT_ERR_ARG;  // before packing into p32[12] / g32[12]
  const unsigned rivals = flags & (NTT_PLAN_STOCKHAM | NTT_PLAN_GZKP | NTT_PLAN_NAIVE | NTT_PLAN_NO_SWAP | kBealtoFlags);
  if (rivals & (rivals - 1)) return NTT_ERR_ARG;  // one rival schedule per plan
  if ((flags & NTT_PLAN_IN_PLACE) && (rivals || (flags & NTT_PLAN_TWIDDLE_ONLY)))
    return NTT_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return NTT_ERR_NODEV;
  if (device < 0 || device >= ndev) return NTT_ERR_ARG;
  uint32_t p32[12] = {0}, g32[12] = {0};
  for (unsigned i = 0; i < limbs64; ++i) {
    p32[2 * i] = (uint32_t)p64[i];
    p32[2 * i + 1] = (uint32_t)(p64[i] >> 32);
    g32[2 * i] = (uint32_t)g64[i];
    g32[2 * i + 1] = (uint32_t)(g64[i] >> 32);
  }
  int rc;
  if (limbs64 == 1) {
    if (p64[0] >= (1ull << 31)) return NTT_ERR_FIELD;  // `long long` path: 31-bit primes
    if (flags & NTT_PLAN_IN_PLACE) {  // in place needs 8-B scratch elements (the caller's layout)
      auto impl = std::make_unique<PlanImpl<EngPI>>();
      rc = impl->init(p32, g32, log_n, device, flags);
      out = std::move(impl);
    } else {
      auto impl = std::make_unique<PlanImpl<EngP>>();
      rc = impl->init(p32, g32, log_n, device, flags);
      out = std::move(impl);
    }
  } else if (limbs64 == 4) {
    auto impl = std::make_unique<PlanImpl<Eng256>>();
    rc = impl->init(p32, g32, log_n, device, flags);
    out = std::move(impl);
  } else if (limbs64 == 6) {
    // the 384-bit element layout: 256-bit arithmetic when the modulus allows it (BN254 Fr,
    // BLS12-381 Fr: the upper two 64-bit limbs of every element are zero), 14 limbs otherwise
    if (p64[4] == 0 && p64[5] == 0 && (p64[3] >> 63) == 0 && (flags & NTT_PLAN_IN_PLACE)) {
      // in place: the intermediates live in the caller's 48-B elements (no 32-B plan scratch)
      auto impl = std::make_unique<PlanImpl<Eng256wI>>();
      rc = impl->init(p32, g32, log_n, device, flags);
      out = std::move(impl);
    } else if (p64[4] == 0 && p64[5] == 0 && (p64[3] >> 63) == 0) {
      auto impl = std::make_unique<PlanImpl<Eng256w>>();
      rc = impl->init(p32, g32, log_n, device, flags);
      out = std::move(impl);
    } else {
      auto impl = std::make_unique<PlanImpl<Eng384>>();
      rc = impl->init(p32, g32, log_n, device, flags);
      out = std::move(impl);
    }
  } else {
    return NTT_ERR_ARG;
  }
  if (rc != NTT_OK) out.reset();
  return rc;
}

// BASELINE config 2 (2^20, 4 x 64-bit limbs): a single transform runs fastest on 4096-element tiles,
// one 1024-thread workgroup per CU, in two passes (10 + 10) instead of three (7 + 7 + 6): 0.105
// against 0.114 ms (BN254), 0.102 against 0.108 (BLS12-381), DESIGN §4.  Batched calls keep the
// 1024-element tiles, which overlap the batch's transforms better (batch 4: 0.082 against 0.091 ms
// per transform).  So a default 4-limb plan of 2^20 holds a second plan of 4096-element tiles for
// one vector's transforms (forward, inverse, coset, polymul).  Environment NTT_WIDE_TILES=0: none.
static bool wide_tiles_enabled() {
  static const bool on = [] {
    const char* v = getenv("NTT_WIDE_TILES");
    return !(v && *v == '0');
  }();
  return on;
}

// The second plan is an optimisation: when it cannot be built the plan runs alone, and nothing of the
// failure may leak into the plan's calls.  A failed hipMalloc inside its init leaves the error as the
// thread's last HIP error, which the next launch check (hipGetLastError) would return as NTT_ERR_HIP
// from a healthy plan, so it is cleared here.  It is not attempted at all when the
// device is short of memory (its scratch and tables take ~100 MiB at 2^20).  In the checked build
// (NTT_DEBUG_CHECKS, libntt_debug.so) only, NTT_TEST_WIDE_FAIL=1 makes the attempt fail through a
// refused allocation (tests/test_gpu_wide_tiles.py); the product build has no such hook.
static constexpr size_t kWideMinFreeBytes = 512ull << 20;
// NTT_PLAN_SINGLE_LAUNCH plans (BASELINE config 2's "single-kernel" form) get the second plan too:
// their batch-1 transforms are then ONE launch of the two passes (k_fused2b; in place k_fused2bi),
// and the second plan is kept only if that single launch is available (single_launch_ready).  An
// in-place single-launch plan sends only its plain forward / inverse there (wide_transforms_only).
static bool wide_flags_ok(unsigned flags) {
  const unsigned f = flags & ~NTT_PLAN_MONTGOMERY_IO;
  return f == 0 || f == NTT_PLAN_SINGLE_LAUNCH || f == (NTT_PLAN_SINGLE_LAUNCH | NTT_PLAN_IN_PLACE);
}
// 2^24 (the headline) on the same tiles in two passes, 12 + 12 with one column per column-pass tile:
// one HBM round trip of the vector fewer than 8 + 8 + 8 on the 1024-element tiles.
// NTT_TWO_PASS_24=1 routes a default 2^24 4-limb plan's single-vector transforms there.
static bool two_pass_24_enabled() {
  static const bool on = [] {
    const char* v = getenv("NTT_TWO_PASS_24");
    return v && *v == '1';
  }();
  return on;
}
static void make_wide_plan(std::unique_ptr<PlanBase>& out, const uint64_t* p64, const uint64_t* g64,
                           unsigned limbs64, unsigned log_n, int device, unsigned flags) {
  if (limbs64 != 4 || !wide_flags_ok(flags) || !wide_tiles_enabled()) return;
  if (log_n == 24) {
    if (!two_pass_24_enabled() || (flags & ~NTT_PLAN_MONTGOMERY_IO)) return;
  } else if (log_n != 20) {
    return;
  }
  if ((flags & NTT_PLAN_IN_PLACE) && (flags & NTT_PLAN_MONTGOMERY_IO)) return;
  uint32_t p32[12] = {0}, g32[12] = {0};
  for (unsigned i = 0; i < 4; ++i) {
    p32[2 * i] = (uint32_t)p64[i];
    p32[2 * i + 1] = (uint32_t)(p64[i] >> 32);
    g32[2 * i] = (uint32_t)g64[i];
    g32[2 * i + 1] = (uint32_t)(g64[i] >> 32);
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != device) (void)hipSetDevice(device);
  size_t free_b = 0, total_b = 0;
  const bool room = hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b >= kWideMinFreeBytes;
  if (room) {
#if NTT_DEBUG_CHECKS
    const char* tf = getenv("NTT_TEST_WIDE_FAIL");
    const bool refuse = tf && tf[0] == '1';
#else
    constexpr bool refuse = false;
#endif
    if (refuse) {
      void* p = nullptr;
      if (hipMalloc(&p, ~(size_t)0 >> 4) == hipSuccess) (void)hipFree(p);  // refused: the sticky error
    } else {
      auto impl = std::make_unique<PlanImpl<Eng256T>>();
      if (impl->init(p32, g32, log_n, device, flags) == NTT_OK &&
          (!(flags & NTT_PLAN_SINGLE_LAUNCH) || impl->single_launch_ready()))
        out = std::move(impl);
    }
  }
  if (!out) (void)hipGetLastError();  // the plan runs alone, with a clean error state
  if (cur != device) (void)hipSetDevice(cur);
}

static int set_err(int rc) {
  g_last_error = rc;
  return rc;
}

}  // namespace

struct ntt_plan {
  std::unique_ptr<PlanBase> impl;
  std::unique_ptr<PlanBase> wide;  // one vector's transforms of a 2^20 4-limb plan (make_wide_plan)
  PlanBase* last = nullptr;        // the plan that ran the latest transform (ntt_plan_last_launch_ms)
  // In-place single-launch plans: the second plan runs the plain forward / inverse only (its
  // k_fused2bi); polymul, cosets and the fused pointwise inverse stay on the 1024-element tiles.
  bool wide_transforms_only() const {
    return wide && (wide->flags & NTT_PLAN_IN_PLACE) && (wide->flags & NTT_PLAN_SINGLE_LAUNCH);
  }
  // The plan that transforms `batch` vectors (plain forward / inverse: transform = true), remembered
  // for the profiling readers.
  PlanBase& exec(unsigned batch, bool transform = false) {
    last = (wide && batch == 1 && (transform || !wide_transforms_only())) ? wide.get() : impl.get();
    return *last;
  }
};

extern "C" {

static int create_plan(ntt_plan** out, const uint64_t* modulus, const uint64_t* generator, unsigned limbs64,
                       unsigned log_n, int device, unsigned flags, bool allow_wide) {
  if (!out || !modulus || !generator) return set_err(NTT_ERR_ARG);
  *out = nullptr;
  std::unique_ptr<PlanBase> impl;
  int rc = make_plan(impl, modulus, generator, limbs64, log_n, device, flags);
  if (rc != NTT_OK) return set_err(rc);
  std::unique_ptr<PlanBase> wide;
  if (allow_wide) make_wide_plan(wide, modulus, generator, limbs64, log_n, device, flags);
  *out = new ntt_plan{std::move(impl), std::move(wide)};
  return set_err(NTT_OK);
}

int ntt_plan_create_custom_ex(ntt_plan** out, const uint64_t* modulus, const uint64_t* generator, unsigned limbs64,
                              unsigned log_n, int device, unsigned flags) {
  return create_plan(out, modulus, generator, limbs64, log_n, device, flags, true);
}

int ntt_plan_create_custom(ntt_plan** out, const uint64_t* modulus, const uint64_t* generator, unsigned limbs64,
                           unsigned log_n, int device) {
  return ntt_plan_create_custom_ex(out, modulus, generator, limbs64, log_n, device, 0);
}

int ntt_plan_create(ntt_plan** out, int field_id, unsigned log_n, unsigned limbs64, int device) {
  return ntt_plan_create_ex(out, field_id, log_n, limbs64, device, 0);
}

static int create_field_plan(ntt_plan** out, int field_id, unsigned log_n, unsigned limbs64, int device,
                             unsigned flags, bool allow_wide) {
  if (field_id < 0 || field_id > 2) return set_err(NTT_ERR_ARG);
  if (limbs64 != 1 && limbs64 != 4 && limbs64 != 6) return set_err(NTT_ERR_ARG);
  if (limbs64 == 1 && field_id != NTT_FIELD_P469762049) return set_err(NTT_ERR_ARG);
  const FieldDef& F = kFields[field_id];
  uint64_t p[6] = {0}, g[6] = {0};
  for (unsigned i = 0; i < limbs64 && i < 4; ++i) p[i] = F.p[i];
  g[0] = F.g;
  return create_plan(out, p, g, limbs64, log_n, device, flags, allow_wide);
}

int ntt_plan_create_ex(ntt_plan** out, int field_id, unsigned log_n, unsigned limbs64, int device, unsigned flags) {
  return create_field_plan(out, field_id, log_n, limbs64, device, flags, true);
}

// Every entry point that launches work runs it on the plan's device (saved and restored around
// the call), so a caller whose current device differs still gets the right one.  A plan whose
// watchdog has tripped (PlanBase::h_watch) refuses work with NTT_ERR_DEVICE until
// ntt_plan_device_status clears the report.
extern "C++" template <class F>
static int on_device(ntt_plan* plan, F&& f, bool check_watchdog = true) {
  if (!plan || !plan->impl) return set_err(NTT_ERR_ARG);
  if (check_watchdog && (plan->impl->tripped() || (plan->wide && plan->wide->tripped())))
    return set_err(NTT_ERR_DEVICE);
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != plan->impl->device) (void)hipSetDevice(plan->impl->device);
  const int rc = f(*plan->impl);
  if (cur != plan->impl->device) (void)hipSetDevice(cur);
  return set_err(rc);
}

extern "C++" inline hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }

int ntt_forward(ntt_plan* plan, void* d, void* s) {
  return on_device(plan, [&](PlanBase&) { return plan->exec(1, true).run(d, 1, false, S(s)); });
}
int ntt_inverse(ntt_plan* plan, void* d, void* s) {
  return on_device(plan, [&](PlanBase&) { return plan->exec(1, true).run(d, 1, true, S(s)); });
}
int ntt_forward_batch(ntt_plan* plan, void* d, unsigned b, void* s) {
  return on_device(plan, [&](PlanBase&) { return plan->exec(b, true).run(d, b, false, S(s)); });
}
int ntt_inverse_batch(ntt_plan* plan, void* d, unsigned b, void* s) {
  return on_device(plan, [&](PlanBase&) { return plan->exec(b, true).run(d, b, true, S(s)); });
}

static int run_coset(ntt_plan* plan, void* d, const uint64_t* shift, bool inv, void* s) {
  return on_device(plan, [&](PlanBase&) {
    PlanBase& P = plan->exec(1);
    const unsigned limbs64 = P.elem_bytes >= 32 ? P.elem_bytes / 8 : 1;
    return P.coset(d, shift, limbs64, inv, S(s));
  });
}
int ntt_forward_coset(ntt_plan* plan, void* d, const uint64_t* shift, void* s) { return run_coset(plan, d, shift, false, s); }
int ntt_inverse_coset(ntt_plan* plan, void* d, const uint64_t* shift, void* s) { return run_coset(plan, d, shift, true, s); }

int ntt_pointwise_mul(ntt_plan* plan, const void* a, const void* b, void* c, void* s) {
  return on_device(plan, [&](PlanBase& P) { return P.pointwise(a, b, c, S(s)); });
}

int ntt_count_noncanonical(ntt_plan* plan, const void* d, uint64_t count, uint64_t* bad, void* s) {
  return on_device(plan, [&](PlanBase& P) { return P.count_noncanonical(d, count, bad, S(s)); });
}

int ntt_plan_device_status(ntt_plan* plan, unsigned* bad) {
  if (!bad) return set_err(NTT_ERR_ARG);
  return on_device(plan, [&](PlanBase& P) {
    int rc = P.device_status(bad);
    unsigned b2 = 0;
    if (rc == NTT_OK && plan->wide && (rc = plan->wide->device_status(&b2)) == NTT_OK) *bad |= b2;
    return rc;
  }, false);
}

int ntt_plan_set_watchdog(ntt_plan* plan, unsigned spins) {
  if (!plan || !plan->impl) return set_err(NTT_ERR_ARG);
  plan->impl->wd_spins = spins;
  if (plan->wide) plan->wide->wd_spins = spins;
  return set_err(NTT_OK);
}

int ntt_polymul(ntt_plan* plan, void* a, void* b, void* c, void* s) {
  return on_device(plan, [&](PlanBase&) { return plan->exec(1).polymul(a, b, c, S(s)); });
}

int ntt_inverse_pointwise_batch(ntt_plan* plan, const void* a, const void* b, void* c, unsigned batch, void* s) {
  return on_device(plan, [&](PlanBase&) { return plan->exec(batch).inverse_pointwise(a, b, c, batch, S(s)); });
}

int ntt_fill(ntt_plan* plan, void* d, int kind, uint64_t seed, void* s) {
  return on_device(plan, [&](PlanBase& P) { return P.fill(d, P.n, kind, seed, 0, 64, 0, S(s)); });
}

int ntt_fill_map(ntt_plan* plan, void* d, uint64_t count, int kind, uint64_t seed, uint64_t row0, unsigned log_inner,
                 unsigned log_stride, void* s) {
  return on_device(plan, [&](PlanBase& P) { return P.fill(d, count, kind, seed, row0, log_inner, log_stride, S(s)); });
}

int ntt_twiddle_pack(ntt_plan* plan, const void* src, void* dst, unsigned log_rows, unsigned log_row_len,
                     unsigned log_block, uint64_t row0, int inverse, void* s) {
  return ntt_twiddle_pack_ex(plan, src, dst, log_rows, log_row_len, log_block, row0, inverse,
                             1ull << (log_rows + log_block), s);
}

int ntt_twiddle_pack_ex(ntt_plan* plan, const void* src, void* dst, unsigned log_rows, unsigned log_row_len,
                        unsigned log_block, uint64_t row0, int inverse, uint64_t peer_stride, void* s) {
  if (log_rows + log_block >= 64) return set_err(NTT_ERR_ARG);
  return on_device(plan, [&](PlanBase& P) {
    return P.twiddle_pack(src, dst, log_rows, log_row_len, log_block, row0, inverse != 0, peer_stride, S(s));
  });
}

int ntt_transpose(ntt_plan* plan, const void* src, void* dst, unsigned log_rows, unsigned log_cols, void* s) {
  return ntt_transpose_ex(plan, src, dst, log_rows, log_cols, log_rows, 1ull << (log_rows + log_cols), s);
}

int ntt_transpose_ex(ntt_plan* plan, const void* src, void* dst, unsigned log_rows, unsigned log_cols,
                     unsigned log_block_rows, uint64_t block_stride, void* s) {
  if (log_rows + log_cols >= 64) return set_err(NTT_ERR_ARG);
  return on_device(plan, [&](PlanBase& P) {
    return P.transpose(src, dst, log_rows, log_cols, log_block_rows, block_stride, S(s));
  });
}

int ntt_plan_info(const ntt_plan* plan, uint64_t* n, unsigned* elem_bytes, unsigned* npasses, unsigned radix_log[8]) {
  if (!plan || !plan->impl) return NTT_ERR_ARG;
  const PlanBase& P = plan->wide ? *plan->wide : *plan->impl;  // one vector's schedule
  if (n) *n = P.n;
  if (elem_bytes) *elem_bytes = P.elem_bytes;
  if (npasses) *npasses = P.npass;
  if (radix_log)
    for (int i = 0; i < 8; ++i) radix_log[i] = P.r[i];
  return NTT_OK;
}

static int set_profiling(PlanBase& P, int enable) {
  if (enable && !P.ev[0][0]) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(P.device);
    for (auto& row : P.ev)
      for (auto& e : row)
        if (hipEventCreate(&e) != hipSuccess) { (void)hipSetDevice(cur); return NTT_ERR_HIP; }
    (void)hipSetDevice(cur);
  }
  P.profiling = enable != 0;
  P.nrec = 0;
  P.ev_used = 0;
  return NTT_OK;
}

// Group mode (PlanBase::begin): the next transform on the plan starts a new slot, the later ones
// continue it until the next call.
int ntt_plan_profile_group(ntt_plan* plan) {
  if (!plan || !plan->impl) return set_err(NTT_ERR_ARG);
  for (PlanBase* P : {plan->impl.get(), plan->wide.get()})
    if (P) P->grouped = P->group_new = true;
  return set_err(NTT_OK);
}

// Labels of the launches of the latest recorded transform (or group), comma-separated, in launch
// order: the same intervals as ntt_plan_last_launch_ms.
int ntt_plan_last_launch_labels(ntt_plan* plan, char* buf, unsigned cap) {
  if (!plan || !plan->impl || !buf || cap == 0) return set_err(NTT_ERR_ARG);
  PlanBase& P = plan->last ? *plan->last : *plan->impl;
  std::string out;
  for (unsigned i = 1; i < P.ev_used && P.nrec; ++i) {
    const char* l = P.lab[P.slot][i];
    if (l[0] == '-' && l[1] == 0) continue;
    if (!out.empty()) out += ',';
    out += l;
  }
  if (out.size() + 1 > cap) return set_err(NTT_ERR_ARG);
  memcpy(buf, out.c_str(), out.size() + 1);
  return set_err(NTT_OK);
}

int ntt_plan_set_profiling(ntt_plan* plan, int enable) {
  if (!plan || !plan->impl) return set_err(NTT_ERR_ARG);
  int rc = set_profiling(*plan->impl, enable);
  if (rc == NTT_OK && plan->wide) rc = set_profiling(*plan->wide, enable);
  return set_err(rc);
}

// Average per-launch durations over the transforms recorded since profiling was enabled (at most
// the last 64); waits for the most recent one.
int ntt_plan_last_launch_ms(ntt_plan* plan, float* ms, unsigned max_launches, unsigned* nlaunches) {
  if (!plan || !plan->impl || !ms) return set_err(NTT_ERR_ARG);
  PlanBase& P = plan->last ? *plan->last : *plan->impl;  // the plan that ran the latest transform
  const unsigned k = P.ev_used ? P.ev_used - 1 : 0;  // intervals of the latest slot (gaps included)
  auto gap = [&](unsigned i) {
    const char* l = P.lab[P.slot][i + 1];
    return l[0] == '-' && l[1] == 0;
  };
  unsigned nl = 0;
  for (unsigned i = 0; i < k; ++i) nl += gap(i) ? 0u : 1u;
  if (nlaunches) *nlaunches = P.nrec ? nl : 0u;
  if (nl == 0 || P.nrec == 0) return set_err(NTT_OK);
  if (hipEventSynchronize(P.ev[P.slot][k]) != hipSuccess) return set_err(NTT_ERR_HIP);
  const unsigned nslots = P.nrec < PlanBase::kSlots ? P.nrec : PlanBase::kSlots;
  unsigned j = 0;
  for (unsigned i = 0; i < k && j < max_launches; ++i) {
    if (gap(i)) continue;
    double acc = 0;
    for (unsigned sl = 0; sl < nslots; ++sl) {
      float t = 0;
      if (hipEventElapsedTime(&t, P.ev[sl][i], P.ev[sl][i + 1]) != hipSuccess) return set_err(NTT_ERR_HIP);
      acc += t;
    }
    ms[j++] = (float)(acc / nslots);
  }
  return set_err(NTT_OK);
}

int ntt_plan_destroy(ntt_plan* plan) {
  delete plan;
  return NTT_OK;
}

const char* ntt_strerror(int status) {
  switch (status) {
    case NTT_OK: return "ok";
    case NTT_ERR_ARG: return "invalid argument";
    case NTT_ERR_HIP: return "HIP runtime error";
    case NTT_ERR_RCCL: return "RCCL error";
    case NTT_ERR_FIELD: return "unsupported modulus or no root of unity of this order";
    case NTT_ERR_NODEV: return "no HIP device";
    case NTT_ERR_DEVICE:
      return "an inter-workgroup wait of an earlier call gave up (watchdog): that call's output is wrong; "
             "ntt_plan_device_status clears the report";
    default: return "unknown status";
  }
}

int ntt_last_error(void) { return g_last_error; }

// ---------------------------------------------------------------- reference-shaped shims
// Plans are cached per (modulus, generator, limbs, log_n, device) like a persistent version of the
// reference drivers' per-call table setup.  Threads calling a shim with the same key share the plan
// and its scratch, so each cached plan has its own lock, held for the whole blocking call
// (tests/test_gpu_threads.py: without it, concurrent calls overwrote each other's scratch).
namespace {
struct CachedPlan {
  std::unique_ptr<ntt_plan> plan;
  std::mutex run_mu;
  uint64_t last_use = 0;
  hipEvent_t done = nullptr;  // the blocking shims wait on this, like the reference's cudaEventSynchronize
  ~CachedPlan() {
    if (done) (void)hipEventDestroy(done);
  }
};
}  // namespace
static std::mutex g_cache_mu;
// Heap-held and never destroyed: cached plans outliving main() are not torn down after the HIP runtime
// (static destructors run in an unspecified order relative to it); ntt_shim_cache_clear frees them.
static auto& g_cache = *new std::map<std::tuple<std::vector<uint64_t>, std::vector<uint64_t>, unsigned, unsigned, int>,
                                     std::shared_ptr<CachedPlan>>();
static uint64_t g_cache_tick = 0;
// At most NTT_SHIM_CACHE_PLANS (default 8) cached plans; the least recently used one is dropped
// when a new key arrives (a call still running on it keeps it alive through its shared_ptr).
static size_t shim_cache_cap() {
  static const size_t cap = [] {
    const char* v = getenv("NTT_SHIM_CACHE_PLANS");
    const long c = v ? atol(v) : 8;
    return (size_t)(c > 0 ? c : 1);
  }();
  return cap;
}

static std::shared_ptr<CachedPlan> cached_plan(const uint64_t* p, const uint64_t* g, unsigned limbs64, unsigned log_n,
                                               int* rc) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  auto key = std::make_tuple(std::vector<uint64_t>(p, p + limbs64), std::vector<uint64_t>(g, g + limbs64), limbs64,
                             log_n, dev);
  std::lock_guard<std::mutex> lk(g_cache_mu);
  auto it = g_cache.find(key);
  if (it != g_cache.end()) {
    it->second->last_use = ++g_cache_tick;
    *rc = NTT_OK;
    return it->second;
  }
  ntt_plan* pl = nullptr;
  *rc = ntt_plan_create_custom(&pl, p, g, limbs64, log_n, dev);
  if (*rc != NTT_OK) return nullptr;
  while (g_cache.size() >= shim_cache_cap()) {
    auto lru = g_cache.begin();
    for (auto jt = g_cache.begin(); jt != g_cache.end(); ++jt)
      if (jt->second->last_use < lru->second->last_use) lru = jt;
    g_cache.erase(lru);
  }
  auto e = std::make_shared<CachedPlan>();
  e->plan.reset(pl);
  e->last_use = ++g_cache_tick;
  g_cache[key] = e;
  return e;
}

extern "C" void ntt_shim_cache_clear(void) {
  std::lock_guard<std::mutex> lk(g_cache_mu);
  g_cache.clear();
}

// Forward on the default stream, then wait for an event recorded after it (GZKP-NTT.cu:1547 waits on
// its own event the same way), under the plan's lock: work the caller runs on other non-blocking
// streams is not waited on.  A tripped watchdog (the plan's report, read after the wait) is this
// call's error, and is cleared so that the cached plan serves the next call.
static int blocking_forward(const std::shared_ptr<CachedPlan>& cp, void* d) {
  std::lock_guard<std::mutex> lk(cp->run_mu);
  int rc = ntt_forward(cp->plan.get(), d, nullptr);
  if (rc == NTT_OK && !cp->done && hipEventCreateWithFlags(&cp->done, hipEventDisableTiming) != hipSuccess) {
    cp->done = nullptr;
    rc = NTT_ERR_HIP;
  }
  if (rc == NTT_OK && (hipEventRecord(cp->done, nullptr) != hipSuccess || hipEventSynchronize(cp->done) != hipSuccess))
    rc = NTT_ERR_HIP;
  for (PlanBase* P : {cp->plan->impl.get(), cp->plan->wide.get()}) {
    if (P && P->tripped()) {
      P->clear_trip();
      if (rc == NTT_OK) rc = NTT_ERR_DEVICE;
    }
  }
  return set_err(rc);
}

void SSIP(long long* x, long long omega, unsigned log_n) {
  const uint64_t p = 469762049ull, g = (uint64_t)omega;
  int rc = NTT_OK;
  std::shared_ptr<CachedPlan> pl = cached_plan(&p, &g, 1, log_n, &rc);
  if (!pl) { set_err(rc); return; }
  blocking_forward(pl, x);
}

int NTT_GZKP_64(long long* data, const void* /*reverse*/, long long len, long long omega, int /*B*/, int /*G*/,
                long long /*reverse_num*/) {
  if (len <= 0 || (len & (len - 1))) return set_err(NTT_ERR_ARG);
  const unsigned log_n = (unsigned)__builtin_ctzll((unsigned long long)len);
  const uint64_t p = 469762049ull, g = (uint64_t)omega;
  int rc = NTT_OK;
  std::shared_ptr<CachedPlan> pl = cached_plan(&p, &g, 1, log_n, &rc);
  if (!pl) return set_err(rc);
  return blocking_forward(pl, data);
}

int NTT_GZKP_256(uint32_t* data, uint32_t len, const void* /*reverse*/, uint32_t /*reverse_len*/,
                 const uint32_t prime[8], const uint32_t omega[8], uint32_t /*B*/, uint32_t /*G*/) {
  if (!data || !prime || !omega || len == 0 || (len & (len - 1))) return set_err(NTT_ERR_ARG);
  const unsigned log_n = (unsigned)__builtin_ctz(len);
  uint64_t p[4], g[4];
  for (int i = 0; i < 4; ++i) {
    p[i] = (uint64_t)prime[2 * i] | ((uint64_t)prime[2 * i + 1] << 32);
    g[i] = (uint64_t)omega[2 * i] | ((uint64_t)omega[2 * i + 1] << 32);
  }
  int rc = NTT_OK;
  std::shared_ptr<CachedPlan> pl = cached_plan(p, g, 4, log_n, &rc);
  if (!pl) return set_err(rc);
  return blocking_forward(pl, data);
}

}  // extern "C"

// ---------------------------------------------------------------- library-internal (ntt_internal.hpp)
namespace ntt {
int plan_run_fs(ntt_plan* plan, const void* in, const void* in2, void* out, unsigned batch, bool inverse,
                const FsIO& io, hipStream_t st) {
  if (!plan || !plan->impl) return NTT_ERR_ARG;
  return plan->impl->run_fs(in, in2, out, batch, inverse, io, st);
}
int plan_build_fs_table(ntt_plan* plan, void* table, unsigned log_rows, unsigned log_cols, uint64_t row0,
                        uint64_t col0, bool inverse, hipStream_t st, unsigned scale_log) {
  if (!plan || !plan->impl) return NTT_ERR_ARG;
  return plan->impl->build_fs_table(table, log_rows, log_cols, row0, col0, inverse, scale_log, st);
}
size_t plan_table_entry_bytes(const ntt_plan* plan) { return plan && plan->impl ? plan->impl->table_entry_bytes() : 0; }
int plan_device(const ntt_plan* plan) { return plan && plan->impl ? plan->impl->device : -1; }
int plan_create_internal(ntt_plan** out, int field_id, unsigned log_n, unsigned limbs64, int device) {
  return create_field_plan(out, field_id, log_n, limbs64, device, 0, false);
}
unsigned plan_max_radix_for(const ntt_plan* plan, unsigned log_x) {
  return plan && plan->impl ? plan->impl->max_radix_for(log_x) : 99u;
}
unsigned plan_passes_for(const ntt_plan* plan, unsigned log_x) {
  return plan && plan->impl ? plan->impl->passes_for(log_x) : 99u;
}
}  // namespace ntt
