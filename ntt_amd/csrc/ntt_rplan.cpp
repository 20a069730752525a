// One rank of the distributed four-step NTT: the local steps around the all-to-all,
// fused so that no separate twiddle, pack or transpose pass touches HBM.
//
//   n = n1 n2 with n1 >= n2: the fewest pass kernels in total, then the smallest largest radix, then the
//   most balanced split (choose_split; ntt_rplan_info reports it); rank g of G owns
//   r = n1/G rows and c = n2/G columns.  Layouts (ntt.h):
//     row layout     [r][n2]: local (a, j2)  = x[g r + a + n1 j2]
//     column layout  [n1][c]: local (k1, kc) = X[g c + kc + n2 k1]   (transform index fastest)
//
//   forward rows  : r length-n2 transforms of the row layout; the last pass multiplies output k2 of
//                   row a by w_n^((g r + a) k2) (per-rank table) and stores it straight into the
//                   send buffer's peer chunk k2 / c at [a][k2 mod c]                   (Mode B out)
//   exchange      : the caller's all-to-all of equal chunks; recv = [G][r][c] = [n1][c]
//   forward cols  : c interleaved length-n1 transforms read recv as it arrived (Mode I) -> x
//   inverse cols  : c interleaved inverse transforms of x (optionally of x * y: polymul, the
//                   product taken at the first pass's load); the last pass multiplies by
//                   w_n^-(j1 (g c + kc)) and writes send = [n1][c], whose peer chunks are contiguous
//   inverse rows  : r inverse length-n2 transforms reading recv = [G][c][r... ] through the chunk map
//                   (Mode B in) -> row layout
// The buffers are the caller's ([G][nvec][r c] elements each), so the exchange can be RCCL through
// torch.distributed, ncclAllToAll in ntt_mplan, or device copies between virtual ranks.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/ntt.h"
#include "ntt_internal.hpp"
#include "ntt_kernels.hpp"

using namespace ntt;

struct ntt_rplan {
  int world = 1, rank = 0, device = 0;
  unsigned log_n = 0, log_n1 = 0, log_n2 = 0, log_g = 0, log_r = 0, log_c = 0;
  size_t elem_bytes = 0;
  ntt_plan *rows = nullptr, *cols = nullptr, *tw = nullptr;
  void* tab_fwd = nullptr;  // [r][n2]: w_n^((g r + a) k2)
  void* tab_inv = nullptr;  // [n1][c]: w_n^-(j1 (g c + kc)) (times n2^-1 when rows_no_scale)
  // the row transforms are single-pass: their inverse's n2^-1 is folded into tab_inv (the inverse
  // columns' epilogue), so the inverse rows run without their scaling product
  bool rows_no_scale = false;
  ~ntt_rplan() {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    if (tab_fwd) (void)hipFree(tab_fwd);
    if (tab_inv) (void)hipFree(tab_inv);
    if (rows) ntt_plan_destroy(rows);
    if (cols) ntt_plan_destroy(cols);
    if (tw) ntt_plan_destroy(tw);
    (void)hipSetDevice(cur);
  }
  uint64_t chunk() const { return 1ull << (log_r + log_c); }
};

namespace {

struct DeviceScope {
  int cur = 0;
  bool moved = false;
  explicit DeviceScope(int dev) {
    (void)hipGetDevice(&cur);
    if (cur != dev) moved = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceScope() {
    if (moved) (void)hipSetDevice(cur);
  }
};

hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }

bool nvec_ok(unsigned nvec, unsigned slot) { return (nvec == 1 || nvec == 2) && slot < nvec; }

// one-level map: p -> (p >> lc) ps + (b << lc) + (p mod 2^lc)
FsMap map1(unsigned lc, uint64_t ps) { return FsMap{lc, lc, ps, 0}; }
// two-level map: peer blocks of ps, column pieces of ps2 within them (FsMap, ntt_kernels.hpp)
FsMap map2(unsigned lc, uint64_t ps, unsigned lc2, uint64_t ps2) { return FsMap{lc, lc2, ps, ps2}; }

// The split n = n1 n2 (log_n2 returned): fewest pass kernels over the row (length n2) and column
// (length n1) transforms, then the smallest largest radix among those passes, then the most balanced
// split.  2^24 on the 256-bit engines: 12 + 12 takes 2 + 2 passes; 14 + 10, 15 + 9 and 16 + 8 take
// 2 + 1 (the rows one workgroup tile each), as many HBM passes as the one-GPU transform, and 16 + 8 has
// the smallest radices (8 + 8 column passes, radix-256 rows): its rank-local launches measured 1.06 /
// 1.07 / 1.13 x (1/G of the one-GPU transform) at G = 2 / 4 / 8, against 1.09 / 1.12 / 1.16 x for
// 14 + 10 (round 5, profiles/r05_ranklocal/).  14 + 10 runs 5.25 products per element in its radix-1024
// row launch where 16 + 8 runs 4.06 (the one-GPU transform's count).  2^28 stays 14 + 14 (4 passes of
// radix 2^7).
unsigned choose_split(const ntt_plan* tw, unsigned log_n, unsigned log_g) {
  const unsigned bal = log_n / 2;
  if (const char* e = std::getenv("NTT_FS_LOG_N2")) {  // experiments (tools/ab_env.sh): a fixed n2
    const unsigned v = (unsigned)std::atoi(e);
    if (v >= 3 && v >= log_g && v <= bal) return v;
  }
  unsigned best = bal, best_p = ~0u, best_r = ~0u;
  for (unsigned s2 = bal; s2 >= 3 && s2 >= log_g; --s2) {
    const unsigned p = plan_passes_for(tw, log_n - s2) + plan_passes_for(tw, s2);
    const unsigned r1 = plan_max_radix_for(tw, log_n - s2), r2 = plan_max_radix_for(tw, s2);
    const unsigned r = r1 > r2 ? r1 : r2;
    if (p < best_p || (p == best_p && r < best_r)) {
      best_p = p;
      best_r = r;
      best = s2;
    }
  }
  return best;
}

// grid.y of a row launch is its row count: launches of at most 2^15 rows
constexpr uint64_t kMaxRowsPerLaunch = 1ull << 15;

// a row piece [row0, row0 + nrows) of the r local rows
bool range_ok(const ntt_rplan* rp, uint64_t row0, uint64_t nrows) {
  const uint64_t r = 1ull << rp->log_r;
  return nrows >= 1 && row0 < r && nrows <= r - row0;
}

// Pieces of the two-sided pipelined exchange (FourStep, ntt_amd/distributed.py): P_r row pieces of
// ra = r / P_r rows, P_c column pieces of cm = c / P_c columns (powers of two).  Exchange blocks, one
// per peer of nvec r c elements:
//   forward [i][v][k][ra][cm]  written by forward_rows_piece (row piece i), read by forward_cols_piece
//                              (column piece k: rows j1 = h r + i ra + a' of every peer h)
//   inverse [k][i][ra][cm]     written by inverse_cols_piece (column piece k), read by
//                              inverse_rows_piece (row piece i)
// With P_r = P_c = 1 both are the [G][nvec][r][c] blocks of the row-range entry points.
bool pieces_ok(const ntt_rplan* rp, unsigned rpc, unsigned cpc, unsigned& lra, unsigned& lcm) {
  if (rpc == 0 || cpc == 0 || (rpc & (rpc - 1)) || (cpc & (cpc - 1))) return false;
  const unsigned lp = (unsigned)__builtin_ctz(rpc), lq = (unsigned)__builtin_ctz(cpc);
  if (lp > rp->log_r || lq > rp->log_c) return false;
  lra = rp->log_r - lp;
  lcm = rp->log_c - lq;
  return true;
}

}  // namespace

extern "C" {

int ntt_rplan_create(ntt_rplan** out, int field_id, unsigned log_n, unsigned limbs64, int world, int rank,
                     int device) {
  if (!out) return NTT_ERR_ARG;
  *out = nullptr;
  if (world < 1 || (world & (world - 1)) || rank < 0 || rank >= world || log_n > 40) return NTT_ERR_ARG;
  auto rp = new ntt_rplan();
  rp->world = world;
  rp->rank = rank;
  rp->device = device;
  rp->log_n = log_n;
  rp->log_g = (unsigned)__builtin_ctz((unsigned)world);
  // every local transform has >= 8 points (one or more pass kernels) and >= 1 row / column per rank
  if (log_n / 2 < 3 || rp->log_g > log_n / 2) {
    delete rp;
    return NTT_ERR_ARG;
  }
  DeviceScope scope(device);
  int rc = ntt_plan_create_ex(&rp->tw, field_id, log_n, limbs64, device, NTT_PLAN_TWIDDLE_ONLY);
  if (rc == NTT_OK) {
    rp->log_n2 = choose_split(rp->tw, log_n, rp->log_g);
    rp->log_n1 = log_n - rp->log_n2;
    rp->log_r = rp->log_n1 - rp->log_g;
    rp->log_c = rp->log_n2 - rp->log_g;
    rc = plan_create_internal(&rp->rows, field_id, rp->log_n2, limbs64, device);
  }
  if (rc == NTT_OK) rc = plan_create_internal(&rp->cols, field_id, rp->log_n1, limbs64, device);
  if (rc == NTT_OK) {
    uint64_t n = 0;
    unsigned eb = 0;
    ntt_plan_info(rp->rows, &n, &eb, nullptr, nullptr);
    rp->elem_bytes = eb;
    const size_t tb = plan_table_entry_bytes(rp->tw);
    const size_t local = 1ull << (log_n - rp->log_g);
    if (hipMalloc(&rp->tab_fwd, local * tb) != hipSuccess || hipMalloc(&rp->tab_inv, local * tb) != hipSuccess)
      rc = NTT_ERR_HIP;
  }
  if (rc == NTT_OK) {
    const uint64_t g = (uint64_t)rank;
    // single-pass row transforms leave n2^-1 to the inverse epilogue table: ask the rows plan itself
    // which schedule it runs, not the twiddle plan
    rp->rows_no_scale = plan_passes_for(rp->rows, rp->log_n2) == 1;
    rc = plan_build_fs_table(rp->tw, rp->tab_fwd, rp->log_r, rp->log_n2, g << rp->log_r, 0, false, nullptr);
    if (rc == NTT_OK)
      rc = plan_build_fs_table(rp->tw, rp->tab_inv, rp->log_n1, rp->log_c, 0, g << rp->log_c, true, nullptr,
                               rp->rows_no_scale ? rp->log_n2 : 0u);
    if (rc == NTT_OK && hipDeviceSynchronize() != hipSuccess) rc = NTT_ERR_HIP;
  }
  if (rc != NTT_OK) {
    delete rp;
    return rc;
  }
  *out = rp;
  return NTT_OK;
}

int ntt_rplan_info(const ntt_rplan* rp, uint64_t* local_n, uint64_t* chunk, unsigned* log_n1, unsigned* log_n2,
                   unsigned* elem_bytes) {
  if (!rp) return NTT_ERR_ARG;
  if (local_n) *local_n = 1ull << (rp->log_n - rp->log_g);
  if (chunk) *chunk = rp->chunk();
  if (log_n1) *log_n1 = rp->log_n1;
  if (log_n2) *log_n2 = rp->log_n2;
  if (elem_bytes) *elem_bytes = (unsigned)rp->elem_bytes;
  return NTT_OK;
}

int ntt_rplan_forward_rows_range(ntt_rplan* rp, const void* d_x, void* d_send, unsigned nvec, unsigned slot,
                                 uint64_t row0, uint64_t nrows, void* s) {
  if (!rp || !d_x || !d_send || !nvec_ok(nvec, slot) || !range_ok(rp, row0, nrows)) return NTT_ERR_ARG;
  if (nrows > kMaxRowsPerLaunch) {
    for (uint64_t a = 0; a < nrows; a += kMaxRowsPerLaunch) {
      const uint64_t m = nrows - a < kMaxRowsPerLaunch ? nrows - a : kMaxRowsPerLaunch;
      if (int rc = ntt_rplan_forward_rows_range(rp, d_x, d_send, nvec, slot, row0 + a, m, s)) return rc;
    }
    return NTT_OK;
  }
  DeviceScope scope(rp->device);
  // batch index b of the launch is local row row0 + b: shift the input rows, the epilogue table rows
  // and the Mode B output map (row a lands at a c within every peer chunk) by row0
  FsIO io;
  io.fs = FS_MAP_OUT;
  io.mout = map1(rp->log_c, nvec * rp->chunk());
  io.tw_epi = static_cast<const char*>(rp->tab_fwd) + (row0 << rp->log_n2) * plan_table_entry_bytes(rp->tw);
  const void* src = static_cast<const char*>(d_x) + (row0 << rp->log_n2) * rp->elem_bytes;
  void* dst = static_cast<char*>(d_send) + (slot * rp->chunk() + (row0 << rp->log_c)) * rp->elem_bytes;
  return plan_run_fs(rp->rows, src, nullptr, dst, (unsigned)nrows, false, io, S(s));
}

int ntt_rplan_forward_rows(ntt_rplan* rp, const void* d_x, void* d_send, unsigned nvec, unsigned slot, void* s) {
  if (!rp) return NTT_ERR_ARG;
  return ntt_rplan_forward_rows_range(rp, d_x, d_send, nvec, slot, 0, 1ull << rp->log_r, s);
}

int ntt_rplan_forward_cols(ntt_rplan* rp, const void* d_recv, void* d_x, unsigned nvec, unsigned slot, void* s) {
  if (!rp || !d_x || !d_recv || !nvec_ok(nvec, slot)) return NTT_ERR_ARG;
  DeviceScope scope(rp->device);
  FsIO io;
  io.fs = FS_IL | (nvec > 1 ? FS_MAP_IN : 0u);
  io.il = rp->log_c;
  io.min = map1(rp->log_r + rp->log_c, nvec * rp->chunk());
  const void* src = static_cast<const char*>(d_recv) + slot * rp->chunk() * rp->elem_bytes;
  return plan_run_fs(rp->cols, src, nullptr, d_x, 1, false, io, S(s));
}

int ntt_rplan_inverse_cols(ntt_rplan* rp, const void* d_x, const void* d_y, void* d_send, void* s) {
  if (!rp || !d_x || !d_send) return NTT_ERR_ARG;
  DeviceScope scope(rp->device);
  FsIO io;
  io.fs = FS_IL;
  io.il = rp->log_c;
  io.tw_epi = rp->tab_inv;
  return plan_run_fs(rp->cols, d_x, d_y, d_send, 1, true, io, S(s));
}

int ntt_rplan_inverse_rows_range(ntt_rplan* rp, const void* d_recv, void* d_out, uint64_t row0, uint64_t nrows,
                                 void* s) {
  if (!rp || !d_recv || !d_out || !range_ok(rp, row0, nrows)) return NTT_ERR_ARG;
  if (nrows > kMaxRowsPerLaunch) {
    for (uint64_t a = 0; a < nrows; a += kMaxRowsPerLaunch) {
      const uint64_t m = nrows - a < kMaxRowsPerLaunch ? nrows - a : kMaxRowsPerLaunch;
      if (int rc = ntt_rplan_inverse_rows_range(rp, d_recv, d_out, row0 + a, m, s)) return rc;
    }
    return NTT_OK;
  }
  DeviceScope scope(rp->device);
  FsIO io;
  io.fs = FS_MAP_IN;
  io.min = map1(rp->log_c, rp->chunk());
  io.no_scale = rp->rows_no_scale;
  const void* src = static_cast<const char*>(d_recv) + (row0 << rp->log_c) * rp->elem_bytes;
  void* dst = static_cast<char*>(d_out) + (row0 << rp->log_n2) * rp->elem_bytes;
  return plan_run_fs(rp->rows, src, nullptr, dst, (unsigned)nrows, true, io, S(s));
}

int ntt_rplan_inverse_rows(ntt_rplan* rp, const void* d_recv, void* d_out, void* s) {
  if (!rp) return NTT_ERR_ARG;
  return ntt_rplan_inverse_rows_range(rp, d_recv, d_out, 0, 1ull << rp->log_r, s);
}

int ntt_rplan_forward_rows_piece(ntt_rplan* rp, const void* d_x, void* d_send, unsigned nvec, unsigned slot,
                                 unsigned piece, unsigned row_pieces, unsigned col_pieces, void* s) {
  unsigned lra = 0, lcm = 0;
  if (!rp || !d_x || !d_send || !nvec_ok(nvec, slot) || !pieces_ok(rp, row_pieces, col_pieces, lra, lcm) ||
      piece >= row_pieces)
    return NTT_ERR_ARG;
  DeviceScope scope(rp->device);
  const uint64_t ra = 1ull << lra, cm = 1ull << lcm, c = 1ull << rp->log_c;
  for (uint64_t a0 = 0; a0 < ra; a0 += kMaxRowsPerLaunch) {
    const uint64_t m = ra - a0 < kMaxRowsPerLaunch ? ra - a0 : kMaxRowsPerLaunch;
    const uint64_t row0 = piece * ra + a0;
    // output k2 of launch row b: peer k2 >> log c, column piece (k2 mod c) >> log cm, row a0 + b
    FsIO io;
    io.fs = FS_MAP_OUT;
    io.mout = map2(rp->log_c, nvec * rp->chunk(), lcm, ra * cm);
    io.tw_epi = static_cast<const char*>(rp->tab_fwd) + (row0 << rp->log_n2) * plan_table_entry_bytes(rp->tw);
    const void* src = static_cast<const char*>(d_x) + (row0 << rp->log_n2) * rp->elem_bytes;
    void* dst = static_cast<char*>(d_send) + ((piece * nvec + slot) * ra * c + a0 * cm) * rp->elem_bytes;
    if (int rc = plan_run_fs(rp->rows, src, nullptr, dst, (unsigned)m, false, io, S(s))) return rc;
  }
  return NTT_OK;
}

int ntt_rplan_forward_cols_piece(ntt_rplan* rp, const void* d_recv, void* d_x, unsigned nvec, unsigned slot,
                                 unsigned piece, unsigned row_pieces, unsigned col_pieces, void* s) {
  unsigned lra = 0, lcm = 0;
  if (!rp || !d_recv || !d_x || !nvec_ok(nvec, slot) || !pieces_ok(rp, row_pieces, col_pieces, lra, lcm) ||
      piece >= col_pieces)
    return NTT_ERR_ARG;
  DeviceScope scope(rp->device);
  const uint64_t ra = 1ull << lra, cm = 1ull << lcm, c = 1ull << rp->log_c;
  // cm interleaved transforms; element j1 = (h P_r + i) ra + a' of transform kc' at that block's unit
  FsIO io;
  io.fs = FS_IL | FS_MAP_IN | FS_MAP_OUT;
  io.il = lcm;
  io.min = map1(lra + lcm, nvec * ra * c);
  io.mout = map1(lcm, c);  // column layout [n1][c], columns piece cm + [0, cm)
  const void* src = static_cast<const char*>(d_recv) + (slot * ra * c + piece * ra * cm) * rp->elem_bytes;
  void* dst = static_cast<char*>(d_x) + piece * cm * rp->elem_bytes;
  return plan_run_fs(rp->cols, src, nullptr, dst, 1, false, io, S(s));
}

int ntt_rplan_inverse_cols_piece(ntt_rplan* rp, const void* d_x, const void* d_y, void* d_send, unsigned piece,
                                 unsigned row_pieces, unsigned col_pieces, void* s) {
  unsigned lra = 0, lcm = 0;
  if (!rp || !d_x || !d_send || !pieces_ok(rp, row_pieces, col_pieces, lra, lcm) || piece >= col_pieces)
    return NTT_ERR_ARG;
  DeviceScope scope(rp->device);
  const uint64_t cm = 1ull << lcm, c = 1ull << rp->log_c;
  FsIO io;
  io.fs = FS_IL | FS_MAP_IN | FS_MAP_OUT | FS_MAP_EPI;
  io.il = lcm;
  io.min = map1(lcm, c);                          // columns piece cm + [0, cm) of [n1][c] (and of y)
  io.mout = map1(rp->log_r + lcm, rp->chunk());  // j1 = h r + a -> block h, unit piece, row a
  io.mepi = map1(lcm, c);                         // the [n1][c] epilogue table
  io.tw_epi = static_cast<const char*>(rp->tab_inv) + piece * cm * plan_table_entry_bytes(rp->tw);
  const size_t off = piece * cm * rp->elem_bytes;
  const void* src = static_cast<const char*>(d_x) + off;
  const void* y = d_y ? static_cast<const char*>(d_y) + off : nullptr;
  void* dst = static_cast<char*>(d_send) + (piece << (rp->log_r + lcm)) * rp->elem_bytes;
  return plan_run_fs(rp->cols, src, y, dst, 1, true, io, S(s));
}

int ntt_rplan_inverse_rows_piece(ntt_rplan* rp, const void* d_recv, void* d_out, unsigned piece, unsigned row_pieces,
                                 unsigned col_pieces, void* s) {
  unsigned lra = 0, lcm = 0;
  if (!rp || !d_recv || !d_out || !pieces_ok(rp, row_pieces, col_pieces, lra, lcm) || piece >= row_pieces)
    return NTT_ERR_ARG;
  DeviceScope scope(rp->device);
  const uint64_t ra = 1ull << lra, cm = 1ull << lcm;
  for (uint64_t a0 = 0; a0 < ra; a0 += kMaxRowsPerLaunch) {
    const uint64_t m = ra - a0 < kMaxRowsPerLaunch ? ra - a0 : kMaxRowsPerLaunch;
    const uint64_t row0 = piece * ra + a0;
    // input k2 of launch row b: block k2 >> log c, unit (k2 mod c) >> log cm, row row0 + b
    FsIO io;
    io.fs = FS_MAP_IN;
    io.min = map2(rp->log_c, rp->chunk(), lcm, (1ull << rp->log_r) * cm);
    io.no_scale = rp->rows_no_scale;
    const void* src = static_cast<const char*>(d_recv) + row0 * cm * rp->elem_bytes;
    void* dst = static_cast<char*>(d_out) + (row0 << rp->log_n2) * rp->elem_bytes;
    if (int rc = plan_run_fs(rp->rows, src, nullptr, dst, (unsigned)m, true, io, S(s))) return rc;
  }
  return NTT_OK;
}

int ntt_rplan_fill(ntt_rplan* rp, void* d_x, int kind, uint64_t seed, void* s) {
  if (!rp || !d_x) return NTT_ERR_ARG;
  // local element i = (a, j2) of the row layout: global j = g r + a + n1 j2
  return ntt_fill_map(rp->tw, d_x, 1ull << (rp->log_n - rp->log_g), kind, seed, (uint64_t)rp->rank << rp->log_r,
                      rp->log_n2, rp->log_n1, s);
}

int ntt_rplan_set_profiling(ntt_rplan* rp, int enable) {
  if (!rp) return NTT_ERR_ARG;
  int rc = ntt_plan_set_profiling(rp->rows, enable);
  return rc ? rc : ntt_plan_set_profiling(rp->cols, enable);
}

int ntt_rplan_last_launch_ms(ntt_rplan* rp, int which, float* ms, unsigned max_launches, unsigned* nlaunches) {
  if (!rp || (which != 0 && which != 1)) return NTT_ERR_ARG;
  return ntt_plan_last_launch_ms(which ? rp->cols : rp->rows, ms, max_launches, nlaunches);
}

int ntt_rplan_last_launch_labels(ntt_rplan* rp, int which, char* buf, unsigned cap) {
  if (!rp || (which != 0 && which != 1)) return NTT_ERR_ARG;
  return ntt_plan_last_launch_labels(which ? rp->cols : rp->rows, buf, cap);
}

int ntt_rplan_profile_group(ntt_rplan* rp) {
  if (!rp) return NTT_ERR_ARG;
  int rc = ntt_plan_profile_group(rp->rows);
  return rc ? rc : ntt_plan_profile_group(rp->cols);
}

int ntt_rplan_destroy(ntt_rplan* rp) {
  delete rp;
  return NTT_OK;
}

}  // extern "C"
