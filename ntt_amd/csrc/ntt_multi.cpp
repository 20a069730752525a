// Single-process multi-GPU four-step (SURVEY §8b `ntt_mplan_*`, §8e): one plan object drives G
// devices of one node, with the transpose as ONE RCCL all-to-all over xGMI per transform.
//
// The layouts are those of ntt_amd/distributed.py (the one-process-per-GPU form of the same
// schedule): n = n1 n2 (the rank plans' split, ntt_rplan.cpp choose_split), r = n1 / G rows and c = n2 / G
// columns per device.
//   input  (row layout):    device g holds [r][n2], element (a, j2) = x[g r + a + n1 j2]
//   output (column layout): device g holds [n1][c], element (k1, kc) = X[g c + kc + n2 k1]
// Forward on every device (its ntt_rplan, ntt_rplan.cpp): batched n2-point NTTs of its rows whose
// last pass applies w_n^(j1 k2) and stores straight into the per-peer chunks -> all-to-all (RCCL,
// grouped over the devices) -> interleaved n1-point NTTs reading the chunks as they arrived.  The
// inverse mirrors it (column layout in, row layout out).  All work is asynchronous on the callers'
// per-device streams.  The reference has no multi-GPU code.
//
// Pipelined exchange on both sides (the schedule of FourStep, ntt_amd/distributed.py): P_r row pieces
// x P_c column pieces (ntt_rplan_*_piece; every exchange unit is one contiguous run of a peer block).
// Forward: row piece i is exchanged (grouped ncclSend / ncclRecv on a per-device communication
// stream, ordered by events) while the row transforms of piece i + 1 run; the last row piece goes out
// column piece by column piece, and the column transforms of piece k start when its unit has arrived.
// The inverse mirrors it.  Default 1 x 1 (one whole-block exchange); ntt_mplan_set_pieces /
// ntt_mplan_set_pieces2 select pieces.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ntt.h"

namespace {

// RCCL is resolved at first use, not linked: a process that already carries an RCCL (PyTorch's
// bundled one) keeps using that single copy, and single-GPU users never load it at all.
struct Rccl {
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllToAll)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  bool ok() const {
    return CommInitAll && CommDestroy && AllToAll && GroupStart && GroupEnd && Send && Recv && CommAbort;
  }
};

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = RTLD_DEFAULT;
    // NTT_RCCL_LIBRARY: an explicit RCCL (or a fault-injecting stand-in, tests/test_gpu_mplan_faults.py).
    // Absolute paths only (no search-path lookup), and the override is announced on stderr.
    if (const char* lib = getenv("NTT_RCCL_LIBRARY"); lib && *lib) {
      if (lib[0] != '/') {
        fprintf(stderr, "libntt: NTT_RCCL_LIBRARY must be an absolute path; ignored: %s\n", lib);
        return x;
      }
      fprintf(stderr, "libntt: multi-GPU collectives from NTT_RCCL_LIBRARY=%s\n", lib);
      h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
      if (!h) return x;
    } else if (!dlsym(h, "ncclCommInitAll")) {
      h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
      if (!h) return x;
    }
    x.CommInitAll = reinterpret_cast<decltype(x.CommInitAll)>(dlsym(h, "ncclCommInitAll"));
    x.CommDestroy = reinterpret_cast<decltype(x.CommDestroy)>(dlsym(h, "ncclCommDestroy"));
    x.AllToAll = reinterpret_cast<decltype(x.AllToAll)>(dlsym(h, "ncclAllToAll"));
    x.GroupStart = reinterpret_cast<decltype(x.GroupStart)>(dlsym(h, "ncclGroupStart"));
    x.GroupEnd = reinterpret_cast<decltype(x.GroupEnd)>(dlsym(h, "ncclGroupEnd"));
    x.Send = reinterpret_cast<decltype(x.Send)>(dlsym(h, "ncclSend"));
    x.Recv = reinterpret_cast<decltype(x.Recv)>(dlsym(h, "ncclRecv"));
    x.CommAbort = reinterpret_cast<decltype(x.CommAbort)>(dlsym(h, "ncclCommAbort"));
    return x;
  }();
  return r;
}

}  // namespace

struct ntt_mplan {
  int ngpus = 0;
  unsigned log_n = 0, log_g = 0, log_n1 = 0, log_n2 = 0, log_r = 0, log_c = 0;
  unsigned elem_bytes = 0;
  std::vector<int> dev;
  std::vector<ntt_rplan*> rp;       // device g's local steps (ntt_rplan.cpp)
  std::vector<void*> send, recv;    // [G][chunk] per device
  std::vector<void*> send2, recv2;  // [G][2][chunk]: the polymul's batched (a, b) exchange, on first use
  std::vector<ncclComm_t> comm;
  std::vector<hipStream_t> cstream;   // per-device communication stream (pipelined exchange)
  std::vector<hipEvent_t> ev_ready;   // per device: compute -> communication ordering
  std::vector<hipEvent_t> ev_done;    // per device and piece: arrival of piece i (kMaxPieces each)
  unsigned pieces = 1;      // row pieces P_r (power of two)
  unsigned col_pieces = 1;  // column pieces P_c (power of two)
  // set when an exchange failed: the communicators were aborted (a peer may have posted its part of
  // the collective) and every later call returns NTT_ERR_RCCL
  bool broken = false;

  ~ntt_mplan() {
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (size_t g = 0; g < dev.size(); ++g) {
      (void)hipSetDevice(dev[g]);
      if (g < comm.size() && comm[g]) rccl().CommDestroy(comm[g]);
      if (g < cstream.size() && cstream[g]) (void)hipStreamDestroy(cstream[g]);
      if (g < ev_ready.size() && ev_ready[g]) (void)hipEventDestroy(ev_ready[g]);
      for (size_t i = g * kMaxPieces; i < (g + 1) * kMaxPieces && i < ev_done.size(); ++i)
        if (ev_done[i]) (void)hipEventDestroy(ev_done[i]);
      for (auto* v : {&send, &recv, &send2, &recv2})
        if (g < v->size() && (*v)[g]) (void)hipFree((*v)[g]);
      if (g < rp.size() && rp[g]) ntt_rplan_destroy(rp[g]);
    }
    (void)hipSetDevice(cur);
  }
  static constexpr unsigned kMaxPieces = 16;
  size_t local_n() const { return 1ull << (log_n - log_g); }
  hipEvent_t done(int g, unsigned i) const { return ev_done[g * kMaxPieces + i]; }
  hipStream_t stream(void* const* streams, int g) const {
    return streams ? static_cast<hipStream_t>(streams[g]) : nullptr;
  }
};

namespace {

struct DeviceGuard {
  int cur = 0;
  DeviceGuard() { (void)hipGetDevice(&cur); }
  ~DeviceGuard() { (void)hipSetDevice(cur); }
};

// RCCL moves at most 2^31 - 1 bytes per peer per collective (a 2 GiB per-peer chunk arrived half
// copied with ncclAllToAll: 2^26 BN254 on one device, tests/test_gpu_fullsize.py), so per-peer chunks
// above kMaxPeerBytes are exchanged as grouped ncclSend/ncclRecv pieces instead.
constexpr size_t kMaxPeerBytes = size_t(1) << 30;

// A call failed inside a grouped exchange.  If it failed on device g > 0, devices 0..g-1 already
// posted their part: the closed group launched a partial all-to-all whose kernels wait for peers that
// never come, and a stream drain would block forever.  Aborting every communicator ends those
// operations (RCCL's documented recovery); the plan is then unusable and every later call returns
// NTT_ERR_RCCL.  The caller's drain() follows.
int abort_comms(ntt_mplan* m) {
  const Rccl& R = rccl();
  for (size_t g = 0; g < m->comm.size(); ++g) {
    if (!m->comm[g]) continue;
    (void)hipSetDevice(m->dev[g]);
    (void)R.CommAbort(m->comm[g]);
    m->comm[g] = nullptr;
  }
  m->broken = true;
  return NTT_ERR_RCCL;
}

// All-to-all of per-peer chunks of `words` 64-bit words: send[g] = [G][words] -> recv[g] = [G][words].
int exchange(ntt_mplan* m, const std::vector<void*>& send, const std::vector<void*>& recv, size_t words,
             void* const* streams) {
  const Rccl& R = rccl();
  if (R.GroupStart() != ncclSuccess) return NTT_ERR_RCCL;
  ncclResult_t st = ncclSuccess;
  if (words * 8 <= kMaxPeerBytes) {
    for (int g = 0; g < m->ngpus && st == ncclSuccess; ++g) {
      (void)hipSetDevice(m->dev[g]);  // inside the group: RCCL calls carry their communicator's device
      st = R.AllToAll(send[g], recv[g], words, ncclUint64, m->comm[g], m->stream(streams, g));
    }
  } else {
    const size_t piece = kMaxPeerBytes / 8;
    for (int g = 0; g < m->ngpus && st == ncclSuccess; ++g) {
      (void)hipSetDevice(m->dev[g]);  // inside the group: RCCL calls carry their communicator's device
      hipStream_t s = m->stream(streams, g);
      auto* sb = static_cast<uint64_t*>(send[g]);
      auto* rb = static_cast<uint64_t*>(recv[g]);
      for (int h = 0; h < m->ngpus && st == ncclSuccess; ++h)
        for (size_t off = 0; off < words && st == ncclSuccess; off += piece) {
          const size_t cnt = words - off < piece ? words - off : piece;
          st = R.Send(sb + h * words + off, cnt, ncclUint64, h, m->comm[g], s);
          if (st == ncclSuccess) st = R.Recv(rb + h * words + off, cnt, ncclUint64, h, m->comm[g], s);
        }
    }
  }
  // always close the group: the calls already issued for other devices are launched (or dropped) by
  // RCCL as a unit, never left pending in the thread's group state
  const ncclResult_t end = R.GroupEnd();
  return (st == ncclSuccess && end == ncclSuccess) ? NTT_OK : abort_comms(m);
}

size_t peer_elems(const ntt_mplan* m) {  // per-peer chunk of one vector: r * c = local_n / G elements
  return 1ull << (m->log_r + m->log_c);
}
size_t chunk_words(const ntt_mplan* m) { return peer_elems(m) * (m->elem_bytes / 8); }

// Runs of every peer block (blocks of peer_elems elements; runs (offset, length) in elements) as
// grouped ncclSend / ncclRecv on the communication streams.
struct Run {
  size_t off, len;
};
int exchange_runs(ntt_mplan* m, const std::vector<void*>& send, const std::vector<void*>& recv, size_t peer_elems,
                  const std::vector<Run>& runs) {
  const Rccl& R = rccl();
  const size_t E = m->elem_bytes / 8, piece = kMaxPeerBytes / 8;
  if (R.GroupStart() != ncclSuccess) return NTT_ERR_RCCL;
  ncclResult_t st = ncclSuccess;
  for (int g = 0; g < m->ngpus && st == ncclSuccess; ++g) {
    (void)hipSetDevice(m->dev[g]);  // inside the group: RCCL calls carry their communicator's device
    auto* sb = static_cast<uint64_t*>(send[g]);
    auto* rb = static_cast<uint64_t*>(recv[g]);
    for (int h = 0; h < m->ngpus && st == ncclSuccess; ++h)
      for (const Run& u : runs) {
        const size_t base = (h * peer_elems + u.off) * E, words = u.len * E;
        for (size_t off = 0; off < words && st == ncclSuccess; off += piece) {
          const size_t cnt = words - off < piece ? words - off : piece;
          st = R.Send(sb + base + off, cnt, ncclUint64, h, m->comm[g], m->cstream[g]);
          if (st == ncclSuccess) st = R.Recv(rb + base + off, cnt, ncclUint64, h, m->comm[g], m->cstream[g]);
        }
      }
  }
  const ncclResult_t end = R.GroupEnd();
  return (st == ncclSuccess && end == ncclSuccess) ? NTT_OK : abort_comms(m);
}

// comm stream of every device waits for the work enqueued so far on its compute stream
int order_comm_after_compute(ntt_mplan* m, void* const* streams) {
  for (int g = 0; g < m->ngpus; ++g) {
    if (hipSetDevice(m->dev[g]) != hipSuccess) return NTT_ERR_HIP;
    if (hipEventRecord(m->ev_ready[g], m->stream(streams, g)) != hipSuccess ||
        hipStreamWaitEvent(m->cstream[g], m->ev_ready[g], 0) != hipSuccess)
      return NTT_ERR_HIP;
  }
  return NTT_OK;
}

// compute stream of every device waits for piece i's arrival (recorded on its comm stream)
int order_compute_after_piece(ntt_mplan* m, void* const* streams, unsigned i) {
  for (int g = 0; g < m->ngpus; ++g) {
    if (hipSetDevice(m->dev[g]) != hipSuccess) return NTT_ERR_HIP;
    if (hipStreamWaitEvent(m->stream(streams, g), m->done(g, i), 0) != hipSuccess) return NTT_ERR_HIP;
  }
  return NTT_OK;
}

int record_piece(ntt_mplan* m, unsigned i) {
  for (int g = 0; g < m->ngpus; ++g) {
    if (hipSetDevice(m->dev[g]) != hipSuccess) return NTT_ERR_HIP;
    if (hipEventRecord(m->done(g, i), m->cstream[g]) != hipSuccess) return NTT_ERR_HIP;
  }
  return NTT_OK;
}

// After a failed step the other devices may still hold queued work that reads or writes the
// caller's buffers: wait for every device's stream before reporting the error, so the caller can
// free or reuse them.
int drain(ntt_mplan* m, void* const* streams, int rc) {
  for (int g = 0; g < m->ngpus; ++g) {
    (void)hipSetDevice(m->dev[g]);
    (void)hipStreamSynchronize(m->stream(streams, g));
    if (g < (int)m->cstream.size() && m->cstream[g]) (void)hipStreamSynchronize(m->cstream[g]);
  }
  return rc;
}

int alloc_pair(std::vector<void*>& v, int g, size_t bytes) {
  if (v[g]) return NTT_OK;
  if (hipMalloc(&v[g], bytes) != hipSuccess) {
    v[g] = nullptr;
    return NTT_ERR_HIP;
  }
  return NTT_OK;
}

int ensure_pair_buffers(ntt_mplan* m) {
  if (m->send2.empty()) {
    m->send2.assign(m->ngpus, nullptr);
    m->recv2.assign(m->ngpus, nullptr);
  }
  for (int g = 0; g < m->ngpus; ++g) {
    (void)hipSetDevice(m->dev[g]);
    if (int rc = alloc_pair(m->send2, g, 2 * m->local_n() * m->elem_bytes)) return rc;
    if (int rc = alloc_pair(m->recv2, g, 2 * m->local_n() * m->elem_bytes)) return rc;
  }
  return NTT_OK;
}

// Forward of nv vectors in row layout to column layout with ONE exchange: v[k][g] is vector k's
// share on device g; the per-peer chunks of all vectors travel together ([G][nv][chunk]).
int forward_vectors(ntt_mplan* m, void* const* const* v, int nv, void* const* streams) {
  const std::vector<void*>& sb = nv == 1 ? m->send : m->send2;
  const std::vector<void*>& rb = nv == 1 ? m->recv : m->recv2;
  if (m->pieces == 1 && m->col_pieces == 1) {
    for (int g = 0; g < m->ngpus; ++g)
      for (int k = 0; k < nv; ++k)
        if (int rc = ntt_rplan_forward_rows(m->rp[g], v[k][g], sb[g], (unsigned)nv, (unsigned)k,
                                            m->stream(streams, g)))
          return rc;
    if (int rc = exchange(m, sb, rb, nv * chunk_words(m), streams)) return rc;
  } else {
    // row piece i's exchange overlaps the row transforms of piece i + 1; the last row piece goes out
    // per column piece, whose column transforms start as soon as that unit has arrived
    // one peer block = the nv vectors' r x c chunks ([G][nv][r c] send / receive buffers)
    const unsigned P = m->pieces, Q = m->col_pieces;
    const size_t c = 1ull << m->log_c, ra = (1ull << m->log_r) / P, cm = c / Q, peer = nv * peer_elems(m);
    for (unsigned i = 0; i < P; ++i) {
      for (int g = 0; g < m->ngpus; ++g)
        for (int k = 0; k < nv; ++k)
          if (int rc = ntt_rplan_forward_rows_piece(m->rp[g], v[k][g], sb[g], (unsigned)nv, (unsigned)k, i, P, Q,
                                                    m->stream(streams, g)))
            return rc;
      if (int rc = order_comm_after_compute(m, streams)) return rc;
      if (i + 1 < P) {
        if (int rc = exchange_runs(m, sb, rb, peer, {Run{i * nv * ra * c, nv * ra * c}})) return rc;
        continue;
      }
      for (unsigned q = 0; q < Q; ++q) {
        std::vector<Run> units;
        for (int k = 0; k < nv; ++k) units.push_back(Run{(i * nv + k) * ra * c + q * ra * cm, ra * cm});
        if (int rc = exchange_runs(m, sb, rb, peer, units)) return rc;
        if (int rc = record_piece(m, q)) return rc;
      }
    }
    for (unsigned q = 0; q < Q; ++q) {  // event q: unit q of the last row piece and everything before it
      if (int rc = order_compute_after_piece(m, streams, q)) return rc;
      for (int g = 0; g < m->ngpus; ++g)
        for (int k = 0; k < nv; ++k)
          if (int rc = ntt_rplan_forward_cols_piece(m->rp[g], rb[g], v[k][g], (unsigned)nv, (unsigned)k, q, P, Q,
                                                    m->stream(streams, g)))
            return rc;
    }
    return NTT_OK;
  }
  for (int g = 0; g < m->ngpus; ++g)
    for (int k = 0; k < nv; ++k)
      if (int rc = ntt_rplan_forward_cols(m->rp[g], rb[g], v[k][g], (unsigned)nv, (unsigned)k, m->stream(streams, g)))
        return rc;
  return NTT_OK;
}

// Inverse from column layout to row layout; with b (polymul) the first column pass starts from the
// pointwise product a * b and the result lands in `out`.
int inverse_vector(ntt_mplan* m, void* const* a, void* const* b, void* const* out, void* const* streams) {
  const unsigned P = m->pieces, Q = m->col_pieces;
  if (P == 1 && Q == 1) {
    for (int g = 0; g < m->ngpus; ++g)
      if (int rc = ntt_rplan_inverse_cols(m->rp[g], a[g], b ? b[g] : nullptr, m->send[g], m->stream(streams, g)))
        return rc;
    if (int rc = exchange(m, m->send, m->recv, chunk_words(m), streams)) return rc;
    for (int g = 0; g < m->ngpus; ++g)
      if (int rc = ntt_rplan_inverse_rows(m->rp[g], m->recv[g], out[g], m->stream(streams, g))) return rc;
    return NTT_OK;
  }
  // column piece q's exchange overlaps the column transforms of piece q + 1; the last column piece
  // goes out per row piece, whose inverse row transforms start as soon as that unit has arrived
  const size_t r = 1ull << m->log_r, ra = r / P, cm = (1ull << m->log_c) / Q, peer = peer_elems(m);
  for (unsigned q = 0; q < Q; ++q) {
    for (int g = 0; g < m->ngpus; ++g)
      if (int rc = ntt_rplan_inverse_cols_piece(m->rp[g], a[g], b ? b[g] : nullptr, m->send[g], q, P, Q,
                                                m->stream(streams, g)))
        return rc;
    if (int rc = order_comm_after_compute(m, streams)) return rc;
    if (q + 1 < Q) {
      if (int rc = exchange_runs(m, m->send, m->recv, peer, {Run{q * r * cm, r * cm}})) return rc;
      continue;
    }
    for (unsigned i = 0; i < P; ++i) {
      if (int rc = exchange_runs(m, m->send, m->recv, peer, {Run{q * r * cm + i * ra * cm, ra * cm}})) return rc;
      if (int rc = record_piece(m, i)) return rc;
    }
  }
  for (unsigned i = 0; i < P; ++i) {
    if (int rc = order_compute_after_piece(m, streams, i)) return rc;
    for (int g = 0; g < m->ngpus; ++g)
      if (int rc = ntt_rplan_inverse_rows_piece(m->rp[g], m->recv[g], out[g], i, P, Q, m->stream(streams, g)))
        return rc;
  }
  return NTT_OK;
}

}  // namespace

extern "C" {

int ntt_mplan_create(ntt_mplan** out, int field_id, unsigned log_n, unsigned limbs64, int ngpus, const int* devices) {
  if (!out || ngpus < 1 || (ngpus & (ngpus - 1)) || !devices) return NTT_ERR_ARG;
  *out = nullptr;
  DeviceGuard guard;
  auto m = new ntt_mplan();
  m->ngpus = ngpus;
  m->log_n = log_n;
  m->log_g = (unsigned)__builtin_ctz((unsigned)ngpus);
  if (m->log_g > log_n / 2) { delete m; return NTT_ERR_ARG; }
  m->dev.assign(devices, devices + ngpus);
  m->rp.assign(ngpus, nullptr);
  m->send.assign(ngpus, nullptr);
  m->recv.assign(ngpus, nullptr);
  int rc = NTT_OK;
  for (int g = 0; g < ngpus && rc == NTT_OK; ++g) {
    if (hipSetDevice(devices[g]) != hipSuccess) { rc = NTT_ERR_HIP; break; }
    rc = ntt_rplan_create(&m->rp[g], field_id, log_n, limbs64, ngpus, g, devices[g]);
    if (rc == NTT_OK) {
      unsigned eb = 0, l1 = 0, l2 = 0;
      ntt_rplan_info(m->rp[g], nullptr, nullptr, &l1, &l2, &eb);
      m->elem_bytes = eb;
      m->log_n1 = l1;  // the rank plans' split (the same on every device)
      m->log_n2 = l2;
      m->log_r = l1 - m->log_g;
      m->log_c = l2 - m->log_g;
      if (alloc_pair(m->send, g, m->local_n() * eb) || alloc_pair(m->recv, g, m->local_n() * eb)) rc = NTT_ERR_HIP;
    }
  }
  if (rc == NTT_OK) {
    m->comm.assign(ngpus, nullptr);
    if (!rccl().ok() || rccl().CommInitAll(m->comm.data(), ngpus, devices) != ncclSuccess) rc = NTT_ERR_RCCL;
  }
  if (rc == NTT_OK) {
    m->cstream.assign(ngpus, nullptr);
    m->ev_ready.assign(ngpus, nullptr);
    m->ev_done.assign((size_t)ngpus * ntt_mplan::kMaxPieces, nullptr);
    for (int g = 0; g < ngpus && rc == NTT_OK; ++g) {
      (void)hipSetDevice(devices[g]);
      if (hipStreamCreateWithFlags(&m->cstream[g], hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&m->ev_ready[g], hipEventDisableTiming) != hipSuccess)
        rc = NTT_ERR_HIP;
      for (unsigned i = 0; i < ntt_mplan::kMaxPieces && rc == NTT_OK; ++i)
        if (hipEventCreateWithFlags(&m->ev_done[g * ntt_mplan::kMaxPieces + i], hipEventDisableTiming) != hipSuccess)
          rc = NTT_ERR_HIP;
    }
    // one whole-block exchange per transform by default (DistNTT.auto_pieces): the pipelined pieces
    // never measured a gain on one GPU and their timings varied run to run, so they
    // are opt-in (ntt_mplan_set_pieces2) until a multi-GPU node shows that they win
    m->pieces = m->col_pieces = 1;
  }
  if (rc != NTT_OK) {
    delete m;
    return rc;
  }
  *out = m;
  return NTT_OK;
}

int ntt_forward_multi(ntt_mplan* m, void* const* d_data, void* const* streams) {
  if (!m || !d_data) return NTT_ERR_ARG;
  if (m->broken) return NTT_ERR_RCCL;
  DeviceGuard guard;
  void* const* v[1] = {d_data};
  const int rc = forward_vectors(m, v, 1, streams);
  return rc ? drain(m, streams, rc) : NTT_OK;
}

int ntt_inverse_multi(ntt_mplan* m, void* const* d_data, void* const* streams) {
  if (!m || !d_data) return NTT_ERR_ARG;
  if (m->broken) return NTT_ERR_RCCL;
  DeviceGuard guard;
  const int rc = inverse_vector(m, d_data, nullptr, d_data, streams);
  return rc ? drain(m, streams, rc) : NTT_OK;
}

int ntt_polymul_multi(ntt_mplan* m, void* const* d_a, void* const* d_b, void* const* d_c, void* const* streams) {
  if (!m || !d_a || !d_b || !d_c) return NTT_ERR_ARG;
  if (m->broken) return NTT_ERR_RCCL;
  DeviceGuard guard;
  if (int rc = ensure_pair_buffers(m)) return rc;
  bool same = true;  // squaring: a == b on every device -> one forward transform
  for (int g = 0; g < m->ngpus; ++g) same = same && d_a[g] == d_b[g];
  void* const* v[2] = {d_a, d_b};
  int rc = same ? forward_vectors(m, v, 1, streams) : forward_vectors(m, v, 2, streams);
  if (rc == NTT_OK) rc = inverse_vector(m, d_a, d_b, d_c, streams);
  return rc ? drain(m, streams, rc) : NTT_OK;
}

int ntt_mplan_fill(ntt_mplan* m, void* const* d_data, int kind, uint64_t seed, void* const* streams) {
  if (!m || !d_data) return NTT_ERR_ARG;
  DeviceGuard guard;
  for (int g = 0; g < m->ngpus; ++g) {
    (void)hipSetDevice(m->dev[g]);
    if (int rc = ntt_rplan_fill(m->rp[g], d_data[g], kind, seed, m->stream(streams, g))) return rc;
  }
  return NTT_OK;
}

int ntt_mplan_set_pieces2(ntt_mplan* m, unsigned row_pieces, unsigned col_pieces) {
  if (!m || row_pieces < 1 || col_pieces < 1 || (row_pieces & (row_pieces - 1)) || (col_pieces & (col_pieces - 1)) ||
      row_pieces > ntt_mplan::kMaxPieces || col_pieces > ntt_mplan::kMaxPieces || row_pieces > (1u << m->log_r) ||
      col_pieces > (1u << m->log_c))
    return NTT_ERR_ARG;
  m->pieces = row_pieces;
  m->col_pieces = col_pieces;
  return NTT_OK;
}

int ntt_mplan_set_pieces(ntt_mplan* m, unsigned pieces) {
  // row pieces only (the round-2 entry point); a count that is not a power of two rounds down
  if (!m || pieces < 1 || pieces > ntt_mplan::kMaxPieces || pieces > (1u << m->log_r)) return NTT_ERR_ARG;
  unsigned p = 1;
  while (p * 2 <= pieces) p *= 2;
  return ntt_mplan_set_pieces2(m, p, 1);
}

int ntt_mplan_info(const ntt_mplan* m, uint64_t* local_n, unsigned* log_n1, unsigned* log_n2) {
  if (!m) return NTT_ERR_ARG;
  if (local_n) *local_n = m->local_n();
  if (log_n1) *log_n1 = m->log_n1;
  if (log_n2) *log_n2 = m->log_n2;
  return NTT_OK;
}

int ntt_mplan_destroy(ntt_mplan* m) {
  delete m;
  return NTT_OK;
}

}  // extern "C"
