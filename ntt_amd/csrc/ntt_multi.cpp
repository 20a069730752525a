// Single-process multi-GPU four-step (SURVEY §8b `ntt_mplan_*`, §8e): one plan object drives G
// devices of one node, with the transpose as ONE RCCL all-to-all over xGMI per transform.
//
// The layouts are those of ntt_amd/distributed.py (the one-process-per-GPU form of the same
// schedule): n = n1 n2, n1 = 2^ceil(L/2), n2 = 2^floor(L/2), r = n1 / G rows and c = n2 / G
// columns per device.
//   input  (row layout):    device g holds [r][n2], element (a, j2) = x[g r + a + n1 j2]
//   output (column layout): device g holds [c][n1], element (kc, k1) = X[g c + kc + n2 k1]
// Forward on every device: batched n2-point NTTs of its rows -> twiddle w_n^(j1 k2) fused with the
// pack into per-peer chunks -> all-to-all (RCCL, grouped over the devices) -> local transpose ->
// batched n1-point NTTs.  The inverse mirrors it (column layout in, row layout out).  All work is
// asynchronous on the callers' per-device streams.  The reference has no multi-GPU code.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

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
  bool ok() const { return CommInitAll && CommDestroy && AllToAll && GroupStart && GroupEnd; }
};

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = RTLD_DEFAULT;
    if (!dlsym(h, "ncclCommInitAll")) {
      h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
      if (!h) return x;
    }
    x.CommInitAll = reinterpret_cast<decltype(x.CommInitAll)>(dlsym(h, "ncclCommInitAll"));
    x.CommDestroy = reinterpret_cast<decltype(x.CommDestroy)>(dlsym(h, "ncclCommDestroy"));
    x.AllToAll = reinterpret_cast<decltype(x.AllToAll)>(dlsym(h, "ncclAllToAll"));
    x.GroupStart = reinterpret_cast<decltype(x.GroupStart)>(dlsym(h, "ncclGroupStart"));
    x.GroupEnd = reinterpret_cast<decltype(x.GroupEnd)>(dlsym(h, "ncclGroupEnd"));
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
  std::vector<ntt_plan*> rows, cols, tw;
  std::vector<void*> send, recv;
  std::vector<ncclComm_t> comm;

  ~ntt_mplan() {
    int cur = 0;
    hipGetDevice(&cur);
    for (size_t g = 0; g < dev.size(); ++g) {
      hipSetDevice(dev[g]);
      if (g < comm.size() && comm[g]) rccl().CommDestroy(comm[g]);
      if (g < send.size() && send[g]) hipFree(send[g]);
      if (g < recv.size() && recv[g]) hipFree(recv[g]);
      if (g < cols.size() && cols[g] && cols[g] != rows[g]) ntt_plan_destroy(cols[g]);
      if (g < rows.size() && rows[g]) ntt_plan_destroy(rows[g]);
      if (g < tw.size() && tw[g]) ntt_plan_destroy(tw[g]);
    }
    hipSetDevice(cur);
  }
  size_t local_n() const { return 1ull << (log_n - log_g); }
  hipStream_t stream(void* const* streams, int g) const {
    return streams ? static_cast<hipStream_t>(streams[g]) : nullptr;
  }
};

namespace {

struct DeviceGuard {
  int cur = 0;
  DeviceGuard() { hipGetDevice(&cur); }
  ~DeviceGuard() { hipSetDevice(cur); }
};

int exchange(ntt_mplan* m, void* const* streams) {
  // per-peer chunk: r * c elements, moved as 64-bit words
  const size_t words = (1ull << (m->log_r + m->log_c)) * (m->elem_bytes / 8);
  const Rccl& R = rccl();
  if (R.GroupStart() != ncclSuccess) return NTT_ERR_RCCL;
  for (int g = 0; g < m->ngpus; ++g) {
    hipSetDevice(m->dev[g]);
    if (R.AllToAll(m->send[g], m->recv[g], words, ncclUint64, m->comm[g], m->stream(streams, g)) != ncclSuccess) {
      R.GroupEnd();
      return NTT_ERR_RCCL;
    }
  }
  return R.GroupEnd() == ncclSuccess ? NTT_OK : NTT_ERR_RCCL;
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
  m->log_n1 = (log_n + 1) / 2;
  m->log_n2 = log_n / 2;
  if (m->log_g > m->log_n2) { delete m; return NTT_ERR_ARG; }
  m->log_r = m->log_n1 - m->log_g;
  m->log_c = m->log_n2 - m->log_g;
  m->elem_bytes = 8 * limbs64;
  m->dev.assign(devices, devices + ngpus);
  m->rows.assign(ngpus, nullptr);
  m->cols.assign(ngpus, nullptr);
  m->tw.assign(ngpus, nullptr);
  m->send.assign(ngpus, nullptr);
  m->recv.assign(ngpus, nullptr);
  int rc = NTT_OK;
  for (int g = 0; g < ngpus && rc == NTT_OK; ++g) {
    if (hipSetDevice(devices[g]) != hipSuccess) { rc = NTT_ERR_HIP; break; }
    rc = ntt_plan_create(&m->rows[g], field_id, m->log_n2, limbs64, devices[g]);
    if (rc == NTT_OK)
      rc = (m->log_n1 == m->log_n2) ? (m->cols[g] = m->rows[g], NTT_OK)
                                    : ntt_plan_create(&m->cols[g], field_id, m->log_n1, limbs64, devices[g]);
    if (rc == NTT_OK) rc = ntt_plan_create_ex(&m->tw[g], field_id, log_n, limbs64, devices[g], NTT_PLAN_TWIDDLE_ONLY);
    if (rc == NTT_OK && (hipMalloc(&m->send[g], m->local_n() * m->elem_bytes) != hipSuccess ||
                         hipMalloc(&m->recv[g], m->local_n() * m->elem_bytes) != hipSuccess))
      rc = NTT_ERR_HIP;
  }
  if (rc == NTT_OK) {
    m->comm.assign(ngpus, nullptr);
    if (!rccl().ok() || rccl().CommInitAll(m->comm.data(), ngpus, devices) != ncclSuccess) rc = NTT_ERR_RCCL;
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
  DeviceGuard guard;
  const uint64_t r = 1ull << m->log_r;
  for (int g = 0; g < m->ngpus; ++g) {
    hipSetDevice(m->dev[g]);
    void* s = m->stream(streams, g);
    if (int rc = ntt_forward_batch(m->rows[g], d_data[g], (unsigned)r, s)) return rc;
    if (int rc = ntt_twiddle_pack(m->tw[g], d_data[g], m->send[g], m->log_r, m->log_n2, m->log_c, (uint64_t)g * r,
                                  0, s))
      return rc;
  }
  if (int rc = exchange(m, streams)) return rc;
  for (int g = 0; g < m->ngpus; ++g) {
    hipSetDevice(m->dev[g]);
    void* s = m->stream(streams, g);
    // recv = [G][r][c] = [n1][c] -> [c][n1]
    if (int rc = ntt_transpose(m->tw[g], m->recv[g], d_data[g], m->log_n1, m->log_c, s)) return rc;
    if (int rc = ntt_forward_batch(m->cols[g], d_data[g], 1u << m->log_c, s)) return rc;
  }
  return NTT_OK;
}

int ntt_inverse_multi(ntt_mplan* m, void* const* d_data, void* const* streams) {
  if (!m || !d_data) return NTT_ERR_ARG;
  DeviceGuard guard;
  const uint64_t c = 1ull << m->log_c;
  for (int g = 0; g < m->ngpus; ++g) {
    hipSetDevice(m->dev[g]);
    void* s = m->stream(streams, g);
    if (int rc = ntt_inverse_batch(m->cols[g], d_data[g], (unsigned)c, s)) return rc;
    if (int rc = ntt_twiddle_pack(m->tw[g], d_data[g], m->send[g], m->log_c, m->log_n1, m->log_r, (uint64_t)g * c,
                                  1, s))
      return rc;
  }
  if (int rc = exchange(m, streams)) return rc;
  for (int g = 0; g < m->ngpus; ++g) {
    hipSetDevice(m->dev[g]);
    void* s = m->stream(streams, g);
    // recv = [G][c][r] = [n2][r] -> [r][n2]
    if (int rc = ntt_transpose(m->tw[g], m->recv[g], d_data[g], m->log_n2, m->log_r, s)) return rc;
    if (int rc = ntt_inverse_batch(m->rows[g], d_data[g], 1u << m->log_r, s)) return rc;
  }
  return NTT_OK;
}

int ntt_mplan_fill(ntt_mplan* m, void* const* d_data, int kind, uint64_t seed, void* const* streams) {
  if (!m || !d_data) return NTT_ERR_ARG;
  DeviceGuard guard;
  for (int g = 0; g < m->ngpus; ++g) {
    hipSetDevice(m->dev[g]);
    // local element i = (a, j2) -> global row g r + a, column j2: j = g r + a + n1 j2
    if (int rc = ntt_fill_map(m->tw[g], d_data[g], m->local_n(), kind, seed, (uint64_t)g << m->log_r, m->log_n2,
                              m->log_n1, m->stream(streams, g)))
      return rc;
  }
  return NTT_OK;
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
