/* Stand-in for the RCCL entry points libntt's multi-GPU plan resolves (ntt_amd/csrc/ntt_multi.cpp,
 * loaded through NTT_RCCL_LIBRARY by tests/test_gpu_mplan_faults.py and tests/test_gpu_mplan_copy.py).
 * Test-only; host functions only (the copies are hipMemcpyAsync calls).
 *
 * NTT_STUB_MODE=copy: a working single-GPU RCCL.  The "devices" of ncclCommInitAll may repeat (the one
 * GPU G times); communicator i is rank i.  Inside a group, ncclSend / ncclRecv / ncclAllToAll are
 * queued; ncclGroupEnd pairs every send of rank g to peer h with the next receive of rank h from g
 * (FIFO per pair), checks that the counts agree and that every run lies inside the allocation its
 * pointer belongs to (hipMemGetAddressRange), and then copies each pair on the receiver's stream,
 * ordered after the sender's stream and before the sender's later work (events both ways).  Any
 * mismatch or out-of-allocation run fails the group (ncclInvalidUsage) and counts a violation
 * (stub_violations()); stub_bytes() reports the bytes copied.
 *
 * Otherwise (fault mode), communicator set-up succeeds and data-path calls fail:
 *   * NTT_STUB_OK_CALLS unset or 0: every call fails with ncclSystemError (2) -- a failure on the
 *     first device of a group, before any peer has posted;
 *   * NTT_STUB_OK_CALLS = k > 0: the first k calls "succeed" and the later ones fail -- a failure on
 *     device g > 0 after devices 0..g-1 posted their part.  A successful call behaves like a posted
 *     collective whose peers never arrive: it enqueues a host function on its stream that blocks
 *     until ncclCommAbort is called (or, after 20 s, gives up and records a hang), so a caller that
 *     drains its streams without aborting the communicators hangs exactly as it would on RCCL.
 * stub_aborts() / stub_hung() report what happened.  Build:
 *   gcc -shared -fPIC -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include rccl_stub.c -L/opt/rocm/lib -lamdhip64 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

typedef void* ncclComm_t;
typedef int ncclResult_t;
#define MAX_RANKS 64
static char fake_comm[MAX_RANKS];
static volatile int g_aborted = 0, g_hung = 0, g_aborts = 0;
static int g_calls = 0;

int stub_aborts(void) { return g_aborts; }
int stub_hung(void) { return g_hung; }

static int copy_mode(void) {
  const char* m = getenv("NTT_STUB_MODE");
  return m && strcmp(m, "copy") == 0;
}

/* ------------------------------------------------------------------ fault mode */
static void blocker(void* arg) {
  (void)arg;
  for (int i = 0; i < 2000 && !g_aborted; ++i) usleep(10000);
  if (!g_aborted) g_hung = 1;
}

static ncclResult_t data_call(void* stream) {
  const char* v = getenv("NTT_STUB_OK_CALLS");
  const int ok = v ? atoi(v) : 0;
  if (g_calls++ < ok) {
    if (hipLaunchHostFunc((hipStream_t)stream, blocker, NULL) != hipSuccess) return 2;
    return 0;
  }
  return 2;
}

/* ------------------------------------------------------------------ copy mode */
enum { OP_SEND = 0, OP_RECV = 1, OP_A2A = 2 };
typedef struct {
  int kind, rank, peer, used;
  char* ptr;   /* send / recv buffer (A2A: send) */
  char* ptr2;  /* A2A: recv */
  size_t bytes;  /* per peer */
  hipStream_t stream;
} Op;
static Op* g_ops = NULL;
static size_t g_nops = 0, g_cap = 0;
static int g_depth = 0, g_nranks = 0;
static long long g_violations = 0, g_bytes = 0;

long long stub_violations(void) { return g_violations; }
long long stub_bytes(void) { return g_bytes; }

static size_t type_bytes(int t) {
  switch (t) {
    case 0: case 1: return 1;  /* int8 / uint8 */
    case 6: return 2;          /* float16 */
    case 2: case 3: case 7: return 4;
    default: return 8;         /* int64 / uint64 / float64 */
  }
}

static int rank_of(ncclComm_t c) { return (int)((char*)c - fake_comm); }

static void push(Op o) {
  if (g_nops == g_cap) {
    g_cap = g_cap ? 2 * g_cap : 256;
    g_ops = (Op*)realloc(g_ops, g_cap * sizeof(Op));
  }
  g_ops[g_nops++] = o;
}

/* the run [p, p + bytes) must lie inside one allocation */
static int in_allocation(const char* p, size_t bytes, const char* what, int rank, int peer) {
  void* base = NULL;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, (void*)p) != hipSuccess) {
    fprintf(stderr, "rccl_stub: %s of rank %d (peer %d) at %p: not a device allocation\n", what, rank, peer, p);
    return 0;
  }
  if (p + bytes > (char*)base + size) {
    fprintf(stderr, "rccl_stub: %s of rank %d (peer %d): %zu bytes at offset %zu overrun the %zu-byte allocation\n",
            what, rank, peer, bytes, (size_t)(p - (char*)base), size);
    return 0;
  }
  return 1;
}

/* dst on rs after src's writer (ss); ss's later work after the copy */
static int ordered_copy(char* dst, const char* src, size_t bytes, hipStream_t ss, hipStream_t rs) {
  hipEvent_t a, b;
  if (hipEventCreateWithFlags(&a, hipEventDisableTiming) != hipSuccess) return 0;
  if (hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) return 0;
  int ok = hipEventRecord(a, ss) == hipSuccess && hipStreamWaitEvent(rs, a, 0) == hipSuccess &&
           hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, rs) == hipSuccess &&
           hipEventRecord(b, rs) == hipSuccess && hipStreamWaitEvent(ss, b, 0) == hipSuccess;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  g_bytes += (long long)bytes;
  return ok;
}

static ncclResult_t flush_group(void) {
  int bad = 0;
  /* all-to-alls: rank g's send block h -> rank h's recv block g; all ranks of the group must be present */
  for (size_t i = 0; i < g_nops; ++i) {
    Op* o = &g_ops[i];
    if (o->kind != OP_A2A || o->used) continue;
    Op* part[MAX_RANKS] = {0};
    for (size_t j = i; j < g_nops; ++j)
      if (g_ops[j].kind == OP_A2A && !g_ops[j].used && !part[g_ops[j].rank]) part[g_ops[j].rank] = &g_ops[j];
    for (int g = 0; g < g_nranks; ++g)
      if (!part[g] || part[g]->bytes != o->bytes) {
        fprintf(stderr, "rccl_stub: all-to-all without a matching part from rank %d\n", g);
        bad = 1;
      }
    if (bad) break;
    for (int g = 0; g < g_nranks; ++g) {
      part[g]->used = 1;
      bad |= !in_allocation(part[g]->ptr, o->bytes * g_nranks, "all-to-all send", g, -1);
      bad |= !in_allocation(part[g]->ptr2, o->bytes * g_nranks, "all-to-all recv", g, -1);
    }
    for (int g = 0; g < g_nranks && !bad; ++g)
      for (int h = 0; h < g_nranks && !bad; ++h)
        bad |= !ordered_copy(part[h]->ptr2 + (size_t)g * o->bytes, part[g]->ptr + (size_t)h * o->bytes, o->bytes,
                             part[g]->stream, part[h]->stream);
  }
  /* point to point: FIFO per (sender, receiver) pair */
  for (size_t i = 0; i < g_nops && !bad; ++i) {
    Op* s = &g_ops[i];
    if (s->kind != OP_SEND || s->used) continue;
    Op* r = NULL;
    for (size_t j = 0; j < g_nops; ++j)
      if (g_ops[j].kind == OP_RECV && !g_ops[j].used && g_ops[j].rank == s->peer && g_ops[j].peer == s->rank) {
        r = &g_ops[j];
        break;
      }
    if (!r || r->bytes != s->bytes) {
      fprintf(stderr, "rccl_stub: send %d -> %d of %zu bytes has no matching receive\n", s->rank, s->peer, s->bytes);
      bad = 1;
      break;
    }
    s->used = r->used = 1;
    bad |= !in_allocation(s->ptr, s->bytes, "send", s->rank, s->peer);
    bad |= !in_allocation(r->ptr, r->bytes, "recv", r->rank, r->peer);
    if (!bad) bad |= !ordered_copy(r->ptr, s->ptr, s->bytes, s->stream, r->stream);
  }
  for (size_t i = 0; i < g_nops && !bad; ++i)
    if (!g_ops[i].used) {
      fprintf(stderr, "rccl_stub: unmatched %s of rank %d\n", g_ops[i].kind == OP_RECV ? "receive" : "call",
              g_ops[i].rank);
      bad = 1;
    }
  g_nops = 0;
  if (bad) ++g_violations;
  return bad ? 5 /* ncclInvalidUsage */ : 0;
}

/* ------------------------------------------------------------------ entry points */
ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist) {
  (void)devlist;
  if (ndev > MAX_RANKS) return 4;
  for (int i = 0; i < ndev; ++i) comm[i] = &fake_comm[i];
  g_nranks = ndev;
  return 0;
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  (void)comm;
  return 0;
}
ncclResult_t ncclCommAbort(ncclComm_t comm) {
  (void)comm;
  g_aborted = 1;
  ++g_aborts;
  return 0;
}
ncclResult_t ncclGroupStart(void) {
  ++g_depth;
  return 0;
}
ncclResult_t ncclGroupEnd(void) {
  if (g_depth > 0) --g_depth;
  return (copy_mode() && g_depth == 0) ? flush_group() : 0;
}
ncclResult_t ncclAllToAll(const void* s, void* r, size_t count, int type, ncclComm_t comm, void* stream) {
  if (!copy_mode()) return data_call(stream);
  Op o = {OP_A2A, rank_of(comm), -1, 0, (char*)s, (char*)r, count * type_bytes(type), (hipStream_t)stream};
  push(o);
  return g_depth ? 0 : flush_group();
}
ncclResult_t ncclSend(const void* s, size_t count, int type, int peer, ncclComm_t comm, void* stream) {
  if (!copy_mode()) return data_call(stream);
  Op o = {OP_SEND, rank_of(comm), peer, 0, (char*)s, NULL, count * type_bytes(type), (hipStream_t)stream};
  push(o);
  return g_depth ? 0 : flush_group();
}
ncclResult_t ncclRecv(void* r, size_t count, int type, int peer, ncclComm_t comm, void* stream) {
  if (!copy_mode()) return data_call(stream);
  Op o = {OP_RECV, rank_of(comm), peer, 0, (char*)r, NULL, count * type_bytes(type), (hipStream_t)stream};
  push(o);
  return g_depth ? 0 : flush_group();
}
