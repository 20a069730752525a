/* Fault-injecting stand-in for the RCCL entry points libntt's multi-GPU plan resolves
 * (ntt_amd/csrc/ntt_multi.cpp, loaded through NTT_RCCL_LIBRARY by tests/test_gpu_mplan_faults.py).
 * Test-only; no GPU code (host functions only).
 *
 * Communicator set-up succeeds.  Data-path calls (ncclAllToAll / ncclSend / ncclRecv):
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
#include <stdlib.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

typedef void* ncclComm_t;
typedef int ncclResult_t;
static char fake_comm[64];
static volatile int g_aborted = 0, g_hung = 0, g_aborts = 0;
static int g_calls = 0;

int stub_aborts(void) { return g_aborts; }
int stub_hung(void) { return g_hung; }

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

ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist) {
  (void)devlist;
  for (int i = 0; i < ndev; ++i) comm[i] = &fake_comm[i % 64];
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
ncclResult_t ncclGroupStart(void) { return 0; }
ncclResult_t ncclGroupEnd(void) { return 0; }
ncclResult_t ncclAllToAll(const void* s, void* r, size_t count, int type, ncclComm_t comm, void* stream) {
  (void)s; (void)r; (void)count; (void)type; (void)comm;
  return data_call(stream);
}
ncclResult_t ncclSend(const void* s, size_t count, int type, int peer, ncclComm_t comm, void* stream) {
  (void)s; (void)count; (void)type; (void)peer; (void)comm;
  return data_call(stream);
}
ncclResult_t ncclRecv(void* r, size_t count, int type, int peer, ncclComm_t comm, void* stream) {
  (void)r; (void)count; (void)type; (void)peer; (void)comm;
  return data_call(stream);
}
