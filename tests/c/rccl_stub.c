/* Fault-injecting stand-in for the five RCCL entry points libntt's multi-GPU plan resolves
 * (ntt_amd/csrc/ntt_multi.cpp, loaded through NTT_RCCL_LIBRARY by tests/test_gpu_mplan_faults.py).
 * Communicator set-up succeeds; every data-path call fails with ncclSystemError (2), as an RCCL
 * failure in the middle of a grouped all-to-all would.  Test-only; no GPU code. */
#include <stddef.h>
#include <stdint.h>

typedef void* ncclComm_t;
typedef int ncclResult_t;
static char fake_comm[64];

ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist) {
  (void)devlist;
  for (int i = 0; i < ndev; ++i) comm[i] = &fake_comm[i % 64];
  return 0;
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  (void)comm;
  return 0;
}
ncclResult_t ncclGroupStart(void) { return 0; }
ncclResult_t ncclGroupEnd(void) { return 0; }
ncclResult_t ncclAllToAll(const void* s, void* r, size_t count, int type, ncclComm_t comm, void* stream) {
  (void)s; (void)r; (void)count; (void)type; (void)comm; (void)stream;
  return 2;
}
ncclResult_t ncclSend(const void* s, size_t count, int type, int peer, ncclComm_t comm, void* stream) {
  (void)s; (void)count; (void)type; (void)peer; (void)comm; (void)stream;
  return 2;
}
ncclResult_t ncclRecv(void* r, size_t count, int type, int peer, ncclComm_t comm, void* stream) {
  (void)r; (void)count; (void)type; (void)peer; (void)comm; (void)stream;
  return 2;
}
