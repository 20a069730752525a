/* Compiled drop-in caller of libntt.so through include/ntt.h — plain C, no Python, no ctypes.
 *
 * It mirrors the reference's own self-checking mains, which are the only callers of its NTT entry
 * points: GZKP-NTT.cu:1560-1721 (x_j = j at n = 2^26, SSIP(data_d, root, bits) at :1710),
 * big-num.cu:389-467 (NTT_GZKP<TPI,BITS>(data_d, length, reverse2_d, reverse_num, prime, omega, 5, 8)
 * at :458 for n = 2^5 .. 2^12 over cgbn_mem_t<256> with prime = P, omega = root) and
 * parallel-load.cu:258-346 (NTT_GZKP(data_d, reverse2_d, length, root, 7, 8, reverse_num) at :319).
 * The reference mains compare with their CPU NTT; this program prints what it computed
 * ("<entry> <log_n> <k> <value>") and tests/test_gpu_dropin_c.py compares it with the reference's
 * outputs (tests/golden/ref_p469762049.npz) and the closed-form KAT.
 *
 * Build: tests/test_gpu_dropin_c.py (gcc -std=c11 against include/ntt.h, -lntt -lamdhip64).
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ntt.h"

#define P 469762049ll /* GZKP-NTT.cu:7 */
#define ROOT 3ll      /* GZKP-NTT.cu:8 */

static int fail(const char* what, int rc) {
  fprintf(stderr, "FAIL %s: %d (%s)\n", what, rc, ntt_strerror(rc));
  return 1;
}

#define HIPCHECK(x)                                                  \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "FAIL %s: %s\n", #x, hipGetErrorString(e_));   \
      return 1;                                                      \
    }                                                                \
  } while (0)

/* sampled outputs of an n-point transform held in host memory */
static void print_samples(const char* tag, unsigned log_n, const long long* v, size_t stride) {
  const size_t n = (size_t)1 << log_n;
  const size_t ks[6] = {0, 1, 2, 3, n / 2, n - 1};
  for (int i = 0; i < 6; ++i) printf("%s %u %zu %lld\n", tag, log_n, ks[i], v[ks[i] * stride]);
}

/* SSIP: GZKP-NTT.cu main, n = 2^26, x_j = j, in place on a device long long buffer */
static int run_ssip(void) {
  const unsigned bits = 26;
  const size_t n = (size_t)1 << bits;
  long long* h = (long long*)malloc(n * sizeof(long long));
  long long* d = NULL;
  for (size_t i = 0; i < n; ++i) h[i] = (long long)i;
  HIPCHECK(hipMalloc((void**)&d, n * sizeof(long long)));
  HIPCHECK(hipMemcpy(d, h, n * sizeof(long long), hipMemcpyHostToDevice));
  SSIP(d, ROOT, bits);
  if (ntt_last_error() != NTT_OK) return fail("SSIP", ntt_last_error());
  HIPCHECK(hipMemcpy(h, d, n * sizeof(long long), hipMemcpyDeviceToHost));
  print_samples("SSIP", bits, h, 1);
  HIPCHECK(hipFree(d));
  free(h);
  return 0;
}

/* The SSIP call site with no plan scratch (NTT_PLAN_IN_PLACE): the reference's self-sort-in-place
 * property kept (GZKP-NTT.cu:1359-1449), n = 2^26, x_j = j, the same outputs as SSIP. */
static int run_inplace(void) {
  const unsigned bits = 26;
  const size_t n = (size_t)1 << bits;
  ntt_plan* plan = NULL;
  int rc = ntt_plan_create_ex(&plan, NTT_FIELD_P469762049, bits, 1, 0, NTT_PLAN_IN_PLACE);
  if (rc != NTT_OK) return fail("ntt_plan_create_ex(NTT_PLAN_IN_PLACE)", rc);
  long long* h = (long long*)malloc(n * sizeof(long long));
  long long* d = NULL;
  for (size_t i = 0; i < n; ++i) h[i] = (long long)i;
  HIPCHECK(hipMalloc((void**)&d, n * sizeof(long long)));
  HIPCHECK(hipMemcpy(d, h, n * sizeof(long long), hipMemcpyHostToDevice));
  if ((rc = ntt_forward(plan, d, NULL)) != NTT_OK) return fail("ntt_forward (in place)", rc);
  HIPCHECK(hipMemcpy(h, d, n * sizeof(long long), hipMemcpyDeviceToHost));
  print_samples("INPLACE_SSIP", bits, h, 1);
  if ((rc = ntt_inverse(plan, d, NULL)) != NTT_OK) return fail("ntt_inverse (in place)", rc);
  HIPCHECK(hipMemcpy(h, d, n * sizeof(long long), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n; ++i)
    if (h[i] != (long long)i) return fail("in-place inverse round trip", -102);
  printf("INPLACE_ROUNDTRIP %u ok\n", bits);
  ntt_plan_destroy(plan);
  HIPCHECK(hipFree(d));
  free(h);
  return 0;
}

/* NTT_GZKP<8,256>: big-num.cu main, n = 2^5 .. 2^12, cgbn_mem_t<256> (8 x u32 LE) elements */
static int run_gzkp256(void) {
  uint32_t prime[8] = {0}, omega[8] = {0};
  prime[0] = (uint32_t)P; /* int64_to_cgbn<BITS>(P) */
  omega[0] = (uint32_t)ROOT;
  for (unsigned bits = 5; bits <= 12; ++bits) {
    const size_t n = (size_t)1 << bits;
    uint32_t* h = (uint32_t*)calloc(n * 8, sizeof(uint32_t));
    uint32_t* d = NULL;
    for (size_t i = 0; i < n; ++i) h[8 * i] = (uint32_t)i;
    HIPCHECK(hipMalloc((void**)&d, n * 32));
    HIPCHECK(hipMemcpy(d, h, n * 32, hipMemcpyHostToDevice));
    const int rc = NTT_GZKP_256(d, (uint32_t)n, NULL, 0, prime, omega, 5, 8);
    if (rc != NTT_OK) return fail("NTT_GZKP_256", rc);
    HIPCHECK(hipMemcpy(h, d, n * 32, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; ++i) {
      for (int w = 1; w < 8; ++w)
        if (h[8 * i + w]) return fail("NTT_GZKP_256 upper words", -100);
      printf("GZKP256 %u %zu %u\n", bits, i, h[8 * i]);
    }
    HIPCHECK(hipFree(d));
    free(h);
  }
  return 0;
}

/* NTT_GZKP (64-bit): parallel-load.cu main, n = 2^26, x_j = j, B = 7, G = 8 */
static int run_gzkp64(void) {
  const unsigned bits = 26;
  const size_t n = (size_t)1 << bits;
  long long* h = (long long*)malloc(n * sizeof(long long));
  long long* d = NULL;
  for (size_t i = 0; i < n; ++i) h[i] = (long long)i;
  HIPCHECK(hipMalloc((void**)&d, n * sizeof(long long)));
  HIPCHECK(hipMemcpy(d, h, n * sizeof(long long), hipMemcpyHostToDevice));
  const int rc = NTT_GZKP_64(d, NULL, (long long)n, ROOT, 7, 8, 0);
  if (rc != NTT_OK) return fail("NTT_GZKP_64", rc);
  HIPCHECK(hipMemcpy(h, d, n * sizeof(long long), hipMemcpyDeviceToHost));
  print_samples("GZKP64", bits, h, 1);
  HIPCHECK(hipFree(d));
  free(h);
  return 0;
}

/* Plan API on its own stream: BN254 Fr 2^20 forward of x_j = j, then the inverse round trip. */
static int run_plan(void) {
  const unsigned bits = 20;
  const size_t n = (size_t)1 << bits;
  ntt_plan* plan = NULL;
  hipStream_t s;
  int rc = ntt_plan_create(&plan, NTT_FIELD_BN254_FR, bits, 4, 0);
  if (rc != NTT_OK) return fail("ntt_plan_create", rc);
  HIPCHECK(hipStreamCreate(&s));
  uint64_t* h = (uint64_t*)calloc(n * 4, sizeof(uint64_t));
  void* d = NULL;
  for (size_t i = 0; i < n; ++i) h[4 * i] = i;
  HIPCHECK(hipMalloc(&d, n * 32));
  HIPCHECK(hipMemcpyAsync(d, h, n * 32, hipMemcpyHostToDevice, s));
  if ((rc = ntt_forward(plan, d, s)) != NTT_OK) return fail("ntt_forward", rc);
  HIPCHECK(hipMemcpyAsync(h, d, n * 32, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  const size_t ks[4] = {0, 1, n / 2, n - 1};
  for (int i = 0; i < 4; ++i) {
    const uint64_t* e = h + 4 * ks[i];
    printf("PLAN_BN254 %u %zu %016llx%016llx%016llx%016llx\n", bits, ks[i], (unsigned long long)e[3],
           (unsigned long long)e[2], (unsigned long long)e[1], (unsigned long long)e[0]);
  }
  if ((rc = ntt_inverse(plan, d, s)) != NTT_OK) return fail("ntt_inverse", rc);
  HIPCHECK(hipMemcpyAsync(h, d, n * 32, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  for (size_t i = 0; i < n; ++i)
    if (h[4 * i] != i || h[4 * i + 1] || h[4 * i + 2] || h[4 * i + 3]) return fail("inverse round trip", -101);
  printf("PLAN_BN254_ROUNDTRIP %u ok\n", bits);
  ntt_plan_destroy(plan);
  HIPCHECK(hipStreamDestroy(s));
  HIPCHECK(hipFree(d));
  free(h);
  return 0;
}

/* error paths through the same header */
static int run_errors(void) {
  ntt_plan* plan = NULL;
  uint32_t prime[8] = {(uint32_t)P}, omega[8] = {(uint32_t)ROOT};
  if (ntt_plan_create(&plan, NTT_FIELD_BN254_FR, 10, 7, 0) != NTT_ERR_ARG) return fail("limbs64 = 7 accepted", 0);
  if (ntt_plan_create(&plan, 9, 10, 4, 0) != NTT_ERR_ARG) return fail("field 9 accepted", 0);
  if (ntt_plan_create(&plan, NTT_FIELD_P469762049, 27, 1, 0) != NTT_ERR_FIELD) return fail("2^27 | P-1 accepted", 0);
  if (NTT_GZKP_256(NULL, 48, NULL, 0, prime, omega, 5, 8) != NTT_ERR_ARG) return fail("len 48 accepted", 0);
  if (ntt_last_error() != NTT_ERR_ARG) return fail("ntt_last_error", ntt_last_error());
  printf("ERRORS ok\n");
  return 0;
}

/* `dropin bench [log_n] [steps]`: the headline transform timed from C alone (no Python): a BN254 Fr
 * plan, vector B (seed 2) via ntt_fill, 50 warm-up forwards past the clock ramp, then `steps`
 * forwards between two HIP events on the plan's stream.  Not part of "all". */
static int run_bench(int argc, char** argv) {
  const unsigned bits = argc > 2 ? (unsigned)atoi(argv[2]) : 24;
  const int steps = argc > 3 ? atoi(argv[3]) : 100;
  ntt_plan* plan = NULL;
  hipStream_t s;
  hipEvent_t e0, e1;
  void* d = NULL;
  int rc = ntt_plan_create(&plan, NTT_FIELD_BN254_FR, bits, 4, 0);
  if (rc != NTT_OK) return fail("ntt_plan_create", rc);
  HIPCHECK(hipStreamCreate(&s));
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  HIPCHECK(hipMalloc(&d, ((size_t)1 << bits) * 32));
  if ((rc = ntt_fill(plan, d, 1, 2, s)) != NTT_OK) return fail("ntt_fill", rc);
  for (int i = 0; i < 50; ++i)
    if ((rc = ntt_forward(plan, d, s)) != NTT_OK) return fail("ntt_forward", rc);
  HIPCHECK(hipEventRecord(e0, s));
  for (int i = 0; i < steps; ++i)
    if ((rc = ntt_forward(plan, d, s)) != NTT_OK) return fail("ntt_forward", rc);
  HIPCHECK(hipEventRecord(e1, s));
  HIPCHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
  printf("BENCH_BN254 2^%u forward: %.4f ms per transform, %.4g field-elements/s (%d steps)\n", bits,
         ms / steps, (double)((size_t)1 << bits) / (ms / steps * 1e-3), steps);
  ntt_plan_destroy(plan);
  HIPCHECK(hipFree(d));
  HIPCHECK(hipEventDestroy(e0));
  HIPCHECK(hipEventDestroy(e1));
  HIPCHECK(hipStreamDestroy(s));
  return 0;
}

int main(int argc, char** argv) {
  const char* which = argc > 1 ? argv[1] : "all";
  if (!strcmp(which, "bench")) return run_bench(argc, argv);
  int all = strcmp(which, "all") == 0;
  if ((all || !strcmp(which, "ssip")) && run_ssip()) return 1;
  if ((all || !strcmp(which, "gzkp256")) && run_gzkp256()) return 1;
  if ((all || !strcmp(which, "gzkp64")) && run_gzkp64()) return 1;
  if ((all || !strcmp(which, "plan")) && run_plan()) return 1;
  if ((all || !strcmp(which, "inplace")) && run_inplace()) return 1;
  if ((all || !strcmp(which, "errors")) && run_errors()) return 1;
  printf("DONE\n");
  return 0;
}
