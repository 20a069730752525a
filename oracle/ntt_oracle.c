/* CPU oracle for the NTT hot path — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain C (gcc) restatement of the reference's CPU transform, used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg.  Nothing in ntt_amd/ links or
 * loads this library.
 *
 *   oracle_ntt_u64   — NTT() of src/GZKP-NTT.cu:30-48 (64-bit path, any prime < 2^31): bit-reverse
 *                      (reverse table GZKP-NTT.cu:1580-1582) then radix-2 DIT, stage twiddle
 *                      gap = qpow(root, (P-1)/(stride<<1)), w advanced by w = gap*w per offset.
 *   oracle_ssip_u64  — NTT_pro1 + NTT_pro2 of src/self-sort-in-place.cu:79-128.
 *   oracle_ntt_mp    — the same DIT definition for a multi-precision prime of 1..6 64-bit limbs
 *                      (src/big-num.cu:37-55 applied to cgbn_mem_t<bits> data; the reference's
 *                      256-bit path is modulus-generic, big-num.cu:68,173).  Elements are canonical,
 *                      little-endian limbs; modular products are Montgomery (R = 2^(64*limbs)) with
 *                      explicit to/from conversion, mirroring bn2mont/mont_mul/mont2bn
 *                      (impl_cuda.cu:980-1024) semantically.
 *   inverse          — GZKP-NTT.cu:1725-1732: forward with inv(root), then multiply by inv(n).
 *   oracle_eval_random_mp — the definition X_k = sum_j x_j w^(jk) (GZKP-NTT.cu:30-48) evaluated
 *                      directly at sampled k for SURVEY §8d's synthetic vector B generated on the
 *                      fly: spot checks of 2^28 transforms (C4) without an FFT or an 8-GiB copy.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ 64-bit path */
static int64_t qpow64(int64_t x, int64_t y, int64_t p) {
  int64_t base = 1;
  x %= p;
  while (y) {
    if (y & 1) base = (int64_t)((u128)base * (uint64_t)x % (uint64_t)p);
    x = (int64_t)((u128)x * (uint64_t)x % (uint64_t)p);
    y >>= 1;
  }
  return base;
}

static void bitrev_permute64(int64_t* d, uint32_t log_n) {
  uint64_t n = 1ull << log_n;
  uint32_t* rev = (uint32_t*)calloc(n, sizeof(uint32_t));
  for (uint64_t i = 1; i < n; i++) rev[i] = (rev[i >> 1] >> 1) | ((uint32_t)(i & 1) << (log_n - 1));
  for (uint64_t i = 0; i < n; i++)
    if (i < rev[i]) { int64_t t = d[i]; d[i] = d[rev[i]]; d[rev[i]] = t; }
  free(rev);
}

/* Forward (inverse != 0: inverse with 1/n scale) NTT over a prime p < 2^62, natural order. */
int oracle_ntt_u64(int64_t* data, uint32_t log_n, int64_t p, int64_t root, int inverse) {
  if (log_n > 40) return -1;
  uint64_t n = 1ull << log_n;
  if (inverse) root = qpow64(root, p - 2, p);
  if (log_n) bitrev_permute64(data, log_n);
  for (uint64_t stride = 1; stride < n; stride <<= 1) {
    int64_t gap = qpow64(root, (p - 1) / (int64_t)(stride << 1), p);
    for (uint64_t start = 0; start < n; start += stride << 1) {
      int64_t w = 1;
      for (uint64_t off = 0; off < stride; off++) {
        int64_t a = data[start + off];
        int64_t b = (int64_t)((u128)(uint64_t)w * (uint64_t)data[start + off + stride] % (uint64_t)p);
        data[start + off] = (a + b) % p;
        data[start + off + stride] = (a - b + p) % p;
        w = (int64_t)((u128)(uint64_t)gap * (uint64_t)w % (uint64_t)p);
      }
    }
  }
  if (inverse) {
    int64_t ni = qpow64((int64_t)(n % (uint64_t)p), p - 2, p);
    for (uint64_t i = 0; i < n; i++) data[i] = (int64_t)((u128)(uint64_t)data[i] * (uint64_t)ni % (uint64_t)p);
  }
  return 0;
}

/* NTT_pro1 + NTT_pro2: the self-sort-in-place CPU dataflow (natural in, natural out). */
int oracle_ssip_u64(int64_t* data, uint32_t log_n, int64_t p, int64_t root) {
  uint64_t len = 1ull << log_n;
  for (uint32_t i = log_n; i > log_n / 2; i--) {
    uint64_t stride = 1ull << (i - 1);
    int64_t gap = qpow64(root, (p - 1) / (int64_t)(stride << 1), p);
    for (uint64_t start = 0; start < len; start += stride << 1) {
      int64_t w = 1;
      for (uint64_t off = 0; off < stride; off++) {
        int64_t a = data[start + off], b = data[start + off + stride];
        data[start + off] = (a + b) % p;
        data[start + off + stride] = (int64_t)((u128)(uint64_t)((a - b + p) % p) * (uint64_t)w % (uint64_t)p);
        w = (int64_t)((u128)(uint64_t)gap * (uint64_t)w % (uint64_t)p);
      }
    }
  }
  for (uint32_t i = log_n / 2; i >= 1; i--) {
    uint64_t stride = 1ull << (i - 1);
    uint64_t pair_stride = 1ull << (log_n - i);
    int64_t gap = qpow64(root, (p - 1) / (int64_t)(stride << 1), p);
    for (uint64_t start = 0; start < len; start += pair_stride << 1) {
      for (uint64_t off0 = 0; off0 < pair_stride; off0 += stride << 1) {
        int64_t w = 1;
        for (uint64_t off = 0; off < stride; off++) {
          uint64_t o = start + off0 + off;
          int64_t a = data[o], b = data[o + stride], c = data[o + pair_stride], d = data[o + pair_stride + stride];
          data[o] = (a + b) % p;
          data[o + stride] = (c + d) % p;
          data[o + pair_stride] = (int64_t)((u128)(uint64_t)((a - b + p) % p) * (uint64_t)w % (uint64_t)p);
          data[o + pair_stride + stride] = (int64_t)((u128)(uint64_t)((c - d + p) % p) * (uint64_t)w % (uint64_t)p);
          w = (int64_t)((u128)(uint64_t)gap * (uint64_t)w % (uint64_t)p);
        }
      }
    }
  }
  return 0;
}

/* ------------------------------------------------------------------ multi-precision path */
#define MAXL 6
typedef struct {
  int L;             /* 64-bit limbs */
  uint64_t p[MAXL];
  uint64_t pinv;     /* -p^-1 mod 2^64 */
  uint64_t r2[MAXL]; /* R^2 mod p */
} mp_field;

static int mp_cmp(const uint64_t* a, const uint64_t* b, int L) {
  for (int i = L - 1; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i] ? 1 : -1;
  }
  return 0;
}
static uint64_t mp_add(uint64_t* r, const uint64_t* a, const uint64_t* b, int L) {
  u128 c = 0;
  for (int i = 0; i < L; i++) { c += (u128)a[i] + b[i]; r[i] = (uint64_t)c; c >>= 64; }
  return (uint64_t)c;
}
static uint64_t mp_sub(uint64_t* r, const uint64_t* a, const uint64_t* b, int L) {
  uint64_t br = 0;
  for (int i = 0; i < L; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    r[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}
static void mp_addmod(uint64_t* r, const uint64_t* a, const uint64_t* b, const mp_field* F) {
  uint64_t t[MAXL];
  uint64_t c = mp_add(t, a, b, F->L);
  if (c || mp_cmp(t, F->p, F->L) >= 0) mp_sub(t, t, F->p, F->L);
  memcpy(r, t, 8 * F->L);
}
static void mp_submod(uint64_t* r, const uint64_t* a, const uint64_t* b, const mp_field* F) {
  uint64_t t[MAXL];
  if (mp_sub(t, a, b, F->L)) mp_add(t, t, F->p, F->L);
  memcpy(r, t, 8 * F->L);
}
/* Montgomery product a*b*R^-1 mod p, CIOS with 64-bit limbs and an explicit top word. */
static void mp_montmul(uint64_t* r, const uint64_t* a, const uint64_t* b, const mp_field* F) {
  int L = F->L;
  uint64_t t[MAXL + 2];
  memset(t, 0, sizeof(t));
  for (int i = 0; i < L; i++) {
    u128 c = 0;
    for (int j = 0; j < L; j++) { c += (u128)a[j] * b[i] + t[j]; t[j] = (uint64_t)c; c >>= 64; }
    c += t[L]; t[L] = (uint64_t)c; t[L + 1] = (uint64_t)(c >> 64);
    uint64_t m = t[0] * F->pinv;
    c = (u128)m * F->p[0] + t[0];
    c >>= 64;
    for (int j = 1; j < L; j++) { c += (u128)m * F->p[j] + t[j]; t[j - 1] = (uint64_t)c; c >>= 64; }
    c += t[L]; t[L - 1] = (uint64_t)c; t[L] = t[L + 1] + (uint64_t)(c >> 64);
  }
  if (t[L] || mp_cmp(t, F->p, L) >= 0) mp_sub(t, t, F->p, L);
  memcpy(r, t, 8 * L);
}
static void mp_to_mont(uint64_t* r, const uint64_t* a, const mp_field* F) { mp_montmul(r, a, F->r2, F); }
static void mp_from_mont(uint64_t* r, const uint64_t* a, const mp_field* F) {
  uint64_t one[MAXL] = {1};
  mp_montmul(r, a, one, F);
}
static int mp_field_init(mp_field* F, const uint64_t* p, int L) {
  if (L < 1 || L > MAXL || !(p[0] & 1)) return -1;
  F->L = L;
  memcpy(F->p, p, 8 * L);
  uint64_t inv = 1;
  for (int i = 0; i < 7; i++) inv *= 2 - p[0] * inv;
  F->pinv = (uint64_t)0 - inv;
  /* R mod p by 64L doublings of 1, then R^2 = (R mod p) doubled 64L more times */
  uint64_t x[MAXL] = {1};
  for (int k = 0; k < 2 * 64 * L; k++) mp_addmod(x, x, x, F);
  memcpy(F->r2, x, 8 * L);
  return 0;
}
/* r = a^e (Montgomery domain in/out), e given as L limbs */
static void mp_pow_mont(uint64_t* r, const uint64_t* a_m, const uint64_t* e, const mp_field* F) {
  uint64_t one[MAXL] = {1}, acc[MAXL], base[MAXL];
  mp_to_mont(acc, one, F);
  memcpy(base, a_m, 8 * F->L);
  for (int i = 0; i < 64 * F->L; i++) {
    if ((e[i / 64] >> (i % 64)) & 1) mp_montmul(acc, acc, base, F);
    mp_montmul(base, base, base, F);
  }
  memcpy(r, acc, 8 * F->L);
}

/* data: n elements of `limbs64` little-endian 64-bit limbs, canonical.  g: generator (limbs64).
 * Forward NTT natural->natural (inverse != 0: inverse incl. 1/n scale).  Returns 0 on success. */
int oracle_ntt_mp(uint64_t* data, uint32_t log_n, uint32_t limbs64, const uint64_t* p, const uint64_t* g,
                  int inverse) {
  mp_field F;
  if (mp_field_init(&F, p, (int)limbs64)) return -1;
  const int L = F.L;
  const uint64_t n = 1ull << log_n;
  uint64_t pm1[MAXL], e[MAXL], gm[MAXL], one[MAXL] = {1};
  mp_sub(pm1, p, one, L);
  mp_to_mont(gm, g, &F);
  if (inverse) { /* g <- g^(p-2) */
    uint64_t two[MAXL] = {2}, pm2[MAXL];
    mp_sub(pm2, p, two, L);
    mp_pow_mont(gm, gm, pm2, &F);
  }
  /* to Montgomery domain */
  for (uint64_t i = 0; i < n; i++) mp_to_mont(data + i * L, data + i * L, &F);
  /* bit reversal */
  if (log_n) {
    uint32_t* rev = (uint32_t*)calloc(n, sizeof(uint32_t));
    for (uint64_t i = 1; i < n; i++) rev[i] = (rev[i >> 1] >> 1) | ((uint32_t)(i & 1) << (log_n - 1));
    uint64_t tmp[MAXL];
    for (uint64_t i = 0; i < n; i++)
      if (i < rev[i]) {
        memcpy(tmp, data + i * L, 8 * L);
        memcpy(data + i * L, data + (uint64_t)rev[i] * L, 8 * L);
        memcpy(data + (uint64_t)rev[i] * L, tmp, 8 * L);
      }
    free(rev);
  }
  for (uint64_t stride = 1, lg = 1; stride < n; stride <<= 1, lg++) {
    /* gap = g^((p-1)/(2*stride)) ; (p-1) >> lg */
    memset(e, 0, sizeof(e));
    for (int i = 0; i < L; i++) {
      e[i] = pm1[i] >> lg;
      if (i + 1 < L && lg) e[i] |= pm1[i + 1] << (64 - lg);
    }
    uint64_t gap[MAXL], w[MAXL], b[MAXL];
    mp_pow_mont(gap, gm, e, &F);
    for (uint64_t start = 0; start < n; start += stride << 1) {
      mp_to_mont(w, one, &F);
      for (uint64_t off = 0; off < stride; off++) {
        uint64_t* pa = data + (start + off) * L;
        uint64_t* pb = data + (start + off + stride) * L;
        mp_montmul(b, w, pb, &F);
        mp_submod(pb, pa, b, &F);
        mp_addmod(pa, pa, b, &F);
        mp_montmul(w, gap, w, &F);
      }
    }
  }
  if (inverse) {
    uint64_t nn[MAXL] = {0}, nm[MAXL], two[MAXL] = {2}, pm2[MAXL];
    nn[0] = n;  /* n < p for every supported field */
    mp_to_mont(nm, nn, &F);
    mp_sub(pm2, p, two, L);
    mp_pow_mont(nm, nm, pm2, &F);
    for (uint64_t i = 0; i < n; i++) mp_montmul(data + i * L, data + i * L, nm, &F);
  }
  for (uint64_t i = 0; i < n; i++) mp_from_mont(data + i * L, data + i * L, &F);
  return 0;
}

/* The same transform with each stage's butterflies split over `threads` OpenMP threads (chunks of
 * one block's offsets; a chunk starts from w = gap^off0).  Used only as the multi-core CPU baseline
 * of bench.py; tests check it against oracle_ntt_mp. */
int oracle_ntt_mp_par(uint64_t* data, uint32_t log_n, uint32_t limbs64, const uint64_t* p, const uint64_t* g,
                      int inverse, int threads) {
  mp_field F;
  if (mp_field_init(&F, p, (int)limbs64)) return -1;
  const int L = F.L;
  const uint64_t n = 1ull << log_n;
  uint64_t pm1[MAXL], gm[MAXL], one[MAXL] = {1};
  mp_sub(pm1, p, one, L);
  mp_to_mont(gm, g, &F);
  if (inverse) {
    uint64_t two[MAXL] = {2}, pm2[MAXL];
    mp_sub(pm2, p, two, L);
    mp_pow_mont(gm, gm, pm2, &F);
  }
  if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(static)
  for (uint64_t i = 0; i < n; i++) mp_to_mont(data + i * L, data + i * L, &F);
  if (log_n) {
    uint32_t* rev = (uint32_t*)calloc(n, sizeof(uint32_t));
    for (uint64_t i = 1; i < n; i++) rev[i] = (rev[i >> 1] >> 1) | ((uint32_t)(i & 1) << (log_n - 1));
#pragma omp parallel for num_threads(threads) schedule(static)
    for (uint64_t i = 0; i < n; i++)
      if (i < rev[i]) {
        uint64_t tmp[MAXL];
        memcpy(tmp, data + i * L, 8 * L);
        memcpy(data + i * L, data + (uint64_t)rev[i] * L, 8 * L);
        memcpy(data + (uint64_t)rev[i] * L, tmp, 8 * L);
      }
    free(rev);
  }
  const uint64_t chunk = 4096; /* butterflies per task */
  for (uint64_t stride = 1, lg = 1; stride < n; stride <<= 1, lg++) {
    uint64_t e[MAXL] = {0}, gap[MAXL];
    for (int i = 0; i < L; i++) {
      e[i] = pm1[i] >> lg;
      if (i + 1 < L && lg) e[i] |= pm1[i + 1] << (64 - lg);
    }
    mp_pow_mont(gap, gm, e, &F);
    /* a task = `bpt` whole blocks (short strides) or one `chunk`-offset slice of a block */
    const uint64_t blocks = n / (2 * stride);
    const uint64_t per_block = (stride + chunk - 1) / chunk;
    const uint64_t bpt = stride >= chunk ? 1 : (chunk / stride < blocks ? chunk / stride : blocks);
    const uint64_t tasks = stride >= chunk ? blocks * per_block : blocks / bpt;
#pragma omp parallel for num_threads(threads) schedule(static)
    for (uint64_t task = 0; task < tasks; task++) {
      uint64_t w[MAXL], b[MAXL], o[MAXL] = {0};
      uint64_t blk0 = task * bpt, off0 = 0, off1 = stride;
      if (stride >= chunk) {
        blk0 = task / per_block;
        off0 = (task % per_block) * chunk;
        off1 = off0 + chunk < stride ? off0 + chunk : stride;
      }
      for (uint64_t blk = blk0; blk < blk0 + bpt; blk++) {
        const uint64_t start = blk * 2 * stride;
        o[0] = off0;
        if (off0)
          mp_pow_mont(w, gap, o, &F);
        else
          mp_to_mont(w, one, &F);
        for (uint64_t off = off0; off < off1; off++) {
          uint64_t* pa = data + (start + off) * L;
          uint64_t* pb = data + (start + off + stride) * L;
          mp_montmul(b, w, pb, &F);
          mp_submod(pb, pa, b, &F);
          mp_addmod(pa, pa, b, &F);
          mp_montmul(w, gap, w, &F);
        }
      }
    }
  }
  if (inverse) {
    uint64_t nn[MAXL] = {0}, nm[MAXL], two[MAXL] = {2}, pm2[MAXL];
    nn[0] = n;
    mp_to_mont(nm, nn, &F);
    mp_sub(pm2, p, two, L);
    mp_pow_mont(nm, nm, pm2, &F);
#pragma omp parallel for num_threads(threads) schedule(static)
    for (uint64_t i = 0; i < n; i++) mp_montmul(data + i * L, data + i * L, nm, &F);
  }
#pragma omp parallel for num_threads(threads) schedule(static)
  for (uint64_t i = 0; i < n; i++) mp_from_mont(data + i * L, data + i * L, &F);
  return 0;
}

/* Pointwise c = a*b mod p over n multi-precision elements (polymul oracle helper). */
int oracle_mul_mp(uint64_t* c, const uint64_t* a, const uint64_t* b, uint64_t n, uint32_t limbs64,
                  const uint64_t* p) {
  mp_field F;
  if (mp_field_init(&F, p, (int)limbs64)) return -1;
  const int L = F.L;
  uint64_t am[MAXL];
  for (uint64_t i = 0; i < n; i++) {
    mp_to_mont(am, a + i * L, &F);
    mp_montmul(c + i * L, am, b + i * L, &F);
  }
  return 0;
}

/* ------------------------------------------------------------------ sampled outputs at full size
 * X_k = sum_j x_j w^(jk), w = g^((p-1)/n), of SURVEY §8d's synthetic vector B -- limb i of x_j is
 * SplitMix64(seed 2^32 + 4j + i) for i < nrand, the last of them masked to top_bits, higher limbs 0
 * (generated on the fly: a 2^28 vector is never stored) -- at `count` indices ks[].  The definition
 * of GZKP-NTT.cu:30-48 evaluated directly (no FFT): Horner over `nch` chunks of j split across
 * `threads` OpenMP threads, chunk c contributing w^(k j0_c) * sum_{j in c} x_j w^(k (j - j0_c)).
 * out: count elements of limbs64 canonical limbs.  Test infrastructure (C4 spot checks). */
static uint64_t splitmix_limb(uint64_t seed, uint64_t j, uint32_t i) {
  uint64_t z = (seed << 32) + 4 * j + i + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* mp_montmul / mp_addmod with the limb count fixed at compile time (the compiler unrolls them): the
 * evaluator's inner loop, 2^28 iterations per sample at C4 */
#define MP_FIXED(NL)                                                                                   \
  static void montmul_##NL(uint64_t* r, const uint64_t* a, const uint64_t* b, const mp_field* F) {    \
    uint64_t t[NL + 2] = {0};                                                                          \
    for (int i = 0; i < NL; i++) {                                                                     \
      u128 c = 0;                                                                                      \
      for (int j = 0; j < NL; j++) { c += (u128)a[j] * b[i] + t[j]; t[j] = (uint64_t)c; c >>= 64; }   \
      c += t[NL]; t[NL] = (uint64_t)c; t[NL + 1] = (uint64_t)(c >> 64);                                \
      uint64_t m = t[0] * F->pinv;                                                                     \
      c = (u128)m * F->p[0] + t[0];                                                                    \
      c >>= 64;                                                                                        \
      for (int j = 1; j < NL; j++) { c += (u128)m * F->p[j] + t[j]; t[j - 1] = (uint64_t)c; c >>= 64; } \
      c += t[NL]; t[NL - 1] = (uint64_t)c; t[NL] = t[NL + 1] + (uint64_t)(c >> 64);                    \
    }                                                                                                  \
    if (t[NL] || mp_cmp(t, F->p, NL) >= 0) mp_sub(t, t, F->p, NL);                                     \
    memcpy(r, t, 8 * NL);                                                                              \
  }
MP_FIXED(1)
MP_FIXED(4)
MP_FIXED(6)

typedef void (*montmul_fn)(uint64_t*, const uint64_t*, const uint64_t*, const mp_field*);

int oracle_eval_random_mp(uint64_t* out, const uint64_t* ks, uint32_t count, uint32_t log_n, uint32_t limbs64,
                          const uint64_t* p, const uint64_t* g, uint64_t seed, uint32_t nrand, uint32_t top_bits,
                          int threads) {
  mp_field F;
  if (mp_field_init(&F, p, (int)limbs64) || nrand < 1 || nrand > limbs64 || top_bits > 64) return -1;
  const int L = F.L;
  const uint64_t n = 1ull << log_n;
  if (threads < 1) threads = 1;
  uint64_t nch = 1; /* a power of two, so that chunks tile [0, n) */
  while (nch * 2 <= (uint64_t)threads * 4 && nch * 2 <= n) nch *= 2;
  const uint64_t len = n / nch;
  uint64_t pm1[MAXL], one[MAXL] = {1}, gm[MAXL], e[MAXL] = {0}, wm[MAXL];
  mp_sub(pm1, p, one, L);
  for (int i = 0; i < L; i++) {
    e[i] = log_n < 64 ? pm1[i] >> log_n : 0;
    if (i + 1 < L && log_n && log_n < 64) e[i] |= pm1[i + 1] << (64 - log_n);
  }
  mp_to_mont(gm, g, &F);
  mp_pow_mont(wm, gm, e, &F); /* w, Montgomery form */
  uint64_t* part = (uint64_t*)calloc((size_t)count * nch * L, 8);
  if (!part) return -1;
  const uint64_t mask = top_bits >= 64 ? ~0ull : ((1ull << top_bits) - 1);
  const montmul_fn mm = L == 4 ? montmul_4 : (L == 6 ? montmul_6 : (L == 1 ? montmul_1 : mp_montmul));
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
  for (uint64_t task = 0; task < (uint64_t)count * nch; task++) {
    const uint64_t s = task / nch, c = task % nch, j0 = c * len;
    uint64_t kk[MAXL] = {0}, wk[MAXL], acc[MAXL] = {0}, x[MAXL], sh[MAXL];
    kk[0] = ks[s] & (n - 1);
    mp_pow_mont(wk, wm, kk, &F); /* w^k, Montgomery form */
    for (uint64_t j = j0 + len; j-- > j0;) {
      mm(acc, acc, wk, &F); /* canonical acc times w^k */
      memset(x, 0, sizeof(x));
      for (uint32_t i = 0; i < nrand; i++) x[i] = splitmix_limb(seed, j, i);
      x[nrand - 1] &= mask;
      mp_addmod(acc, acc, x, &F);
    }
    uint64_t ej[MAXL] = {0};
    /* w^(k j0): exponent k j0 mod n (w has order n) */
    ej[0] = (kk[0] * j0) & (n - 1);
    mp_pow_mont(sh, wm, ej, &F);
    mp_montmul(part + (s * nch + c) * L, acc, sh, &F);
  }
  for (uint32_t s = 0; s < count; s++) {
    uint64_t tot[MAXL] = {0};
    for (uint64_t c = 0; c < nch; c++) mp_addmod(tot, tot, part + (s * nch + c) * L, &F);
    memcpy(out + (size_t)s * L, tot, 8 * L);
  }
  free(part);
  return 0;
}
