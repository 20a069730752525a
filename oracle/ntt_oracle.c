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
