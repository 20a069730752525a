/* C ABI of libntt.so — the MI355X-native drop-in for the reference's NTT host entry points.
 *
 * The reference (tie-pilot-qxw/NTT) has no library API: its entry points are C++ host drivers called
 * from main().  Each function below names the reference interface it replaces.
 *
 *   SSIP(long long* x, long long omega, uint log_n)            GZKP-NTT.cu:1452 (= self-sort-in-place.cu:309)
 *   NTT_GZKP<TPI,BITS>(cgbn_mem_t<bits> data[], uint len, uint2 reverse[], uint reverse_len,
 *                      cgbn_mem_t<bits> prime, cgbn_mem_t<bits> omega, uint B, uint G)
 *                                                               big-num.cu:260-261
 *   NTT_GZKP(long long data[], longlong2 reverse[], long long len, long long omega, int B, int G,
 *            long long reverse_num)                             parallel-load.cu:195 / GZKP-NTT.cu:167
 *   inverse: NTT(..., inv(root)) then * inv(len)               GZKP-NTT.cu:1725-1732 (commented out)
 *
 * Conventions (same as the reference unless stated):
 *   - data is a DEVICE pointer owned by the caller; transforms are in place, natural order in and
 *     out (the reference's SSIP contract), elements canonical (< p), not in Montgomery form;
 *   - element layout = cgbn_mem_t<32*W>: W little-endian 32-bit words (cgbn_cuda.h:51-55), i.e.
 *     limbs64 little-endian 64-bit limbs; the 1-limb P469762049 path uses `long long` elements;
 *   - `omega` arguments are the multiplicative GENERATOR (the reference passes `root`, 3), the
 *     n-th root is omega^((p-1)/n) (GZKP-NTT.cu:1462, big-num.cu:292-296);
 *   - unlike the reference (void, prints timings, default stream, blocking): every call returns a
 *     status (0 ok, < 0 error, see ntt_strerror), prints nothing, and the plan API is asynchronous
 *     on the given hipStream_t (NULL = default stream).  The reference-shaped shims SSIP /
 *     NTT_GZKP_256 keep the reference's blocking behaviour.
 *   - plans are thread-compatible: one plan per thread, or serialise calls on a plan.  A plan's
 *     scratch is shared by its calls, so calls on one plan must also be ordered on the device (the
 *     same stream, or streams the caller orders).  The status of the last call (ntt_last_error) is
 *     kept per thread.  The shims are thread-safe: their plan cache is locked and each cached plan
 *     runs one blocking call at a time.
 */
#ifndef NTT_AMD_NTT_H
#define NTT_AMD_NTT_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define NTT_OK 0
#define NTT_ERR_ARG (-1)      /* invalid field / size / limb count / pointer */
#define NTT_ERR_HIP (-2)      /* HIP runtime error (launch, allocation, copy) */
#define NTT_ERR_RCCL (-3)     /* RCCL error (multi-GPU) */
#define NTT_ERR_FIELD (-4)    /* modulus unsupported (even, too large, no root of unity of order n) */
#define NTT_ERR_NODEV (-5)    /* no HIP device */
#define NTT_ERR_DEVICE (-6)   /* an inter-workgroup wait of an earlier call on this plan gave up at its
                               * watchdog (in-place or single-launch schedules; never expected): that
                               * call's output is wrong.  Every call on the plan returns this until
                               * ntt_plan_device_status clears the report.  The blocking shims return it
                               * for the call itself (and clear it).  The reference asserts instead
                               * (GZKP-NTT.cu:1527). */

/* field ids */
#define NTT_FIELD_P469762049 0   /* 7*2^26+1, generator 3 (GZKP-NTT.cu:7-8) */
#define NTT_FIELD_BN254_FR 1     /* 0x30644e72...f0000001, generator 5 */
#define NTT_FIELD_BLS12_381_FR 2 /* 0x73eda753...00000001, generator 7 */

typedef struct ntt_plan ntt_plan;

/* Create a plan for 2^log_n-point transforms on `device` (twiddle tables and scratch are cached in
 * the plan: the reference rebuilt its tables on every call, GZKP-NTT.cu:1476-1500).
 * limbs64: 1 (P469762049 only, `long long` elements), 4 (256-bit, cgbn_mem_t<256>), 6 (384-bit
 * template).  Replaces the table setup inside SSIP (GZKP-NTT.cu:1452-1505) and NTT_GZKP
 * (big-num.cu:278-309). */
int ntt_plan_create(ntt_plan** out, int field_id, unsigned log_n, unsigned limbs64, int device);

/* Plan flags for the _ex constructors. */
#define NTT_PLAN_TWIDDLE_ONLY 1u /* only the w_n tables: fill / twiddle_pack / transpose, no transforms */
/* Elements are in Montgomery form x R mod p, R = 2^(64 limbs64) (CGBN's bn2mont domain,
 * impl_cuda.cu:980-1010; the form arkworks / sppark / ICICLE callers keep their data in).  The
 * transforms are linear, so forward / inverse / coset are unchanged (NTT(x R) = NTT(x) R); the
 * pointwise product becomes the Montgomery product a b R^-1 so that polymul maps (a R, b R) to
 * (a b) R.  Saves the caller a to/from-Montgomery pass over the data on each side. */
#define NTT_PLAN_MONTGOMERY_IO 2u
/* Rival schedule: forward transforms run as the reference's bellperson / improved_NTT
 * family re-derived for gfx950 — Stockham autosort passes of radix 2^r_i with the twiddle applied to
 * the INPUT of each pass (GZKP-NTT.cu:324-386 FIELD_radix_fft; :556-1296 improved_NTT_v1..v4, whose
 * grouping / coalescing / bank-conflict variants the wave64 LDS-staged kernels subsume), ping-pong
 * between two plan buffers, no final digit-reversal pass.  Same contract and results as the default
 * four-step DIF schedule; kept to measure against it (tools/bench_rivals.py).  P469762049 (1 limb)
 * and 4-limb plans, single transforms (batch 1); other calls use the default schedule. */
#define NTT_PLAN_STOCKHAM 4u
/* Rival schedule: forward transforms run as the reference's GZKP(B, G) (GZKP-NTT.cu:
 * 115-165, driver 167-233; parallel-load.cu:114-193 for P): a bit-reversal permutation pass
 * (`rearrange`), then in-place radix-2 DIT rounds, B of them per pass over tiles of G adjacent
 * columns, re-derived as: the permutation into a plan buffer, a first pass of contiguous radix-2^r_0
 * DFTs, then passes that multiply their inputs by w_N^(c d) (per-pass tables) and run radix-2^r_i
 * DFTs in place over stride-2^(r_0 + .. + r_{i-1}) columns.  Same contract and results as the
 * default schedule; P469762049 (1 limb) and 4-limb plans, single transforms (batch 1).
 * NTT_PLAN_STOCKHAM and NTT_PLAN_GZKP are exclusive. */
#define NTT_PLAN_GZKP 8u
/* In place, no scratch (the reference's self-sort-in-place property, SSIP_NTT_stage2's mirror pairs,
 * GZKP-NTT.cu:1359-1449): the plan owns no n-element buffer.  The radices are arranged as a
 * palindrome (R_1 = R_p, middle radices symmetric; one pass more than the default schedule when
 * log_n admits no palindrome of that length, e.g. odd log_n over an even pass count), every pass
 * writes the positions it read, and the digit reversal (an involution) is fused into the final
 * pass: each final tile writes natural positions once the mirror slab has been read (k_final_ipn,
 * bounded waits reported by ntt_plan_device_status); batched calls take a separate pass of disjoint
 * tile-pair swaps instead.  Same contract and results as the default schedule, within ~1 % of its
 * time on the 256-bit path.  P469762049 plans run on 8-B scratch elements for it (the default P
 * plan keeps 4-B ones); 6 x 64-bit plans of a modulus < 2^255 keep their intermediates in the
 * caller's 48-B elements (the default 6-limb plan uses 32-B scratch).  Sizes with no palindrome the
 * pass kernels accept (2^11 and 2^13 on the 1024-element tiles; P: 2^15, 2^17, 2^19 on its
 * 8192-element tiles) and the rival schedules return NTT_ERR_ARG. */
#define NTT_PLAN_IN_PLACE 16u
/* Single-launch schedule (BASELINE config 2, "single-kernel self-sort-in-place"; the reference runs
 * 2^20 as 4 launches, GZKP-NTT.cu:1509-1545): a forward / inverse of a 4-limb BN254 / BLS12-381 plan
 * runs as ONE persistent launch.  At 2^20 (round 5): the two passes of 4096-element tiles (10 + 10)
 * with one grid barrier (k_fused2b); with NTT_PLAN_IN_PLACE too, no scratch and a second barrier
 * before the digit-reversed stores (k_fused2bi).  Other 3-pass sizes (2^18 .. 2^24): two grid-wide
 * barriers (k_fused3b; the default) or the passes' tiles handed between workgroups through dependency
 * counters (k_fused3; environment NTT_FUSED_MODE=0); in place (2^18, 2^19): three barriers
 * (k_fused3bi).  Same contract and results as the default schedule; batch 1; other plans and calls
 * ignore the flag.
 * The grid-barrier forms are plain launches of at most as many workgroups as the device keeps
 * resident (the plan's occupancy query).  The library orders them per device (round 6): a single
 * launch enqueued on another stream than the device's previous one waits for it, so two
 * single-launch plans on two streams never split the device between them (on one stream nothing is
 * added).  CUs held by anything else (another process, a persistent kernel of the caller's) can still
 * keep part of a launch waiting; every wait is bounded, so the call then returns garbage and the
 * plan's next call NTT_ERR_DEVICE (ntt_plan_device_status), never a hang.  The in-place forms
 * (k_fused2bi, k_fused3bi) check residency before their first store: such a call stores nothing and
 * the caller's buffer keeps its input.  (The cooperative-launch switch NTT_FUSED_COOP was retired in
 * round 6.)
 * ntt_plan_device_status reports a wait that gave up (a watchdog; never expected). */
#define NTT_PLAN_SINGLE_LAUNCH 32u
/* Rival schedule, the reference's `naive` (GZKP-NTT.cu:59-95, big-num.cu:67-170): the bit reversal,
 * then log2 n radix-2 DIT rounds of one launch each (a thread per butterfly, w from an n/2-entry power
 * table, the reference's `roots`).  Forward single transforms of P469762049 and 4-limb plans; the
 * plan's other calls run the default schedule.  Exclusive with the other rivals and with
 * NTT_PLAN_IN_PLACE. */
#define NTT_PLAN_NAIVE 64u
/* Rival schedule, the reference's `naive_no_swap` (GZKP-NTT.cu:237-296; its main checks it against
 * the CPU NTT, GZKP-NTT.cu:1653-1660): a radix-2 Stockham autosort -- log2 n rounds of one launch
 * each, round s reading x[i], x[i + n/2] and writing y[2i - k], y[2i - k + 2^s] (k = i mod 2^s,
 * w = w_n^(k n / 2^(s+1)) from the n/2-entry power table), ping-pong between the caller's buffer and
 * a plan buffer, natural order in and out, no bit reversal.  When log2 n is odd the last round lands
 * in the plan buffer and one device copy brings it back.  Forward single transforms of P469762049 and
 * 4-limb plans; the plan's other calls run the default schedule.  Exclusive with the other rivals and
 * with NTT_PLAN_IN_PLACE. */
#define NTT_PLAN_NO_SWAP 128u
/* Rival schedules, the reference's bealto.com radix-2^deg Stockham family (round 6): log2 n / deg
 * rounds of one launch each, ping-pong between the caller's buffer and a plan buffer, natural order
 * in and out.  A group of 2^deg elements x[index + i t] (t = n / 2^deg) is multiplied by
 * w^((n >> lgp >> deg) k i) (k = index mod 2^lgp), transformed by deg radix-2 rounds in LDS with the
 * 2^(max_deg-1)-entry table pq, and written to y[((index - k) << deg) + k + i 2^lgp]; two elements per
 * thread.  The variants differ only in how threads, groups and LDS rows map (the reference's access
 * patterns, kept for comparison):
 *   NTT_PLAN_BELLPERSON   bellperson_baseline / FIELD_radix_fft_revised (GZKP-NTT.cu:391-553): one
 *                         group per workgroup, deg <= 8, inputs bit-reversed into LDS, DIT rounds;
 *   NTT_PLAN_IMPROVED_V1  improve_grouped (GZKP-NTT.cu:556-630, 721-804): 32 groups per workgroup,
 *                         deg <= 3, DIF rounds, outputs bit-reversed from LDS;
 *   NTT_PLAN_IMPROVED_V2  improve_group_coalesced_read (632-719, 806-890): v1 with the load map
 *                         transposed, consecutive threads reading consecutive groups;
 *   NTT_PLAN_IMPROVED_V3  improve_group_coalesced_read_and_write (892-1075): v2 with the stores on
 *                         the load map too (after the first round);
 *   NTT_PLAN_IMPROVED_V4  improve_reduce_bank_conflict (1077-1296): v3 with each group's LDS row
 *                         padded by one element.
 * The reference runs them on P469762049 (`long long`); here forward single transforms of P469762049
 * and 4-limb plans, the plan's other calls on the default schedule.  Exclusive with the other rivals
 * and with NTT_PLAN_IN_PLACE. */
#define NTT_PLAN_BELLPERSON 256u
#define NTT_PLAN_IMPROVED_V1 512u
#define NTT_PLAN_IMPROVED_V2 1024u
#define NTT_PLAN_IMPROVED_V3 2048u
#define NTT_PLAN_IMPROVED_V4 4096u
int ntt_plan_create_ex(ntt_plan** out, int field_id, unsigned log_n, unsigned limbs64, int device, unsigned flags);
/* Device-side status of a plan (blocking: synchronises the device, then reads and clears it).
 * *bad bit 0: an inter-workgroup wait gave up at its watchdog (NTT_PLAN_SINGLE_LAUNCH, or the fused
 * digit reversal of NTT_PLAN_IN_PLACE): that call's output is wrong (the workgroup that gave up
 * skipped its stores), and until this call clears the report every other call on the plan returns
 * NTT_ERR_DEVICE.  The checked build (ntt_amd/libntt_debug.so,
 * same ABI, `python -m ntt_amd.build --debug`) adds, from checks inside every pass kernel:
 *   0x100  an element index outside its buffer (the access went to element 0 instead)
 *   0x200  a caller input element >= p (the inputs must be canonical, as in the reference)
 *   0x400  an intermediate >= 2p (a lazy-reduction bound broke)
 *   0x800  an output element >= p
 * The product build never sets these bits. */
int ntt_plan_device_status(ntt_plan* plan, unsigned* bad);
/* Poll limit of the plan's bounded inter-workgroup waits (default 2^21, about 2 s; read at each
 * launch).  0 makes every wait that is not already satisfied give up at once: a test hook for the
 * NTT_ERR_DEVICE path (tests/test_gpu_watchdog.py). */
int ntt_plan_set_watchdog(ntt_plan* plan, unsigned spins);

/* Modulus-generic plan, like big-num.cu's `prime` / `omega` kernel arguments (big-num.cu:68,173,260):
 * modulus and generator given as limbs64 little-endian 64-bit limbs.  Accepted moduli: odd primes
 * with 2^log_n | p - 1 and, by limb count, p < 2^30 (1 limb: lazy values up to 4p must fit 32 bits,
 * so e.g. the 31-bit 2013265921 returns NTT_ERR_FIELD), p < 2^255 (4 limbs), p < 2^(29*14-6) with 2p
 * below 2^383 (6 limbs). */
int ntt_plan_create_custom(ntt_plan** out, const uint64_t* modulus, const uint64_t* generator, unsigned limbs64,
                           unsigned log_n, int device);

int ntt_plan_create_custom_ex(ntt_plan** out, const uint64_t* modulus, const uint64_t* generator, unsigned limbs64,
                              unsigned log_n, int device, unsigned flags);

/* Forward NTT in place, natural -> natural (SSIP GZKP-NTT.cu:1452, NTT_GZKP big-num.cu:260). */
int ntt_forward(ntt_plan* plan, void* d_data, void* hip_stream);
/* Inverse NTT in place including the n^-1 scale (GZKP-NTT.cu:1725-1732). */
int ntt_inverse(ntt_plan* plan, void* d_data, void* hip_stream);
/* `batch` independent transforms laid out back to back (stride 2^log_n elements). */
int ntt_forward_batch(ntt_plan* plan, void* d_data, unsigned batch, void* hip_stream);
int ntt_inverse_batch(ntt_plan* plan, void* d_data, unsigned batch, void* hip_stream);

/* Coset NTT, the low-degree-extension step of the GZKP provers the reference targets:
 *   forward:  X_k = sum_j x_j (c w^k)^j = NTT(x_j c^j)          (evaluations on the coset c<w>)
 *   inverse:  x_j = c^-j INTT(X)_j                               (interpolation from the coset)
 * `shift` = c as limbs64 little-endian 64-bit limbs, canonical and nonzero (e.g. the field's
 * multiplicative generator).  The plan caches the c^j tables of the last shift. */
int ntt_forward_coset(ntt_plan* plan, void* d_data, const uint64_t* shift, void* hip_stream);
int ntt_inverse_coset(ntt_plan* plan, void* d_data, const uint64_t* shift, void* hip_stream);

/* Pointwise product c = a * b mod p over 2^log_n elements (polynomial-multiply middle step);
 * a b R^-1 with NTT_PLAN_MONTGOMERY_IO. */
int ntt_pointwise_mul(ntt_plan* plan, const void* d_a, const void* d_b, void* d_c, void* hip_stream);
/* Cyclic polynomial product c = a * b of length 2^log_n: forward(a), forward(b), then the inverse
 * of their pointwise product into c (multi-pass 256-bit plans fuse the pointwise product into the
 * inverse's first pass).  a and b are overwritten with their transforms; c may alias a or b. */
int ntt_polymul(ntt_plan* plan, void* d_a, void* d_b, void* d_c, void* hip_stream);
/* Second half of a polymul over `batch` transforms laid out back to back: c = INTT(a * b) for a, b
 * already forward-transformed (fused into the inverse's first pass where the plan allows it).
 * c may alias a or b; a may equal b (squaring).  The distributed polymul runs it on each rank's
 * column-layout shares (ntt_polymul_multi, ntt_amd/distributed.py). */
int ntt_inverse_pointwise_batch(ntt_plan* plan, const void* d_a, const void* d_b, void* d_c, unsigned batch,
                                void* hip_stream);

/* Canonical-range check of a caller buffer (the contract every transform assumes: elements < p,
 * upper limbs zero).  The reference's only guard is CGBN's padded-store `BAD LIMB` trap
 * (impl_cuda.cu:1402-1408); this is a query instead: *bad = number of the `count` elements that are
 * not < p.  Blocking on hip_stream. */
int ntt_count_noncanonical(ntt_plan* plan, const void* d_data, uint64_t count, uint64_t* bad, void* hip_stream);

/* Fill a device vector with the SURVEY §8d synthetic inputs: kind 0 = x_j = j (the reference's
 * input, GZKP-NTT.cu:1587), kind 1 = SplitMix64 limbs with the top limb masked (seeded). */
int ntt_fill(ntt_plan* plan, void* d_data, int kind, uint64_t seed, void* hip_stream);

/* Fill `count` local elements: element i gets the synthetic value of global index
 * j = row0 + (i >> log_inner) + ((i mod 2^log_inner) << log_stride)  (log_inner >= 64: j = i).
 * Used to lay out one rank's share of a distributed vector. */
int ntt_fill_map(ntt_plan* plan, void* d_data, uint64_t count, int kind, uint64_t seed, uint64_t row0,
                 unsigned log_inner, unsigned log_stride, void* hip_stream);

/* ---------------------------------------------------------------- multi-GPU four-step, local steps
 * (the exchange itself is an RCCL all-to-all issued by the caller)
 * twiddle_pack: src = [2^log_rows][2^log_row_len] row-major; element (a, b) is multiplied by
 * w_n^((row0 + a) * b) (w_n^-1 if inverse; n = 2^log_n of the plan) and written to
 * dst[b >> log_block][a][b mod 2^log_block]: one contiguous chunk per destination rank.
 * transpose: dst[c][r] = src[r][c] for a 2^log_rows x 2^log_cols matrix of elements. */
int ntt_twiddle_pack(ntt_plan* plan, const void* d_src, void* d_dst, unsigned log_rows, unsigned log_row_len,
                     unsigned log_block, uint64_t row0, int inverse, void* hip_stream);
int ntt_transpose(ntt_plan* plan, const void* d_src, void* d_dst, unsigned log_rows, unsigned log_cols,
                  void* hip_stream);
/* The same with explicit chunk strides (several vectors exchanged in one all-to-all, e.g. the
 * distributed polymul's a and b): twiddle_pack writes peer chunk q at dst + q * peer_stride
 * elements (peer_stride >= 2^(log_rows + log_block)); transpose reads source rows in blocks of
 * 2^log_block_rows rows, block q starting at src + q * block_stride elements. */
int ntt_twiddle_pack_ex(ntt_plan* plan, const void* d_src, void* d_dst, unsigned log_rows, unsigned log_row_len,
                        unsigned log_block, uint64_t row0, int inverse, uint64_t peer_stride, void* hip_stream);
int ntt_transpose_ex(ntt_plan* plan, const void* d_src, void* d_dst, unsigned log_rows, unsigned log_cols,
                     unsigned log_block_rows, uint64_t block_stride, void* hip_stream);

/* Per-launch timing for benchmarks: when enabled, every transform records HIP events on its
 * stream between its kernel launches (a ring of 64 transforms, no host synchronisation);
 * ntt_plan_last_launch_ms returns per-launch durations (ms) averaged over the transforms recorded
 * since profiling was enabled (the last 64 at most), waiting for the most recent one; for the
 * schedule the most recent call ran (single-vector or batched, see ntt_plan_info). */
int ntt_plan_set_profiling(ntt_plan* plan, int enable);
int ntt_plan_last_launch_ms(ntt_plan* plan, float* ms, unsigned max_launches, unsigned* nlaunches);
/* The same launches' labels, comma-separated, in launch order: a kind letter and the pass's log2
 * radix (c column pass, "s" appended when it reads a Shoup-pair outer table; f final pass; s one
 * transform per workgroup; r several per workgroup; i in-place final pass with the digit reversal;
 * d digit-reversal swap; b single launch; n naive), "" when unlabelled.  NTT_ERR_ARG when `cap`
 * bytes do not hold them.  New (round 6): benchmarks pair per-launch PMC bytes with launches by
 * label, not by position. */
int ntt_plan_last_launch_labels(ntt_plan* plan, char* buf, unsigned cap);
/* Group mode: from this call on, the plan's transforms accumulate into ONE record (timings and
 * labels) until the next call, so that ntt_plan_last_launch_ms reports every launch of a caller-level
 * operation made of several transforms (the rank plan's row transforms of 2^15 rows each); the time
 * between two transforms of a group is not reported. */
int ntt_plan_profile_group(ntt_plan* plan);

/* Plan introspection: n, bytes per element, number of passes and their log2 radices (of a
 * single-vector transform: a default or Montgomery-I/O 4 x 64-bit plan of exactly 2^20 runs those on
 * 4096-element tiles in two passes, 10 + 10, and batched calls on 1024-element tiles, 7 + 7 + 6;
 * environment NTT_WIDE_TILES=0 keeps every call on the latter). */
int ntt_plan_info(const ntt_plan* plan, uint64_t* n, unsigned* elem_bytes, unsigned* npasses, unsigned radix_log[8]);
int ntt_plan_destroy(ntt_plan* plan);
const char* ntt_strerror(int status);

/* ---------------------------------------------------------------- reference-shaped shims */
/* SSIP(x, omega, log_n): P469762049 path, long long elements in device memory, blocking,
 * default stream (GZKP-NTT.cu:1452).  Prints nothing; errors are reported by the return value of
 * ntt_last_error(). */
void SSIP(long long* x, long long omega, unsigned log_n);
/* NTT_GZKP<8,256>(data, len, reverse, reverse_len, prime, omega, B, G) (big-num.cu:260): 256-bit
 * elements (8 x u32 LE), any odd prime < 2^255 given as 8 u32 words, omega = generator.  reverse /
 * reverse_len / B / G are accepted for signature compatibility and ignored (the transform is
 * self-sorting).  Blocking, default stream.  Returns a status. */
int NTT_GZKP_256(uint32_t* data, uint32_t len, const void* reverse, uint32_t reverse_len, const uint32_t prime[8],
                 const uint32_t omega[8], uint32_t B, uint32_t G);
/* NTT_GZKP(data, reverse, len, omega, B, G, reverse_num) for P469762049 (parallel-load.cu:195). */
int NTT_GZKP_64(long long* data, const void* reverse, long long len, long long omega, int B, int G,
                long long reverse_num);
int ntt_last_error(void);
/* The shims cache one plan per (modulus, generator, limbs, size, device) -- the reference rebuilt
 * its tables on every call (GZKP-NTT.cu:1476-1500, big-num.cu:278-309) -- keeping at most
 * NTT_SHIM_CACHE_PLANS (environment, default 8) and dropping the least recently used one beyond
 * that.  This releases every cached plan (a shim call still running keeps its plan until it returns). */
void ntt_shim_cache_clear(void);

/* ---------------------------------------------------------------- one rank of the distributed four-step
 * New (the reference has no multi-GPU code).  The local steps of rank `rank` of `world`
 * around the all-to-all, fused so that no separate twiddle, pack or transpose pass runs: the row
 * transforms' last pass applies w_n^(j1 k2) and stores straight into the peer chunks, and the column
 * transforms read the received chunks in place (2^log_c interleaved transforms).  Layouts as the
 * multi-GPU plan below: row layout [r][n2], column layout [n1][c]; the split n1 x n2 is the plan's
 * (ntt_rplan_info), the same for every rank of one (field, log_n, limbs64, world).  Send / receive buffers are the
 * caller's: [world][nvec][chunk] elements (chunk = r c, ntt_rplan_info), exchanged by the caller
 * as ONE all-to-all of equal chunks (RCCL, device copies, ...).  nvec = 2 carries two vectors per
 * exchange (polymul: slot 0 = a, slot 1 = b).  All calls are asynchronous on hip_stream. */
typedef struct ntt_rplan ntt_rplan;
int ntt_rplan_create(ntt_rplan** out, int field_id, unsigned log_n, unsigned limbs64, int world, int rank,
                     int device);
int ntt_rplan_info(const ntt_rplan* rp, uint64_t* local_n, uint64_t* chunk, unsigned* log_n1, unsigned* log_n2,
                   unsigned* elem_bytes);
/* row layout x (unchanged) -> send slot `slot` of nvec */
int ntt_rplan_forward_rows(ntt_rplan* rp, const void* d_x, void* d_send, unsigned nvec, unsigned slot,
                           void* hip_stream);
/* recv slot `slot` of nvec -> column layout x */
int ntt_rplan_forward_cols(ntt_rplan* rp, const void* d_recv, void* d_x, unsigned nvec, unsigned slot,
                           void* hip_stream);
/* column layout x (times y, pointwise, when y != NULL: the polymul's product) -> send (nvec = 1) */
int ntt_rplan_inverse_cols(ntt_rplan* rp, const void* d_x, const void* d_y, void* d_send, void* hip_stream);
/* recv (nvec = 1) -> row layout out (1/n included over both halves) */
int ntt_rplan_inverse_rows(ntt_rplan* rp, const void* d_recv, void* d_out, void* hip_stream);
/* The same two row steps over local rows [row0, row0 + nrows) only (1 <= nrows, row0 + nrows <= r).
 * Rows [row0, row0 + nrows) of every peer chunk form the contiguous run
 * [row0 c, (row0 + nrows) c) of that chunk, so a caller can exchange each piece as soon as it is written
 * (forward) or transform each piece as soon as it has arrived (inverse): the exchange of one piece
 * overlaps the row transforms of the next. */
int ntt_rplan_forward_rows_range(ntt_rplan* rp, const void* d_x, void* d_send, unsigned nvec, unsigned slot,
                                 uint64_t row0, uint64_t nrows, void* hip_stream);
int ntt_rplan_inverse_rows_range(ntt_rplan* rp, const void* d_recv, void* d_out, uint64_t row0, uint64_t nrows,
                                 void* hip_stream);
/* Pieces on BOTH sides of the exchange (ntt_amd/distributed.py FourStep): row_pieces P_r and
 * col_pieces P_c, powers of two (<= r and <= c); ra = r / P_r, cm = c / P_c.  Exchange blocks (one
 * per peer, nvec r c elements each) in these entry points' own layouts:
 *   forward [i][v][k][ra][cm]: forward_rows_piece(i) writes row piece i of vector `slot`;
 *     forward_cols_piece(k) transforms column piece k (columns k cm + [0, cm) of the column layout)
 *     once units (i, v, k) of every peer i have arrived -- row piece i of all vectors is one run
 *     [i nvec ra c, (i + 1) nvec ra c) of each block, unit (i, v, k) the run of ra cm elements at
 *     (i nvec + v) ra c + k ra cm;
 *   inverse [k][i][ra][cm]: inverse_cols_piece(k) (times y, same layout as x, if y != NULL) writes
 *     column piece k = the run [k r cm, (k + 1) r cm) of each block; inverse_rows_piece(i) transforms
 *     row piece i once the units (k, i) = runs of ra cm elements at k r cm + i ra cm have arrived.
 * So the exchange can overlap the row transforms before it and the column transforms after it
 * (forward), or the column transforms before it and the row transforms after it (inverse).  With
 * P_r = P_c = 1 the layouts are the [G][nvec][r][c] blocks above. */
int ntt_rplan_forward_rows_piece(ntt_rplan* rp, const void* d_x, void* d_send, unsigned nvec, unsigned slot,
                                 unsigned piece, unsigned row_pieces, unsigned col_pieces, void* hip_stream);
int ntt_rplan_forward_cols_piece(ntt_rplan* rp, const void* d_recv, void* d_x, unsigned nvec, unsigned slot,
                                 unsigned piece, unsigned row_pieces, unsigned col_pieces, void* hip_stream);
int ntt_rplan_inverse_cols_piece(ntt_rplan* rp, const void* d_x, const void* d_y, void* d_send, unsigned piece,
                                 unsigned row_pieces, unsigned col_pieces, void* hip_stream);
int ntt_rplan_inverse_rows_piece(ntt_rplan* rp, const void* d_recv, void* d_out, unsigned piece, unsigned row_pieces,
                                 unsigned col_pieces, void* hip_stream);
/* this rank's row-layout share of the global synthetic vector (kinds as ntt_fill) */
int ntt_rplan_fill(ntt_rplan* rp, void* d_x, int kind, uint64_t seed, void* hip_stream);
/* per-launch timing of the row (which = 0) or column (1) transforms, as ntt_plan_last_launch_ms */
int ntt_rplan_set_profiling(ntt_rplan* rp, int enable);
int ntt_rplan_last_launch_ms(ntt_rplan* rp, int which, float* ms, unsigned max_launches, unsigned* nlaunches);
int ntt_rplan_last_launch_labels(ntt_rplan* rp, int which, char* buf, unsigned cap);
/* the row and column plans' group mode (ntt_plan_profile_group): call at the start of every four-step
 * transform, so that the timings report each of its launches (e.g. the row transform's launches of
 * 2^15 rows each at world size 1) */
int ntt_rplan_profile_group(ntt_rplan* rp);
int ntt_rplan_destroy(ntt_rplan* rp);

/* ---------------------------------------------------------------- single-process multi-GPU
 * New (the reference has no multi-GPU code).  One plan drives `ngpus` devices of one node (power of
 * two); a transform is the four-step with ONE RCCL all-to-all over xGMI (ncclCommInitAll over
 * `devices`).  d_data[g] / hip_streams[g] belong to devices[g] (streams may be NULL = default
 * streams); each d_data[g] holds n / ngpus elements.  Device g runs ntt_rplan rank g.  Layouts (as
 * ntt_amd/distributed.py), with n = n1 n2, r = n1/ngpus, c = n2/ngpus, where the plan picks the split
 * (ntt_mplan_info / ntt_rplan_info): the fewest pass kernels, then the smallest largest radix, then
 * the most balanced split (2^24 on the 256-bit engines: n1 = 2^16, n2 = 2^8):
 *   forward input  (row layout):    d_data[g] = [r][n2], element (a, j2) = x[g r + a + n1 j2]
 *   forward output (column layout): d_data[g] = [n1][c], element (k1, kc) = X[g c + kc + n2 k1]
 * The inverse takes the column layout back to the row layout (1/n included).  Asynchronous. */
typedef struct ntt_mplan ntt_mplan;
int ntt_mplan_create(ntt_mplan** out, int field_id, unsigned log_n, unsigned limbs64, int ngpus, const int* devices);
int ntt_forward_multi(ntt_mplan* plan, void* const* d_data, void* const* hip_streams);
int ntt_inverse_multi(ntt_mplan* plan, void* const* d_data, void* const* hip_streams);
/* Distributed cyclic polynomial product (BASELINE config 5): d_a[g], d_b[g] hold the
 * row-layout shares of a and b; on return d_c[g] holds the row-layout share of c = a * b (length n)
 * and d_a / d_b hold the column-layout shares of their forward transforms.  Forward(a) and
 * forward(b) share ONE all-to-all (each peer chunk carries both), the pointwise product is local
 * and fused into the inverse's first column pass, and the inverse's all-to-all brings c back to
 * the row layout: two exchanges for the three transforms.  d_c may alias d_a or d_b. */
int ntt_polymul_multi(ntt_mplan* plan, void* const* d_a, void* const* d_b, void* const* d_c, void* const* hip_streams);
/* each device's row-layout share of the global synthetic vector (kinds as ntt_fill) */
int ntt_mplan_fill(ntt_mplan* plan, void* const* d_data, int kind, uint64_t seed, void* const* hip_streams);
int ntt_mplan_info(const ntt_mplan* plan, uint64_t* local_n, unsigned* log_n1, unsigned* log_n2);
/* Pieces of the pipelined exchange on both sides (powers of two, <= 16, row_pieces <= r, col_pieces
 * <= c; the ntt_rplan_*_piece layouts): row piece i's exchange (grouped ncclSend / ncclRecv on a
 * per-device communication stream) overlaps the row transforms of piece i + 1, the last row piece
 * goes out per column piece and each column piece's transforms start when it has arrived (the
 * inverse mirrors it).  Default: 1 x 1, one whole-block exchange per transform (the pieces have
 * not yet measured a gain). */
int ntt_mplan_set_pieces2(ntt_mplan* plan, unsigned row_pieces, unsigned col_pieces);
/* Row pieces only (1..16, <= r; rounded down to a power of two), one column piece. */
int ntt_mplan_set_pieces(ntt_mplan* plan, unsigned pieces);
int ntt_mplan_destroy(ntt_mplan* plan);

#ifdef __cplusplus
}
#endif
#endif
