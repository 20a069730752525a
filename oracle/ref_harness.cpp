// Harness around the reference's OWN CPU transforms — TEST INFRASTRUCTURE ONLY (the checker).
//
// oracle/Makefile (target `ref`) compiles the reference's host-only CPU code straight from
// /root/reference (never copied into this repository): the leading part of each source up to its
// first __global__/__device__ definition, with only the `#include <cuda_runtime.h>` line dropped
// (that part uses no CUDA type or call).  Outputs go to oracle/_ref/ (git-ignored):
//   libref_gzkp.so  <- src/GZKP-NTT.cu:1-48        NTT (radix-2 DIT after bit reversal), qpow, inv
//   libref_ssip.so  <- src/self-sort-in-place.cu:1-128  NTT, NTT_dif, NTT_pro1, NTT_pro2
// This file adds the extern "C" entry points ctypes binds (oracle/ref_c.py).  The field is the
// reference's compile-time P = 469762049 with root = 3 (GZKP-NTT.cu:7-8).
#include <cstdint>
#include <vector>

#if defined(REF_GZKP) || defined(REF_SSIP)
void NTT(long long data[], long long reverse[], long long len, long long omega);
#endif
#ifdef REF_SSIP
void NTT_dif(long long data[], long long reverse[], unsigned log_len, long long omega);
void NTT_pro1(long long data[], unsigned log_len, long long omega);
void NTT_pro2(long long data[], unsigned log_len, long long omega);
#endif

namespace {
const long long kP = 469762049;  // GZKP-NTT.cu:7

long long powmod(long long x, long long y) {
    long long r = 1;
    x %= kP;
    while (y) {
        if (y & 1) r = r * x % kP;
        x = x * x % kP;
        y >>= 1;
    }
    return r;
}

// the bit-reversal table exactly as the reference's main builds it (GZKP-NTT.cu:1580-1582)
std::vector<long long> reverse_table(unsigned bits) {
    long long len = 1ll << bits;
    std::vector<long long> rev(len, 0);
    for (long long i = 0; i < len; i++)
        rev[i] = bits ? ((rev[i >> 1] >> 1) | ((i & 1ll) << (bits - 1))) : 0;
    return rev;
}
}  // namespace

extern "C" {

long long ref_modulus(void) { return kP; }

// forward: NTT(data, reverse, len, omega) as main calls it with omega = root (GZKP-NTT.cu:1595);
// inverse: the commented-out recipe of GZKP-NTT.cu:1725-1732 — NTT(..., inv(omega)) then * inv(len).
int ref_ntt(long long* data, unsigned log_n, long long omega, int inverse) {
    if (log_n > 30) return -1;
    std::vector<long long> rev = reverse_table(log_n);
    long long len = 1ll << log_n;
    NTT(data, rev.data(), len, inverse ? powmod(omega, kP - 2) : omega);
    if (inverse) {
        long long co = powmod(len, kP - 2);
        for (long long i = 0; i < len; i++) data[i] = data[i] * co % kP;
    }
    return 0;
}

#ifdef REF_SSIP
// self-sort-in-place CPU spec: NTT_pro1 then NTT_pro2 (self-sort-in-place.cu:79-128)
int ref_ssip_pro(long long* data, unsigned log_n, long long omega) {
    if (log_n > 30) return -1;
    NTT_pro1(data, log_n, omega);
    NTT_pro2(data, log_n, omega);
    return 0;
}

// DIF followed by the bit-reversal permutation (self-sort-in-place.cu:53-77)
int ref_ntt_dif(long long* data, unsigned log_n, long long omega) {
    if (log_n > 30) return -1;
    std::vector<long long> rev = reverse_table(log_n);
    NTT_dif(data, rev.data(), log_n, omega);
    return 0;
}
#endif
}
