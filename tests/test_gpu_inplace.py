"""NTT_PLAN_IN_PLACE: the transform with no plan scratch (the reference's self-sort-in-place
property: SSIP_NTT_stage2's mirror pairs, GZKP-NTT.cu:1359-1449, leave the result in natural order in
the caller's buffer with no second buffer).  Palindromic pass sequence, every pass writes the
positions it read, then k_digitrev_swap exchanges tile pairs (the digit reversal is an involution).
Pins: the C oracle (GZKP-NTT.cu:30-48 restated; itself pinned against the reference's outputs,
tests/test_oracle_ref.py) element by element, and bit-for-bit agreement with the default schedule."""
import os

import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8"))))


def _plan(fid, log_n, L=4, in_place=True, **kw):
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=fid, log_n=log_n, limbs64=L, in_place=in_place, **kw)


def _host(t, L):
    return t.cpu().numpy().view(np.uint64).reshape(-1, L)


def _is_palindrome(r):
    return list(r) == list(reversed(r))


# sizes whose palindromic schedule is the default pass count (12, 16, 17, 20, 23) and ones that take
# a pass more (15: 5+5+5, 25: 5+5+5+5+5)
@pytest.mark.parametrize("fid,log_n", [(1, 12), (2, 15), (1, 16), (2, 17), (1, 20), (1, 23), (2, 25)])
def test_in_place_matches_oracle_and_default(fid, log_n):
    p, g = R.FIELDS[fid]
    ip = _plan(fid, log_n)
    df = _plan(fid, log_n, in_place=False)
    assert _is_palindrome(ip.passes) and sum(ip.passes) == log_n, ip.passes
    a = ip.fill(ip.empty(), "random", seed=100 + log_n)
    b = a.clone()
    x = _host(a, 4).copy()
    ip.forward(a)
    df.forward(b)
    assert torch.equal(a, b), (fid, log_n, ip.passes, df.passes)
    if log_n <= 20:
        assert np.array_equal(_host(a, 4), OC.ntt_mp_par(x, p, g, THREADS))
    ip.inverse(a)
    assert np.array_equal(_host(a, 4), x)


def test_in_place_2pow24_bn254_elementwise():
    """The headline size: forward element by element against the threaded C oracle, inverse round trip."""
    p, g = R.FIELDS[1]
    ip = _plan(1, 24)
    assert ip.passes == [8, 8, 8]
    a = ip.fill(ip.empty(), "random", seed=24)
    x = _host(a, 4).copy()
    ip.forward(a)
    assert np.array_equal(_host(a, 4), OC.ntt_mp_par(x, p, g, THREADS))
    ip.inverse(a)
    assert np.array_equal(_host(a, 4), x)


def test_in_place_2pow28_bn254_matches_default():
    """C4's n on one GPU (7+7+7+7, two middle digits reversed by the swap): equal to the default
    schedule on the device, KAT of x_j = j at sampled k, round trip."""
    fid, log_n = 1, 28
    p, g = R.FIELDS[fid]
    n = 1 << log_n
    ip = _plan(fid, log_n)
    assert ip.passes == [7, 7, 7, 7]
    a = ip.fill(ip.empty(), "random", seed=28)
    ref = a.clone()
    ip.forward(a)
    df = _plan(fid, log_n, in_place=False)
    df.forward(ref)
    assert torch.equal(a, ref)
    del ref, df
    torch.cuda.empty_cache()
    ip.inverse(a)
    x = ip.fill(ip.empty(), "random", seed=28)
    assert torch.equal(a, x)
    del x
    ip.fill(a, "iota")
    ip.forward(a)
    rng = np.random.default_rng(2828)
    for k in [0, 1, n - 1] + [int(v) for v in rng.integers(0, n, 8)]:
        v = sum(int(w) << (64 * i) for i, w in enumerate(a[k].cpu().numpy().view(np.uint64)))
        assert v == R.kat_xj(n, p, g, k), k


def test_in_place_plan_owns_no_scratch():
    """The default plan holds an n x 32-B scratch vector; the in-place plan does not."""
    log_n = 24
    torch.cuda.synchronize()
    f0, _ = torch.cuda.mem_get_info()
    df = _plan(1, log_n, in_place=False)
    torch.cuda.synchronize()
    f1, _ = torch.cuda.mem_get_info()
    ip = _plan(1, log_n)
    torch.cuda.synchronize()
    f2, _ = torch.cuda.mem_get_info()
    used_df, used_ip = f0 - f1, f1 - f2
    assert used_df - used_ip >= (1 << log_n) * 32 * 0.99, (used_df, used_ip)
    ip.close()
    df.close()


def test_in_place_batch_polymul_coset():
    fid, log_n, batch = 2, 16, 3
    p, g = R.FIELDS[fid]
    ip = _plan(fid, log_n)
    df = _plan(fid, log_n, in_place=False)
    a = torch.cat([ip.fill(ip.empty(), "random", seed=7 + i) for i in range(batch)]).contiguous()
    b = a.clone()
    ip.forward_batch(a, batch)
    df.forward_batch(b, batch)
    assert torch.equal(a, b)
    ip.inverse_batch(a, batch)
    df.inverse_batch(b, batch)
    assert torch.equal(a, b)
    # polymul: c = a * b mod (x^n - 1), the fused product in the inverse's first pass, and squaring
    u = ip.fill(ip.empty(), "random", seed=8)
    v = ip.fill(ip.empty(), "random", seed=9)
    c1, c2 = ip.empty(), df.empty()
    ip.polymul(u.clone(), v.clone(), c1)
    df.polymul(u.clone(), v.clone(), c2)
    assert torch.equal(c1, c2)
    s1 = u.clone()
    ip.polymul(s1, s1, s1)
    s2 = u.clone()
    df.polymul(s2, s2, s2)
    assert torch.equal(s1, s2)
    # coset forward / inverse
    shift = 5
    w1, w2 = u.clone(), u.clone()
    ip.forward_coset(w1, shift)
    df.forward_coset(w2, shift)
    assert torch.equal(w1, w2)
    ip.inverse_coset(w1, shift)
    assert torch.equal(w1, u)


def test_in_place_384bit_class():
    """14-limb engine (moduli above 2^255 in the 6 x 64-bit layout: scratch element = caller element)."""
    from tests.test_gpu_parity import _big_ntt_prime, _to_dev
    from ntt_amd.ntt import NTTPlan
    p, g = _big_ntt_prime(380, 24)
    rng = np.random.default_rng(380)
    for log_n in (12, 14, 16):
        n = 1 << log_n
        vals = [int.from_bytes(rng.bytes(48), "little") % p for _ in range(n)]
        x = OC.ints_to_limbs(vals, 6)
        pl = NTTPlan(log_n=log_n, limbs64=6, modulus=p, generator=g, in_place=True)
        assert _is_palindrome(pl.passes), pl.passes
        t = _to_dev(x, 6)
        pl.forward(t)
        assert np.array_equal(_host(t, 6), OC.ntt_mp(x, p, g, False)), log_n
        pl.inverse(t)
        assert np.array_equal(_host(t, 6), x), log_n


@pytest.mark.parametrize("fid,log_n", [(2, 12), (1, 16), (2, 20), (1, 23)])
def test_in_place_6limb_layout_matches_oracle_and_default(fid, log_n):
    """C3's 6 x 64-bit layout in place: the intermediates live in the caller's
    48-B elements (Eng256wI), 256-bit arithmetic; equal to the default 6-limb plan and to the oracle."""
    p, g = R.FIELDS[fid]
    ip = _plan(fid, log_n, 6)
    df = _plan(fid, log_n, 6, in_place=False)
    assert _is_palindrome(ip.passes) and sum(ip.passes) == log_n, ip.passes
    a = ip.fill(ip.empty(), "random", seed=600 + log_n)
    b = a.clone()
    x = _host(a, 6).copy()
    ip.forward(a)
    df.forward(b)
    assert torch.equal(a, b), (fid, log_n, ip.passes, df.passes)
    if log_n <= 20:
        assert np.array_equal(_host(a, 6), OC.ntt_mp_par(x, p, g, THREADS))
    ip.inverse(a)
    assert np.array_equal(_host(a, 6), x)


def test_in_place_6limb_2pow24_bls_elementwise():
    """BASELINE C3 (2^24 BLS12-381 Fr, 6 x 64-bit limbs) in place: forward and inverse element by
    element against the threaded C oracle (GZKP-NTT.cu:30-48 restated; inverse GZKP-NTT.cu:1725-1732)."""
    p, g = R.FIELDS[2]
    ip = _plan(2, 24, 6)
    assert ip.passes == [8, 8, 8]
    a = ip.fill(ip.empty(), "random", seed=3)
    x = _host(a, 6).copy()
    ip.forward(a)
    assert np.array_equal(_host(a, 6), OC.ntt_mp_par(x, p, g, THREADS))
    a.copy_(torch.from_numpy(x.view(np.int64)).to(a.device))
    ip.inverse(a)
    assert np.array_equal(_host(a, 6), OC.ntt_mp_par(x, p, g, THREADS, inverse=True))


GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_p469762049.npz"))


@pytest.mark.parametrize("log_n", [14, 16, 18, 20, 21, 22, 24, 26])
def test_in_place_p_path_vs_reference_outputs(log_n):
    """The reference's own field and SSIP contract (`long long` elements, P = 469762049, x_j = j and a
    seeded vector): sampled outputs of the reference's CPU NTT (tests/golden/ref_p469762049.npz),
    bit-for-bit agreement with the default schedule, round trip.  P plans with NTT_PLAN_IN_PLACE run
    on 8-B scratch elements (EngPI) and the 8192-element tiles (palindromes with r_1 + r_p >= 13)."""
    n = 1 << log_n
    ip = _plan(0, log_n, 1)
    assert _is_palindrome(ip.passes) and sum(ip.passes) == log_n, ip.passes
    idx = torch.from_numpy(GOLD[f"samp_idx_{log_n}"]).to("cuda:0") if f"samp_idx_{log_n}" in GOLD else None
    t = torch.arange(n, dtype=torch.int64, device="cuda:0")
    ip.forward(t)
    if idx is not None:
        assert np.array_equal(t[idx].cpu().numpy(), GOLD[f"samp_iota_{log_n}"])
    x = OC.random_limbs(0, n, seed=2000 + log_n, L=1)[:, 0].astype(np.int64)
    a = torch.from_numpy(x).to("cuda:0")
    b = a.clone()
    ip.forward(a)
    _plan(0, log_n, 1, in_place=False).forward(b)
    assert torch.equal(a, b)
    if idx is not None:
        assert np.array_equal(a[idx].cpu().numpy(), GOLD[f"samp_rand_{log_n}"])
    if log_n <= 16:
        p, g = R.FIELDS[0]
        assert np.array_equal(a.cpu().numpy(), OC.ntt_u64(x, p, g))
    ip.inverse(a)
    assert np.array_equal(a.cpu().numpy(), x)


@pytest.mark.parametrize("kw", [dict(fid=0, log_n=15, L=1),            # P: no palindrome with r_1 + r_p >= 13
                                dict(fid=1, log_n=11, L=4),            # no palindrome with r_1 + r_p >= 10
                                dict(fid=1, log_n=13, L=4),            # ... and r_{p-1} + r_p >= 10
                                dict(fid=1, log_n=16, L=4, stockham=True)])
def test_in_place_rejected(kw):
    kw = dict(kw)
    fid, log_n, L = kw.pop("fid"), kw.pop("log_n"), kw.pop("L")
    with pytest.raises(Exception):
        _plan(fid, log_n, L, **kw)
