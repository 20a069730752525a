"""Full-size GPU parity, element by element and for the multi-GPU configs.

* 2^24 random vectors compared with the threaded C oracle (oracle_ntt_mp_par, a restatement of
  GZKP-NTT.cu:30-48 pinned in test_oracle.py / test_oracle_ref.py): BN254 forward and inverse (the
  headline), BLS12-381 Fr forward and inverse in the 4 and 6 x 64-bit layouts (C3), the 8-B P path
  at 2^26;
* C4's four-step at 2^28 over 8 virtual ranks (one GPU, exchange = device copies): the closed-form
  KAT of x_j = j at sampled k of the gathered column layout, plus the inverse round trip;
* the single-process multi-GPU plan (ntt_mplan_*, RCCL) at 2^26 and 2^28 on the visible devices;
* C5's polymul at 2^24 (degree < 2^23 inputs from vector B, seeds 5 and 6), element by element;
* C4 at 2^28 on SURVEY §8d's random vector B (seed 4), both as the plain one-GPU transform and as the
  four-step over 8 virtual ranks: sampled outputs against the definition evaluated directly on the
  CPU (oracle_eval_random_mp, Horner over the on-the-fly generated vector; pinned against the
  oracle's NTT in test_oracle.py).
"""
import os

import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8"))))


def _plan(fid, log_n, L):
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=fid, log_n=log_n, limbs64=L, device=0)


def _host(t, L):
    return t.cpu().numpy().view(np.uint64).reshape(-1, L)


@pytest.mark.parametrize("fid,L,seed", [(1, 4, 24), (2, 6, 3), (2, 4, 3)])
def test_2pow24_elementwise_vs_threaded_oracle(fid, L, seed):
    p, g = R.FIELDS[fid]
    pl = _plan(fid, 24, L)
    t = pl.empty()
    pl.fill(t, "random", seed=seed)
    x = _host(t, L).copy()
    pl.forward(t)
    exp = OC.ntt_mp_par(x, p, g, THREADS)
    assert np.array_equal(_host(t, L), exp), (fid, L, "forward")
    del exp
    t.copy_(torch.from_numpy(x.view(np.int64)).to(t.device))
    pl.inverse(t)
    exp = OC.ntt_mp_par(x, p, g, THREADS, inverse=True)
    assert np.array_equal(_host(t, L), exp), (fid, L, "inverse")


def test_p_path_2pow26_elementwise():
    p, g = R.FIELDS[0]
    pl = _plan(0, 26, 1)
    t = pl.empty()
    pl.fill(t, "random", seed=26)
    x = t.cpu().numpy().copy()
    pl.forward(t)
    assert np.array_equal(t.cpu().numpy(), OC.ntt_u64(x, p, g))
    pl.inverse(t)
    assert np.array_equal(t.cpu().numpy(), x)


def _kat_check_columns(shares, layouts, n, p, g, L, ks):
    for k in ks:
        k2, k1 = k % layouts[0].n2, k // layouts[0].n2
        rank, kc = k2 // layouts[0].c, k2 % layouts[0].c
        row = shares[rank][k1 * layouts[0].c + kc].cpu().numpy().view(np.uint64).reshape(-1)  # [n1][c]
        v = sum(int(row[i]) << (64 * i) for i in range(L))
        assert v == R.kat_xj(n, p, g, k), k


def _row_index(lay, device):
    i = torch.arange(lay.local_n, dtype=torch.int64, device=device)
    return lay.rank * lay.r + (i >> lay.log_n2) + lay.n1 * (i & (lay.n2 - 1))


def test_c4_fourstep_2pow28_eight_virtual_ranks():
    from ntt_amd.distributed import VirtualRanks
    fid, L, log_n, world = 1, 4, 28, 8
    p, g = R.FIELDS[fid]
    n = 1 << log_n
    vr = VirtualRanks(fid, log_n, L, world, pieces=4)  # the pipelined exchange, as timed in bench_configs
    assert (vr.layout0.log_n1, vr.layout0.log_n2) == (14, 14)  # SURVEY §8e's C4 split (4 passes either way)
    xs = vr.fill(vr.empty(), "iota")
    vr.forward(xs)
    rng = np.random.default_rng(4)
    ks = [0, 1, 2, 3, n // 2, n - 1] + [int(k) for k in rng.integers(0, n, 30)]
    _kat_check_columns(xs, vr.layouts, n, p, g, L, ks)
    vr.inverse(xs)
    for lay, t in zip(vr.layouts, xs):
        assert torch.equal(t[:, 0], _row_index(lay, t.device)) and not bool(t[:, 1:].any()), lay.rank


@pytest.mark.parametrize("log_n", [26, 28])
def test_mplan_large_kat_and_round_trip(log_n):
    from ntt_amd.distributed import MultiPlan
    fid, L = 1, 4
    p, g = R.FIELDS[fid]
    n = 1 << log_n
    mp = MultiPlan(fid, log_n, L, devices=list(range(torch.cuda.device_count())))
    xs = mp.fill(mp.empty(), "iota")
    mp.forward(xs)
    rng = np.random.default_rng(log_n)
    ks = [0, 1, 2, 3, n // 2, n - 1] + [int(k) for k in rng.integers(0, n, 30)]
    _kat_check_columns(xs, mp.layouts, n, p, g, L, ks)
    mp.inverse(xs)
    for lay, t in zip(mp.layouts, xs):
        assert torch.equal(t[:, 0], _row_index(lay, t.device)) and not bool(t[:, 1:].any())
    del mp


def test_c5_polymul_2pow24_elementwise_vs_threaded_oracle():
    """C5: a, b of degree < 2^23 drawn from vector B (seeds 5 and 6), c = a * b of
    length 2^24 by the fused ntt_polymul, every coefficient against the oracle's forward transforms,
    pointwise product and inverse (GZKP-NTT.cu:30-48, 1725-1732).  With deg a + deg b < 2^24 the
    cyclic product is the plain polynomial product."""
    fid, L, log_n = 1, 4, 24
    p, g = R.FIELDS[fid]
    n, half = 1 << log_n, 1 << (log_n - 1)
    pl = _plan(fid, log_n, L)
    a = pl.fill(pl.empty(), "random", seed=5)
    b = pl.fill(pl.empty(), "random", seed=6)
    a[half:] = 0
    b[half:] = 0
    ah, bh = _host(a, L).copy(), _host(b, L).copy()
    c = pl.empty()
    pl.polymul(a, b, c)
    got = _host(c, L)
    A = OC.ntt_mp_par(ah, p, g, THREADS)
    B = OC.ntt_mp_par(bh, p, g, THREADS)
    exp = OC.ntt_mp_par(OC.mul_mp(A, B, p), p, g, THREADS, inverse=True)
    assert np.array_equal(got, exp)
    assert not got[n - 1].any()  # degree < 2^24 - 1


C4_SEED = 4
C4_KS = [1, 0x5A5A5A5, (1 << 28) - 3]  # a low, a scattered and a top index (~4 s each on 16 cores)


@pytest.fixture(scope="module")
def c4_expected():
    return OC.eval_random(1, 28, C4_SEED, C4_KS, 4, threads=THREADS)


def test_c4_random_2pow28_plain_sampled_vs_definition(c4_expected):
    pl = _plan(1, 28, 4)
    t = pl.fill(pl.empty(), "random", seed=C4_SEED)
    pl.forward(t)
    got = OC.limbs_to_ints(_host(t[C4_KS], 4))
    assert got == c4_expected
    del t, pl


def test_c4_random_2pow28_fourstep_sampled_vs_definition(c4_expected):
    from ntt_amd.distributed import VirtualRanks
    vr = VirtualRanks(1, 28, 4, 8, pieces=4)
    xs = vr.fill(vr.empty(), "random", seed=C4_SEED)
    vr.forward(xs)
    L0 = vr.layout0
    got = []
    for k in C4_KS:
        k2, k1 = k % L0.n2, k // L0.n2
        rank, kc = k2 // L0.c, k2 % L0.c
        got.append(OC.limbs_to_ints(_host(xs[rank][k1 * L0.c + kc].reshape(1, 4), 4))[0])
    assert got == c4_expected
