"""C4 element by element: 2^28 BN254 Fr, SURVEY §8d vector B (seed 4),
forward and inverse, every coefficient against the threaded C oracle (oracle_ntt_mp_par: the
restatement of GZKP-NTT.cu:30-48 and of the inverse recipe GZKP-NTT.cu:1725-1732, pinned in
test_oracle.py / test_oracle_ref.py), both as the plain one-GPU transform and as the four-step over 8
virtual ranks (one GPU; the all-to-all = device copies, pipelined in 4 pieces as in bench_configs)
gathered through the [n1][c] column-layout / [r][n2] row-layout index maps of DistNTT.

The expected vectors are computed once per module (~25-30 s of oracle time each on 16 threads).
Host memory: the input and both expected vectors, 8 GiB each, plus one gathered result.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8"))))
FID, L, LOG_N, SEED, WORLD = 1, 4, 28, 4, 8


def _plan():
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=FID, log_n=LOG_N, limbs64=L, device=0)


def _host(t):
    return t.cpu().numpy().view(np.uint64).reshape(-1, L)


@pytest.fixture(scope="module")
def vec_b():
    pl = _plan()
    t = pl.fill(pl.empty(), "random", seed=SEED)
    x = _host(t).copy()
    del t, pl
    torch.cuda.empty_cache()
    # the device generator is the host generator: the first 2^16 rows
    assert np.array_equal(OC.random_limbs(FID, 1 << 16, SEED, L), x[:1 << 16])
    return x


@pytest.fixture(scope="module")
def fwd_expected(vec_b):
    p, g = R.FIELDS[FID]
    return OC.ntt_mp_par(vec_b, p, g, THREADS)


@pytest.fixture(scope="module")
def inv_expected(vec_b):
    p, g = R.FIELDS[FID]
    return OC.ntt_mp_par(vec_b, p, g, THREADS, inverse=True)


def _mismatch(got, exp):
    bad = np.nonzero((got != exp).any(axis=1))[0]
    return f"{len(bad)} of {len(exp)} coefficients differ, first at {bad[:5].tolist()}"


def test_c4_plain_forward_elementwise(vec_b, fwd_expected):
    pl = _plan()
    t = pl.empty()
    t.copy_(torch.from_numpy(vec_b.view(np.int64)).to(t.device))
    pl.forward(t)
    got = _host(t)
    assert np.array_equal(got, fwd_expected), _mismatch(got, fwd_expected)
    del t, pl, got
    torch.cuda.empty_cache()


def test_c4_plain_inverse_elementwise(vec_b, inv_expected):
    pl = _plan()
    t = pl.empty()
    t.copy_(torch.from_numpy(vec_b.view(np.int64)).to(t.device))
    pl.inverse(t)
    got = _host(t)
    assert np.array_equal(got, inv_expected), _mismatch(got, inv_expected)
    del t, pl, got
    torch.cuda.empty_cache()


def _vr():
    from ntt_amd.distributed import VirtualRanks
    vr = VirtualRanks(FID, LOG_N, L, WORLD, pieces=4)
    assert (vr.layout0.log_n1, vr.layout0.log_n2) == (14, 14)
    return vr


def test_c4_fourstep_forward_elementwise(fwd_expected):
    vr = _vr()
    xs = vr.fill(vr.empty(), "random", seed=SEED)  # row layout of vector B (DistNTT's fill map)
    vr.forward(xs)
    L0 = vr.layout0
    # column layout: rank g holds [n1][c], (k1, kc) = X[g c + kc + n2 k1]  ->  [n1][G][c] is natural order
    nat = torch.stack([t.view(L0.n1, L0.c, L) for t in xs], dim=1).reshape(-1, L)
    del xs
    got = _host(nat)
    del nat, vr
    torch.cuda.empty_cache()
    assert np.array_equal(got, fwd_expected), _mismatch(got, fwd_expected)


def test_c4_fourstep_inverse_elementwise(vec_b, inv_expected):
    vr = _vr()
    L0 = vr.layout0
    dev = torch.device("cuda:0")
    src = torch.from_numpy(vec_b.view(np.int64)).to(dev).view(L0.n1, WORLD, L0.c, L)
    xs = [src[:, g].contiguous().view(-1, L) for g in range(WORLD)]  # column layout of vector B
    del src
    vr.inverse(xs)
    # row layout: rank g holds [r][n2], (a, j2) = x[g r + a + n1 j2]  ->  [n1][n2]^T is natural order
    nat = torch.cat([t.view(L0.r, L0.n2, L) for t in xs], dim=0).transpose(0, 1).reshape(-1, L)
    del xs
    got = _host(nat)
    del nat, vr
    torch.cuda.empty_cache()
    assert np.array_equal(got, inv_expected), _mismatch(got, inv_expected)
