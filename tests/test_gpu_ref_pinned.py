"""GPU outputs against the REFERENCE'S OWN outputs (tests/golden/ref_p469762049.npz, made by
tests/golden/make_ref_vectors.py from the reference's CPU NTT compiled out of /root/reference).

Every entry point that can run the reference's field P = 469762049 is checked against them: the
8-B ``long long`` plan path and the reference-shaped ``SSIP`` shim (GZKP-NTT.cu:1452), the 256-bit
``NTT_GZKP_256`` shim with the zero-padded P (big-num.cu:260) and the 48-B (6 x 64-bit) layout.
Full vectors at 2^0..2^12, the inverse recipe (GZKP-NTT.cu:1725-1732), and 64 sampled outputs of
x_j = j and of the seeded vector at 2^16..2^26.
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle_c as OC
from oracle import ref_c

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_p469762049.npz"))
P = 469762049


def _rand(log_n, seed):
    return OC.random_limbs(0, 1 << log_n, seed=seed, L=1)[:, 0].astype(np.int64)


def _plan(log_n, L):
    from ntt_amd.ntt import NTTPlan
    if L == 1:
        return NTTPlan(field_id=0, log_n=log_n, limbs64=1, device=0)
    return NTTPlan(log_n=log_n, limbs64=L, modulus=P, generator=3, device=0)


def _dev(x, L):
    h = np.zeros((x.size, L), dtype=np.int64)
    h[:, 0] = x
    t = torch.from_numpy(h).to("cuda:0")
    return t.reshape(-1) if L == 1 else t


def _low(t, L):
    a = t.cpu().numpy()
    if L == 1:
        return a.reshape(-1)
    assert not a[:, 1:].any()
    return a[:, 0]


@pytest.mark.parametrize("L", [1, 4, 6])
def test_full_vectors_vs_reference(L):
    for log_n in range(0, 13):
        n = 1 << log_n
        pl = _plan(log_n, L)
        t = _dev(np.arange(n, dtype=np.int64), L)
        pl.forward(t)
        assert np.array_equal(_low(t, L), GOLD[f"fwd_iota_{log_n}"]), (L, log_n)
        x = _rand(log_n, 1000 + log_n)
        t = _dev(x, L)
        pl.forward(t)
        assert np.array_equal(_low(t, L), GOLD[f"fwd_rand_{log_n}"]), (L, log_n)
        t = _dev(x, L)
        pl.inverse(t)
        assert np.array_equal(_low(t, L), GOLD[f"inv_rand_{log_n}"]), (L, log_n)


@pytest.mark.parametrize("L,log_n", [(1, 16), (1, 20), (1, 22), (1, 24), (1, 26), (4, 16), (4, 20), (4, 22),
                                     (4, 24), (6, 20)])
def test_sampled_vs_reference(L, log_n):
    n = 1 << log_n
    idx = torch.from_numpy(GOLD[f"samp_idx_{log_n}"]).to("cuda:0")
    pl = _plan(log_n, L)
    t = _dev(np.arange(n, dtype=np.int64), L)
    pl.forward(t)
    assert np.array_equal(_low(t[idx], L), GOLD[f"samp_iota_{log_n}"]), (L, log_n)
    t = _dev(_rand(log_n, 2000 + log_n), L)
    pl.forward(t)
    assert np.array_equal(_low(t[idx], L), GOLD[f"samp_rand_{log_n}"]), (L, log_n)


def test_ssip_shim_vs_reference():
    """The reference-shaped entry point itself (blocking, default stream)."""
    from ntt_amd.ntt import SSIP
    for log_n in list(range(1, 13)) + [16, 20, 24, 26]:
        n = 1 << log_n
        key = f"fwd_rand_{log_n}" if log_n <= 12 else f"samp_rand_{log_n}"
        x = torch.from_numpy(_rand(log_n, (1000 if log_n <= 12 else 2000) + log_n)).to("cuda:0")
        SSIP(x, 3, log_n)
        got = x.cpu().numpy()
        if log_n > 12:
            got = got[GOLD[f"samp_idx_{log_n}"]]
        assert np.array_equal(got, GOLD[key]), log_n
        del n


def test_ntt_gzkp_256_shim_vs_reference():
    from ntt_amd.ntt import NTT_GZKP
    for log_n in range(5, 13):  # big-num.cu main's sizes
        x = _rand(log_n, 1000 + log_n)
        t = _dev(x, 4)
        NTT_GZKP(t, 1 << log_n, P, 3)
        assert np.array_equal(_low(t, 4), GOLD[f"fwd_rand_{log_n}"]), log_n


@pytest.mark.skipif(not ref_c.available(), reason="oracle/_ref (the reference's CPU NTT) not built")
def test_live_reference_2pow22_elementwise():
    """The full 2^22 output of the reference's own CPU NTT (run on this box's host) vs the GPU."""
    log_n = 22
    x = _rand(log_n, 77)
    exp = ref_c.ntt(x)
    for L in (1, 4):
        pl = _plan(log_n, L)
        t = _dev(x, L)
        pl.forward(t)
        assert np.array_equal(_low(t, L), exp), L
        pl.inverse(t)
        assert np.array_equal(_low(t, L), x), L
