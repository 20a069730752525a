"""GPU parity of the SURVEY §8f widenings: the coset (low-degree-extension) transform and the
Montgomery-form I/O plan flag, bit-exact against oracle/ntt_ref.py (coset_ntt, coset_intt,
kat_coset_xj, to_mont).  The reference has neither (parity unpinned by the reference itself; the
oracle definitions are pinned against the DFT definition in tests/test_oracle.py)."""
import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu

CASES = [(1, 4), (2, 4), (1, 6), (0, 1), (0, 4)]


def _plan(fid, log_n, L, **kw):
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=fid, log_n=log_n, limbs64=L, device=0, **kw)


def _dev(vals, L):
    from ntt_amd.ntt import to_device
    return to_device(vals, L, "cuda:0")


def _ints(t):
    from ntt_amd.ntt import from_device
    return from_device(t)


@pytest.mark.parametrize("fid,L", CASES)
def test_coset_forward_inverse_small(fid, L):
    p, g = R.FIELDS[fid]
    for log_n in (0, 1, 2, 5, 9, 12):
        n = 1 << log_n
        pl = _plan(fid, log_n, L)
        x = R.random_vector(fid, n, seed=700 + log_n)
        for c in (g, pow(g, 5, p), p - 1):
            t = _dev(x, L)
            pl.forward_coset(t, c)
            got = _ints(t)
            assert got == R.coset_ntt(x, p, g, c), (fid, L, log_n, c)
            pl.inverse_coset(t, c)
            assert _ints(t) == x, (fid, L, log_n, c)


@pytest.mark.parametrize("fid,L,log_n", [(1, 4, 16), (2, 4, 20), (1, 4, 24), (2, 6, 18)])
def test_coset_large_kat_and_round_trip(fid, L, log_n):
    p, g = R.FIELDS[fid]
    n = 1 << log_n
    pl = _plan(fid, log_n, L)
    t = pl.empty()
    pl.fill(t, "iota")
    pl.forward_coset(t, g)
    host = t.cpu().numpy().view(np.uint64).reshape(n, L)
    rng = np.random.default_rng(log_n)
    ks = [0, 1, n // 2, n - 1] + [int(k) for k in rng.integers(0, n, 12)]
    for k in ks:
        v = sum(int(host[k, i]) << (64 * i) for i in range(L))
        assert v == R.kat_coset_xj(n, p, g, g, k), (fid, L, log_n, k)
    pl.inverse_coset(t, g)
    back = t.cpu().numpy().view(np.uint64).reshape(n, L)
    assert np.array_equal(back[:, 0], np.arange(n, dtype=np.uint64)) and not back[:, 1:].any()


@pytest.mark.parametrize("fid,L", [(1, 4), (2, 4), (2, 6), (0, 1)])
def test_montgomery_io(fid, L):
    """Transforms commute with the Montgomery map; the pointwise product / polymul become
    Montgomery products: polymul(aR, bR) = (a b) R."""
    p, g = R.FIELDS[fid]
    for log_n in (3, 12, 16):
        n = 1 << log_n
        pm = _plan(fid, log_n, L, montgomery_io=True)
        a = R.random_vector(fid, n, seed=900 + log_n)
        b = R.random_vector(fid, n, seed=901 + log_n)
        aM = [R.to_mont(v, p, L) for v in a]
        bM = [R.to_mont(v, p, L) for v in b]
        t = _dev(aM, L)
        pm.forward(t)
        A = R.ntt_dit(a, p, g)
        assert _ints(t) == [R.to_mont(v, p, L) for v in A], (fid, L, log_n)
        ta, tb, tc = _dev(aM, L), _dev(bM, L), _dev([0] * n, L)
        pm.polymul(ta, tb, tc)
        assert _ints(tc) == [R.to_mont(v, p, L) for v in R.polymul(a, b, p, g)], (fid, L, log_n)
