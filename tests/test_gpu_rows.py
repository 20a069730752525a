"""GPU parity of KIND_ROWS: batches of short single-tile transforms (n = 2^3..2^7) run TILE / n transforms
per workgroup (ntt_forward_batch / ntt_inverse_batch of short vectors, and the four-step's row launches
of such n, ntt_rplan); 2^8 and 2^9 keep one transform per workgroup and are checked alongside.
Every transform of the batch is compared with the C oracle (GZKP-NTT.cu:30-48 restated); batches that
the per-workgroup count does not divide take KIND_SINGLE and are checked the same way.
"""
import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu

TILE_LOG = 10  # the 256-bit engines' tile: 1024 elements


def _plan(fid, log_n, L):
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=fid, log_n=log_n, limbs64=L, device=0)


def _to_dev(arr, L):
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.int64)).to("cuda:0").reshape(-1, L)


def _host(t, L):
    return t.cpu().numpy().view(np.uint64).reshape(-1, L)


def _check_batch(fid, L, log_n, batch, x):
    p, g = R.FIELDS[fid]
    pl = _plan(fid, log_n, L)
    t = pl.empty(batch)
    t.copy_(_to_dev(x, L))
    pl.forward_batch(t, batch)
    got = _host(t, L)
    n = 1 << log_n
    for s in range(batch):
        exp = OC.ntt_mp(x[s * n:(s + 1) * n], p, g, False)
        assert np.array_equal(got[s * n:(s + 1) * n], exp), (fid, log_n, batch, s)
    pl.inverse_batch(t, batch)
    assert np.array_equal(_host(t, L), x), (fid, log_n, batch)
    # the inverse alone, against the oracle's inverse
    t.copy_(_to_dev(x, L))
    pl.inverse_batch(t, batch)
    got = _host(t, L)
    for s in range(batch):
        exp = OC.ntt_mp(x[s * n:(s + 1) * n], p, g, True)
        assert np.array_equal(got[s * n:(s + 1) * n], exp), ("inverse", fid, log_n, batch, s)


@pytest.mark.parametrize("fid,L", [(1, 4), (2, 4), (2, 6)])  # (2, 6): the 48-B layout engine
@pytest.mark.parametrize("log_n", [3, 4, 5, 6, 7, 8, 9])
def test_rows_batch_vs_oracle(fid, L, log_n):
    per_wg = 1 << (TILE_LOG - log_n)
    for batch in (per_wg, 3 * per_wg, 3 * per_wg + 1):  # KIND_ROWS, KIND_ROWS, KIND_SINGLE (not divisible)
        x = np.concatenate([OC.random_limbs(fid, 1 << log_n, seed=1000 * log_n + s, L=L) for s in range(batch)])
        _check_batch(fid, L, log_n, batch, x)


@pytest.mark.parametrize("log_n", [3, 6, 7, 8])
def test_rows_edge_values(log_n):
    """Every input p - 1 and alternating 0 / p - 1 (the lazy butterflies' largest intermediate bounds)."""
    fid, L = 1, 4
    p, _ = R.FIELDS[fid]
    n = 1 << log_n
    batch = 2 << (TILE_LOG - log_n)
    vals = np.empty(n * batch, dtype=object)
    vals[: n * batch // 2] = p - 1
    vals[n * batch // 2:] = [(p - 1) if i % 2 else 0 for i in range(n * batch // 2)]
    x = np.array([[(int(v) >> (64 * k)) & (2**64 - 1) for k in range(L)] for v in vals], dtype=np.uint64)
    _check_batch(fid, L, log_n, batch, x)


@pytest.mark.parametrize("log_n", [7, 8])
def test_rows_large_batch_round_trip(log_n):
    """2^15 rows in one call (2^8: the four-step's row-launch shape at 2^24): sampled transforms
    against the oracle, then the inverse round trip on all of them."""
    fid, L, batch = 1, 4, 1 << 15
    p, g = R.FIELDS[fid]
    n = 1 << log_n
    from ntt_amd.ntt import NTTPlan
    pl = _plan(fid, log_n, L)
    t = pl.empty(batch)
    NTTPlan(fid, log_n + 15, L).fill(t, "random", seed=7)
    x = _host(t, L).copy()
    pl.forward_batch(t, batch)
    got = _host(t, L)
    for s in (0, 1, 2, 3, 4097, batch - 1):
        assert np.array_equal(got[s * n:(s + 1) * n], OC.ntt_mp(x[s * n:(s + 1) * n], p, g, False)), s
    pl.inverse_batch(t, batch)
    assert np.array_equal(_host(t, L), x)


@pytest.mark.parametrize("fid,L", [(1, 4), (2, 6)])
def test_rows_montgomery_io(fid, L):
    """NTT_PLAN_MONTGOMERY_IO through KIND_ROWS: every transform of the batch commutes with the
    Montgomery map (forward(a R) = forward(a) R), and the inverse brings the batch back."""
    from ntt_amd.ntt import NTTPlan
    p, g = R.FIELDS[fid]
    log_n = 6
    n, batch = 1 << log_n, 2 << (TILE_LOG - 6)
    pm = NTTPlan(field_id=fid, log_n=log_n, limbs64=L, device=0, montgomery_io=True)
    vecs = [R.random_vector(fid, n, seed=1200 + s) for s in range(batch)]
    words = lambda v: [(int(v) >> (64 * k)) & (2**64 - 1) for k in range(L)]
    x = np.array([words(R.to_mont(v, p, L)) for vec in vecs for v in vec], dtype=np.uint64)
    t = pm.empty(batch)
    t.copy_(_to_dev(x, L))
    pm.forward_batch(t, batch)
    got = _host(t, L)
    for s, vec in enumerate(vecs):
        exp = np.array([words(R.to_mont(v, p, L)) for v in R.ntt_dit(vec, p, g)], dtype=np.uint64)
        assert np.array_equal(got[s * n:(s + 1) * n], exp), (fid, s)
    pm.inverse_batch(t, batch)
    assert np.array_equal(_host(t, L), x)


@pytest.mark.parametrize("log_n", [3, 5, 6, 7, 9])
def test_rows_p_field_vs_oracle(log_n):
    """P469762049 (8-B elements, 8192-element tiles): KIND_ROWS up to 2^6 points; 2^7 and up keep one
    transform per workgroup.  Every transform against the reference-pinned C oracle, both directions."""
    from ntt_amd.ntt import NTTPlan
    p, g = R.FIELDS[0]
    n = 1 << log_n
    per_wg = 1 << (13 - log_n)
    pl = NTTPlan(field_id=0, log_n=log_n, limbs64=1, device=0)
    for batch in (per_wg, 2 * per_wg + 1):
        x = np.concatenate([OC.random_limbs(0, n, seed=3000 * log_n + s, L=1)[:, 0] for s in range(batch)])
        x = x.astype(np.int64) % p  # canonical inputs (as test_gpu_parity does for P)
        t = torch.from_numpy(x.copy()).to("cuda:0")
        pl.forward_batch(t, batch)
        got = t.cpu().numpy()
        for s in range(batch):
            assert np.array_equal(got[s * n:(s + 1) * n], OC.ntt_u64(x[s * n:(s + 1) * n], p, g)), (log_n, batch, s)
        pl.inverse_batch(t, batch)
        assert np.array_equal(t.cpu().numpy(), x), (log_n, batch)
