"""GPU parity on the edge vectors of SURVEY §8d (zeros, all p-1, deltas) and on adversarial inputs
that push the kernels' lazy bounds (unnormalised butterflies, quotient-estimate reductions) to
their maxima.  Every check is bit-exact: against the C oracle (a restatement of
GZKP-NTT.cu:30-48) where it is fast, and against closed forms at the multi-pass sizes:

* constant c:        X_0 = n c mod p, X_k = 0 (k != 0)
* delta c at j0:     X_k = c w^(j0 k)
* zeros:             zeros
"""
import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu

FIELD_CASES = [(1, 4), (2, 4), (1, 6), (2, 6), (0, 4)]


def _plan(fid, log_n, L):
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=fid, log_n=log_n, limbs64=L, device=0)


def _limbs(values, L):
    out = np.zeros((len(values), L), dtype=np.uint64)
    for j, v in enumerate(values):
        for i in range(L):
            out[j, i] = (v >> (64 * i)) & ((1 << 64) - 1)
    return out


def _const_limbs(v, n, L):
    row = _limbs([v], L)[0]
    return np.tile(row, (n, 1))


def _values(arr):
    L = arr.shape[1]
    return [sum(int(arr[j, i]) << (64 * i) for i in range(L)) for j in range(arr.shape[0])]


def _run(pl, host, inverse=False):
    t = torch.from_numpy(np.ascontiguousarray(host).view(np.int64)).to("cuda:0").reshape(host.shape)
    (pl.inverse if inverse else pl.forward)(t)
    # the checked build (libntt_debug.so, tests/test_gpu_debug_build.py) checks every lazy bound in the
    # kernels: these inputs drive them to their maxima, so no check may fire; the product build reports 0
    assert pl.device_status() == 0, hex(pl.device_status())
    return t.cpu().numpy().view(np.uint64).reshape(host.shape)


@pytest.mark.parametrize("fid,L", FIELD_CASES)
@pytest.mark.parametrize("log_n", [3, 11, 12, 16, 20])
def test_constant_and_zero_vectors(fid, L, log_n):
    p, g = R.FIELDS[fid]
    n = 1 << log_n
    pl = _plan(fid, log_n, L)
    assert not _run(pl, np.zeros((n, L), dtype=np.uint64)).any()
    for c in (p - 1, p - 2, (p - 1) // 2, 1):
        got = _run(pl, _const_limbs(c, n, L))
        assert _values(got[:1]) == [n * c % p], (fid, L, log_n, c)
        assert not got[1:].any(), (fid, L, log_n, c)
        # inverse of the constant: X_0 = c (n^-1 n), X_k = 0
        got = _run(pl, _const_limbs(c, n, L), inverse=True)
        assert _values(got[:1]) == [c] and not got[1:].any(), (fid, L, log_n, c)


@pytest.mark.parametrize("fid,L", FIELD_CASES)
@pytest.mark.parametrize("log_n", [12, 18, 22])
def test_deltas(fid, L, log_n):
    p, g = R.FIELDS[fid]
    n = 1 << log_n
    w = R.root_of_unity(p, g, n)
    pl = _plan(fid, log_n, L)
    rng = np.random.default_rng(log_n + 7 * fid)
    ks = [0, 1, 2, n // 2, n - 1] + [int(k) for k in rng.integers(0, n, 16)]
    for j0 in (0, 1, n - 1, n // 3):
        c = p - 1
        host = np.zeros((n, L), dtype=np.uint64)
        host[j0] = _limbs([c], L)[0]
        got = _run(pl, host)
        vals = _values(got[ks])
        assert vals == [c * pow(w, j0 * k, p) % p for k in ks], (fid, L, log_n, j0)


@pytest.mark.parametrize("fid,L", FIELD_CASES)
def test_adversarial_near_p_against_oracle(fid, L):
    """x_j in {p-1, p-2, 0} patterns and p-1-(small): every butterfly sum/difference sits at its
    lazy bound; compared element by element with the C oracle through the multi-pass path."""
    p, g = R.FIELDS[fid]
    for log_n in (12, 14, 16):
        n = 1 << log_n
        rng = np.random.default_rng(log_n)
        pattern = rng.integers(0, 4, n)
        vals = [(p - 1, p - 2, 0, p - 1 - int(rng.integers(0, 1 << 20)))[int(s)] for s in pattern]
        x = _limbs(vals, L)
        got = _run(_plan(fid, log_n, L), x)
        exp = OC.ntt_mp(x, p, g, False)
        assert np.array_equal(got, exp), (fid, L, log_n)


@pytest.mark.parametrize("fid,L", [(1, 4), (2, 6), (0, 1), (0, 4)])
def test_count_noncanonical(fid, L):
    """ntt_count_noncanonical: synthetic inputs are canonical; p, p + 1 and all-ones limbs are not,
    p - 1 is."""
    from ntt_amd.ntt import NTTPlan, to_device
    p, _ = R.FIELDS[fid]
    pl = NTTPlan(fid, 12, L)
    t = pl.fill(pl.empty(), "random", seed=3)
    assert pl.count_noncanonical(t) == 0
    bad = to_device([p, p + 1, (1 << (64 * L - 1)) - 1, p - 1], L)
    t[5:9] = bad
    t[20] = -1  # all limbs 0xffff...: not a residue in any layout
    assert pl.count_noncanonical(t) == 4


RIVAL_SCHEDULES = ["stockham", "gzkp", "naive", "no_swap", "bellperson", "v1", "v2", "v3", "v4"]


@pytest.mark.parametrize("sched", RIVAL_SCHEDULES)
@pytest.mark.parametrize("fid,L", [(1, 4), (2, 4), (0, 1)])
def test_rival_schedules_on_edge_vectors(fid, L, sched):
    """The rival schedules (test_gpu_rivals.py) on the same adversarial inputs: near-p patterns against
    the oracle, and the constant p - 1 (X_0 = n (p - 1), the rest 0); through the checked build no
    lazy-bound or output check may fire (k_bealto's rounds keep < 4p between LDS stages)."""
    from ntt_amd.ntt import NTTPlan
    p, g = R.FIELDS[fid]
    for log_n in (14, 16):  # the multi-pass rivals need >= 2 passes of the P tile (2^13)
        n = 1 << log_n
        pl = NTTPlan(field_id=fid, log_n=log_n, limbs64=L, device=0, stockham=sched == "stockham",
                     gzkp=sched == "gzkp", naive=sched == "naive", no_swap=sched == "no_swap",
                     bealto=sched if sched in ("bellperson", "v1", "v2", "v3", "v4") else "")
        rng = np.random.default_rng(log_n + 3)
        pattern = rng.integers(0, 4, n)
        vals = [(p - 1, p - 2, 0, p - 1 - int(rng.integers(0, 1 << 20)))[int(s)] for s in pattern]
        x = _limbs(vals, L)
        got = _run(pl, x) if L > 1 else _run1(pl, x)
        assert np.array_equal(got, OC.ntt_mp(x, p, g, False)), (fid, L, log_n, sched)
        c = _const_limbs(p - 1, n, L)
        got = _run(pl, c) if L > 1 else _run1(pl, c)
        assert _values(got[:1]) == [n * (p - 1) % p] and not got[1:].any(), (fid, L, log_n, sched)


def _run1(pl, host):
    """_run for the 1-limb (`long long`) layout: a flat tensor"""
    t = torch.from_numpy(np.ascontiguousarray(host[:, 0]).view(np.int64)).to("cuda:0")
    pl.forward(t)
    assert pl.device_status() == 0, hex(pl.device_status())
    return t.cpu().numpy().view(np.uint64).reshape(host.shape)
