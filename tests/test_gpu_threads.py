"""The reference-shaped shims (SSIP, NTT_GZKP_256) called from several host threads at once.

The shims keep one cached plan per (modulus, generator, size, device) -- the persistent form of the
reference drivers' per-call table setup (GZKP-NTT.cu:1452-1558, big-num.cu:260-353) -- so threads
transforming different buffers of the same size share a plan and its scratch.  ctypes releases the
GIL around each call, so these threads really overlap.  Also: the error state is per thread
(ntt_last_error), so one thread's failing calls never show up as another thread's error.
"""
import ctypes as C
import threading

import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu
THREADS, ROUNDS = 8, 6


def _run_threads(fn, n):
    errs = []

    def wrap(i):
        try:
            fn(i)
        except BaseException as e:  # noqa: BLE001 -- reported below
            errs.append((i, repr(e)))

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "thread hung"
    assert not errs, errs


def test_ntt_gzkp_256_shim_concurrent_same_plan():
    """8 threads x 6 calls of NTT_GZKP_256 on their own BN254 vectors (one shared cached plan)."""
    from ntt_amd.ntt import NTT_GZKP
    fid, L, log_n = 1, 4, 16
    p, g = R.FIELDS[fid]
    n = 1 << log_n
    xs = [OC.random_limbs(fid, n, 100 + i, L) for i in range(THREADS)]
    exp = [OC.ntt_mp(x, p, g) for x in xs]
    dev = [torch.from_numpy(x.view(np.int64)).to("cuda:0") for x in xs]

    def work(i):
        for r in range(ROUNDS):
            t = dev[i].clone()
            NTT_GZKP(t, n, p, g)
            got = t.cpu().numpy().view(np.uint64).reshape(-1, L)
            assert np.array_equal(got, exp[i]), (i, r)

    _run_threads(work, THREADS)


def test_ssip_shim_concurrent_same_plan():
    """8 threads x 6 calls of SSIP at 2^18 over P (the reference's own entry point and field)."""
    from ntt_amd.ntt import SSIP
    p, g = R.FIELDS[0]
    n = 1 << 18
    rng = np.random.default_rng(5)
    xs = [rng.integers(0, p, n, dtype=np.int64) for _ in range(THREADS)]
    exp = [OC.ntt_u64(x, p, g) for x in xs]

    def work(i):
        for r in range(ROUNDS):
            t = torch.from_numpy(xs[i]).to("cuda:0")
            SSIP(t, g, 18)
            assert np.array_equal(t.cpu().numpy(), exp[i]), (i, r)

    _run_threads(work, THREADS)


def test_error_state_is_per_thread():
    """One thread keeps failing (NTT_GZKP_256 with a non-power-of-two length: NTT_ERR_ARG) while
    another keeps succeeding through SSIP: each sees only its own ntt_last_error."""
    from ntt_amd import lib as _L
    lib = _L.load()
    p = R.FIELDS[0][0]
    x = torch.arange(1 << 12, dtype=torch.int64, device="cuda:0")
    p32 = (C.c_uint32 * 8)(*[(p >> (32 * i)) & 0xFFFFFFFF for i in range(8)])
    g32 = (C.c_uint32 * 8)(3, 0, 0, 0, 0, 0, 0, 0)
    stop = threading.Event()
    seen = {"bad": set(), "good": set()}

    def bad(_):
        while not stop.is_set():
            rc = lib.NTT_GZKP_256(C.c_void_p(x.data_ptr()), 3, None, 0, p32, g32, 5, 8)
            seen["bad"].add((rc, lib.ntt_last_error()))

    def good(_):
        for _ in range(200):
            y = x.clone()
            lib.SSIP(C.c_void_p(y.data_ptr()), 3, 12)
            seen["good"].add(lib.ntt_last_error())
        stop.set()

    _run_threads(lambda i: (bad if i == 0 else good)(i), 2)
    assert seen["good"] == {0}
    assert all(rc != 0 and err == rc for rc, err in seen["bad"])
