"""The single launches wait across workgroups, so they need their workgroups resident together
(ADVICE r05 medium).  Two guarantees, tested deterministically:

* ordering (ntt_plan.cpp FusedSerial): single launches on one device run one after another, whatever
  streams and plans they come from.  Stream 1 gets a ~1 s sleep kernel, then plan A's single launch;
  stream 2 gets plan B's.  B must not have run while stream 1 still sleeps (B waits for A, A for the
  sleep), and both results must equal the default schedule's with no watchdog report.  B is 2^18 (its
  256 workgroups fit beside the sleep kernel), so without the ordering it would finish at once.
* residency (ntt_kernels_impl.hpp residency_wait): an in-place single launch whose workgroups cannot
  all be resident (a helper kernel, tests/c/occupy.hip, holds 100 KiB of LDS on a few CUs) gives up
  before its first store: the caller's buffer is unchanged, the call is reported (NTT_ERR_DEVICE at
  the next call, ntt_plan_device_status bit 0), and the plan is correct again afterwards.

The reference never waits across blocks: one launch per stage (GZKP-NTT.cu:1509-1545)."""
import ctypes
import os
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OCC = os.path.join(ROOT, "tests", "c", "libocc.so")


def _occ():
    if not os.path.exists(OCC):
        pytest.skip("tests/c/libocc.so not built (python tests/occupy_build.py)")
    lib = ctypes.CDLL(OCC)
    lib.occ_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
    lib.occ_launch.restype = ctypes.c_int
    return lib


def _sleep(ms):
    """a ~ms sleep kernel on the current stream (torch's: one wave, no LDS)"""
    torch.cuda._sleep(int(ms * 2.0e6))  # clock cycles at ~2 GHz


@pytest.mark.parametrize("in_place", [False, True], ids=["scratch", "in_place"])
def test_single_launches_on_two_streams_run_in_order(in_place):
    from ntt_amd.ntt import NTTPlan
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep unavailable")
    a = NTTPlan(1, 20, 4, single_launch=True, in_place=in_place)   # k_fused2b / k_fused2bi
    b = NTTPlan(1, 18, 4, single_launch=True, in_place=in_place)   # k_fused3b / k_fused3bi
    ra, rb = NTTPlan(1, 20, 4), NTTPlan(1, 18, 4)
    xa = a.fill(a.empty(), "random", seed=71)
    xb = b.fill(b.empty(), "random", seed=72)
    wa, wb = xa.clone(), xb.clone()
    ra.forward(wa)
    rb.forward(wb)
    ya, yb = xa.clone(), xb.clone()
    a.forward(ya.clone())  # build both single-launch schedules before the timed part
    b.forward(yb.clone())
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        _sleep(1000)
    a.forward(ya, stream=s1)
    b.forward(yb, stream=s2)
    b_done_early = s2.query()
    s1_busy = not s1.query()
    s1.synchronize()
    s2.synchronize()
    assert s1_busy, "the sleep kernel ended before the check: the test proves nothing"
    assert not b_done_early, "plan B's single launch ran beside plan A's (no ordering)"
    assert torch.equal(ya, wa) and torch.equal(yb, wb)
    assert a.device_status() == 0 and b.device_status() == 0


_CHILD_3BI = r"""
import ctypes, sys, time, torch
sys.path.insert(0, {root!r})
from ntt_amd import lib as L
from ntt_amd.ntt import NTTPlan
occ = ctypes.CDLL({occ!r})
occ.occ_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
pl = NTTPlan(1, 20, 4, in_place=True, single_launch=True)
assert pl.passes == [7, 6, 7], pl.passes  # k_fused3bi: 1024 tiles, one per workgroup slot of the chip
ref = NTTPlan(1, 20, 4)
x = pl.fill(pl.empty(), "random", seed=81)
want = x.clone(); ref.forward(want)
y = x.clone(); pl.forward(y); torch.cuda.synchronize()
assert torch.equal(y, want) and pl.device_status() == 0
side = torch.cuda.Stream()
assert occ.occ_launch(8, 100 * 1024, 1500.0, ctypes.c_void_p(side.cuda_stream)) == 0
time.sleep(0.1)
pl.set_watchdog(1 << 14)
y = x.clone(); pl.forward(y); torch.cuda.synchronize()
assert torch.equal(y, x), "an abandoned in-place launch stored"
try:
    pl.forward(x.clone()); print("no error"); sys.exit(1)
except L.NTTError as e:
    assert e.status == L.NTT_ERR_DEVICE
assert pl.device_status() & 1
pl.set_watchdog()
y = x.clone(); pl.forward(y); torch.cuda.synchronize()
assert torch.equal(y, want) and pl.device_status() == 0
print("child ok")
"""


def test_in_place_single_launch_without_residency_stores_nothing():
    """k_fused2bi (2^20 in place, 256 workgroups of 144 KiB LDS, one per CU) with a few CUs held by
    the helper kernel: the launch gives up before any store."""
    from ntt_amd import lib as L
    from ntt_amd.ntt import NTTPlan
    occ = _occ()
    pl = NTTPlan(1, 20, 4, in_place=True, single_launch=True)
    assert pl.passes == [10, 10]
    ref = NTTPlan(1, 20, 4)
    x = pl.fill(pl.empty(), "random", seed=82)
    want = x.clone()
    ref.forward(want)
    y = x.clone()
    pl.forward(y)  # healthy first (builds the single-launch schedule)
    torch.cuda.synchronize()
    assert torch.equal(y, want) and pl.device_status() == 0

    side = torch.cuda.Stream()
    assert occ.occ_launch(8, 100 * 1024, 1500.0, ctypes.c_void_p(side.cuda_stream)) == 0
    time.sleep(0.1)  # the helper's workgroups hold their CUs
    pl.set_watchdog(1 << 14)  # give up after ~16 ms of polls, well inside the helper's 1.5 s
    y = x.clone()
    pl.forward(y)
    torch.cuda.synchronize()  # the last workgroups run once the helper is done, see the decision and leave
    assert torch.equal(y, x), "an abandoned in-place launch stored"
    with pytest.raises(L.NTTError) as ei:
        pl.forward(x.clone())
    assert ei.value.status == L.NTT_ERR_DEVICE
    assert pl.device_status() & 1

    pl.set_watchdog()
    y = x.clone()
    pl.forward(y)
    torch.cuda.synchronize()
    assert torch.equal(y, want) and pl.device_status() == 0


def test_three_pass_in_place_single_launch_without_residency_stores_nothing():
    """The same for k_fused3bi (2^20 in place on 1024-element tiles: NTT_WIDE_TILES=0, read once per
    process, so in a child process): 1024 workgroups, four per CU."""
    _occ()
    env = dict(os.environ, NTT_WIDE_TILES="0")
    r = subprocess.run([sys.executable, "-c", _CHILD_3BI.format(root=ROOT, occ=OCC)], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0 and "child ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
