"""BASELINE config 2 as a single kernel (VERDICT r02 missing 1): NTT_PLAN_SINGLE_LAUNCH runs a 3-pass
transform as ONE persistent launch, in both forms (NTT_FUSED_MODE, read when a plan builds its fused
schedule): "1" two grid barriers (k_fused3b, the default; a plain launch since round 5, the cooperative
launch retired in round 6), "0" the passes'
tiles handed between workgroups through dependency counters (k_fused3).  Checked bit for bit against the threaded C oracle (GZKP-NTT.cu:30-48, inverse
GZKP-NTT.cu:1725-1732) at C2's 2^20 on vectors A (x_j = j, the reference's input) and B, against the
default 3-launch schedule at every fused size 2^18..2^24 for BN254 and BLS12-381 (4 limbs), over
repeated calls (the counters re-zero themselves), and that exactly one launch ran with the watchdog
silent."""
import os

import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8"))))


def _plan(fid, log_n, single):
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=fid, log_n=log_n, limbs64=4, device=0, single_launch=single)


def _host(t):
    return t.cpu().numpy().view(np.uint64).reshape(-1, 4)


@pytest.fixture(params=["1", "0"], ids=["barriers", "dataflow"])
def fused_mode(request, monkeypatch):
    monkeypatch.setenv("NTT_FUSED_MODE", request.param)
    return request.param


@pytest.mark.parametrize("kind", ["iota", "random"])
def test_c2_2pow20_single_launch_vs_oracle(kind):
    """C2 as ONE kernel (round 5): the two passes of the 4096-element tiles (10 + 10) with one grid
    barrier, a plain launch (k_fused2b)."""
    fid, log_n = 1, 20
    p, g = R.FIELDS[fid]
    pl = _plan(fid, log_n, True)
    assert pl.passes == [10, 10]
    t = pl.fill(pl.empty(), kind, seed=2)
    x = _host(t).copy()
    pl.set_profiling(True)
    pl.forward(t)
    launches = pl.last_launch_ms()
    pl.set_profiling(False)
    assert len(launches) == 1, launches  # one kernel for the whole transform
    assert np.array_equal(_host(t), OC.ntt_mp_par(x, p, g, THREADS))
    if kind == "iota":
        n = 1 << log_n
        got = _host(t)
        for k in (0, 1, 2, n // 2, n - 1):
            assert OC.limbs_to_ints(got[k:k + 1])[0] == R.kat_xj(n, p, g, k)
    t.copy_(torch.from_numpy(x.view(np.int64)).to(t.device))
    pl.inverse(t)
    assert np.array_equal(_host(t), OC.ntt_mp_par(x, p, g, THREADS, inverse=True))
    assert pl.device_status() == 0


@pytest.mark.parametrize("fid", [1, 2])
@pytest.mark.parametrize("log_n", [18, 19, 20, 21, 22, 23, 24])
def test_single_launch_matches_default_schedule(fid, log_n, fused_mode):
    ref = _plan(fid, log_n, False)
    fused = _plan(fid, log_n, True)
    # 2^20 plans report their single-vector schedule, the 4096-element tiles' 10 + 10 (k_fused2b)
    assert fused.passes == ref.passes and len(fused.passes) == (2 if log_n == 20 else 3)
    a = ref.fill(ref.empty(), "random", seed=log_n)
    b = a.clone()
    x = a.clone()
    fused.set_profiling(True)
    for _ in range(3):  # repeated calls: every launch must leave the counters zeroed
        ref.forward(a)
        fused.forward(b)
        assert torch.equal(a, b), log_n
        ref.inverse(a)
        fused.inverse(b)
        assert torch.equal(a, b), log_n
    assert torch.equal(b, x)  # round trip
    assert len(fused.last_launch_ms()) == 1
    fused.set_profiling(False)
    assert fused.device_status() == 0


def test_single_launch_edges_and_interleaving():
    """Edge vectors (zeros, p - 1 everywhere, deltas) through the fused kernel, interleaved with a
    default-schedule plan of the same size on the same stream."""
    fid, log_n = 1, 20
    p, g = R.FIELDS[fid]
    n = 1 << log_n
    ref = _plan(fid, log_n, False)
    fused = _plan(fid, log_n, True)
    pm1 = OC.ints_to_limbs([p - 1], 4)[0]
    for name in ("zeros", "pm1", "delta0", "deltaN"):
        h = np.zeros((n, 4), dtype=np.uint64)
        if name == "pm1":
            h[:] = pm1
        elif name == "delta0":
            h[0] = pm1
        elif name == "deltaN":
            h[n - 1] = pm1
        a = torch.from_numpy(h.view(np.int64)).to("cuda:0")
        b = a.clone()
        ref.forward(a)
        fused.forward(b)
        assert torch.equal(a, b), name
    assert fused.device_status() == 0


# ---- the in-place single launch (BASELINE C2's "single-kernel self-sort-in-place")
def _ip_plan(fid, log_n, single=True):
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=fid, log_n=log_n, limbs64=4, device=0, single_launch=single, in_place=True)


@pytest.mark.parametrize("kind", ["iota", "random"])
def test_c2_2pow20_in_place_single_launch_vs_oracle(kind):
    """2^20 BN254 as ONE kernel with no scratch (round 5: k_fused2bi on 4096-element tiles): pass 1 in
    place, the final pass's digit reversal behind a second grid barrier.  Bit for bit against the
    threaded C oracle (forward and inverse), the KAT of x_j = j, exactly one launch, and no plan
    buffer."""
    fid, log_n = 1, 20
    p, g = R.FIELDS[fid]
    pl = _ip_plan(fid, log_n)
    assert pl.passes == [10, 10]
    t = pl.fill(pl.empty(), kind, seed=2)
    x = _host(t).copy()
    pl.set_profiling(True)
    pl.forward(t)
    launches = pl.last_launch_ms()
    pl.set_profiling(False)
    assert len(launches) == 1, launches
    assert np.array_equal(_host(t), OC.ntt_mp_par(x, p, g, THREADS))
    if kind == "iota":
        n = 1 << log_n
        got = _host(t)
        for k in (0, 1, 2, n // 2, n - 1):
            assert OC.limbs_to_ints(got[k:k + 1])[0] == R.kat_xj(n, p, g, k)
    t.copy_(torch.from_numpy(x.view(np.int64)).to(t.device))
    pl.inverse(t)
    assert np.array_equal(_host(t), OC.ntt_mp_par(x, p, g, THREADS, inverse=True))
    assert pl.device_status() == 0


@pytest.mark.parametrize("fid", [1, 2])
@pytest.mark.parametrize("log_n", [18, 19, 20, 21])
def test_in_place_single_launch_matches_default(fid, log_n):
    """2^18..2^20 run as one launch (every final tile resident); 2^21 has more tiles than the device
    keeps resident and falls back to the in-place multi-launch schedule.  Both equal the default plan,
    over repeated calls (the barrier words re-arm) and the round trip."""
    ip = _ip_plan(fid, log_n)
    df = _plan(fid, log_n, False)
    for seed in (1, 2, 3):
        a = ip.fill(ip.empty(), "random", seed=seed)
        b = a.clone()
        x = a.clone()
        ip.set_profiling(True)
        ip.forward(a)
        nl = len(ip.last_launch_ms())
        ip.set_profiling(False)
        df.forward(b)
        assert torch.equal(a, b), (fid, log_n, seed)
        assert nl == (1 if log_n <= 20 else 3), nl
        ip.inverse(a)
        assert torch.equal(a, x)
    assert ip.device_status() == 0


_PLAIN_LAUNCH_CHECK = r"""
import sys, torch
sys.path.insert(0, {root!r})
from ntt_amd.ntt import NTTPlan
for log_n, ip in ((18, False), (20, False), (18, True), (20, True)):
    ref = NTTPlan(1, log_n, 4)
    one = NTTPlan(1, log_n, 4, single_launch=True, in_place=ip)
    x = ref.fill(ref.empty(), "random", seed=7)
    a, b = x.clone(), x.clone()
    ref.forward(a)
    for _ in range(3):  # repeated calls: the barrier words re-zero themselves
        b.copy_(x)
        one.forward(b)
    assert torch.equal(a, b), (log_n, ip)
    one.inverse(b)
    assert torch.equal(b, x), (log_n, ip)
    assert one.device_status() == 0
print("plain-launch ok")
"""


@pytest.mark.parametrize("env", [{"NTT_WIDE_TILES": "0", "NTT_FUSED_MODE": "1"},
                                 {"NTT_WIDE_TILES": "0", "NTT_FUSED_MODE": "0"}],
                         ids=["three_pass_2pow20_barriers", "three_pass_2pow20_dataflow"])
def test_grid_barrier_forms_in_child_processes(env):
    """Environment switches are read once per process, so in a child process: NTT_WIDE_TILES=0, the
    1024-element-tile single launches at 2^20 too (k_fused3b / k_fused3 / k_fused3bi, as before round
    5).  Each gives the default schedule's results.  (Round 6 retired the cooperative-launch switch,
    NTT_FUSED_COOP: VERDICT r05 item 5.)"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _PLAIN_LAUNCH_CHECK.format(root=root)], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "plain-launch ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
