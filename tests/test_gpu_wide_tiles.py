"""BASELINE config 2 (2^20, 4 x 64-bit limbs) on 4096-element tiles: a default 4-limb plan of 2^20
runs one vector's transforms (forward, inverse, coset, polymul, fused pointwise inverse) on a
second plan of 4096-element tiles in two passes (10 + 10), and batched calls on the 1024-element
tiles (7 + 7 + 6).  Checked bit for bit against the threaded C oracle (GZKP-NTT.cu:30-48, inverse
GZKP-NTT.cu:1725-1732), against the batched path of the same plan, and against a child process
with the second plan switched off (NTT_WIDE_TILES=0, read once per process) for every routed call."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8"))))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _host(t):
    return t.cpu().numpy().view(np.uint64).reshape(-1, 4)


@pytest.mark.parametrize("fid", [1, 2])
@pytest.mark.parametrize("kind", ["iota", "random"])
def test_wide_tiles_vs_oracle(fid, kind):
    from ntt_amd.ntt import NTTPlan
    p, g = R.FIELDS[fid]
    pl = NTTPlan(fid, 20, 4)
    assert pl.passes == [10, 10]
    t = pl.fill(pl.empty(), kind, seed=3)
    x = _host(t).copy()
    pl.set_profiling(True)
    pl.forward(t)
    assert len(pl.last_launch_ms()) == 2  # two passes
    assert np.array_equal(_host(t), OC.ntt_mp_par(x, p, g, THREADS))
    t.copy_(torch.from_numpy(x.view(np.int64)).to(t.device))
    pl.inverse(t)
    assert len(pl.last_launch_ms()) == 2
    pl.set_profiling(False)
    assert np.array_equal(_host(t), OC.ntt_mp_par(x, p, g, THREADS, inverse=True))
    assert pl.device_status() == 0


def test_batch_one_and_batched_paths_agree():
    """Batch 1 runs on the 4096-element tiles (2 launches), batch 2 on the 1024-element tiles
    (3 launches): same outputs, interleaved on one plan."""
    from ntt_amd.ntt import NTTPlan
    pl = NTTPlan(1, 20, 4)
    n = pl.n
    b = pl.empty(2)
    bv = b.view(2, n, -1)
    for i in range(2):
        pl.fill(bv[i], "random", seed=11 + i)
    x0, x1 = bv[0].clone(), bv[1].clone()
    pl.set_profiling(True)
    for _ in range(2):
        pl.forward_batch(b, 2)
        assert len(pl.last_launch_ms()) == 3
        pl.forward(x0)
        assert len(pl.last_launch_ms()) == 2
        pl.forward(x1)
        assert torch.equal(bv[0], x0) and torch.equal(bv[1], x1)
        pl.inverse_batch(b, 2)
        pl.inverse(x0)
        pl.inverse(x1)
        assert torch.equal(bv[0], x0) and torch.equal(bv[1], x1)
    pl.set_profiling(False)


_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, {root!r})
from ntt_amd.ntt import NTTPlan
out = {{}}
for fid in (1, 2):
    for mont in (False, True):
        pl = NTTPlan(fid, 20, 4, montgomery_io=mont)
        a = pl.fill(pl.empty(), "random", seed=21 + fid)
        b = pl.fill(pl.empty(), "random", seed=31 + fid)
        c = pl.empty()
        t = a.clone(); pl.forward(t); out[f"fwd{{fid}}{{int(mont)}}"] = t.cpu().numpy()
        t = a.clone(); pl.inverse(t); out[f"inv{{fid}}{{int(mont)}}"] = t.cpu().numpy()
        t = a.clone(); pl.forward_coset(t, 7); out[f"cf{{fid}}{{int(mont)}}"] = t.cpu().numpy()
        t = a.clone(); pl.inverse_coset(t, 7); out[f"ci{{fid}}{{int(mont)}}"] = t.cpu().numpy()
        pl.polymul(a.clone(), b.clone(), c); out[f"pm{{fid}}{{int(mont)}}"] = c.cpu().numpy()
        pl.inverse_pointwise_batch(a, b, c, 1); out[f"ip{{fid}}{{int(mont)}}"] = c.cpu().numpy()
        out[f"passes{{fid}}{{int(mont)}}"] = np.array(pl.passes)
np.savez({path!r}, **out)
print("child ok")
"""


def test_routed_calls_match_the_1024_tile_plan(tmp_path):
    """forward, inverse, coset both ways, polymul and the fused pointwise inverse of a 2^20 plan
    (BN254, BLS12-381; canonical and Montgomery I/O) against the same calls with NTT_WIDE_TILES=0."""
    from ntt_amd.ntt import NTTPlan
    path = str(tmp_path / "ref.npz")
    env = dict(os.environ, NTT_WIDE_TILES="0")
    r = subprocess.run([sys.executable, "-c", _CHILD.format(root=ROOT, path=path)], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "child ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    ref = np.load(path)
    for fid in (1, 2):
        for mont in (False, True):
            k = f"{fid}{int(mont)}"
            assert list(ref["passes" + k]) == [7, 7, 6]
            pl = NTTPlan(fid, 20, 4, montgomery_io=mont)
            assert pl.passes == [10, 10]
            a = pl.fill(pl.empty(), "random", seed=21 + fid)
            b = pl.fill(pl.empty(), "random", seed=31 + fid)
            c = pl.empty()
            t = a.clone(); pl.forward(t); assert np.array_equal(t.cpu().numpy(), ref["fwd" + k]), k
            t = a.clone(); pl.inverse(t); assert np.array_equal(t.cpu().numpy(), ref["inv" + k]), k
            t = a.clone(); pl.forward_coset(t, 7); assert np.array_equal(t.cpu().numpy(), ref["cf" + k]), k
            t = a.clone(); pl.inverse_coset(t, 7); assert np.array_equal(t.cpu().numpy(), ref["ci" + k]), k
            pl.polymul(a.clone(), b.clone(), c); assert np.array_equal(c.cpu().numpy(), ref["pm" + k]), k
            pl.inverse_pointwise_batch(a, b, c, 1); assert np.array_equal(c.cpu().numpy(), ref["ip" + k]), k
            assert pl.device_status() == 0


def test_other_plans_keep_their_tiles():
    """Only default (or Montgomery-I/O, or single-launch) 4-limb plans of exactly 2^20 take the second
    plan."""
    from ntt_amd.ntt import NTTPlan
    assert NTTPlan(1, 19, 4).passes == [7, 6, 6]
    assert NTTPlan(1, 21, 4).passes == [7, 7, 7]
    if os.environ.get("NTT_TWO_PASS_24") != "1":  # the 12 + 12 A/B switch is off by default
        assert NTTPlan(1, 24, 4).passes == [8, 8, 8]
    assert len(NTTPlan(1, 20, 4, in_place=True).passes) == 3
    # round 5: single-launch plans of 2^20 run the two passes as one launch (k_fused2b / k_fused2bi)
    assert NTTPlan(1, 20, 4, single_launch=True).passes == [10, 10]
    assert NTTPlan(1, 20, 4, single_launch=True, in_place=True).passes == [10, 10]
    assert len(NTTPlan(2, 20, 6).passes) == 3


def test_custom_modulus_plan_and_256_bit_shim_take_the_two_pass_plan():
    """ntt_plan_create_custom with a 4-limb modulus at 2^20 and the reference-shaped NTT_GZKP_256
    shim (its cached plan) run the 4096-element tiles too, with the named plan's results."""
    from ntt_amd.ntt import NTT_GZKP, NTTPlan
    p, g = R.FIELDS[1]
    named = NTTPlan(1, 20, 4)
    custom = NTTPlan(log_n=20, limbs64=4, modulus=p, generator=g)
    assert named.passes == custom.passes == [10, 10]
    x = named.fill(named.empty(), "random", seed=41)
    a, b, c = x.clone(), x.clone(), x.clone()
    named.forward(a)
    custom.forward(b)
    NTT_GZKP(c.view(-1), 1 << 20, p, g)
    assert torch.equal(a, b) and torch.equal(a, c)
    custom.inverse(b)
    assert torch.equal(b, x)


_CHILD_TWO_PASS = r"""
import sys, torch
sys.path.insert(0, {root!r})
from ntt_amd.ntt import NTTPlan
for fid in (1, 2):
    pl = NTTPlan(fid, 24, 4)
    assert pl.passes == [12, 12], pl.passes
    n = pl.n
    b = pl.empty(2)
    bv = b.view(2, n, -1)
    pl.fill(bv[0], "random", seed=61 + fid)
    pl.fill(bv[1], "iota")
    x0, x1 = bv[0].clone(), bv[1].clone()
    pl.set_profiling(True)
    pl.forward(x0)
    assert len(pl.last_launch_ms()) == 2
    pl.set_profiling(False)
    pl.forward(x1)
    pl.forward_batch(b, 2)  # 8 + 8 + 8 on the 1024-element tiles
    assert torch.equal(bv[0], x0) and torch.equal(bv[1], x1), fid
    pl.inverse(x0); pl.inverse(x1); pl.inverse_batch(b, 2)
    assert torch.equal(bv[0], x0) and torch.equal(bv[1], x1), fid
    assert pl.device_status() == 0
print("child ok")
"""


def test_two_pass_24_switch_is_bit_exact():
    """NTT_TWO_PASS_24=1 (an A/B switch: measured slower): a 2^24 4-limb
    plan runs one vector's transforms as 12 + 12 on 4096-element tiles, one column per column-pass
    tile.  Forward and inverse, BN254 and BLS12-381, bit for bit against the same plan's batched
    8 + 8 + 8 path."""
    env = dict(os.environ, NTT_TWO_PASS_24="1")
    r = subprocess.run([sys.executable, "-c", _CHILD_TWO_PASS.format(root=ROOT)], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0 and "child ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


_CHILD_FAIL = r"""
import sys, numpy as np, torch
sys.path.insert(0, {root!r})
from ntt_amd.ntt import NTTPlan
pl = NTTPlan(1, 20, 4)  # the second plan's init is refused (NTT_TEST_WIDE_FAIL=1)
assert pl.passes == [7, 7, 6], pl.passes
x = pl.fill(pl.empty(), "random", seed=51)
t = x.clone()
pl.forward(t)  # the first call on the plan: must not see the refused allocation's error
y = t.clone()
pl.inverse(y)
assert torch.equal(y, x)
np.save({path!r}, t.cpu().numpy())
print("child ok")
"""


def test_failed_second_plan_leaves_no_error_behind(tmp_path):
    """when the 4096-element-tile plan cannot be built (its allocation refused),
    the plan runs alone on 1024-element tiles and its first forward returns NTT_OK with the same
    output as a plan that has the second plan (the refused allocation's sticky error is cleared).
    The refusal hook exists in the checked build only: the child loads libntt_debug.so."""
    from ntt_amd.ntt import NTTPlan
    dbg = os.path.join(ROOT, "ntt_amd", "libntt_debug.so")
    if not os.path.exists(dbg):
        pytest.skip("checked build not built (python -m ntt_amd.build --debug)")
    path = str(tmp_path / "fail.npy")
    env = dict(os.environ, NTT_TEST_WIDE_FAIL="1", NTT_LIB_PATH=dbg)
    r = subprocess.run([sys.executable, "-c", _CHILD_FAIL.format(root=ROOT, path=path)], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "child ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    pl = NTTPlan(1, 20, 4)
    assert pl.passes == [10, 10]
    t = pl.fill(pl.empty(), "random", seed=51)
    pl.forward(t)
    assert np.array_equal(t.cpu().numpy(), np.load(path))


_CHILD_NO_HOOK = r"""
import sys
sys.path.insert(0, {root!r})
from ntt_amd.ntt import NTTPlan
assert NTTPlan(1, 20, 4).passes == [10, 10]
print("child ok")
"""


def test_product_build_has_no_failure_hook():
    """NTT_TEST_WIDE_FAIL is read by the checked build only; the product library
    builds its second plan regardless."""
    env = dict(os.environ, NTT_TEST_WIDE_FAIL="1")
    env.pop("NTT_LIB_PATH", None)
    r = subprocess.run([sys.executable, "-c", _CHILD_NO_HOOK.format(root=ROOT)], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0 and "child ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_launch_labels_name_the_schedule():
    """ntt_plan_last_launch_labels (round 6): the kinds and radices of the latest transform's launches,
    the names bench.py pairs PMC bytes by (tools/pmc_to_traffic.py derives them from kernel names)."""
    from ntt_amd.ntt import NTTPlan
    for fid, log_n, kw, want in [(1, 24, {}, ["c8", "c8s", "f8"]), (1, 20, {}, ["c10", "f10"]),
                                 (1, 20, {"single_launch": True}, ["b"]), (1, 8, {}, ["s8"])]:
        pl = NTTPlan(fid, log_n, 4, **kw)
        t = pl.fill(pl.empty(), "random", seed=9)
        pl.set_profiling(True)
        pl.forward(t)
        assert pl.last_launch_labels() == want, (log_n, kw, pl.last_launch_labels())
        assert len(pl.last_launch_ms()) == len(want)
        pl.set_profiling(False)
    pl = NTTPlan(1, 20, 4)
    b = pl.empty(2)
    pl.fill(b.view(2, pl.n, -1)[0], "random", seed=1)
    pl.set_profiling(True)
    pl.forward_batch(b, 2)  # batched: the 1024-element tiles, 7 + 7 + 6
    assert pl.last_launch_labels() == ["c7", "c7s", "f6"], pl.last_launch_labels()
    pl.set_profiling(False)
