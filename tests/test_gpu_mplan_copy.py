"""The single-process multi-GPU plan (ntt_mplan, ntt_amd/csrc/ntt_multi.cpp) end to end over G ranks
on ONE GPU: the RCCL stand-in in copy mode (tests/c/rccl_stub.c, NTT_STUB_MODE=copy) accepts the
one device G times and performs every grouped ncclSend / ncclRecv / ncclAllToAll as device copies,
after checking that sends and receives pair up with equal counts and that every run lies inside
its buffer's allocation.

This is the test that was missing for ADVICE r03 (high): the pipelined exchange used G x the peer
block stride, so every send / receive to a peer h >= 1 ran past the end of the exchange buffers --
invisible at G = 1 and with a stand-in that moved no data.  Here the C++ schedule's exchange units
must move the right bytes: the gathered column layout equals the single-GPU transform, the inverse
returns the row layout, and the distributed polymul equals the single-GPU product, bit for bit, for
G = 2, 4, 8 with and without pieces.  Runs in a child process so the stand-in never meets PyTorch's
RCCL."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes, sys
sys.path.insert(0, ROOT)
import torch
from ntt_amd.distributed import MultiPlan
from ntt_amd.ntt import NTTPlan
stub = ctypes.CDLL(STUB)
stub.stub_violations.restype = ctypes.c_longlong
stub.stub_bytes.restype = ctypes.c_longlong

def col_index(lay):
    i = torch.arange(lay.local_n, dtype=torch.int64, device="cuda:0")
    return lay.rank * lay.c + (i & (lay.c - 1)) + lay.n2 * (i >> lay.log_c)

def row_index(lay):
    i = torch.arange(lay.local_n, dtype=torch.int64, device="cuda:0")
    return lay.rank * lay.r + (i >> lay.log_n2) + lay.n1 * (i & (lay.n2 - 1))

for (G, fid, L, log_n, P, Q) in CASES:
    ref = NTTPlan(fid, log_n, L)
    x = ref.fill(ref.empty(), "random", seed=7)
    X = x.clone()
    ref.forward(X)
    a = ref.fill(ref.empty(), "random", seed=8)
    b = ref.fill(ref.empty(), "random", seed=9)
    c = ref.empty()
    ref.polymul(a.clone(), b.clone(), c)
    mp = MultiPlan(fid, log_n, L, devices=[0] * G, pieces=P, col_pieces=Q)
    xs = mp.fill(mp.empty(), "random", seed=7)
    for lay, t in zip(mp.layouts, xs):
        assert torch.equal(t, x[row_index(lay)]), ("row layout", G, log_n)
    shares = [t.clone() for t in xs]
    before = stub.stub_bytes()
    mp.forward(xs)
    torch.cuda.synchronize()
    moved = stub.stub_bytes() - before
    for lay, t in zip(mp.layouts, xs):
        assert torch.equal(t, X[col_index(lay)]), ("forward", G, log_n, P, Q, lay.rank)
    # every element crosses the exchange once: G ranks x G peers x r c elements
    assert moved == x.numel() * 8, (moved, x.numel() * 8)
    mp.inverse(xs)
    torch.cuda.synchronize()
    for s, t in zip(shares, xs):
        assert torch.equal(s, t), ("inverse", G, log_n, P, Q)
    As = mp.fill(mp.empty(), "random", seed=8)
    Bs = mp.fill(mp.empty(), "random", seed=9)
    Cs = mp.empty()
    mp.polymul(As, Bs, Cs)
    torch.cuda.synchronize()
    for lay, t in zip(mp.layouts, Cs):
        assert torch.equal(t, c[row_index(lay)]), ("polymul", G, log_n, P, Q, lay.rank)
    del mp
    print("OK", G, fid, L, log_n, P, Q, flush=True)
print("VIOLATIONS", stub.stub_violations(), flush=True)
'''

CASES = [(2, 1, 4, 16, 1, 1), (2, 1, 4, 16, 2, 4), (4, 1, 4, 16, 1, 1), (4, 1, 4, 16, 4, 2),
         (8, 1, 4, 18, 1, 1), (8, 1, 4, 18, 2, 2), (8, 1, 4, 20, 4, 4), (4, 2, 6, 16, 2, 2),
         (2, 0, 1, 16, 2, 2), (8, 0, 1, 18, 4, 4)]


def _build_stub(stub, src):
    if not os.path.exists(stub) or os.path.getmtime(stub) < os.path.getmtime(src):
        subprocess.run(["gcc", "-shared", "-fPIC", "-O2", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-o",
                        stub, src, "-L/opt/rocm/lib", "-lamdhip64"], check=True)


def test_mplan_over_copy_stub_matches_single_gpu():
    stub = os.path.join(ROOT, "tests", "c", "librccl_stub.so")
    src = os.path.join(ROOT, "tests", "c", "rccl_stub.c")
    _build_stub(stub, src)
    env = dict(os.environ, NTT_RCCL_LIBRARY=stub, NTT_STUB_MODE="copy")
    code = f"ROOT = {ROOT!r}\nSTUB = {stub!r}\nCASES = {CASES!r}\n" + CHILD
    r = subprocess.run([sys.executable, "-u", "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert r.stdout.count("OK ") == len(CASES), r.stdout
    assert "VIOLATIONS 0" in r.stdout, r.stdout
