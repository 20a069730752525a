"""Fault path of the single-process multi-GPU plan: with an RCCL whose
data-path calls fail (tests/c/rccl_stub.c, loaded through NTT_RCCL_LIBRARY), ntt_forward_multi /
ntt_inverse_multi / ntt_polymul_multi return NTT_ERR_RCCL after draining every device's stream
(ntt_multi.cpp: exchange() always closes the RCCL group; drain() waits on the streams), and the
process and device stay usable: the plan is destroyed and a single-GPU transform still runs and is
correct.  Runs in a child process so the stand-in RCCL never meets PyTorch's."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys
sys.path.insert(0, ROOT)
import numpy as np, torch
from ntt_amd.distributed import MultiPlan
from ntt_amd.lib import NTTError
from ntt_amd.ntt import NTTPlan
from oracle import oracle_c as OC, ntt_ref as R
mp = MultiPlan(1, 14, 4, devices=[0])
xs = mp.fill(mp.empty(), "random", seed=1)
for name, call in (("forward", lambda: mp.forward(xs)), ("inverse", lambda: mp.inverse(xs)),
                   ("polymul", lambda: mp.polymul(xs, [x.clone() for x in xs], [x.clone() for x in xs]))):
    try:
        call()
        print("NO-ERROR", name)
        sys.exit(3)
    except NTTError as e:
        assert e.status == -3, (name, e.status)
        print("RCCL-ERROR", name, flush=True)
del mp
torch.cuda.synchronize()
pl = NTTPlan(1, 12, 4)
t = pl.fill(pl.empty(), "random", seed=2)
x = t.cpu().numpy().view(np.uint64).copy()
pl.forward(t)
p, g = R.FIELDS[1]
assert np.array_equal(t.cpu().numpy().view(np.uint64), OC.ntt_mp(x, p, g))
print("HEALTHY")
'''


def _build_stub(stub, src):
    if not os.path.exists(stub) or os.path.getmtime(stub) < os.path.getmtime(src):
        subprocess.run(["gcc", "-shared", "-fPIC", "-O2", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-o",
                        stub, src, "-L/opt/rocm/lib", "-lamdhip64"], check=True)


def test_rccl_failure_is_reported_and_drained():
    stub = os.path.join(ROOT, "tests", "c", "librccl_stub.so")
    src = os.path.join(ROOT, "tests", "c", "rccl_stub.c")
    _build_stub(stub, src)
    env = dict(os.environ, NTT_RCCL_LIBRARY=stub)
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + CHILD], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert r.stdout.count("RCCL-ERROR") == 3 and "HEALTHY" in r.stdout


# A failure on device g > 0 of a grouped exchange: device 0's part is posted and
# "waits for its peers" (the stand-in blocks its stream until ncclCommAbort), device 1's call fails.
# The plan must abort every communicator before draining, return NTT_ERR_RCCL instead of hanging, and
# refuse later calls.  Two "devices" are the one GPU twice (the stand-in accepts any device list).
CHILD_MID = r"""
import ctypes, sys, time
sys.path.insert(0, ROOT)
import torch
from ntt_amd.distributed import MultiPlan
from ntt_amd.lib import NTTError
mp = MultiPlan(1, 14, 4, devices=[0, 0], pieces=PIECES)
xs = mp.fill(mp.empty(), "random", seed=1)
torch.cuda.synchronize()
t0 = time.time()
try:
    mp.forward(xs)
    print("NO-ERROR"); sys.exit(3)
except NTTError as e:
    assert e.status == -3, e.status
dt = time.time() - t0
stub = ctypes.CDLL(STUB)
print("ABORTS", stub.stub_aborts(), "HUNG", stub.stub_hung(), "SECONDS", round(dt, 2), flush=True)
for call in (lambda: mp.forward(xs), lambda: mp.inverse(xs)):
    try:
        call(); print("NO-ERROR-AFTER"); sys.exit(4)
    except NTTError as e:
        assert e.status == -3, e.status
del mp
torch.cuda.synchronize()
print("DONE")
"""


@pytest.mark.parametrize("pieces", [1, 2])
def test_rccl_failure_on_second_device_aborts_instead_of_hanging(pieces):
    stub = os.path.join(ROOT, "tests", "c", "librccl_stub.so")
    src = os.path.join(ROOT, "tests", "c", "rccl_stub.c")
    _build_stub(stub, src)
    env = dict(os.environ, NTT_RCCL_LIBRARY=stub, NTT_STUB_OK_CALLS="1")
    code = f"ROOT = {ROOT!r}\nSTUB = {stub!r}\nPIECES = {pieces}\n" + CHILD_MID
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("ABORTS")][0].split()
    aborts, hung, secs = int(line[1]), int(line[3]), float(line[5])
    assert aborts == 2 and hung == 0 and secs < 15, line
    assert "DONE" in r.stdout
