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


def test_rccl_failure_is_reported_and_drained():
    stub = os.path.join(ROOT, "tests", "c", "librccl_stub.so")
    src = os.path.join(ROOT, "tests", "c", "rccl_stub.c")
    if not os.path.exists(stub) or os.path.getmtime(stub) < os.path.getmtime(src):
        subprocess.run(["gcc", "-shared", "-fPIC", "-O2", "-o", stub, src], check=True)
    env = dict(os.environ, NTT_RCCL_LIBRARY=stub)
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + CHILD], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert r.stdout.count("RCCL-ERROR") == 3 and "HEALTHY" in r.stdout
