"""Plan memory: the reference-shaped shims keep at most NTT_SHIM_CACHE_PLANS cached
plans (least recently used dropped; ntt_shim_cache_clear releases them all), and a plan builds its
inverse outer-twiddle tables only at the first inverse call (a forward-only plan holds one
direction).  Run in a child process so the cache cap is read fresh."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys
sys.path.insert(0, ROOT)
import ctypes
import numpy as np, torch
from ntt_amd import lib as L
from ntt_amd.ntt import SSIP, NTTPlan
from oracle import oracle_c as OC
lib = L.load()
P = 469762049

def free():
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info()[0]

# three SSIP sizes through a 2-plan cache, round robin: every call must still be exact
xs = {lg: np.arange(1 << lg, dtype=np.int64) for lg in (16, 18, 20)}
refs = {lg: OC.ntt_u64(x, P, 3) for lg, x in xs.items()}
for _ in range(3):
    for lg, x in xs.items():
        t = torch.from_numpy(x).cuda()
        SSIP(t, 3, lg)
        assert np.array_equal(t.cpu().numpy(), refs[lg]), lg
f0 = free()
lib.ntt_shim_cache_clear()
f1 = free()
assert f1 >= f0, (f0, f1)
print("CACHE-OK", f1 - f0)

# lazy inverse tables: 2^22 BN254, the pass-1 table alone is 2^22 x 32 B = 128 MiB
pl = NTTPlan(1, 22, 4)
t = pl.fill(pl.empty(), "random", seed=3)
x = t.clone()
pl.forward(t)
a = free()
pl.inverse(t)
b = free()
assert torch.equal(t, x)
grown = a - b
assert grown >= (1 << 22) * 32, grown
print("LAZY-OK", grown)
'''


def test_shim_cache_cap_clear_and_lazy_inverse_tables():
    env = dict(os.environ, NTT_SHIM_CACHE_PLANS="2")
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + CHILD], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "CACHE-OK" in r.stdout and "LAZY-OK" in r.stdout
