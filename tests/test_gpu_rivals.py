"""The rival schedules, same contract as the default schedule and so the same pins --
the reference's own outputs (tests/golden/ref_p469762049.npz) on its field P, the C oracle for
BN254 / BLS12-381 Fr, and bit-for-bit agreement with the default four-step DIF schedule:
* "stockham": the bellperson / improved_NTT_v1..v4 family (GZKP-NTT.cu:324-386 FIELD_radix_fft,
  :556-1296) as Stockham autosort pass kernels (KIND_STOCKHAM, plan flag NTT_PLAN_STOCKHAM);
* "gzkp": GZKP(B, G) (GZKP-NTT.cu:115-233; parallel-load.cu for P): bit reversal, then in-place DIT
  passes with input twiddles (KIND_DIT, plan flag NTT_PLAN_GZKP)."""
import os

import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_p469762049.npz"))
THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8"))))


RIVALS = ["stockham", "gzkp"]


def _plan(fid, log_n, L, sched):
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=fid, log_n=log_n, limbs64=L, stockham=sched == "stockham", gzkp=sched == "gzkp")


@pytest.mark.parametrize("sched", RIVALS)
@pytest.mark.parametrize("log_n", [16, 20, 22, 24, 26])
def test_rival_p_path_vs_reference_outputs(log_n, sched):
    n = 1 << log_n
    idx = torch.from_numpy(GOLD[f"samp_idx_{log_n}"]).to("cuda:0")
    pl = _plan(0, log_n, 1, sched)
    t = torch.arange(n, dtype=torch.int64, device="cuda:0")
    pl.forward(t)
    assert np.array_equal(t[idx].cpu().numpy(), GOLD[f"samp_iota_{log_n}"])
    t = torch.from_numpy(OC.random_limbs(0, n, seed=2000 + log_n, L=1)[:, 0].astype(np.int64)).to("cuda:0")
    pl.forward(t)
    assert np.array_equal(t[idx].cpu().numpy(), GOLD[f"samp_rand_{log_n}"])
    pl.inverse(t)  # the inverse runs the default schedule
    assert np.array_equal(t.cpu().numpy(), OC.random_limbs(0, n, seed=2000 + log_n, L=1)[:, 0].astype(np.int64))


@pytest.mark.parametrize("sched", RIVALS)
@pytest.mark.parametrize("fid,L,log_n", [(0, 1, 14), (0, 1, 18), (1, 4, 11), (1, 4, 13), (1, 4, 16), (2, 4, 17),
                                         (1, 4, 20)])
def test_rival_matches_oracle_and_default_schedule(fid, L, log_n, sched):
    p, g = R.FIELDS[fid]
    st = _plan(fid, log_n, L, sched)
    df = _plan(fid, log_n, L, "default")
    a = st.fill(st.empty(), "random", seed=log_n)
    b = a.clone()
    x = a.cpu().numpy().view(np.uint64).reshape(-1, L).copy()
    st.forward(a)
    df.forward(b)
    assert torch.equal(a, b), (fid, L, log_n, st.passes)
    got = a.cpu().numpy().view(np.uint64).reshape(-1, L)
    if L == 1:
        assert np.array_equal(got[:, 0].astype(np.int64), OC.ntt_u64(x[:, 0].astype(np.int64), p, g))
    else:
        assert np.array_equal(got, OC.ntt_mp(x, p, g))


@pytest.mark.parametrize("sched", RIVALS)
def test_rival_2pow24_bn254_elementwise(sched):
    p, g = R.FIELDS[1]
    st = _plan(1, 24, 4, sched)
    a = st.fill(st.empty(), "random", seed=24)
    x = a.cpu().numpy().view(np.uint64).reshape(-1, 4).copy()
    st.forward(a)
    assert np.array_equal(a.cpu().numpy().view(np.uint64).reshape(-1, 4), OC.ntt_mp_par(x, p, g, THREADS))


def test_rival_flags_are_exclusive():
    from ntt_amd.ntt import NTTPlan
    with pytest.raises(Exception):
        NTTPlan(field_id=1, log_n=12, limbs64=4, stockham=True, gzkp=True)
