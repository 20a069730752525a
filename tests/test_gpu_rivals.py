"""The rival schedules, same contract as the default schedule and so the same pins --
the reference's own outputs (tests/golden/ref_p469762049.npz) on its field P, the C oracle for
BN254 / BLS12-381 Fr, and bit-for-bit agreement with the default four-step DIF schedule:
* "stockham": the bellperson / improved_NTT_v1..v4 family (GZKP-NTT.cu:324-386 FIELD_radix_fft,
  :556-1296) as Stockham autosort pass kernels (KIND_STOCKHAM, plan flag NTT_PLAN_STOCKHAM);
* "gzkp": GZKP(B, G) (GZKP-NTT.cu:115-233; parallel-load.cu for P): bit reversal, then in-place DIT
  passes with input twiddles (KIND_DIT, plan flag NTT_PLAN_GZKP);
* "naive": the reference's `naive` (GZKP-NTT.cu:59-95, big-num.cu:67-170): bit reversal, then one
  radix-2 DIT round per launch (k_naive_round, plan flag NTT_PLAN_NAIVE);
* "no_swap": the reference's `naive_no_swap` (GZKP-NTT.cu:237-296, checked against the CPU NTT in its
  main, :1653-1660): a radix-2 Stockham autosort, one round per launch, natural order in and out
  (k_noswap_round, plan flag NTT_PLAN_NO_SWAP);
* "bellperson", "v1".."v4": the same family as the reference ships it, kernel for kernel -- rounds of
  2^deg-point groups in LDS, one launch per round (k_bealto; FIELD_radix_fft_revised / bellperson_baseline,
  GZKP-NTT.cu:391-553, and improve_grouped, improve_group_coalesced_read, ..._and_write and
  improve_reduce_bank_conflict with improved_NTT_v1..v4, :556-1296; plan flags NTT_PLAN_BELLPERSON,
  NTT_PLAN_IMPROVED_V1..V4)."""
import os

import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_p469762049.npz"))
THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8"))))


BEALTO = ["bellperson", "v1", "v2", "v3", "v4"]
RIVALS = ["stockham", "gzkp", "naive", "no_swap"] + BEALTO


def _plan(fid, log_n, L, sched):
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=fid, log_n=log_n, limbs64=L, stockham=sched == "stockham", gzkp=sched == "gzkp",
                   naive=sched == "naive", no_swap=sched == "no_swap", bealto=sched if sched in BEALTO else "")


def _bealto_rounds(sched, log_n):
    """the reference's round degrees: max_deg = min(8 - log_g, log_n), log_g 0 (bellperson) or 5"""
    md = min(8 if sched == "bellperson" else 3, log_n)
    out, lgp = [], 0
    while lgp < log_n:
        out.append(min(md, log_n - lgp))
        lgp += out[-1]
    return out


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


@pytest.mark.parametrize("sched", RIVALS[:4] + ["bellperson"])
def test_rival_2pow24_bn254_elementwise(sched):
    p, g = R.FIELDS[1]
    st = _plan(1, 24, 4, sched)
    a = st.fill(st.empty(), "random", seed=24)
    x = a.cpu().numpy().view(np.uint64).reshape(-1, 4).copy()
    st.forward(a)
    assert np.array_equal(a.cpu().numpy().view(np.uint64).reshape(-1, 4), OC.ntt_mp_par(x, p, g, THREADS))


def test_rival_flags_are_exclusive():
    from ntt_amd.ntt import NTTPlan
    for kw in ({"stockham": True, "gzkp": True}, {"stockham": True, "naive": True}, {"gzkp": True, "naive": True},
               {"naive": True, "in_place": True}, {"no_swap": True, "naive": True}, {"no_swap": True, "in_place": True}):
        with pytest.raises(Exception):
            NTTPlan(field_id=1, log_n=12, limbs64=4, **kw)
    for kw in ({"bealto": "v1", "naive": True}, {"bealto": "bellperson", "stockham": True},
               {"bealto": "v4", "in_place": True}):
        with pytest.raises(Exception):
            NTTPlan(field_id=1, log_n=12, limbs64=4, **kw)
    with pytest.raises(ValueError):
        NTTPlan(field_id=1, log_n=12, limbs64=4, bealto="v5")
    for kw in ({"naive": True}, {"no_swap": True}, {"bealto": "v2"}):
        with pytest.raises(Exception):  # the rivals cover P and the 4 x 64-bit layout
            NTTPlan(field_id=2, log_n=12, limbs64=6, **kw)


@pytest.mark.parametrize("sched", BEALTO[1:])
def test_bealto_2pow24_bn254_matches_default(sched):
    """2^24 BN254 (BASELINE config 2's size) on the improved kernels: 8 rounds of 2^3-point groups,
    equal to the default schedule (pinned to the oracle above) element for element"""
    st = _plan(1, 24, 4, sched)
    df = _plan(1, 24, 4, "default")
    a = st.fill(st.empty(), "random", seed=124)
    b = a.clone()
    st.set_profiling(True)
    st.forward(a)
    assert st.last_launch_labels() == ["v3"] * 8
    st.set_profiling(False)
    df.forward(b)
    assert torch.equal(a, b)


@pytest.mark.parametrize("sched", ["naive", "no_swap"] + BEALTO)
@pytest.mark.parametrize("fid,L,log_n", [(0, 1, 1), (0, 1, 2), (0, 1, 5), (1, 4, 1), (1, 4, 3), (2, 4, 9),
                                         (0, 1, 11), (1, 4, 7)])
def test_naive_small_sizes_vs_oracle(fid, L, log_n, sched):
    """The radix-2 rivals have no tile constraints: every size from 2 points (odd and even round
    counts: no_swap's odd ones end in the plan buffer and are copied back), forward against the
    oracle, the plan's (default-schedule) inverse back to the input; the launch groups recorded."""
    p, g = R.FIELDS[fid]
    pl = _plan(fid, log_n, L, sched)
    a = pl.fill(pl.empty(), "random", seed=7 + log_n)
    x = a.cpu().numpy().view(np.uint64).reshape(-1, L).copy()
    pl.set_profiling(True)
    pl.forward(a)
    # naive: [bit reversal, the log2 n rounds]; no_swap: [the log2 n rounds]; the bealto family: one
    # interval per round (labels g<deg> / v<deg>) and the copy back after an odd round count
    if sched in BEALTO:
        rounds = _bealto_rounds(sched, log_n)
        want = [("g" if sched == "bellperson" else "v") + str(d) for d in rounds] + (["cp"] if len(rounds) & 1 else [])
        assert pl.last_launch_labels() == want
        assert len(pl.last_launch_ms()) == len(want)
    else:
        assert len(pl.last_launch_ms()) == (2 if sched == "naive" else 1)
    pl.set_profiling(False)
    got = a.cpu().numpy().view(np.uint64).reshape(-1, L)
    if L == 1:
        assert np.array_equal(got[:, 0].astype(np.int64), OC.ntt_u64(x[:, 0].astype(np.int64), p, g))
    else:
        assert np.array_equal(got, OC.ntt_mp(x, p, g))
    pl.inverse(a)
    assert np.array_equal(a.cpu().numpy().view(np.uint64).reshape(-1, L), x)
