"""Pin the oracle against the REFERENCE'S OWN CPU transforms (not a restatement of them).

``tests/golden/ref_p469762049.npz`` holds outputs of the reference's ``NTT`` (src/GZKP-NTT.cu:30-48),
its inverse recipe (GZKP-NTT.cu:1725-1732), ``NTT_pro1``+``NTT_pro2`` and ``NTT_dif``
(src/self-sort-in-place.cu:53-128), compiled from /root/reference by ``make -C oracle ref`` and run by
``tests/golden/make_ref_vectors.py``.  The field is the reference's P = 469762049, the only one its
runnable code has.  The multi-precision oracle (the checker of the BN254 / BLS12-381 GPU tests) is
modulus-generic, so running it on the zero-padded P pins its code path against the same outputs.

When oracle/_ref is built (this container, or a box that received the built .so files), the live
reference is also compared against the oracle on fresh seeds.
"""
import os

import numpy as np
import pytest

from oracle import ntt_ref as R
from oracle import oracle_c as OC
from oracle import ref_c

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_p469762049.npz"))
P = R.P469762049


def _rand(log_n, seed):
    return OC.random_limbs(0, 1 << log_n, seed=seed, L=1)[:, 0].astype(np.int64)


def _padded(x, L):
    out = np.zeros((x.size, L), dtype=np.uint64)
    out[:, 0] = x.astype(np.uint64)
    return out


@pytest.mark.parametrize("log_n", range(0, 13))
def test_c_oracle_matches_reference_fixtures(log_n):
    n = 1 << log_n
    x = _rand(log_n, 1000 + log_n)
    assert np.array_equal(OC.ntt_u64(np.arange(n), P, 3), GOLD[f"fwd_iota_{log_n}"])
    assert np.array_equal(OC.ntt_u64(x, P, 3), GOLD[f"fwd_rand_{log_n}"])
    assert np.array_equal(OC.ntt_u64(x, P, 3, inverse=True), GOLD[f"inv_rand_{log_n}"])


@pytest.mark.parametrize("L", [1, 4, 6])
def test_multiprecision_oracle_matches_reference_fixtures(L):
    """The BN254/BLS checker's code path (oracle_ntt_mp, 1/4/6 x 64-bit limbs) on the reference's P."""
    for log_n in range(0, 13):
        x = _rand(log_n, 1000 + log_n)
        got = OC.ntt_mp(_padded(x, L), P, 3)
        assert np.array_equal(got[:, 0].astype(np.int64), GOLD[f"fwd_rand_{log_n}"]) and not got[:, 1:].any()
        got = OC.ntt_mp(_padded(x, L), P, 3, inverse=True)
        assert np.array_equal(got[:, 0].astype(np.int64), GOLD[f"inv_rand_{log_n}"])


def test_python_oracle_matches_reference_fixtures():
    for log_n in range(0, 11):
        x = [int(v) for v in _rand(log_n, 1000 + log_n)]
        assert R.ntt_dit(x, P, 3) == GOLD[f"fwd_rand_{log_n}"].tolist()
        assert R.ssip_pro(x, P, 3) == GOLD[f"ssip_rand_{log_n}"].tolist()
        assert R.intt(GOLD[f"fwd_rand_{log_n}"].tolist(), P, 3) == x
    # the reference's SSIP CPU spec and DIF agree with its DIT NTT (natural order in and out)
    for log_n in range(0, 11):
        assert np.array_equal(GOLD[f"ssip_rand_{log_n}"], GOLD[f"fwd_rand_{log_n}"])
        assert np.array_equal(GOLD[f"dif_rand_{log_n}"], GOLD[f"fwd_rand_{log_n}"])


@pytest.mark.parametrize("log_n", [16, 20, 22, 24, 26])
def test_sampled_reference_outputs(log_n):
    idx = GOLD[f"samp_idx_{log_n}"]
    n = 1 << log_n
    # x_j = j: the closed form (any size), which the GPU tests use at full sizes
    assert [R.kat_xj(n, P, 3, int(k)) for k in idx] == GOLD[f"samp_iota_{log_n}"].tolist()
    if log_n <= 22:
        got = OC.ntt_u64(_rand(log_n, 2000 + log_n), P, 3)
        assert np.array_equal(got[idx], GOLD[f"samp_rand_{log_n}"])


def test_reference_2pow26_head_matches_survey_run():
    assert GOLD["samp_iota_26"][:4].tolist() == [95869806, 352459684, 445876816, 262883937]


@pytest.mark.skipif(not ref_c.available() and not os.path.isdir(ref_c.REF_SRC), reason="oracle/_ref not built")
def test_live_reference_against_oracle():
    assert ref_c.build()
    for log_n in list(range(0, 15)) + [18]:
        for seed in (5, 6):
            x = _rand(log_n, seed)
            exp = ref_c.ntt(x)
            assert np.array_equal(OC.ntt_u64(x, P, 3), exp), (log_n, seed)
            assert np.array_equal(ref_c.ssip_pro(x), exp)
            assert np.array_equal(OC.ntt_u64(x, P, 3, inverse=True), ref_c.ntt(x, inverse=True))
            if log_n <= 12:
                got = OC.ntt_mp(_padded(x, 4), P, 3)
                assert np.array_equal(got[:, 0].astype(np.int64), exp)
