"""The compiled C drop-in caller (tests/c/dropin.c: include/ntt.h + libntt.so, no Python on the
call path) at the reference mains' own call sites, sizes and inputs, checked against the
reference's outputs (tests/golden/ref_p469762049.npz) and the closed-form KAT of x_j = j.

Call sites mirrored: GZKP-NTT.cu:1710 SSIP(data_d, root, 26); big-num.cu:458 NTT_GZKP<8,256> for
n = 2^5..2^12; parallel-load.cu:319 NTT_GZKP(data_d, reverse2_d, 2^26, root, 7, 8, reverse_num).
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import ntt_ref as R

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_p469762049.npz"))


@pytest.fixture(scope="module")
def dropin_output():
    from tests.dropin_build import build
    exe = build()
    r = subprocess.run([exe, "all"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = {}
    for line in r.stdout.splitlines():
        parts = line.split()
        out.setdefault(parts[0], []).append(parts[1:])
    assert "DONE" in out
    return out


def test_ssip_call_site(dropin_output):
    gold = dict(zip(GOLD["samp_idx_26"].tolist(), GOLD["samp_iota_26"].tolist()))
    n = 1 << 26
    for log_n, k, v in dropin_output["SSIP"]:
        k, v = int(k), int(v)
        assert v == R.kat_xj(n, R.P469762049, 3, k)
        if k in gold:
            assert v == gold[k]


def test_in_place_ssip_call_site(dropin_output):
    """NTT_PLAN_IN_PLACE at the SSIP call site: the same outputs as SSIP (the reference's 2^26 values),
    round trip through the in-place inverse."""
    gold = dict(zip(GOLD["samp_idx_26"].tolist(), GOLD["samp_iota_26"].tolist()))
    n = 1 << 26
    assert len(dropin_output["INPLACE_SSIP"]) == 6
    for log_n, k, v in dropin_output["INPLACE_SSIP"]:
        k, v = int(k), int(v)
        assert v == R.kat_xj(n, R.P469762049, 3, k)
        if k in gold:
            assert v == gold[k]
    assert dropin_output["INPLACE_ROUNDTRIP"] == [["26", "ok"]]


def test_gzkp256_call_site(dropin_output):
    got = {}
    for log_n, k, v in dropin_output["GZKP256"]:
        got.setdefault(int(log_n), {})[int(k)] = int(v)
    assert sorted(got) == list(range(5, 13))
    for log_n, vals in got.items():
        assert [vals[k] for k in range(1 << log_n)] == GOLD[f"fwd_iota_{log_n}"].tolist(), log_n


def test_gzkp64_call_site(dropin_output):
    n = 1 << 26
    for log_n, k, v in dropin_output["GZKP64"]:
        assert int(v) == R.kat_xj(n, R.P469762049, 3, int(k))


def test_plan_api_bn254(dropin_output):
    p, g = R.FIELDS[1]
    n = 1 << 20
    for log_n, k, hexv in dropin_output["PLAN_BN254"]:
        assert int(hexv, 16) == R.kat_xj(n, p, g, int(k))
    assert dropin_output["PLAN_BN254_ROUNDTRIP"] == [["20", "ok"]]
    assert dropin_output["ERRORS"] == [["ok"]]
