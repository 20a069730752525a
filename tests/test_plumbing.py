"""Config C1 (CPU plumbing): the restated datapath_demo / twiddlecheck helpers reproduce the outputs
captured from the reference's own Python scripts, and the 2^12 BN254 CPU transform matches the
oracle."""
import json
import os

from ntt_amd import plumbing
from oracle import ntt_ref as R

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_datapath_map_matches_reference_stdout():
    ref = open(os.path.join(GOLD, "datapath_demo_lgp4.txt")).read()
    rows = plumbing.datapath_map(4)
    assert len(rows) == 256 and all(len(r) == 16 for r in rows)
    assert plumbing.format_datapath_map(rows) == ref


def test_datapath_map_is_a_permutation():
    # every one of the 4096 outputs of the radix-16 pass is written exactly once
    for lgp in (0, 4, 8):
        flat = [v for row in plumbing.datapath_map(lgp) for v in row]
        assert sorted(flat) == list(range(4096))


def test_twiddlecheck_matches_reference_output():
    d = json.load(open(os.path.join(GOLD, "twiddlecheck.json")))
    assert plumbing.twiddle_exponents(d["target"], d["origin"], d["omega"]) == d["reference_output"]


def test_c1_cpu_ntt_2pow12_bn254():
    X = plumbing.cpu_ntt_c1(12)
    p, g = R.FIELDS[1]
    assert X == R.ntt_dit(list(range(1 << 12)), p, g)
