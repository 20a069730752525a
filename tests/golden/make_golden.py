"""Generate the committed golden fixtures under tests/golden/ (run in the build container only).

Sources:
* ``datapath_demo_lgp4.txt`` — stdout of the reference's own ``src/datapath_demo.py`` (run with
  MPLBACKEND=Agg; the scatter plot is discarded).  This pins ``ntt_amd.plumbing.datapath_map``.
* ``twiddlecheck.json``     — inputs fed on stdin to the reference's own ``src/twiddlecheck.py`` and
  the exponents it printed.  This pins ``ntt_amd.plumbing.twiddle_exponents`` and the reference's
  hard-coded omega_256 = 338628632 (twiddlecheck.py:11).
* ``ntt_vectors.json``      — forward NTT vectors from the Python oracle (oracle/ntt_ref.py), which is
  itself pinned by the closed-form KAT and by the reference-run values in SURVEY.md §0.3; full
  vectors for small n, sampled (k, X_k) for larger n.

The reference tree is never read at test time; only these data files travel.
Usage: python tests/golden/make_golden.py [/root/reference]
"""
from __future__ import annotations

import json
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import ntt_ref as R  # noqa: E402


def run_reference_python(ref: str) -> None:
    env = dict(os.environ, MPLBACKEND="Agg")
    out = subprocess.run([sys.executable, os.path.join(ref, "src", "datapath_demo.py")], env=env,
                         capture_output=True, text=True, check=True, timeout=600).stdout
    with open(os.path.join(HERE, "datapath_demo_lgp4.txt"), "w") as f:
        f.write(out)

    # twiddlecheck: origin random nonzero, target = origin * w256^e mod P with known e.
    rng = random.Random(2024)
    P = R.P469762049
    w = 338628632
    origin = [rng.randrange(1, P) for _ in range(256)]
    exps = [rng.randrange(0, 256) for _ in range(256)]
    target = [o * pow(w, e, P) % P for o, e in zip(origin, exps)]
    stdin = " ".join(map(str, target)) + "\n" + " ".join(map(str, origin)) + "\n"
    out = subprocess.run([sys.executable, os.path.join(ref, "src", "twiddlecheck.py")], input=stdin,
                         capture_output=True, text=True, check=True, timeout=600).stdout
    printed = [int(t) for t in out.split()]
    with open(os.path.join(HERE, "twiddlecheck.json"), "w") as f:
        json.dump({"omega": w, "origin": origin, "target": target, "reference_output": printed}, f)


def ntt_vectors() -> None:
    out = {"fields": {}, "vectors": []}
    for fid, (p, g) in R.FIELDS.items():
        out["fields"][str(fid)] = {"p": hex(p), "g": g, "name": R.FIELD_NAMES[fid]}
    for fid, (p, g) in R.FIELDS.items():
        for log_n in range(0, 11 if fid == 0 else 9):
            n = 1 << log_n
            for kind in ("iota", "random"):
                x = R.iota_vector(n) if kind == "iota" else R.random_vector(fid, n, seed=1)
                X = R.ntt_dit(x, p, g)
                out["vectors"].append({"field": fid, "log_n": log_n, "input": kind, "seed": 1,
                                       "x": [hex(v) for v in x], "X": [hex(v) for v in X]})
        # sampled KAT outputs at larger sizes (iota input)
        for log_n in (12, 16, 20, 24) + ((26,) if fid == 0 else (28,)):
            if log_n > R.two_adicity(p):
                continue
            n = 1 << log_n
            ks = sorted({0, 1, 2, 3, n // 2, n - 1} | {random.Random(log_n).randrange(n) for _ in range(8)})
            out["vectors"].append({"field": fid, "log_n": log_n, "input": "iota",
                                   "sampled": {str(k): hex(R.kat_xj(n, p, g, k)) for k in ks}})
    with open(os.path.join(HERE, "ntt_vectors.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    if os.path.isdir(ref):
        run_reference_python(ref)
    else:
        print("reference tree absent: keeping the committed reference-derived fixtures")
    ntt_vectors()
