"""bench.py's host logic on the CPU (no GPU calls): the launcher refuses more ranks than visible
devices, the column-layout assembly of the post-timing parity check, and its closed-form KAT."""
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from ntt_amd.distributed import Layout  # noqa: E402


def test_spawn_refuses_more_ranks_than_devices():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "NTT_BENCH_EXCHANGE")}
    env["HIP_VISIBLE_DEVICES"] = ""  # no device visible, even on a GPU box
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.stdout, r.stderr)
    assert "refusing" in r.stderr


def test_assemble_columns_restores_natural_order():
    for log_n, world, log_n2, tail in [(12, 2, 6, ()), (12, 4, 5, (4,)), (14, 8, 7, (6,))]:
        n = 1 << log_n
        X = torch.arange(n * (int(np.prod(tail)) if tail else 1), dtype=torch.int64).reshape((n,) + tail)
        parts = []
        for g in range(world):
            L = Layout(log_n, world, g, log_n2)
            idx = torch.tensor([L.col_global(i) for i in range(L.local_n)])
            parts.append(X[idx])
        L = Layout(log_n, world, 0, log_n2)
        assert torch.equal(bench.assemble_columns(parts, L.n1, L.c), X)


def test_kat_check_matches_the_definition():
    from ntt_amd.fields import field_params
    for fid, log_n in [(0, 6), (1, 5), (2, 4)]:
        p, g = field_params(fid)
        n = 1 << log_n
        w = pow(g, (p - 1) // n, p)
        X = [sum(j * pow(w, j * k, p) for j in range(n)) % p for k in range(n)]
        ks = list(range(n))
        assert bench._kat_check(fid, log_n, 4, X, ks)
        bad = list(X)
        bad[3] = (bad[3] + 1) % p
        assert not bench._kat_check(fid, log_n, 4, bad, ks)
        assert bench._to_ints(torch.tensor([[5, 0, 0, 0], [-1, 1, 0, 0]])) == [5, (1 << 64) - 1 + (1 << 64)]


def test_launcher_parent_never_loads_torch():
    """spawn_ranks (``python bench.py --gpus N`` without a launcher) counts devices in a child process:
    the parent that later starts the ranks never imports torch, so it cannot have touched the HIP
    runtime (here no device is visible, so it refuses after counting)."""
    code = ("import os, sys, types; sys.path.insert(0, %r); os.environ['HIP_VISIBLE_DEVICES'] = ''\n"
            "os.environ.pop('NTT_BENCH_EXCHANGE', None)\n"
            "import bench\n"
            "rc = bench.spawn_ranks(types.SimpleNamespace(gpus=2))\n"
            "assert rc == 2, rc\n"
            "assert 'torch' not in sys.modules, 'the launcher parent imported torch'\n"
            "print('parent clean')\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "parent clean" in r.stdout, (r.stdout, r.stderr)


def test_cpu_baseline_fields():
    """The cpu_baseline object (§8d: the C oracle on the host's CPU share, the CPU model recorded) on a
    small size: value, unit, cores, kind, sample, cpu_model, and the 1-core samples."""
    import bench
    cb = bench.cpu_baseline(1, 4, 10)
    assert cb["value"] > 0 and cb["unit"] == "field-elements/s" and cb["kind"] == "port"
    assert cb["cores"] >= 1 and isinstance(cb["cpu_model"], str) and cb["cpu_model"]
    assert cb["single_core"]["cores"] == 1 and cb["reference_field_single_core"]["cores"] == 1
    # C1 and 2^20 in full, 2^24 once, 2^28 extrapolated and labelled
    c = cb["configs"]
    assert set(c) == {"C1_2^12_python", "C1_2^12_c", "2^20", "2^24", "2^28_extrapolated"}
    assert all(v["value"] > 0 and v["seconds"] > 0 and v["cores"] >= 1 for v in c.values())
    assert c["2^28_extrapolated"]["extrapolated"] is True and "EXTRAPOLATED" in c["2^28_extrapolated"]["sample"]
    assert not any(v.get("extrapolated") for k, v in c.items() if k != "2^28_extrapolated")
    assert c["2^20"]["single_core"]["cores"] == 1


def test_traffic_pairs_by_launch_label():
    """PMC bytes attach to this run's launches only when the summary's launches
    are the same kernels in the same order (labels from tools/pmc_to_traffic.py vs the plan's
    ntt_plan_last_launch_labels), one timing per launch; else no traffic."""
    ent = {"launch_bytes": [0.806e9, 0.806e9, 1.25e9, 1.147e9], "launch_labels": ["r8", "r8", "c8", "c8s"]}
    ok, why = bench.pair_traffic(ent, ["r8", "r8", "c8", "c8s"], [0.30, 0.30, 0.55, 0.47])
    assert ok == ent["launch_bytes"] and why is None
    # round 5's world-1 four-step: one row launch missing from the timings -> refused, not shifted
    bad, why = bench.pair_traffic(ent, ["r8", "c8", "c8s"], [0.316, 0.583, 0.490])
    assert bad is None and "not this run's launches" in why
    bad, why = bench.pair_traffic(ent, ["r8", "r8", "c8", "c8s"], [0.30, 0.55, 0.47])
    assert bad is None
    bad, why = bench.pair_traffic({"launch_bytes": [1.0, 2.0]}, ["c8", "f8"], [0.5, 0.4])
    assert bad is None and "without per-launch labels" in why
    bad, why = bench.pair_traffic(None, ["c8"], [0.5])
    assert bad is None


def test_pmc_labels_from_kernel_names():
    """tools/pmc_to_traffic.py names launches as the plan does (include/ntt.h ntt_plan_last_launch_labels)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_to_traffic import launch_label
    E = "ntt::Eng29<9, 8, 0, 0>"
    assert launch_label(f"void ntt::k_pass<{E}, 8, 0, true, true, 0, true, 0, false>(unsigned int const*)") == "c8"
    assert launch_label(f"void ntt::k_pass<{E}, 8, 0, true, true, 0, true, 0, true>(unsigned int const*)") == "c8s"
    assert launch_label(f"void ntt::k_pass<{E}, 8, 1, false, true, 0, true, 0, false>(x)") == "f8"
    assert launch_label("void ntt::k_pass<ntt::Eng32<1, 2, 0>, 6, 5, false, true, 0, true, 2, false>(x)") == "r6"
    assert launch_label(f"void ntt::k_final_ipn<{E}, 8>(unsigned int*)") == "i8"
    assert launch_label("void ntt::k_fused2b<ntt::Eng29<9, 8, 0, 12>, 10, 10>(x)") == "b"
    assert launch_label("void ntt::k_build_tw<ntt::Eng29<9, 8, 0, 0> >(x)") == ""


def test_device_probe_failure_is_reported(monkeypatch):
    """a failing device-count child is a reported failure, not '0 devices'."""
    import pytest
    monkeypatch.setattr(sys, "executable", "/bin/false")
    with pytest.raises(SystemExit) as ei:
        bench.visible_devices()
    assert "probe failed" in str(ei.value)
