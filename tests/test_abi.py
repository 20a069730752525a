"""The C-ABI library loads and exports every symbol declared in include/*.h (no GPU needed)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")


def declared_functions():
    names = set()
    for f in os.listdir(INCLUDE):
        if not f.endswith(".h"):
            continue
        text = open(os.path.join(INCLUDE, f)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", text, flags=re.M):
            name = m.group(1)
            if name in ("if", "while", "for", "return", "sizeof", "defined"):
                continue
            names.add(name)
    return sorted(names)


def test_headers_declare_the_entry_points():
    names = declared_functions()
    for must in ("ntt_plan_create", "ntt_forward", "ntt_inverse", "ntt_plan_destroy", "SSIP", "NTT_GZKP_256",
                 "ntt_twiddle_pack", "ntt_transpose", "ntt_fill_map"):
        assert must in names, must


def test_library_exports_every_declared_symbol():
    from ntt_amd import lib as L
    assert os.path.exists(L.LIB_PATH), "libntt.so missing: run __graft_entry__.build()"
    so = C.CDLL(L.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(so, n)]
    assert not missing, missing


def test_checked_build_exports_the_same_abi():
    """ntt_amd/libntt_debug.so (NTT_DEBUG_CHECKS) is a drop-in for libntt.so: every declared symbol."""
    from ntt_amd import build as B
    if not os.path.exists(B.DEBUG_LIB):
        pytest.skip("libntt_debug.so not built (python -m ntt_amd.build --debug)")
    so = C.CDLL(B.DEBUG_LIB)
    missing = [n for n in declared_functions() if not hasattr(so, n)]
    assert not missing, missing


def test_python_prototypes_cover_header():
    from ntt_amd import lib as L
    missing = [n for n in declared_functions() if n not in L.PROTOTYPES]
    assert not missing, missing


def test_strerror_without_gpu():
    from ntt_amd import lib as L
    so = L.load()
    assert so.ntt_strerror(0) == b"ok"
    assert so.ntt_strerror(-4).startswith(b"unsupported")


def test_plan_create_reports_no_device_or_bad_args_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    from ntt_amd import lib as L
    so = L.load()
    h = C.c_void_p()
    st = so.ntt_plan_create(C.byref(h), 1, 10, 4, 0)
    assert st in (-5, -2)  # no device
    assert so.ntt_plan_create(C.byref(h), 7, 10, 4, 0) == -1  # bad field id


def test_mplan_create_fails_cleanly_without_gpu_or_bad_args():
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    from ntt_amd import lib as L
    so = L.load()
    h = C.c_void_p()
    devs = (C.c_int * 3)(0, 1, 2)
    assert so.ntt_mplan_create(C.byref(h), 1, 16, 4, 3, devs) == -1  # not a power of two
    assert so.ntt_mplan_create(C.byref(h), 1, 2, 4, 8, devs) == -1   # 2^2 cannot split over 8
    st = so.ntt_mplan_create(C.byref(h), 1, 16, 4, 1, devs)
    assert st in (-5, -2, -1) and not h.value
    assert so.ntt_forward_multi(None, None, None) == -1
    assert so.ntt_mplan_destroy(None) == 0


def test_piece_entry_points_reject_null_plans_without_gpu():
    """The two-sided piece entry points (ntt_rplan_*_piece, ntt_mplan_set_pieces2) check their plan
    before touching a device."""
    from ntt_amd import lib as L
    so = L.load()
    assert so.ntt_rplan_forward_rows_piece(None, None, None, 1, 0, 0, 1, 1, None) == -1
    assert so.ntt_rplan_forward_cols_piece(None, None, None, 1, 0, 0, 1, 1, None) == -1
    assert so.ntt_rplan_inverse_cols_piece(None, None, None, None, 0, 1, 1, None) == -1
    assert so.ntt_rplan_inverse_rows_piece(None, None, None, 0, 1, 1, None) == -1
    assert so.ntt_mplan_set_pieces2(None, 1, 1) == -1


def test_limb_counts_outside_1_4_6_are_rejected_before_any_packing():
    """limbs64 >= 7 used to overrun the 12-word modulus buffers; now NTT_ERR_ARG."""
    from ntt_amd import lib as L
    so = L.load()
    h = C.c_void_p()
    for limbs in (0, 2, 3, 5, 7, 8, 64):
        assert so.ntt_plan_create_ex(C.byref(h), 1, 10, limbs, 0, 0) == -1, limbs
        p = (C.c_uint64 * 8)(*([0xFFFFFFFF00000001] + [0] * 7))
        g = (C.c_uint64 * 8)(*([7] + [0] * 7))
        assert so.ntt_plan_create_custom(C.byref(h), p, g, limbs, 10, 0) == -1, limbs
        assert not h.value


def test_compiled_c_caller_builds_against_header_and_library():
    """tests/c/dropin.c (a plain-C caller of include/ntt.h) compiles with -Werror and links
    libntt.so: the header is valid C and every symbol it calls is exported."""
    import shutil
    if not shutil.which("gcc") or not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"):
        pytest.skip("gcc / ROCm headers unavailable")
    from tests.dropin_build import build
    assert os.access(build(), os.X_OK)


def test_python_constants_match_the_header():
    """Every NTT_PLAN_* / NTT_ERR_* / NTT_FIELD_* / NTT_OK value ntt_amd.lib mirrors equals the
    header's #define, and every such #define is mirrored."""
    from ntt_amd import lib as L
    text = open(os.path.join(INCLUDE, "ntt.h")).read()
    defs = {m.group(1): int(m.group(2)) for m in
            re.finditer(r"^#define\s+(NTT_(?:PLAN|ERR|FIELD)_\w+|NTT_OK)\s+\(?(-?\d+)u?\)?", text, flags=re.M)}
    assert "NTT_PLAN_NAIVE" in defs and "NTT_PLAN_NO_SWAP" in defs and "NTT_ERR_DEVICE" in defs
    for name, value in defs.items():
        assert hasattr(L, name), name
        assert getattr(L, name) == value, (name, getattr(L, name), value)


def test_conflicting_schedule_flags_are_rejected_without_a_device():
    """One rival schedule per plan, and none with NTT_PLAN_IN_PLACE: refused before any device
    query, so NTT_ERR_ARG here on a machine with no GPU."""
    from ntt_amd import lib as L
    so = L.load()
    h = C.c_void_p()
    rivals = (L.NTT_PLAN_STOCKHAM, L.NTT_PLAN_GZKP, L.NTT_PLAN_NAIVE, L.NTT_PLAN_NO_SWAP, L.NTT_PLAN_BELLPERSON,
              L.NTT_PLAN_IMPROVED_V1, L.NTT_PLAN_IMPROVED_V2, L.NTT_PLAN_IMPROVED_V3, L.NTT_PLAN_IMPROVED_V4)
    bad = [a | b for i, a in enumerate(rivals) for b in rivals[i + 1:]]
    bad += [r | L.NTT_PLAN_IN_PLACE for r in rivals] + [L.NTT_PLAN_IN_PLACE | L.NTT_PLAN_TWIDDLE_ONLY]
    for flags in bad:
        assert so.ntt_plan_create_ex(C.byref(h), 1, 12, 4, 0, flags) == L.NTT_ERR_ARG, flags
        assert not h.value


def test_bealto_kwarg_is_checked_before_the_library():
    """NTTPlan(bealto=...) names one of the five bealto-family schedules; anything else is refused
    before a plan (or a device) is touched."""
    import pytest as _pt
    from ntt_amd import lib as L
    from ntt_amd.ntt import BEALTO_FLAGS, NTTPlan
    assert BEALTO_FLAGS == {"bellperson": L.NTT_PLAN_BELLPERSON, "v1": L.NTT_PLAN_IMPROVED_V1,
                            "v2": L.NTT_PLAN_IMPROVED_V2, "v3": L.NTT_PLAN_IMPROVED_V3, "v4": L.NTT_PLAN_IMPROVED_V4}
    for bad in ("v0", "v5", "Bellperson", "stockham"):
        with _pt.raises(ValueError):
            NTTPlan(1, 12, 4, bealto=bad)
