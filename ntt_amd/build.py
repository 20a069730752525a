"""Build libntt.so (HIP kernels for gfx950 + the C ABI) in-tree with hipcc.

The shared library lands next to this file (``ntt_amd/libntt.so``) so it travels with the repo
snapshot to the GPU box.  Translation units compile in parallel and are rebuilt only when a source
or header is newer than the object.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# Variants beside the product: NTT_BUILD_TAG=<tag> NTT_BUILD_DEFINES="-DX=1 ..." builds
# ntt_amd/libntt_<tag>.so from ntt_amd/_build_<tag>/ (experiments); NTT_LIB_PATH selects it at load
# time.  build_debug() is the checked build (NTT_DEBUG_CHECKS, libntt_debug.so).
_TAG = os.environ.get("NTT_BUILD_TAG", "")
_DEFINES = os.environ.get("NTT_BUILD_DEFINES", "").split()


def _paths(tag: str):
    return (os.path.join(HERE, "_build" + (f"_{tag}" if tag else "")),
            os.path.join(HERE, "libntt" + (f"_{tag}" if tag else "") + ".so"))


BUILD, LIB = _paths(_TAG)
DEBUG_LIB = _paths("debug")[1]
INCLUDE = os.path.join(os.path.dirname(HERE), "include")

# slowest translation units first (the pool runs them in list order)
SOURCES = ["ntt_e256_fused.hip"]  # the fused single-launch 3-pass schedule (NTT_PLAN_SINGLE_LAUNCH)
SOURCES += ["ntt_e256t_fused.hip"]  # the two-pass single launch on 4096-element tiles (2^20)
SOURCES += [f"ntt_{e}_{k}.hip" for e in ("e384", "e256", "e256w", "ep") for k in ("col", "single", "fin", "misc")]
SOURCES += ["ntt_e256_stk.hip", "ntt_ep_stk.hip"]  # the bellperson-family rival schedule (NTT_PLAN_STOCKHAM)
SOURCES += ["ntt_e256_dit.hip", "ntt_ep_dit.hip"]  # the GZKP(B, G) rival schedule (NTT_PLAN_GZKP)
SOURCES += ["ntt_e256_rows.hip", "ntt_e256w_rows.hip", "ntt_ep_rows.hip"]  # batched single-tile transforms, several per workgroup (KIND_ROWS)
SOURCES += [f"ntt_epi_{k}.hip" for k in ("col", "single", "fin", "misc")]  # P with 8-B scratch (NTT_PLAN_IN_PLACE)
SOURCES += [f"ntt_e256wi_{k}.hip" for k in ("col", "single", "fin", "misc")]  # 48-B in place (NTT_PLAN_IN_PLACE)
SOURCES += [f"ntt_e256t_{k}.hip" for k in ("col", "single", "fin", "misc")]  # 4096-element tiles (2^20 single transforms)
SOURCES += ["ntt_plan.cpp", "ntt_rplan.cpp", "ntt_multi.cpp"]
ARCH = os.environ.get("NTT_OFFLOAD_ARCH", "gfx950")


def source_hash() -> str:
    """16-hex digest of every kernel / C-ABI source and header: tags measurements (PMC traffic in
    profiles/pmc_summary.json) with the code they were taken on, so bench.py never reports stale bytes."""
    import hashlib
    h = hashlib.sha256()
    for d in (CSRC, INCLUDE):
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".hpp", ".cpp", ".h")):
                h.update(f.encode())
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()[:16]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain (ROCm) is required to build libntt.so")


def _deps() -> float:
    latest = 0.0
    for d in (CSRC, INCLUDE):
        for f in os.listdir(d):
            if f.endswith((".hpp", ".h")):
                latest = max(latest, os.path.getmtime(os.path.join(d, f)))
    return latest


def _compile(src: str, hdr_mtime: float, build_dir: str, defines) -> str:
    s = os.path.join(CSRC, src)
    o = os.path.join(build_dir, src + ".o")
    if os.path.exists(o) and os.path.getmtime(o) >= max(os.path.getmtime(s), hdr_mtime):
        return o
    cmd = [hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-c", s, "-o", o,
           "-I", CSRC, "-I", INCLUDE, "-Wno-pass-failed", "-Wno-unused-command-line-argument", *defines]
    if src.endswith(".cpp"):
        cmd[1:1] = ["-x", "hip"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-4000:]}")
    return o


def build(verbose: bool = False, jobs: int | None = None, tag: str | None = None, defines=None) -> str:
    """Build libntt.so (or the variant `tag` with extra -D `defines`; default: NTT_BUILD_TAG /
    NTT_BUILD_DEFINES from the environment).  Incremental: objects newer than their sources stay."""
    build_dir, lib = _paths(_TAG if tag is None else tag)
    defines = _DEFINES if defines is None else list(defines)
    os.makedirs(build_dir, exist_ok=True)
    hdr = _deps()
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4)))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr, build_dir, defines), srcs))
    if not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib + ".tmp", *objs]
        cmd += ["-ldl"]  # RCCL is dlopen-ed by ntt_multi.cpp at first multi-GPU use
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        os.replace(lib + ".tmp", lib)
    if verbose:
        print(f"built {lib}")
    return lib


def build_debug(verbose: bool = False, jobs: int | None = None) -> str:
    """The checked build ntt_amd/libntt_debug.so (NTT_DEBUG_CHECKS=1: index bounds, canonical inputs
    and outputs, lazy bounds inside the kernels; ntt_plan_device_status reports violations).  Same
    C ABI; select it with NTT_LIB_PATH.  Slower: for debugging callers, never measured."""
    return build(verbose, jobs, tag="debug", defines=["-DNTT_DEBUG_CHECKS=1"])


if __name__ == "__main__":
    if "--debug" in sys.argv:
        build_debug(verbose=True)
    else:
        build(verbose=True)
    sys.exit(0)
