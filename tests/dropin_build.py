"""Build tests/c/dropin (the compiled C caller of include/ntt.h + libntt.so) with gcc."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "dropin.c")
OUT = os.path.join(ROOT, "tests", "c", "dropin")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def build() -> str:
    deps = [SRC, os.path.join(ROOT, "include", "ntt.h"), os.path.join(ROOT, "ntt_amd", "libntt.so")]
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(d) for d in deps):
        return OUT
    cmd = ["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
           f"-I{ROCM}/include", f"-I{ROOT}/include", SRC, "-o", OUT + ".tmp",
           f"-L{ROOT}/ntt_amd", "-lntt", f"-L{ROCM}/lib", "-lamdhip64",
           "-Wl,-rpath,$ORIGIN/../../ntt_amd", f"-Wl,-rpath,{ROCM}/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT
