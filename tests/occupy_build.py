"""Build tests/c/libocc.so (tests/c/occupy.hip: a kernel that holds CUs for a while) with hipcc, for the
GPU tests of the single launches' ordering and residency (tests/test_gpu_fused_order.py).  Built on
the CPU beside the product (__graft_entry__.build()); the .so travels to the GPU box."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "occupy.hip")
OUT = os.path.join(ROOT, "tests", "c", "libocc.so")


def build() -> str:
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= os.path.getmtime(SRC):
        return OUT
    hipcc = os.environ.get("HIPCC") or "/opt/rocm/bin/hipcc"
    arch = os.environ.get("NTT_OFFLOAD_ARCH", "gfx950")
    subprocess.run([hipcc, "-O2", f"--offload-arch={arch}", "-shared", "-fPIC", SRC, "-o", OUT + ".tmp"], check=True,
                   capture_output=True, text=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build())
