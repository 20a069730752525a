"""Resolve a glog-style crash trace ("    @     0x7581f148d59e (unknown)") against a /proc/<pid>/maps
dump of the same process (tools/exit_crash_probe.py) into library + offset, then into function names
with llvm-symbolizer (the libraries are the same image's, so they can be read here).

    python tools/symbolize_trace.py CRASH_LOG MAPS [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess

SYMBOLIZER = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def load_maps(path):
    out = []
    for line in open(path):
        parts = line.split()
        if len(parts) < 6 or not parts[5].startswith("/"):
            continue
        lo, hi = (int(v, 16) for v in parts[0].split("-"))
        off = int(parts[2], 16)
        out.append((lo, hi, off, parts[5]))
    return out


def resolve(addr, maps):
    for lo, hi, off, path in maps:
        if lo <= addr < hi:
            return path, addr - lo + off
    return None, None


def symbolize(path, offset):
    if not os.path.exists(path) or not os.path.exists(SYMBOLIZER):
        return None
    r = subprocess.run([SYMBOLIZER, "--obj", path, "--demangle", "--functions=linkage", hex(offset)],
                       capture_output=True, text=True)
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    return lines[0] if lines else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("maps")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    maps = load_maps(a.maps)
    frames = []
    text = open(a.log, errors="replace").read()
    pc = re.search(r"PC: @\s+(0x[0-9a-f]+)", text)
    addrs = ([int(pc.group(1), 16)] if pc else []) + [int(m.group(1), 16) for m in
                                                      re.finditer(r"^\s+@\s+(0x[0-9a-f]+)", text, re.M)]
    for i, ad in enumerate(addrs):
        path, off = resolve(ad, maps)
        # return addresses point after the call: symbolize addr - 1 (not for the PC itself)
        sym = symbolize(path, off - (0 if (pc and i == 0) else 1)) if path else None
        frames.append({"addr": hex(ad), "lib": path, "offset": hex(off) if off is not None else None, "symbol": sym})
        print(f"{hex(ad)}  {os.path.basename(path) if path else '?'}+{hex(off) if off is not None else '?'}  {sym or ''}")
    if a.json:
        json.dump(frames, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
