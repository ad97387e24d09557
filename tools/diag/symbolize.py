"""Offline symbolizer for tools/diag/crashtrace.c dumps (diagnostics only).

Scans the raw stack bytes for words that point into an executable mapping, maps each
to (library, file offset -> vaddr) and names the nearest symbol with addr2line / nm.
Return addresses left on the stack by live frames come out in call order (innermost
first); stale words from dead frames can appear too, so read it as a likely chain.

Usage: python tools/diag/symbolize.py PREFIX [--root DIR]
  PREFIX.{regs,stack,maps} as written by crashtrace.c; --root maps box paths (the repo
  root on the GPU box) to this container's tree.
"""
import argparse
import bisect
import os
import struct
import subprocess
import sys


def parse_maps(path):
    maps = []
    for line in open(path):
        parts = line.split()
        if len(parts) < 6 or "x" not in parts[1]:
            continue
        lo, hi = (int(x, 16) for x in parts[0].split("-"))
        maps.append((lo, hi, int(parts[2], 16), parts[5]))
    return maps


_LOADS = {}


def load_segments(lib):
    if lib not in _LOADS:
        segs = []
        out = subprocess.run(["readelf", "-lW", lib], capture_output=True, text=True).stdout
        for line in out.splitlines():
            f = line.split()
            if f and f[0] == "LOAD":
                segs.append((int(f[1], 16), int(f[2], 16), int(f[4], 16)))  # off, vaddr, filesz
        _LOADS[lib] = segs
    return _LOADS[lib]


_SYMS = {}


def dyn_symbols(lib):
    if lib not in _SYMS:
        syms = []
        for flag in ([], ["-D"]):
            out = subprocess.run(["nm", "-C", "--defined-only", *flag, lib], capture_output=True,
                                 text=True).stdout
            for line in out.splitlines():
                f = line.split(None, 2)
                if len(f) == 3 and f[1] in "tTwW":
                    syms.append((int(f[0], 16), f[2]))
        syms.sort()
        _SYMS[lib] = ([a for a, _ in syms], [s for _, s in syms])
    return _SYMS[lib]


def name_of(lib, vaddr):
    addrs, names = dyn_symbols(lib)
    i = bisect.bisect_right(addrs, vaddr) - 1
    return f"{names[i]}+{vaddr - addrs[i]:#x}" if i >= 0 else "?"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--root", default=None, help="box repo root to replace by this repo")
    a = ap.parse_args()
    maps = parse_maps(a.prefix + ".maps")
    regs = dict(l.split() for l in open(a.prefix + ".regs"))
    data = open(a.prefix + ".stack", "rb").read()
    here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    words = [int(regs["rip"], 16)] + [struct.unpack_from("<Q", data, i)[0]
                                      for i in range(0, len(data) - 7, 8)]
    seen = 0
    for w in words:
        for lo, hi, off, lib in maps:
            if lo <= w < hi:
                path = lib
                if a.root and path.startswith(a.root):
                    path = here + path[len(a.root):]
                if not os.path.exists(path):
                    print(f"{w:#x} {lib} (file absent here)")
                    break
                foff = w - lo + off
                vaddr = None
                for so, sv, sz in load_segments(path):
                    if so <= foff < so + sz:
                        vaddr = foff - so + sv
                if vaddr is None:
                    break
                print(f"{w:#x} {os.path.basename(lib)} {name_of(path, vaddr)}")
                seen += 1
                break
        if seen >= 80:
            break


if __name__ == "__main__":
    sys.exit(main())
