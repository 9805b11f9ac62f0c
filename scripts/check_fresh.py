#!/usr/bin/env python3
"""Fail (exit 3) when an in-tree built library is older than a source it is built from, so a
GPU run never tests a stale libpob.so / _pob / oracle build against fresh sources (the GPU
box runs the prebuilt files; the oracle is rebuilt there from its source when stale, the
HIP library is not)."""
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(ROOT, "po-brax_amd", "csrc")
checks = [
    (os.path.join(ROOT, "po-brax_amd", "po_brax_amd", "libpob.so"),
     glob.glob(os.path.join(CS, "*.h")) + glob.glob(os.path.join(CS, "*.hip")) + [os.path.join(CS, "pob_system.cpp"),
                                                                                  os.path.join(ROOT, "include", "pob.h")]),
    (glob.glob(os.path.join(ROOT, "po-brax_amd", "po_brax_amd", "_pob*.so"))[0],
     [os.path.join(CS, "pob_py.cpp"), os.path.join(ROOT, "include", "pob.h")]),
]
bad = []
for lib, srcs in checks:
    t = os.path.getmtime(lib)
    bad += [(lib, s) for s in srcs if os.path.getmtime(s) > t]
for lib, s in bad:
    print(f"STALE: {os.path.relpath(lib, ROOT)} is older than {os.path.relpath(s, ROOT)}", file=sys.stderr)
sys.exit(3 if bad else 0)
