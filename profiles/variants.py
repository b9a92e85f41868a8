#!/usr/bin/env python3
"""Build measurement variants of the library (macro switches) into
nip_amd/_lib/variants/ and, on the GPU box, bench each one.

  python profiles/variants.py build NAME=DEF1,DEF2 ...     (here)
  python profiles/variants.py bench                        (GPU box)
"""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "nip_amd", "_lib", "variants")


def build(specs):
    from nip_amd import build as b
    for spec in specs:
        name, _, defs = spec.partition("=")
        out = os.path.join(VDIR, "libnip_amd_%s.so" % name)
        b.build(defines=[d for d in defs.split(",") if d], out=out)
        print("built", out)


def bench(extra):
    for so in sorted(glob.glob(os.path.join(VDIR, "*.so"))):
        env = dict(os.environ, NIPAMD_LIB=so)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", *extra],
                           env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode or not line:
            print(os.path.basename(so), "FAILED", r.returncode, r.stderr[-500:], flush=True)
            continue
        d = json.loads(line[-1])
        print("%-28s %.4g seq-ts/s  kernel %.4f ms  frac %.3f" % (
            os.path.basename(so), d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"]), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        bench(sys.argv[2:])
