#!/usr/bin/env python3
"""Build the product library of another git revision for an interleaved A/B
on one GPU box (profiles/r03/ab_bench.sh):
    python profiles/r04/build_ab.py REV NAME [DEFINE...]  ->  nip_amd/_lib/ab/NAME.so
(REV "WORKTREE": the working tree's own sources, e.g. for a stamps build)
The revision's csrc and headers are extracted to /tmp and compiled with that
revision's own build.py (same flags), so only the kernels differ."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rev, name, defines = sys.argv[1], sys.argv[2], sys.argv[3:]
    tmp = "/tmp/ab_" + name
    subprocess.check_call(["rm", "-rf", tmp])
    os.makedirs(tmp)
    files = ["nip_amd/csrc", "nip_amd/build.py", "nip_amd/__init__.py", "nip_amd/em.py", "nip_amd/synth.py", "include"]
    if rev == "WORKTREE":
        subprocess.check_call(["tar", "-c", "-f", tmp + ".tar", "-C", ROOT, *files])
        subprocess.check_call(["tar", "-x", "-f", tmp + ".tar", "-C", tmp])
    else:
        arch = subprocess.run(["git", "-C", ROOT, "archive", rev, *files], check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", tmp], input=arch, check=True)
    out = os.path.join(ROOT, "nip_amd", "_lib", "ab", name + ".so")
    code = ("import sys; sys.path.insert(0, %r); from nip_amd import build as b; print(b.build(out=%r, defines=%r))"
            % (tmp, out, defines))
    subprocess.check_call([sys.executable, "-c", code])


if __name__ == "__main__":
    main()
