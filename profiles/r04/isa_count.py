#!/usr/bin/env python3
"""Static instruction count of chain_row64_kernel's filter step (config 5),
from the gfx950 ISA the product build compiles (hipcc -S, same flags):
every basic block holding one step's 64 v_fmac_f64_dpp, classified by
instruction kind.  Writes profiles/r04/isa_row64_step.json, which bench.py
reads for config 5's issue roof:
    floor cycles per step = VALU x 4 (one wave64 VALU op per 4 cycles on a
    16-lane SIMD) + SALU / s_nop / s_waitcnt x 1 + the rescale every 4th step
    python profiles/r04/isa_count.py"""
import collections
import json
import os
import re
import subprocess
import statistics

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def main():
    src = os.path.join(ROOT, "nip_amd", "csrc", "chain_wide4.hip")
    out = "/tmp/isa_row64.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC",
                           "-mllvm", "-amdgpu-mfma-vgpr-form", "-I" + os.path.join(ROOT, "include"),
                           "-I" + os.path.join(ROOT, "nip_amd", "csrc"), "-S", "--cuda-device-only", src, "-o", out])
    s = open(out).read()
    name = [n for n in re.findall(r"^(_Z\S*chain_wide4_kernelILb1ELi1E\S*):", s, re.M)][0]
    body = s[s.index(name + ":"):]
    body = body[:body.index(".Lfunc_end")]
    # the filter loops: every block annotated as part of an inner loop whose
    # blocks hold 64 v_fmac_f64_dpp per step; per-step averages over a whole
    # loop iteration (8 steps, their rescales every 4th, the chunk's overhead)
    loops = collections.defaultdict(collections.Counter)
    cur = None
    for line in body.split("\n"):
        l = line.strip()
        m = re.match(r"^(\.LBB\S+|; %bb\.\d+):\s*;?\s*(.*)$", l) or re.match(r"^(; %bb\.\d+):(.*)$", l)
        if m:
            ann = m.group(2)
            h = re.search(r"Header=(\S+)", ann)
            if "Inner Loop Header" in ann:
                cur = m.group(1).rstrip(":").lstrip(".").replace("LBB", "BB")
            elif h:
                cur = h.group(1)
            else:
                cur = None
            continue
        if cur is not None and l and not l.startswith((".", ";")):
            loops[cur][l.split()[0]] += 1
    per = []
    for h, c in loops.items():
        n = c["v_fmac_f64_dpp"]
        if n == 0 or n % 64:
            continue
        k = n // 64
        v = sum(x for op, x in c.items() if op.startswith("v_"))
        sl = sum(x for op, x in c.items() if op.startswith("s_"))
        ds = sum(x for op, x in c.items() if op.startswith("ds_"))
        per.append((h, k, v / k, sl / k, ds / k))
    # the full-chunk fast path: one basic block of 8 steps (512 v_fmac_f64_dpp)
    fast = []
    cur = None
    for line in body.split("\n"):
        l = line.strip()
        if re.match(r"^(\.LBB\S+|; %bb\.\d+):", l):
            cur = collections.Counter()
            fast.append(cur)
            continue
        if cur is not None and l and not l.startswith((".", ";")):
            cur[l.split()[0]] += 1
    fast = [c for c in fast if c["v_fmac_f64_dpp"] == 512]

    def per_step(c, k):
        return (sum(x for op, x in c.items() if op.startswith("v_")) / k,
                sum(x for op, x in c.items() if op.startswith("s_")) / k,
                sum(x for op, x in c.items() if op.startswith("ds_")) / k)
    fp = [per_step(c, 8) for c in fast]
    use = fp if fp else [x[2:] for x in per]
    rec = {
        "kernel": name, "source": "nip_amd/csrc/chain_wide4.hip r64_filter<FWD, NC=1>",
        "loops": [{"header": h, "steps": k, "valu_per_step": v, "salu_per_step": sl, "ds_per_step": ds}
                  for h, k, v, sl, ds in per],
        "fast_path_blocks": len(fp),
        "valu_per_step": statistics.median(x[0] for x in use),
        "salu_per_step": statistics.median(x[1] for x in use),
        "ds_per_step": statistics.median(x[2] for x in use),
        "note": "static counts per step of the filter's full-chunk path (one basic block of 8 unrolled steps "
                "with 64 v_fmac_f64_dpp each and their rescales every 4th step; loops: whole loop bodies incl. "
                "the checked tail path), both directions and both phases",
    }
    with open(os.path.join(HERE, "isa_row64_step.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
