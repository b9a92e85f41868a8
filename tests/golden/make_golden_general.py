#!/usr/bin/env python3
"""Golden fixtures for the general join-tree engine, from the reference's OWN
code (oracle/_ref: the reference's nippotential / nipjointree / nipgraph
sources compiled unmodified, nip.c's time loops restated in
oracle/ref/nipref_harness.c).

Run in the build container (where /root/reference exists and oracle/_ref is
built):  python tests/golden/make_golden_general.py
Writes tests/golden/gen_*.npz: forward_backward_inference / forward_inference
posteriors of EVERY variable and ll, e_step counts / ll / BAD_LUCK flags and
an em_learn curve, for slices outside the interface-chain plan: several
interface variables, evidence on hidden parents and on non-leaf variables,
random DBNs with and without an interface.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from nip_amd import synth  # noqa: E402  (synthetic spec generator only)
from oracle import bind  # noqa: E402
from oracle.netfile import read_net  # noqa: E402


def contract_spec(name):
    c = json.load(open(os.path.join(HERE, "index_contract.json")))[name]
    return [tuple(n) for n in c["nodes"]], [(ch, ps, d) for ch, ps, d in c["potentials"]]


def demo1_spec_native():
    ns = read_net(os.path.join(HERE, "demo1.net"))
    return [(n.symbol, len(n.states), n.next) for n in ns.nodes], \
        [(p.child, p.parents, p.data) for p in ns.potentials]


# name, spec, observed symbols (None: every non-OLD_OUTGOING variable with
# probability 1/2, seeded), B, T, seed, missing rate
CASES = [
    ("fhmm", synth.factorial_spec(4, 3, 5), ["O1"], 6, 20, 1, 0.1),
    ("coupled", synth.coupled_spec(3, 4, 3), ["A1", "B1"], 6, 20, 2, 0.1),
    ("demo1_hidden_obs", demo1_spec_native(), ["A1", "B1", "D1"], 5, 16, 3, 0.1),
    ("nonleaf", synth.nonleaf_spec(4, 3, 3), ["O1", "Q1"], 6, 18, 4, 0.15),
    ("nonleaf_q_only", synth.nonleaf_spec(4, 3, 3), ["Q1"], 5, 18, 5, 0.0),
    ("hmm_obs_hidden", synth.hmm_spec(4, 5, seed=77), ["M1", "P1"], 5, 15, 6, 0.5),
    # complete data: e_step / em_learn parity without the missing-value quirk
    ("em_fhmm", synth.factorial_spec(3, 2, 4), ["O1"], 6, 24, 7, 0.0),
    ("em_coupled", synth.coupled_spec(2, 3, 3), ["A1", "B1"], 6, 24, 8, 0.0),
    ("em_demo1_hidden_obs", demo1_spec_native(), ["A1", "B1", "D1"], 5, 20, 9, 0.0),
    ("em_nonleaf", synth.nonleaf_spec(3, 3, 2), ["O1", "Q1"], 6, 20, 10, 0.0),
]
RAND = ["rand00", "rand04", "rand05", "rand08", "rand11", "rand14", "rand17", "rand25",
        "rand30", "rand31", "rand49", "rand51", "rand53", "rand58"]


def main():
    assert bind.ref_available(), "build oracle/_ref first"
    cases = list(CASES)
    for k, name in enumerate(RAND):
        cases.append((name, contract_spec(name), None, 4, 12, 100 + k, 0.1))
    for name, (nodes, pots), osyms, B, T, seed, miss in cases:
        ref = bind.RefHarness(synth.spec_to_replay(nodes, pots))
        d = ref.desc
        syms = [v["symbol"] for v in d["vars"]]
        r = np.random.default_rng(seed)
        if osyms is None:
            ov = [i for i, v in enumerate(d["vars"]) if not (v["if"] & 4) and r.random() < 0.5]
            if not ov:
                ov = [len(syms) - 1]
        else:
            ov = [syms.index(s) for s in osyms]
        q = list(range(len(syms)))                 # every variable
        cards = [d["vars"][v]["card"] for v in ov]
        obs = np.stack([np.stack([r.integers(0, c, size=T) for c in cards], 1) for _ in range(B)]).astype(np.int32)
        obs[r.random(obs.shape) < miss] = -1
        posts, lls, fposts, flls = [], [], [], []
        for b in range(B):
            p, l = ref.fb(obs[b], ov, q)
            fp, fl = ref.fb(obs[b], ov, q, filter_only=True)
            posts.append(p); lls.append(l); fposts.append(fp); flls.append(fl)
        ps = ref.param_size()
        cnt, ell, bad = ref.estep(obs, ov, np.ones(ps))
        init = synth.uniform01(2000 + seed, ps) + 0.05
        it, curve = ref.em(obs, ov, init, 1e-6, 8)
        np.savez_compressed(os.path.join(HERE, "gen_%s.npz" % name),
                            spec=np.array(json.dumps([[list(n) for n in nodes],
                                                      [[ch, list(ps), None if dd is None else
                                                        [float(x) for x in np.ravel(dd)]]
                                                       for ch, ps, dd in pots]])),
                            obs=obs, obs_vars=np.array(ov, np.int32), query=np.array(q, np.int32),
                            post=np.stack(posts), ll=np.array(lls), fpost=np.stack(fposts),
                            fll=np.array(flls), counts=cnt, estep_ll=ell, estep_bad=bad,
                            em_init=init, em_iters=np.array(it), em_curve=curve)
        print(name, "vars", len(syms), "obs", ov, "bad", int(bad.sum()), "em", it)


if __name__ == "__main__":
    main()
