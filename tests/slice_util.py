"""Helpers for the single-slice API tests (test_slice.py, test_gpu_slice.py):
write a model spec as a Hugin .net file, and run a slice script
(oracle/ref/slice_script.h) on both sides of the drop-in -- the reference's
own code through the harness (nh_slice) and libnip.so through
tests/_bin/slice_driver."""
import ctypes as C
import json
import os
import subprocess
import tempfile

import numpy as np

from oracle import bind, netfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
DRIVER = os.path.join(ROOT, "tests", "_bin", "slice_driver")
REF_DRIVER = os.path.join(ROOT, "oracle", "_ref", "slice_ref")
_REPLAYS = tempfile.mkdtemp(prefix="nip_replays_")


def spec_to_net(nodes, pots, path):
    """nodes: (symbol, card, next symbol or None); pots: (child, parents in
    file order, data in textual order)."""
    out = ["net", "{", "    node_size = (80 40);", "}"]
    for sym, card, nxt in nodes:
        out += [f"node {sym}", "{", f'    label = "{sym}";',
                "    states = (" + " ".join(f'"s{i}"' for i in range(card)) + ");"]
        if nxt:
            out.append(f'    NIP_next = "{nxt}";')
        out.append("}")
    for child, parents, data in pots:
        head = f"potential ({child} | {' '.join(parents)})" if parents else f"potential ({child})"
        body = [] if data is None else ["    data = (" + " ".join(repr(float(x)) for x in data) + ");"]
        out += [head, "{", *body, "}"]
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    return path


def contract_models():
    c = json.load(open(os.path.join(GOLD, "index_contract.json")))
    return {k: ([tuple(n) for n in v["nodes"]], [tuple(p) for p in v["potentials"]])
            for k, v in c.items() if isinstance(v["potentials"], list)}


def ref_slice(net, script):
    """The script over the reference's own code (oracle/_ref/slice_ref, a
    process of its own); None when the reference crashes on it."""
    replay = os.path.join(_REPLAYS, "%x.replay" % (hash(os.path.abspath(net)) & 0xFFFFFFFFFFFF))
    if not os.path.exists(replay):
        with open(replay, "w") as f:
            f.write(netfile.read_net(net).replay())
    r = subprocess.run([REF_DRIVER, replay, script], capture_output=True, text=True, timeout=120)
    if r.returncode < 0:
        return None
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def compat_slice(net, script):
    """The script over libnip.so (compat headers)."""
    r = subprocess.run([DRIVER, net, script], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout


def first_diff(a, b):
    for i, (x, y) in enumerate(zip(a.splitlines(), b.splitlines())):
        if x != y:
            return f"line {i}:\n ref {x[:300]}\n got {y[:300]}"
    return f"lengths {len(a)} vs {len(b)}"


def model_info(net):
    """(cards, independent var indices, parents) of the parsed model."""
    spec = netfile.read_net(net)
    cards = [len(n.states) for n in spec.nodes]
    syms = [n.symbol for n in spec.nodes]
    parents = [[] for _ in syms]
    for p in spec.potentials:
        parents[syms.index(p.child)] = [syms.index(s) for s in p.parents]
    return cards, parents


def random_script(net, seed, propagate=True, soft=True, joint=True):
    """A seeded script: reset, priors, evidence (hard and soft, some on
    zero-likelihood states to force global retractions), propagation
    (make_consistent or a collect/distribute pair from a random clique),
    masses, marginals, joint distributions and full dumps."""
    rng = np.random.default_rng(seed)
    cards, parents = model_info(net)
    nv = len(cards)
    ncl = len(bind.RefHarness(netfile.read_net(net).replay()).desc["cliques"])
    cmds = ["reset", "priors 0"]
    if propagate:
        cmds.append("consistent")
    cmds += ["mass", "dump"]
    for step in range(3):
        for v in rng.permutation(nv)[: max(1, nv // 2)]:
            if soft and rng.random() < 0.3:
                p = rng.random(cards[v])
                p[rng.integers(cards[v])] = 0.0
                cmds.append(f"soft {v} " + " ".join(repr(float(x)) for x in p))
            else:
                cmds.append(f"obs {v} {int(rng.integers(cards[v]))}")
        if propagate:
            if rng.random() < 0.7:
                cmds.append("consistent")
            else:
                c = int(rng.integers(ncl))
                cmds += [f"collect {c}", f"distribute {c}"]
        cmds += ["mass", "dump"]
        for v in range(nv):
            cmds.append(f"prob {v}")
        if joint:
            k = int(rng.integers(1, min(3, nv) + 1))
            vs = rng.choice(nv, size=k, replace=False)
            cmds.append(f"joint {k} " + " ".join(str(int(v)) for v in vs))
        if step == 1:
            cmds += ["reset", "priors 1"]
    return " ".join(cmds)
