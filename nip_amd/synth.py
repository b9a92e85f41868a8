"""Synthetic workloads of SURVEY.md 8(d) (no datasets are fetched).

* CPT entries are 0.05 + U[0,1) from splitmix64(seed=12345), normalised per
  parent configuration in the file's child-fastest layout (the parser then
  applies the reference's own re-normalisation, huginnet.y:635-636).
* Observations are i.i.d. uniform over the observed variable's states from
  splitmix64(seed=1).
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n outputs of splitmix64 starting from `seed` (vectorised)."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform01(seed: int, n: int) -> np.ndarray:
    return (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def cpt(seed: int, child_card: int, parent_configs: int) -> np.ndarray:
    """Textual-order data of a `potential (child | parents)` block."""
    d = 0.05 + uniform01(seed, child_card * parent_configs)
    d = d.reshape(parent_configs, child_card)
    return (d / d.sum(axis=1, keepdims=True)).ravel()


def hmm_spec(N: int = 16, M: int = 16, seed: int = 12345, proper: bool = False):
    """HMM-shaped DBN of config 2 (structure of examples/model.net).

    proper=True declares M1, P1, P0 in that order, so the reference's CPT
    re-normalisation runs over the child of each family (the lowest ID): the
    transition and emission rows then sum to 1, and so do the step masses
    of missing observations -- sums sitting right at a power of two."""
    nodes = [("P0", N, "P1"), ("P1", N, None), ("M1", M, None)]
    if proper:
        nodes = [nodes[2], nodes[1], nodes[0]]
    pots = [
        ("M1", ["P1"], cpt(seed, M, N)),
        ("P1", ["P0"], cpt(seed + 1, N, N)),
        ("P0", [], cpt(seed + 2, N, 1)),
    ]
    return nodes, pots


def demo1_spec(card: int = 32, seed: int = 12345):
    """examples/demo1.net structure with every variable at `card` states (config 3)."""
    nodes = [("A1", card, None), ("B1", card, None), ("C0", card, "C1"),
             ("C1", card, None), ("D1", card, None)]
    pots = [
        ("A1", ["C1"], cpt(seed, card, card)),
        ("B1", ["C1"], cpt(seed + 1, card, card)),
        ("C0", [], cpt(seed + 2, card, 1)),
        ("D1", [], cpt(seed + 3, card, 1)),
        ("C1", ["D1", "C0"], cpt(seed + 4, card, card * card)),
    ]
    return nodes, pots


def wide_spec(card: int = 64, obs_card: int = 16, seed: int = 12345):
    """X0 (NIP_next X1), Y1, Z1, X1 at `card` states, O1
    observed at `obs_card`; potentials (X1 | X0 Y1 Z1), (O1 | X1) and priors
    X0, Y1, Z1, so the in-clique {X0, Y1, Z1, X1} holds card^4 entries."""
    nodes = [("X0", card, "X1"), ("Y1", card, None), ("Z1", card, None),
             ("X1", card, None), ("O1", obs_card, None)]
    pots = [
        ("X1", ["X0", "Y1", "Z1"], cpt(seed, card, card ** 3)),
        ("O1", ["X1"], cpt(seed + 1, obs_card, card)),
        ("X0", [], cpt(seed + 2, card, 1)),
        ("Y1", [], cpt(seed + 3, card, 1)),
        ("Z1", [], cpt(seed + 4, card, 1)),
    ]
    return nodes, pots


def factorial_spec(a: int = 4, b: int = 3, m: int = 5, seed: int = 12345):
    """Factorial HMM: two hidden chains X (a states) and Y (b states) with one
    observation O1 of both -- a two-variable interface {X1, Y1} (general
    join-tree engine)."""
    nodes = [("X0", a, "X1"), ("Y0", b, "Y1"), ("X1", a, None), ("Y1", b, None), ("O1", m, None)]
    pots = [
        ("X1", ["X0"], cpt(seed, a, a)),
        ("Y1", ["Y0"], cpt(seed + 1, b, b)),
        ("O1", ["X1", "Y1"], cpt(seed + 2, m, a * b)),
        ("X0", [], cpt(seed + 3, a, 1)),
        ("Y0", [], cpt(seed + 4, b, 1)),
    ]
    return nodes, pots


def coupled_spec(a: int = 3, b: int = 4, m: int = 3, seed: int = 12345):
    """Two coupled chains: X1 | X0 Y0 and Y1 | Y0 X0, each with its own
    observed child (A1 | X1, B1 | Y1)."""
    nodes = [("X0", a, "X1"), ("Y0", b, "Y1"), ("X1", a, None), ("Y1", b, None),
             ("A1", m, None), ("B1", m + 1, None)]
    pots = [
        ("X1", ["X0", "Y0"], cpt(seed, a, a * b)),
        ("Y1", ["Y0", "X0"], cpt(seed + 1, b, a * b)),
        ("A1", ["X1"], cpt(seed + 2, m, a)),
        ("B1", ["Y1"], cpt(seed + 3, m + 1, b)),
        ("X0", [], cpt(seed + 4, a, 1)),
        ("Y0", [], cpt(seed + 5, b, 1)),
    ]
    return nodes, pots


def nonleaf_spec(n: int = 4, m: int = 3, k: int = 3, seed: int = 12345):
    """HMM whose observation O1 has an observed child Q1 of its own (a
    non-leaf observed variable)."""
    nodes = [("P0", n, "P1"), ("P1", n, None), ("O1", m, None), ("Q1", k, None)]
    pots = [
        ("P1", ["P0"], cpt(seed, n, n)),
        ("O1", ["P1"], cpt(seed + 1, m, n)),
        ("Q1", ["O1"], cpt(seed + 2, k, m)),
        ("P0", [], cpt(seed + 3, n, 1)),
    ]
    return nodes, pots


def observations(B: int, T: int, card: int, seed: int = 1, n_obs: int = 1) -> np.ndarray:
    """int32 [B, T, n_obs] uniform states."""
    u = splitmix64(seed, B * T * n_obs) % np.uint64(card)
    return u.astype(np.int32).reshape(B, T, n_obs)


def spec_to_replay(nodes, pots) -> str:
    """Replay stream for oracle/ref/nipref_harness.c (test helper)."""
    idx = {n[0]: i for i, n in enumerate(nodes)}
    out = ["V %d" % len(nodes)]
    for s, c, nx in nodes:
        out.append("%s %d %d" % (s, c, idx[nx] if nx else -1))
    out.append("P %d" % len(pots))
    for ch, ps, d in pots:
        d = [] if d is None else list(np.asarray(d, np.float64).ravel())
        out.append(" ".join([str(idx[ch]), str(len(ps))] + [str(idx[p]) for p in ps]
                            + [str(len(d))] + ["%.17g" % x for x in d]))
    return "\n".join(out) + "\n"
