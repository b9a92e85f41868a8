"""Index contract: the product's host join-tree
compiler reproduces the reference's clique order, dimension order, sepsets,
link order, family cliques/mappings, interface lists and original tables
bit-exactly (fixtures from the reference's own nipgraph/nipjointree code)."""
import hashlib
import json
import os

import numpy as np
import pytest

import nip_amd
from nip_amd import synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CONTRACT = json.load(open(os.path.join(GOLD, "index_contract.json")))
GRAPHS = json.load(open(os.path.join(GOLD, "graph_cliques.json")))


def model_of(entry, name):
    if name == "demo1_card32":
        return nip_amd.Model.from_spec(*synth.demo1_spec(32))
    nodes = [tuple(n) for n in entry["nodes"]]
    pots = [tuple(p) for p in entry["potentials"]]
    return nip_amd.Model.from_spec(nodes, pots)


def assert_same_desc(got, want):
    for c in got["cliques"]:
        if "original_sha256" in [k for w in want["cliques"] for k in w]:
            pass
    for cg, cw in zip(got["cliques"], want["cliques"]):
        if "original_sha256" in cw:
            a = np.asarray(cg.pop("original"), np.float64)
            assert hashlib.sha256(a.tobytes()).hexdigest() == cw["original_sha256"]
            assert len(a) == cw["original_len"]
            cw = {k: v for k, v in cw.items() if not k.startswith("original_")}
        assert cg == cw
    assert {k: v for k, v in got.items() if k != "cliques"} == \
           {k: v for k, v in want.items() if k != "cliques"}


@pytest.mark.parametrize("name", sorted(CONTRACT))
def test_index_contract(name):
    entry = CONTRACT[name]
    got = json.loads(json.dumps(model_of(entry, name).desc()))
    assert_same_desc(got, json.loads(json.dumps(entry["desc"])))


@pytest.mark.parametrize("name", ["model", "demo1"])
def test_net_reader(name):
    got = nip_amd.Model.from_net(os.path.join(GOLD, name + ".net")).desc()
    assert_same_desc(json.loads(json.dumps(got)), json.loads(json.dumps(CONTRACT[name]["desc"])))


def test_graphtest7_known_answer():
    """test/graphtest.c Test 7: cliques ABC BCD EGH DEF CEG CDE, in that order."""
    g = GRAPHS["graphtest7"]
    cl = nip_amd.graph_cliques(g["card"], g["edges"], set_parents=False)
    assert ["".join("ABCDEFGH"[v] for v in c) for c in cl] == ["ABC", "BCD", "EGH", "DEF", "CEG", "CDE"]


@pytest.mark.parametrize("name", sorted(GRAPHS))
def test_graph_cliques(name):
    g = GRAPHS[name]
    assert nip_amd.graph_cliques(g["card"], g["edges"], False) == g["cliques_noparents"]
    assert nip_amd.graph_cliques(g["card"], g["edges"], True) == g["cliques_parents"]


def test_m_step_tables():
    """m_step (nip.c:2010-2071) re-initialises the tables bit-exactly."""
    for name in ("fb_hmm16.npz", "fb_demo1.npz", "fb_model_T24.npz"):
        z = np.load(os.path.join(GOLD, name))
        m = model_of(CONTRACT[str(z["model"])], str(z["model"]))
        m.m_step(z["em_init"])
        o = np.concatenate([m.original(c) for c in range(len(m.desc()["cliques"]))])
        assert np.array_equal(o, z["mstep_originals"])


def test_chain_plan_recognition():
    m = nip_amd.Model.from_spec(*synth.hmm_spec(16, 16))
    assert m.gpu_supported([m.variable("M1")], [m.variable("P1")])
    d = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    # demo1: interface C, hidden independent parent D1 folded into the
    # transition, observed leaf children A1, B1 (SURVEY 8(d) config 3 shape)
    assert d.gpu_supported([d.variable("A1"), d.variable("B1")], [d.variable("C1")])
    assert d.gpu_supported([d.variable("B1")], [d.variable("C1")])
    # every variable of the slice can be queried (derived marginals: prev, hidden parent, children)
    assert d.gpu_supported([d.variable("A1")], [d.variable(v) for v in ("D1", "C0", "B1", "A1")])
    # evidence on a folded parent: outside the chain plan; the automatic choice
    # serves it on the evidence-indexed chain (opchain.cpp)
    d.set_engine(nip_amd.ENGINE_CHAIN)
    assert not d.gpu_supported([d.variable("D1")], [d.variable("C1")])
    d.set_engine(nip_amd.ENGINE_AUTO)
    assert d.gpu_supported([d.variable("D1")], [d.variable("C1")])
    # a slice with two interface variables is a chain over the joint interface
    # state (compile.cpp build_joint_chain_plan) for fb / filter of the
    # interface variables, their previous-slice copies and leaf children;
    # evidence on the previous slice stays on the general engine
    nodes = [("a0", 2, "a1"), ("b0", 2, "b1"), ("a1", 2, None), ("b1", 2, None), ("o", 2, None)]
    pots = [("a0", [], None), ("b0", [], None), ("a1", ["a0"], None), ("b1", ["b0", "a1"], None),
            ("o", ["b1"], None)]
    w = nip_amd.Model.from_spec(nodes, pots)
    w.set_engine(nip_amd.ENGINE_CHAIN)
    assert w.gpu_supported([w.variable("o")], [w.variable("a1")])
    assert w.gpu_supported([w.variable("o"), w.variable("b1")], [w.variable("a1"), w.variable("b1")])
    assert w.gpu_supported([w.variable("o")], [w.variable("a0"), w.variable("b0")])
    assert not w.gpu_supported([w.variable("a0")], [w.variable("a1")])   # evidence on the previous slice
    assert w.estep_supported()          # joint e_step: the HMM e_step kernel over the joint state
    c = nip_amd.Model.from_spec(*synth.coupled_spec())
    c.set_engine(nip_amd.ENGINE_CHAIN)
    assert c.gpu_supported([c.variable("A1"), c.variable("B1")], [c.variable("X1")])
    assert not c.estep_supported()      # two observed children: e_step on the general engine
    w.set_engine(nip_amd.ENGINE_AUTO)
    assert w.gpu_supported([w.variable("o")], [w.variable("a1")])
    assert w.estep_supported()
    assert w.set_engine(nip_amd.ENGINE_JTREE) == nip_amd.ENGINE_AUTO
