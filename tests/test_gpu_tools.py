"""The nipinference counterpart (nip_amd/_lib/nipamd_inference, SURVEY 8(d)
config 1) end to end on the GPU: data file in, posterior file out, against
the CPU oracle run on the same series (oracle/datafile.py for the file
format, oracle/nip_oracle.c for the posteriors).

Tolerance: the output is "%f" text (6 decimals), so each printed value must
be within 5e-7 (+1e-12) of the oracle's posterior; the printed average
log-likelihood ("%g", 6 significant digits) within 1e-5 relative.
"""
import os
import re
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
pytest.importorskip("torch")

import nip_amd
from nip_amd import build
from oracle import datafile as ref
from oracle.bind import PortOracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOOL = os.path.join(build.LIB_DIR, "nipamd_inference")
DBL_MAX = np.finfo(np.float64).max


def write_data(path, header, series):
    with open(path, "w") as f:
        f.write(" ".join(header) + "\n")
        for s in series:
            for row in s:
                f.write(" ".join(row) + "\n")
            f.write("\n")


def run_tool(net, data, var, out, tool=TOOL):
    r = subprocess.run([tool, net, data, var, out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"Average log\. likelihood = (\S+)", r.stdout)
    return float(m.group(1))


def parse_output(path):
    blocks, cur = [], []
    lines = open(path).read().split("\n")
    header = lines[0].split(",")
    for ln in lines[1:]:
        if ln == "":
            if cur:
                blocks.append(np.array(cur))
            cur = []
        else:
            cur.append([float(x) for x in ln.split(",")])
    return header, blocks


def check(net, header, series, var, tmp_path, tool=TOOL):
    m = nip_amd.Model.from_net(net)
    data, out = str(tmp_path / "data.txt"), str(tmp_path / "post.txt")
    write_data(data, header, series)
    avg = run_tool(net, data, var, out, tool)
    got_header, blocks = parse_output(out)
    v = m.variable(var)
    assert got_header == m.state_names(v)
    # oracle: the same file through the reference-format reader, then fb per series
    syms = [d["symbol"] for d in m.desc()["vars"]]
    rs, ov = ref.read_timeseries(data, syms, [m.state_names(i) for i in range(m.num_vars)])
    orc = PortOracle(m.desc())
    assert len(blocks) == len(rs)
    acc = 0.0
    for b, s in zip(blocks, rs):
        post, ll = orc.fb(np.array(s, np.int32).reshape(len(s), len(ov)), ov, [v])
        assert b.shape == post.shape             # zero mass: both all-zero rows, ll -DBL_MAX
        assert np.abs(b - post).max() <= 5e-7 + 1e-12
        acc += ll / len(s)
    acc /= len(rs)
    assert abs(avg - acc) <= 1e-5 * abs(acc)


def test_inference_model_net(tmp_path):
    """examples/model.net with M1 observed (and some nulls), ragged series."""
    rng = np.random.default_rng(4)
    series = []
    for T in (24, 1, 7, 24, 13, 2):
        series.append([[rng.choice(["0", "1", "2", "null"], p=[0.4, 0.3, 0.2, 0.1])] for _ in range(T)])
    check(os.path.join(GOLD, "model.net"), ["M1"], series, "P1", tmp_path)


def test_inference_interface_evidence(tmp_path):
    """P1 itself observed in some steps (nipinference marks every variable)."""
    rng = np.random.default_rng(9)
    series = []
    for T in (10, 10, 3):
        rows = []
        for _ in range(T):
            p1 = rng.choice(["F", "f", "u", "null", "null", "null"])
            rows.append([p1, rng.choice(["0", "1", "null"])])
        series.append(rows)
    check(os.path.join(GOLD, "model.net"), ["P1", "M1"], series, "P1", tmp_path)


def test_inference_demo1(tmp_path):
    """demo1.net: two observed children (A1, B1) and an ignored column."""
    m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    a, b = m.state_names(m.variable("A1")), m.state_names(m.variable("B1"))
    rng = np.random.default_rng(1)
    series = [[[rng.choice(a + ["null"]), "x", rng.choice(b)] for _ in range(T)] for T in (5, 9, 5)]
    check(os.path.join(GOLD, "demo1.net"), ["A1", "junk", "B1"], series, "C1", tmp_path)


MAP_TOOL = os.path.join(build.LIB_DIR, "nipamd_map")


def check_map(net, header, series, tmp_path, tool=MAP_TOOL):
    """nipamd_map's output file against nipmap.c restated over the oracle's
    smoothed marginals of every hidden variable (first strictly greater state
    from 0, nipmap.c:154-160); a state within 1e-9 of the maximum is a tie
    either implementation may pick."""
    m = nip_amd.Model.from_net(net)
    data, out = str(tmp_path / "data.txt"), str(tmp_path / "map.txt")
    write_data(data, header, series)
    r = subprocess.run([tool, net, data, out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    syms = [d["symbol"] for d in m.desc()["vars"]]
    names = [m.state_names(i) for i in range(m.num_vars)]
    rs, ov = ref.read_timeseries(data, syms, names)
    hidden = [v for v in range(m.num_vars) if v not in ov]
    text = open(out).read()
    lines = text.split("\n")
    assert lines[0] == " ".join(syms[v] for v in hidden)
    orc = PortOracle(m.desc())
    i = 1
    for s in rs:
        post, _ = orc.fb(np.array(s, np.int32).reshape(len(s), len(ov)), ov, hidden)
        for t in range(len(s)):
            assert lines[i].endswith(" ")
            got = lines[i][:-1].split(" ")
            i += 1
            off = 0
            for h, v in enumerate(hidden):
                row = post[t, off:off + m.card(v)]
                off += m.card(v)
                best, mx = 0, 0.0
                for j, x in enumerate(row):
                    if x > mx:
                        best, mx = j, x
                if got[h] != names[v][best]:
                    j = names[v].index(got[h])
                    assert abs(row[j] - row[best]) <= 1e-9, (t, syms[v], got[h], names[v][best], row)
        assert lines[i] == ""
        i += 1
    assert text.endswith("\n\n")


def test_map_model_net(tmp_path):
    """examples/model.net with M1 observed: MAP of P0 (the previous slice) and P1."""
    rng = np.random.default_rng(12)
    series = [[[rng.choice(["0", "1", "2", "null"], p=[0.4, 0.3, 0.2, 0.1])] for _ in range(T)]
              for T in (24, 3, 24, 1, 9)]
    check_map(os.path.join(GOLD, "model.net"), ["M1"], series, tmp_path)


def test_map_demo1_hidden_parent(tmp_path):
    """demo1.net with A1, B1 observed: MAP of C0, C1 and the hidden parent D1."""
    m = nip_amd.Model.from_net(os.path.join(GOLD, "demo1.net"))
    a, b = m.state_names(m.variable("A1")), m.state_names(m.variable("B1"))
    rng = np.random.default_rng(2)
    series = [[[rng.choice(a + ["null"]), rng.choice(b)] for _ in range(T)] for T in (6, 6, 11)]
    check_map(os.path.join(GOLD, "demo1.net"), ["A1", "B1"], series, tmp_path)
