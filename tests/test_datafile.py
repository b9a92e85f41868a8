"""Time-series data files: nip_amd's reader and writer
against the CPU restatement of the reference (oracle/datafile.py, which
follows nipparsers.c / nip.c line by line).  No GPU needed.

Crafted files cover every branch of the reference's structure rules: empty
lines before and after the header, single and repeated series separators,
comma and white-space separators, empty fields, missing-value tokens, unknown
states, columns that are not model variables, short lines (trailing entries
stay 0, nip.c:620-651) and lines longer than the 10000-byte read buffer.
"""
import os
import random

import numpy as np
import pytest

import nip_amd
from oracle import datafile as ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def model():
    return nip_amd.Model.from_net(os.path.join(GOLD, "model.net"))


def model_desc(m):
    n = m.num_vars
    syms = [v["symbol"] for v in m.desc()["vars"]]
    return syms, [m.state_names(v) for v in range(n)]


def check(m, path):
    got, ov = nip_amd.read_timeseries(m, path)
    syms, states = model_desc(m)
    want, wov = ref.read_timeseries(path, syms, states)
    assert ov == wov
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g.shape == (len(w), len(ov))
        assert g.tolist() == w
    return got, ov


CRAFTED = {
    "plain": "P1 M1\nF 0\nf 1\n\n! 4\nu 3\n",
    "commas": "P1,M1\nF,0\nf,1\n\n!,4\n",
    "blank_before_and_after_header": "\n\n  \nP1 M1\n\n\nF 0\nf 1\n\n\n\n! 4\n\n",
    "missing_tokens": "P1 M1\nnull 0\nF N/A\n<null> <null>\nq 7\n",
    "empty_fields": "P1,,M1\n,F,,0,\nf,,1\n",
    "extra_columns": "X P1 Y M1 Z\n1 F 2 0 3\n1 f 2 1 3\n",
    "only_observation": "M1\n0\n1\n2\n\n3\n",
    "short_lines": "P1 M1\nF\nf 1\n\n\n\nu\n",
    "long_lines": "P1 M1\n" + "F 0 " + "x" * 12000 + "\nf 1\n",
    "whitespace_mix": "P1\tM1\r\nF\t0\r\n \t \r\nf  ,  1\r\n",
    "no_model_columns": "A B\n1 2\n3 4\n\n5 6\n",
    "trailing_separators": "P1 M1,\nF 0,\n,f 1,,\n",
}


@pytest.mark.parametrize("name", sorted(CRAFTED))
def test_reader_crafted(model, tmp_path, name):
    p = tmp_path / (name + ".txt")
    p.write_text(CRAFTED[name])
    check(model, str(p))


def test_reader_values(model, tmp_path):
    p = tmp_path / "v.txt"
    p.write_text(CRAFTED["missing_tokens"])
    got, ov = check(model, str(p))
    assert ov == [model.variable("P1"), model.variable("M1")]
    assert got[0].tolist() == [[-1, 0], [0, -1], [-1, -1], [-1, -1]]
    p.write_text(CRAFTED["short_lines"])
    got, _ = check(model, str(p))
    assert [g.tolist() for g in got] == [[[0, 0], [1, 1]], [[2, 0]]]


def test_reader_random_files(model, tmp_path):
    rng = random.Random(5)
    syms, states = model_desc(model)
    for case in range(40):
        cols = rng.sample(["P0", "P1", "M1", "junk"], rng.randint(1, 4))
        lines = [rng.choice(["", " "]) for _ in range(rng.randint(0, 2))]
        lines.append(rng.choice([" ", ",", ", "]).join(cols))
        for _ in range(rng.randint(1, 5)):
            lines += ["" for _ in range(rng.randint(0, 2))]
            for _ in range(rng.randint(1, 6)):
                row = []
                for c in cols[:rng.randint(len(cols) - 1 if rng.random() < 0.8 else 0, len(cols))]:
                    if c in syms and rng.random() < 0.8:
                        row.append(rng.choice(states[syms.index(c)]))
                    else:
                        row.append(rng.choice(["null", "N/A", "<null>", "zz", "9"]))
                lines.append(rng.choice([" ", ",", " , ", "\t"]).join(row))
        p = tmp_path / ("r%d.txt" % case)
        p.write_text("\n".join(lines) + rng.choice(["", "\n", "\n\n"]))
        check(model, str(p))


def test_reader_errors(model, tmp_path):
    with pytest.raises(nip_amd.NipError):
        nip_amd.read_timeseries(model, str(tmp_path / "missing.txt"))
    p = tmp_path / "header_only.txt"
    p.write_text("P1 M1\n\n")
    with pytest.raises(nip_amd.NipError):
        nip_amd.read_timeseries(model, str(p))


def test_writer_matches_reference_text(model, tmp_path):
    rng = np.random.default_rng(2)
    v = model.variable("P1")
    posts = []
    for T in (3, 1, 5):
        x = rng.random((T, 4))
        x[0, 1] = 0.0
        x[-1, 2] = 1.0 / 3.0
        posts.append(x / x.sum(axis=1, keepdims=True))
    p = tmp_path / "out.txt"
    nip_amd.write_uncertainseries(model, str(p), v, posts)
    assert p.read_text() == ref.write_uncertainseries_text(model.state_names(v), posts)
