"""libnip.so's potential / join-tree / single-slice API on the host
(nippotential.h, nipjointree.h and nip.h's reset_model,
use_priors, insert_*, model_prob_mass, get_probability,
get_joint_probability), against the reference's OWN compiled code.

These scripts do no propagation (make_consistent / collect / distribute run
on the GPU: tests/test_gpu_slice.py), so they need no GPU.  Everything is
compared bit for bit (doubles printed as %a):
  - test/potentialtest.c, the reference's own unit test, compiled unmodified
    against include/compat + libnip.so and against the reference's sources:
    identical output, md5 ac8ecd1b... (SURVEY 8(c) known answer);
  - seeded single-slice scripts (tests/slice_util.py: hard and soft
    evidence incl. zero->nonzero likelihood changes that force global
    retractions, priors with and without history, masses, every variable's
    marginal, joint distributions, full table dumps) on 65 compiled models,
    the harness running the same script over the reference's nipjointree.c
    / nippotential.c.
get_joint_probability follows the reference's nip_gather_joint_probability
(nipjointree.c:1198-1402) where that function stays inside its arrays; where
the reference reads or writes outside them (the result is undefined there,
and for some variable sets it corrupts its heap) libnip.so returns NULL, so
those lines are only required to be NULL on our side.
"""
import ctypes
import glob
import hashlib
import os
import re
import subprocess

import pytest

import nip_amd
from nip_amd import build
from oracle import bind

import slice_util as su

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def need(path):
    if not os.access(path, os.X_OK):
        pytest.skip(f"{path} not built (no reference tree where the build ran)")
    return path


def test_potentialtest_identical_to_reference():
    ours = subprocess.run([need(os.path.join(build.REF_BIN_DIR, "potentialtest"))],
                          capture_output=True, check=True).stdout
    ref = subprocess.run([need(os.path.join(ROOT, "oracle", "_ref", "reftests", "potentialtest"))],
                         capture_output=True, check=True).stdout
    assert ours == ref
    assert hashlib.md5(ours).hexdigest().startswith("ac8ecd1b")


def compat_declared():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "compat", "*.h")):
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        syms |= set(re.findall(r"^\s*(?:const\s+)?[\w]+[\s\*]+\**(\w+)\s*\([^;{]*\)\s*;", text, re.M))
    return syms


def test_compat_exports_every_declared_symbol():
    lib = ctypes.CDLL(build.COMPAT_LIB)
    syms = compat_declared()
    for must in ("nip_general_marginalise", "nip_update_potential", "nip_collect_evidence",
                 "nip_distribute_evidence", "make_consistent", "reset_model", "use_priors",
                 "insert_ts_step", "insert_soft_evidence", "model_prob_mass", "get_probability",
                 "get_joint_probability", "nip_probability_mass", "nip_global_retraction"):
        assert must in syms, must
    missing = [s for s in sorted(syms) if not hasattr(lib, s)]
    assert not missing, missing


def models():
    return sorted(su.contract_models().items())


@pytest.fixture(scope="module")
def nets(tmp_path_factory):
    d = tmp_path_factory.mktemp("nets")
    out = {name: su.spec_to_net(nodes, pots, str(d / (name + ".net"))) for name, (nodes, pots) in models()}
    out["model"] = os.path.join(su.GOLD, "model.net")
    out["demo1"] = os.path.join(su.GOLD, "demo1.net")
    return out


def compare(net, script):
    ref = su.ref_slice(net, script)
    got = su.compat_slice(net, script)
    if ref is None:                 # the reference crashed (its gather's heap corruption)
        ref = su.ref_slice(net, script.split(" joint ")[0])
        assert ref is not None
        got = su.compat_slice(net, script.split(" joint ")[0])
    rl, gl = ref.splitlines(), got.splitlines()
    assert len(rl) == len(gl)
    for a, b in zip(rl, gl):
        if b == "joint null":
            continue                # undefined in the reference (see the module doc)
        assert a == b, su.first_diff(ref, got)
    return ref


@pytest.mark.skipif(not os.path.exists(su.REF_DRIVER), reason="oracle/_ref not built")
def test_host_slice_scripts_bit_identical(nets):
    joints = 0
    for name in sorted(nets):
        for seed in range(2):
            out = compare(nets[name], su.random_script(nets[name], seed, propagate=False))
            joints += sum(1 for l in out.splitlines() if l.startswith("joint") and l != "joint null")
    assert joints > 50              # the defined joint distributions were compared too


@pytest.mark.skipif(not os.path.exists(su.REF_DRIVER), reason="oracle/_ref not built")
def test_model_join_tree_matches_reference(nets):
    """parse_model's host join tree: every clique table, sepset and family as
    the reference builds them (a dump right after parsing)."""
    for name in ("model", "demo1", "rand05", "rand31"):
        compare(nets[name], "dump " + " ".join(f"prob {v}" for v in range(len(su.model_info(nets[name])[0]))))
