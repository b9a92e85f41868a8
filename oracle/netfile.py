"""Minimal Hugin .net reader -- TEST INFRASTRUCTURE ONLY (oracle).

Turns a .net file (or an in-memory model spec) into the "replay stream" that
oracle/ref/nipref_harness.c replays through the reference's own model-building
calls, in the order src/huginnet.y's grammar actions run them:

  * nodeDeclaration (huginnet.y:321-387): one variable per `node`, in file
    order -- this order fixes the variable IDs (nipvariable.c:60,72), which in
    turn fix every clique's dimension order;
  * potentialDeclaration (huginnet.y:582-780): parents in FILE order here; the
    harness reverses them exactly as the grammar's prepend does (:753-766);
  * NIP_next (huginnet.y persistenceDeclaration) -> index of the next-slice node.

This module is independent of the product's own .net reader.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field

_TOK = re.compile(r'"[^"]*"|[A-Za-z_][A-Za-z0-9_.\-]*|[-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?|[(){}=;|]')


@dataclass
class Node:
    symbol: str
    states: list
    next: str | None = None


@dataclass
class Potential:
    child: str
    parents: list            # file order
    data: list | None        # flattened textual order, or None for "{ }"


@dataclass
class NetSpec:
    nodes: list = field(default_factory=list)
    potentials: list = field(default_factory=list)

    def index(self, sym):
        for i, n in enumerate(self.nodes):
            if n.symbol == sym:
                return i
        raise KeyError(sym)

    def replay(self) -> str:
        """Token stream consumed by nh_build()."""
        out = ["V %d" % len(self.nodes)]
        for n in self.nodes:
            nxt = self.index(n.next) if n.next else -1
            out.append("%s %d %d" % (n.symbol, len(n.states), nxt))
        out.append("P %d" % len(self.potentials))
        for p in self.potentials:
            par = [self.index(s) for s in p.parents]
            d = p.data or []
            out.append(" ".join([str(self.index(p.child)), str(len(par))]
                                + [str(i) for i in par] + [str(len(d))]
                                + ["%.17g" % x for x in d]))
        return "\n".join(out) + "\n"


def _strip_comments(text: str) -> str:
    lines = []
    for line in text.splitlines():
        out, inq = [], False
        for ch in line:
            if ch == '"':
                inq = not inq
            if ch == '%' and not inq:
                break
            out.append(ch)
        lines.append("".join(out))
    return "\n".join(lines)


def parse_net(text: str) -> NetSpec:
    toks = _TOK.findall(_strip_comments(text))
    spec = NetSpec()
    i = 0

    def skip_block(j):
        depth = 0
        while j < len(toks):
            if toks[j] == '{':
                depth += 1
            elif toks[j] == '}':
                depth -= 1
                if depth == 0:
                    return j + 1
            j += 1
        return j

    while i < len(toks):
        t = toks[i]
        if t == 'net':
            i = skip_block(i + 1)
        elif t in ('node', 'discrete'):
            if t == 'discrete':
                i += 1
            sym = toks[i + 1]
            i += 2
            assert toks[i] == '{'
            i += 1
            states, nxt = [], None
            while toks[i] != '}':
                key = toks[i]
                assert toks[i + 1] == '='
                j = i + 2
                vals = []
                if toks[j] == '(':
                    j += 1
                    while toks[j] != ')':
                        vals.append(toks[j])
                        j += 1
                    j += 1
                else:
                    vals.append(toks[j])
                    j += 1
                assert toks[j] == ';'
                if key == 'states':
                    states = [v.strip('"') for v in vals]
                elif key == 'NIP_next':
                    nxt = vals[0].strip('"')
                i = j + 1
            i += 1
            spec.nodes.append(Node(sym, states, nxt))
        elif t == 'potential':
            assert toks[i + 1] == '('
            child = toks[i + 2]
            j = i + 3
            parents = []
            if toks[j] == '|':
                j += 1
                while toks[j] != ')':
                    parents.append(toks[j])
                    j += 1
            assert toks[j] == ')'
            j += 1
            assert toks[j] == '{'
            j += 1
            data = None
            while toks[j] != '}':
                if toks[j] == 'data':
                    j += 2  # 'data' '='
                    vals = []
                    while toks[j] != ';':
                        if toks[j] not in '()':
                            vals.append(float(toks[j]))
                        j += 1
                    data = vals
                    j += 1
                else:
                    while toks[j] != ';':
                        j += 1
                    j += 1
            spec.potentials.append(Potential(child, parents, data))
            i = j + 1
        else:
            i += 1
    return spec


def read_net(path: str) -> NetSpec:
    with open(path) as f:
        return parse_net(f.read())
