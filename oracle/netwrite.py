"""CPU restatement of the reference's write_model (src/nip.c:298-484) -- TEST
INFRASTRUCTURE ONLY (the checker for nip_amd's .net writer).

nip.c is not compiled here, so this follows its print
statements line by line over the join-tree description the host compiler
exports (bit-exact with the reference, tests/test_compiler.py):
  header            nip.c:334-348   (NET_LANG_V1 undefined: "net {...}")
  node blocks       nip.c:351-366   (NIP_next of v->previous, as written there)
  priors            nip.c:369-390   (independent variables, "%f  ", 7 per line)
  conditionals      nip.c:393-469   (family marginal, nip_normalise_cpd, " %f ",
                                     parent-configuration comments)
nip_general_marginalise / nip_normalise_cpd / nip_inverse_mapping follow
src/nippotential.c:267-311, 363-383, 251-264.
"""
import re

PER_LINE = 7                    # POTENTIAL_ELEMENTS_PER_LINE, nip.c:26


def net_layout(text):
    """label / position per node and the net block's node_size (what
    huginnet.y keeps: label default " ", position 100 100, node_size 80 60)."""
    ns = re.search(r"\bnet\s*\{[^}]*?node_size\s*=\s*\(\s*(\S+)\s+(\S+)\s*\)", text)
    node_size = (abs(int(float(ns.group(1)))), abs(int(float(ns.group(2))))) if ns else (80, 60)
    nodes = {}
    for m in re.finditer(r"\bnode\s+(\S+)\s*\{(.*?)\}", text, re.S):
        body = m.group(2)
        lab = re.search(r'label\s*=\s*"([^"]*)"', body)
        pos = re.search(r"position\s*=\s*\(\s*(\S+)\s+(\S+)\s*\)", body)
        nodes[m.group(1)] = (lab.group(1) if lab else " ",
                             (abs(int(float(pos.group(1)))), abs(int(float(pos.group(2))))) if pos else (100, 100))
    return node_size, nodes


def _family_table(desc, v):
    V = desc["vars"]
    var = V[v]
    c = desc["cliques"][var["family"]]
    ccard = [V[u]["card"] for u in c["vars"]]
    dcard = [var["card"]] + [V[p]["card"] for p in var["parents"]]
    size = 1
    for d in dcard:
        size *= d
    dest = [0.0] * size
    idx = [0] * len(ccard)
    fm = var["family_mapping"]
    for x in c["original"]:
        di, stride = 0, 1
        for k, d in enumerate(dcard):
            di += idx[fm[k]] * stride
            stride *= d
        dest[di] += x
        for k in range(len(idx)):
            idx[k] += 1
            if idx[k] < ccard[k]:
                break
            idx[k] = 0
    n = var["card"]
    for b in range(0, size, n):
        s = sum(dest[b:b + n])
        if s != 0.0:
            for x in range(n):
                dest[b + x] /= s
    return dest


def write_model_text(desc, state_names, node_size, layout, independent, children):
    V = desc["vars"]
    out = ["net\n", "{\n", "    node_size = (%d %d);\n" % node_size, "}\n"]
    for i, v in enumerate(V):
        label, pos = layout.get(v["symbol"], (" ", (100, 100)))
        names = state_names[i]
        out += ["\n", "node %s\n" % v["symbol"], "{\n", '    label = "%s";\n' % label,
                "    position = (%d %d);\n" % pos, "    states = ("]
        for s in names[:-1]:
            out.append(' "%s" \n              ' % s)
        out.append(' "%s" );\n' % names[-1])
        if v["previous"] >= 0:
            out.append('    NIP_next = "%s";\n' % V[v["previous"]]["symbol"])
        out.append("}\n")
    for i in independent:
        v = V[i]
        out += ["\n", "potential (%s)\n" % v["symbol"], "{\n", "    data = ( "]
        for j, x in enumerate(v["prior"]):
            if j > 0 and j % PER_LINE == 0:
                out.append("\n             ")
            out.append("%f  " % x)
        out += [");\n", "}\n"]
    for i in children:
        v = V[i]
        par = v["parents"]
        out += ["\n", "potential (%s | " % v["symbol"]]
        for j in range(len(par) - 1, 0, -1):
            out.append("%s " % V[par[j]]["symbol"])
        out += ["%s)\n" % V[par[0]]["symbol"], "{ \n", "    data = ("]
        p = _family_table(desc, i)
        n = v["card"]
        y = 0
        for j, x in enumerate(p):
            new = j % n == 0
            if j > 0 and (new or (n > PER_LINE and y % PER_LINE == 0)):
                if new:
                    out.append(" % ")
                    r = (j - 1) // n
                    pv = []
                    for q in par:
                        pv.append(r % V[q]["card"])
                        r //= V[q]["card"]
                    for k in range(len(par) - 1, -1, -1):
                        out.append("%s=%s " % (V[par[k]]["symbol"], state_names[par[k]][pv[k]]))
                out.append("\n            ")
                y = 0
            out.append(" %f " % x)
            y += 1
        out += [");\n", "}\n"]
    return "".join(out)
