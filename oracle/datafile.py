"""CPU restatement of the reference's time-series data files -- TEST
INFRASTRUCTURE ONLY (the checker for nip_amd's reader/writer; never imported
by the product).

Follows the reference line by line, including its two-pass structure:
  nip_count_tokens / nip_tokenise   src/nipstring.c:36-99, 101-199
                                    (q_strings = 0, sep_tokens = 0, wspace_sep = 1)
  nip_open_data_file                src/nipparsers.c:48-367 (nodenames = 1)
  nip_next_line_tokens              src/nipparsers.c:441-522
  read_timeseries                   src/nip.c:512-667
  nip_variable_state_index          src/nipvariable.c:239-247
  write_uncertainseries             src/nip.c:815-893
nipparsers.c is not compiled here: its build needs the NIP_ERROR_* codes,
which the tree uses but never defines, so this
restatement is pinned by crafted files that exercise each branch.
"""

MAX_LINELENGTH = 10000          # src/nipparsers.h:30
SEP = ","                       # NIP_FIELD_SEPARATOR, src/nip.h:54


def _lines(path):
    """fgets(buf, MAX_LINELENGTH, f): at most MAX_LINELENGTH - 1 bytes per read."""
    with open(path, "rb") as f:
        data = f.read()
    out, i = [], 0
    while i < len(data):
        j = data.find(b"\n", i)
        end = len(data) if j < 0 else j + 1
        end = min(end, i + MAX_LINELENGTH - 1)
        out.append(data[i:end].decode("latin-1"))
        i = end
    return out


WS = " \t\n\v\f\r"              # C isspace() in the "C" locale


def tokens(line):
    """nip_tokenise(line, n, 0, &SEP, 1, 0, 1): state 0 waits for a token,
    state 1 is inside one; a separator or white space ends it."""
    out, state, cur = [], 0, []
    for ch in line:
        if ch == SEP:
            if state == 1:
                out.append("".join(cur))
            state = 0
        elif state == 0:
            if ch not in WS:
                cur = [ch]
                state = 1
        elif ch in WS:
            out.append("".join(cur))
            state = 0
        else:
            cur.append(ch)
    if state == 1:
        out.append("".join(cur))
    return out


def open_data_file(path):
    """nip_open_data_file(path, ',', 0, 1): node symbols, rows per series."""
    lines = _lines(path)
    # pass 1: count the time series (nipparsers.c:117-150)
    ndatarows, linecounter, empty, state = 0, 0, 0, 2
    label_line, current = -1, 0
    for ln in lines:
        n = len(tokens(ln))
        current += 1
        if n == 0:
            linecounter = 0
            empty += 1
            if state or empty > 1:
                continue
        else:
            linecounter += 1
            empty = 0
            if state > 0:
                if state > 1:
                    label_line = current
                    linecounter = 0
                state -= 1
            if state == 0 and linecounter == 1:
                ndatarows += 1
    # pass 2: node symbols and rows per series (nipparsers.c:167-352)
    datarows = [0] * ndatarows
    symbols = None
    linecounter, empty, state, tscounter = 0, 0, 2, 0
    for ln in lines:
        toks = tokens(ln)
        if not toks:
            empty += 1
            continue
        if empty:
            linecounter = 1
            if state < 1:
                tscounter += 1
        else:
            linecounter += 1
        empty = 0
        if state > 0:
            state -= 1
        if state:
            symbols = toks
        else:
            datarows[tscounter] += 1
    return {"symbols": symbols or [], "datarows": datarows, "label_line": label_line, "lines": lines}


def read_timeseries(path, var_symbols, var_states):
    """read_timeseries(model, path): (series [T][n_obs] lists, observed model
    variable indices).  var_symbols / var_states describe the model."""
    df = open_data_file(path)
    N = len(df["datarows"])
    if N < 1:
        return [], []
    col_var = [var_symbols.index(s) if s in var_symbols else -1 for s in df["symbols"]]
    observed = [v for v in col_var if v >= 0]
    # nip_next_line_tokens: data lines in file order, skipping empty lines and the label line
    rows = []
    for k, ln in enumerate(df["lines"], start=1):
        t = tokens(ln)
        if not t or k == df["label_line"]:
            continue
        rows.append(t[:len(df["symbols"])])
    out, r = [], 0
    for n in range(N):
        ser = []
        for _ in range(df["datarows"][n]):
            t = rows[r]
            r += 1
            rec = [0] * len(observed)                 # calloc
            k = 0
            for i in range(len(df["symbols"])):
                if i == len(t):
                    break                              # the line was too short
                v = col_var[i]
                if v >= 0:
                    st = var_states[v]
                    rec[k] = st.index(t[i]) if t[i] in st else -1
                    k += 1
            ser.append(rec)
        out.append(ser)
    return out, observed


def write_uncertainseries_text(state_names, posts):
    """The text write_uncertainseries() produces for one variable."""
    s = SEP.join(state_names) + "\n"
    for p in posts:
        for row in p:
            s += SEP.join("%f" % x for x in row) + "\n"
        s += "\n"
    return s
