"""Parse C/OpenCL array initialisers out of the reference's table files.

Tooling only (runs in the build container where /root/reference exists).  Used by
gen_tables.py to emit this repo's compact table header and by the table tests to
check that header against the reference's constants.cl / mip_matrix.cl.
"""
import re

REF_ROOT = "/root/reference"


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def parse_arrays(path):
    """Return {name: flat list of numbers} for every `name[..] = { ... };` in path."""
    src = _strip_comments(open(path).read())
    out = {}
    pat = re.compile(r"([A-Za-z_][A-Za-z_0-9]*)\s*((?:\[[^\]]*\])+)\s*=\s*\{")
    pos = 0
    while True:
        m = pat.search(src, pos)
        if not m:
            break
        name = m.group(1)
        depth, i = 1, m.end()
        while depth:
            c = src[i]
            depth += (c == "{") - (c == "}")
            i += 1
        body = src[m.end():i - 1].replace("{", ",").replace("}", ",")
        vals = []
        for tok in body.split(","):
            tok = tok.strip()
            if not tok:
                continue
            try:
                vals.append(eval(tok, {"__builtins__": {}}))
            except Exception:
                vals.append(None)
        out[name] = vals
        pos = i
    return out


def parse_rows(path, name):
    """Return the list of inner `{...}` rows of a 2-D initialiser (rows may be short)."""
    src = _strip_comments(open(path).read())
    m = re.search(r"\b" + re.escape(name) + r"\s*((?:\[[^\]]*\])+)\s*=\s*\{", src)
    depth, i = 1, m.end()
    rows, cur = [], None
    while depth:
        c = src[i]
        if c == "{":
            depth += 1
            cur = i + 1
        elif c == "}":
            if depth == 2:
                rows.append([int(t) for t in src[cur:i].replace("\n", " ").split(",") if t.strip()])
            depth -= 1
        i += 1
    return rows
