"""Writes tests/golden/ref_store_methods.json: the full signature of every public
method each reference store class declares (src/main/java/com/intel/distml/util/store/
*.java) and of DataStore (util/DataStore.java:17-58) — modifiers, return type, name,
parameter types and `throws` clause, no parameter names, no bodies, no source text —
so tests/test_java_dropin.py can check, here and on machines without the reference,
that every GPU subclass (integration/jni/Gpu*Store*.java) overrides each of them with
the same signature. No JDK exists in the image, so a wrong parameter
type (an overload instead of an override) or an added checked exception would
otherwise go unnoticed.
Run: python tests/golden/make_ref_store_methods.py"""
import json
import os
import re

REF = "/root/reference/src/main/java/com/intel/distml/util"
HERE = os.path.dirname(os.path.abspath(__file__))
# a class member declared on one line at the top level of a class body (4-space indent)
DECL = re.compile(r"^    (public|protected)((?: (?:abstract|static|final|synchronized))*) "
                  r"([\w\[\]<>.,? ]+?) (\w+)\(([^)]*)\)\s*(?:throws ([\w.,\s]+?))?\s*[{;]", re.M)


def _split_params(s):
    """Parameter types of a parameter list: depth-0 commas (generics kept), the last
    token of each parameter (its name) dropped, `final` ignored."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    types = []
    for p in out:
        toks = [t for t in p.split() if t != "final"]
        types.append(re.sub(r"\s+", "", "".join(toks[:-1])) if len(toks) > 1 else toks[0])
    return types


def signatures(src):
    """Every one-line public / protected method declaration of a Java class body:
    {"mods", "ret", "name", "params", "throws"} (constructors excluded)."""
    sigs = []
    for m in DECL.finditer(src):
        vis, mods, ret, name, params, throws = m.groups()
        if ret.strip() in ("class", "interface", "enum") or "class" in ret.split():
            continue
        sigs.append({"mods": [vis] + mods.split(), "ret": re.sub(r"\s+", "", ret), "name": name,
                     "params": _split_params(params),
                     "throws": sorted(t.strip() for t in throws.split(",")) if throws else []})
    return sigs


def methods(ref=REF):
    out = {}
    store = os.path.join(ref, "store")
    files = [("DataStore", os.path.join(ref, "DataStore.java"))] + \
            [(f[:-5], os.path.join(store, f)) for f in sorted(os.listdir(store)) if f.endswith(".java")]
    for cls, path in files:
        src = open(path, errors="replace").read()
        out[cls] = sorted(signatures(src), key=lambda s: (s["name"], s["params"]))
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "ref_store_methods.json"), "w") as fh:
        json.dump(methods(), fh, indent=1)
        fh.write("\n")
