"""Writes tests/golden/ref_store_methods.json: the names of the public methods each
reference store class declares (src/main/java/com/intel/distml/util/store/*.java;
names only, no source text), so tests/test_java_dropin.py can check that every
GPU subclass (integration/jni/Gpu*Store*.java) overrides each of them, here and on
machines without the reference.
Run: python tests/golden/make_ref_store_methods.py"""
import json
import os
import re

REF = "/root/reference/src/main/java/com/intel/distml/util/store"
HERE = os.path.dirname(os.path.abspath(__file__))
METHOD = re.compile(r"^    public (?!class\b|static\b)[\w\[\]<>.]+ (\w+)\(", re.M)


def methods(ref=REF):
    out = {}
    for f in sorted(os.listdir(ref)):
        if f.endswith(".java"):
            src = open(os.path.join(ref, f), errors="replace").read()
            out[f[:-5]] = sorted(set(METHOD.findall(src)))
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "ref_store_methods.json"), "w") as fh:
        json.dump(methods(), fh, indent=1)
        fh.write("\n")
