"""Writes tests/golden/ref_line_counts.json: the line count of every .java /
.scala file under /root/reference (data about the reference, no source text),
so tests/test_citations.py can check every `File.java:N-M` citation in this
repo lies inside the cited file, here and on machines without the reference.
Run: python tests/golden/make_ref_line_counts.py"""
import json
import os

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def counts(ref=REF):
    out = {}
    for dp, _, fn in os.walk(ref):
        for f in fn:
            if f.endswith((".java", ".scala")):
                p = os.path.join(dp, f)
                out[os.path.relpath(p, ref)] = sum(1 for _ in open(p, errors="replace"))
    return dict(sorted(out.items()))


if __name__ == "__main__":
    with open(os.path.join(HERE, "ref_line_counts.json"), "w") as fh:
        json.dump(counts(), fh, indent=1)
        fh.write("\n")
