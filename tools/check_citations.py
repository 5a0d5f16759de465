#!/usr/bin/env python3
"""Audit of the reference citations (file:line) in this repository's sources.

Every `name.ext:N` / `name.ext:N-M` (comma lists too) in the product, oracle, tests,
tools and docs is resolved against /root/reference: a path with a directory part is
looked up under the reference root and its bpf/ and bpf/lib/ subtrees, a bare file
name under the reference tree (bpf/lib/ first).  A citation is BAD when the file does
not exist there or the range runs past the end of the file.  Usage:

    python tools/check_citations.py            # report, exit 1 on any bad citation
    python tools/check_citations.py --show     # also print the first cited line of each

Only runs where /root/reference exists (the build container); tests/test_citations.py
wraps it.
"""
from __future__ import annotations

import os
import re
import sys

REF = os.environ.get("CV_REFERENCE", "/root/reference")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCAN_DIRS = ("cilium_amd", "oracle", "include", "tests", "tools")
SCAN_FILES = ("DESIGN.md", "INTEGRATION.md", "README.md", "bench.py", "__graft_entry__.py")
EXTS = (".c", ".h", ".hpp", ".hip", ".cpp", ".py", ".md", ".sh")
# reference source kinds a citation can name
CITE = re.compile(r"(?<![\w/.-])((?:[\w.-]+/)*[\w.-]+\.(?:c|h|go|sh|rst|yaml|t))"
                  r":(\d+(?:-\d+)?(?:,\s?\d+(?:-\d+)?)*)")
# files of this repository that share a name with a reference file are not citations
OWN = {"cv_oracle.c", "cv_oracle.h", "cilium_hip.h", "ref_probe.c", "cv_common.hpp"}

_index = None


def _ref_index():
    global _index
    if _index is None:
        _index = {}
        for d, _, files in os.walk(REF):
            if "/vendor" in d or "/.git" in d:
                continue
            for f in files:
                _index.setdefault(f, []).append(os.path.join(d, f))
    return _index


def resolve(path):
    if "/" in path:
        for base in ("", "bpf", "bpf/lib"):
            p = os.path.join(REF, base, path)
            if os.path.isfile(p):
                return p
        tail = path.split("/")[-1]
        cands = [c for c in _ref_index().get(tail, []) if c.endswith("/" + path)]
        return cands[0] if cands else None
    cands = _ref_index().get(path, [])
    if not cands:
        return None
    for pref in ("/bpf/lib/", "/bpf/", "/pkg/", "/daemon/"):
        for c in cands:
            if pref in c[len(REF):]:
                return c
    return cands[0]


_lines = {}


def nlines(p):
    if p not in _lines:
        with open(p, "rb") as f:
            _lines[p] = f.read().decode("utf-8", "replace").split("\n")
    return _lines[p]


def scan():
    files = [os.path.join(ROOT, f) for f in SCAN_FILES]
    for d in SCAN_DIRS:
        for dp, _, fs in os.walk(os.path.join(ROOT, d)):
            if "__pycache__" in dp or "/_" in dp[len(ROOT):]:
                continue
            files += [os.path.join(dp, f) for f in fs if f.endswith(EXTS)]
    out = []
    for fp in files:
        if not os.path.isfile(fp) or fp.endswith("check_citations.py"):
            continue
        with open(fp, encoding="utf-8", errors="replace") as f:
            for ln, line in enumerate(f, 1):
                for m in CITE.finditer(line):
                    name, ranges = m.group(1), m.group(2)
                    if name.split("/")[-1] in OWN or name.startswith(("tests/", "tools/", "profiles/", "oracle/")):
                        continue
                    out.append((os.path.relpath(fp, ROOT), ln, name, ranges))
    return out


def check(show=False):
    bad, good = [], 0
    for src, ln, name, ranges in scan():
        p = resolve(name)
        if p is None:
            bad.append((src, ln, f"{name}:{ranges}", "file not in the reference"))
            continue
        L = nlines(p)
        n = len(L) - (1 if L and L[-1] == "" else 0)
        for r in re.split(r",\s?", ranges):
            a, _, b = r.partition("-")
            a, b = int(a), int(b or a)
            if b < a or b > n or a < 1:
                bad.append((src, ln, f"{name}:{r}", f"past the end ({os.path.relpath(p, REF)} has {n} lines)"))
            else:
                good += 1
                if show:
                    print(f"{src}:{ln}: {name}:{r} -> {L[a - 1].strip()[:90]}")
    return good, bad


def main():
    if not os.path.isdir(REF):
        print(f"{REF} absent: nothing to check")
        return 0
    good, bad = check("--show" in sys.argv)
    for src, ln, cite, why in bad:
        print(f"BAD {src}:{ln}: {cite}: {why}")
    print(f"{good} citation ranges resolve, {len(bad)} bad")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
