"""Every reference citation (file:line) in the sources resolves to an existing
reference file and stays inside it (tools/check_citations.py).  Runs where the
reference tree is present (the build container)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import check_citations as cc  # noqa: E402


@pytest.mark.skipif(not os.path.isdir(cc.REF), reason="reference tree absent")
def test_citations_resolve():
    good, bad = cc.check()
    assert good > 300
    assert not bad, "\n".join(f"{s}:{ln}: {c}: {why}" for s, ln, c, why in bad)
