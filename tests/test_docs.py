"""Every profiles/ file the documentation cites exists (globs must match at least one file)."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "README.md", "INTEGRATION.md"]


@pytest.mark.parametrize("doc", DOCS)
def test_profile_citations_resolve(doc):
    text = open(os.path.join(ROOT, doc)).read()
    missing = []
    for m in re.finditer(r"profiles/([A-Za-z0-9_.*\-/]+)", text):
        name = m.group(1).rstrip(".")
        if not name or name.endswith("/"):
            continue
        if not glob.glob(os.path.join(ROOT, "profiles", name)):
            missing.append(name)
    assert not missing, "%s cites missing profiles: %s" % (doc, sorted(set(missing)))
