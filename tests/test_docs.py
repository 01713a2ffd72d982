"""docs/COMPONENTS.md maps SURVEY.md's inventory to file:line definitions; scripts/doc_refs.py keeps those
line numbers true to the tree."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import doc_refs  # noqa: E402


def test_component_map_line_references_are_current():
    problems = doc_refs.check(os.path.join(ROOT, "docs", "COMPONENTS.md"), fix=False)
    assert problems == [], "stale references (python scripts/doc_refs.py --fix):\n" + "\n".join(problems)


def test_checker_finds_and_fixes_a_stale_reference(tmp_path):
    good = doc_refs.definitions("ncc/app.py", "main")
    assert good
    doc = tmp_path / "doc.md"
    doc.write_text(f"| x | `ncc/app.py:{good[0] + 3}` `main`, `ncc/kube/transport.py` pool `:1` `ConnectionPool` |\n")
    problems = doc_refs.check(str(doc), fix=True)
    assert len(problems) == 2 and "defined at line" in problems[0]
    assert doc_refs.check(str(doc), fix=False) == []
    assert f"`ncc/app.py:{good[0]}` `main`" in doc.read_text()
