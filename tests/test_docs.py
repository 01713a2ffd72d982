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


def test_every_environment_variable_is_documented():
    """docs/ENVIRONMENT.md lists every NCC_* variable (or compile-time macro) the sources read."""
    import re
    names = set()
    for base in ("ncc", "native", "bench", "scripts"):
        for dirpath, _dirs, files in os.walk(os.path.join(ROOT, base)):
            for f in files:
                if f.endswith((".py", ".cpp", ".hpp")):
                    with open(os.path.join(dirpath, f), errors="replace") as fh:
                        names.update(re.findall(r"NCC_[A-Z][A-Z_]*[A-Z]", fh.read()))
    with open(os.path.join(ROOT, "bench.py")) as fh:
        names.update(re.findall(r"NCC_[A-Z][A-Z_]*[A-Z]", fh.read()))
    with open(os.path.join(ROOT, "docs", "ENVIRONMENT.md")) as fh:
        doc = fh.read()
    documented = set(re.findall(r"NCC_[A-Z][A-Z_]*[A-Z]", doc))
    missing = {n for n in names if n not in documented and not any(n.startswith(p) for p in ("NCC_OPT_",))}
    assert not missing, sorted(missing)


def test_profile_archive_round_trip(tmp_path, monkeypatch):
    """scripts/archive_profiles.py: a packed run directory reads back file for file (JSON and text)."""
    import json
    import sys
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import archive_profiles as ap
    monkeypatch.setattr(ap, "ROOT", str(tmp_path))
    rd = tmp_path / "profiles" / "r9"
    (rd / "keepme").mkdir(parents=True)
    (rd / "run1").mkdir()
    (rd / "run1" / "a.json").write_text('{"value": 1}\n')
    (rd / "run1" / "a.err").write_text("tail of stderr\n")
    (rd / "README.md").write_text("# index\n")
    (rd / "keepme" / "b.json").write_text("{}")
    packed, left = ap.pack(str(rd), {"keepme"})
    assert packed == 2 and left == 2
    assert not (rd / "run1").exists() and (rd / "README.md").exists() and (rd / "keepme" / "b.json").exists()
    assert json.loads(ap.show(str(rd / "run1" / "a.json"))) == {"value": 1}
    assert ap.show(str(rd / "run1" / "a.err")) == "tail of stderr\n"
    assert ap.show(str(rd / "keepme" / "b.json")) == "{}"
