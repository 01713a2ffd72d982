"""The static-analysis gate (scripts/lint.py; the reference's go vet / staticcheck step) runs in the suite."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import lint  # noqa: E402


def test_repository_is_lint_clean(capsys):
    assert lint.main([]) == 0, capsys.readouterr().out


def test_checks_fire(tmp_path):
    bad = tmp_path / "bad.py"
    bad.write_text(
        "import os\nimport json\n\n\ndef f(x=[]):\n    try:\n        return f'plain' if x is 'a' else json\n"
        "    except:\n        return {'k': 1, 'k': 2}\n\n\ndef test_a():\n    pass\n\n\ndef test_a():\n    pass\n"
        "\n\nok = f'{1:05d}'\n")
    codes = sorted(c for _, _, c, _ in lint.lint_file(str(bad)))
    assert codes == ["B006", "E722", "F401", "F541", "F601", "F632", "F811"]
