#!/usr/bin/env python
"""Static checks for the Python sources (the CI lint gate; the reference runs gofmt, go vet and
golangci-lint/staticcheck — /root/reference/.github/workflows/build.yaml:33-42, .golangci.yaml).

No third-party linter is needed (none is installable offline); the checks are the pyflakes/vet class
of mistakes that compile fine and fail at run time or silently:

* F401  imported name never used (module re-exports in `__init__.py`/`__all__` and `# noqa` excepted)
* F811  a function/class redefined in the same scope before any use (a duplicate test silently drops
        the first one)
* F541  f-string without placeholders
* F601  duplicate constant key in a dict literal
* F632  `is` / `is not` against a str/bytes/number literal
* E722  bare `except:`
* B006  mutable default argument (list/dict/set literal)
* E999  syntax error

Usage: python scripts/lint.py [paths...]   (default: ncc bench tests scripts bench.py __graft_entry__.py setup.py)
Exit status 1 when anything is found.  CI additionally runs `ruff check` when it can install it.
"""
from __future__ import annotations

import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = ["ncc", "bench", "tests", "scripts", "native", "bench.py", "__graft_entry__.py", "setup.py"]


def _files(paths):
    for p in paths:
        p = os.path.join(ROOT, p) if not os.path.isabs(p) else p
        if os.path.isfile(p) and p.endswith(".py"):
            yield p
        elif os.path.isdir(p):
            for d, dirs, fs in os.walk(p):
                dirs[:] = [x for x in dirs if not x.startswith((".", "__pycache__", "build"))]
                for f in sorted(fs):
                    if f.endswith(".py"):
                        yield os.path.join(d, f)


class _Checker(ast.NodeVisitor):
    def __init__(self, path: str, src: str):
        self.path = path
        self.lines = src.splitlines()
        self.out: list[tuple] = []
        self.used: set[str] = set()
        self.imports: list[tuple] = []  # (name, node)
        self.is_init = os.path.basename(path) == "__init__.py"
        self.all_names: set[str] = set()
        self.specs: set[int] = set()

    def report(self, node, code, msg):
        line = self.lines[node.lineno - 1] if 0 < node.lineno <= len(self.lines) else ""
        if "noqa" in line:
            return
        self.out.append((self.path, node.lineno, code, msg))

    # -- names
    def visit_Name(self, node):
        self.used.add(node.id)
        self.generic_visit(node)

    def visit_Attribute(self, node):
        self.generic_visit(node)

    def visit_Import(self, node):
        for a in node.names:
            name = a.asname or a.name.split(".")[0]
            self.imports.append((name, node))
        self.generic_visit(node)

    def visit_ImportFrom(self, node):
        if node.module == "__future__":
            return
        for a in node.names:
            if a.name == "*":
                continue
            self.imports.append((a.asname or a.name, node))
        self.generic_visit(node)

    def visit_Assign(self, node):
        for t in node.targets:
            if isinstance(t, ast.Name) and t.id == "__all__" and isinstance(node.value, (ast.List, ast.Tuple)):
                self.all_names |= {e.value for e in node.value.elts if isinstance(e, ast.Constant)}
        self.generic_visit(node)

    # -- checks
    def visit_FormattedValue(self, node):
        if node.format_spec is not None:  # `{x:05d}`: the spec is a JoinedStr of its own
            self.specs.add(id(node.format_spec))
        self.generic_visit(node)

    def visit_JoinedStr(self, node):
        if id(node) not in self.specs and not any(isinstance(v, ast.FormattedValue) for v in node.values):
            self.report(node, "F541", "f-string without placeholders")
        self.generic_visit(node)

    def visit_Dict(self, node):
        seen = set()
        for k in node.keys:
            if isinstance(k, ast.Constant):
                if k.value in seen:
                    self.report(k, "F601", f"duplicate dict key {k.value!r}")
                seen.add(k.value)
        self.generic_visit(node)

    def visit_Compare(self, node):
        for op, right in zip(node.ops, node.comparators):
            if isinstance(op, (ast.Is, ast.IsNot)) and isinstance(right, ast.Constant) and \
                    isinstance(right.value, (str, bytes, int, float)) and not isinstance(right.value, bool):
                self.report(node, "F632", "`is` comparison with a literal")
        self.generic_visit(node)

    def visit_ExceptHandler(self, node):
        if node.type is None:
            self.report(node, "E722", "bare `except:`")
        self.generic_visit(node)

    def _defaults(self, node):
        for d in list(node.args.defaults) + [x for x in node.args.kw_defaults if x is not None]:
            if isinstance(d, (ast.List, ast.Dict, ast.Set)):
                self.report(d, "B006", "mutable default argument")

    def visit_FunctionDef(self, node):
        self._defaults(node)
        self.generic_visit(node)

    visit_AsyncFunctionDef = visit_FunctionDef

    def check_redefinitions(self, body, scope_used):
        defined: dict[str, ast.AST] = {}
        for stmt in body:
            if isinstance(stmt, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
                if any(isinstance(d, ast.Name) and d.id in ("overload", "property") or
                       isinstance(d, ast.Attribute) and d.attr in ("setter", "getter", "deleter", "register")
                       for d in stmt.decorator_list):
                    continue
                prev = defined.get(stmt.name)
                if prev is not None:
                    self.report(stmt, "F811", f"redefinition of {stmt.name!r} from line {prev.lineno}")
                defined[stmt.name] = stmt
                if isinstance(stmt, ast.ClassDef):
                    self.check_redefinitions(stmt.body, scope_used)
            elif isinstance(stmt, (ast.If, ast.Try)):
                continue  # conditional definitions (fallback implementations) are deliberate
            else:
                # a use between two definitions makes the second one a deliberate rebinding
                for n in ast.walk(stmt):
                    if isinstance(n, ast.Name) and n.id in defined:
                        defined.pop(n.id, None)

    def finish(self, tree):
        self.check_redefinitions(tree.body, self.used)
        # names used only inside string annotations count as used
        for node in ast.walk(tree):
            if isinstance(node, ast.Constant) and isinstance(node.value, str) and node.value.isidentifier():
                self.used.add(node.value)
            elif isinstance(node, ast.Constant) and isinstance(node.value, str) and "." in node.value:
                self.used.add(node.value.split(".")[0])
        if self.is_init:
            return
        for name, node in self.imports:
            if name not in self.used and name not in self.all_names:
                self.report(node, "F401", f"{name!r} imported but unused")


def lint_file(path: str) -> list:
    with open(path, encoding="utf-8") as f:
        src = f.read()
    try:
        tree = ast.parse(src, path)
    except SyntaxError as e:
        return [(path, e.lineno or 0, "E999", str(e))]
    c = _Checker(path, src)
    c.visit(tree)
    c.finish(tree)
    return c.out


def main(argv=None) -> int:
    paths = (argv if argv is not None else sys.argv[1:]) or DEFAULT
    found = []
    for p in _files(paths):
        found += lint_file(p)
    for path, line, code, msg in sorted(found):
        print(f"{os.path.relpath(path, ROOT)}:{line}: {code} {msg}")
    print(f"{len(found)} finding(s)", file=sys.stderr)
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main())
