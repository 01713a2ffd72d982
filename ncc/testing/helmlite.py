"""A small Go text/template + Sprig interpreter: renders this repository's Helm chart without `helm`.

`helm template` is not available where the test suite runs (no network, no Go toolchain), yet the chart
in deploy/helm/nexus-configuration-controller has logic worth pinning — the leader-election branches,
`dig` defaults, the health port taken apart with `splitList`, the three ClusterRoles built from a
`range` over `dict`s.  This module implements the subset of the template language the chart uses, with
Go's semantics where they matter:

* actions `{{ }}` with trim markers `{{-` / `-}}`, comments `{{/* */}}`;
* `if` / `else if` / `else`, `with` / `else`, `range` (with `$v :=` / `$i, $v :=`), `define`, `end`;
* pipelines `a | f b` (the piped value is the last argument), parenthesised sub-pipelines,
  variables (`$`, `$x := ...`, `$x.field`), fields (`.Values.a.b`), string/number/bool literals;
* Go truthiness (false, 0, nil, "" and empty collections are false);
* functions: include, tpl-free Sprig subset — default, dig, quote, squote, toYaml, toJson, nindent,
  indent, trunc, trimSuffix, trimPrefix, replace, printf, contains, hasPrefix, list, dict, index, last,
  first, splitList, join, int, toString, lower, upper, trim, eq, ne, lt, gt, not, and, or, empty,
  required, fail, ternary, len.

`render_chart(chart_dir, values_overrides, release=...)` returns {template file name: rendered text},
like `helm template` (values.yaml deep-merged with the overrides; `.Chart`, `.Release`, `.Values`).
tests/test_helm_chart.py renders the chart in several configurations and parses every document.
`.github/workflows/ci.yaml` also runs the real `helm lint` / `helm template` there.
"""
from __future__ import annotations

import copy
import json
import os
import re

import yaml

__all__ = ["render", "render_chart", "TemplateError"]


class TemplateError(Exception):
    pass


# ------------------------------------------------------------------------------------------- lexing
_ACTION = re.compile(r"\{\{(-\s)?(.*?)(\s-)?\}\}", re.S)


def _split(src: str) -> list:
    """[("text", s) | ("action", s)] with trim markers applied to the neighbouring text."""
    out = []
    pos = 0
    trim_next = False
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if trim_next:
            text = text.lstrip(" \t\r\n")
        if m.group(1):
            text = text.rstrip(" \t\r\n")
        if text:
            out.append(("text", text))
        body = m.group(2).strip()
        if not (body.startswith("/*") and body.endswith("*/")):
            out.append(("action", body))
        trim_next = bool(m.group(3))
        pos = m.end()
    text = src[pos:]
    if trim_next:
        text = text.lstrip(" \t\r\n")
    if text:
        out.append(("text", text))
    return out


_TOKEN = re.compile(r"""
    (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<raw>`[^`]*`)
  | (?P<decl>:=)
  | (?P<assign>=)
  | (?P<num>-?\d+(?:\.\d+)?)
  | (?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)
  | (?P<field>(?:\.[A-Za-z0-9_]+)+|\.)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<lp>\()
  | (?P<rp>\))
  | (?P<pipe>\|)
  | (?P<comma>,)
  | (?P<ws>\s+)
""", re.X)


def _tokens(s: str) -> list:
    out = []
    pos = 0
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if m is None:
            raise TemplateError(f"cannot parse {s[pos:pos + 30]!r} in action {{{{ {s} }}}}")
        kind = m.lastgroup
        if kind != "ws":
            out.append((kind, m.group()))
        pos = m.end()
    return out


# ------------------------------------------------------------------------------------------- parsing
class _Node:
    __slots__ = ("kind", "a", "b", "c", "d")

    def __init__(self, kind, a=None, b=None, c=None, d=None):
        self.kind, self.a, self.b, self.c, self.d = kind, a, b, c, d


def _parse(items: list, defines: dict) -> list:
    pos = 0

    def block(stop: tuple) -> tuple:
        nonlocal pos
        body = []
        while pos < len(items):
            kind, s = items[pos]
            if kind == "text":
                body.append(_Node("text", s))
                pos += 1
                continue
            word = s.split(None, 1)[0] if s else ""
            if word in stop or (word == "else" and "else" in stop):
                return body, s
            pos += 1
            rest = s[len(word):].strip()
            if word == "if":
                body.append(cond_chain("if", rest))
            elif word == "with":
                then, term = block(("end", "else"))
                other = None
                if term.startswith("else"):
                    pos += 1
                    other, _ = block(("end",))
                pos += 1
                body.append(_Node("with", rest, then, other))
            elif word == "range":
                then, term = block(("end", "else"))
                other = None
                if term.startswith("else"):
                    pos += 1
                    other, _ = block(("end",))
                pos += 1
                body.append(_Node("range", rest, then, other))
            elif word == "define":
                name = json.loads(rest)
                inner, _ = block(("end",))
                pos += 1
                defines[name] = inner
            else:
                body.append(_Node("action", s))
        if stop:
            raise TemplateError(f"missing {{{{ end }}}} (looking for {stop})")
        return body, ""

    def cond_chain(kind: str, expr: str) -> _Node:
        nonlocal pos
        then, term = block(("end", "else"))
        other = None
        if term.startswith("else"):
            pos += 1
            rest = term[4:].strip()
            if rest.startswith("if "):
                return _Node(kind, expr, then, [cond_chain("if", rest[3:].strip())])
            other, _ = block(("end",))
            pos += 1
            return _Node(kind, expr, then, other)
        pos += 1
        return _Node(kind, expr, then, other)

    body, _ = block(())
    return body


# ------------------------------------------------------------------------------------------- values
def _truthy(v) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, tuple, dict)):
        return len(v) > 0
    return True


def _to_string(v) -> str:
    if v is None:
        return ""
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, (dict, list)):
        return _go_print(v)
    return str(v)


def _go_print(v) -> str:
    """fmt's %v of maps and slices (only used for odd debugging output)."""
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{_go_print(v[k])}" for k in sorted(v)) + "]"
    if isinstance(v, list):
        return "[" + " ".join(_go_print(x) for x in v) + "]"
    return _to_string(v)


def _go_quote(s: str) -> str:
    return json.dumps(s, ensure_ascii=False)


def _to_yaml(v) -> str:
    if v is None:
        return "null"
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=True, allow_unicode=True).rstrip("\n")


def _indent(n, s) -> str:
    pad = " " * int(n)
    return "\n".join(pad + line for line in _to_string(s).split("\n"))


def _printf(fmt, *args) -> str:
    out, i = [], 0
    parts = re.split(r"(%[-+# 0]*\d*(?:\.\d+)?[sdvqtf%])", fmt)
    for p in parts:
        if not p.startswith("%") or len(p) < 2:
            out.append(p)
            continue
        verb = p[-1]
        if verb == "%":
            out.append("%")
            continue
        a = args[i] if i < len(args) else None
        i += 1
        if verb == "q":
            out.append(_go_quote(_to_string(a)))
        elif verb == "d":
            out.append(str(int(a)))
        else:
            out.append(_to_string(a))
    return "".join(out)


def _dig(*args):
    *keys, default, d = args
    cur = d
    for k in keys:
        if not isinstance(cur, dict) or k not in cur:
            return default
        cur = cur[k]
    return cur


def _index(coll, *keys):
    cur = coll
    for k in keys:
        if isinstance(cur, dict):
            cur = cur.get(k)
        elif isinstance(cur, (list, tuple)):
            cur = cur[int(k)]
        else:
            raise TemplateError(f"index of {type(cur).__name__}")
    return cur


def _required(msg, v):
    if v is None or v == "":
        raise TemplateError(msg)
    return v


def _fail(msg):
    raise TemplateError(msg)


_FUNCS = {
    "default": lambda d, *v: v[0] if v and _truthy(v[0]) else d,
    "dig": _dig,
    "quote": lambda *a: " ".join(_go_quote(_to_string(x)) for x in a if x is not None),
    "squote": lambda *a: " ".join("'" + _to_string(x) + "'" for x in a if x is not None),
    "toYaml": _to_yaml,
    "toJson": lambda v: json.dumps(v, separators=(",", ":"), ensure_ascii=False),
    "nindent": lambda n, s: "\n" + _indent(n, s),
    "indent": _indent,
    "trunc": lambda n, s: _to_string(s)[:int(n)] if int(n) >= 0 else _to_string(s)[int(n):],
    "trimSuffix": lambda suf, s: _to_string(s)[:-len(suf)] if suf and _to_string(s).endswith(suf) else _to_string(s),
    "trimPrefix": lambda pre, s: _to_string(s)[len(pre):] if pre and _to_string(s).startswith(pre) else _to_string(s),
    "trim": lambda s: _to_string(s).strip(),
    "lower": lambda s: _to_string(s).lower(),
    "upper": lambda s: _to_string(s).upper(),
    "replace": lambda old, new, s: _to_string(s).replace(old, new),
    "printf": _printf,
    "contains": lambda sub, s: _to_string(sub) in _to_string(s),
    "hasPrefix": lambda pre, s: _to_string(s).startswith(_to_string(pre)),
    "list": lambda *a: list(a),
    "dict": lambda *a: {_to_string(a[i]): (a[i + 1] if i + 1 < len(a) else "") for i in range(0, len(a), 2)},
    "index": _index,
    "last": lambda l: l[-1] if l else None,
    "first": lambda l: l[0] if l else None,
    "splitList": lambda sep, s: _to_string(s).split(sep),
    "join": lambda sep, l: sep.join(_to_string(x) for x in l),
    "int": lambda v: int(float(v)) if _to_string(v).strip() not in ("", "None") else 0,
    "toString": _to_string,
    "eq": lambda a, *b: any(a == x for x in b),
    "ne": lambda a, b: a != b,
    "lt": lambda a, b: a < b,
    "gt": lambda a, b: a > b,
    "not": lambda v: not _truthy(v),
    "and": lambda *a: next((x for x in a if not _truthy(x)), a[-1]),
    "or": lambda *a: next((x for x in a if _truthy(x)), a[-1]),
    "empty": lambda v: not _truthy(v),
    "required": _required,
    "fail": _fail,
    "ternary": lambda a, b, c: a if _truthy(c) else b,
    "len": lambda v: len(v) if v is not None else 0,
}


# ------------------------------------------------------------------------------------------- evaluation
class _Scope:
    def __init__(self, root, parent=None):
        self.vars = {"$": root} if parent is None else {}
        self.parent = parent

    def get(self, name):
        s = self
        while s is not None:
            if name in s.vars:
                return s.vars[name]
            s = s.parent
        raise TemplateError(f"undefined variable {name}")

    def set(self, name, v, declare: bool):
        if declare:
            self.vars[name] = v
            return
        s = self
        while s is not None:
            if name in s.vars:
                s.vars[name] = v
                return
            s = s.parent
        raise TemplateError(f"assignment to undeclared variable {name}")


def _field(v, path: list):
    for p in path:
        if isinstance(v, dict):
            v = v.get(p)
        elif v is None:
            return None
        else:
            v = getattr(v, p, None)
    return v


class _Renderer:
    def __init__(self, defines: dict):
        self.defines = defines
        self.depth = 0

    def render(self, nodes, dot, scope) -> str:
        out = []
        for n in nodes:
            k = n.kind
            if k == "text":
                out.append(n.a)
            elif k == "action":
                v = self.pipeline(n.a, dot, scope, allow_decl=True)
                if v is not _NOTHING:
                    out.append(_to_string(v))
            elif k == "if":
                if _truthy(self.pipeline(n.a, dot, scope)):
                    out.append(self.render(n.b, dot, _Scope(None, scope)))
                elif n.c is not None:
                    out.append(self.render(n.c, dot, _Scope(None, scope)))
            elif k == "with":
                v = self.pipeline(n.a, dot, scope)
                if _truthy(v):
                    out.append(self.render(n.b, v, _Scope(None, scope)))
                elif n.c is not None:
                    out.append(self.render(n.c, dot, _Scope(None, scope)))
            elif k == "range":
                out.append(self.range(n, dot, scope))
        return "".join(out)

    def range(self, n, dot, scope) -> str:
        expr = n.a
        names = []
        m = re.match(r"^(\$\w*)(?:\s*,\s*(\$\w*))?\s*:=\s*(.*)$", expr, re.S)
        if m:
            names = [x for x in (m.group(1), m.group(2)) if x]
            expr = m.group(3)
        coll = self.pipeline(expr, dot, scope)
        if not _truthy(coll):
            return self.render(n.c, dot, _Scope(None, scope)) if n.c is not None else ""
        pairs = sorted(coll.items()) if isinstance(coll, dict) else list(enumerate(coll))
        out = []
        for key, val in pairs:
            s = _Scope(None, scope)
            if len(names) == 1:
                s.vars[names[0]] = val
            elif len(names) == 2:
                s.vars[names[0]], s.vars[names[1]] = key, val
            out.append(self.render(n.b, val, s))
        return "".join(out)

    def include(self, name, dot) -> str:
        body = self.defines.get(name)
        if body is None:
            raise TemplateError(f"no template {name!r}")
        self.depth += 1
        if self.depth > 100:
            raise TemplateError("include nesting too deep")
        try:
            return self.render(body, dot, _Scope(dot))
        finally:
            self.depth -= 1

    # -- expressions
    def pipeline(self, expr: str, dot, scope, allow_decl: bool = False):
        toks = _tokens(expr)
        if len(toks) >= 2 and toks[0][0] == "var" and toks[1][0] in ("decl", "assign"):
            if not allow_decl and toks[1][0] == "decl":
                raise TemplateError(f"declaration not allowed here: {expr}")
            v = self._pipe(toks[2:], dot, scope)
            scope.set(toks[0][1], v, toks[1][0] == "decl")
            return _NOTHING
        return self._pipe(toks, dot, scope)

    def _pipe(self, toks, dot, scope):
        cmds, cur, depth = [], [], 0
        for t in toks:
            if t[0] == "lp":
                depth += 1
            elif t[0] == "rp":
                depth -= 1
            if t[0] == "pipe" and depth == 0:
                cmds.append(cur)
                cur = []
            else:
                cur.append(t)
        cmds.append(cur)
        val = _NOTHING
        for c in cmds:
            val = self._command(c, dot, scope, val)
        return val

    def _args(self, toks, dot, scope) -> list:
        out, i = [], 0
        while i < len(toks):
            t = toks[i]
            if t[0] == "lp":
                depth, j = 1, i + 1
                while depth:
                    if toks[j][0] == "lp":
                        depth += 1
                    elif toks[j][0] == "rp":
                        depth -= 1
                    j += 1
                out.append(self._pipe(toks[i + 1:j - 1], dot, scope))
                i = j
                continue
            out.append(self._operand(t, dot, scope))
            i += 1
        return out

    def _operand(self, t, dot, scope):
        kind, s = t
        if kind == "str":
            return json.loads(s)
        if kind == "raw":
            return s[1:-1]
        if kind == "num":
            return float(s) if "." in s else int(s)
        if kind == "field":
            return dot if s == "." else _field(dot, s[1:].split("."))
        if kind == "var":
            name, *path = s.split(".")
            return _field(scope.get(name), path)
        if kind == "ident":
            if s in ("true", "false"):
                return s == "true"
            if s == "nil":
                return None
            return _Func(s)
        raise TemplateError(f"unexpected token {s!r}")

    def _command(self, toks, dot, scope, piped):
        if not toks:
            raise TemplateError("empty command")
        head = toks[0]
        if head[0] == "lp":  # a parenthesised pipeline used as a value
            vals = self._args(toks, dot, scope)
            if len(vals) != 1 or piped is not _NOTHING:
                raise TemplateError("a parenthesised value takes no arguments")
            return vals[0]
        args = self._args(toks[1:], dot, scope)
        if piped is not _NOTHING:
            args.append(piped)
        if head[0] == "ident" and head[1] not in ("true", "false", "nil"):
            name = head[1]
            if name == "include":
                return self.include(args[0], args[1] if len(args) > 1 else None)
            fn = _FUNCS.get(name)
            if fn is None:
                raise TemplateError(f"function {name!r} not supported")
            return fn(*args)
        if args:
            raise TemplateError(f"{head[1]} is not a function")
        return self._operand(head, dot, scope)


class _Func(str):
    pass


_NOTHING = object()


# ------------------------------------------------------------------------------------------- API
def render(templates: dict, values: dict, chart: dict | None = None, release: dict | None = None) -> dict:
    """Render {name: source} templates; files starting with `_` only contribute `define`s."""
    defines: dict = {}
    parsed = {name: _parse(_split(src), defines) for name, src in sorted(templates.items())}
    chart = chart or {}
    root = {
        "Values": values,
        "Chart": {"Name": chart.get("name", ""), "Version": chart.get("version", ""),
                  "AppVersion": chart.get("appVersion", "")},
        "Release": {"Name": "release-name", "Namespace": "default", "Service": "Helm", "IsInstall": True,
                    **(release or {})},
        "Capabilities": {"KubeVersion": {"Version": "v1.33.0"}},
    }
    r = _Renderer(defines)
    return {name: r.render(nodes, root, _Scope(root)) for name, nodes in parsed.items()
            if not os.path.basename(name).startswith("_")}


def _merge(base: dict, over: dict) -> dict:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def render_chart(chart_dir: str, overrides: dict | None = None, release: dict | None = None) -> dict:
    """`helm template` of a chart directory: {template file name: rendered text}."""
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        values = yaml.safe_load(f) or {}
    tdir = os.path.join(chart_dir, "templates")
    templates = {}
    for fn in sorted(os.listdir(tdir)):
        if fn.endswith((".yaml", ".yml", ".tpl")):
            with open(os.path.join(tdir, fn)) as f:
                templates[fn] = f.read()
    return render(templates, _merge(values, overrides or {}), chart, release)
