"""Render the charts under ``helm-charts/`` without the helm binary.

    python tools/helm_lite.py helm-charts/seldon-abtest --name my-ab [--namespace ns] [--set a.b=c ...]

Implements the subset of Go templates the charts use -- and the charts keep
to it, so ``helm template`` and this renderer produce the same documents:

* ``{{ .Values.a.b }}``, ``{{ .Release.Name }}``, ``{{ .Release.Namespace }}``,
  ``{{ .Chart.Name }}``, ``{{ .Chart.Version }}``, ``{{ $var }}`` / ``{{ $var.field }}``
* ``{{ .Files.Get "files/x" }}`` (a file of the chart), pipelines ``| toJson``,
  ``| quote``, ``| default <literal>``, ``| indent N``, ``| nindent N``
* ``{{ if X }} ... {{ else }} ... {{ end }}`` (X: a path, ``not`` path, or
  ``eq`` path "literal"), ``{{ range $k, $v := X }}``, ``{{ range $v := X }}``
* ``{{-`` / ``-}}`` whitespace trimming and ``{{/* comments */}}``.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
from typing import Any, Dict, List, Optional, Tuple

import yaml

TOKEN = re.compile(r"\{\{(-?)\s*(.*?)\s*(-?)\}\}", re.S)


def _tokens(src: str) -> List[Tuple[str, str]]:
    out: List[Tuple[str, str]] = []
    pos = 0
    for m in TOKEN.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip()
        if out and out[-1][0] == "trim_next":
            out.pop()
            text = text.lstrip()
        out.append(("text", text))
        body = m.group(2)
        if not body.startswith("/*"):
            out.append(("action", body))
        if m.group(3):
            out.append(("trim_next", ""))
        pos = m.end()
    text = src[pos:]
    if out and out[-1][0] == "trim_next":
        out.pop()
        text = text.lstrip()
    out.append(("text", text))
    return out


def _parse(tokens: List[Tuple[str, str]], i: int = 0, stop=("end",)) -> Tuple[List, int, str]:
    nodes: List = []
    while i < len(tokens):
        kind, val = tokens[i]
        if kind == "text":
            nodes.append(("text", val))
            i += 1
            continue
        head = val.split()[0] if val.split() else ""
        if head in stop:
            return nodes, i + 1, head
        if head == "if":
            body, i, end = _parse(tokens, i + 1, ("else", "end"))
            other: List = []
            if end == "else":
                other, i, _ = _parse(tokens, i, ("end",))
            nodes.append(("if", val[2:].strip(), body, other))
        elif head == "range":
            body, i, _ = _parse(tokens, i + 1, ("end",))
            nodes.append(("range", val[5:].strip(), body))
        else:
            nodes.append(("expr", val))
            i += 1
    return nodes, i, ""


def _lookup(path: str, ctx: Dict[str, Any]) -> Any:
    if path.startswith("$"):
        name, _, rest = path.partition(".")
        cur = ctx["vars"].get(name)
    else:
        cur, rest = ctx["root"], path.lstrip(".")
    for part in filter(None, rest.split(".")):
        cur = cur.get(part) if isinstance(cur, dict) else None
    return cur


def _literal(tok: str) -> Any:
    if tok.startswith('"'):
        return json.loads(tok)
    try:
        return json.loads(tok)
    except ValueError:
        return tok


def _value(expr: str, ctx: Dict[str, Any]) -> Any:
    stages = [s.strip() for s in expr.split("|")]
    head = stages[0].split()
    if head[0] == ".Files.Get":
        with open(os.path.join(ctx["root"]["_chart_dir"], _literal(head[1]))) as f:
            v = f.read()
    elif head[0] == "not":
        v = not _truthy(_lookup(head[1], ctx))
    elif head[0] == "eq":
        a = _lookup(head[1], ctx) if head[1].startswith((".", "$")) else _literal(head[1])
        v = a == _literal(head[2])
    elif head[0].startswith((".", "$")):
        v = _lookup(head[0], ctx)
    else:
        v = _literal(head[0])
    for st in stages[1:]:
        fn, *args = st.split(None, 1)
        if fn == "toJson":
            v = json.dumps(v, separators=(",", ":"))
        elif fn == "quote":
            v = json.dumps("" if v is None else str(v))
        elif fn == "default":
            if not _truthy(v):
                v = _literal(args[0])
        elif fn in ("indent", "nindent"):
            pad = " " * int(args[0])
            v = "\n".join(pad + ln if ln else ln for ln in _str(v).split("\n"))
            if fn == "nindent":
                v = "\n" + v
        else:
            raise ValueError(f"helm_lite: unsupported function {fn!r}")
    return v


def _truthy(v: Any) -> bool:
    return v not in (None, False, 0, "", [], {})


def _str(v: Any) -> str:
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def _render(nodes: List, ctx: Dict[str, Any]) -> str:
    out = []
    for n in nodes:
        if n[0] == "text":
            out.append(n[1])
        elif n[0] == "expr":
            out.append(_str(_value(n[1], ctx)))
        elif n[0] == "if":
            out.append(_render(n[2] if _truthy(_value(n[1], ctx)) else n[3], ctx))
        elif n[0] == "range":
            lhs, _, src = n[1].partition(":=")
            names = [x.strip() for x in lhs.split(",")]
            coll = _value(src.strip(), ctx) or []
            items = sorted(coll.items()) if isinstance(coll, dict) else list(enumerate(coll))
            for k, v in items:
                vars_ = dict(ctx["vars"])
                if len(names) == 2:
                    vars_[names[0]], vars_[names[1]] = k, v
                else:
                    vars_[names[0]] = v
                out.append(_render(n[2], {**ctx, "vars": vars_}))
    return "".join(out)


def _set(values: Dict, dotted: str, raw: str) -> None:
    cur = values
    parts = dotted.split(".")
    for p in parts[:-1]:
        cur = cur.setdefault(p, {})
    cur[parts[-1]] = yaml.safe_load(raw)


def _merge(a: Dict, b: Dict) -> Dict:
    out = dict(a)
    for k, v in b.items():
        out[k] = _merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def render_chart(chart_dir: str, name: str, namespace: str = "default", values: Optional[Dict] = None,
                 sets: Optional[List[str]] = None) -> List[Dict]:
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        vals = yaml.safe_load(f) or {}
    vals = _merge(vals, values or {})
    for s in sets or []:
        k, _, v = s.partition("=")
        _set(vals, k, v)
    root = {"Values": vals, "Release": {"Name": name, "Namespace": namespace},
            "Chart": {"Name": chart.get("name"), "Version": chart.get("version")}, "_chart_dir": chart_dir}
    docs: List[Dict] = []
    tdir = os.path.join(chart_dir, "templates")
    for fn in sorted(os.listdir(tdir)):
        if fn.startswith("_") or not fn.endswith((".yaml", ".json")):
            continue
        with open(os.path.join(tdir, fn)) as f:
            nodes, _, _ = _parse(_tokens(f.read()))
        text = _render(nodes, {"root": root, "vars": {}})
        for d in yaml.safe_load_all(text):
            if d:
                docs.append(d)
    return docs


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="helm_lite")
    ap.add_argument("chart")
    ap.add_argument("--name", default="release")
    ap.add_argument("--namespace", default="default")
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args(argv)
    sys.stdout.write(yaml.safe_dump_all(render_chart(a.chart, a.name, a.namespace, sets=a.set), sort_keys=False))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
