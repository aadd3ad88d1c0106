"""A small Go text/template interpreter, enough to render the bundled Helm charts in tests (no helm binary here).

Covers the subset the charts use: ``{{- ... -}}`` whitespace trimming, comments, ``if / else if / else``,
``range`` over lists and maps (``$k, $v :=``), ``with``, variable declaration ``$x := ...``, field chains on
``.`` / ``$`` / variables, parenthesised sub-pipelines, pipelines (``a | f b``: the value becomes the last
argument), and the functions printf, trunc, trimSuffix, trimPrefix, toYaml, nindent, indent, quote, squote,
int, default, required, eq / ne / lt / le / gt / ge, and / or / not, len, upper / lower. Anything else raises, so
a chart using a construct outside the subset fails its test instead of rendering wrongly.
"""
from __future__ import annotations

import os
import re

import yaml

_ACTION = re.compile(r"\{\{(-?)\s*(.*?)\s*(-?)\}\}", re.S)


class TemplateError(Exception):
    pass


# ------------------------------------------------------------------------------------------------ lexing
def _segments(src: str):
    """[(kind, text)] with kind 'text' / 'action', whitespace trim markers applied."""
    out, pos = [], 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip(" \t\r\n")
        out.append(["text", text])
        out.append(["action", m.group(2), bool(m.group(3))])
        pos = m.end()
    out.append(["text", src[pos:]])
    # right trim: strip the leading whitespace of the text after a "-}}"
    for i, seg in enumerate(out):
        if seg[0] == "action" and seg[2] and i + 1 < len(out):
            out[i + 1][1] = out[i + 1][1].lstrip(" \t\r\n")
    return [(s[0], s[1]) for s in out if not (s[0] == "text" and s[1] == "")]


_TOK = re.compile(r'\s*(?:("(?:[^"\\]|\\.)*")|(`[^`]*`)|(:=|\(|\)|\||,)|([^\s()|,]+))')


def _tokens(expr: str) -> list[str]:
    toks, pos = [], 0
    expr = expr.strip()
    while pos < len(expr):
        m = _TOK.match(expr, pos)
        if not m or m.end() == pos:
            raise TemplateError(f"cannot tokenize {expr[pos:]!r}")
        toks.append(next(g for g in m.groups() if g is not None))
        pos = m.end()
    return toks


# ------------------------------------------------------------------------------------------------ parsing
def _parse(segs):
    """Nested node list: ('text', s) | ('expr', toks) | ('if', [(cond, body)...], else_body) | ('range', ...) |
    ('with', toks, body, else_body)."""
    pos = 0

    def block(stops):
        nonlocal pos
        nodes = []
        while pos < len(segs):
            kind, text = segs[pos]
            if kind == "text":
                nodes.append(("text", text))
                pos += 1
                continue
            if text.startswith("/*"):
                pos += 1
                continue
            word = text.split(None, 1)[0] if text else ""
            if word in stops:
                return nodes, word, text
            pos += 1
            if word == "if":
                branches, else_body = [(_tokens(text[2:]), None)], []
                body, stop, stext = block(("else", "end"))
                branches[-1] = (branches[-1][0], body)
                while stop == "else":
                    pos += 1
                    rest = stext[4:].strip()
                    if rest.startswith("if "):
                        cond = _tokens(rest[3:])
                        body, stop, stext = block(("else", "end"))
                        branches.append((cond, body))
                    else:
                        else_body, stop, stext = block(("end",))
                pos += 1  # end
                nodes.append(("if", branches, else_body))
            elif word in ("range", "with"):
                head = text[len(word):].strip()
                body, stop, _ = block(("else", "end"))
                else_body = []
                if stop == "else":
                    pos += 1
                    else_body, stop, _ = block(("end",))
                pos += 1
                nodes.append((word, head, body, else_body))
            elif word in ("end", "else"):
                raise TemplateError(f"unexpected {{{{ {text} }}}}")
            else:
                nodes.append(("expr", text))
        if stops:
            raise TemplateError(f"missing {{{{ end }}}} (expected one of {stops})")
        return nodes, None, None

    nodes, _, _ = block(())
    return nodes


# ------------------------------------------------------------------------------------------------ evaluation
def _truthy(v) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return True


def _fmt(v) -> str:
    if v is None:
        return "<no value>"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, (dict, list)):
        raise TemplateError(f"cannot print a {type(v).__name__} directly (use toYaml)")
    return str(v)


def _printf(fmt, *args):
    """Go fmt.Sprintf for the verbs charts use: %s %v %d %f %q %%."""
    res, ai, i = [], 0, 0
    for m in re.finditer(r"%([-+ 0#]*\d*(?:\.\d+)?)([svdqf%])", fmt):
        res.append(fmt[i:m.start()])
        i = m.end()
        flags, verb = m.group(1), m.group(2)
        if verb == "%":
            res.append("%")
            continue
        a = args[ai]
        ai += 1
        if verb in ("s", "v"):
            res.append(_fmt(a))
        elif verb == "d":
            res.append(("%" + flags + "d") % int(a))
        elif verb == "f":
            res.append(("%" + flags + "f") % float(a))
        else:  # q
            res.append('"' + str(a).replace('"', '\\"') + '"')
    res.append(fmt[i:])
    return "".join(res)


def _to_yaml(v) -> str:
    if v is None:
        return "null"
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=True).rstrip("\n")


def _indent(n, s):
    return "\n".join((" " * int(n) + line) if line else line for line in str(s).split("\n"))


def _required(msg, v):
    if not _truthy(v):
        raise TemplateError(msg)
    return v


def _num(v):
    return v if isinstance(v, (int, float)) else float(v)


FUNCS = {
    "printf": _printf,
    "trunc": lambda n, s: str(s)[:int(n)],
    "trimSuffix": lambda suf, s: str(s)[:-len(suf)] if suf and str(s).endswith(suf) else str(s),
    "trimPrefix": lambda pre, s: str(s)[len(pre):] if pre and str(s).startswith(pre) else str(s),
    "toYaml": _to_yaml,
    "nindent": lambda n, s: "\n" + _indent(n, s),
    "indent": _indent,
    "quote": lambda *a: " ".join('"' + _fmt(x).replace("\\", "\\\\").replace('"', '\\"') + '"' for x in a),
    "squote": lambda *a: " ".join("'" + _fmt(x) + "'" for x in a),
    "int": lambda v: int(float(v)) if v not in (None, "") else 0,
    "default": lambda d, *v: v[0] if v and _truthy(v[0]) else d,
    "required": _required,
    "eq": lambda a, *b: any(a == x for x in b),
    "ne": lambda a, b: a != b,
    "lt": lambda a, b: _num(a) < _num(b),
    "le": lambda a, b: _num(a) <= _num(b),
    "gt": lambda a, b: _num(a) > _num(b),
    "ge": lambda a, b: _num(a) >= _num(b),
    "and": lambda *a: next((x for x in a if not _truthy(x)), a[-1]),
    "or": lambda *a: next((x for x in a if _truthy(x)), a[-1]),
    "not": lambda a: not _truthy(a),
    "len": lambda a: len(a),
    "upper": lambda s: str(s).upper(),
    "lower": lambda s: str(s).lower(),
}


class _Scope:
    def __init__(self, dot, root, variables):
        self.dot, self.root, self.vars = dot, root, variables


def _field(obj, path: str):
    for part in [p for p in path.split(".") if p]:
        if isinstance(obj, dict):
            obj = obj.get(part)
        else:
            obj = getattr(obj, part, None)
    return obj


def _operand(tok: str, sc: _Scope):
    if tok.startswith('"'):
        return bytes(tok[1:-1], "utf-8").decode("unicode_escape")
    if tok.startswith("`"):
        return tok[1:-1]
    if tok in ("true", "false"):
        return tok == "true"
    if tok == "nil":
        return None
    if re.fullmatch(r"-?\d+", tok):
        return int(tok)
    if re.fullmatch(r"-?\d+\.\d*", tok):
        return float(tok)
    if tok == ".":
        return sc.dot
    if tok.startswith("."):
        return _field(sc.dot, tok)
    if tok.startswith("$"):
        name, _, rest = tok.partition(".")
        if name == "$":
            base = sc.root
        elif name in sc.vars:
            base = sc.vars[name]
        else:
            raise TemplateError(f"undefined variable {name}")
        return _field(base, rest)
    raise TemplateError(f"unknown operand {tok!r}")


def _split_pipe(toks):
    parts, cur, depth = [], [], 0
    for t in toks:
        if t == "(":
            depth += 1
        elif t == ")":
            depth -= 1
        if t == "|" and depth == 0:
            parts.append(cur)
            cur = []
        else:
            cur.append(t)
    parts.append(cur)
    return parts


def _args(toks, sc):
    """Evaluate a token list into argument values (parenthesised groups are sub-pipelines)."""
    vals, i = [], 0
    while i < len(toks):
        t = toks[i]
        if t == "(":
            depth, j = 1, i + 1
            while depth:
                depth += {"(": 1, ")": -1}.get(toks[j], 0)
                j += 1
            vals.append(_pipeline(toks[i + 1:j - 1], sc))
            i = j
        else:
            vals.append(("func", t) if t in FUNCS else ("val", _operand(t, sc)))
            i += 1
    return vals


def _command(toks, sc, piped=None, has_piped=False):
    vals = _args(toks, sc)
    if not vals:
        raise TemplateError("empty command")
    head = vals[0]
    rest = [v[1] if isinstance(v, tuple) else v for v in vals[1:]]
    if has_piped:
        rest.append(piped)
    if isinstance(head, tuple) and head[0] == "func":
        return FUNCS[head[1]](*rest)
    if rest and not has_piped:
        raise TemplateError(f"{toks[0]!r} is not a function")
    return head[1] if isinstance(head, tuple) else head


def _pipeline(toks, sc):
    decl = None
    if len(toks) > 2 and toks[1] == ":=" and toks[0].startswith("$"):
        decl, toks = toks[0], toks[2:]
    val, has = None, False
    for part in _split_pipe(toks):
        val = _command(part, sc, val, has)
        has = True
    if decl:
        sc.vars[decl] = val
        return ""
    return val


def _render(nodes, sc: _Scope, out: list):
    for n in nodes:
        kind = n[0]
        if kind == "text":
            out.append(n[1])
        elif kind == "expr":
            v = _pipeline(_tokens(n[1]), sc)
            if not (isinstance(v, str) and v == "" and ":=" in n[1]):
                out.append(_fmt(v))
        elif kind == "if":
            for cond, body in n[1]:
                if _truthy(_pipeline(cond, sc)):
                    _render(body, sc, out)
                    break
            else:
                _render(n[2], sc, out)
        elif kind == "with":
            v = _pipeline(_tokens(n[1]), sc)
            if _truthy(v):
                _render(n[2], _Scope(v, sc.root, dict(sc.vars)), out)
            else:
                _render(n[3], sc, out)
        elif kind == "range":
            toks = _tokens(n[1])
            kv = []
            if ":=" in toks:
                i = toks.index(":=")
                kv = [t for t in toks[:i] if t != ","]
                toks = toks[i + 1:]
            coll = _pipeline(toks, sc)
            items = sorted(coll.items()) if isinstance(coll, dict) else list(enumerate(coll or []))
            if not items:
                _render(n[3], sc, out)
            for k, v in items:
                inner = _Scope(v, sc.root, dict(sc.vars))
                if len(kv) == 2:
                    inner.vars[kv[0]], inner.vars[kv[1]] = k, v
                elif len(kv) == 1:
                    inner.vars[kv[0]] = v
                _render(n[2], inner, out)


def _merge(base: dict, over: dict) -> dict:
    out = dict(base)
    for k, v in (over or {}).items():
        out[k] = _merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def render_chart(chart_dir: str, values: dict | None = None, release: str = "demo", namespace: str = "default"):
    """{template file name: rendered text} of a chart directory, with ``values`` merged over values.yaml."""
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        vals = yaml.safe_load(f) or {}
    ctx = {"Values": _merge(vals, values or {}),
           "Release": {"Name": release, "Namespace": namespace, "Service": "Helm"},
           "Chart": {"Name": chart["name"], "Version": chart.get("version"), "AppVersion": chart.get("appVersion")}}
    out = {}
    tdir = os.path.join(chart_dir, "templates")
    for name in sorted(os.listdir(tdir)):
        if not name.endswith((".yaml", ".yml", ".tpl")) or name.startswith("_"):
            continue
        with open(os.path.join(tdir, name)) as f:
            nodes = _parse(_segments(f.read()))
        buf: list = []
        _render(nodes, _Scope(ctx, ctx, {}), buf)
        out[name] = "".join(buf)
    return out


def render_docs(chart_dir: str, values: dict | None = None, release: str = "demo") -> list[dict]:
    """Every YAML document the chart renders (empty documents dropped)."""
    docs = []
    for text in render_chart(chart_dir, values, release).values():
        docs += [d for d in yaml.safe_load_all(text) if d]
    return docs
