"""Jinja2 templating with the Ansible filter/test subset the provisioning roles use.

Recursive templating of strings inside dicts/lists, "naked" conditional evaluation for ``when`` /
``failed_when`` / ``changed_when`` / ``until``, lazily templated variables (a var whose value is itself a
template is resolved on use, like Ansible's HostVars), and filters: default/d, bool, int, float, string,
lower/upper, length/count, join, split, replace, regex_replace, regex_search, to_json/from_json,
to_yaml/from_yaml, to_nice_yaml, b64encode/b64decode, basename/dirname, ipaddr (address / network /
netmask / prefix / nth host), unique, union, difference, intersect, first/last, min/max, mandatory,
quote, version_compare (+ ``version`` test), dict2items/items2dict, combine, selectattr via Jinja.
"""
from __future__ import annotations

import base64
import ipaddress
import json
import os
import re
import shlex

import jinja2
import yaml
from jinja2 import StrictUndefined
from jinja2.nativetypes import NativeEnvironment


class TemplateError(Exception):
    pass


def _bool(v):
    if isinstance(v, bool):
        return v
    if isinstance(v, (int, float)):
        return v != 0
    return str(v).strip().lower() in ("yes", "on", "1", "true", "y", "t")


def _ver(v):
    parts = re.split(r"[.\-+]", str(v).lstrip("vV"))
    out = []
    for p in parts:
        m = re.match(r"(\d+)(.*)", p)
        out.append((int(m.group(1)), m.group(2)) if m else (-1, p))
    return out


def _version_compare(a, b, op=">=", strict=False):
    a, b = _ver(a), _ver(b)
    n = max(len(a), len(b))
    a += [(0, "")] * (n - len(a))
    b += [(0, "")] * (n - len(b))
    ops = {"<": a < b, "lt": a < b, "<=": a <= b, "le": a <= b, ">": a > b, "gt": a > b, ">=": a >= b,
           "ge": a >= b, "==": a == b, "eq": a == b, "!=": a != b, "ne": a != b}
    return ops[op]


def _ipaddr(value, query=""):
    try:
        if "/" in str(value):
            iface = ipaddress.ip_interface(str(value))
        else:
            iface = ipaddress.ip_interface(str(value) + "/32")
    except ValueError:
        return False
    if query in ("", None):
        return str(value)
    if query == "address":
        return str(iface.ip)
    if query == "network":
        return str(iface.network.network_address)
    if query == "netmask":
        return str(iface.network.netmask)
    if query == "prefix":
        return iface.network.prefixlen
    if query == "broadcast":
        return str(iface.network.broadcast_address)
    if isinstance(query, int) or str(query).isdigit():
        return str(iface.network.network_address + int(query)) + f"/{iface.network.prefixlen}"
    return str(value)


def _regex_replace(s, pattern, repl="", ignorecase=False):
    return re.sub(pattern, repl, str(s), flags=re.I if ignorecase else 0)


def _regex_search(s, pattern, *groups):
    m = re.search(pattern, str(s))
    if not m:
        return None
    if groups:
        return [m.group(int(str(g).lstrip("\\"))) for g in groups]
    return m.group(0)


def _mandatory(v):
    if isinstance(v, jinja2.Undefined):
        raise TemplateError("mandatory variable is undefined")
    return v


def _combine(*dicts, recursive=False):
    out = {}
    for d in dicts:
        if recursive:
            for k, v in d.items():
                if isinstance(v, dict) and isinstance(out.get(k), dict):
                    out[k] = _combine(out[k], v, recursive=True)
                else:
                    out[k] = v
        else:
            out.update(d)
    return out


def _default(value, default_value="", boolean=False):
    if isinstance(value, jinja2.Undefined) or (boolean and not value):
        return default_value
    return value


FILTERS = {
    "default": _default,
    "d": _default,
    "bool": _bool,
    "to_json": lambda v, **k: json.dumps(v, **k),
    "to_nice_json": lambda v, indent=4: json.dumps(v, indent=indent, sort_keys=True),
    "from_json": lambda v: json.loads(v),
    "to_yaml": lambda v, **k: yaml.safe_dump(v, default_flow_style=True).strip(),
    "to_nice_yaml": lambda v, indent=2: yaml.safe_dump(v, default_flow_style=False, indent=indent),
    "from_yaml": lambda v: yaml.safe_load(v),
    "b64encode": lambda v: base64.b64encode(str(v).encode()).decode(),
    "b64decode": lambda v: base64.b64decode(str(v).encode()).decode(),
    "basename": lambda v: os.path.basename(str(v)),
    "dirname": lambda v: os.path.dirname(str(v)),
    "ipaddr": _ipaddr,
    "ipv4": _ipaddr,
    "regex_replace": _regex_replace,
    "regex_search": _regex_search,
    "unique": lambda v: list(dict.fromkeys(v)),
    "union": lambda a, b: list(dict.fromkeys(list(a) + list(b))),
    "difference": lambda a, b: [x for x in a if x not in b],
    "intersect": lambda a, b: [x for x in a if x in b],
    "mandatory": _mandatory,
    "quote": lambda v: shlex.quote(str(v)),
    "version_compare": _version_compare,
    "combine": _combine,
    "dict2items": lambda d: [{"key": k, "value": v} for k, v in d.items()],
    "items2dict": lambda l: {i["key"]: i["value"] for i in l},
    "split": lambda s, sep=None: str(s).split(sep),
    "string": str,
    "type_debug": lambda v: type(v).__name__,
}

TESTS = {
    "version": _version_compare,
    "version_compare": _version_compare,
    "succeeded": lambda r: isinstance(r, dict) and not r.get("failed", False),
    "success": lambda r: isinstance(r, dict) and not r.get("failed", False),
    "failed": lambda r: isinstance(r, dict) and bool(r.get("failed", False)),
    "changed": lambda r: isinstance(r, dict) and bool(r.get("changed", False)),
    "skipped": lambda r: isinstance(r, dict) and bool(r.get("skipped", False)),
    "match": lambda s, p: re.match(p, str(s)) is not None,
    "search": lambda s, p: re.search(p, str(s)) is not None,
    "regex": lambda s, p: re.search(p, str(s)) is not None,
}


class _Undef(jinja2.ChainableUndefined):
    pass


def _make_env(native: bool):
    cls = NativeEnvironment if native else jinja2.Environment
    env = cls(undefined=StrictUndefined, keep_trailing_newline=True, trim_blocks=True, lstrip_blocks=False,
              extensions=["jinja2.ext.do", "jinja2.ext.loopcontrols"])
    env.filters.update(FILTERS)
    env.tests.update(TESTS)
    return env


_ENV_STR = _make_env(False)
_ENV_NATIVE = _make_env(True)


class VarView(dict):
    """Variable mapping whose string values that are templates are rendered lazily on access."""

    def __init__(self, base: dict, depth: int = 0):
        super().__init__(base)
        self._depth = depth

    def __getitem__(self, key):
        v = super().__getitem__(key)
        if isinstance(v, str) and ("{{" in v or "{%" in v) and self._depth < 16:
            return render(v, VarView(dict(self), self._depth + 1))
        return v


def has_template(s) -> bool:
    return isinstance(s, str) and ("{{" in s or "{%" in s)


def render(value, variables: dict):
    """Template a value; strings that are exactly one expression keep their native type."""
    if isinstance(value, str):
        if not has_template(value):
            return value
        ctx = variables if isinstance(variables, VarView) else VarView(variables)
        stripped = value.strip()
        try:
            if stripped.startswith("{{") and stripped.endswith("}}") and stripped.count("{{") == 1:
                out = _ENV_NATIVE.from_string(stripped).render(ctx)
                return out
            return _ENV_STR.from_string(value).render(ctx)
        except jinja2.UndefinedError as e:
            raise TemplateError(f"undefined variable in {value!r}: {e}") from e
        except jinja2.TemplateError as e:
            raise TemplateError(f"template error in {value!r}: {e}") from e
    if isinstance(value, dict):
        return {render(k, variables): render(v, variables) for k, v in value.items()}
    if isinstance(value, list):
        return [render(v, variables) for v in value]
    return value


def render_text(text: str, variables: dict) -> str:
    """Template a whole file (the ``template`` module); always returns text."""
    ctx = variables if isinstance(variables, VarView) else VarView(variables)
    try:
        return _ENV_STR.from_string(text).render(ctx)
    except jinja2.UndefinedError as e:
        raise TemplateError(f"undefined variable in template: {e}") from e
    except jinja2.TemplateError as e:
        raise TemplateError(f"template error: {e}") from e


def evaluate(cond, variables: dict) -> bool:
    """Evaluate a ``when``-style condition (string expression, bool, or list = AND)."""
    if cond is None:
        return True
    if isinstance(cond, bool):
        return cond
    if isinstance(cond, list):
        return all(evaluate(c, variables) for c in cond)
    if isinstance(cond, (int, float)):
        return bool(cond)
    expr = str(cond).strip()
    if has_template(expr) and expr.startswith("{{") and expr.endswith("}}"):
        expr = expr[2:-2]
    ctx = variables if isinstance(variables, VarView) else VarView(variables)
    try:
        out = _ENV_NATIVE.from_string("{{ (" + expr + ") }}").render(ctx)
    except jinja2.UndefinedError as e:
        raise TemplateError(f"undefined variable in condition {cond!r}: {e}") from e
    except jinja2.TemplateError as e:
        raise TemplateError(f"bad condition {cond!r}: {e}") from e
    if isinstance(out, str):
        return _bool(out)
    return bool(out)
