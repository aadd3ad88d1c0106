"""Jinja2 templating with the Ansible filter/test subset the provisioning roles use.

Recursive templating of strings inside dicts/lists, "naked" conditional evaluation for ``when`` /
``failed_when`` / ``changed_when`` / ``until``, lazily templated variables (a var whose value is itself a
template is resolved on use through a custom Jinja context, like Ansible's HostVars; recursion is bounded),
a sandboxed environment (API-supplied config values cannot reach Python internals), and filters: default/d, bool, int, float, string,
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
import threading

import jinja2
import yaml
from jinja2 import StrictUndefined
from jinja2.nativetypes import NativeCodeGenerator, NativeTemplate, native_concat
from jinja2.runtime import Context, missing
from jinja2.sandbox import ImmutableSandboxedEnvironment, SecurityError


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
    for d in map(_data, dicts):
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


def _data(v):
    """Plain data for serialising filters: lazily bound dicts / lists become dicts / lists of expanded values."""
    if isinstance(v, Unsafe):
        return str.__str__(v)
    if isinstance(v, dict):
        return {_data(k): _data(v[k]) for k in v.keys()}
    if isinstance(v, (list, tuple)):
        return [_data(x) for x in v]
    return v


FILTERS = {
    "default": _default,
    "d": _default,
    "bool": _bool,
    "to_json": lambda v, **k: json.dumps(_data(v), **k),
    "to_nice_json": lambda v, indent=4: json.dumps(_data(v), indent=indent, sort_keys=True),
    "from_json": lambda v: json.loads(v),
    "to_yaml": lambda v, **k: yaml.safe_dump(_data(v), default_flow_style=True).strip(),
    "to_nice_yaml": lambda v, indent=2: yaml.safe_dump(_data(v), default_flow_style=False, indent=indent),
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


class TemplateRecursionError(TemplateError):
    pass


class Unsafe(str):
    """A string that is data, never a template (Ansible's ``!unsafe``): user content such as Helm values
    is wrapped in it so ``{{ ... }}`` inside it is written out literally instead of being evaluated."""


def mark_unsafe(value):
    """Recursively wrap the strings of a JSON-like value in :class:`Unsafe`."""
    if isinstance(value, str):
        return Unsafe(value)
    if isinstance(value, dict):
        return {mark_unsafe(k): mark_unsafe(v) for k, v in value.items()}
    if isinstance(value, (list, tuple)):
        return [mark_unsafe(v) for v in value]
    return value


_MAX_DEPTH = 16
_tls = threading.local()


def _expand(value, root):
    """Resolve a variable's value on use: a string that is itself a template is rendered against ``root``
    (Ansible templates variables lazily, so role defaults may reference inventory / extra vars), and a dict
    is wrapped so its templated members resolve the same way when they are looked up."""
    if isinstance(value, str):
        if not has_template(value):
            return value
        depth = getattr(_tls, "depth", 0)
        if depth >= _MAX_DEPTH:
            raise TemplateRecursionError(f"recursive loop detected in template string: {value!r}")
        _tls.depth = depth + 1
        try:
            return render(value, root)
        finally:
            _tls.depth = depth
    if type(value) is dict:
        return _BoundVars(value, root)
    if isinstance(value, list) and any(has_template(x) for x in value):
        return [_expand(x, root) for x in value]
    return value


class _BoundVars(dict):
    """A dict-valued variable whose templated members render against the enclosing variable set."""

    def __init__(self, base: dict, root):
        super().__init__(base)
        self._root = root

    def __getitem__(self, key):
        return _expand(super().__getitem__(key), self._root)

    def get(self, key, default=None):
        return self[key] if key in self else default

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def values(self):
        return [self[k] for k in self.keys()]


class LazyVars(_BoundVars):
    """A variable set (e.g. one host's ``hostvars`` entry) whose templated values render against itself."""

    def __init__(self, base: dict):
        super().__init__(base, None)
        self._root = self


class _LazyContext(Context):
    def resolve_or_missing(self, key):
        v = super().resolve_or_missing(key)
        if v is missing:
            return v
        return _expand(v, self.parent)


class _SandboxedNativeEnvironment(ImmutableSandboxedEnvironment):
    """Sandboxed environment whose single-expression renders keep their Python type."""

    code_generator_class = NativeCodeGenerator
    concat = staticmethod(native_concat)


_SandboxedNativeEnvironment.template_class = NativeTemplate


class _ChainableStrictUndefined(StrictUndefined):
    """Strict, but attribute / item access on an undefined value yields another undefined (Ansible's
    AnsibleUndefined behaviour): ``reg.stdout_lines | default([])`` works when ``reg`` was never registered
    (its task was skipped), while printing, iterating or comparing an undefined still raises."""

    __slots__ = ()

    def __getattr__(self, name):
        if name[:2] == "__":
            raise AttributeError(name)
        return _ChainableStrictUndefined(name=f"{self._undefined_name}.{name}" if self._undefined_name else name)

    def __getitem__(self, key):
        return _ChainableStrictUndefined(name=f"{self._undefined_name}[{key!r}]")


def _make_env(native: bool):
    # Sandboxed: cluster configs and execution params come from API users (item MANAGERs) and are merged
    # into the variables, so a template must not reach Python internals (attribute walks to globals, etc.).
    cls = _SandboxedNativeEnvironment if native else ImmutableSandboxedEnvironment
    env = cls(undefined=_ChainableStrictUndefined, keep_trailing_newline=True, trim_blocks=True, lstrip_blocks=False,
              extensions=["jinja2.ext.do", "jinja2.ext.loopcontrols"])
    env.context_class = _LazyContext
    env.filters.update(FILTERS)
    env.tests.update(TESTS)
    return env


_ENV_STR = _make_env(False)
_ENV_NATIVE = _make_env(True)


def _plain(variables) -> dict:
    return variables if isinstance(variables, dict) else dict(variables)


def has_template(s) -> bool:
    return isinstance(s, str) and not isinstance(s, Unsafe) and ("{{" in s or "{%" in s)


def render(value, variables: dict):
    """Template a value; strings that are exactly one expression keep their native type."""
    if isinstance(value, str):
        if not has_template(value):
            return value
        ctx = _plain(variables)
        stripped = value.strip()
        try:
            if stripped.startswith("{{") and stripped.endswith("}}") and stripped.count("{{") == 1:
                out = _ENV_NATIVE.from_string(stripped).render(ctx)
                return out
            return _ENV_STR.from_string(value).render(ctx)
        except TemplateError:
            raise
        except SecurityError as e:
            raise TemplateError(f"unsafe template {value!r}: {e}") from e
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
    try:
        return _ENV_STR.from_string(text).render(_plain(variables))
    except TemplateError:
        raise
    except SecurityError as e:
        raise TemplateError(f"unsafe template: {e}") from e
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
    try:
        out = _ENV_NATIVE.from_string("{{ (" + expr + ") }}").render(_plain(variables))
    except TemplateError:
        raise
    except SecurityError as e:
        raise TemplateError(f"unsafe condition {cond!r}: {e}") from e
    except jinja2.UndefinedError as e:
        raise TemplateError(f"undefined variable in condition {cond!r}: {e}") from e
    except jinja2.TemplateError as e:
        raise TemplateError(f"bad condition {cond!r}: {e}") from e
    if isinstance(out, str):
        return _bool(out)
    return bool(out)
