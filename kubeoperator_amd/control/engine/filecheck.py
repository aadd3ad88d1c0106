"""Structural checks of rendered files before the engine uploads them (``template`` / ``copy content=``).

The reference's roles hand rendered files straight to the tools on the host -- containerd, kubeadm, kubectl
(core/resource/kubeasz/roles/kube-master/tasks/main.yml:1-127) -- and learn about a template typo only when that
command fails halfway through an install. Here every rendered file of a structured type is parsed first, on the
control node, and a broken one fails its template step with the parser's message:

* ``*.toml``: TOML (containerd ``config.toml``, registry ``hosts.toml``);
* ``*.yaml`` / ``*.yml``: every YAML document; documents whose ``apiVersion`` / ``kind`` appear in
  ``resources/schemas/kubernetes_config_keys.yml`` (kubeadm Init / Cluster / Join, Kubelet and KubeProxy
  configuration) are also checked key by key against it -- a misspelt kubeadm key fails here, not in ``kubeadm init``;
* ``*.json``: JSON (Grafana dashboards, CNI configuration).

A task can opt out with ``validate: false`` (payload that only looks structured).
"""
from __future__ import annotations

import functools
import json
import os
import posixpath

import yaml

try:  # Python 3.11+
    import tomllib as _toml
except ModuleNotFoundError:  # pragma: no cover - this image runs 3.10, where tomli is the same parser
    import tomli as _toml


class FileCheckError(ValueError):
    """A rendered file that does not parse, or a configuration document with an unknown key."""


@functools.lru_cache(maxsize=1)
def config_schemas() -> dict:
    from ..conf import RESOURCE_DIR

    with open(os.path.join(RESOURCE_DIR, "schemas", "kubernetes_config_keys.yml")) as f:
        return yaml.safe_load(f)


def _unknown_keys(doc, schema, prefix: str = "") -> list[str]:
    """Dotted paths of keys in ``doc`` that ``schema`` does not allow (``"*"`` allows anything below)."""
    if schema == "*" or not isinstance(schema, dict):
        return []
    if not isinstance(doc, dict):
        return [f"{prefix or '<root>'}: expected a mapping, got {type(doc).__name__}"]
    bad = []
    for k, v in doc.items():
        path = f"{prefix}.{k}" if prefix else str(k)
        if k not in schema:
            bad.append(path)
        else:
            bad += _unknown_keys(v, schema[k], path)
    return bad


def check_config_document(doc: dict) -> None:
    """Key check of one Kubernetes component-configuration document (no-op for kinds without a schema)."""
    if not isinstance(doc, dict):
        return
    api, kind = doc.get("apiVersion"), doc.get("kind")
    schemas = config_schemas()
    if api in schemas:
        if kind not in schemas[api]:
            raise FileCheckError(f"{api}: unknown kind {kind!r} (known: {', '.join(sorted(schemas[api]))})")
        bad = _unknown_keys(doc, schemas[api][kind])
        if bad:
            raise FileCheckError(f"{api} {kind}: unknown key(s) {', '.join(bad)}")


def check(path: str, data: bytes) -> str | None:
    """Parse ``data`` as the type ``path`` names; returns the type checked (None: not a structured type) or raises
    ``FileCheckError`` naming the file and the problem."""
    name = posixpath.basename(path).lower()
    try:
        if name.endswith(".toml"):
            _toml.loads(data.decode())
            return "toml"
        if name.endswith((".yaml", ".yml")):
            for doc in yaml.safe_load_all(data.decode()):
                check_config_document(doc)
            return "yaml"
        if name.endswith(".json"):
            json.loads(data.decode())
            return "json"
    except FileCheckError as e:
        raise FileCheckError(f"{path}: {e}") from None
    except (UnicodeDecodeError, ValueError, yaml.YAMLError) as e:  # tomllib / json errors are ValueErrors
        raise FileCheckError(f"{path}: {type(e).__name__}: {e}") from None
    return None
