"""Process configuration of the control plane (reference: ``core/apps/kubeoperator/conf.py:31-361``).

Three-tier lookup with the reference's semantics: an UPPERCASE key in ``config.yml`` wins, then an
environment variable of the same name ("true"/"false" coerced to bool), then the built-in default; values
are coerced to the type of the default (so ``HTTP_LISTEN_PORT=9000`` in the environment is an int).

Differences by design: the store is SQLite (WAL) under ``DATA_DIR`` instead of MySQL, the job broker is
the store itself instead of Redis, and there is no Elasticsearch -- system logs and events are JSONL
files searched in-process. ``SECRET_KEY`` is generated and persisted under ``DATA_DIR`` on first start
instead of being committed to the repository.
"""
from __future__ import annotations

import os
import secrets
import threading

import yaml

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
RESOURCE_DIR = os.path.join(PKG_DIR, "resources")

DEFAULTS = {
    "DEBUG": False,
    "LOG_LEVEL": "INFO",
    "DATA_DIR": os.path.join(os.path.expanduser("~"), ".kubeoperator"),
    "DB_URL": "",  # default: sqlite:///<DATA_DIR>/kubeoperator.db
    "SECRET_KEY": "",
    "HTTP_BIND_HOST": "0.0.0.0",
    "HTTP_LISTEN_PORT": 8000,
    "WORKER_CONCURRENCY": 4,  # reference: celery -c 4 (core/kubeops.py:28)
    "ANSIBLE_FORKS": 5,  # reference: forks=5 (ansible_api/ansible/runner.py:39)
    "JWT_EXPIRATION_HOURS": 12,  # reference: settings.py:218-223
    "JWT_AUTH_HEADER_PREFIX": "JWT",
    "DEFAULT_TRANSPORT": "ssh",  # ssh | local | fake
    "PACKAGE_DIR": "",  # default: <DATA_DIR>/packages
    "TERRAFORM_BIN": "terraform",
    "KUBECTL_BIN": "kubectl",
    "ADMIN_PASSWORD": "kubeoperator@admin123",
    "DEFAULT_HOST_USER": "root",
    "DEFAULT_HOST_PASSWORD": "KubeOperator@2019",
    "WEBKUBECTL_URL": "http://webkubectl:8080",
    "MONITOR_INTERVAL_S": 300,
}


class Config(dict):
    def __init__(self, defaults=None, path: str | None = None):
        super().__init__()
        self.defaults = dict(DEFAULTS if defaults is None else defaults)
        self.path = path
        if path and os.path.isfile(path):
            self.load_yaml(path)

    def load_yaml(self, path: str) -> None:
        with open(path) as f:
            data = yaml.safe_load(f) or {}
        for k, v in data.items():
            if str(k).isupper():
                self[k] = v

    def _coerce(self, key, value):
        d = self.defaults.get(key)
        if d is None or value is None:
            return value
        try:
            if isinstance(d, bool):
                if isinstance(value, str):
                    return value.strip().lower() in ("1", "true", "yes", "on")
                return bool(value)
            if isinstance(d, int):
                return int(value)
            if isinstance(d, float):
                return float(value)
        except (TypeError, ValueError):
            return d
        return value

    def __getitem__(self, key):
        v = dict.get(self, key)
        if v is not None:
            return self._coerce(key, v)
        env = os.environ.get(key)
        if env is not None:
            if env.lower() in ("true", "false"):
                return env.lower() == "true"
            return self._coerce(key, env)
        return self.defaults.get(key)

    def get(self, key, default=None):
        v = self[key]
        return default if v is None else v

    def __getattr__(self, item):
        if item.startswith("_") or item in ("defaults", "path"):
            raise AttributeError(item)
        return self[item]

    # derived paths ------------------------------------------------------------------------------
    @property
    def data_dir(self) -> str:
        d = self["DATA_DIR"]
        os.makedirs(d, exist_ok=True)
        return d

    @property
    def db_url(self) -> str:
        return self["DB_URL"] or f"sqlite:///{os.path.join(self.data_dir, 'kubeoperator.db')}"

    @property
    def package_dir(self) -> str:
        d = self["PACKAGE_DIR"] or os.path.join(self.data_dir, "packages")
        os.makedirs(d, exist_ok=True)
        return d

    def secret_key(self) -> str:
        k = self["SECRET_KEY"]
        if k:
            return k
        p = os.path.join(self.data_dir, "secret_key")
        if os.path.exists(p):
            with open(p) as f:
                return f.read().strip()
        k = secrets.token_urlsafe(48)
        with open(p, "w") as f:
            f.write(k)
        os.chmod(p, 0o600)
        return k


_cfg: Config | None = None
_lock = threading.Lock()


def get_config() -> Config:
    global _cfg
    with _lock:
        if _cfg is None:
            path = os.environ.get("KUBEOPERATOR_CONFIG")
            if not path:
                for cand in ("config.yml", "config.yaml"):
                    if os.path.isfile(cand):
                        path = cand
                        break
            _cfg = Config(path=path)
        return _cfg


def set_config(cfg: Config) -> None:
    global _cfg
    with _lock:
        _cfg = cfg
