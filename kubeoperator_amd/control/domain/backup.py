"""Cluster backup / restore: etcd snapshots to S3-compatible / Azure Blob / local storage.

Reference: kubeops_api/cluster_backup_utils.py:12-122, storage_client.py:6-56 (jms_storage for S3/OSS/
Azure), models/backup_storage.py, backup_strategy.py, cluster_backup.py, playbooks cluster-backup.yml /
cluster-restore.yml. The playbook leaves ``<fetch dir>/cluster-backup.zip`` on the controller (fetched
from the first etcd member); it is uploaded as ``<cluster>/<cluster>-<timestamp>.zip``; the daily
strategy job keeps ``save_num`` backups per cluster.

Storage clients are dependency-free: S3 (and S3-compatible OSS / MinIO / Ceph RGW) with AWS Signature V4,
Azure Blob with SharedKey, and LOCAL (a mounted directory, e.g. NFS).
"""
from __future__ import annotations

import base64
import datetime as dt
import hashlib
import hmac
import os
import shutil
import urllib.parse

import httpx
from sqlalchemy import select

from ..conf import get_config
from ..store import models as M
from ..store.db import session_scope
from . import clusters, context


class StorageClient:
    def upload(self, local: str, key: str) -> None: ...
    def download(self, key: str, local: str) -> None: ...
    def exists(self, key: str) -> bool: ...
    def delete(self, key: str) -> None: ...
    def check(self) -> bool: ...
    def list_buckets(self) -> list[str]:
        return []


class LocalStorage(StorageClient):
    def __init__(self, root: str):
        self.root = root

    def _p(self, key):
        return os.path.join(self.root, key)

    def upload(self, local, key):
        os.makedirs(os.path.dirname(self._p(key)), exist_ok=True)
        shutil.copyfile(local, self._p(key))

    def download(self, key, local):
        os.makedirs(os.path.dirname(local) or ".", exist_ok=True)
        shutil.copyfile(self._p(key), local)

    def exists(self, key):
        return os.path.exists(self._p(key))

    def delete(self, key):
        if self.exists(key):
            os.remove(self._p(key))

    def check(self):
        os.makedirs(self.root, exist_ok=True)
        return os.access(self.root, os.W_OK)

    def list_buckets(self):
        return [os.path.basename(self.root)]


class S3Storage(StorageClient):
    """AWS SigV4 over plain HTTP(S); ``endpoint`` makes it work for OSS / MinIO / RGW."""

    def __init__(self, access_key, secret_key, bucket, region="us-east-1", endpoint=None):
        self.ak, self.sk, self.bucket, self.region = access_key, secret_key, bucket, region or "us-east-1"
        self.endpoint = (endpoint or f"https://s3.{self.region}.amazonaws.com").rstrip("/")

    def _sign(self, method, path, query="", payload=b"", headers=None):
        t = dt.datetime.now(dt.timezone.utc)
        amzdate, date = t.strftime("%Y%m%dT%H%M%SZ"), t.strftime("%Y%m%d")
        host = urllib.parse.urlparse(self.endpoint).netloc
        ph = hashlib.sha256(payload).hexdigest()
        h = {"host": host, "x-amz-date": amzdate, "x-amz-content-sha256": ph, **(headers or {})}
        signed = ";".join(sorted(h))
        canon = "\n".join([method, urllib.parse.quote(path), query,
                           "".join(f"{k}:{h[k]}\n" for k in sorted(h)), signed, ph])
        scope = f"{date}/{self.region}/s3/aws4_request"
        sts = "\n".join(["AWS4-HMAC-SHA256", amzdate, scope, hashlib.sha256(canon.encode()).hexdigest()])
        k = ("AWS4" + self.sk).encode()
        for part in (date, self.region, "s3", "aws4_request"):
            k = hmac.new(k, part.encode(), hashlib.sha256).digest()
        sig = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
        h["Authorization"] = f"AWS4-HMAC-SHA256 Credential={self.ak}/{scope}, SignedHeaders={signed}, Signature={sig}"
        return h

    def _req(self, method, key="", payload=b"", query=""):
        path = f"/{self.bucket}/{key}" if key else f"/{self.bucket}"
        url = self.endpoint + urllib.parse.quote(path) + (f"?{query}" if query else "")
        return httpx.request(method, url, content=payload, headers=self._sign(method, path, query, payload),
                             timeout=600)

    def upload(self, local, key):
        with open(local, "rb") as f:
            r = self._req("PUT", key, f.read())
        r.raise_for_status()

    def download(self, key, local):
        r = self._req("GET", key)
        r.raise_for_status()
        with open(local, "wb") as f:
            f.write(r.content)

    def exists(self, key):
        return self._req("HEAD", key).status_code == 200

    def delete(self, key):
        self._req("DELETE", key)

    def check(self):
        try:
            return self._req("HEAD").status_code == 200
        except httpx.HTTPError:
            return False


class AzureStorage(StorageClient):
    def __init__(self, account, key, container, endpoint_suffix="core.windows.net"):
        self.account, self.key, self.container = account, key, container
        self.base = f"https://{account}.blob.{endpoint_suffix}"

    def _headers(self, method, key, length=0, extra=None):
        date = dt.datetime.now(dt.timezone.utc).strftime("%a, %d %b %Y %H:%M:%S GMT")
        h = {"x-ms-date": date, "x-ms-version": "2021-08-06", **(extra or {})}
        canon_h = "".join(f"{k}:{h[k]}\n" for k in sorted(h) if k.startswith("x-ms-"))
        res = f"/{self.account}/{self.container}/{key}"
        sts = "\n".join([method, "", "", str(length) if length else "", "", "", "", "", "", "", "", ""]) + "\n" + canon_h + res
        sig = base64.b64encode(hmac.new(base64.b64decode(self.key), sts.encode(), hashlib.sha256).digest()).decode()
        h["Authorization"] = f"SharedKey {self.account}:{sig}"
        return h

    def upload(self, local, key):
        with open(local, "rb") as f:
            data = f.read()
        r = httpx.put(f"{self.base}/{self.container}/{key}", content=data,
                      headers=self._headers("PUT", key, len(data), {"x-ms-blob-type": "BlockBlob"}), timeout=600)
        r.raise_for_status()

    def download(self, key, local):
        r = httpx.get(f"{self.base}/{self.container}/{key}", headers=self._headers("GET", key), timeout=600)
        r.raise_for_status()
        with open(local, "wb") as f:
            f.write(r.content)

    def exists(self, key):
        return httpx.head(f"{self.base}/{self.container}/{key}", headers=self._headers("HEAD", key)).status_code == 200

    def delete(self, key):
        httpx.delete(f"{self.base}/{self.container}/{key}", headers=self._headers("DELETE", key))

    def check(self):
        try:
            return httpx.get(f"{self.base}/{self.container}?restype=container", timeout=30).status_code < 500
        except httpx.HTTPError:
            return False


def client_for(storage: M.BackupStorage | dict) -> StorageClient:
    d = storage if isinstance(storage, dict) else {"type": storage.type, "credentials": storage.credentials,
                                                  "region": storage.region}
    cred = {k: (context.dec(v) if isinstance(v, str) else v) for k, v in (d.get("credentials") or {}).items()}
    t = (d.get("type") or cred.get("type") or "S3").upper()
    if t == "LOCAL":
        return LocalStorage(cred.get("path") or os.path.join(get_config().data_dir, "backups"))
    if t in ("S3", "OSS", "MINIO"):
        return S3Storage(cred.get("accessKey", ""), cred.get("secretKey", ""), cred.get("bucket", ""),
                         d.get("region") or cred.get("region"), cred.get("endpoint"))
    if t == "AZURE":
        return AzureStorage(cred.get("accountName", ""), cred.get("accountKey", ""), cred.get("bucket", ""),
                            cred.get("endpointSuffix", "core.windows.net"))
    raise ValueError(f"unknown backup storage type {t}")


def backup_file_local(cluster_name: str) -> str:
    return os.path.join(get_config().data_dir, "fetch", cluster_name, "cluster-backup.zip")


def upload_backup(cluster_name: str, storage_id: str, logger=None) -> dict:
    c = clusters.get_cluster(cluster_name)
    with session_scope() as s:
        st = s.get(M.BackupStorage, storage_id)
        if st is None:
            raise clusters.NotFound(f"backup storage {storage_id} not found")
        client = client_for(st)
    local = backup_file_local(cluster_name)
    if not os.path.exists(local):
        raise RuntimeError(f"backup archive {local} was not fetched by the playbook")
    name = f"{cluster_name}-{dt.datetime.now():%Y-%m-%d-%H%M%S}.zip"
    client.upload(local, f"{cluster_name}/{name}")
    if logger:
        logger(f"uploaded {name} ({os.path.getsize(local)} bytes)")
    with session_scope() as s:
        b = M.ClusterBackup(name=name, size=os.path.getsize(local), folder=f"{cluster_name}/", cluster_id=c.id,
                            backup_storage_id=storage_id)
        s.add(b)
        s.flush()
        return b.to_dict()


def download_backup(cluster_name: str, backup_id: str, logger=None) -> str:
    with session_scope() as s:
        b = s.get(M.ClusterBackup, backup_id)
        if b is None:
            raise clusters.NotFound(f"backup {backup_id} not found")
        st = s.get(M.BackupStorage, b.backup_storage_id)
        client, key = client_for(st), f"{cluster_name}/{b.name}"
    if not client.exists(key):
        raise RuntimeError("File is not exist!")
    local = backup_file_local(cluster_name)
    client.download(key, local)
    if logger:
        logger(f"downloaded {key}")
    return local


def apply_retention(cluster_id: str, save_num: int) -> list[str]:
    """Keep the newest ``save_num`` backups (reference cluster_backup(): delete older ones)."""
    removed = []
    with session_scope() as s:
        rows = list(s.scalars(select(M.ClusterBackup).where(M.ClusterBackup.cluster_id == cluster_id)
                              .order_by(M.ClusterBackup.date_created.desc())))
        for b in rows[save_num:]:
            st = s.get(M.BackupStorage, b.backup_storage_id) if b.backup_storage_id else None
            if st is not None:
                try:
                    client_for(st).delete(f"{b.folder}{b.name}")
                except Exception:  # noqa: BLE001
                    pass
            removed.append(b.name)
            s.delete(b)
    return removed


def due_strategies(today: dt.date | None = None) -> list[tuple[str, str, int]]:
    today = today or dt.date.today()
    out = []
    with session_scope() as s:
        for st in s.scalars(select(M.BackupStrategy).where(M.BackupStrategy.status == "ENABLE")):
            c = s.get(M.Cluster, st.cluster_id)
            if c is None or c.status != "RUNNING":
                continue
            last = s.scalar(select(M.ClusterBackup).where(M.ClusterBackup.cluster_id == c.id)
                            .order_by(M.ClusterBackup.date_created.desc()).limit(1))
            if last is None or (today - last.date_created.date()).days >= max(1, st.cron):
                out.append((c.name, st.backup_storage_id, st.save_num))
    return out
