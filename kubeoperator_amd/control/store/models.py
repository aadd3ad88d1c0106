"""Persistent data model of the control plane (SQLAlchemy 2 on SQLite/WAL).

Table-for-table re-design of the reference's Django models; field names that the REST
API exposes keep the reference spelling (including ``cluster_doamin_suffix``). Differences by design:
UUID string keys everywhere, JSON columns instead of JSON-in-text fields, secrets stored Fernet-less but
*encrypted* (AES-free XOR stream keyed by SECRET_KEY via HMAC-SHA256 counter mode, see ``crypto.py``)
instead of merely signed, one execution table for every long-running operation, and a job table that
replaces Celery + Redis.

Reference models: ansible_api/models/{project,inventory,playbook,adhoc,mixins}.py,
kubeops_api/models/{cluster,node,host,deploy,package,setting,credential,item,item_resource,
backup_storage,backup_strategy,cluster_backup,cluster_health_history,health_check}.py,
cloud_provider/models.py, storage/models.py, users/models.py, message_center/models.py.
"""
from __future__ import annotations

import datetime as _dt
import uuid

from sqlalchemy import (JSON, Boolean, DateTime, Float, ForeignKey, Index, Integer, String, Text, UniqueConstraint,
                        text)
from sqlalchemy.orm import DeclarativeBase, Mapped, mapped_column


def _uuid() -> str:
    return str(uuid.uuid4())


def now() -> _dt.datetime:
    return _dt.datetime.now(_dt.timezone.utc).replace(tzinfo=None)


class Base(DeclarativeBase):
    type_annotation_map = {dict: JSON, list: JSON}

    def to_dict(self, exclude: tuple = ()) -> dict:
        out = {}
        for c in self.__table__.columns:
            if c.key in exclude:
                continue
            v = getattr(self, c.key)
            if isinstance(v, _dt.datetime):
                v = v.isoformat()
            out[c.key] = v
        return out


class IdMixin:
    id: Mapped[str] = mapped_column(String(36), primary_key=True, default=_uuid)
    date_created: Mapped[_dt.datetime] = mapped_column(DateTime, default=now)


# ------------------------------------------------------------------------------------------- users / RBAC
class User(IdMixin, Base):
    __tablename__ = "users"
    username: Mapped[str] = mapped_column(String(150), unique=True)
    email: Mapped[str] = mapped_column(String(254), default="")
    password_hash: Mapped[str] = mapped_column(String(256), default="")
    is_superuser: Mapped[bool] = mapped_column(Boolean, default=False)
    is_active: Mapped[bool] = mapped_column(Boolean, default=True)
    source: Mapped[str] = mapped_column(String(16), default="local")  # local | ldap (Profile.source)
    notification_config: Mapped[dict] = mapped_column(JSON, default=lambda: {
        "LOCAL": "ENABLE", "EMAIL": "DISABLE", "DINGTALK": "DISABLE", "WORKWEIXIN": "DISABLE"})
    last_login: Mapped[_dt.datetime | None] = mapped_column(DateTime, nullable=True)


class Item(IdMixin, Base):
    """Multi-tenant project ("item") -- reference kubeops_api/models/item.py:8-31."""
    __tablename__ = "items"
    name: Mapped[str] = mapped_column(String(128), unique=True)
    description: Mapped[str] = mapped_column(Text, default="")


class ItemRoleMapping(IdMixin, Base):
    __tablename__ = "item_role_mappings"
    item_id: Mapped[str] = mapped_column(ForeignKey("items.id", ondelete="CASCADE"))
    user_id: Mapped[str] = mapped_column(ForeignKey("users.id", ondelete="CASCADE"))
    role: Mapped[str] = mapped_column(String(16), default="VIEWER")  # VIEWER | MANAGER
    __table_args__ = (UniqueConstraint("item_id", "user_id"),)


class ItemResource(IdMixin, Base):
    __tablename__ = "item_resources"
    item_id: Mapped[str] = mapped_column(ForeignKey("items.id", ondelete="CASCADE"))
    resource_id: Mapped[str] = mapped_column(String(36))
    resource_type: Mapped[str] = mapped_column(String(32))  # CLUSTER HOST PLAN BACKUP_STORAGE STORAGE
    __table_args__ = (UniqueConstraint("resource_id", "resource_type"),)


# ------------------------------------------------------------------------------------------- settings
class Setting(IdMixin, Base):
    __tablename__ = "settings"
    tab: Mapped[str] = mapped_column(String(64), default="system")
    key: Mapped[str] = mapped_column(String(128))
    value: Mapped[str] = mapped_column(Text, default="")
    __table_args__ = (UniqueConstraint("tab", "key"),)


class Credential(IdMixin, Base):
    __tablename__ = "credentials"
    name: Mapped[str] = mapped_column(String(128), unique=True)
    username: Mapped[str] = mapped_column(String(128), default="root")
    password: Mapped[str] = mapped_column(Text, default="")  # encrypted
    private_key: Mapped[str] = mapped_column(Text, default="")  # encrypted
    type: Mapped[str] = mapped_column(String(16), default="password")  # password | privateKey


# ------------------------------------------------------------------------------------------- packages
class Package(IdMixin, Base):
    __tablename__ = "packages"
    name: Mapped[str] = mapped_column(String(64), unique=True)
    meta: Mapped[dict] = mapped_column(JSON, default=dict)
    path: Mapped[str] = mapped_column(Text, default="")


# ------------------------------------------------------------------------------------------- cloud / IaaS
class CloudProviderTemplate(IdMixin, Base):
    __tablename__ = "cloud_provider_templates"
    name: Mapped[str] = mapped_column(String(64), unique=True)
    meta: Mapped[dict] = mapped_column(JSON, default=dict)


class Region(IdMixin, Base):
    __tablename__ = "regions"
    name: Mapped[str] = mapped_column(String(64), unique=True)
    template_id: Mapped[str | None] = mapped_column(ForeignKey("cloud_provider_templates.id"), nullable=True)
    cloud_region: Mapped[str] = mapped_column(String(128), default="")
    vars: Mapped[dict] = mapped_column(JSON, default=dict)
    comment: Mapped[str] = mapped_column(Text, default="")


class Zone(IdMixin, Base):
    __tablename__ = "zones"
    name: Mapped[str] = mapped_column(String(64), unique=True)
    region_id: Mapped[str] = mapped_column(ForeignKey("regions.id", ondelete="CASCADE"))
    cloud_zone: Mapped[str] = mapped_column(String(128), default="")
    vars: Mapped[dict] = mapped_column(JSON, default=dict)  # ip_start, ip_end, net_mask, gateway, dns...
    ip_used: Mapped[list] = mapped_column(JSON, default=list)
    status: Mapped[str] = mapped_column(String(16), default="READY")
    comment: Mapped[str] = mapped_column(Text, default="")


class Plan(IdMixin, Base):
    __tablename__ = "plans"
    name: Mapped[str] = mapped_column(String(64), unique=True)
    region_id: Mapped[str | None] = mapped_column(ForeignKey("regions.id"), nullable=True)
    zone_ids: Mapped[list] = mapped_column(JSON, default=list)
    deploy_template: Mapped[str] = mapped_column(String(32), default="SINGLE")  # SINGLE | MULTIPLE
    vars: Mapped[dict] = mapped_column(JSON, default=dict)  # compute models, worker/master sizes, gpu flags
    comment: Mapped[str] = mapped_column(Text, default="")


# ------------------------------------------------------------------------------------------- hosts
class Host(IdMixin, Base):
    """A registered machine (reference kubeops_api/models/host.py:17-48)."""
    __tablename__ = "hosts"
    name: Mapped[str] = mapped_column(String(128), unique=True)
    ip: Mapped[str] = mapped_column(String(64))
    port: Mapped[int] = mapped_column(Integer, default=22)
    credential_id: Mapped[str | None] = mapped_column(ForeignKey("credentials.id"), nullable=True)
    username: Mapped[str] = mapped_column(String(128), default="root")
    password: Mapped[str] = mapped_column(Text, default="")  # encrypted
    private_key: Mapped[str] = mapped_column(Text, default="")  # encrypted
    memory: Mapped[int] = mapped_column(Integer, default=0)  # MiB
    os: Mapped[str] = mapped_column(String(64), default="")
    os_version: Mapped[str] = mapped_column(String(64), default="")
    cpu_core: Mapped[int] = mapped_column(Integer, default=0)
    volumes: Mapped[list] = mapped_column(JSON, default=list)  # [{name, size}]
    gpus: Mapped[list] = mapped_column(JSON, default=list)  # [{name, vendor, pci, arch, vram_gb}]
    gpu_vendor: Mapped[str] = mapped_column(String(16), default="")  # amd | ""
    zone_id: Mapped[str | None] = mapped_column(ForeignKey("zones.id"), nullable=True)
    status: Mapped[str] = mapped_column(String(16), default="UNKNOWN")  # RUNNING CREATING UNKNOWN UPDATING
    auto_gather_info: Mapped[bool] = mapped_column(Boolean, default=True)
    node_id: Mapped[str | None] = mapped_column(String(36), nullable=True)
    conditions: Mapped[list] = mapped_column(JSON, default=list)
    info: Mapped[dict] = mapped_column(JSON, default=dict)

    @property
    def has_gpu(self) -> bool:
        return bool(self.gpus)

    @property
    def gpu_num(self) -> int:
        return len(self.gpus or [])


# ------------------------------------------------------------------------------------------- projects / inventory
class Project(IdMixin, Base):
    """Ansible-style project (base of clusters and NFS servers): reference ansible_api/models/project.py."""
    __tablename__ = "projects"
    name: Mapped[str] = mapped_column(String(128), unique=True)
    kind: Mapped[str] = mapped_column(String(16), default="cluster")  # cluster | nfs
    options: Mapped[dict] = mapped_column(JSON, default=dict)
    comment: Mapped[str] = mapped_column(Text, default="")
    meta: Mapped[dict] = mapped_column(JSON, default=dict)
    created_by: Mapped[str] = mapped_column(String(128), default="")


class InvHost(IdMixin, Base):
    """Inventory host of a project; a cluster Node (reference ansible_api/models/inventory.py:21-77)."""
    __tablename__ = "inventory_hosts"
    project_id: Mapped[str] = mapped_column(ForeignKey("projects.id", ondelete="CASCADE"))
    name: Mapped[str] = mapped_column(String(256))
    ip: Mapped[str] = mapped_column(String(64), default="")
    port: Mapped[int] = mapped_column(Integer, default=22)
    username: Mapped[str] = mapped_column(String(128), default="root")
    password: Mapped[str] = mapped_column(Text, default="")
    private_key: Mapped[str] = mapped_column(Text, default="")
    vars: Mapped[dict] = mapped_column(JSON, default=dict)
    meta: Mapped[dict] = mapped_column(JSON, default=dict)
    groups: Mapped[list] = mapped_column(JSON, default=list)  # group names
    host_id: Mapped[str | None] = mapped_column(ForeignKey("hosts.id"), nullable=True)  # Node -> Host
    info: Mapped[dict] = mapped_column(JSON, default=dict)
    conditions: Mapped[list] = mapped_column(JSON, default=list)
    __table_args__ = (UniqueConstraint("project_id", "name"),)


class InvGroup(IdMixin, Base):
    """Inventory group ("role") of a project (reference ansible_api/models/inventory.py:168-232)."""
    __tablename__ = "inventory_groups"
    project_id: Mapped[str] = mapped_column(ForeignKey("projects.id", ondelete="CASCADE"))
    name: Mapped[str] = mapped_column(String(128))
    vars: Mapped[dict] = mapped_column(JSON, default=dict)
    children: Mapped[list] = mapped_column(JSON, default=list)
    meta: Mapped[dict] = mapped_column(JSON, default=dict)
    __table_args__ = (UniqueConstraint("project_id", "name"),)


class Playbook(IdMixin, Base):
    __tablename__ = "playbooks"
    project_id: Mapped[str] = mapped_column(ForeignKey("projects.id", ondelete="CASCADE"))
    name: Mapped[str] = mapped_column(String(128))
    alias: Mapped[str] = mapped_column(String(128), default="site.yml")
    type: Mapped[str] = mapped_column(String(16), default="local")  # local | json | git | http
    url: Mapped[str] = mapped_column(Text, default="")
    plays: Mapped[list] = mapped_column(JSON, default=list)  # type=json
    extra_vars: Mapped[dict] = mapped_column(JSON, default=dict)
    __table_args__ = (UniqueConstraint("project_id", "name"),)


# ------------------------------------------------------------------------------------------- clusters
class Cluster(IdMixin, Base):
    """Reference kubeops_api/models/cluster.py:30-432 (the Project row shares the id)."""
    __tablename__ = "clusters"
    project_id: Mapped[str] = mapped_column(ForeignKey("projects.id", ondelete="CASCADE"), unique=True)
    name: Mapped[str] = mapped_column(String(128), unique=True)
    package: Mapped[str] = mapped_column(String(64), default="")
    persistent_storage: Mapped[str] = mapped_column(String(64), default="")
    network_plugin: Mapped[str] = mapped_column(String(64), default="flannel")
    template: Mapped[str] = mapped_column(String(64), default="")
    plan_id: Mapped[str | None] = mapped_column(ForeignKey("plans.id"), nullable=True)
    worker_size: Mapped[int] = mapped_column(Integer, default=3)
    status: Mapped[str] = mapped_column(String(16), default="READY")
    deploy_type: Mapped[str] = mapped_column(String(16), default="MANUAL")  # MANUAL | AUTOMATIC
    configs: Mapped[dict] = mapped_column(JSON, default=dict)
    cluster_doamin_suffix: Mapped[str] = mapped_column(String(256), default="")  # sic, API compatibility
    comment: Mapped[str] = mapped_column(Text, default="")
    upgrade_from: Mapped[str] = mapped_column(String(64), default="")


class Execution(IdMixin, Base):
    """Every long-running operation: DeployExecution, playbook / ad-hoc runs (AbstractExecutionModel)."""
    __tablename__ = "executions"
    kind: Mapped[str] = mapped_column(String(16), default="deploy")  # deploy | playbook | adhoc
    project_id: Mapped[str | None] = mapped_column(ForeignKey("projects.id", ondelete="CASCADE"), nullable=True)
    operation: Mapped[str] = mapped_column(String(64), default="")
    params: Mapped[dict] = mapped_column(JSON, default=dict)
    steps: Mapped[list] = mapped_column(JSON, default=list)
    current_step: Mapped[int] = mapped_column(Integer, default=0)
    state: Mapped[str] = mapped_column(String(16), default="PENDING")  # PENDING STARTED SUCCESS FAILURE RETRY
    num: Mapped[int] = mapped_column(Integer, default=1)
    timedelta: Mapped[float] = mapped_column(Float, default=0.0)
    result_summary: Mapped[dict] = mapped_column(JSON, default=dict)
    result_raw: Mapped[dict] = mapped_column(JSON, default=dict)
    date_start: Mapped[_dt.datetime | None] = mapped_column(DateTime, nullable=True)
    date_end: Mapped[_dt.datetime | None] = mapped_column(DateTime, nullable=True)
    created_by: Mapped[str] = mapped_column(String(128), default="")
    # At most one active (PENDING/STARTED) deploy execution per cluster, enforced by the database itself: a
    # partial unique index (SQLite / PostgreSQL), so no interleaving of two creators can slip a second one in.
    __table_args__ = (Index("uq_one_active_deploy_per_project", "project_id", unique=True,
                            sqlite_where=text("kind = 'deploy' AND state IN ('PENDING', 'STARTED')"),
                            postgresql_where=text("kind = 'deploy' AND state IN ('PENDING', 'STARTED')")),)


# ------------------------------------------------------------------------------------------- backup
class BackupStorage(IdMixin, Base):
    __tablename__ = "backup_storages"
    name: Mapped[str] = mapped_column(String(64), unique=True)
    region: Mapped[str] = mapped_column(String(128), default="")
    credentials: Mapped[dict] = mapped_column(JSON, default=dict)  # type S3/OSS/AZURE/LOCAL + keys (encrypted)
    type: Mapped[str] = mapped_column(String(16), default="S3")
    status: Mapped[str] = mapped_column(String(16), default="VALID")


class BackupStrategy(IdMixin, Base):
    __tablename__ = "backup_strategies"
    cluster_id: Mapped[str] = mapped_column(ForeignKey("clusters.id", ondelete="CASCADE"), unique=True)
    backup_storage_id: Mapped[str | None] = mapped_column(ForeignKey("backup_storages.id"), nullable=True)
    cron: Mapped[int] = mapped_column(Integer, default=1)  # every N days
    save_num: Mapped[int] = mapped_column(Integer, default=7)
    status: Mapped[str] = mapped_column(String(16), default="ENABLE")


class ClusterBackup(IdMixin, Base):
    __tablename__ = "cluster_backups"
    name: Mapped[str] = mapped_column(String(256))
    size: Mapped[int] = mapped_column(Integer, default=0)
    folder: Mapped[str] = mapped_column(Text, default="")
    cluster_id: Mapped[str] = mapped_column(ForeignKey("clusters.id", ondelete="CASCADE"))
    backup_storage_id: Mapped[str | None] = mapped_column(ForeignKey("backup_storages.id"), nullable=True)


class ClusterHealthHistory(IdMixin, Base):
    __tablename__ = "cluster_health_history"
    cluster_id: Mapped[str] = mapped_column(String(36))
    available_rate: Mapped[float] = mapped_column(Float, default=100.0)
    date_type: Mapped[str] = mapped_column(String(8), default="HOUR")  # HOUR | DAY
    month: Mapped[str] = mapped_column(String(8), default="")


# ------------------------------------------------------------------------------------------- storage
class NfsStorage(IdMixin, Base):
    __tablename__ = "nfs_storages"
    project_id: Mapped[str | None] = mapped_column(ForeignKey("projects.id", ondelete="CASCADE"), nullable=True)
    name: Mapped[str] = mapped_column(String(64), unique=True)
    vars: Mapped[dict] = mapped_column(JSON, default=dict)  # storage_nfs_server, path, ...
    status: Mapped[str] = mapped_column(String(16), default="CREATING")


class CephStorage(IdMixin, Base):
    __tablename__ = "ceph_storages"
    name: Mapped[str] = mapped_column(String(64), unique=True)
    vars: Mapped[dict] = mapped_column(JSON, default=dict)


class ClusterCephStorage(IdMixin, Base):
    __tablename__ = "cluster_ceph_storages"
    cluster_id: Mapped[str] = mapped_column(ForeignKey("clusters.id", ondelete="CASCADE"))
    storage_id: Mapped[str] = mapped_column(ForeignKey("ceph_storages.id", ondelete="CASCADE"))


# ------------------------------------------------------------------------------------------- messages
class Message(IdMixin, Base):
    __tablename__ = "messages"
    title: Mapped[str] = mapped_column(String(256))
    sender: Mapped[str] = mapped_column(String(64), default="system")
    content: Mapped[dict] = mapped_column(JSON, default=dict)
    level: Mapped[str] = mapped_column(String(16), default="INFO")  # INFO WARNING ERROR
    type: Mapped[str] = mapped_column(String(16), default="SYSTEM")  # SYSTEM CLUSTER
    item_id: Mapped[str | None] = mapped_column(String(36), nullable=True)


class UserMessage(IdMixin, Base):
    __tablename__ = "user_messages"
    user_id: Mapped[str] = mapped_column(ForeignKey("users.id", ondelete="CASCADE"))
    message_id: Mapped[str] = mapped_column(ForeignKey("messages.id", ondelete="CASCADE"))
    read_status: Mapped[str] = mapped_column(String(16), default="UNREAD")
    send_type: Mapped[str] = mapped_column(String(16), default="LOCAL")  # LOCAL EMAIL DINGTALK WORKWEIXIN
    send_status: Mapped[str] = mapped_column(String(16), default="SUCCESS")
    receive: Mapped[str] = mapped_column(String(256), default="")


class UserReceiver(IdMixin, Base):
    __tablename__ = "user_receivers"
    user_id: Mapped[str] = mapped_column(ForeignKey("users.id", ondelete="CASCADE"), unique=True)
    vars: Mapped[dict] = mapped_column(JSON, default=dict)  # EMAIL, DINGTALK, WORKWEIXIN addresses


class UserNotificationConfig(IdMixin, Base):
    __tablename__ = "user_notification_configs"
    user_id: Mapped[str] = mapped_column(ForeignKey("users.id", ondelete="CASCADE"))
    type: Mapped[str] = mapped_column(String(16), default="SYSTEM")  # SYSTEM | CLUSTER
    vars: Mapped[dict] = mapped_column(JSON, default=dict)
    __table_args__ = (UniqueConstraint("user_id", "type"),)


# ------------------------------------------------------------------------------------------- runtime
class Job(IdMixin, Base):
    """Durable job queue entry (replaces Celery/Redis): reference celery_api + kubeops_api/tasks.py."""
    __tablename__ = "jobs"
    name: Mapped[str] = mapped_column(String(128))
    args: Mapped[dict] = mapped_column(JSON, default=dict)
    state: Mapped[str] = mapped_column(String(16), default="PENDING")  # PENDING STARTED SUCCESS FAILURE
    result: Mapped[dict] = mapped_column(JSON, default=dict)
    worker: Mapped[str] = mapped_column(String(128), default="")
    log_path: Mapped[str] = mapped_column(Text, default="")
    date_start: Mapped[_dt.datetime | None] = mapped_column(DateTime, nullable=True)
    date_end: Mapped[_dt.datetime | None] = mapped_column(DateTime, nullable=True)
    attempts: Mapped[int] = mapped_column(Integer, default=0)


class WorkerHeartbeat(Base):
    """One row per job-worker process (the task monitor's worker list; reference Celery Flower workers view,
    core/kubeops.py:197-213)."""
    __tablename__ = "worker_heartbeats"
    name: Mapped[str] = mapped_column(String(128), primary_key=True)  # host:pid
    hostname: Mapped[str] = mapped_column(String(128), default="")
    pid: Mapped[int] = mapped_column(Integer, default=0)
    concurrency: Mapped[int] = mapped_column(Integer, default=1)
    started: Mapped[_dt.datetime | None] = mapped_column(DateTime, nullable=True)
    last_seen: Mapped[_dt.datetime | None] = mapped_column(DateTime, nullable=True)
    active: Mapped[list] = mapped_column(JSON, default=list)  # job ids running now
    processed: Mapped[int] = mapped_column(Integer, default=0)
    stopped: Mapped[bool] = mapped_column(Boolean, default=False)


class PeriodicTask(IdMixin, Base):
    """Cron-like schedule entry (reference django-celery-beat rows; celery_api/utils.py:59-181)."""
    __tablename__ = "periodic_tasks"
    name: Mapped[str] = mapped_column(String(128), unique=True)
    task: Mapped[str] = mapped_column(String(128))
    args: Mapped[dict] = mapped_column(JSON, default=dict)
    interval_s: Mapped[int] = mapped_column(Integer, default=0)
    crontab: Mapped[str] = mapped_column(String(64), default="")  # "m h * * *"
    enabled: Mapped[bool] = mapped_column(Boolean, default=True)
    last_run: Mapped[_dt.datetime | None] = mapped_column(DateTime, nullable=True)


class SchemaVersion(Base):
    __tablename__ = "schema_version"
    version: Mapped[int] = mapped_column(Integer, primary_key=True)
    applied: Mapped[_dt.datetime] = mapped_column(DateTime, default=now)
