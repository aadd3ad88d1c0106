"""Domain layer of the control plane: plan, clusters, deploy state machine, hosts & AMD GPU detection,
packages, IaaS providers, backup/restore, storage, monitoring/health/grade, message center, users/RBAC."""
from . import backup, cloud, clusters, context, deploy, hosts, messages, monitor, packages, plan, storage, tasks, users

__all__ = ["backup", "cloud", "clusters", "context", "deploy", "hosts", "messages", "monitor", "packages", "plan",
           "storage", "tasks", "users"]
