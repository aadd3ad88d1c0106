"""Job runtime (queue + workers + per-job logs) and periodic scheduler; replaces Celery/Redis/beat."""
from . import jobs, scheduler
from .jobs import JobLogger, WorkerPool, run_inline, submit, tail, task

__all__ = ["jobs", "scheduler", "JobLogger", "WorkerPool", "run_inline", "submit", "tail", "task"]
