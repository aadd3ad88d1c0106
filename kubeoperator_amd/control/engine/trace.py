"""Timing spans of an execution: step -> playbook -> play -> task -> host.

The reference records one ``timedelta`` per execution (``ansible_api/models/mixins.py:74-82``) and Ansible's
per-task ``delta`` inside the callback details (``ansible/callback.py:69-77``); where an install spends its
minutes is not recorded anywhere. Here every level is a span with wall-clock start / end, status and a few
attributes (module, changed, rc). A finished execution's spans are exported

* as Chrome trace-event JSON (``traceEvents``, complete events ``ph: "X"``): one track for the controller
  (steps, playbooks, plays, tasks) and one per host (the module runs), viewable in Perfetto / chrome://tracing;
* as a summary: per step, the slowest tasks and per-host busy time -- what the UI's deploy tab shows;
* as the ``kubeoperator_task_seconds`` histogram (per module and status) on ``/metrics``.
"""
from __future__ import annotations

import itertools
import threading
import time
from dataclasses import dataclass, field


@dataclass
class Span:
    id: int
    name: str
    kind: str  # step | playbook | play | task | host
    parent: int | None
    start: float
    end: float | None = None
    host: str | None = None
    status: str = "running"
    attrs: dict = field(default_factory=dict)

    @property
    def seconds(self) -> float:
        return (self.end if self.end is not None else time.time()) - self.start

    def to_dict(self) -> dict:
        return {"id": self.id, "name": self.name, "kind": self.kind, "parent": self.parent, "start": self.start,
                "end": self.end, "seconds": round(self.seconds, 6), "host": self.host, "status": self.status,
                "attrs": self.attrs}


class Tracer:
    """Thread-safe span recorder. The controller-side spans nest through a stack (the runner is sequential
    at task level); host spans, started from the runner's worker threads, name their task span explicitly."""

    def __init__(self, on_host_span=None):
        self.spans: list[Span] = []
        self._ids = itertools.count(1)
        self._lock = threading.Lock()
        self._stack: list[int] = []
        self._by_id: dict[int, Span] = {}
        self.on_host_span = on_host_span

    def begin(self, name: str, kind: str, host: str | None = None, parent: int | None = None, **attrs) -> int:
        with self._lock:
            sid = next(self._ids)
            if parent is None and kind != "host" and self._stack:
                parent = self._stack[-1]
            sp = Span(sid, str(name), kind, parent, time.time(), host=host, attrs=dict(attrs))
            self.spans.append(sp)
            self._by_id[sid] = sp
            if kind != "host":
                self._stack.append(sid)
            return sid

    def end(self, sid: int, status: str = "ok", **attrs) -> None:
        with self._lock:
            sp = self._by_id[sid]
            sp.end = time.time()
            sp.status = status
            sp.attrs.update(attrs)
            if sp.kind != "host":
                # close anything left open beneath it (an exception unwound the runner)
                while self._stack and self._stack[-1] != sid:
                    inner = self._by_id[self._stack.pop()]
                    if inner.end is None:
                        inner.end, inner.status = sp.end, "aborted"
                if self._stack:
                    self._stack.pop()
        if sp.kind == "host" and self.on_host_span is not None:
            self.on_host_span(sp)

    def current(self) -> int | None:
        with self._lock:
            return self._stack[-1] if self._stack else None

    def span(self, name: str, kind: str, **attrs):
        return _SpanCtx(self, name, kind, attrs)

    # ---------------------------------------------------------------------------------------- exports
    def to_list(self) -> list[dict]:
        with self._lock:
            return [s.to_dict() for s in self.spans]


class _SpanCtx:
    def __init__(self, tracer: Tracer, name: str, kind: str, attrs: dict):
        self.t, self.name, self.kind, self.attrs = tracer, name, kind, attrs
        self.sid = None
        self.status = "ok"

    def __enter__(self):
        self.sid = self.t.begin(self.name, self.kind, **self.attrs)
        return self

    def __exit__(self, et, ev, tb):
        self.t.end(self.sid, "error" if et is not None else self.status)
        return False


def chrome_trace(spans: list[dict], process: str = "execution") -> dict:
    """Chrome trace-event JSON: controller spans on track 0, each host's module runs on its own track."""
    if not spans:
        return {"traceEvents": [], "displayTimeUnit": "ms"}
    t0 = min(s["start"] for s in spans)
    hosts = sorted({s["host"] for s in spans if s["kind"] == "host" and s["host"]})
    tid = {h: i + 1 for i, h in enumerate(hosts)}
    ev = [{"ph": "M", "name": "process_name", "pid": 1, "args": {"name": process}},
          {"ph": "M", "name": "thread_name", "pid": 1, "tid": 0, "args": {"name": "controller"}}]
    ev += [{"ph": "M", "name": "thread_name", "pid": 1, "tid": tid[h], "args": {"name": h}} for h in hosts]
    for s in spans:
        end = s["end"] if s["end"] is not None else s["start"] + s["seconds"]
        ev.append({"name": s["name"], "cat": s["kind"], "ph": "X", "pid": 1,
                   "tid": tid.get(s["host"], 0) if s["kind"] == "host" else 0,
                   "ts": round((s["start"] - t0) * 1e6, 1), "dur": round(max(0.0, end - s["start"]) * 1e6, 1),
                   "args": {"status": s["status"], **s["attrs"]}})
    return {"traceEvents": ev, "displayTimeUnit": "ms"}


def summary(spans: list[dict], top: int = 10) -> dict:
    """Per step: wall seconds, its slowest tasks (wall, slowest host) and per-host busy seconds."""
    by_id = {s["id"]: s for s in spans}

    def ancestor(s, kind):
        while s is not None and s["kind"] != kind:
            s = by_id.get(s["parent"])
        return s

    steps = {}
    order = []
    for s in spans:
        if s["kind"] == "step":
            steps[s["id"]] = {"step": s["name"], "seconds": round(s["seconds"], 3), "status": s["status"],
                              "tasks": [], "hosts": {}}
            order.append(s["id"])
    loose = {"step": "(no step)", "seconds": 0.0, "status": "ok", "tasks": [], "hosts": {}}
    host_spans: dict[int, list] = {}
    for s in spans:
        if s["kind"] == "host":
            host_spans.setdefault(s["parent"], []).append(s)
    for s in spans:
        if s["kind"] == "task":
            st = ancestor(s, "step")
            hs = host_spans.get(s["id"], [])
            slow = max(hs, key=lambda h: h["seconds"], default=None)
            (steps[st["id"]] if st else loose)["tasks"].append(
                {"task": s["name"], "seconds": round(s["seconds"], 3), "hosts": len(hs),
                 "slowest_host": slow["host"] if slow else None,
                 "slowest_host_seconds": round(slow["seconds"], 3) if slow else None})
        elif s["kind"] == "host":
            st = ancestor(s, "step")
            d = (steps[st["id"]] if st else loose)["hosts"]
            d[s["host"]] = round(d.get(s["host"], 0.0) + s["seconds"], 3)
    out = []
    for sid in order + ([None] if loose["tasks"] else []):
        d = steps[sid] if sid is not None else loose
        d["task_count"] = len(d["tasks"])
        d["tasks"] = sorted(d["tasks"], key=lambda x: -x["seconds"])[:top]
        out.append(d)
    return {"steps": out, "total_seconds": round(sum(d["seconds"] for d in out), 3)}
