"""REST ``/api/v1`` + WebSocket API of the control plane (replaces the reference's Django REST Framework
views and Channels consumers; route table in SURVEY.md §1.1, reference ``core/apps/kubeoperator/urls.py:23-50``,
``kubeops_api/api_url.py``, ``kubeops_api/api.py``, ``users/urls.py``, ``celery_api/urls``,
``cloud_provider/api.py``, ``storage/api.py``, ``message_center/api_url.py``, ``log/api.py``).

Compatibility contract kept from the reference:
* auth header ``Authorization: JWT <token>`` (``Bearer`` accepted too), tokens from ``POST token/auth/``,
  ``POST token/refresh/`` (12 h expiry, 7 day refresh window);
* resource paths and trailing slashes, lookup fields (clusters by ``name``, packages by ``name``, configs by
  ``key``), the ``cluster_doamin_suffix`` field spelling, deploy execution body ``{operation, params}``;
* item-based RBAC: non-superusers only see resources of their items; cluster deletion and operations need the
  MANAGER role (reference ``api.py:49-73``, ``apis/item.py``);
* list endpoints answer a plain JSON list, or the DRF page shape ``{count, next, previous, results}`` when
  ``?page=`` / ``?limit=`` is given (reference host list is paginated).

The app is a plain ASGI application (FastAPI/Starlette); ``server.py`` serves it (HTTP + WebSocket) without
uvicorn's optional websocket dependencies. Blocking domain calls run in Starlette's thread pool.
"""
from __future__ import annotations

import asyncio
import datetime as dt
import json
import os
import time
from typing import Any

from fastapi import APIRouter, Depends, FastAPI, Request, WebSocket, WebSocketDisconnect
from fastapi.responses import FileResponse, JSONResponse, PlainTextResponse, RedirectResponse, Response
from sqlalchemy import select

from ... import __version__
from ..conf import get_config
from ..domain import backup, cloud, clusters, deploy, hosts, messages, monitor, packages, plan, storage, users
from ..domain import context
from ..domain.users import AuthError, Forbidden
from ..runtime import jobs
from ..store import models as M
from ..store.db import session_scope

API = "/api/v1"
UI_DIR = os.path.join(os.path.dirname(os.path.dirname(__file__)), "ui")


def _is_ipv4(v: str) -> bool:
    import ipaddress

    try:
        return isinstance(ipaddress.ip_address(v), ipaddress.IPv4Address)
    except ValueError:
        return False


class HTTPError(Exception):
    def __init__(self, status: int, detail: Any):
        self.status, self.detail = status, detail


# ------------------------------------------------------------------------------------------------ helpers
def _auth_token(headers) -> str | None:
    h = headers.get("authorization") or ""
    prefix = str(get_config()["JWT_AUTH_HEADER_PREFIX"])
    for p in (prefix, "Bearer", "JWT"):
        if h.startswith(p + " "):
            return h[len(p) + 1:].strip()
    return None


def current_user(request: Request) -> M.User:
    tok = _auth_token(request.headers) or request.query_params.get("token")
    if not tok:
        raise HTTPError(401, "Authentication credentials were not provided.")
    try:
        return users.user_from_token(tok)
    except AuthError as e:
        raise HTTPError(401, str(e)) from e


def superuser(request: Request) -> M.User:
    u = current_user(request)
    if not u.is_superuser:
        raise HTTPError(403, "You do not have permission to perform this action.")
    return u


async def raw_body(request: Request) -> bytes:
    return await request.body()


async def body(request: Request) -> dict:
    """The request's JSON (or form) payload. Handlers take it as a ``Depends(body)`` parameter and are plain
    ``def`` functions, so FastAPI runs their blocking store / SSH / password-hash work in its thread pool
    instead of on the event loop that serves every websocket."""
    raw = await request.body()
    if not raw:
        return {}
    ctype = request.headers.get("content-type", "")
    if "application/x-www-form-urlencoded" in ctype:
        from urllib.parse import parse_qsl

        return dict(parse_qsl(raw.decode()))
    try:
        data = json.loads(raw)
    except ValueError as e:
        raise HTTPError(400, f"JSON parse error: {e}") from e
    if not isinstance(data, (dict, list)):
        raise HTTPError(400, "expected a JSON object")
    return data


def parse_multipart(ctype: str, raw: bytes) -> dict[str, tuple[str | None, bytes]]:
    """Minimal multipart/form-data parser (python-multipart is not available): name -> (filename, data)."""
    bnd = None
    for part in ctype.split(";"):
        part = part.strip()
        if part.startswith("boundary="):
            bnd = part[9:].strip('"')
    if not bnd:
        raise HTTPError(400, "multipart boundary missing")
    out = {}
    for chunk in raw.split(b"--" + bnd.encode()):
        chunk = chunk.strip(b"\r\n")
        if not chunk or chunk == b"--":
            continue
        head, _, data = chunk.partition(b"\r\n\r\n")
        disp = {}
        for line in head.decode(errors="replace").split("\r\n"):
            if line.lower().startswith("content-disposition:"):
                for kv in line.split(";")[1:]:
                    k, _, v = kv.strip().partition("=")
                    disp[k] = v.strip('"')
        if "name" in disp:
            out[disp["name"]] = (disp.get("filename"), data)
    return out


def paginate(request: Request, rows: list) -> Any:
    q = request.query_params
    if "page" not in q and "limit" not in q:
        return rows
    if "page" in q:
        size = int(q.get("size") or q.get("page_size") or 10)
        page = max(1, int(q["page"]))
        off = (page - 1) * size
    else:
        size, off = int(q["limit"]), int(q.get("offset", 0))
    nxt = off + size < len(rows)
    return {"count": len(rows), "next": nxt or None, "previous": off > 0 or None, "results": rows[off:off + size]}


def _visible(user: M.User, rtype: str, rows: list[dict], key: str = "id") -> list[dict]:
    ids = users.visible_resources(user, rtype)
    return rows if ids is None else [r for r in rows if r[key] in ids]


def _cluster_for(user: M.User, name: str, manage: bool = False) -> M.Cluster:
    c = clusters.get_cluster(name)
    ids = users.visible_resources(user, "CLUSTER")
    if ids is not None and c.id not in ids:
        raise HTTPError(404, f"cluster {name} not found")
    if manage:
        users.require_manager(user, c.id, "CLUSTER")
    return c


def _scrub(d: dict, *secret_keys) -> dict:
    for k in secret_keys:
        if k in d:
            d[k] = ""
    return d


def _row(model, rid: str) -> M.Base:
    with session_scope() as s:
        r = s.get(model, rid)
        if r is None:
            r = s.scalar(select(model).where(model.name == rid)) if hasattr(model, "name") else None
        if r is None:
            raise HTTPError(404, f"{model.__name__} {rid} not found")
        return r


# ------------------------------------------------------------------------------------------------ generic CRUD
def crud(router: APIRouter, path: str, model, rtype: str | None = None, secrets: tuple = (), encrypt: tuple = (),
         admin_write: bool = True, on_create=None, on_delete=None, to_dict=None, paginated: bool = False):
    """list/create on ``path`` and retrieve/update/delete on ``path/<id or name>/`` (DRF ModelViewSet shape)."""
    cols = {c.name for c in model.__table__.columns} - {"id", "date_created"}
    render = to_dict or (lambda r: _scrub(r.to_dict(), *secrets))

    def _apply(row, data):
        for k, v in data.items():
            if k in cols:
                if k in encrypt:
                    if v in (None, ""):
                        continue
                    v = context.enc(v) if isinstance(v, str) else {kk: context.enc(vv) if isinstance(vv, str) else vv
                                                                   for kk, vv in v.items()}
                setattr(row, k, v)

    @router.get(path)
    def _list(request: Request):
        u = current_user(request)
        with session_scope() as s:
            rows = [render(r) for r in s.scalars(select(model).order_by(model.date_created))]
        if rtype:
            rows = _visible(u, rtype, rows)
        return paginate(request, rows) if paginated or "page" in request.query_params else rows

    @router.post(path, status_code=201)
    def _create(request: Request, data: dict = Depends(body)):
        u = superuser(request) if admin_write else current_user(request)
        with session_scope() as s:
            if "name" in cols and data.get("name") and s.scalar(select(model).where(model.name == data["name"])):
                raise HTTPError(400, {"name": [f"{model.__name__} with this name already exists."]})
            row = model()
            _apply(row, data)
            s.add(row)
            s.flush()
            rid = row.id
        if on_create:
            on_create(rid, data, u)
        if rtype and data.get("item_name"):
            users.add_item_resources(data["item_name"], rtype, [rid])
        return render(_row(model, rid))

    @router.get(path + "{rid}/")
    def _get(rid: str, request: Request):
        current_user(request)
        return render(_row(model, rid))

    def _update(rid: str, request: Request, data: dict = Depends(body)):
        superuser(request) if admin_write else current_user(request)
        r = _row(model, rid)
        with session_scope() as s:
            row = s.get(model, r.id)
            _apply(row, data)
        return render(_row(model, r.id))

    router.put(path + "{rid}/")(_update)
    router.patch(path + "{rid}/")(_update)

    @router.delete(path + "{rid}/", status_code=204)
    def _delete(rid: str, request: Request):
        superuser(request) if admin_write else current_user(request)
        r = _row(model, rid)
        if on_delete:
            on_delete(r)
        with session_scope() as s:
            s.delete(s.get(model, r.id))
            s.query(M.ItemResource).filter(M.ItemResource.resource_id == r.id).delete()
        return Response(status_code=204)


# ------------------------------------------------------------------------------------------------ app
def create_app() -> FastAPI:
    # FastAPI's own /docs pages load swagger-ui from a CDN and render blank offline: the API explorer here is one
    # self-contained page (api/explorer.html, no external assets), served where the reference serves its schema
    # views (kubeoperator/urls.py:44-47): /swagger/, /docs/, /redoc/, plus the raw schema at /docs.json, /docs.yaml
    app = FastAPI(title="KubeOperator-AMD", version=__version__, docs_url=None, redoc_url=None,
                  openapi_url="/swagger.json")
    r = APIRouter(prefix=API)

    explorer = os.path.join(os.path.dirname(os.path.abspath(__file__)), "explorer.html")

    def _explorer():
        with open(explorer) as f:
            return Response(f.read(), media_type="text/html")

    for _p in ("/swagger/", "/docs/", "/redoc/"):
        app.get(_p, include_in_schema=False)(_explorer)

    @app.get("/docs.json", include_in_schema=False)
    def docs_json():
        return JSONResponse(app.openapi())

    @app.get("/docs.yaml", include_in_schema=False)
    def docs_yaml():
        import yaml

        return Response(yaml.safe_dump(app.openapi(), sort_keys=False), media_type="application/yaml")

    @app.exception_handler(HTTPError)
    async def _h1(_, e: HTTPError):
        return JSONResponse({"detail": e.detail} if not isinstance(e.detail, dict) else e.detail, status_code=e.status)

    @app.exception_handler(clusters.NotFound)
    async def _h2(_, e):
        return JSONResponse({"detail": str(e)}, status_code=404)

    @app.exception_handler(clusters.Conflict)
    async def _h3(_, e):
        return JSONResponse({"detail": str(e)}, status_code=400)

    @app.exception_handler(AuthError)
    async def _h4(_, e):
        return JSONResponse({"detail": str(e)}, status_code=401)

    @app.exception_handler(Forbidden)
    async def _h5(_, e):
        return JSONResponse({"detail": str(e)}, status_code=403)

    @app.exception_handler(ValueError)
    async def _h6(_, e):
        return JSONResponse({"detail": str(e)}, status_code=400)

    @app.exception_handler(KeyError)
    async def _h7(_, e):
        return JSONResponse({"detail": f"missing field {e}"}, status_code=400)

    # ------------------------------------------------------------------ users / auth (users/urls.py:13-23)
    @r.post("/token/auth/")
    def token_auth(request: Request, d: dict = Depends(body)):
        return users.authenticate(d.get("username", ""), d.get("password", ""))

    @r.post("/token/refresh/")
    def token_refresh(request: Request, d: dict = Depends(body)):
        return users.refresh(d.get("token", ""))

    @r.get("/profile/")
    def my_profile(request: Request):
        return users.profile(current_user(request))

    @r.put("/profile/")
    def update_profile(request: Request, d: dict = Depends(body)):
        u = current_user(request)
        with session_scope() as s:
            row = s.get(M.User, u.id)
            if "email" in d:
                row.email = d["email"]
            if "notification_config" in d:
                row.notification_config = d["notification_config"]
        return users.profile(_row(M.User, u.id))

    @r.put("/password/")
    def change_password(request: Request, d: dict = Depends(body)):
        u = current_user(request)
        users.set_password(u.id, d.get("original"), d["password"])
        return {"msg": "ok"}

    @r.get("/users/")
    def list_users(request: Request):
        current_user(request)
        with session_scope() as s:
            rows = list(s.scalars(select(M.User).order_by(M.User.date_created)))
        return paginate(request, [users.profile(u) for u in rows])

    @r.post("/users/", status_code=201)
    def create_user(request: Request, d: dict = Depends(body)):
        superuser(request)
        return users.create_user(d["username"], d.get("password", ""), d.get("email", ""),
                                 bool(d.get("is_superuser", False)))

    @r.get("/users/{uid}/")
    def get_user(uid: str, request: Request):
        current_user(request)
        return users.profile(_user(uid))

    @r.put("/users/{uid}/")
    @r.patch("/users/{uid}/")
    def update_user(uid: str, request: Request, d: dict = Depends(body)):
        superuser(request)
        u = _user(uid)
        with session_scope() as s:
            row = s.get(M.User, u.id)
            for k in ("email", "is_superuser", "is_active"):
                if k in d:
                    setattr(row, k, d[k])
        if d.get("password"):
            users.set_password(u.id, None, d["password"], check_original=False)
        return users.profile(_user(u.id))

    @r.delete("/users/{uid}/", status_code=204)
    def delete_user(uid: str, request: Request):
        me = superuser(request)
        u = _user(uid)
        if u.id == me.id or u.username == "admin":
            raise HTTPError(400, "cannot delete yourself or the admin user")
        with session_scope() as s:
            s.delete(s.get(M.User, u.id))
        return Response(status_code=204)

    @r.post("/users/sync/")
    def users_sync(request: Request):
        superuser(request)
        return {"job_id": jobs.submit("sync_ldap_users", {})}

    @r.get("/profiles/")
    def list_profiles(request: Request):
        current_user(request)
        with session_scope() as s:
            rows = list(s.scalars(select(M.User)))
        return [users.profile(u) for u in rows]

    @r.get("/version/")
    def version():
        return {"version": __version__, "arch": "gfx950", "accelerator": "AMD Instinct MI355X"}

    # ------------------------------------------------------------------ clusters (kubeops_api/api.py:42-255)
    @r.get("/clusters/")
    def list_clusters(request: Request):
        u = current_user(request)
        with session_scope() as s:
            rows = list(s.scalars(select(M.Cluster).order_by(M.Cluster.date_created)))
        data = _visible(u, "CLUSTER", [clusters.cluster_dict(c) for c in rows])
        item = request.query_params.get("item")
        if item:
            data = [c for c in data if c.get("item_name") == item]
        return paginate(request, data)

    @r.post("/clusters/", status_code=201)
    def create_cluster(request: Request, d: dict = Depends(body)):
        u = current_user(request)
        if not u.is_superuser:
            item = d.get("item_name")
            with session_scope() as s:
                it = s.scalar(select(M.Item).where(M.Item.name == item)) if item else None
            if it is None or users.role_in(u, it.id) != "MANAGER":
                raise HTTPError(403, "creating a cluster requires the MANAGER role of its item")
        out = clusters.create_cluster(d, created_by=u.username)
        for n in d.get("nodes") or []:
            clusters.add_node(d["name"], n)
        return clusters.cluster_dict(clusters.get_cluster(out["id"]))

    @r.get("/clusters/{name}/")
    def get_cluster(name: str, request: Request):
        return clusters.cluster_dict(_cluster_for(current_user(request), name))

    @r.patch("/clusters/{name}/")
    @r.put("/clusters/{name}/")
    def update_cluster(name: str, request: Request, d: dict = Depends(body)):
        c = _cluster_for(current_user(request), name, manage=True)
        with session_scope() as s:
            row = s.get(M.Cluster, c.id)
            for k in ("comment", "worker_size", "persistent_storage", "cluster_doamin_suffix"):
                if k in d:
                    setattr(row, k, d[k])
        return clusters.cluster_dict(clusters.get_cluster(c.id))

    @r.delete("/clusters/{name}/", status_code=204)
    def delete_cluster(name: str, request: Request):
        u = current_user(request)
        c = _cluster_for(u, name, manage=True)
        if c.status not in ("READY", "ERROR") and not u.is_superuser:
            raise HTTPError(400, f"cluster is {c.status}; uninstall it first")
        clusters.delete_cluster(c.name, force=u.is_superuser)
        monitor.delete_cluster_data(c.name)
        return Response(status_code=204)

    @r.get("/clusters/{name}/configs/")
    def list_configs(name: str, request: Request):
        c = _cluster_for(current_user(request), name)
        return [{"key": k, "value": v} for k, v in (c.configs or {}).items()]

    @r.post("/clusters/{name}/configs/", status_code=201)
    def set_config(name: str, request: Request, d: dict = Depends(body)):
        c = _cluster_for(current_user(request), name, manage=True)
        clusters.set_config(c.name, d["key"], d.get("value"))
        return {"key": d["key"], "value": d.get("value")}

    @r.get("/clusters/{name}/configs/{key}/")
    def get_config_key(name: str, key: str, request: Request):
        c = _cluster_for(current_user(request), name)
        if key not in (c.configs or {}):
            raise HTTPError(404, f"config {key} not set")
        return {"key": key, "value": c.configs[key]}

    @r.put("/clusters/{name}/configs/{key}/")
    def put_config_key(name: str, key: str, request: Request, d: dict = Depends(body)):
        c = _cluster_for(current_user(request), name, manage=True)
        clusters.set_config(c.name, key, d.get("value"))
        return {"key": key, "value": d.get("value")}

    @r.delete("/clusters/{name}/configs/{key}/", status_code=204)
    def del_config_key(name: str, key: str, request: Request):
        c = _cluster_for(current_user(request), name, manage=True)
        clusters.del_config(c.name, key)
        return Response(status_code=204)

    @r.get("/clusters/{name}/nodes/")
    def list_nodes(name: str, request: Request):
        c = _cluster_for(current_user(request), name)
        return paginate(request, clusters.list_nodes(c.name))

    @r.post("/clusters/{name}/nodes/", status_code=201)
    def add_node(name: str, request: Request, _data: dict = Depends(body)):
        c = _cluster_for(current_user(request), name, manage=True)
        return clusters.add_node(c.name, _data)

    @r.get("/clusters/{name}/nodes/{node}/")
    def get_node(name: str, node: str, request: Request):
        c = _cluster_for(current_user(request), name)
        for n in clusters.list_nodes(c.name):
            if n["name"] == node or n["id"] == node:
                return n
        raise HTTPError(404, f"node {node} not found")

    @r.delete("/clusters/{name}/nodes/{node}/", status_code=204)
    def delete_node(name: str, node: str, request: Request):
        c = _cluster_for(current_user(request), name, manage=True)
        clusters.remove_node_record(c.name, node)
        return Response(status_code=204)

    @r.get("/clusters/{name}/roles/")
    def list_roles(name: str, request: Request):
        c = _cluster_for(current_user(request), name)
        inv = context.project_inventory(c.project_id)
        return [{"name": g, "vars": inv.groups[g].vars, "children": inv.groups[g].children,
                 "hosts": inv.group_hosts(g)} for g in inv.groups if g not in ("all", "ungrouped")]

    @r.get("/clusters/{name}/roles/{role}/")
    def get_role(name: str, role: str, request: Request):
        for g in list_roles(name, request):
            if g["name"] == role:
                return g
        raise HTTPError(404, f"role {role} not found")

    @r.get("/clusters/{name}/executions/")
    def list_executions(name: str, request: Request):
        c = _cluster_for(current_user(request), name)
        with session_scope() as s:
            rows = list(s.scalars(select(M.Execution).where(M.Execution.project_id == c.project_id,
                                                            M.Execution.kind == "deploy")
                                  .order_by(M.Execution.date_created.desc())))
        return paginate(request, [_exec_dict(e) for e in rows])

    @r.post("/clusters/{name}/executions/", status_code=201)
    def create_execution(name: str, request: Request, d: dict = Depends(body)):
        u = current_user(request)
        c = _cluster_for(u, name, manage=True)
        return deploy.create(c.name, d.get("operation", ""), d.get("params") or {}, user=u.username)

    def _own_execution(name: str, eid: str, request: Request):
        """The execution, only through the cluster it belongs to (no reading other clusters' runs by id)."""
        c = _cluster_for(current_user(request), name)
        with session_scope() as s:
            e = s.get(M.Execution, eid)
            if e is None or e.project_id != c.project_id:
                raise HTTPError(404, f"execution {eid} not found in cluster {name}")
        return c

    @r.get("/clusters/{name}/executions/{eid}/")
    def get_execution(name: str, eid: str, request: Request):
        _own_execution(name, eid, request)
        return deploy.get(eid)

    @r.get("/clusters/{name}/executions/{eid}/trace/")
    def get_execution_trace(name: str, eid: str, request: Request, view: str = "chrome"):
        """Timing spans of the execution: ``view=chrome`` (trace-event JSON for Perfetto / chrome://tracing),
        ``summary`` (per step: slowest tasks, per-host busy time) or ``spans``."""
        _own_execution(name, eid, request)
        if view not in ("chrome", "summary", "spans"):
            raise HTTPError(400, "view must be chrome, summary or spans")
        return deploy.get_trace(eid, view)

    @r.get("/clusters/{name}/apps/")
    def list_cluster_apps(name: str, request: Request):
        """Helm releases deployed through ``app-deploy`` executions (training runs carry their result)."""
        c = _cluster_for(current_user(request), name)
        return clusters.list_apps(c.name)

    @r.get("/apps/catalog/")
    def app_catalog(request: Request):
        """Bundled charts and their default values (the app store content shipped with the operator)."""
        current_user(request)
        import yaml as _yaml

        from ..domain import plan as _plan
        root = os.path.join(_plan.PLAYBOOK_DIR, "roles", "kubeapps", "files", "charts")
        out = []
        for d in sorted(os.listdir(root)):
            try:
                with open(os.path.join(root, d, "Chart.yaml")) as f:
                    meta = _yaml.safe_load(f)
                with open(os.path.join(root, d, "values.yaml")) as f:
                    values = _yaml.safe_load(f) or {}
            except OSError:
                continue
            out.append({"name": meta.get("name", d), "version": meta.get("version"),
                        "description": meta.get("description", ""), "values": values})
        return out

    @r.get("/cluster/config")
    @r.get("/cluster/config/")
    def cluster_plan(request: Request):
        current_user(request)
        return plan.load_plan()

    @r.get("/cluster/{cid}/download/")
    def download_kubeconfig(cid: str, request: Request):
        c = _cluster_for(current_user(request), cid)
        return PlainTextResponse(clusters.fetch_kubeconfig(c.name),
                                 headers={"Content-Disposition": f'attachment; filename="{c.name}-kubeconfig"'})

    @r.get("/cluster/{cid}/token/")
    def cluster_token(cid: str, request: Request):
        c = _cluster_for(current_user(request), cid)
        return {"token": clusters.cluster_token(c.name)}

    @r.get("/cluster/{cid}/webkubectl/token/")
    def webkubectl_token(cid: str, request: Request):
        import base64

        import httpx

        c = _cluster_for(current_user(request), cid)
        cfg = clusters.fetch_kubeconfig(c.name)
        url = str(get_config()["WEBKUBECTL_URL"]).rstrip("/")
        try:
            resp = httpx.post(f"{url}/api/kube-config", json={"name": c.name,
                              "kubeConfig": base64.b64encode(cfg.encode()).decode()}, timeout=10)
            return resp.json()
        except Exception as e:  # noqa: BLE001
            raise HTTPError(502, f"webkubectl unavailable: {e}") from e

    @r.get("/cluster/{cid}/grade/")
    def cluster_grade(cid: str, request: Request):
        c = _cluster_for(current_user(request), cid)
        return monitor.grade(c.name)

    def _cached(name):
        data = monitor.get_cluster_data(name)
        if data is None:
            try:
                data = monitor.set_cluster_data(name)
            except Exception as e:  # noqa: BLE001
                raise HTTPError(503, f"cluster data unavailable: {e}") from e
        return data

    @r.get("/cluster/{name}/health/{ns}/")
    def cluster_health(name: str, ns: str, request: Request):
        c = _cluster_for(current_user(request), name)
        h = monitor.cluster_health(c.name)
        if ns not in ("all", ""):
            h = dict(h, pods=[p for p in _cached(c.name)["pods"] if p["namespace"] == ns])
        return h

    @r.post("/cluster/{name}/monitor/refresh/")
    def cluster_monitor_refresh(name: str, request: Request):
        """Collect the cluster's dashboard data now instead of at the next 5-minute tick (UI dashboard refresh)."""
        c = _cluster_for(current_user(request), name)
        try:
            d = monitor.set_cluster_data(c.name)
        except Exception as e:  # noqa: BLE001 -- cluster API unreachable: the cached blob stays
            raise HTTPError(502, f"monitoring data of {c.name} not refreshed: {e}") from e
        return {"name": c.name, "date": d["date"]}

    @r.get("/cluster/{name}/component/")
    def cluster_components(name: str, request: Request):
        c = _cluster_for(current_user(request), name)
        return [d for d in _cached(c.name)["deployments"] if d["namespace"] == "kube-system"]

    @r.get("/cluster/{name}/namespace/")
    def cluster_namespaces(name: str, request: Request):
        c = _cluster_for(current_user(request), name)
        return _cached(c.name)["namespaces"]

    @r.get("/cluster/{name}/storage/")
    def cluster_storage(name: str, request: Request):
        c = _cluster_for(current_user(request), name)
        k8s, _, _ = monitor._clients(c)
        return {"storage_classes": k8s.get("/apis/storage.k8s.io/v1/storageclasses").get("items", []),
                "pvcs": k8s.get("/api/v1/persistentvolumeclaims").get("items", [])}

    @r.get("/cluster/{name}/checkNodes/")
    def check_nodes(name: str, request: Request):
        c = _cluster_for(current_user(request), name)
        return monitor.node_health(c.name)

    @r.get("/cluster/{name}/syncNodeTime/")
    def sync_node_time(name: str, request: Request):
        c = _cluster_for(current_user(request), name)
        return monitor.node_time_skew(c.name)

    @r.post("/cluster/{name}/event/")
    def cluster_events(name: str, request: Request, d: dict = Depends(body)):
        c = _cluster_for(current_user(request), name)
        return monitor.search_events(c.name, limit=int(d.get("limit", 100)), offset=int(d.get("offset", 0)),
                                     type_=d.get("type"))

    @r.get("/clusterHealthHistory/{pid}/")
    def health_history(pid: str, request: Request):
        current_user(request)
        c = clusters.get_cluster(_cluster_id_from_project(pid))
        return monitor.availability_history(c.id, request.query_params.get("type", "HOUR"))

    @r.get("/dashboard/{project}/{item}/")
    def dashboard(project: str, item: str, request: Request):
        u = current_user(request)
        names = [c["name"] for c in list_clusters(request)] if project in ("all", "") else [project]
        if item not in ("all", ""):
            names = [n for n in names if clusters.cluster_dict(clusters.get_cluster(n)).get("item_name") == item]
        out = {"clusters": [], "gpu_total": 0, "gpu_allocatable": 0, "restart_pods": [], "error_pods": [],
               "warn_containers": []}
        for n in names:
            d = monitor.get_cluster_data(n)
            if not d:
                continue
            out["clusters"].append(d)
            for k in ("gpu_total", "gpu_allocatable"):
                out[k] += d.get(k, 0)
            for k in ("restart_pods", "error_pods", "warn_containers"):
                out[k] += d.get(k, [])
        out["user"] = u.username
        return out

    # ------------------------------------------------------------------ packages / hosts / credentials
    @r.get("/packages/")
    def list_packages(request: Request):
        current_user(request)
        return packages.sync_packages()

    @r.get("/packages/{name}/")
    def get_package(name: str, request: Request):
        current_user(request)
        return packages.get_package(name)

    crud(r, "/credential/", M.Credential, secrets=("password", "private_key"), encrypt=("password", "private_key"))

    @r.get("/host/")
    def list_hosts(request: Request):
        u = current_user(request)
        with session_scope() as s:
            ids = [h.id for h in s.scalars(select(M.Host).order_by(M.Host.date_created))]
        return paginate(request, _visible(u, "HOST", [hosts.host_dict(i) for i in ids]))

    @r.post("/host/", status_code=201)
    def create_host(request: Request, d: dict = Depends(body)):
        u = current_user(request)
        out = hosts.create_host(d, check_ssh=bool(d.get("check_ssh", True)))
        if d.get("item_name"):
            users.add_item_resources(d["item_name"], "HOST", [out["id"]])
        return out

    @r.get("/host/{hid}/")
    def get_host(hid: str, request: Request):
        current_user(request)
        return hosts.host_dict(_row(M.Host, hid).id)

    @r.post("/host/{hid}/sync/")
    def sync_host(hid: str, request: Request):
        current_user(request)
        h = _row(M.Host, hid)
        return {"job_id": jobs.submit("sync_host_info", {"host_id": h.id})}

    @r.post("/host/{hid}/gpu-check/")
    def gpu_check_host(hid: str, request: Request):
        """Read-only GPU node check (kfd topology, rocminfo agents, amd-smi inventory) through the engine."""
        current_user(request)
        h = _row(M.Host, hid)
        return hosts.check_gpu_node(h.id)

    @r.delete("/host/{hid}/", status_code=204)
    def delete_host(hid: str, request: Request):
        superuser(request)
        h = _row(M.Host, hid)
        if h.node_id:
            raise HTTPError(400, f"host {h.name} is used by a cluster node")
        with session_scope() as s:
            s.delete(s.get(M.Host, h.id))
        return Response(status_code=204)

    @r.post("/host/import/")
    def import_hosts(request: Request, raw: bytes = Depends(raw_body)):
        superuser(request)
        ctype = request.headers.get("content-type", "")
        if ctype.startswith("multipart/"):
            parts = parse_multipart(ctype, raw)
            fname, data = parts.get("file") or next(iter(parts.values()))
        else:
            fname, data = request.query_params.get("filename", "hosts.csv"), raw
        return hosts.import_hosts(fname or "hosts.csv", data, check_ssh=request.query_params.get("check_ssh") != "false")

    @r.post("/file/upload/")
    def upload_file(request: Request, raw: bytes = Depends(raw_body)):
        current_user(request)
        ctype = request.headers.get("content-type", "")
        parts = parse_multipart(ctype, raw) if ctype.startswith("multipart/") else {"file": ("upload.bin", raw)}
        up = os.path.join(get_config().data_dir, "uploads")
        os.makedirs(up, exist_ok=True)
        saved = []
        for _, (fname, data) in parts.items():
            if fname:
                p = os.path.join(up, os.path.basename(fname))
                with open(p, "wb") as f:
                    f.write(data)
                saved.append({"name": os.path.basename(fname), "size": len(data), "path": p})
        return saved

    # ------------------------------------------------------------------ backup (api.py:331-425)
    crud(r, "/backupStorage/", M.BackupStorage, rtype="BACKUP_STORAGE", encrypt=("credentials",),
         to_dict=lambda b: dict(b.to_dict(), credentials={k: ("" if k in ("secretKey", "accountKey", "password")
                                                              else v) for k, v in (b.credentials or {}).items()}))

    @r.post("/backupStorage/check")
    @r.post("/backupStorage/check/")
    def check_storage(request: Request, d: dict = Depends(body)):
        current_user(request)
        try:
            return {"message": "OK" if backup.client_for(d).check() else "FAILED"}
        except Exception as e:  # noqa: BLE001
            return {"message": f"FAILED: {e}"}

    @r.post("/backupStorage/getBuckets")
    @r.post("/backupStorage/getBuckets/")
    def get_buckets(request: Request, d: dict = Depends(body)):
        current_user(request)
        return backup.client_for(d).list_buckets()

    crud(r, "/backupStrategy/", M.BackupStrategy, admin_write=False)

    @r.get("/clusterBackup/{pid}/")
    def list_backups(pid: str, request: Request):
        current_user(request)
        cid = _cluster_id_from_project(pid)
        with session_scope() as s:
            return [b.to_dict() for b in s.scalars(select(M.ClusterBackup).where(M.ClusterBackup.cluster_id == cid)
                                                    .order_by(M.ClusterBackup.date_created.desc()))]

    @r.delete("/clusterBackup/{bid}/delete/", status_code=204)
    def delete_backup(bid: str, request: Request):
        current_user(request)
        b = _row(M.ClusterBackup, bid)
        with session_scope() as s:
            st = s.get(M.BackupStorage, b.backup_storage_id)
            c = s.get(M.Cluster, b.cluster_id)
            if st is not None and c is not None:
                try:
                    backup.client_for(st).delete(f"{c.name}/{b.name}")
                except Exception:  # noqa: BLE001
                    pass
            s.delete(s.get(M.ClusterBackup, b.id))
        return Response(status_code=204)

    @r.put("/clusterBackup/restore/")
    @r.post("/clusterBackup/restore/")
    def restore_backup(request: Request, d: dict = Depends(body)):
        u = current_user(request)
        b = _row(M.ClusterBackup, d.get("id") or d["clusterBackupId"])
        c = _cluster_for(u, b.cluster_id, manage=True)
        return deploy.create(c.name, "restore", {"clusterBackupId": b.id}, user=u.username)

    # ------------------------------------------------------------------ items / RBAC (apis/item.py)
    crud(r, "/items/", M.Item)

    @r.get("/item/profiles/{item}/")
    def item_profiles(item: str, request: Request):
        current_user(request)
        it = _row(M.Item, item)
        with session_scope() as s:
            return [{"user_id": m.user_id, "username": s.get(M.User, m.user_id).username, "role": m.role}
                    for m in s.scalars(select(M.ItemRoleMapping).where(M.ItemRoleMapping.item_id == it.id))]

    @r.post("/item/profiles/{item}/")
    def set_item_profiles(item: str, request: Request, d: dict = Depends(body)):
        superuser(request)
        it = _row(M.Item, item)
        users.set_item_profiles(it.name, d if isinstance(d, list) else d.get("profiles", []))
        return item_profiles(item, request)

    @r.get("/resource/item/clusters/")
    def item_clusters(request: Request):
        u = current_user(request)
        return _visible(u, "CLUSTER", [clusters.cluster_dict(c) for c in _all(M.Cluster)])

    @r.get("/resource/{item}/")
    def item_resources(item: str, request: Request):
        current_user(request)
        it = _row(M.Item, item)
        with session_scope() as s:
            return [x.to_dict() for x in s.scalars(select(M.ItemResource).where(M.ItemResource.item_id == it.id))]

    @r.get("/resource/{item}/{rtype}/")
    def item_resources_type(item: str, rtype: str, request: Request):
        return [x for x in item_resources(item, request) if x["resource_type"] == rtype.upper()]

    @r.post("/resource/{item}/{rtype}/")
    def add_item_resources(item: str, rtype: str, request: Request, d: dict = Depends(body)):
        superuser(request)
        it = _row(M.Item, item)
        users.add_item_resources(it.name, rtype.upper(), d if isinstance(d, list) else d.get("ids", []))
        return item_resources_type(item, rtype, request)

    @r.delete("/resource/{item}/{rtype}/{rid}/", status_code=204)
    def del_item_resource(item: str, rtype: str, rid: str, request: Request):
        superuser(request)
        it = _row(M.Item, item)
        with session_scope() as s:
            s.query(M.ItemResource).filter(M.ItemResource.item_id == it.id, M.ItemResource.resource_id == rid,
                                           M.ItemResource.resource_type == rtype.upper()).delete()
        return Response(status_code=204)

    # ------------------------------------------------------------------ settings (api.py:517-529)
    @r.get("/settings")
    @r.get("/settings/")
    def get_settings(request: Request):
        current_user(request)
        st = context.get_settings(request.query_params.get("tab"))
        return {k: ("" if "PASSWORD" in k.upper() or "SECRET" in k.upper() else v) for k, v in st.items()}

    @r.post("/settings")
    @r.post("/settings/")
    def set_settings(request: Request, d: dict = Depends(body)):
        superuser(request)
        context.set_settings(d, tab=request.query_params.get("tab", "system"))
        return context.get_settings(request.query_params.get("tab"))

    # ------------------------------------------------------------------ DNS (ui/src/app/dns/dns.service.ts)
    # Cluster-wide resolvers for the nodes: stored as the "dns" settings tab, so every execution's extra vars carry
    # dns1 / dns2 to the nameserver role (a zone's own dns1 / dns2 override them: zone vars are applied later).
    @r.get("/dns/")
    def get_dns(request: Request):
        current_user(request)
        st = context.get_settings("dns")
        return {"id": "dns", "dns1": st.get("dns1", ""), "dns2": st.get("dns2", "")}

    @r.post("/dns/update/")
    def update_dns(request: Request, d: dict = Depends(body)):
        superuser(request)
        vals = {k: str(d.get(k) or "").strip() for k in ("dns1", "dns2")}
        for k, v in vals.items():
            if v and not _is_ipv4(v):
                raise HTTPError(400, {k: [f"not an IPv4 address: {v!r}"]})
        context.set_settings(vals, tab="dns")
        return {"id": "dns", **vals}

    # ------------------------------------------------------------------ cloud provider (cloud_provider/api.py)
    @r.get("/provider/template/")
    def provider_templates(request: Request):
        current_user(request)
        return [t.to_dict() for t in _all(M.CloudProviderTemplate)]

    crud(r, "/regions/", M.Region)
    crud(r, "/zones/", M.Zone, on_delete=_zone_in_use, on_create=lambda rid, data, u: cloud.on_zone_create(rid))
    crud(r, "/plans/", M.Plan, rtype="PLAN")

    @r.post("/cloud/region/")
    def cloud_regions(request: Request, _data: dict = Depends(body)):
        current_user(request)
        return cloud.list_regions_from_cloud(_data)

    @r.get("/cloud/compute/")
    def compute_models(request: Request):
        current_user(request)
        return cloud.compute_models()

    @r.get("/cloud/{region}/zone/")
    def cloud_zones(region: str, request: Request):
        current_user(request)
        reg = _row(M.Region, region)
        return cloud.list_zones_from_cloud(dict(reg.vars or {}, provider=_provider_of(reg)), reg.cloud_region)

    @r.get("/cloud/{region}/flavor/")
    def cloud_flavors(region: str, request: Request):
        current_user(request)
        reg = _row(M.Region, region)
        return cloud.list_flavors(dict(reg.vars or {}, provider=_provider_of(reg)), reg.cloud_region)

    # ------------------------------------------------------------------ storage (storage/api.py)
    @r.get("/storage/nfs/")
    def list_nfs(request: Request):
        current_user(request)
        return storage.list_nfs()

    @r.post("/storage/nfs/", status_code=201)
    def create_nfs(request: Request, _data: dict = Depends(body)):
        superuser(request)
        return storage.create_nfs(_data)

    @r.delete("/storage/nfs/{name}/", status_code=204)
    def delete_nfs(name: str, request: Request):
        superuser(request)
        storage.delete_nfs(name)
        return Response(status_code=204)

    @r.get("/storage/ceph/")
    def list_ceph(request: Request):
        current_user(request)
        return storage.list_ceph()

    @r.post("/storage/ceph/", status_code=201)
    def create_ceph(request: Request, _data: dict = Depends(body)):
        superuser(request)
        return storage.create_ceph(_data)

    @r.delete("/storage/ceph/{name}/", status_code=204)
    def delete_ceph(name: str, request: Request):
        superuser(request)
        storage.delete_ceph(name)
        return Response(status_code=204)

    # ------------------------------------------------------------------ logs / notifications
    @r.post("/log/")
    def search_log(request: Request, d: dict = Depends(body)):
        current_user(request)
        return monitor.search_system_log(d.get("level"), d.get("keywords"), int(d.get("days", 7)),
                                         int(d.get("limit", 50)), int(d.get("offset", 0)))

    @r.get("/notification/subscribe/")
    def get_subscribe(request: Request):
        u = current_user(request)
        with session_scope() as s:
            return [c.to_dict() for c in s.scalars(select(M.UserNotificationConfig)
                                                   .where(M.UserNotificationConfig.user_id == u.id))]

    @r.put("/notification/subscribe/")
    @r.post("/notification/subscribe/")
    def set_subscribe(request: Request, d: dict = Depends(body)):
        u = current_user(request)
        with session_scope() as s:
            row = s.scalar(select(M.UserNotificationConfig).where(M.UserNotificationConfig.user_id == u.id,
                                                                  M.UserNotificationConfig.type == d.get("type", "SYSTEM")))
            if row is None:
                row = M.UserNotificationConfig(user_id=u.id, type=d.get("type", "SYSTEM"))
                s.add(row)
            row.vars = d.get("vars", {})
        return get_subscribe(request)

    @r.get("/notification/receiver/")
    def get_receiver(request: Request):
        u = current_user(request)
        with session_scope() as s:
            row = s.scalar(select(M.UserReceiver).where(M.UserReceiver.user_id == u.id))
            return row.to_dict() if row else {"user_id": u.id, "vars": {}}

    @r.put("/notification/receiver/")
    @r.post("/notification/receiver/")
    def set_receiver(request: Request, d: dict = Depends(body)):
        u = current_user(request)
        with session_scope() as s:
            row = s.scalar(select(M.UserReceiver).where(M.UserReceiver.user_id == u.id))
            if row is None:
                row = M.UserReceiver(user_id=u.id)
                s.add(row)
            row.vars = d.get("vars", d)
        return get_receiver(request)

    @r.get("/notification/userMessage/")
    def user_messages(request: Request):
        u = current_user(request)
        q = request.query_params
        size = int(q.get("size", q.get("limit", 50)))
        off = (int(q.get("page", 1)) - 1) * size if "page" in q else int(q.get("offset", 0))
        return messages.user_messages(u.id, q.get("readStatus") or q.get("read_status"), size, off)

    @r.put("/notification/userMessage/")
    @r.post("/notification/userMessage/read/")
    def mark_messages(request: Request, d: dict = Depends(body)):
        u = current_user(request)
        ids = d if isinstance(d, list) else d.get("ids")
        return {"updated": messages.mark_read(u.id, ids)}

    @r.get("/notification/userMessage/unread/")
    def unread(request: Request):
        return {"unread": messages.unread_count(current_user(request).id)}

    @r.post("/notification/email/check/")
    def check_email(request: Request, d: dict = Depends(body)):
        superuser(request)
        ok = messages.send_email(d, d.get("SMTP_TEST_USER") or d.get("SMTP_USERNAME", ""), "KubeOperator test",
                                 "test message")
        return {"success": ok}

    @r.post("/notification/workWeixin/check/")
    def check_ww(request: Request, d: dict = Depends(body)):
        superuser(request)
        try:
            return {"success": messages.send_workweixin(d, d.get("WORKWEIXIN_TEST_USER", "@all"), "KubeOperator test")}
        except Exception as e:  # noqa: BLE001
            return {"success": False, "detail": str(e)}

    # ------------------------------------------------------------------ task monitor (the reference's Flower)
    @r.get("/tasks/")
    def task_list(request: Request):
        """Recent jobs, newest first; filters state / name, limit (default 100, at most 1000)."""
        superuser(request)
        q = request.query_params
        limit = min(1000, int(q.get("limit", 100) or 100))
        with session_scope() as s:
            stmt = select(M.Job).order_by(M.Job.date_created.desc()).limit(limit)
            if q.get("state"):
                stmt = stmt.where(M.Job.state == q["state"].upper())
            if q.get("name"):
                stmt = stmt.where(M.Job.name == q["name"])
            rows = list(s.scalars(stmt))
            return [{"id": j.id, "name": j.name, "state": j.state, "worker": j.worker, "attempts": j.attempts,
                     "args": j.args, "date_created": j.date_created, "date_start": j.date_start, "date_end": j.date_end,
                     "runtime_s": (j.date_end - j.date_start).total_seconds() if j.date_end and j.date_start else None,
                     "error": (j.result or {}).get("error")} for j in rows]

    @r.get("/tasks/stats/")
    def task_stats(request: Request):
        superuser(request)
        hours = request.query_params.get("hours")
        since = M.now() - dt.timedelta(hours=float(hours)) if hours else None
        return {"tasks": jobs.stats(since), "registered": jobs.registered_tasks()}

    @r.get("/tasks/workers/")
    def task_workers(request: Request):
        superuser(request)
        return jobs.workers()

    @r.get("/tasks/periodic/")
    def task_periodic(request: Request):
        superuser(request)
        with session_scope() as s:
            return [{"name": p.name, "task": p.task, "crontab": p.crontab, "interval_s": p.interval_s,
                     "enabled": p.enabled, "last_run": p.last_run}
                    for p in s.scalars(select(M.PeriodicTask).order_by(M.PeriodicTask.name))]

    @r.post("/tasks/{jid}/revoke/")
    def task_revoke(jid: str, request: Request):
        superuser(request)
        try:
            changed, state = jobs.revoke(jid)
        except KeyError:
            raise HTTPError(404, f"task {jid} not found")
        if not changed:
            raise HTTPError(409, f"task {jid} is {state}: only a PENDING task can be revoked")
        return {"id": jid, "state": state}

    @r.post("/tasks/{jid}/retry/")
    def task_retry(jid: str, request: Request):
        superuser(request)
        try:
            return {"id": jobs.retry(jid), "retry_of": jid}
        except KeyError:
            raise HTTPError(404, f"task {jid} not found")
        except ValueError as e:
            raise HTTPError(409, str(e))

    # ------------------------------------------------------------------ tasks (celery_api/api.py:15-37)
    @r.get("/tasks/{jid}/result/")
    def task_result(jid: str, request: Request):
        current_user(request)
        j = jobs.get(jid)
        if j is None:
            raise HTTPError(404, f"task {jid} not found")
        return {"id": j.id, "name": j.name, "state": j.state, "result": j.result,
                "date_start": j.date_start, "date_end": j.date_end}

    @r.get("/tasks/{jid}/log/")
    def task_log(jid: str, request: Request):
        current_user(request)
        off = int(request.query_params.get("mark", request.query_params.get("offset", 0)) or 0)
        data, end = jobs.tail(jobs.log_path(jid), off, 1 << 20)
        j = jobs.get(jid)
        return {"data": data, "mark": end, "end": j is not None and j.state in ("SUCCESS", "FAILURE", "REVOKED")}

    # ------------------------------------------------------------------ training chart (bundled workload)
    @r.get("/train/presets/")
    def train_presets(request: Request):
        current_user(request)
        from ...models.config import CONFIGS

        return {k: {"params": v.num_params(), "layers": v.n_layers, "hidden": v.hidden} for k, v in CONFIGS.items()}

    app.include_router(r)

    # ------------------------------------------------------------------ websockets (ws.py consumers)
    async def _ws_auth(ws: WebSocket) -> bool:
        tok = ws.query_params.get("token") or _auth_token(ws.headers)
        try:
            await asyncio.to_thread(users.user_from_token, tok or "")
            return True
        except AuthError:
            await ws.close(code=4401)
            return False

    @app.websocket("/ws/progress/{eid}/")
    async def ws_progress(ws: WebSocket, eid: str):
        """Push DeployExecution.to_json() every second (reference kubeops_api/ws.py:8-31)."""
        if not await _ws_auth(ws):
            return
        await ws.accept()
        try:
            while True:
                data = await asyncio.to_thread(deploy.to_json, eid)
                await ws.send_text(json.dumps(data, default=str))
                if data.get("state") in ("SUCCESS", "FAILURE"):
                    break
                await asyncio.sleep(float(ws.query_params.get("interval", 1.0)))
        except (WebSocketDisconnect, clusters.NotFound):
            return
        await ws.close()

    @app.websocket("/ws/tasks/{jid}/log/")
    async def ws_task_log(ws: WebSocket, jid: str):
        """Tail the job log: up to 4 KiB every 0.2 s (reference celery_api/ws.py:8-42)."""
        if not await _ws_auth(ws):
            return
        await ws.accept()
        off = 0
        path = jobs.log_path(jid)
        idle_after_end = 0
        try:
            while True:
                data, off2 = await asyncio.to_thread(jobs.tail, path, off, 4096)
                if data:
                    await ws.send_text(json.dumps({"message": data}))
                    off = off2
                    continue
                j = await asyncio.to_thread(jobs.get, jid)
                if j is not None and j.state in ("SUCCESS", "FAILURE", "REVOKED"):
                    idle_after_end += 1
                    if idle_after_end > 2:
                        break
                await asyncio.sleep(0.2)
        except WebSocketDisconnect:
            return
        await ws.close()

    # ------------------------------------------------------------------ web UI
    @app.get("/")
    def root():
        return RedirectResponse("/ui/")

    @app.get("/flower/")
    def flower():
        """The reference proxies Celery Flower here (kubeoperator/celery_flower.py:13-22): its task monitor is
        the UI's tasks view."""
        return RedirectResponse("/ui/#/tasks")

    @app.get("/ui/{path:path}")
    def ui(path: str):
        p = os.path.normpath(os.path.join(UI_DIR, path or "index.html"))
        if not p.startswith(UI_DIR) or not os.path.isfile(p):
            p = os.path.join(UI_DIR, "index.html")
        return FileResponse(p)

    @app.get("/metrics")
    def prometheus_metrics():
        from ..runtime import metrics

        return Response(metrics.exposition(), media_type="text/plain; version=0.0.4")

    @app.get("/healthz")
    def healthz():
        return {"ok": True, "time": time.time()}

    return app


# ------------------------------------------------------------------------------------------------ small helpers
def _user(uid: str) -> M.User:
    with session_scope() as s:
        u = s.get(M.User, uid) or s.scalar(select(M.User).where(M.User.username == uid))
    if u is None:
        raise HTTPError(404, f"user {uid} not found")
    return u


def _all(model) -> list:
    with session_scope() as s:
        return list(s.scalars(select(model).order_by(model.date_created)))


def _exec_dict(e: M.Execution) -> dict:
    d = e.to_dict(exclude=("result_raw",))
    return d


def _cluster_id_from_project(pid: str) -> str:
    with session_scope() as s:
        c = s.scalar(select(M.Cluster).where((M.Cluster.project_id == pid) | (M.Cluster.id == pid)
                                             | (M.Cluster.name == pid)))
        if c is None:
            raise HTTPError(404, f"cluster {pid} not found")
        return c.id


def _zone_in_use(z: M.Zone) -> None:
    with session_scope() as s:
        if s.scalar(select(M.Host).where(M.Host.zone_id == z.id)) is not None or z.ip_used:
            raise HTTPError(400, f"zone {z.name} is in use")


def _provider_of(reg: M.Region) -> str:
    with session_scope() as s:
        t = s.get(M.CloudProviderTemplate, reg.template_id) if reg.template_id else None
        return t.name if t else (reg.vars or {}).get("provider", "")


def json_default(o):
    if isinstance(o, (dt.datetime, dt.date)):
        return o.isoformat()
    return str(o)
