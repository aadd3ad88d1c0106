"""Users, authentication (JWT / password / LDAP) and item-based RBAC.

Reference: users/models.py:9-26 (Profile.source local/ldap), users/api.py:17-90, authentication/ldap.py,
sync/ldap.py, kubeops_api/models/item.py + item_resource.py, apis/item.py:24-234,
settings.py:218-223 (JWT: header prefix ``JWT``, 12 h expiry, refresh allowed).

JWT is HS256 implemented on the stdlib (PyJWT is not available). The token payload carries the profile
incl. ``item_role_mappings`` like the reference's jwt_response_payload_handler.
"""
from __future__ import annotations

import base64
import datetime as dt
import hashlib
import hmac
import json
import time

from sqlalchemy import select

from ..conf import get_config
from ..store import models as M
from ..store.crypto import hash_password, verify_password
from ..store.db import session_scope
from . import context


class AuthError(Exception):
    pass


class Forbidden(Exception):
    pass


def _b64(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def _unb64(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def jwt_encode(payload: dict, key: str | None = None) -> str:
    key = key or get_config().secret_key()
    head = _b64(json.dumps({"alg": "HS256", "typ": "JWT"}, separators=(",", ":")).encode())
    body = _b64(json.dumps(payload, separators=(",", ":"), default=str).encode())
    sig = _b64(hmac.new(key.encode(), f"{head}.{body}".encode(), hashlib.sha256).digest())
    return f"{head}.{body}.{sig}"


def jwt_decode(token: str, key: str | None = None, verify_exp: bool = True) -> dict:
    key = key or get_config().secret_key()
    try:
        head, body, sig = token.split(".")
    except ValueError as e:
        raise AuthError("malformed token") from e
    good = _b64(hmac.new(key.encode(), f"{head}.{body}".encode(), hashlib.sha256).digest())
    if not hmac.compare_digest(good, sig):
        raise AuthError("bad token signature")
    payload = json.loads(_unb64(body))
    if verify_exp and payload.get("exp", 0) < time.time():
        raise AuthError("token expired")
    return payload


def profile(user: M.User) -> dict:
    with session_scope() as s:
        maps = [{"item_id": m.item_id, "item_name": s.get(M.Item, m.item_id).name, "role": m.role}
                for m in s.scalars(select(M.ItemRoleMapping).where(M.ItemRoleMapping.user_id == user.id))]
    return {"id": user.id, "username": user.username, "email": user.email, "is_superuser": user.is_superuser,
            "is_active": user.is_active, "source": user.source, "item_role_mappings": maps,
            "notification_config": user.notification_config}


def issue_token(user: M.User, orig_iat: float | None = None) -> dict:
    hours = int(get_config()["JWT_EXPIRATION_HOURS"])
    now = time.time()
    payload = {"user_id": user.id, "username": user.username, "exp": int(now + hours * 3600),
               "orig_iat": int(orig_iat or now), "profile": profile(user)}
    return {"token": jwt_encode(payload), "user": payload["profile"]}


def authenticate(username: str, password: str) -> dict:
    with session_scope() as s:
        u = s.scalar(select(M.User).where(M.User.username == username))
    if u is not None and u.source == "local":
        if not u.is_active or not verify_password(password, u.password_hash):
            raise AuthError("unable to log in with provided credentials")
    elif context.get_settings("ldap").get("AUTH_LDAP_ENABLE") in ("true", "True", True):
        u = ldap_authenticate(username, password)
        if not u.is_active:
            raise AuthError("unable to log in with provided credentials")
    else:
        raise AuthError("unable to log in with provided credentials")
    with session_scope() as s:
        s.get(M.User, u.id).last_login = M.now()
    return issue_token(u)


def refresh(token: str) -> dict:
    p = jwt_decode(token, verify_exp=True)
    with session_scope() as s:
        u = s.get(M.User, p["user_id"])
    if u is None or not u.is_active:
        raise AuthError("user inactive")
    if time.time() - p.get("orig_iat", 0) > 7 * 86400:
        raise AuthError("refresh has expired")
    return issue_token(u, p.get("orig_iat"))


def user_from_token(token: str) -> M.User:
    p = jwt_decode(token)
    with session_scope() as s:
        u = s.get(M.User, p["user_id"])
    if u is None or not u.is_active:
        raise AuthError("user inactive or deleted")
    return u


def create_user(username: str, password: str, email: str = "", is_superuser: bool = False, source="local") -> dict:
    with session_scope() as s:
        if s.scalar(select(M.User).where(M.User.username == username)) is not None:
            raise ValueError(f"user {username} exists")
        u = M.User(username=username, email=email, is_superuser=is_superuser, source=source,
                   password_hash=hash_password(password) if password else "")
        s.add(u)
        s.flush()
        return profile(u)


def set_password(user_id: str, original: str | None, new: str, check_original: bool = True) -> None:
    with session_scope() as s:
        u = s.get(M.User, user_id)
        if check_original and not verify_password(original or "", u.password_hash):
            raise AuthError("original password is wrong")
        u.password_hash = hash_password(new)


# ------------------------------------------------------------------------------------------- LDAP
def _ldap_settings() -> dict:
    st = context.get_settings("ldap")
    if not st.get("AUTH_LDAP_SERVER_URI"):
        raise AuthError("LDAP server URI is not configured")
    return st


def _ldap_service_conn(st: dict):
    from .ldap_client import LDAPConnection

    conn = LDAPConnection(st["AUTH_LDAP_SERVER_URI"])
    if st.get("AUTH_LDAP_BIND_DN"):
        conn.bind(st["AUTH_LDAP_BIND_DN"], st.get("AUTH_LDAP_BIND_PASSWORD", ""))
    return conn


def _attr_map(st: dict) -> dict:
    try:
        return json.loads(st.get("AUTH_LDAP_USER_ATTR_MAP") or '{"username": "uid", "email": "mail"}')
    except ValueError:
        return {"username": "uid", "email": "mail"}


def ldap_authenticate(username: str, password: str) -> M.User:
    """Find the user's entry with the service account (AUTH_LDAP_SEARCH_OU, ``|``-separated bases, and
    AUTH_LDAP_SEARCH_FILTER), then bind as that DN with the given password (reference
    users/authentication/ldap.py). The user name is escaped before it goes into the filter."""
    from .ldap_client import LDAPConnection, LDAPError, escape_filter_value

    st = _ldap_settings()
    amap = _attr_map(st)
    flt = (st.get("AUTH_LDAP_SEARCH_FILTER") or f"({amap.get('username', 'uid')}=%(user)s)") % {
        "user": escape_filter_value(username)}
    try:
        with _ldap_service_conn(st) as conn:
            hits = []
            for base in (st.get("AUTH_LDAP_SEARCH_OU") or "").split("|"):
                if base.strip():
                    hits += conn.search(base.strip(), flt, attributes=[amap.get("email", "mail")], size_limit=2)
        if not hits:
            raise AuthError("LDAP user not found")
        if len({h["dn"].lower() for h in hits}) > 1:
            # ambiguous search (several entries over the bases): never bind as whichever the server lists first
            raise AuthError("LDAP search matched more than one entry")
        found = hits[0]
        with LDAPConnection(st["AUTH_LDAP_SERVER_URI"]) as user_conn:
            user_conn.bind(found["dn"], password)
    except LDAPError as e:
        raise AuthError("invalid LDAP credentials" if e.code == 49 else f"LDAP error: {e}") from e
    except OSError as e:
        raise AuthError(f"LDAP server unreachable: {e}") from e
    email = (found["attrs"].get(amap.get("email", "mail")) or [""])[0]
    with session_scope() as s:
        u = s.scalar(select(M.User).where(M.User.username == username))
        if u is None:
            u = M.User(username=username, source="ldap", email=email)
            s.add(u)
            s.flush()
        elif u.source != "ldap":
            raise AuthError("a local user with this name exists")
        uid = u.id
    with session_scope() as s:
        u = s.get(M.User, uid)
        s.expunge(u)
        return u


def sync_ldap_users() -> int:
    """Import every person entry under the search bases as an LDAP user (reference users/sync/ldap.py)."""
    st = context.get_settings("ldap")
    if str(st.get("AUTH_LDAP_ENABLE")) not in ("true", "True") or not st.get("AUTH_LDAP_SERVER_URI"):
        return 0
    amap = _attr_map(st)
    uattr, eattr = amap.get("username", "uid"), amap.get("email", "mail")
    n = 0
    with _ldap_service_conn(st) as conn:
        for base in (st.get("AUTH_LDAP_SEARCH_OU") or "").split("|"):
            if not base.strip():
                continue
            for e in conn.search(base.strip(), "(|(objectClass=person)(objectClass=inetOrgPerson))", [uattr, eattr]):
                name = (e["attrs"].get(uattr) or [""])[0]
                if not name:
                    continue
                with session_scope() as s:
                    if s.scalar(select(M.User).where(M.User.username == name)) is None:
                        s.add(M.User(username=name, source="ldap", email=(e["attrs"].get(eattr) or [""])[0]))
                        n += 1
    return n


# ------------------------------------------------------------------------------------------- items / RBAC
def items_for(user: M.User) -> list[str]:
    """Item ids a user can see (superusers: all)."""
    with session_scope() as s:
        if user.is_superuser:
            return [i.id for i in s.scalars(select(M.Item))]
        return [m.item_id for m in s.scalars(select(M.ItemRoleMapping).where(M.ItemRoleMapping.user_id == user.id))]


def role_in(user: M.User, item_id: str) -> str | None:
    if user.is_superuser:
        return "MANAGER"
    with session_scope() as s:
        m = s.scalar(select(M.ItemRoleMapping).where(M.ItemRoleMapping.user_id == user.id,
                                                     M.ItemRoleMapping.item_id == item_id))
        return m.role if m else None


def visible_resources(user: M.User, resource_type: str) -> set[str] | None:
    """Resource ids of a type visible to the user; None = everything (superuser)."""
    if user.is_superuser:
        return None
    ids = items_for(user)
    with session_scope() as s:
        return {r.resource_id for r in s.scalars(select(M.ItemResource).where(
            M.ItemResource.item_id.in_(ids), M.ItemResource.resource_type == resource_type))}


def require_manager(user: M.User, resource_id: str, resource_type: str) -> None:
    """MANAGER of an item owning the resource (or superuser) -- e.g. to delete / operate a cluster."""
    if user.is_superuser:
        return
    with session_scope() as s:
        rows = list(s.scalars(select(M.ItemResource).where(M.ItemResource.resource_id == resource_id,
                                                           M.ItemResource.resource_type == resource_type)))
    if not any(role_in(user, r.item_id) == "MANAGER" for r in rows):
        raise Forbidden("requires MANAGER role on the resource's item")


def set_item_profiles(item_name: str, mappings: list[dict]) -> None:
    with session_scope() as s:
        item = s.scalar(select(M.Item).where(M.Item.name == item_name))
        s.query(M.ItemRoleMapping).filter(M.ItemRoleMapping.item_id == item.id).delete()
        for m in mappings:
            u = s.scalar(select(M.User).where((M.User.username == m.get("username")) | (M.User.id == m.get("user_id"))))
            if u is not None:
                s.add(M.ItemRoleMapping(item_id=item.id, user_id=u.id, role=m.get("role", "VIEWER")))


def add_item_resources(item_name: str, resource_type: str, ids: list[str]) -> None:
    with session_scope() as s:
        item = s.scalar(select(M.Item).where(M.Item.name == item_name))
        for rid in ids:
            if s.scalar(select(M.ItemResource).where(M.ItemResource.resource_id == rid,
                                                     M.ItemResource.resource_type == resource_type)) is None:
                s.add(M.ItemResource(item_id=item.id, resource_id=rid, resource_type=resource_type))


def now_iso() -> str:
    return dt.datetime.utcnow().isoformat()
