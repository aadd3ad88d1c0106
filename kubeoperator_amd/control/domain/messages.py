"""Message center: per-user fan-out of cluster / system messages over LOCAL, EMAIL, DINGTALK, WORKWEIXIN.

Reference: message_center/models.py:14-113, message_client.py:21-186 (``insert_message`` :84-104 fans a
message out to every user of the message's item according to each user's subscription config, then
sends email / DingTalk in threads). Settings keys: ``SMTP_*``, ``DINGTALK_*``, ``WORKWEIXIN_*``.
External deliveries run on a small thread pool and record send_status per user message.
"""
from __future__ import annotations

import base64
import concurrent.futures as cf
import hashlib
import hmac
import json
import logging
import smtplib
import time
import urllib.parse
from email.mime.text import MIMEText

import httpx
from sqlalchemy import func, select

from ..store import models as M
from ..store.db import session_scope
from . import context

log = logging.getLogger("kubeoperator.messages")
_pool = cf.ThreadPoolExecutor(max_workers=4, thread_name_prefix="kop-notify")
SEND_TYPES = ("LOCAL", "EMAIL", "DINGTALK", "WORKWEIXIN")


def _recipients(s, item_id):
    users = list(s.scalars(select(M.User).where(M.User.is_active.is_(True))))
    if not item_id:
        return users
    members = {m.user_id for m in s.scalars(select(M.ItemRoleMapping).where(M.ItemRoleMapping.item_id == item_id))}
    return [u for u in users if u.is_superuser or u.id in members]


def insert_message(msg: dict, sync: bool = False) -> str:
    with session_scope() as s:
        m = M.Message(title=msg.get("title", ""), sender=msg.get("sender", "system"), content=msg.get("content", {}),
                      level=msg.get("level", "INFO"), type=msg.get("type", "SYSTEM"), item_id=msg.get("item_id"))
        s.add(m)
        s.flush()
        mid = m.id
        jobs = []
        for u in _recipients(s, m.item_id):
            cfg = dict(u.notification_config or {})
            nc = s.scalar(select(M.UserNotificationConfig).where(M.UserNotificationConfig.user_id == u.id,
                                                                 M.UserNotificationConfig.type == m.type))
            if nc is not None:
                cfg.update(nc.vars or {})
            rcv = s.scalar(select(M.UserReceiver).where(M.UserReceiver.user_id == u.id))
            for t in SEND_TYPES:
                if cfg.get(t, "DISABLE") != "ENABLE":
                    continue
                receive = (rcv.vars or {}).get(t, "") if rcv is not None else ""
                if t == "EMAIL" and not receive:
                    receive = u.email
                um = M.UserMessage(user_id=u.id, message_id=mid, send_type=t, receive=receive,
                                   send_status="SUCCESS" if t == "LOCAL" else "PENDING")
                s.add(um)
                s.flush()
                if t != "LOCAL":
                    jobs.append((um.id, t, receive))
    for umid, t, receive in jobs:
        f = _pool.submit(_deliver, umid, t, receive, msg)
        if sync:
            f.result()
    return mid


def _deliver(user_message_id: str, send_type: str, receive: str, msg: dict) -> None:
    ok = False
    try:
        st = context.get_settings()
        text = f"[KubeOperator] {msg.get('title', '')}: {json.dumps(msg.get('content', {}), ensure_ascii=False)}"
        if send_type == "EMAIL" and st.get("SMTP_STATUS") == "ENABLE" and receive:
            ok = send_email(st, receive, msg.get("title", ""), text)
        elif send_type == "DINGTALK" and st.get("DINGTALK_STATUS") == "ENABLE":
            ok = send_dingtalk(st, receive, text)
        elif send_type == "WORKWEIXIN" and st.get("WORKWEIXIN_STATUS") == "ENABLE":
            ok = send_workweixin(st, receive, text)
    except Exception:  # noqa: BLE001
        log.exception("delivery %s failed", send_type)
    with session_scope() as s:
        um = s.get(M.UserMessage, user_message_id)
        if um is not None:
            um.send_status = "SUCCESS" if ok else "FAILED"


def send_email(st: dict, to: str, subject: str, body: str) -> bool:
    m = MIMEText(body, "plain", "utf-8")
    m["Subject"], m["From"], m["To"] = subject, st.get("SMTP_USERNAME", ""), to
    port = int(st.get("SMTP_PORT", 465))
    cls = smtplib.SMTP_SSL if port == 465 else smtplib.SMTP
    with cls(st.get("SMTP_ADDRESS", "localhost"), port, timeout=30) as srv:
        if st.get("SMTP_USERNAME"):
            srv.login(st["SMTP_USERNAME"], st.get("SMTP_PASSWORD", ""))
        srv.sendmail(st.get("SMTP_USERNAME", ""), [to], m.as_string())
    return True


def _dingtalk_url(st: dict) -> str:
    url = st.get("DINGTALK_WEBHOOK", "")
    secret = st.get("DINGTALK_SECRET", "")
    if secret:
        ts = str(round(time.time() * 1000))
        sign = base64.b64encode(hmac.new(secret.encode(), f"{ts}\n{secret}".encode(), hashlib.sha256).digest())
        url += f"&timestamp={ts}&sign={urllib.parse.quote_plus(sign)}"
    return url


def send_dingtalk(st: dict, receive: str, text: str) -> bool:
    body = {"msgtype": "text", "text": {"content": text}, "at": {"atMobiles": [receive] if receive else []}}
    r = httpx.post(_dingtalk_url(st), json=body, timeout=15)
    return r.status_code == 200 and r.json().get("errcode", 1) == 0


def send_workweixin(st: dict, receive: str, text: str) -> bool:
    tok = httpx.get("https://qyapi.weixin.qq.com/cgi-bin/gettoken",
                    params={"corpid": st.get("WORKWEIXIN_CORP_ID", ""), "corpsecret": st.get("WORKWEIXIN_SECRET", "")},
                    timeout=15).json().get("access_token")
    r = httpx.post(f"https://qyapi.weixin.qq.com/cgi-bin/message/send?access_token={tok}",
                   json={"touser": receive, "msgtype": "text", "agentid": st.get("WORKWEIXIN_AGENT_ID", ""),
                         "text": {"content": text}}, timeout=15)
    return r.status_code == 200 and r.json().get("errcode", 1) == 0


def user_messages(user_id: str, read_status: str | None = None, limit: int = 50, offset: int = 0) -> dict:
    with session_scope() as s:
        q = select(M.UserMessage, M.Message).join(M.Message, M.Message.id == M.UserMessage.message_id).where(
            M.UserMessage.user_id == user_id, M.UserMessage.send_type == "LOCAL")
        if read_status:
            q = q.where(M.UserMessage.read_status == read_status)
        total = s.scalar(select(func.count()).select_from(q.subquery()))
        rows = s.execute(q.order_by(M.UserMessage.date_created.desc()).limit(limit).offset(offset)).all()
        return {"count": total, "results": [{**um.to_dict(), "message_detail": m.to_dict()} for um, m in rows]}


def unread_count(user_id: str) -> int:
    with session_scope() as s:
        return s.scalar(select(func.count()).select_from(M.UserMessage).where(
            M.UserMessage.user_id == user_id, M.UserMessage.send_type == "LOCAL",
            M.UserMessage.read_status == "UNREAD")) or 0


def mark_read(user_id: str, ids: list[str] | None = None) -> int:
    with session_scope() as s:
        q = select(M.UserMessage).where(M.UserMessage.user_id == user_id, M.UserMessage.read_status == "UNREAD")
        n = 0
        for um in s.scalars(q):
            if ids is None or um.id in ids:
                um.read_status = "READ"
                n += 1
        return n
