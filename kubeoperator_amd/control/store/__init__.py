"""Control-plane persistence: SQLAlchemy models, sessions, secret encryption."""
from . import models
from .db import init_db, session, session_scope

__all__ = ["models", "init_db", "session", "session_scope"]
