"""HTTP / WebSocket API of the control plane."""
from .app import create_app

__all__ = ["create_app"]
