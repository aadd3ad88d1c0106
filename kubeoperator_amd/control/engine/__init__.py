"""Execution engine: inventory, Jinja templating, transports (ssh/local/fake), modules, playbook runner."""
from .inventory import Inventory
from .modules import MODULES, module_names
from .runner import PlaybookError, ResultCallback, Runner
from .transport import FakeTransport, HostConn, LocalTransport, SSHTransport, Transport, Unreachable, make_transport

__all__ = ["Inventory", "MODULES", "module_names", "PlaybookError", "ResultCallback", "Runner", "FakeTransport",
           "HostConn", "LocalTransport", "SSHTransport", "Transport", "Unreachable", "make_transport"]
