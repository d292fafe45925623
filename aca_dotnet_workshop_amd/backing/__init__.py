"""Backing-services emulator (Cosmos DB / Service Bus / Storage / Key Vault / SendGrid /
Redis equivalents) built on the native engines, plus its async client."""
from .auth import AccessPolicy, RoleAssignment
from .client import BackingClient, BackingError, EtagConflict, backing_url

__all__ = ["AccessPolicy", "RoleAssignment", "BackingClient", "BackingError", "EtagConflict", "backing_url",
           "BackingServices", "serve_backing"]


def __getattr__(name: str):
    """The server (and through it the columnar query engine) loads on first use only: services
    that just need the client -- the processor's SendGrid-API notifier -- do not import it."""
    if name in ("BackingServices", "serve_backing"):
        from . import server
        return getattr(server, name)
    raise AttributeError(name)
