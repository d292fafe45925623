"""Backing-services emulator (Cosmos DB / Service Bus / Storage / Key Vault / SendGrid /
Redis equivalents) built on the native engines, plus its async client."""
from .auth import AccessPolicy, RoleAssignment
from .client import BackingClient, BackingError, EtagConflict, backing_url
from .server import BackingServices, serve_backing

__all__ = ["AccessPolicy", "RoleAssignment", "BackingClient", "BackingError", "EtagConflict", "backing_url",
           "BackingServices", "serve_backing"]
