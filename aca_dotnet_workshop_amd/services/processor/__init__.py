"""Backend processor service (reference TasksTracker.Processor.Backend.Svc)."""
from .app import ROLE, create_app, main

__all__ = ["ROLE", "create_app", "main"]
