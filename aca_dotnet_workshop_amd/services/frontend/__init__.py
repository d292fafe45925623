"""Web portal service (reference TasksTracker.WebPortal.Frontend.Ui)."""
from .app import ROLE, create_app, main

__all__ = ["ROLE", "create_app", "main"]
