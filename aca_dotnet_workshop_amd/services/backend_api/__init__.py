"""Backend API service (reference TasksTracker.TasksManager.Backend.Api)."""
from .app import ROLE, create_app, main
from .managers import FakeTasksManager, TasksManager, TasksStoreManager

__all__ = ["ROLE", "create_app", "main", "FakeTasksManager", "TasksManager", "TasksStoreManager"]
