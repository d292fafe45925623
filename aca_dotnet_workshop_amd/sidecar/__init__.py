"""The sidecar runtime (``daprd`` equivalent): building-block API, components, delivery."""
from . import bindings, pubsub, secrets, state  # noqa: F401  (register component types)
from .base import RuntimeContext, supported_types
from .components import Component, ComponentError, SubscriptionSpec, from_dict, load_file, load_paths
from .registry import NameResolver
from .runtime import Sidecar, make_cloudevent

__all__ = ["RuntimeContext", "supported_types", "Component", "ComponentError", "SubscriptionSpec", "from_dict",
           "load_file", "load_paths", "NameResolver", "Sidecar", "make_cloudevent"]
