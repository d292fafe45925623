"""Application SDK for talking to the sidecar (the Dapr .NET SDK equivalent)."""
from .aspnet import cloud_events_middleware, map_subscribe_handler, subscriptions, topic
from .client import (DaprClient, InvocationError, QueryResponse, SidecarClient, StateItem, client_from_config,
                     sidecar_base_url)

__all__ = ["cloud_events_middleware", "map_subscribe_handler", "subscriptions", "topic", "DaprClient",
           "InvocationError", "QueryResponse", "SidecarClient", "StateItem", "sidecar_base_url",
           "client_from_config"]
