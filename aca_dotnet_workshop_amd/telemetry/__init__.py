"""Observability: tracing (App Insights equivalent), structured logs, metrics, app map."""
from .logging import configure_logging
from .metrics import REGISTRY, Counter, Gauge, Histogram, Registry, metrics_middleware
from .tracing import (Span, Tracer, configure, current_span, current_trace_id, current_traceparent,
                      parse_traceparent, server_middleware, tracer)

__all__ = ["configure_logging", "REGISTRY", "Counter", "Gauge", "Histogram", "Registry", "metrics_middleware",
           "Span", "Tracer", "configure", "current_span", "current_trace_id", "current_traceparent",
           "parse_traceparent", "server_middleware", "tracer"]
