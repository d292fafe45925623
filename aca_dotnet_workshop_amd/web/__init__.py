"""HTTP server, client and application framework (the Kestrel / ASP.NET Core equivalent)."""
from .app import Route, WebApp, read_model, run_app, to_response
from .client import ClientResponse, HttpClient
from .http import (Headers, HTTPError, Request, Response, empty, html_response, json_response, problem,
                   redirect, text_response)
from .server import HttpServer, serve

__all__ = ["Route", "WebApp", "read_model", "run_app", "to_response", "ClientResponse", "HttpClient",
           "Headers", "HTTPError", "Request", "Response", "empty", "html_response", "json_response",
           "problem", "redirect", "text_response", "HttpServer", "serve"]
