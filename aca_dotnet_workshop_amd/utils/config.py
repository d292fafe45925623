"""Layered configuration, equivalent of ASP.NET Core's default configuration stack.

Reference behaviour reproduced (SURVEY.md §5 "Config / flag system"):
* ``appsettings.json`` -> ``appsettings.{Environment}.json`` -> environment variables ->
  command-line ``--Key=Value``; later layers win.
* Keys are case-insensitive and hierarchical with ``:`` (``BackendApiConfig:BaseUrlExternalHttp``,
  reference Frontend.Ui/Program.cs:17); environment variables use ``__`` as the separator
  (``SendGrid__IntegrationEnabled``, reference bicep/modules/container-apps/processor-backend-service.bicep:148-151).
* The environment name comes from ``ASPNETCORE_ENVIRONMENT`` / ``DOTNET_ENVIRONMENT`` /
  ``APP_ENVIRONMENT`` (default ``Production``), as in Properties/launchSettings.json.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Any, Iterable, Mapping

_TRUE = {"true", "1", "yes", "on"}
_FALSE = {"false", "0", "no", "off", ""}


def _flatten(prefix: str, value: Any, out: dict[str, Any]) -> None:
    if isinstance(value, Mapping):
        for k, v in value.items():
            _flatten(f"{prefix}:{k}" if prefix else str(k), v, out)
    elif isinstance(value, list):
        for i, v in enumerate(value):
            _flatten(f"{prefix}:{i}" if prefix else str(i), v, out)
    else:
        out[prefix] = value


class Configuration:
    """Flat, case-insensitive ``path -> value`` view over the merged layers."""

    def __init__(self, layers: Iterable[Mapping[str, Any]] = ()) -> None:
        self._data: dict[str, Any] = {}
        self._orig: dict[str, str] = {}
        for layer in layers:
            self.add(layer)

    # -- building -------------------------------------------------------------
    def add(self, layer: Mapping[str, Any]) -> "Configuration":
        flat: dict[str, Any] = {}
        _flatten("", layer, flat)
        for k, v in flat.items():
            self._data[k.lower()] = v
            self._orig[k.lower()] = k
        return self

    def add_json_file(self, path: str | os.PathLike, optional: bool = True) -> "Configuration":
        p = Path(path)
        if not p.exists():
            if optional:
                return self
            raise FileNotFoundError(p)
        text = p.read_text(encoding="utf-8-sig")
        return self.add(json.loads(text) if text.strip() else {})

    def add_environment(self, environ: Mapping[str, str] | None = None, prefix: str = "") -> "Configuration":
        env = os.environ if environ is None else environ
        layer: dict[str, Any] = {}
        for k, v in env.items():
            if prefix and not k.startswith(prefix):
                continue
            key = k[len(prefix):].replace("__", ":")
            layer[key] = v
        for k, v in layer.items():
            self._data[k.lower()] = v
            self._orig[k.lower()] = k
        return self

    def add_command_line(self, argv: Iterable[str]) -> "Configuration":
        args = list(argv)
        i = 0
        while i < len(args):
            a = args[i]
            if a.startswith("--") and "=" in a:
                k, v = a[2:].split("=", 1)
                self._data[k.replace("__", ":").lower()] = v
            elif a.startswith("--") and i + 1 < len(args) and not args[i + 1].startswith("--"):
                self._data[a[2:].replace("__", ":").lower()] = args[i + 1]
                i += 1
            i += 1
        return self

    def set(self, key: str, value: Any) -> None:
        self._data[key.lower()] = value

    # -- reading --------------------------------------------------------------
    def get(self, key: str, default: Any = None) -> Any:
        return self._data.get(key.lower(), default)

    def __getitem__(self, key: str) -> Any:
        return self._data.get(key.lower())

    def __contains__(self, key: str) -> bool:
        return key.lower() in self._data

    def get_str(self, key: str, default: str | None = None) -> str | None:
        v = self.get(key)
        return default if v is None else str(v)

    def get_bool(self, key: str, default: bool = False) -> bool:
        v = self.get(key)
        if v is None:
            return default
        if isinstance(v, bool):
            return v
        s = str(v).strip().lower()
        if s in _TRUE:
            return True
        if s in _FALSE:
            return False
        raise ValueError(f"configuration value {key}={v!r} is not a boolean")

    def get_int(self, key: str, default: int = 0) -> int:
        v = self.get(key)
        return default if v is None or v == "" else int(v)

    def get_float(self, key: str, default: float = 0.0) -> float:
        v = self.get(key)
        return default if v is None or v == "" else float(v)

    def section(self, prefix: str) -> dict[str, Any]:
        """Nested dict of everything under ``prefix`` (original key casing)."""
        p = prefix.lower() + ":"
        out: dict[str, Any] = {}
        for k, v in self._data.items():
            if k.startswith(p):
                parts = self._orig.get(k, k)[len(p):].split(":")
                cur = out
                for part in parts[:-1]:
                    cur = cur.setdefault(part, {})
                cur[parts[-1]] = v
        return out

    def as_dict(self) -> dict[str, Any]:
        return {self._orig.get(k, k): v for k, v in self._data.items()}


def environment_name(environ: Mapping[str, str] | None = None) -> str:
    env = os.environ if environ is None else environ
    for k in ("ASPNETCORE_ENVIRONMENT", "DOTNET_ENVIRONMENT", "APP_ENVIRONMENT"):
        if env.get(k):
            return env[k]
    return "Production"


def load_configuration(content_root: str | os.PathLike | None = None,
                       environ: Mapping[str, str] | None = None,
                       argv: Iterable[str] = (),
                       overrides: Mapping[str, Any] | None = None) -> Configuration:
    """``WebApplication.CreateBuilder`` configuration defaults."""
    cfg = Configuration()
    env_name = environment_name(environ)
    if content_root is not None:
        root = Path(content_root)
        cfg.add_json_file(root / "appsettings.json")
        cfg.add_json_file(root / f"appsettings.{env_name}.json")
    cfg.add_environment(environ)
    cfg.add_command_line(argv)
    if overrides:
        cfg.add(overrides)
    cfg.set("Environment", env_name)
    return cfg
