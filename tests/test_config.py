"""Layered configuration (ASP.NET Core semantics) and SDK endpoint resolution."""
import json

import pytest

from aca_dotnet_workshop_amd.sdk.client import sidecar_base_url
from aca_dotnet_workshop_amd.utils.config import Configuration, environment_name, load_configuration


def test_layering_env_and_command_line(tmp_path):
    (tmp_path / "appsettings.json").write_text(json.dumps({
        "Logging": {"LogLevel": {"Default": "Information"}}, "SendGrid": {"IntegrationEnabled": False},
        "BackendApiConfig": {"BaseUrlExternalHttp": "https://x"}}))
    (tmp_path / "appsettings.Development.json").write_text(json.dumps({"Logging": {"LogLevel": {"Default": "Debug"}}}))
    env = {"ASPNETCORE_ENVIRONMENT": "Development", "SendGrid__IntegrationEnabled": "true"}
    cfg = load_configuration(tmp_path, environ=env, argv=["--BackendApiConfig:BaseUrlExternalHttp=https://y"])
    assert cfg.get("Environment") == "Development"
    assert cfg.get_str("logging:loglevel:default") == "Debug"        # case-insensitive, env file layered
    assert cfg.get_bool("SendGrid:IntegrationEnabled") is True        # env var with __ separator wins
    assert cfg.get_str("BackendApiConfig:BaseUrlExternalHttp") == "https://y"  # command line wins
    assert cfg.section("Logging") == {"LogLevel": {"Default": "Debug"}}
    with pytest.raises(ValueError):
        Configuration([{"x": "maybe"}]).get_bool("x")
    assert environment_name({}) == "Production"


def test_sidecar_endpoint_resolution():
    assert sidecar_base_url({}) == "http://127.0.0.1:3500"
    assert sidecar_base_url({"DAPR_HTTP_PORT": "3501"}) == "http://127.0.0.1:3501"
    assert sidecar_base_url({"TT_SIDECAR_UDS": "/tmp/s.sock"}) == "unix:/tmp/s.sock:"


def test_tune_gc_knob():
    import gc
    from aca_dotnet_workshop_amd.services.hosting import tune_gc
    before = gc.get_threshold()
    try:
        assert tune_gc({"TT_GC_GEN0": "0"}) is False and gc.get_threshold() == before
        assert tune_gc({"TT_GC_GEN0": "12345"}) is True and gc.get_threshold()[0] == 12345
    finally:
        gc.unfreeze()
        gc.set_threshold(*before)
