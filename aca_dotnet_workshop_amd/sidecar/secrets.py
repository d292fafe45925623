"""Secret store components and the secrets building block.

Types:
* ``secretstores.azure.keyvault`` -- vault in the backing emulator (reference
  aca-components/containerapps-secretstore-kv.yaml:1-7, bicep dapr-components.bicep:73-90);
* ``secretstores.local.file``   -- JSON file, nested keys flattened with ``nestedSeparator``;
* ``secretstores.local.env``    -- process environment;
* the built-in ACA *app secrets* store used for ``secretRef`` entries of components that
  name no ``secretStoreComponent`` (ACA ``secrets:`` + ``secretRef``, reference
  processor-backend-service.bicep:121-130); it reads ``TT_APP_SECRETS`` (JSON object).
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Any

from .base import ComponentBase, RuntimeContext, register
from .components import Component, ComponentError

APP_SECRETS_STORE = "__aca_app_secrets__"


class SecretStore(ComponentBase):
    async def get(self, key: str, metadata: dict[str, str] | None = None) -> dict[str, str] | None:
        raise NotImplementedError

    async def bulk(self) -> dict[str, dict[str, str]]:
        raise NotImplementedError


def _flatten(prefix: str, v: Any, sep: str, out: dict[str, str]) -> None:
    if isinstance(v, dict):
        for k, x in v.items():
            _flatten(f"{prefix}{sep}{k}" if prefix else str(k), x, sep, out)
    else:
        out[prefix] = v if isinstance(v, str) else json.dumps(v)


@register("secretstores.local.file")
class LocalFileSecretStore(SecretStore):
    async def init(self) -> None:
        path = self.comp.get("secretsFile")
        if not path:
            raise ComponentError(f"{self.name}: secretsFile is required")
        p = Path(path)
        if not p.is_absolute() and self.comp.source and self.comp.source != "<inline>":
            cand = Path(self.comp.source).parent / p
            if cand.exists():
                p = cand
        data = json.loads(p.read_text())
        self.multi = self.comp.get_bool("multiValued")
        self.data: dict[str, Any] = data
        self.flat: dict[str, str] = {}
        _flatten("", data, self.comp.get("nestedSeparator", ":") or ":", self.flat)

    async def get(self, key, metadata=None):
        if self.multi and isinstance(self.data.get(key), dict):
            return {k: (v if isinstance(v, str) else json.dumps(v)) for k, v in self.data[key].items()}
        v = self.flat.get(key)
        return None if v is None else {key: v}

    async def bulk(self):
        return {k: {k: v} for k, v in self.flat.items()}


@register("secretstores.local.env")
class EnvSecretStore(SecretStore):
    async def init(self) -> None:
        self.prefix = self.comp.get("prefix", "") or ""

    async def get(self, key, metadata=None):
        v = self.ctx.environ.get(self.prefix + key)
        return None if v is None else {key: v}

    async def bulk(self):
        return {k[len(self.prefix):]: {k[len(self.prefix):]: v} for k, v in self.ctx.environ.items()
                if k.startswith(self.prefix)}


@register("secretstores.azure.keyvault")
class KeyVaultSecretStore(SecretStore):
    async def init(self) -> None:
        self.vault = self.comp.get("vaultName")
        if not self.vault:
            raise ComponentError(f"{self.name}: vaultName is required")
        self.client = self.ctx.backing(self.comp)

    async def get(self, key, metadata=None):
        v = await self.client.kv_get(self.vault, key)
        return None if v is None else {key: v}

    async def bulk(self):
        out = {}
        for name in await self.client.kv_list(self.vault):
            v = await self.client.kv_get(self.vault, name)
            if v is not None:
                out[name] = {name: v}
        return out


class AppSecretsStore(SecretStore):
    """ACA container-app secrets (``secrets:`` on the app, referenced by ``secretRef``)."""

    def __init__(self, ctx: RuntimeContext) -> None:
        super().__init__(Component(APP_SECRETS_STORE, "secretstores.aca.appsecrets"), ctx)
        raw = ctx.environ.get("TT_APP_SECRETS", "")
        self.secrets: dict[str, str] = json.loads(raw) if raw else {}

    async def get(self, key, metadata=None):
        v = self.secrets.get(key)
        return None if v is None else {key: v}

    async def bulk(self):
        return {k: {k: v} for k, v in self.secrets.items()}
