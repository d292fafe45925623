"""Access control for the backing services: account keys and managed-identity RBAC.

Reference parity:
* Backend API identity: "Cosmos DB Built-in Data Contributor" on the account and
  "Azure Service Bus Data Sender" on the topic (webapi-backend-service.bicep:146-165);
* Processor identity: "Azure Service Bus Data Receiver" (processor-backend-service.bicep:190-198)
  and "Key Vault Secrets User" (secrets/processor-backend-service-secrets.bicep:66-74);
* self-hosted components authenticate with keys / connection strings instead
  (components/dapr-statestore-cosmos.yaml:11-12 ``masterKey``).

A request carries ``x-tt-identity: <principal>`` (managed identity) and/or
``x-tt-key: <key>``.  In ``open`` mode (local dev, the default) everything is allowed;
in ``enforce`` mode a request needs either the resource's key or a role assignment whose
scope is a prefix of the resource scope.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any

ROLE_ACTIONS: dict[str, set[str]] = {
    "Cosmos DB Built-in Data Contributor": {"cosmos.read", "cosmos.write"},
    "Cosmos DB Built-in Data Reader": {"cosmos.read"},
    "Azure Service Bus Data Sender": {"sb.send"},
    "Azure Service Bus Data Receiver": {"sb.receive"},
    "Azure Service Bus Data Owner": {"sb.send", "sb.receive", "sb.manage"},
    "Key Vault Secrets User": {"kv.get"},
    "Key Vault Secrets Officer": {"kv.get", "kv.set"},
    "Storage Queue Data Contributor": {"queue.send", "queue.receive"},
    "Storage Blob Data Contributor": {"blob.read", "blob.write"},
    "Owner": {"*"},
}


@dataclass
class RoleAssignment:
    principal: str
    role: str
    scope: str


@dataclass
class AccessPolicy:
    mode: str = "open"
    assignments: list[RoleAssignment] = field(default_factory=list)
    keys: dict[str, str] = field(default_factory=dict)  # scope -> key

    @classmethod
    def from_dict(cls, d: dict[str, Any] | None) -> "AccessPolicy":
        d = d or {}
        return cls(mode=d.get("mode", "open"),
                   assignments=[RoleAssignment(a["principal"], a["role"], a["scope"]) for a in d.get("roleAssignments", [])],
                   keys=dict(d.get("keys", {})))

    def to_dict(self) -> dict[str, Any]:
        return {"mode": self.mode, "keys": self.keys,
                "roleAssignments": [{"principal": a.principal, "role": a.role, "scope": a.scope} for a in self.assignments]}

    def check(self, action: str, scope: str, identity: str | None, key: str | None) -> bool:
        if self.mode != "enforce":
            return True
        if key:
            for kscope, k in self.keys.items():
                if scope.startswith(kscope) and key == k:
                    return True
        if identity:
            for a in self.assignments:
                if a.principal != identity or not scope.startswith(a.scope):
                    continue
                acts = ROLE_ACTIONS.get(a.role, set())
                if "*" in acts or action in acts:
                    return True
        return False
