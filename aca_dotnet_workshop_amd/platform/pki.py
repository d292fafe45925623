"""Environment PKI: the certificate authority of a Container Apps environment.

ACA terminates TLS at the environment's ingress (HTTPS for external ingress, HTTP redirected
to HTTPS unless ``allowInsecure``) and Dapr runs mutual TLS between sidecars with
certificates issued per app-id by its Sentry CA (reference docs/aca/03-aca-dapr-integration/
index.md:36).  ``EnvironmentPki`` is that CA, built with the ``openssl`` command line:

* ``ca.crt`` / ``ca.key``     -- the environment root (EC P-256, 10 years);
* ``workload(app_id)``        -- a sidecar identity: SAN ``DNS:<app-id>`` and
  ``URI:spiffe://<trust-domain>/ns/default/<app-id>``, usable as TLS server *and* client
  certificate (``serverAuth, clientAuth``) -- what both ends of a sidecar-to-sidecar call
  present and verify;
* ``server(name, hosts)``     -- the ingress / app certificate for ``localhost`` /
  ``127.0.0.1`` and the given names.

Issued files are cached under the directory; keys are created 0600.
"""
from __future__ import annotations

import os
import ssl
import subprocess
from dataclasses import dataclass
from pathlib import Path


class PkiError(RuntimeError):
    pass


@dataclass(frozen=True)
class CertPair:
    cert: str
    key: str
    ca: str

    def server_context(self, require_client_cert: bool = False) -> ssl.SSLContext:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        ctx.load_cert_chain(self.cert, self.key)
        if require_client_cert:
            ctx.load_verify_locations(self.ca)
            ctx.verify_mode = ssl.CERT_REQUIRED
        return ctx

    def client_context(self, present_cert: bool = True) -> ssl.SSLContext:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        ctx.load_verify_locations(self.ca)
        if present_cert:
            ctx.load_cert_chain(self.cert, self.key)
        return ctx

    def as_config(self) -> dict[str, str]:
        return {"cert": self.cert, "key": self.key, "ca": self.ca}


def _openssl(*args: str, stdin: bytes | None = None) -> None:
    try:
        p = subprocess.run(["openssl", *args], input=stdin, capture_output=True, timeout=60)
    except FileNotFoundError as e:
        raise PkiError("the openssl command line is required for the environment PKI") from e
    if p.returncode != 0:
        raise PkiError(f"openssl {' '.join(args[:2])}: {p.stderr.decode(errors='replace')[-400:]}")


class EnvironmentPki:
    def __init__(self, directory: str | os.PathLike, trust_domain: str = "taskstracker.local") -> None:
        self.dir = Path(directory)
        self.dir.mkdir(parents=True, exist_ok=True)
        os.chmod(self.dir, 0o700)
        self.trust_domain = trust_domain
        self.ca_crt = self.dir / "ca.crt"
        self.ca_key = self.dir / "ca.key"
        if not (self.ca_crt.exists() and self.ca_key.exists()):
            self._make_ca()

    def _newkey(self, path: Path) -> None:
        old = os.umask(0o077)
        try:
            _openssl("ecparam", "-name", "prime256v1", "-genkey", "-noout", "-out", str(path))
        finally:
            os.umask(old)

    def _make_ca(self) -> None:
        self._newkey(self.ca_key)
        _openssl("req", "-x509", "-new", "-key", str(self.ca_key), "-sha256", "-days", "3650",
                 "-subj", f"/O=Container Apps environment/CN={self.trust_domain} root",
                 "-addext", "basicConstraints=critical,CA:TRUE", "-addext", "keyUsage=critical,keyCertSign,cRLSign",
                 "-out", str(self.ca_crt))

    def _issue(self, name: str, cn: str, sans: list[str], usage: str, days: int = 825) -> CertPair:
        crt, key, csr, ext = (self.dir / f"{name}.crt", self.dir / f"{name}.key", self.dir / f"{name}.csr",
                              self.dir / f"{name}.ext")
        if crt.exists() and key.exists():
            return CertPair(str(crt), str(key), str(self.ca_crt))
        self._newkey(key)
        _openssl("req", "-new", "-key", str(key), "-subj", f"/O={self.trust_domain}/CN={cn}", "-out", str(csr))
        ext.write_text("basicConstraints=critical,CA:FALSE\nkeyUsage=critical,digitalSignature,keyEncipherment\n"
                       f"extendedKeyUsage={usage}\nsubjectAltName={','.join(sans)}\n")
        _openssl("x509", "-req", "-in", str(csr), "-CA", str(self.ca_crt), "-CAkey", str(self.ca_key),
                 "-CAcreateserial", "-days", str(days), "-sha256", "-extfile", str(ext), "-out", str(crt))
        csr.unlink(missing_ok=True)
        ext.unlink(missing_ok=True)
        return CertPair(str(crt), str(key), str(self.ca_crt))

    def workload(self, app_id: str) -> CertPair:
        """Sidecar identity for ``app_id`` (server + client auth)."""
        return self._issue(f"workload-{app_id}", app_id,
                           [f"DNS:{app_id}", f"URI:spiffe://{self.trust_domain}/ns/default/{app_id}"],
                           "serverAuth,clientAuth")

    def server(self, name: str, hosts: list[str] = ()) -> CertPair:
        """TLS server certificate (ingress, ``--app-ssl`` apps) for localhost + ``hosts``."""
        sans = ["DNS:localhost", "IP:127.0.0.1", *[f"DNS:{h}" for h in hosts if h]]
        return self._issue(f"server-{name}", name, sans, "serverAuth")
