"""A local container registry -- the Azure Container Registry of the reference's deployment.

The reference builds its three images into ACR (`az acr build`, docs/aca/01-deploy-api-to-aca),
or imports them from GHCR in CI (.github/workflows/infra-deploy.yml `create-acr`), and the
container apps pull them through a user-assigned managed identity holding **AcrPull**
(bicep/modules/container-apps.bicep:113-127, container-apps/*.bicep `registries:` blocks).

Here a registry is a directory (``<root>/<name>/``) with the layout of an OCI distribution
store: content-addressed blobs shared by all repositories, manifests by digest, and tags per
repository.  ``push`` takes the OCI image-layout archives ``platform image`` builds; ``resolve``
turns ``<name>.azurecr.io/<repo>:<tag>`` or ``...@sha256:<digest>`` into a manifest digest;
``unpack`` extracts an image's root filesystem once per digest into a cache.  Pull permission is
the platform's business (it checks the app identity's AcrPull role before calling ``unpack``).
"""
from __future__ import annotations

import gzip
import hashlib
import io
import json
import os
import shutil
import tarfile
import tempfile
from pathlib import Path
from typing import Any

LOGIN_SUFFIX = ".azurecr.io"


class RegistryError(Exception):
    pass


def default_root() -> Path:
    """``$TT_CONTAINER_REGISTRY_ROOT`` or a per-user directory: registries outlive environments,
    like ACR outlives a resource group's container apps."""
    env = os.environ.get("TT_CONTAINER_REGISTRY_ROOT")
    return Path(env) if env else Path(tempfile.gettempdir()) / f"tt-acr-{os.getuid()}"


def _sha(b: bytes) -> str:
    return "sha256:" + hashlib.sha256(b).hexdigest()


class LocalRegistry:
    def __init__(self, name: str, root: str | os.PathLike | None = None) -> None:
        if not name or "/" in name:
            raise RegistryError(f"bad registry name {name!r}")
        self.name = name
        self.dir = Path(root or default_root()) / name
        self.login_server = f"{name}{LOGIN_SUFFIX}"

    # ------------------------------------------------------------------ layout
    def _blob(self, digest: str) -> Path:
        algo, hexd = digest.split(":", 1)
        if algo != "sha256" or len(hexd) != 64 or any(c not in "0123456789abcdef" for c in hexd):
            raise RegistryError(f"bad digest {digest!r}")
        return self.dir / "blobs" / "sha256" / hexd

    def _tag_file(self, repo: str, tag: str) -> Path:
        if ".." in repo.split("/") or not tag or "/" in tag:
            raise RegistryError(f"bad reference {repo}:{tag}")
        return self.dir / "repositories" / repo / "tags" / tag

    def _put_blob(self, data: bytes) -> str:
        d = _sha(data)
        p = self._blob(d)
        if not p.exists():
            p.parent.mkdir(parents=True, exist_ok=True)
            tmp = p.with_suffix(f".tmp{os.getpid()}")
            tmp.write_bytes(data)
            os.replace(tmp, p)
        return d

    def read_blob(self, digest: str) -> bytes:
        p = self._blob(digest)
        if not p.exists():
            raise RegistryError(f"blob {digest} not found in {self.login_server}")
        data = p.read_bytes()
        if _sha(data) != digest:
            raise RegistryError(f"blob {digest} is corrupt")
        return data

    # ------------------------------------------------------------------ push / resolve
    def push(self, archive: str | os.PathLike, repo: str, tag: str = "latest") -> str:
        """``docker push`` of an OCI image-layout archive; returns the manifest digest."""
        self.create()  # a push to a registry nobody created yet creates it (the dev-loop shortcut)
        with tarfile.open(archive) as tf:
            index = json.load(tf.extractfile("index.json"))
            man_digest = index["manifests"][0]["digest"]

            def blob(d: str) -> bytes:
                return tf.extractfile("blobs/sha256/" + d.split(":", 1)[1]).read()
            man_bytes = blob(man_digest)
            man = json.loads(man_bytes)
            for ref in [man["config"]] + man["layers"]:
                data = blob(ref["digest"])
                if _sha(data) != ref["digest"]:
                    raise RegistryError(f"{archive}: blob {ref['digest']} does not match its digest")
                self._put_blob(data)
        if self._put_blob(man_bytes) != man_digest:
            raise RegistryError(f"{archive}: manifest digest mismatch")
        tf_ = self._tag_file(repo, tag)
        tf_.parent.mkdir(parents=True, exist_ok=True)
        tf_.write_text(man_digest)
        return man_digest

    def parse_ref(self, ref: str) -> tuple[str, str]:
        """``<login server>/<repo>[:tag|@digest]`` -> (repo, tag or digest)."""
        server, _, rest = ref.partition("/")
        if server != self.login_server or not rest:
            raise RegistryError(f"{ref!r} is not an image of {self.login_server}")
        if "@" in rest:
            repo, digest = rest.split("@", 1)
            return repo, digest
        repo, _, tag = rest.partition(":")
        return repo, tag or "latest"

    def resolve(self, ref: str) -> str:
        repo, what = self.parse_ref(ref)
        if what.startswith("sha256:"):
            self._blob(what)
            return what
        p = self._tag_file(repo, what)
        if not p.exists():
            raise RegistryError(f"manifest unknown: {ref}")
        return p.read_text().strip()

    def manifest(self, digest: str) -> dict[str, Any]:
        return json.loads(self.read_blob(digest))

    def config(self, digest: str) -> dict[str, Any]:
        return json.loads(self.read_blob(self.manifest(digest)["config"]["digest"]))

    def repositories(self) -> list[dict[str, Any]]:
        out = []
        base = self.dir / "repositories"
        if not base.exists():
            return out
        for tags in sorted(base.rglob("tags")):
            repo = str(tags.parent.relative_to(base))
            out.append({"repository": repo, "tags": {t.name: t.read_text().strip() for t in sorted(tags.iterdir())}})
        return out

    # ------------------------------------------------------------------ create / import
    def exists(self) -> bool:
        return (self.dir / "registry.json").exists()

    def create(self, sku: str = "Basic") -> bool:
        """``az acr create``: True when the registry was created, False when it already existed."""
        if self.exists():
            return False
        self.dir.mkdir(parents=True, exist_ok=True)
        tmp = self.dir / "registry.json.tmp"
        tmp.write_text(json.dumps({"name": self.name, "loginServer": self.login_server, "sku": sku}))
        os.replace(tmp, self.dir / "registry.json")
        return True

    def import_image(self, source: "LocalRegistry", ref: str, image: str, force: bool = False) -> str:
        """``az acr import --source <source>/<repo>:<tag> --image <repo>[:tag]``: copy the manifest
        and its blobs from another registry, tag it here; returns the manifest digest."""
        digest = source.resolve(ref)
        repo, _, tag = image.partition(":")
        tag = tag or "latest"
        tf_ = self._tag_file(repo, tag)
        if tf_.exists() and not force and tf_.read_text().strip() != digest:
            raise RegistryError(f"{self.login_server}/{repo}:{tag} exists (use force to overwrite)")
        man_bytes = source.read_blob(digest)
        man = json.loads(man_bytes)
        for ref_ in [man["config"]] + man["layers"]:
            self._put_blob(source.read_blob(ref_["digest"]))
        self._put_blob(man_bytes)
        tf_.parent.mkdir(parents=True, exist_ok=True)
        tf_.write_text(digest)
        return digest

    # ------------------------------------------------------------------ pull
    def unpack(self, digest: str, cache: str | os.PathLike) -> tuple[Path, dict[str, Any]]:
        """Root filesystem of the image (extracted once per digest under ``cache``) and its
        config.  Layers are verified against their digests before extraction."""
        man = self.manifest(digest)
        cfg = json.loads(self.read_blob(man["config"]["digest"]))
        root = Path(cache) / digest.split(":", 1)[1][:32] / "rootfs"
        done = root.parent / ".complete"
        if not done.exists():
            if root.exists():
                shutil.rmtree(root)
            root.mkdir(parents=True)
            root.chmod(0o755)
            for layer in man["layers"]:
                data = gzip.decompress(self.read_blob(layer["digest"]))
                with tarfile.open(fileobj=io.BytesIO(data)) as lt:
                    for m in lt.getmembers():  # no absolute paths / parent escapes from a layer
                        if m.name.startswith("/") or ".." in Path(m.name).parts:
                            raise RegistryError(f"layer {layer['digest']}: unsafe path {m.name!r}")
                    lt.extractall(root)
            done.write_text(digest)
        return root, cfg
