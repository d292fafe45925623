"""Module 12 (optimise containers): OCI images of the services built without Docker.

The reference's only measured numbers are image sizes (reference
docs/aca/12-optimize-containers/index.md:318-326).  Here the Backend API is packaged as a
``standard`` and a ``chiseled`` image; the archive must be a valid OCI layout (digests match),
the chiseled image must carry no shell and no Python sources and run as non-root, and -- when
the test runs as root -- both images must serve module 1's acceptance request from inside their
own root filesystem (``chroot``), with the native extension loaded."""
import gzip
import hashlib
import io
import json
import os
import tarfile

import pytest

from aca_dotnet_workshop_amd.platform import image


def _read(archive):
    with tarfile.open(archive) as tf:
        blobs = {m.name: tf.extractfile(m).read() for m in tf.getmembers() if m.isfile()}
    return blobs


@pytest.fixture(scope="module")
def built(tmp_path_factory):
    out = tmp_path_factory.mktemp("images")
    closure = image.full_closure("backend_api")
    return {v: image.build_image("backend_api", v, out, closure) for v in ("standard", "chiseled")}


def test_oci_layout_is_consistent(built):
    for r in built.values():
        blobs = _read(r.path)
        assert json.loads(blobs["oci-layout"]) == {"imageLayoutVersion": "1.0.0"}
        index = json.loads(blobs["index.json"])
        md = index["manifests"][0]["digest"]
        man_raw = blobs[f"blobs/sha256/{md.split(':')[1]}"]
        assert "sha256:" + hashlib.sha256(man_raw).hexdigest() == md == r.digest
        man = json.loads(man_raw)
        for d in [man["config"]] + man["layers"]:
            assert "sha256:" + hashlib.sha256(blobs[f"blobs/sha256/{d['digest'].split(':')[1]}"]).hexdigest() == d["digest"]
        cfg = json.loads(blobs[f"blobs/sha256/{man['config']['digest'].split(':')[1]}"])
        layer = gzip.decompress(blobs[f"blobs/sha256/{man['layers'][0]['digest'].split(':')[1]}"])
        assert cfg["rootfs"]["diff_ids"] == ["sha256:" + hashlib.sha256(layer).hexdigest()]
        assert cfg["config"]["Entrypoint"][-1] == "aca_dotnet_workshop_amd.services.backend_api"
        docker = json.loads(blobs["manifest.json"])  # docker-archive view of the same blobs
        assert docker[0]["RepoTags"] == [f"tasksmanager/tasksmanager-backend-api:{r.variant}"]


def test_chiseled_is_minimal_and_nonroot(built):
    std, ch = built["standard"], built["chiseled"]
    assert ch.uncompressed < std.uncompressed and ch.files < std.files
    blobs = _read(ch.path)
    index = json.loads(blobs["index.json"])
    man = json.loads(blobs[f"blobs/sha256/{index['manifests'][0]['digest'].split(':')[1]}"])
    cfg = json.loads(blobs[f"blobs/sha256/{man['config']['digest'].split(':')[1]}"])
    assert cfg["config"]["User"] == f"{image.NONROOT}:{image.NONROOT}"
    layer = gzip.decompress(blobs[f"blobs/sha256/{man['layers'][0]['digest'].split(':')[1]}"])
    with tarfile.open(fileobj=io.BytesIO(layer)) as lt:
        names = {m.name for m in lt.getmembers()}
    assert not any(n.endswith(("bin/sh", "bin/bash", "bin/dash")) for n in names)
    assert not any(n.endswith(".py") for n in names)  # sourceless
    assert "app/aca_dotnet_workshop_amd/services/backend_api/appsettings.json" in names
    assert any(n.startswith("app/aca_dotnet_workshop_amd/native/_ttnative") for n in names)
    assert not any(n.startswith("root/") for n in names)


@pytest.mark.skipif(os.geteuid() != 0, reason="chroot needs root")
@pytest.mark.parametrize("variant", ["standard", "chiseled"])
def test_image_runs_module1_acceptance(built, variant):  # every mode of MODES, incl. gRPC
    v = image.verify_image(built[variant].path, "backend_api")
    assert v["status"] == 200
    tasks = json.loads(v["body"])
    assert len(tasks) == 10 and all(t["taskCreatedBy"] == "tjoudeh@bitoftech.net" for t in tasks)
    # every mode (incl. the gRPC sidecar protocol) finds all the code its paths import
    assert [m["mode"] for m in v["modes"]] == image.MODES["backend_api"]
    assert all(m["clean"] for m in v["modes"]), v["log"][-3000:]


def test_module12_table_for_all_three_services(built, tmp_path_factory, capsys):
    """Module 12's table (docs/aca/12-optimize-containers/index.md:318-326) for every service on
    the current tree: standard vs chiseled -- files, uncompressed and compressed size, Python
    distributions, shared libraries -- printed (``pytest -s``) and the chiseled image smaller on
    every size axis.  The numbers are recorded in profiles/r6_container_images.md."""
    out = tmp_path_factory.mktemp("images3")
    rows = [r.row() for r in built.values()]
    for svc in ("processor", "frontend"):
        closure = image.full_closure(svc)
        rows += [image.build_image(svc, v, out, closure).row() for v in ("standard", "chiseled")]
    by = {(r["service"], r["variant"]): r for r in rows}
    with capsys.disabled():
        for r in rows:
            print(json.dumps({k: r[k] for k in ("service", "variant", "files", "uncompressed_mb", "compressed_mb",
                                                "python_distributions", "shared_libs")}))
    for svc in ("backend_api", "processor", "frontend"):
        std, ch = by[(svc, "standard")], by[(svc, "chiseled")]
        assert ch["files"] < std["files"] and ch["uncompressed_mb"] < std["uncompressed_mb"]
        assert ch["compressed_mb"] < std["compressed_mb"] and ch["shared_libs"] < std["shared_libs"]
        assert ch["python_distributions"] == std["python_distributions"]  # the same code, less base
