"""The workshop modules are executable: every ``bash run`` block of docs/modules/*.md runs and its
``text expect`` lines must appear (aca_dotnet_workshop_amd/utils/docrun.py).  This is how the
reference's manual acceptance checks (M1 10 tasks, M2 403, M4 204 + value, M5 204 +
processor log, M6 blob, M7 cron logs, M9 1 -> 5 -> 1 replicas) are kept true."""
import fcntl
import re
from pathlib import Path

import pytest

from aca_dotnet_workshop_amd.utils.docrun import _check, parse, run_doc

ROOT = Path(__file__).resolve().parents[1]
# every module in the site's nav (mkdocs.yml), whether or not docs/ is in this checkout: the GPU
# box's snapshot leaves docs/ out (.gpurunignore), and its walkthroughs are then skipped, not
# silently uncollected
NAV = sorted(set(re.findall(r"modules/(\d\d-[\w-]+\.md)", (ROOT / "mkdocs.yml").read_text())))
DOCS = [ROOT / "docs" / "modules" / n for n in NAV]


def test_docrun_parser_and_matcher():
    blocks = parse("x\n```bash run timeout=5\necho hi\n```\n```text expect\nh\n...\nre: ^b+$\n```\n"
                   "```bash\nnot run\n```\n```bash cleanup\nrm -f x\n```\n")
    assert [(b.kind, b.code, b.timeout) for b in blocks] == [("run", "echo hi", 5.0), ("cleanup", "rm -f x", 60.0)]
    assert blocks[0].expect == ["h", "re: ^b+$"]
    assert _check(["a", "b", "re: ^c\\d$"], "xa\nb\nc1") is None
    assert _check(["b", "a"], "a\nb") == "a"               # order matters
    assert _check(["open", "api"], "openapi 3 ['/api']") is None  # same line may satisfy several


def test_walkthroughs_exist():
    names = {p.name for p in DOCS}
    assert {"01-deploy-api.md", "09-autoscale.md"} <= names and len(names) == 13


@pytest.mark.parametrize("doc", DOCS, ids=lambda p: p.stem)
def test_walkthrough(doc, tmp_path):
    if not doc.exists():
        pytest.skip(f"{doc.name}: docs/ is not part of this checkout")
    if not any(b.kind == "run" for b in parse(doc.read_text())):
        pytest.skip(f"{doc.name}: no executable blocks")
    # the walkthroughs use the reference's fixed ports (7088, 3500, ...): one at a time
    with open("/tmp/tt-docs-walkthrough.lock", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        failures = run_doc(doc)
    assert not failures, "\n\n".join(failures)
