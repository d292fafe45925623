"""The workshop modules are executable: every ``bash run`` block of docs/modules/*.md runs and its
``text expect`` lines must appear (aca_dotnet_workshop_amd/utils/docrun.py).  This is how the
reference's manual acceptance checks (M1 10 tasks, M2 403, M4 204 + value, M5 204 +
processor log, M6 blob, M7 cron logs, M9 1 -> 5 -> 1 replicas) are kept true."""
import fcntl
from pathlib import Path

import pytest

from aca_dotnet_workshop_amd.utils.docrun import _check, parse, run_doc

ROOT = Path(__file__).resolve().parents[1]
DOCS = sorted(p for p in (ROOT / "docs" / "modules").glob("*.md") if any(b.kind == "run" for b in parse(p.read_text())))


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
    assert {"01-deploy-api.md"} <= names


@pytest.mark.parametrize("doc", DOCS, ids=lambda p: p.stem)
def test_walkthrough(doc, tmp_path):
    # the walkthroughs use the reference's fixed ports (7088, 3500, ...): one at a time
    with open("/tmp/tt-docs-walkthrough.lock", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        failures = run_doc(doc)
    assert not failures, "\n\n".join(failures)
