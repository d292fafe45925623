"""Executable workshop modules: run the fenced commands of a Markdown walkthrough and check
their outputs, so the docs cannot rot.

The reference's modules (docs/aca/*/index.md) are walkthroughs whose acceptance checks are
manual ("you should see 10 tasks", "the response is 403").  Ours are executed:

* a fenced block whose info string is ``bash run`` is executed (in order, in ONE bash
  session per document, from the repository root, so ``export`` and background ``&``
  processes carry over to later blocks); ``bash run timeout=120`` raises the block's budget;
* a ``text expect`` block right after it lists lines that must appear in that block's output,
  in order, each as a substring of some output line (``...`` lines are skipped; a line
  starting with ``re:`` is a regular expression; consecutive expectations may match the same
  output line);
* ``bash cleanup`` blocks always run at the end, even after a failure (``platform down``);
* any other fence (plain ``bash``, ``yaml``, ...) is documentation only.

A block fails when its last command exits non-zero (use ``|| true`` where a failure is the
point) or an expected line is missing.  Every process the session starts is in its own
process group, which is killed when the document finishes.

    python -m aca_dotnet_workshop_amd.utils.docrun docs/modules/04-state-api.md [...]
"""
from __future__ import annotations

import argparse
import os
import re
import signal
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field
from pathlib import Path

REPO_ROOT = Path(__file__).resolve().parents[2]
_FENCE = re.compile(r"^(\s*)(`{3,}|~{3,})\s*([^`]*)$")


@dataclass
class Block:
    kind: str            # run | cleanup
    code: str
    line: int            # 1-based line of the opening fence
    timeout: float = 60.0
    expect: list[str] = field(default_factory=list)


def parse(text: str) -> list[Block]:
    blocks: list[Block] = []
    lines = text.splitlines()
    i = 0
    while i < len(lines):
        m = _FENCE.match(lines[i])
        if not m:
            i += 1
            continue
        indent, fence, info = m.group(1), m.group(2), m.group(3).strip().split()
        body, j = [], i + 1
        while j < len(lines) and not lines[j].strip().startswith(fence):
            body.append(lines[j][len(indent):] if lines[j].startswith(indent) else lines[j])
            j += 1
        lang = info[0] if info else ""
        flags = info[1:]
        if lang in ("bash", "sh", "console") and ("run" in flags or "cleanup" in flags):
            b = Block("cleanup" if "cleanup" in flags else "run", "\n".join(body), i + 1)
            for f in flags:
                if f.startswith("timeout="):
                    b.timeout = float(f.split("=", 1)[1])
            blocks.append(b)
        elif lang == "text" and "expect" in flags:
            prev = next((b for b in reversed(blocks) if b.kind == "run"), None)
            if prev is None:
                raise ValueError(f"line {i + 1}: 'text expect' without a preceding 'bash run' block")
            prev.expect.extend(x.strip() for x in body if x.strip() and x.strip() != "...")
        i = j + 1
    return blocks


def _script(blocks: list[Block]) -> str:
    out = ["set -o pipefail", f"cd {REPO_ROOT}", "export PYTHONPATH=\"$PWD${PYTHONPATH:+:$PYTHONPATH}\"",
           "__tt_cleanup() {"]
    cleanup = [(k, b) for k, b in enumerate(blocks) if b.kind == "cleanup"]
    for k, b in cleanup:
        out += [f"echo '@@TT {k} BEGIN@@'", b.code, f"echo \"@@TT {k} END $?@@\""]
    out += [":", "}", "trap __tt_cleanup EXIT"]
    for k, b in enumerate(blocks):
        if b.kind != "run":
            continue
        out += [f"echo '@@TT {k} BEGIN@@'", b.code, f"echo \"@@TT {k} END $?@@\""]
    return "\n".join(out) + "\n"


def _check(expect: list[str], output: str) -> str | None:
    """None when every expected line appears in order (several may match the same output
    line); else the first missing one."""
    lines = output.splitlines()
    pos = 0
    for e in expect:
        rx = re.compile(e[3:].strip()) if e.startswith("re:") else None
        while pos < len(lines) and not (rx.search(lines[pos]) if rx else e in lines[pos]):
            pos += 1
        if pos == len(lines):
            return e
    return None


def run_doc(path: str | os.PathLike, env: dict[str, str] | None = None, verbose: bool = False) -> list[str]:
    """Run one document; returns failure descriptions (empty = pass)."""
    path = Path(path)
    blocks = parse(path.read_text())
    if not any(b.kind == "run" for b in blocks):
        return []
    budget = sum(b.timeout for b in blocks) + 30
    with tempfile.TemporaryDirectory(prefix="tt-doc-") as tmp:
        script = Path(tmp) / "doc.sh"
        script.write_text(_script(blocks))
        e = dict(os.environ, **(env or {}), TT_DOC_TMP=tmp)
        p = subprocess.Popen(["bash", str(script)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=e,
                             start_new_session=True, cwd=REPO_ROOT)
        t0 = time.monotonic()
        try:
            raw, _ = p.communicate(timeout=budget)
            timed_out = False
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGTERM)
            raw, _ = p.communicate()
            timed_out = True
        finally:
            try:  # background servers the walkthrough started
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
    text = raw.decode(errors="replace")
    if verbose:
        sys.stdout.write(text)
    outputs: dict[int, tuple[str, int | None]] = {}
    cur, buf = None, []
    for ln in text.splitlines():
        m = re.fullmatch(r"@@TT (\d+) (BEGIN|END)(?: (\d+))?@@", ln.strip())
        if m:
            k = int(m.group(1))
            if m.group(2) == "BEGIN":
                cur, buf = k, []
            else:
                outputs[k] = ("\n".join(buf), int(m.group(3)))
                cur = None
            continue
        if cur is not None:
            buf.append(ln)
    if cur is not None:
        outputs[cur] = ("\n".join(buf), None)
    failures = []
    for k, b in enumerate(blocks):
        if b.kind != "run":
            continue
        where = f"{path.name}:{b.line}"
        if k not in outputs:
            failures.append(f"{where}: block did not run (an earlier block stopped the session)")
            break
        out, rc = outputs[k]
        if rc is None:
            failures.append(f"{where}: block did not finish{' (timeout)' if timed_out else ''}\n{b.code}\n--- output\n{out[-3000:]}")
            break
        if rc != 0:
            failures.append(f"{where}: exit status {rc}\n{b.code}\n--- output\n{out[-3000:]}")
            continue
        missing = _check(b.expect, out)
        if missing is not None:
            failures.append(f"{where}: expected {missing!r}\n{b.code}\n--- output\n{out[-3000:]}")
    if verbose:
        print(f"{path}: {len(failures)} failure(s) in {time.monotonic() - t0:.1f}s", file=sys.stderr)
    return failures


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="docrun", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("docs", nargs="+")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    bad = 0
    for d in a.docs:
        fails = run_doc(d, verbose=a.verbose)
        for f in fails:
            print(f"FAIL {f}\n", file=sys.stderr)
        bad += bool(fails)
        print(f"{'FAIL' if fails else 'ok  '} {d}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
