"""Run a CI/CD pipeline file locally: GitHub Actions workflows and Azure DevOps pipelines.

The reference's pipelines only ever run on hosted agents against Azure;
here the same graphs -- lint -> validate -> preview -> (create registry -> import images ->
deploy with registry images | deploy with published images) -> teardown -- drive the local
platform, so they can run, be tested and be shown.  The runner:

* loads ``jobs:`` (GitHub) or ``stages:`` -> ``jobs:`` (Azure DevOps; a stage is one node);
* orders them by ``needs`` / ``dependsOn`` and evaluates their ``if:`` / ``condition:`` with the
  given context (``vars``, ``inputs``/``parameters``, ``github``, ``env``, ``needs``) -- a node
  whose dependencies did not all succeed is skipped, as on the hosted runners;
* expands ``${{ ... }}`` (both dialects) and ``$(VAR)`` (Azure DevOps macros) in ``run:`` /
  ``script:`` steps and runs them with bash (``-e -o pipefail``) in the workspace, with
  ``$GITHUB_ENV`` / ``$GITHUB_OUTPUT`` honoured (step outputs -> job outputs -> ``needs``);
* expands a one-axis ``strategy.matrix`` into one run per value;
* emulates the actions the repo's workflows use: ``actions/checkout`` and
  ``actions/setup-python`` (no-ops: the workspace is the checkout) and ``dorny/paths-filter``
  (from ``github.changed_files``); any other ``uses:`` step is reported as not run.

    python -m aca_dotnet_workshop_amd.utils.pipeline .github/workflows/infra-deploy.yml \\
        --var CONTAINER_REGISTRY_NAME=taskstrackeracr --env ENV_DIR=/tmp/env
"""
from __future__ import annotations

import argparse
import fnmatch
import json
import os
import re
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any

import yaml

ROOT = Path(__file__).resolve().parents[2]


# ------------------------------------------------------------------------------------------
# expressions: GitHub's `${{ }}` language and Azure DevOps' condition functions, one parser
_TOKEN = re.compile(r"\s*(?:(?P<num>\d+(?:\.\d+)?)|(?P<str>'(?:[^']|'')*')|(?P<op>==|!=|&&|\|\||<=|>=|[!<>(),\[\]])"
                    r"|(?P<id>[A-Za-z_][A-Za-z0-9_\-]*(?:\.[A-Za-z0-9_\-*]+)*))")


class ExprError(Exception):
    pass


def _tokens(s: str) -> list[tuple[str, str]]:
    out, i = [], 0
    while i < len(s):
        m = _TOKEN.match(s, i)
        if not m or m.end() == i:
            if s[i:].strip() == "":
                break
            raise ExprError(f"cannot parse {s!r} at {s[i:]!r}")
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
        i = m.end()
    return out


def _truthy(v: Any) -> bool:
    if isinstance(v, str):
        return v != "" and v.lower() != "false"
    return bool(v)


def _loose_eq(a: Any, b: Any) -> bool:
    if isinstance(a, bool) or isinstance(b, bool):
        return _truthy(a) == _truthy(b) if isinstance(a, bool) and isinstance(b, bool) else \
            str(a).lower() == str(b).lower()
    if isinstance(a, str) and isinstance(b, str):
        return a.lower() == b.lower()
    try:
        return float(a) == float(b)
    except (TypeError, ValueError):
        return a == b


class Evaluator:
    def __init__(self, ctx: dict[str, Any], status: dict[str, Any] | None = None) -> None:
        self.ctx = ctx
        self.status = status or {}

    def eval(self, text: str) -> Any:
        self.t = _tokens(text)
        self.i = 0
        v = self._or()
        if self.i != len(self.t):
            raise ExprError(f"trailing tokens in {text!r}")
        return v

    def _peek(self) -> tuple[str, str] | None:
        return self.t[self.i] if self.i < len(self.t) else None

    def _take(self, val: str | None = None) -> tuple[str, str]:
        tok = self._peek()
        if tok is None or (val is not None and tok[1] != val):
            raise ExprError(f"expected {val!r}, got {tok!r}")
        self.i += 1
        return tok

    def _or(self) -> Any:
        v = self._and()
        while self._peek() and self._peek()[1] == "||":
            self._take()
            r = self._and()
            v = v if _truthy(v) else r
        return v

    def _and(self) -> Any:
        v = self._cmp()
        while self._peek() and self._peek()[1] == "&&":
            self._take()
            r = self._cmp()
            v = r if _truthy(v) else v
        return v

    def _cmp(self) -> Any:
        v = self._unary()
        while self._peek() and self._peek()[1] in ("==", "!=", "<", ">", "<=", ">="):
            op = self._take()[1]
            r = self._unary()
            if op == "==":
                v = _loose_eq(v, r)
            elif op == "!=":
                v = not _loose_eq(v, r)
            else:
                v = {"<": float(v) < float(r), ">": float(v) > float(r), "<=": float(v) <= float(r),
                     ">=": float(v) >= float(r)}[op]
        return v

    def _unary(self) -> Any:
        if self._peek() and self._peek()[1] == "!":
            self._take()
            return not _truthy(self._unary())
        return self._primary()

    def _primary(self) -> Any:
        kind, val = self._take()
        if kind == "num":
            return float(val) if "." in val else int(val)
        if kind == "str":
            return val[1:-1].replace("''", "'")
        if val == "(":
            v = self._or()
            self._take(")")
            return v
        if kind != "id":
            raise ExprError(f"unexpected {val!r}")
        if val in ("true", "True"):
            return True
        if val in ("false", "False"):
            return False
        if val == "null":
            return None
        if self._peek() and self._peek()[1] == "(":
            self._take("(")
            args = []
            while self._peek() and self._peek()[1] != ")":
                args.append(self._or())
                if self._peek() and self._peek()[1] == ",":
                    self._take(",")
            self._take(")")
            return self._call(val, args)
        v = self._lookup(val)
        while self._peek() and self._peek()[1] == "[":  # variables['X'] (Azure DevOps)
            self._take("[")
            key = self._or()
            self._take("]")
            v = (v or {}).get(key) if isinstance(v, dict) else None
        return v

    def _lookup(self, path: str) -> Any:
        cur: Any = self.ctx
        for part in path.split("."):
            if isinstance(cur, dict):
                cur = cur.get(part, cur.get(part.lower()) if isinstance(part, str) else None)
            else:
                return None
        return "" if cur is None and path.split(".")[0] in ("vars", "env", "secrets") else cur

    def _call(self, fn: str, args: list[Any]) -> Any:
        f = fn.lower()
        if f in ("success", "succeeded"):
            return self.status.get("deps_ok", True)
        if f == "failure" or f == "failed":
            return self.status.get("deps_failed", False)
        if f == "always":
            return True
        if f == "cancelled" or f == "canceled":
            return False
        if f == "eq":
            return _loose_eq(args[0], args[1])
        if f == "ne":
            return not _loose_eq(args[0], args[1])
        if f == "and":
            return all(_truthy(a) for a in args)
        if f == "or":
            return any(_truthy(a) for a in args)
        if f == "not":
            return not _truthy(args[0])
        if f == "contains":
            hay, needle = args
            if isinstance(hay, (list, tuple)):
                return any(_loose_eq(x, needle) for x in hay)
            return str(needle).lower() in str(hay).lower()
        if f == "startswith":
            return str(args[0]).lower().startswith(str(args[1]).lower())
        if f == "endswith":
            return str(args[0]).lower().endswith(str(args[1]).lower())
        if f == "fromjson":
            return json.loads(args[0]) if isinstance(args[0], str) and args[0] else args[0]
        if f == "tojson":
            return json.dumps(args[0])
        if f == "format":
            s = str(args[0])
            for i, a in enumerate(args[1:]):
                s = s.replace("{%d}" % i, str(a))
            return s
        raise ExprError(f"unknown function {fn}()")


_TEMPLATE = re.compile(r"\$\{\{\s*(.*?)\s*\}\}")
_MACRO = re.compile(r"\$\(([A-Za-z_][A-Za-z0-9_.]*)\)")


def expand(text: str, ev: Evaluator, macros: dict[str, str] | None = None) -> Any:
    """``${{ expr }}`` (a whole-string expression keeps its type) and ``$(VAR)`` macros."""
    if not isinstance(text, str):
        return text
    m = _TEMPLATE.fullmatch(text.strip())
    if m:
        return ev.eval(m.group(1))

    def fmt(v: Any) -> str:
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, (list, dict)):
            return json.dumps(v)
        return "" if v is None else str(v)
    out = _TEMPLATE.sub(lambda mm: fmt(ev.eval(mm.group(1))), text)
    if macros is not None:
        out = _MACRO.sub(lambda mm: macros.get(mm.group(1), mm.group(0)), out)
    return out


def condition(text: Any, ev: Evaluator) -> bool:
    if text is None:
        return _truthy(ev._call("success", []))
    if isinstance(text, bool):
        return text
    s = str(text).strip()
    m = _TEMPLATE.fullmatch(s)
    if m:
        s = m.group(1)
    s = _TEMPLATE.sub(lambda mm: repr(ev.eval(mm.group(1))) if not isinstance(ev.eval(mm.group(1)), bool)
                      else str(ev.eval(mm.group(1))).lower(), s)
    v = ev.eval(s)
    # GitHub: a job condition without a status function is ANDed with success()
    if not re.search(r"\b(success|succeeded|failure|failed|always|cancelled|canceled)\s*\(", s, re.I):
        return _truthy(v) and ev.status.get("deps_ok", True)
    return _truthy(v)


# ------------------------------------------------------------------------------------------
@dataclass
class Step:
    name: str
    run: str | None = None
    uses: str | None = None
    id: str | None = None
    cond: Any = None
    env: dict[str, str] = field(default_factory=dict)
    with_: dict[str, Any] = field(default_factory=dict)


@dataclass
class Job:
    name: str
    needs: list[str]
    cond: Any
    steps: list[Step]
    env: dict[str, str] = field(default_factory=dict)
    outputs: dict[str, str] = field(default_factory=dict)
    matrix: Any = None
    variables: dict[str, str] = field(default_factory=dict)


@dataclass
class Pipeline:
    kind: str
    name: str
    jobs: dict[str, Job]
    env: dict[str, str]
    parameters: dict[str, Any]


def _steps(raw: list[dict]) -> list[Step]:
    out = []
    for i, s in enumerate(raw or []):
        run = s.get("run") or s.get("script") or s.get("bash")
        out.append(Step(name=s.get("name") or s.get("displayName") or (run or s.get("uses") or f"step {i}").split("\n")[0][:60],
                        run=run, uses=s.get("uses"), id=s.get("id") or s.get("name"), cond=s.get("if", s.get("condition")),
                        env={k: str(v) for k, v in (s.get("env") or {}).items()}, with_=s.get("with") or {}))
    return out


def _variables(v: Any) -> dict[str, str]:
    if isinstance(v, dict):
        return {k: str(x) for k, x in v.items()}
    out = {}
    for item in v or []:
        if isinstance(item, dict) and "name" in item:
            out[item["name"]] = str(item.get("value", ""))
    return out


def load(path: str | os.PathLike) -> Pipeline:
    doc = yaml.safe_load(Path(path).read_text()) or {}
    if "jobs" in doc:  # GitHub Actions
        jobs = {}
        for name, j in doc["jobs"].items():
            needs = j.get("needs") or []
            jobs[name] = Job(name, [needs] if isinstance(needs, str) else list(needs), j.get("if"),
                             _steps(j.get("steps")), {k: str(v) for k, v in (j.get("env") or {}).items()},
                             dict(j.get("outputs") or {}), (j.get("strategy") or {}).get("matrix"))
        return Pipeline("github", doc.get("name", Path(path).stem), jobs,
                        {k: str(v) for k, v in (doc.get("env") or {}).items()}, {})
    if "stages" in doc:  # Azure DevOps: one node per stage (its jobs' steps in order)
        params = {p["name"]: p.get("default") for p in doc.get("parameters") or []}
        jobs = {}
        prev: str | None = None
        for st in doc["stages"]:
            name = st["stage"]
            dep = st.get("dependsOn", [prev] if prev else [])
            steps: list[Step] = []
            variables: dict[str, str] = _variables(st.get("variables"))
            for j in st.get("jobs") or []:
                steps += _steps(j.get("steps"))
                variables.update(_variables(j.get("variables")))
            jobs[name] = Job(name, [dep] if isinstance(dep, str) else list(dep or []), st.get("condition"), steps,
                             variables=variables)
            prev = name
        return Pipeline("ado", Path(path).stem, jobs, _variables(doc.get("variables")), params)
    raise ValueError(f"{path}: neither a GitHub workflow (jobs:) nor an Azure DevOps pipeline (stages:)")


@dataclass
class Result:
    job: str
    status: str               # success | failure | skipped
    seconds: float = 0.0
    steps: list[dict] = field(default_factory=list)
    outputs: dict[str, str] = field(default_factory=dict)
    matrix: Any = None


def _paths_filter(step: Step, ctx: dict[str, Any]) -> dict[str, str]:
    filters = step.with_.get("filters")
    filters = yaml.safe_load(filters) if isinstance(filters, str) else (filters or {})
    changed = list((ctx.get("github") or {}).get("changed_files") or [])
    hits = [name for name, pats in filters.items()
            if any(fnmatch.fnmatch(f, p) or fnmatch.fnmatch(f, p.rstrip("*").rstrip("/") + "/*") for f in changed
                   for p in (pats if isinstance(pats, list) else [pats]))]
    out = {"changes": json.dumps(hits)}
    out.update({name: "true" if name in hits else "false" for name in filters})
    return out


def run(pipeline: Pipeline, ctx: dict[str, Any] | None = None, workdir: str | os.PathLike = ROOT,
        env_overrides: dict[str, str] | None = None, timeout: float = 900.0, log=None) -> list[Result]:
    """Run every node in dependency order; returns one Result per node (per matrix value)."""
    ctx = {"vars": {}, "inputs": {}, "github": {}, "secrets": {}, **(ctx or {})}
    params = dict(pipeline.parameters)
    params.update(ctx.get("parameters") or {})
    ctx["parameters"] = params
    gh = ctx["github"] = json.loads(json.dumps(ctx["github"]))  # the caller's context stays untouched
    gh.setdefault("event", {}).setdefault("inputs", {})
    gh["event"]["inputs"].update({k: (str(v).lower() if isinstance(v, bool) else v) for k, v in ctx["inputs"].items()})
    base_env = {**pipeline.env, **(env_overrides or {})}
    results: dict[str, list[Result]] = {}
    done: list[Result] = []
    order = _topo(pipeline)
    for name in order:
        job = pipeline.jobs[name]
        deps = [r for n in job.needs for r in results.get(n, [])]
        deps_ok = all(r.status == "success" for r in deps)
        needs_ctx = {n: {"result": _combined(results.get(n, [])),
                         "outputs": {k: v for r in results.get(n, []) for k, v in r.outputs.items()}} for n in job.needs}
        jctx = {**ctx, "env": {**base_env, **job.env}, "needs": needs_ctx,
                "dependencies": {n: {"result": v["result"]} for n, v in needs_ctx.items()},
                "variables": {**base_env, **job.variables}}
        ev = Evaluator(jctx, {"deps_ok": deps_ok, "deps_failed": any(r.status == "failure" for r in deps)})
        if not condition(job.cond, ev):
            r = Result(name, "skipped")
            results[name] = [r]
            done.append(r)
            if log:
                log(f"[{pipeline.name}] {name}: skipped")
            continue
        values = [None]
        if job.matrix:
            axis, vals = next(iter(job.matrix.items()))
            vals = expand(vals, ev) if isinstance(vals, str) else vals
            values = [{axis: v} for v in (vals or [])]
        results[name] = []
        for mv in values:
            r = _run_job(pipeline, job, {**jctx, "matrix": mv or {}}, ev.status, Path(workdir), base_env, timeout, log)
            r.matrix = mv
            results[name].append(r)
            done.append(r)
        if not values:
            r = Result(name, "skipped")
            results[name] = [r]
            done.append(r)
    return done


def _combined(rs: list[Result]) -> str:
    if not rs:
        return "skipped"
    if any(r.status == "failure" for r in rs):
        return "failure"
    return "success" if all(r.status == "success" for r in rs) else "skipped"


def _topo(p: Pipeline) -> list[str]:
    order, seen = [], set()

    def visit(n: str, stack: tuple = ()) -> None:
        if n in seen:
            return
        if n in stack:
            raise ValueError(f"dependency cycle through {n}")
        for d in p.jobs[n].needs:
            if d not in p.jobs:
                raise ValueError(f"{n} depends on unknown {d}")
            visit(d, stack + (n,))
        seen.add(n)
        order.append(n)
    for n in p.jobs:
        visit(n)
    return order


def _run_job(p: Pipeline, job: Job, jctx: dict, status: dict, workdir: Path, base_env: dict, timeout: float,
             log) -> Result:
    t0 = time.time()
    res = Result(job.name, "success")
    tmp = Path(tempfile.mkdtemp(prefix="tt-pipeline-"))
    genv, gout = tmp / "env", tmp / "output"
    env = dict(os.environ)
    env.update(base_env)
    env.update(job.env)
    env.update(job.variables)
    (tmp / "runner-temp").mkdir()
    env.update({"GITHUB_ENV": str(genv), "GITHUB_OUTPUT": str(gout), "CI": "true", "RUNNER_TEMP": str(tmp / "runner-temp"),
                "PYTHONPATH": str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")})
    steps_ctx: dict[str, dict] = {}
    failed = False
    for st in job.steps:
        jctx = {**jctx, "env": {**jctx["env"], **{k: v for k, v in env.items() if k in base_env or k in job.env}},
                "steps": steps_ctx}
        ev = Evaluator(jctx, {"deps_ok": not failed, "deps_failed": failed})
        rec = {"name": st.name, "status": "success"}
        try:
            if not condition(st.cond, ev):
                rec["status"] = "skipped"
                res.steps.append(rec)
                continue
        except ExprError as e:
            rec.update(status="failure", error=str(e))
            res.steps.append(rec)
            failed = True
            continue
        if st.uses:
            action = st.uses.split("@")[0]
            if action in ("actions/checkout", "actions/setup-python"):
                rec["status"] = "success (workspace)"
            elif action == "dorny/paths-filter":
                outs = _paths_filter(st, jctx)
                steps_ctx[st.id or st.name] = {"outputs": outs}
                rec["outputs"] = outs
            else:
                rec["status"] = "not run (external action)"
            res.steps.append(rec)
            continue
        macros = {**{k: v for k, v in env.items()}, **{k: str(v) for k, v in (jctx.get("parameters") or {}).items()}}
        script = expand(st.run, ev, macros if p.kind == "ado" else None)
        step_env = dict(env)
        step_env.update({k: str(expand(v, ev)) for k, v in st.env.items()})
        genv.write_text("")
        gout.write_text("")
        t = time.time()
        try:
            pr = subprocess.run(["bash", "-e", "-o", "pipefail", "-c", script], cwd=str(workdir), env=step_env,
                                capture_output=True, text=True, timeout=timeout)
            rc, out, err = pr.returncode, pr.stdout, pr.stderr
        except subprocess.TimeoutExpired as e:
            rc, out, err = 124, e.stdout or "", f"timed out after {timeout}s"
        rec.update(rc=rc, seconds=round(time.time() - t, 2), stdout=out[-4000:], stderr=err[-4000:])
        env.update(_kv_file(genv))
        outs = _kv_file(gout)
        if outs:
            steps_ctx[st.id or st.name] = {"outputs": outs}
        if rc != 0:
            rec["status"] = "failure"
            failed = True
        res.steps.append(rec)
        if log:
            log(f"[{p.name}] {job.name}: {st.name} -> {rec['status']} ({rec['seconds']} s)")
        if failed:
            break
    if failed:
        res.status = "failure"
    ev = Evaluator({**jctx, "steps": steps_ctx}, status)
    res.outputs = {k: str(expand(v, ev)) for k, v in job.outputs.items()}
    res.seconds = round(time.time() - t0, 2)
    return res


def _kv_file(path: Path) -> dict[str, str]:
    out: dict[str, str] = {}
    if not path.exists():
        return out
    lines = path.read_text().splitlines()
    i = 0
    while i < len(lines):
        line = lines[i]
        if "<<" in line and "=" not in line.split("<<")[0]:  # NAME<<EOF ... EOF
            name, delim = line.split("<<", 1)
            buf = []
            i += 1
            while i < len(lines) and lines[i] != delim:
                buf.append(lines[i])
                i += 1
            out[name] = "\n".join(buf)
        elif "=" in line:
            k, v = line.split("=", 1)
            out[k] = v
        i += 1
    return out


def summary(results: list[Result]) -> list[str]:
    out = []
    for r in results:
        tag = f"{r.job}[{','.join(f'{k}={v}' for k, v in r.matrix.items())}]" if r.matrix else r.job
        ran = [s for s in r.steps if s["status"] not in ("skipped",)]
        out.append(f"{tag}: {r.status}" + (f" ({len(ran)} steps)" if r.status != "skipped" else ""))
    return out


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="pipeline", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("file")
    ap.add_argument("--var", action="append", default=[], help="NAME=value (repository / pipeline variables)")
    ap.add_argument("--input", action="append", default=[], help="NAME=value (workflow_dispatch inputs)")
    ap.add_argument("--param", action="append", default=[], help="NAME=value (Azure DevOps parameters)")
    ap.add_argument("--env", action="append", default=[], help="NAME=value (override the pipeline's env)")
    ap.add_argument("--github", default="{}", help="JSON merged into the github context (ref, sha, event...)")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)

    def kv(items):
        out = {}
        for it in items:
            k, _, v = it.partition("=")
            out[k] = {"true": True, "false": False}.get(v.lower(), v)
        return out
    p = load(a.file)
    res = run(p, {"vars": kv(a.var), "inputs": kv(a.input), "parameters": kv(a.param), "github": json.loads(a.github)},
              env_overrides={k: str(v) for k, v in kv(a.env).items()},
              log=None if a.json else (lambda s: print(s, file=sys.stderr, flush=True)))
    if a.json:
        print(json.dumps([r.__dict__ for r in res], indent=1, default=str))
    else:
        for line in summary(res):
            print(line)
    return 1 if any(r.status == "failure" for r in res) else 0


if __name__ == "__main__":
    sys.exit(main())
