"""The workshop site: build ``docs/`` into static HTML and publish it to a pages tree.

The reference builds its mkdocs-material site in a container (``make build-docs-website``,
Makefile:1-13) and publishes it three ways: a PR preview under ``pr-preview/pr-<n>/`` of the
``gh-pages`` branch (.github/workflows/preview-docs.yml:44-56), a release copy
(release-docs.yml:38-47) and the Pages deployment of ``main`` (publish-docs.yml:1-32).
mkdocs is not a dependency here; this builder renders the same ``mkdocs.yml`` nav with
markdown-it (CommonMark + tables), rewrites ``.md`` links to ``.html`` and, in strict mode,
fails on a link to a page that does not exist -- what ``mkdocs build --strict`` checks.

    python -m aca_dotnet_workshop_amd.utils.docsite build [--out dist/site]
    python -m aca_dotnet_workshop_amd.utils.docsite publish --site dist/site --pages <dir> [--dest pr-preview/pr-7]
    python -m aca_dotnet_workshop_amd.utils.docsite remove --pages <dir> --dest pr-preview/pr-7
"""
from __future__ import annotations

import argparse
import html
import json
import os
import re
import shutil
import sys
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parents[2]
_LINK = re.compile(r'href="([^"#:]+\.md)(#[^"]*)?"')


def _nav(items, out: list[tuple[str, str, int]], depth: int = 0) -> None:
    for it in items or []:
        for title, target in it.items():
            if isinstance(target, list):
                out.append((title, "", depth))
                _nav(target, out, depth + 1)
            else:
                out.append((title, target, depth))


def _renderer():
    from markdown_it import MarkdownIt
    return MarkdownIt("commonmark", {"html": False}).enable("table")


def build(src: str | os.PathLike = ROOT / "docs", config: str | os.PathLike = ROOT / "mkdocs.yml",
          out: str | os.PathLike = ROOT / "dist" / "site", strict: bool = True) -> dict:
    src, out = Path(src), Path(out)
    cfg = yaml.safe_load(Path(config).read_text())
    nav: list[tuple[str, str, int]] = []
    _nav(cfg.get("nav"), nav)
    if out.exists():
        shutil.rmtree(out)
    out.mkdir(parents=True)
    md = _renderer()
    pages = sorted(p.relative_to(src).as_posix() for p in src.rglob("*.md"))
    missing_nav = [t for _, t, _ in nav if t and t not in pages]
    broken: list[str] = []
    for page in pages:
        body = md.render((src / page).read_text())

        def fix(m: re.Match, page=page) -> str:
            target = (Path(page).parent / m.group(1)).as_posix()
            norm = os.path.normpath(target)
            if norm not in pages:
                broken.append(f"{page} -> {m.group(1)}")
            return f'href="{m.group(1)[:-3]}.html{m.group(2) or ""}"'
        body = _LINK.sub(fix, body)
        depth = page.count("/")
        up = "../" * depth
        items = []
        for title, target, d in nav:
            label = html.escape(title)
            if target:
                cls = ' class="current"' if target == page else ""
                items.append(f'<li style="margin-left:{d}em"><a{cls} href="{up}{target[:-3]}.html">{label}</a></li>')
            else:
                items.append(f'<li style="margin-left:{d}em"><strong>{label}</strong></li>')
        title = next((t for t, p, _ in nav if p == page), page)
        doc = (f"<!doctype html><html><head><meta charset=\"utf-8\"><title>{html.escape(title)} - "
               f"{html.escape(cfg.get('site_name', ''))}</title></head><body>"
               f"<nav><ul>{''.join(items)}</ul></nav><main>{body}</main></body></html>\n")
        dst = out / (page[:-3] + ".html")
        dst.parent.mkdir(parents=True, exist_ok=True)
        dst.write_text(doc)
    for p in src.rglob("*"):  # assets next to the pages (images, snippets, request files)
        if p.is_file() and p.suffix != ".md":
            dst = out / p.relative_to(src)
            dst.parent.mkdir(parents=True, exist_ok=True)
            shutil.copy2(p, dst)
    report = {"pages": len(pages), "nav_entries": sum(1 for _, t, _ in nav if t), "broken_links": broken,
              "missing_nav_pages": missing_nav, "out": str(out)}
    if strict and (broken or missing_nav):
        raise SystemExit(f"docs build failed (strict): {json.dumps(report)}")
    return report


def publish(site: str | os.PathLike, pages: str | os.PathLike, dest: str = "", alias: str | None = None) -> dict:
    """Copy a built site into the pages tree at ``dest`` ('' = the root, keeping the preview
    and release directories that live beside it); ``alias`` also points ``<alias>/`` at it and
    records the version in ``versions.json`` (releases)."""
    site, pages = Path(site), Path(pages)
    pages.mkdir(parents=True, exist_ok=True)
    target = pages / dest if dest else pages
    keep = {"pr-preview", "versions.json"} | {v["version"] for v in _versions(pages)} | \
        {a for v in _versions(pages) for a in v.get("aliases", [])} | ({alias} if alias else set())
    if target.exists():
        for p in target.iterdir():
            if dest or p.name not in keep:
                shutil.rmtree(p) if p.is_dir() else p.unlink()
    shutil.copytree(site, target, dirs_exist_ok=True)
    if alias:
        a = pages / alias
        if a.exists():
            shutil.rmtree(a)
        shutil.copytree(site, a)
        vs = [v for v in _versions(pages) if v["version"] != dest]
        vs.insert(0, {"version": dest, "aliases": [alias]})
        for v in vs[1:]:
            v["aliases"] = [x for x in v.get("aliases", []) if x != alias]
        (pages / "versions.json").write_text(json.dumps(vs, indent=1))
    return {"published": str(target), "files": sum(1 for p in target.rglob("*") if p.is_file())}


def remove(pages: str | os.PathLike, dest: str) -> dict:
    target = Path(pages) / dest
    existed = target.exists()
    if existed:
        shutil.rmtree(target)
    return {"removed": str(target), "existed": existed}


def _versions(pages: Path) -> list[dict]:
    f = pages / "versions.json"
    return json.loads(f.read_text()) if f.exists() else []


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="docsite")
    sub = ap.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("build")
    b.add_argument("--src", default=str(ROOT / "docs"))
    b.add_argument("--config", default=str(ROOT / "mkdocs.yml"))
    b.add_argument("--out", default=str(ROOT / "dist" / "site"))
    b.add_argument("--no-strict", action="store_true")
    p = sub.add_parser("publish")
    p.add_argument("--site", required=True)
    p.add_argument("--pages", required=True)
    p.add_argument("--dest", default="")
    p.add_argument("--alias", default=None)
    r = sub.add_parser("remove")
    r.add_argument("--pages", required=True)
    r.add_argument("--dest", required=True)
    a = ap.parse_args(argv)
    if a.cmd == "build":
        res = build(a.src, a.config, a.out, strict=not a.no_strict)
    elif a.cmd == "publish":
        res = publish(a.site, a.pages, a.dest, a.alias)
    else:
        res = remove(a.pages, a.dest)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
