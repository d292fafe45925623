"""Updates in the native document store keep its secondary indexes and its column mirror exact.

``DocStore::put_at`` carries an unchanged path's index entry and mirror dictionary id over from
the replaced version instead of re-keying it (the overdue sweep's bulk save rewrites ~700 tasks
whose creator, dates and prefix do not change).  This test drives random updates that keep,
change, drop, add and re-type values (including ``0.0`` -> ``-0.0``, ``"1"`` -> ``1``) and checks
every live mirror row and every indexed query against the final documents.
"""
from __future__ import annotations

import json
import random

from aca_dotnet_workshop_amd import native

PATHS = ["owner", "due", "done", "n"]


def _doc(rnd: random.Random) -> dict:
    d = {}
    if rnd.random() < 0.9:
        d["owner"] = rnd.choice(["a@x", "b@x", "c@x", 1, None])
    if rnd.random() < 0.9:
        d["due"] = f"2024-05-{rnd.randrange(1, 6):02d}"
    d["done"] = rnd.random() < 0.5
    d["n"] = rnd.choice([0.0, -0.0, 1, 2.5, "1"])
    d["name"] = "t%d" % rnd.randrange(1000)
    return d


def _mirror_rows(store) -> list[tuple[int, dict]]:
    d = store.mirror_delta(0, 0, 0, [])
    assert d["full"] and d["on"]
    cols = {path: (values, ids) for path, _from, values, ids, _all_str in d["columns"]}
    rows = []
    for r in range(d["n"]):
        if not d["live"][r]:
            continue
        vals = {}
        for p in PATHS:
            values, ids = cols[p]
            if ids[r] >= 0:
                vals[p] = json.loads(values[ids[r]])
        rows.append((int(d["seqs"][r]), vals))
    return rows


def _same(a, b) -> bool:
    # the query engine's equality: type-strict (True != 1, "1" != 1), numbers by value
    if isinstance(a, bool) or isinstance(b, bool):
        return type(a) is type(b) and a == b
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return a == b
    return type(a) is type(b) and a == b


def test_updates_keep_indexes_and_mirror_exact():
    store = native.load().DocStore("", 0, 16)
    rnd = random.Random(7)
    docs: dict[str, dict] = {}
    seq: dict[str, int] = {}
    for i in range(200):
        k = f"t||{i}"
        docs[k] = _doc(rnd)
        seq[k] = i + 1
        store.set(k, json.dumps(docs[k]))
    assert store.mirror_enable(PATHS)
    store.query(json.dumps({"filter": {"EQ": {"owner": "a@x"}}}), "t||")  # builds the owner index
    for step in range(3000):
        k = f"t||{rnd.randrange(220)}"
        if k in docs and rnd.random() < 0.6:  # keep most fields, change one
            d = dict(docs[k])
            f = rnd.choice(PATHS + ["name"])
            if rnd.random() < 0.2:
                d.pop(f, None)
            else:
                d[f] = _doc(rnd).get(f, "x")
        elif k in docs and rnd.random() < 0.1:
            store.delete(k)
            del docs[k]
            continue
        else:
            d = _doc(rnd)
        if k not in seq:
            seq[k] = max(seq.values()) + 1
        elif k not in docs:  # re-created after a delete: a new insertion
            seq[k] = max(seq.values()) + 1
        docs[k] = d
        store.set(k, json.dumps(d))
        if step % 500 == 0:
            store.query(json.dumps({"filter": {"EQ": {"due": "2024-05-01"}}}), "t||")  # a second index

    by_seq = {seq[k]: k for k in docs}
    rows = _mirror_rows(store)
    assert len(rows) == len(docs)
    for s, vals in rows:
        want = docs[by_seq[s]]
        for p in PATHS:
            assert (p in vals) == (p in want), (by_seq[s], p)
            if p in want:
                assert _same(vals[p], want[p]), (by_seq[s], p, vals[p], want[p])

    for path, value in [("owner", "a@x"), ("owner", 1), ("owner", None), ("due", "2024-05-01"), ("due", "2024-05-03")]:
        got = {r["key"] for r in json.loads(store.query(json.dumps({"filter": {"EQ": {path: value}}}), "t||"))["results"]}
        want = {k[len("t||"):] for k, d in docs.items() if path in d and _same(d[path], value)}
        assert got == want, (path, value)
