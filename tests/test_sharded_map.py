"""The store's sharded key map (native/src/shardedmap.hpp) grows its shards at staggered points.

Task ids spread evenly over the shards. With one load limit for all shards, every shard crossed
it within the same ~16k inserts. The whole collection was relinked in one burst, under the store
lock, once per doubling. The headline showed it as slow steps at 150k, 325k and 650k documents.
Each shard now has its own limit, so growths spread over the doubling."""
import collections

import pytest

native = pytest.importorskip("aca_dotnet_workshop_amd.native")


def test_shard_growth_is_spread_over_each_doubling():
    m = native.load()
    growth = m.sharded_map_growth(700_000)
    relinked = collections.Counter()  # nodes relinked per 16,384 inserts (one headline step)
    grown = collections.Counter()
    for i, shards in growth:
        relinked[i // 16384] += shards * i / 64  # a growing shard holds about 1/64 of the keys
        grown[i // 16384] += shards
    late = {w: n / 16384 for w, n in relinked.items() if w >= 4}  # past 64k keys
    assert late, "no growth past 64k keys"
    # equal limits relinked up to 24x a step's inserts within one step (39 of 64 shards at
    # 640k keys); spread over the doubling it stays within a few times
    assert max(late.values()) <= 8, sorted(late.items())
    # every shard still grows: about one growth per shard per doubling (64k -> 700k: ~3.4)
    assert sum(n for w, n in grown.items() if w >= 4) >= 3 * 64
