"""The in-tree builder's staleness rule (native/build.py): a build is dated like the newest source
it was compiled from, so a source saved while the compiler ran makes the next check rebuild."""
import os

from aca_dotnet_workshop_amd.native import build


def test_a_source_saved_during_the_compile_leaves_the_build_stale(tmp_path):
    src, target = tmp_path / "a.hpp", tmp_path / "mod.so"
    src.write_text("v1")
    os.utime(src, (1_000_000, 1_000_000))
    stamp = build._newest([src])  # read when the compile starts
    src.write_text("v2")          # saved while it runs
    os.utime(src, (1_000_050, 1_000_050))
    out = tmp_path / "mod.tmp1.so"
    out.write_text("built from v1")
    build._install(out, target, stamp)
    assert target.read_text() == "built from v1" and not out.exists()
    assert build._stale(target, [src])
    out = tmp_path / "mod.tmp2.so"  # the rebuild, from v2
    out.write_text("built from v2")
    build._install(out, target, build._newest([src]))
    assert not build._stale(target, [src])
