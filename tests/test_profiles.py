"""The committed profiles the bench line attaches (profiles/current/): every
file names the commit and the source digest it was measured at, all of them one measurement, and
the bench's `sources_match` compares that digest with the tree it runs from (no GPU needed)."""
import glob
import json
import os
import sys
import warnings

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

from mpc_arpo_project_amd._lib import source_digest  # noqa: E402

CURRENT = sorted(glob.glob(os.path.join(REPO, "profiles", "current", "*.json")))


def test_current_profiles_are_one_measurement_with_provenance():
    assert CURRENT, "no committed profiles"
    stamps = set()
    for f in CURRENT:
        d = json.load(open(f))
        assert d.get("commit") and d.get("src_digest"), f
        for k in ("batch", "nx", "kind", "concurrent_shards"):
            assert k in d, (f, k)
        stamps.add((d["commit"], d["src_digest"]))
    assert len(stamps) == 1, stamps
    (_, digest), = stamps
    if digest != source_digest():
        # a source change since the profiling run: the bench line says so (sources_match false);
        # re-run tools/profile_r5.sh a/b/d and tools/profile_post.py before the round ends
        warnings.warn(f"profiles/current measured on sources {digest}, tree is {source_digest()}")


def test_bench_reports_whether_the_profile_sources_match():
    import bench

    d = json.load(open(CURRENT[0]))
    assert bench._sources_match(d) is (d["src_digest"] == source_digest())
    assert bench._sources_match({k: v for k, v in d.items() if k != "src_digest"}) is None


def test_source_digest_follows_the_sources(tmp_path, monkeypatch):
    import shutil

    from mpc_arpo_project_amd import _lib

    ref = _lib.source_digest()
    pkg = tmp_path / "pkg"
    shutil.copytree(os.path.join(REPO, "mpc_arpo_project_amd", "csrc"), pkg / "csrc")
    shutil.copytree(os.path.join(REPO, "include"), tmp_path / "include")
    monkeypatch.setattr(_lib, "_HERE", str(pkg))
    a = _lib.source_digest()
    assert a == ref  # content, not location
    with open(pkg / "csrc" / "engine_pair.inc", "a") as fh:
        fh.write("\n// a comment changes the digest too\n")
    assert _lib.source_digest() != a
