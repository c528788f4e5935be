"""Every profiles/ path the documentation and code cite names a committed file
(tools/profile_refs.py also prunes the uncited records)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import profile_refs as P  # noqa: E402


def test_every_cited_profile_path_exists():
    files = P.tracked_profiles()
    if not files:   # not a git checkout (e.g. a copied tree): nothing to check against
        files = [os.path.relpath(os.path.join(dp, f), ROOT) for dp, _, fs in os.walk(os.path.join(ROOT, "profiles"))
                 for f in fs]
    full, _ = P.citations()
    assert len(full) > 40
    missing = [p for p in full if not P.full_matches(p, files)]
    assert not missing, missing


def test_brace_and_glob_citations_expand():
    assert P.expand_braces("profiles/r0{1,2}/x_{a,b}.json") == [
        "profiles/r01/x_a.json", "profiles/r01/x_b.json", "profiles/r02/x_a.json", "profiles/r02/x_b.json"]
    assert P.full_matches("profiles/r05/valu/", ["profiles/r05/valu/a.csv", "profiles/r05/x.csv"]) == \
        ["profiles/r05/valu/a.csv"]
