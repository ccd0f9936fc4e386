"""The exact BestEffort hint merge (koordinator_amd/csrc/ke_merge.h merge_exact, used beyond MERGE_BUDGET
permutations) against the reference's permutation-by-permutation fold (merge_walk, policy.go:198-299) on random
provider lists, compiled for the host with g++ (tests/merge/merge_check.cpp)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def merge_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("merge") / "merge_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-o", exe,
                    os.path.join(HERE, "merge", "merge_check.cpp")], check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_merge_exact_equals_walk(merge_check, seed):
    r = subprocess.run([merge_check, str(seed), "2500"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "fails 0" in r.stdout
