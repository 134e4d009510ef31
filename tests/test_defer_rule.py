"""The deferred-leaf rule (rt_fast.h defer_leaf and its end-of-traversal guard) against the reference
order, on the CPU: tools/defer_probe.c renders sampled rows with the oracle's arithmetic (test
infrastructure: it includes oracle/rt_oracle.c) and, for every segment, traces the ray twice -- in
BVHRayHit's order (main_raytracing.cu:43-71) and with the ray's first big leaf deferred to the end of its
traversal, walked from the bound the rest left, ties decided by DFS order, and the guard's second walk
when the rest's best hit lies below its own leaf box's rounded entry -- and counts the segments whose hit
(distance bits, kind, face) differs.  CPU only."""
import json
import os
import subprocess

import pytest

import rt_testlib as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("defer") / "defer_probe")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-o", exe, os.path.join(ROOT, "tools", "defer_probe.c"),
                    "-lm"], check=True, capture_output=True)
    return exe


def _run(exe, *args):
    env = dict(os.environ, OMP_NUM_THREADS="4")
    out = subprocess.run([exe, T.ASSETS, *map(str, args)], check=True, capture_output=True, text=True, env=env, timeout=600)
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_deferred_tree_leaf_equals_reference_order(probe):
    """4-bunny scene (BASELINE configs[3]): the 12,318-triangle leaf deferred, as the leaf-tree kernels do."""
    d = _run(probe, 1, 320, 180, 2, 12, 1024)
    assert d["giant_segments"] > 5000, d
    assert d["mismatches"] == 0 and d["nan_fallbacks"] == 0, d
    assert d["guard_second_walks"] > 0  # the guard's case occurs in real frames


def test_deferred_big_leaf_equals_reference_order(probe):
    """Bunny scene (BASELINE configs[1]) with its 345-triangle floor leaf deferred (the rule itself; the
    production kernel defers only leaf-tree leaves, §4.1 of DESIGN.md)."""
    d = _run(probe, 0, 640, 360, 2, 4, 9)
    assert d["giant_segments"] > 20000, d
    assert d["mismatches"] == 0 and d["nan_fallbacks"] == 0, d
