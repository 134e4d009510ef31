"""The benchmark line proves itself: bench.py's default run re-renders the frames it timed unsharded,
in plain tile order, and compares the final surface bit for bit (`check_equal`), so the exact launch
shape behind the headline number -- cost-ordered tiles, the measured lane map, the occupancy the probe
picks -- is checked at full size on every run (RayTracing/RayTracing.cpp:231-233: each frame lerps
into the last one, so the final surface carries every frame's pixels).  At N > 1 the compared frame is
the gathered one, and the line carries the per-frame gather time (tests/test_gpu_multi.py
test_bench_two_ranks_without_launcher).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, timeout=240):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, f"exit {r.returncode}: {r.stderr[-3000:]}"
    return r.returncode, json.loads(lines[-1])


@pytest.mark.gpu
def test_bench_cfg2_line_is_bit_exact():
    """The headline workload (config 2) with the bench's own defaults: the line says check_equal."""
    rc, line = _bench(["--config", "cfg2", "--steps", "2", "--warmup", "1", "--no-pmc", "--no-cpu-baseline"])
    assert rc == 0, line
    assert line["check_equal"] is True
    assert line["check"]["frames"] == 3
    assert line["plan"]["kind"].startswith("cost")
    # frame 0 of the exact timed launch shape against the oracle's own full frame (row hashes + RNG states)
    assert line["check_oracle_fixture"]["equal"] is True, line["check_oracle_fixture"]

