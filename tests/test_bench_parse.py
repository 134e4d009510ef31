"""bench.py's reading of rocprofv3 output (CPU): the render kernel is found under its namespaced,
templated name, and a probe dispatch of the other occupancy variant does not mix into the
counters of the production frames.  (Round 3 moved the kernels into `namespace rtk`; the old
name filter silently found no rows and the bench line lost its PMC roofline.)"""
import csv
import os

import bench

W6 = "void rtk::render_fast_kernel_w6<30, false, 17>(rtk::RenderArgs)"
W5 = "void rtk::render_fast_kernel_w5<30, false, 17>(rtk::RenderArgs)"
OTHER = "(anonymous namespace)::init_rng_kernel(rt_rng_state*, unsigned int const*)"


def test_short_names():
    assert bench._short(W6) == "render_fast_kernel_w6<30, false, 17>"
    assert bench._short(OTHER) == "init_rng_kernel"


def _write(path, header, rows):
    with open(path, "w", newline="") as fh:
        w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(header)
        w.writerows(rows)


def test_read_pmc_pass_picks_the_production_variant(tmp_path):
    d = tmp_path / "pass0"
    os.makedirs(d)
    rows = [[OTHER, "SQ_INSTS_VALU", 1.0], [W5, "SQ_INSTS_VALU", 99.0]]
    rows += [[W6, "SQ_INSTS_VALU", v] for v in (10.0, 12.0, 14.0)]
    _write(d / "pmc_counter_collection.csv", ["Kernel_Name", "Counter_Name", "Counter_Value"], rows)
    trace = [[OTHER, 0, 5], [W5, 0, 7_000_000]] + [[W6, 100, 100 + 16_000_000] for _ in range(3)]
    _write(d / "pmc_kernel_trace.csv", ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], trace)
    vals, kernel, dur = bench.read_pmc_pass(str(d))
    assert kernel == "render_fast_kernel_w6<30, false, 17>"
    assert vals == {"SQ_INSTS_VALU": [10.0, 12.0, 14.0]}
    assert dur == [0.016] * 3


def test_read_pmc_pass_empty(tmp_path):
    assert bench.read_pmc_pass(str(tmp_path)) == ({}, None, [])
