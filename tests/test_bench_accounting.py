"""bench.py's roofline accounting on CPU: the per-unit algorithmic bytes of
k_paths and its camera stage, the kernel-name matching that ties the
rocprofv3 counter passes to the timed instantiation, and the counter child's command (the
parent's resolved pixelsamples, not a re-planned one)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_kpaths_bytes_follow_the_per_unit_figures():
    # BENCH_r03's counters (20 launches): VERDICT r3's recomputation, 8.90 GB per launch
    agg = {"medium_lookups": 1813622114, "shadow_lookups": 652134642, "medium_items_in": 1179648000,
           "medium_items_out": 0}
    tot, parts = bench.kpaths_bytes(agg, "zsobol", "grid", False, zsobol_table=True)
    assert parts["density_lookups"] == 32 * (1813622114 + 652134642)
    assert parts["sample_records_written"] == 16 * 1179648000
    assert parts["camera_records_read"] == 68 * 1179648000
    assert tot / 20 / 1e9 == pytest.approx(8.90, abs=0.01)
    # phase events add 5 ZSobol table entries of 4 B each
    agg["medium_items_out"] = 1000
    assert bench.kpaths_bytes(agg, "zsobol")[1]["zsobol_table_reads"] == 20 * 1000
    assert bench.kpaths_bytes(agg, "zsobol", zsobol_table=False)[1]["zsobol_table_reads"] == 0
    assert bench.kpaths_bytes(agg, "independent")[1]["camera_records_read"] == 80 * 1179648000


def test_lookup_bytes_by_medium():
    assert bench.lookup_bytes("grid") == 32
    assert bench.lookup_bytes("nanovdb") == 36
    assert bench.lookup_bytes("nanovdb", emissive=True) == 72     # + the temperature grid
    assert bench.lookup_bytes("rgb") == 8 * 16 * 2
    assert bench.lookup_bytes("rgb", emissive=True) == 384       # sigma_a, sigma_s, Le
    agg = {"medium_lookups": 10, "shadow_lookups": 5, "medium_items_in": 0, "medium_items_out": 0}
    # shadow rays evaluate no emission
    assert bench.kpaths_bytes(agg, "zsobol", "rgb", True)[1]["density_lookups"] == 10 * 384 + 5 * 256


def test_camera_bytes():
    assert bench.camera_bytes(4, "zsobol") == 4 * 88 + 6 * 4
    assert bench.camera_bytes(4, "zsobol", zsobol_table=False) == 4 * 88
    assert bench.camera_bytes(4, "independent") == 400
    # the per-pass ZSobol table: 8-B entries per draw, and its build (8 B written + 4 B of the
    # pixel table read per pixel and dimension) once per launch
    assert bench.camera_bytes(4, "zsobol", pass_dims=64, pixels=2, launches=1) == 4 * 88 + 6 * 8 + 2 * 64 * 12
    assert bench.camera_bytes(8, "zsobol", zsobol_table=False, pass_dims=16, pixels=2, launches=2) == \
        8 * 88 + 12 * 8 + 2 * 2 * 16 * 8
    agg = {"medium_lookups": 0, "shadow_lookups": 0, "medium_items_in": 0, "medium_items_out": 1000}
    assert bench.kpaths_bytes(agg, "zsobol", pass_table=True)[1]["zsobol_table_reads"] == 40 * 1000


def test_kernel_names_match_across_demangled_mangled_and_the_abi_string():
    want = ("false", "true", "3", "0", "false", "false")
    assert bench.kernel_targs("k_paths<false, true, 3, 0, false, false>") == want
    assert bench.kernel_targs("void avr::k_paths<false, true, 3, 0, false, false>(avr::Params)") == want
    assert bench.kernel_targs("_ZN3avr7k_pathsILb0ELb1ELi3ELi0ELb0ELb0EEEvNS_6ParamsE") == want
    assert bench.kernel_targs("_ZN3avr7k_pathsILb0ELb1ELi2ELi0ELb0ELb0EEEvNS_6ParamsE") != want
    assert bench.kernel_targs("void avr::k_paths_camera<3, false>(avr::Params)") is None


def test_counter_child_renders_the_parents_pixelsamples():
    args = bench.parse(["--steps", "20", "--warmup", "5"])
    child = bench.pmc_child_argv(args, 16384)
    i = child.index("--pixelsamples")
    assert child[i + 1] == "16384" and child.count("--pixelsamples") == 1
    assert child[child.index("--steps") + 1] == "2"
    assert child[child.index("--spp-per-step") + 1] == str(args.spp_per_step)
    # the child's own plan would differ (2 steps): the forwarded value is what it renders with
    from acceleratedvolrenderer_amd.launch import sample_plan
    assert sample_plan(1, 2, 1, 64)[0] != 16384
    assert sample_plan(1, 2, 1, 64, pixelsamples=16384)[0] == 16384
