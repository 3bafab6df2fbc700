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
           "medium_items_out": 0, "medium_dda_steps": 19127199408}
    tot, parts, impl = bench.kpaths_bytes(agg, "zsobol", "grid", False, zsobol_table=True)
    assert parts["density_lookups"] == 32 * (1813622114 + 652134642)
    assert parts["sample_records_written"] == 16 * 1179648000
    assert parts["camera_records_read"] == 64 * 1179648000   # round 4: 68 (the light pick apart)
    assert impl["l2_majorant_steps"] == 0        # the 16^3 majorant is staged in LDS
    assert (tot + 4 * 1179648000) / 20 / 1e9 == pytest.approx(8.90, abs=0.01)
    # phase events read 5 ZSobol table entries of 4 B each: implementation bytes, not in the total
    agg["medium_items_out"] = 1000
    t2, _, impl = bench.kpaths_bytes(agg, "zsobol")
    assert impl["zsobol_table_reads"] == 20 * 1000 and t2 == tot
    assert bench.kpaths_bytes(agg, "zsobol", zsobol_table=False)[2]["zsobol_table_reads"] == 0
    assert bench.kpaths_bytes(agg, "independent")[1]["camera_records_read"] == 80 * 1179648000
    # NanoVDB: 4 B per majorant step read through L2 (reported separately, not HBM
    # bytes, so not in the total) and the 4-B apron slot apart
    tv, pv, iv = bench.kpaths_bytes(agg, "zsobol", "nanovdb", majorant_in_lds=False)
    assert iv["l2_majorant_steps"] == 4 * 19127199408 and "majorant_steps" not in pv
    assert tv == tot
    assert iv["vdb_slot_reads"] == 4 * (1813622114 + 652134642)


def test_nanovdb_frac_excludes_the_l2_majorant():
    """BENCH_r05's NanoVDB leg priced on lookups + records only = 7.66 GB per
    launch over 35.9 ms = 0.027 of 8 TB/s; its 16.4 GB of majorant reads per launch (L2) apart."""
    # per launch (4 launches): lookups 2938699472 B / 32, records 943718400 / 16, camera 3774873600 / 64
    L = 4
    agg = {"medium_lookups": L * 2938699472 // 32, "shadow_lookups": 0, "medium_items_in": L * 58982400,
           "medium_items_out": 0, "medium_dda_steps": L * 16403993540 // 4, "ms_medium": L * 35.89823055267334}
    rb = bench.roofline_block(agg, L, "zsobol", "nanovdb", False, True, True)
    assert rb["bytes_per_launch"] / 1e9 == pytest.approx(7.657, abs=0.001)
    assert rb["frac"] == pytest.approx(0.027, abs=0.0005)
    assert rb["l2_majorant"]["bytes_per_launch"] == pytest.approx(16403993540)
    assert bench.roofline_block(agg, L, "zsobol", "grid", False, True, True)["l2_majorant"] is None


def test_traffic_prices_reads_by_request_size():
    ctr = {"TCC_EA0_RDREQ_sum": 60, "TCC_EA0_RDREQ_32B_sum": 10, "TCC_EA0_RDREQ_64B_sum": 20,
           "TCC_EA0_RDREQ_128B_sum": 30, "WRITE_SIZE": 2.0, "FETCH_SIZE": 5.0}
    assert bench.traffic_bytes(ctr) == 32 * 10 + 64 * 20 + 128 * 30 + 2048
    assert bench.traffic_bytes({"FETCH_SIZE": 5.0, "WRITE_SIZE": 1.0}) is None
    names = [c for _, cs in bench.PMC_PASSES for c in cs]
    assert all(c in names for c in bench.RDREQ_SIZES)
    for _, cs in bench.PMC_PASSES:   # TCC block: at most 4 counters a pass (FETCH_SIZE costs 3)
        tcc = sum(3 if c == "FETCH_SIZE" else (2 if c == "WRITE_SIZE" else 1) for c in cs
                  if c.startswith("TCC") or c in ("FETCH_SIZE", "WRITE_SIZE"))
        assert tcc <= 4


def test_roofline_block_reproduces_the_r04_recomputation(monkeypatch):
    """BENCH_r04's counters over 20 launches at the rocprof average 24.213 ms give
    8.90 GB per launch = 0.046 of 8 TB/s, and lookups alone 3.945 GB = 0.020."""
    agg = {"medium_lookups": 1813755508, "shadow_lookups": 652138892, "medium_items_in": 1179648000,
           "medium_items_out": 1054911269, "medium_dda_steps": 19127199408, "ms_medium": 20 * 24.213}
    # round 4's camera record was 68 B (the light pick apart; 64 B since round 5)
    monkeypatch.setitem(bench.BYTES_CAMERA_RECORD_READ, "zsobol", 68)
    rb = bench.roofline_block(agg, 20, "zsobol", "grid", False, True, True)
    assert rb["bytes_per_launch"] / 1e9 == pytest.approx(8.90, abs=0.01)
    assert rb["frac"] == pytest.approx(0.046, abs=0.0005)
    assert rb["density_fetch"]["bytes_per_launch"] / 1e9 == pytest.approx(3.945, abs=0.001)
    assert rb["density_fetch"]["frac"] == pytest.approx(0.020, abs=0.0005)
    assert rb["implementation_bytes_per_launch"]["zsobol_table_reads"] / 1e9 == pytest.approx(2.11, abs=0.01)


def test_lookup_bytes_by_medium():
    assert bench.lookup_bytes("grid") == 32
    assert bench.lookup_bytes("nanovdb") == 32
    assert bench.lookup_bytes("nanovdb", emissive=True) == 64     # + the temperature grid
    assert bench.lookup_bytes("rgb") == 8 * 16 * 2
    assert bench.lookup_bytes("rgb", emissive=True) == 384       # sigma_a, sigma_s, Le
    agg = {"medium_lookups": 10, "shadow_lookups": 5, "medium_items_in": 0, "medium_items_out": 0,
           "medium_dda_steps": 0}
    # shadow rays evaluate no emission
    assert bench.kpaths_bytes(agg, "zsobol", "rgb", True)[1]["density_lookups"] == 10 * 384 + 5 * 256


def test_camera_bytes():
    assert bench.camera_bytes(4, "zsobol") == 4 * 68 + 6 * 4
    assert bench.camera_bytes(4, "zsobol", zsobol_table=False) == 4 * 68
    assert bench.camera_bytes(4, "independent") == 4 * 84
    # the per-pass ZSobol table: 8-B entries per draw, and its build (8 B written + 4 B of the
    # pixel table read per pixel and dimension) once per launch
    assert bench.camera_bytes(4, "zsobol", pass_dims=64, pixels=2, launches=1) == 4 * 68 + 6 * 8 + 2 * 64 * 12
    assert bench.camera_bytes(8, "zsobol", zsobol_table=False, pass_dims=16, pixels=2, launches=2) == \
        8 * 68 + 12 * 8 + 2 * 2 * 16 * 8
    # the pass table built ahead on the side stream (avr_set_pass_table_ahead): the camera
    # stage's interval is the camera kernel alone, so its bytes leave the build out
    assert bench.camera_bytes(4, "zsobol", pass_dims=64, pixels=2, launches=0) == 4 * 68 + 6 * 8
    agg = {"medium_lookups": 0, "shadow_lookups": 0, "medium_items_in": 0, "medium_items_out": 1000,
           "medium_dda_steps": 0}
    assert bench.kpaths_bytes(agg, "zsobol", pass_table=True)[2]["zsobol_table_reads"] == 40 * 1000


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


def _trace_avg_ms(rows, inst, timed):
    """Average duration (ms) of the last `timed` dispatches of one k_paths instantiation in a
    rocprofv3 kernel trace (dispatch order): a leg's timed steps come after its majorant-tuning
    probes and warmup steps."""
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
         for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
         if r["Kernel_Name"] == f"void avr::{inst}(avr::Params)"][-timed:]
    return sum(d) / len(d), len(d)


@pytest.mark.parametrize("tag", ["final", "end"])
def test_r06_line_fracs_reproduce_from_the_committed_kernel_trace(tag):
    """VERDICT r5 item 1's Done: the grid, NanoVDB and fast `frac` of the round-6 line
    (profiles/r06_bench_line_{final,end}.json: mid-round and end of round) from its per-launch
    algorithmic bytes over the kernel's average duration in the committed rocprofv3 trace of the
    same command (profiles/r06_kernel_trace_{final,end}.csv, tools/final_pass.sh `stats`) — separate runs, so within
    2 % — and `traffic_over_algorithmic` as the calibrated counter bytes over those bytes."""
    import csv
    import json
    line = json.load(open(os.path.join(ROOT, "profiles", f"r06_bench_line_{tag}.json")))
    rows = list(csv.DictReader(open(os.path.join(ROOT, "profiles", f"r06_kernel_trace_{tag}.csv"))))
    legs = [(line["roofline"]["instantiation"], line["roofline"], line["steps"]),
            (line["nanovdb"]["instantiation"], line["nanovdb"]["roofline"], line["nanovdb"]["steps"]),
            (line["fast_mode"]["instantiation"], line["fast_mode"]["roofline"], line["steps"])]
    for inst, rb, timed in legs:
        ms, n = _trace_avg_ms(rows, inst, timed)
        assert n == timed, inst
        assert ms == pytest.approx(rb["avg_launch_ms"], rel=0.02), inst
        frac = rb["bytes_per_launch"] / (ms / 1e3) / (rb["peak"] * 1e9)
        assert frac == pytest.approx(rb["frac"], rel=0.02), inst
        assert sum(rb["bytes_parts_per_launch"].values()) == pytest.approx(rb["bytes_per_launch"])
    # NanoVDB's L2 majorant reads are reported apart, not priced in frac
    nv = line["nanovdb"]["roofline"]
    assert "l2_majorant_steps" not in nv["bytes_parts_per_launch"] and nv["l2_majorant"]["bytes_per_launch"] > 0
    for rb in (line["roofline"], line["fast_mode"]["roofline"]):
        assert rb["traffic_over_algorithmic"] == pytest.approx(rb["traffic"] * 1e9 / rb["bytes_per_launch"], rel=0.01)
    assert "r06_fetch_size_calibration.json" in line["roofline"]["traffic_basis"]
    cal = json.load(open(os.path.join(ROOT, "profiles", "r06_fetch_size_calibration.json")))
    for o in ("random", "trace", "shuffled"):   # FETCH_SIZE x 2 = the request-size bytes for 32-B gathers
        assert cal["orders"][o]["fetch_size_correction"] == pytest.approx(2.0, abs=0.01)
