"""CPU tests of the profile tooling: scripts/trace_gaps.py's step timeline and
scripts/train_step_timeline.py's training-step timeline."""
import csv
import json
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def _trace(path, steps, build_ns=100_000, look_ns=8_000, gap_ns=700, prep=("corr_build_split_kernel<f>",),
           graph_every=0, graph_gap_ns=0):
    t, rows = 0, []
    for s in range(steps):
        if graph_every and s and s % graph_every == 0:
            t += graph_gap_ns            # a graph replay boundary before this step
        for name in prep:
            rows.append((name, t, t + build_ns))
            t += build_ns + gap_ns
        for _ in range(12):
            rows.append(("corr_lookup_wide_kernel<4, float, 512, 0>", t, t + look_ns))
            t += look_ns + gap_ns
    rows.append(("at::native::reduce_kernel<...>", t, t + 1000))   # a non-step kernel at the end
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writerows(rows)


def _run(path):
    out = subprocess.run([sys.executable, str(REPO / "scripts" / "trace_gaps.py"), str(path)],
                         capture_output=True, text=True, check=True).stdout
    return json.loads(out)


def test_trace_gaps_step_timeline(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p, steps=6)
    r = _run(p)
    assert r["steps"] == 5                       # the last step has no successor
    assert r["build_us_median"] == 100.0
    assert r["lookup_us_median"] == 8.0
    assert r["step_span_us_median"] == round((100_000 + 12 * 8_000 + 13 * 700) / 1e3, 2)
    assert r["idle_us_per_step_median"] == round(13 * 700 / 1e3, 2)
    assert r["build_in_step_us_median"] == 100.0
    assert r["first_lookup_us_median"] == 8.0
    assert r["idle_us_median_by_boundary"] == {"in_build": 0.0, "build_to_lookup": 0.7,
                                               "between_lookups": round(11 * 0.7, 2),
                                               "step_to_step": 0.7}


def test_trace_gaps_split_build_boundaries(tmp_path):
    """Two build kernels (split pass + DMA build): the gap between them is the
    build's own, and the build's in-step span covers both."""
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p, steps=4, prep=("split_pairs_kernel<false>", "corr_build_dma_kernel<float>"),
           build_ns=50_000)
    r = _run(p)
    assert r["build_us_median"] == 100.0
    assert r["build_in_step_us_median"] == 100.7
    assert r["idle_us_median_by_boundary"]["in_build"] == 0.7


def test_trace_gaps_on_the_fly_block_prep_kernels(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p, steps=4, prep=("transpose_tile_v4_kernel", "avg_pool2x2_nhwc_kernel"),
           build_ns=10_000)
    r = _run(p)
    assert r["steps"] == 3 and r["build_us_median"] == 20.0


def test_trace_gaps_without_steps(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writerow(["corr_lookup_wide_kernel<4>", 0, 10])
    assert _run(p)["steps"] == 0


def test_trace_gaps_means_with_steps_per_graph(tmp_path):
    """Four steps per graph replay: 3 of 4 step boundaries are in-graph, so the
    median hides the replay boundary and the mean carries it per step."""
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p, steps=9, graph_every=4, graph_gap_ns=10_000)
    r = _run(p)
    assert r["steps"] == 8
    assert r["idle_us_median_by_boundary"]["step_to_step"] == 0.7
    assert r["idle_us_mean_by_boundary"]["step_to_step"] == round(0.7 + 2 * 10.0 / 8, 2)
    assert r["idle_us_per_step_mean"] == round(13 * 0.7 + 2 * 10.0 / 8, 2)


def test_bench_profile_config_names_match_gpu_final():
    """bench.py reads its traffic / timeline from profiles/<round>/<config>/, the
    directories scripts/gpu_final.sh writes — one name per configuration, so two
    configurations sharing a workload key (kitti NCHW / NHWC, 1080p alt / full)
    never borrow each other's counters."""
    sys.path.insert(0, str(REPO))
    import bench
    cases = {("sintel", 1, 1, "nchw", "corr"): "sintel", ("sintel", 8, 1, "nchw", "corr"): "sintel_b8",
             ("chairs", 1, 1, "nchw", "corr"): "chairs", ("kitti", 8, 8, "nchw", "corr"): "kitti",
             ("kitti", 8, 8, "nhwc", "corr"): "kitti_nhwc", ("1080p", 1, 1, "nchw", "alt"): "hd_alt",
             ("1080p", 1, 1, "nchw", "corr"): "hd_full"}
    for args, name in cases.items():
        assert bench.profile_config(*args) == name
    script = (REPO / "scripts" / "gpu_final.sh").read_text()
    for name in cases.values():
        assert f"$R/{name} " in script


def test_train_step_timeline(tmp_path):
    """scripts/train_step_timeline.py: steps split at the split pass, the
    second-to-last complete step printed with per-kernel idle and totals."""
    p = tmp_path / "run_kernel_trace.csv"
    rows, t = [], 0
    for _ in range(4):
        for name, dur, gap in (("void (anonymous namespace)::split_pairs_kernel<false, false, 32>(float const*)", 9_000, 0),
                               ("void (anonymous namespace)::corr_build_dma_kernel<float, false, false, 5>(x)", 100_000, 0),
                               ("void at::native::vectorized_elementwise_kernel<4, at::native::FillFunctor<float>>(int)", 5_000, 20_000),
                               ("void (anonymous namespace)::corr_lookup_wide_kernel<4, float, 256, 16>(x)", 8_000, 3_000)):
            t += gap
            rows.append((name, t, t + dur))
            t += dur
        t += 50_000
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writerows(rows)
    out = subprocess.run([sys.executable, str(REPO / "scripts" / "train_step_timeline.py"), str(p)],
                         capture_output=True, text=True, check=True).stdout.splitlines()
    ks = [json.loads(line) for line in out]
    assert [k["kernel"] for k in ks[:-1]] == [
        "split_pairs_kernel", "corr_build_dma_kernel",
        "at::native::vectorized_elementwise_kernel<4, at::native::FillFunctor<float>>",
        "corr_lookup_wide_kernel"]
    assert [k["idle_before_us"] for k in ks[:-1]] == [0.0, 0.0, 20.0, 3.0]
    assert ks[-1] == {"kernels": 4, "kernel_us": 122.0, "idle_us": 23.0, "span_us": 145.0}
