"""bench.py's measurement plumbing on the CPU (no kernel): the config
presets, the kernel names it looks up in rocprofv3 summaries, the committed
profiles it reads `frac_rocprof` / `traffic` from, and the dry-run JSON line
of every config."""
import json
import os
import subprocess
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _args(*argv):
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


@pytest.mark.parametrize("cfg,env,batch,workload,scaling", [
    (0, "SimulatedCars", 65536, "step", "weak"), (1, "SimulatedCars", 1, "closed_loop", "weak"),
    (2, "SimulatedCars", 4096, "step", "weak"), (3, "Unicycle", 4096, "step", "weak"),
    (4, "SimulatedCars", 262144, "step", "strong"), (5, "SimulatedCars", 4096, "sac_update", "weak")])
def test_config_presets_follow_baseline_json(cfg, env, batch, workload, scaling):
    a = _args("--config", str(cfg))
    assert (a.env, a.batch, a.workload, a.scaling) == (env, batch, workload, scaling)
    if cfg == 3:
        assert a.hazards == 3  # BASELINE config 3: the 3-obstacle constraint set


def test_block_size_mirrors_the_library():
    # rcbf_common.hpp block_for_envs: 256 from 65 536 envs, 128 from 32 768, else 64
    assert [bench.block_for_envs(b) for b in (1, 4096, 32767, 32768, 65535, 65536, 262144)] == \
        [64, 64, 64, 128, 128, 256, 256]


def test_kernel_names_and_profile_lookup():
    a = _args()
    assert bench.workload_short(a) == "cars"
    assert bench.dominant_kernels(a, 65536) == ["k_safe_step<0, 0, 1, false, 256, false>"]
    a3 = _args("--config", "3")
    assert bench.workload_short(a3) == "uni3"
    assert bench.dominant_kernels(a3, 4096) == ["k_safe_step<0, 1, 3, false, 64, false>"]
    a5 = _args("--config", "5")
    assert bench.workload_short(a5) == "sacupd_cars_rowsprior_maxstd"  # MAX_STD materialised per env
    assert bench.dominant_kernels(a5, 4096) == ["k_safe_action_jac<0, 0, 1, true, 64>", "k_apply_jac<1, 64>"]
    # the committed r04 summaries of the headline are found and parsed
    us, src = bench.rocprof_kernel_us("cars", 65536, bench.dominant_kernels(a, 65536))
    assert src and src.startswith("profiles/r") and 2.0 < us < 20.0
    tr, tsrc = bench.pmc_traffic_file("cars", 65536)
    assert tsrc and 0.9 < tr / (241 * 65536) < 1.5
    # a kernel name no summary holds gives None, never another kernel's time
    assert bench.rocprof_kernel_us("cars", 65536, ["k_not_a_kernel<0>"]) == (None, None)


def test_rocprof_figure_comes_from_the_same_command_form(tmp_path, monkeypatch):
    """The driver's command (--steps 20 --warmup 5) reads only a trace of that
    command (kernel_stats_driver_form_*), the default form only the long-form
    trace; neither borrows the other's file."""
    assert bench.rocprof_form(20, 5) == "driver" and bench.rocprof_form(1000, 20) == "default"
    prof = tmp_path / "profiles" / "r09"
    prof.mkdir(parents=True)
    head = '"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
    k = "k_safe_step<0, 0, 1, false, 256, false>"
    (prof / "kernel_stats_cars_B65536_r09a.csv").write_text(head + f'"void {k}(x)",10,50000,5000.0,90,1,1,1\n')
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.rocprof_kernel_us("cars", 65536, [k], "default") == (5.0, "profiles/r09/kernel_stats_cars_B65536_r09a.csv")
    assert bench.rocprof_kernel_us("cars", 65536, [k], "driver") == (None, None)
    (prof / "kernel_stats_driver_form_cars_B65536_r09b.csv").write_text(head + f'"void {k}(x)",88,500000,5800.0,90,1,1,1\n')
    assert bench.rocprof_kernel_us("cars", 65536, [k], "driver") == (
        5.8, "profiles/r09/kernel_stats_driver_form_cars_B65536_r09b.csv")
    assert bench.rocprof_kernel_us("cars", 65536, [k], "default")[0] == 5.0


@pytest.mark.parametrize("cfg", [0, 2, 5])
def test_dry_run_line_carries_the_contract_fields(cfg):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-dry-run", "--steps", "5",
                        "--warmup", "1", "--config", str(cfg)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in rec, k
    rf = rec["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_us_rocprof", "frac_rocprof",
              "rocprof_source"):
        assert k in rf, k
    assert rec["config"]["baseline_config"] == (cfg or None)
    # configs 2 and 5 read the materialised sigma[5, 7, 9] rows (+12 B)
    assert rf["bytes_per_env_step"] == {0: 241, 2: 253, 5: 68}[cfg]


def test_rccl_flag_brings_up_the_group_on_one_rank():
    """bench.py --rccl on one rank runs the N > 1 path's process-group code (rendezvous on 127.0.0.1,
    barriers around the timed region, all_gather of the per-rank times, MAX all_reduce): over gloo in
    the CPU dry run, over RCCL on the device (profiles/r05/bench_rccl_world1_r05z.json)."""
    env = {k: v for k, v in os.environ.items() if k not in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-dry-run", "--rccl", "--steps", "4",
                        "--warmup", "1", "--batch", "256"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == 1 and rec["config"]["collectives"].startswith("gloo process group, world 1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-dry-run", "--steps", "4",
                        "--warmup", "1", "--batch", "256"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])["config"]["collectives"] is None


def test_committed_roofline_records_recompute():
    """every committed roofline record (bench.py --record) recomputes its own figures --
    frac from bytes_per_launch and kernel_us_per_step, frac_wall from ms_per_step, the per-step GPU time as the
    median of its dispatch-timestamp runs -- and nests as an untraced run must: in-kernel span <= per-step GPU
    time <= wall time per step.  bench.py finds the driver-form record for the driver's command."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "roofline_record_*.json")))
    assert paths
    for p in paths:
        r = json.load(open(p))
        k_us, wall_us = r["kernel_us_per_step"], r["ms_per_step"] * 1e3
        frac = r["bytes_per_launch"] / (k_us * 1e-6) / 1e9 / r["peak_GBs"]
        assert abs(frac - r["frac"]) <= 0.002, p
        assert abs(r["bytes_per_launch"] / (wall_us * 1e-6) / 1e9 / r["peak_GBs"] - r["frac_wall"]) <= 0.002, p
        runs = r["aql_dispatch_times"]["runs"]
        periods = sorted((x["last_end_ns"] - x["first_start_ns"]) / 1e3 / r["steps"] for x in runs)
        assert abs(periods[len(periods) // 2] - k_us) <= 0.01, p
        assert r["span"]["kernel_span_us_median"] <= k_us <= wall_us + 0.01, p
        assert r["bytes_per_launch"] == r["batch"] * r["bytes_per_env_step"]
    k_us, src = bench.roofline_record("cars", 65536, "driver", "aql")
    assert src and "driver_form" in src and 2.0 < k_us < 6.0
