"""bench.py's driver contract on CPU: 2 ranks over gloo (torch.distributed.run, 127.0.0.1), rank 0 prints ONE
JSON line with the whole-job value, the max-over-ranks time and the BASELINE metric name."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_rank_gloo_json_contract(tmp_path):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29653", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--backend", "torch", "--preset", "cartpole-cpu", "--paths", "4", "--envs", "16", "--tmax", "5",
           "--steps", "2", "--warmup", "1", "--ga-backend", "host", "--solve-seconds", "30"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["metric"] == "env_frames_per_sec_whole_node_pong_pathnet"
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["dtype"] == "fp32" and d["value"] > 0
    # value is the whole-job aggregate: 2 ranks x 4 paths x 16 envs x T=5 per update
    frames = 2 * 4 * 16 * 5 * 2
    assert abs(d["value"] - frames / (d["ms_per_step"] * 2 / 1e3)) / d["value"] < 0.01
    assert d["config"]["global_batch"] == 2 * 4 * 16 * 5 and d["config"]["parallelism"].startswith("dp2")
    # median of 3 windows; the strong-scaling record times the fixed 64-path population split over the 2 ranks
    assert d["windows"] == 3 and len(d["windows_ms_per_step"]) == 3
    assert sorted(d["windows_ms_per_step"])[1] == d["ms_per_step"]
    s = d["strong_scaling"]
    assert s["paths_total"] == 64 and s["paths_per_gpu"] == 32 and s["n_gpus"] == 2 and s["ms_per_update"] > 0
    r = s["in_run_solve"]
    assert r["paths_total"] == 64 and r["paths_per_gpu"] == 32 and r["updates_run"] > 0
