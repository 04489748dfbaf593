"""bench.py's driver contract on CPU: 2 ranks over gloo (torch.distributed.run, 127.0.0.1), rank 0 prints ONE
JSON line with the whole-job value, the max-over-ranks time and the BASELINE metric name."""
import json
import os
import subprocess
import sys
import pytest

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


def test_bench_gpus_flag_self_launches_its_ranks(tmp_path):
    """``bench.py --gpus 2`` outside torchrun starts its own 2 ranks (torch.distributed.run as a child, 127.0.0.1) and
    relays rank 0's single JSON line: n_gpus 2, with the strong-scaling windows and in-run solve of a multi-GPU run."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "torch", "--preset",
           "cartpole-cpu", "--paths", "4", "--envs", "16", "--tmax", "5", "--steps", "2", "--warmup", "1",
           "--windows", "1", "--ga-backend", "host", "--solve-seconds", "20"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"].startswith("dp2")
    s = d["strong_scaling"]
    assert s["n_gpus"] == 2 and s["paths_per_gpu"] == 32 and s["ms_per_update"] > 0
    assert s["in_run_solve"]["updates_run"] > 0


def test_bench_refuses_a_world_size_that_differs_from_gpus(tmp_path):
    """Under torchrun (WORLD_SIZE set), --gpus must equal the world size: exit 2 before any torch import."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--backend", "torch"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr and not r.stdout.strip()


@pytest.mark.gpu
def test_bench_mismatch_guard_on_the_gpu_box(tmp_path):
    """The same guard with the HIP backend on an MI355X box: a torchrun-style environment whose WORLD_SIZE differs
    from --gpus exits 2 before anything touches the GPU (no JSON line, nothing launched)."""
    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29671")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "0"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=4" in r.stderr and not r.stdout.strip(), (r.returncode, r.stderr[-400:])


def test_solve_records_v2_one_per_seed_same_build(tmp_path):
    """bench.solve_records: only v2-criterion records (task horizon + held-out confirmation) of this config and build
    count, one per seed (the latest), wall-limited runs are set apart, unsolved-at-horizon counts as infinite."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from pathnet_gym_amd.algo.solve import CRITERION
    from pathnet_gym_amd.config import preset
    key = bench.solve_key(preset("pong"), "pong")
    cfgd = dict(key, seed=0, ga=True)

    def rec(name, seed, solved, gens, t, stopped="solved", src="aaaa", crit=CRITERION, **kw):
        c = dict(cfgd, seed=seed, **kw)
        d = {"metric": "generations_to_solve", "n_gpus": 1, "criterion": crit, "solved": solved, "stopped": stopped,
             "generations_to_solve": gens if solved else None, "updates_to_solve": gens * 5 if solved else None,
             "frames_to_solve": gens * 100 if solved else None, "finished_at": t, "config": c,
             "build": {"sources_sha256": src}, "candidates": []}
        (tmp_path / name).write_text(json.dumps(d) + "\n")

    rec("a.json", 1, True, 100, 1.0)
    rec("b.json", 1, True, 300, 2.0)                       # a later run of seed 1 replaces a.json
    rec("c.json", 2, False, 0, 1.0, stopped="horizon")     # unsolved at the horizon: counts, as infinite
    rec("d.json", 3, True, 200, 1.0)
    rec("e.json", 4, True, 50, 1.0, src="bbbb")            # another build
    rec("f.json", 5, True, 60, 1.0, crit="old")            # pre-v2 criterion
    rec("g.json", 6, False, 0, 1.0, stopped="wall")        # wall-limited before the horizon
    r = bench.solve_records(key, 1, "aaaa", root=str(tmp_path))
    assert r["seeds"] == 3 and r["solved_seeds"] == 2
    assert [x["seed"] for x in r["runs"]] == [1, 2, 3]
    assert r["runs"][0]["generations"] == 300
    assert r["value"] == 300 and r["min"] == 200 and r["max"] == "unsolved"
    assert r["excluded"] == {"other_config": 0, "pre_v2_criterion": 1, "other_build": 1, "wall_limited": 1}
    assert bench.committed_updates_to_solve.__code__.co_argcount == 2
    # a reproducing certificate (scripts/certify_build.py) links build bbbb to build aaaa: seed 4 now counts for
    # either build; a certificate that did not reproduce links nothing
    (tmp_path / "build_equivalence.json").write_text(json.dumps([
        {"from": "aaaa", "to": "cccc", "reproduces": True, "committed_file": "x"},
        {"from": "cccc", "to": "bbbb", "reproduces": True, "committed_file": "y"},
        {"from": "aaaa", "to": "dddd", "reproduces": False}]))
    rec("h.json", 7, True, 70, 1.0, src="dddd")
    for src in ("aaaa", "bbbb"):
        r = bench.solve_records(key, 1, src, root=str(tmp_path))
        assert [x["seed"] for x in r["runs"]] == [1, 2, 3, 4], src
        assert set(r["equivalent_builds"]) == {"aaaa", "bbbb", "cccc"} - {src}
        assert r["excluded"]["other_build"] == 1              # dddd's record
    assert bench.equivalent_builds("dddd", str(tmp_path)) == {"dddd": None}
