"""bench.py --gpus N (CPU): the argument -> launch-mode logic.
A bare `python bench.py --gpus N` with N > 1 starts its N ranks itself through
a torch.distributed.run child; a launcher whose WORLD_SIZE disagrees with
--gpus is an error; a run whose ranks cannot start exits non-zero and prints
no bench line (never a silent one-GPU line for --gpus 8)."""
import os
import subprocess
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("gpus,env,expect", [
    (1, {}, ("single", 1)),
    (2, {}, ("spawn", 2)),
    (8, {}, ("spawn", 8)),
    (8, {"WORLD_SIZE": ""}, ("spawn", 8)),
    (8, {"WORLD_SIZE": "8"}, ("rank", 8)),
    (1, {"WORLD_SIZE": "1"}, ("single", 1)),
])
def test_launch_plan(gpus, env, expect):
    assert bench.launch_plan(gpus, env) == expect


@pytest.mark.parametrize("gpus,env", [(8, {"WORLD_SIZE": "1"}), (2, {"WORLD_SIZE": "4"}), (0, {}),
                                      (2, {"WORLD_SIZE": "two"})])
def test_launch_plan_rejects(gpus, env):
    with pytest.raises(SystemExit):
        bench.launch_plan(gpus, env)


def test_spawn_command_runs_this_script_per_gpu():
    cmd = bench.spawn_command(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert os.path.samefile(cmd[-5], os.path.join(ROOT, "bench.py"))


def test_spawned_ranks_stdout_carries_only_the_bench_line(monkeypatch, capsys):
    # what a backend library prints on the ranks' stdout (gloo's connection
    # lines) goes to stderr; the bench line and the ranks' exit code pass through
    script = "print('[Gloo] Rank 1 is connected to 1 peer ranks.'); print('{\"metric\": \"m\", \"value\": 1}'); " \
             "print('trailing'); raise SystemExit(3)"
    monkeypatch.setattr(bench, "spawn_command", lambda gpus, argv, port: [sys.executable, "-c", script])
    rc = bench.spawn_ranks(2, [])
    out, err = capsys.readouterr()
    assert rc == 3
    assert out.splitlines() == ['{"metric": "m", "value": 1}']
    assert "[Gloo]" in err and "trailing" in err


def test_bench_line_fields_from_helpers():
    # the algorithmic bytes of config 2: ~0.5 KB per path
    b = bench.algorithmic_bytes(100)
    assert 15.5e6 < b < 16.5e6 and abs(b / 31200 - 512) < 10


def test_rank_abort_record_classifies_peer_stops():
    chunk = 125 * 312
    shard = 1000 * 312
    runs = [(1.0, 14000.0, 1.0),          # found itself
            (0.0, 2 * chunk, 1.0),        # stopped between chunks (a whole number of them)
            (0.0, chunk + 777, 1.0),      # stopped inside a launch by the device flag
            (0.0, float(shard), 1.0)]     # tracked its whole shard: not stopped
    r = bench.rank_abort_record(3, runs, shard, chunk)
    assert r["rank"] == 3 and r["self_found_runs"] == 1
    assert r["peer_stopped_runs"] == 2 and r["peer_stopped_mid_launch_runs"] == 1
    assert r["paths_tracked"] == {"median": int((2 * chunk + chunk + 777) / 2), "min": 14000, "max": shard}


@pytest.mark.timeout(300)
def test_bare_multi_gpu_run_without_gpus_fails_loudly(tmp_path):
    """No GPU here: the bare --gpus 2 run starts two ranks, both fail at
    set_device, and the parent exits non-zero without a JSON line."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"], capture_output=True, text=True, timeout=280,
                       env=env, cwd=str(tmp_path))
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert "torch.distributed" in p.stderr or "ChildFailedError" in p.stderr or "rank" in p.stderr.lower()
