"""bench.py's multi-GPU entry point (the driver's `bench.py --gpus N`): with
no launcher around it, bench.py starts N ranks itself (one process per GPU,
slo_amd.dist.launch_ranks) before anything touches a GPU.  --dry-dist runs
the rank plumbing alone on gloo, so this runs on CPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=180, env=env, cwd=ROOT)


def _line(r):
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout   # rank 0 alone prints
    return json.loads(lines[0])


def test_gpus_2_starts_two_ranks():
    j = _line(_run(["--gpus", "2", "--dry-dist", "--steps", "3", "--warmup", "1"]))
    assert j["n_gpus"] == 2 and j["ranks_seen"] == 2
    assert j["steps"] == 3 and j["warmup"] == 1
    assert j["ms_per_step"] == 20.0   # max over ranks: rank 1's 0.02 s


def test_gpus_1_is_one_rank():
    j = _line(_run(["--gpus", "1", "--dry-dist"], {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29611",
                                                    "RANK": "0", "WORLD_SIZE": "1"}))
    assert j["n_gpus"] == 1


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4", "--dry-dist"], {"RANK": "0", "WORLD_SIZE": "2", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "--gpus 4" in r.stderr


def test_a_failing_rank_fails_the_job():
    # rank 1 exits before the rendezvous: rank 0 would wait for it forever, the launcher stops it
    r = _run(["--gpus", "2", "--dry-dist", "--dry-fail-rank", "1"])
    assert r.returncode == 3
    assert "rank 1 exited with 3" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_launch_ranks_stdout_file_and_time_limit(tmp_path):
    """the Mode S leg's launcher (bench.py modes_leg_launch): every rank's
    stdout into one file, and a group still running at the time limit is
    stopped with 124 instead of holding the bench"""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "sc-lego-loam_amd"))
    from slo_amd import dist as sdist
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "print('{\"rank\": %s, \"world\": %s}' % (os.environ['RANK'], os.environ['WORLD_SIZE']), flush=True)\n"
                      "time.sleep(float(sys.argv[1]))\n")
    with tempfile.TemporaryFile("w+") as f:
        assert sdist.launch_ranks(3, ["0"], str(script), stdout=f, timeout_s=60) == 0
        f.seek(0)
        got = sorted(json.loads(x)["rank"] for x in f.read().splitlines())
    assert got == [0, 1, 2]
    with tempfile.TemporaryFile("w+") as f:
        assert sdist.launch_ranks(2, ["600"], str(script), stdout=f, timeout_s=3) == 124
