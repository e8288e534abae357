"""bench.py's own launcher (`--gpus N` without torch.distributed.run): N rank
processes with the launcher environment, rendezvous on 127.0.0.1, here with
gloo on the CPU; and the loud failure when WORLD_SIZE and --gpus disagree."""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    import torch.distributed as dist
    dist.init_process_group("gloo")
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, (int(os.environ["RANK"]), int(os.environ["LOCAL_RANK"]), sys.argv[1:]))
    rank = dist.get_rank()
    if rank == 0:
        print(json.dumps({"world": dist.get_world_size(), "ranks": got}), flush=True)
    dist.destroy_process_group()
    sys.exit(5 if int(os.environ.get("FAIL_RANK", "-1")) == rank else 0)
""")


def _run(tmp_path, n, extra_env=None):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.spawn_ranks(%d, %r, ['--gpus', '%d', '--steps', '1']))" % (ROOT, n, str(script), n))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=180)


def test_spawn_two_ranks_gloo(tmp_path):
    r = _run(tmp_path, 2)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["world"] == 2
    assert sorted(tuple(x[:2]) for x in out["ranks"]) == [(0, 0), (1, 1)]
    assert all(x[2] == ["--gpus", "2", "--steps", "1"] for x in out["ranks"])


def test_spawn_reports_a_failed_rank(tmp_path):
    r = _run(tmp_path, 2, {"FAIL_RANK": "1"})
    assert r.returncode == 5


def test_world_size_disagreeing_with_gpus_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr
