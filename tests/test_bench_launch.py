"""bench.py's own launcher (CPU): `python bench.py --gpus N` without torchrun starts N rank
processes with the torch.distributed environment set, before anything touches a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]


def test_launcher_spawns_n_ranks():
    for n in (2, 8):
        lines = _run(["--gpus", str(n), "--dry-run"])
        assert sorted(x["rank"] for x in lines) == list(range(n))
        assert all(x["world_size"] == n for x in lines)
        assert all(x["local_rank"] == x["rank"] for x in lines)
        assert all(x["master_addr"] == "127.0.0.1" for x in lines)
        assert len({x["master_port"] for x in lines}) == 1
        assert len({x["pid"] for x in lines}) == n
        # the ranks decide nothing about the GPU before the launch: torch is not even imported
        assert not any(x["torch_imported"] for x in lines)


def test_single_gpu_and_torchrun_env_run_in_process():
    (one,) = _run(["--dry-run"])
    assert one["world_size"] == 1 and one["rank"] == 0
    # under torchrun (WORLD_SIZE set) the process is one rank already: no second launch
    (r,) = _run(["--gpus", "4", "--dry-run"],
                {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3",
                 "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29999"})
    assert (r["rank"], r["world_size"], r["master_port"]) == (3, 4, "29999")
