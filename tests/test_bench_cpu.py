"""bench.py's launcher contract (CPU): `--gpus N` without a torchrun
environment launches N ranks itself; a torchrun environment whose WORLD_SIZE
differs from --gpus is refused before any GPU work."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env_over):
    env = {k: v for k, v in os.environ.items()
           if not k.startswith("FRECSYS_") and k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_over)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=120)


def test_gpus_n_launches_n_ranks():
    r = _run(["--gpus", "4", "--steps", "3", "--print-launch"])
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd
    assert cmd[cmd.index(os.path.join(ROOT, "bench.py")) + 1:] == ["--gpus", "4", "--steps", "3",
                                                                   "--print-launch"]


def test_torchrun_env_is_used_as_is():
    r = _run(["--gpus", "2", "--print-launch"], WORLD_SIZE="2", RANK="1", LOCAL_RANK="1")
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1]) is None  # no second launch


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "--gpus 1 but WORLD_SIZE=2" in r.stderr
    r = _run(["--gpus", "8"], WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE=4" in r.stderr


def test_frecsys_env_refused():
    r = _run(["--gpus", "1"], FRECSYS_DUAL="0")
    assert r.returncode != 0 and "refusing" in r.stderr


def test_default_extras_config5_at_one_gpu_only():
    import bench
    one = bench.default_extras(1).split(",")
    many = bench.default_extras(8).split(",")
    assert "safer2_2m500k_d1024" in one and "safer2_2m500k_d1024" not in many
    assert set(many) == {"safer2_ml20m_d256", "ials_msd_d512"}
    assert bench.WORKLOADS["safer2_2m500k_d1024"]["max_extra_steps"] == 2
    # every default extra is a BASELINE config the bench knows
    assert all(w in bench.WORKLOADS for w in one)
