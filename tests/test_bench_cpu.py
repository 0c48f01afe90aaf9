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


def _plan(r):
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_gpus_n_launches_n_ranks():
    r = _run(["--gpus", "4", "--steps", "3", "--print-launch"])
    cmd = _plan(r)["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd
    assert cmd[cmd.index(os.path.join(ROOT, "bench.py")) + 1:] == ["--gpus", "4", "--steps", "3",
                                                                   "--print-launch"]


def test_torchrun_env_is_used_as_is():
    r = _run(["--gpus", "2", "--print-launch"], WORLD_SIZE="2", RANK="1", LOCAL_RANK="1")
    assert _plan(r)["launch"] is None  # no second launch


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "--gpus 1 but WORLD_SIZE=2" in r.stderr
    r = _run(["--gpus", "8"], WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE=4" in r.stderr


def test_frecsys_env_refused():
    r = _run(["--gpus", "1"], FRECSYS_DUAL="0")
    assert r.returncode != 0 and "refusing" in r.stderr


def test_default_extras_every_config_at_every_n():
    """BASELINE configs[3] and [4] are defined on 8 GPUs: the driver's N = 8
    run measures configs 3, 4 and 5 beside the headline."""
    import bench
    for n in (1, 2, 4, 8):
        assert bench.default_extras(n).split(",") == ["safer2_ml20m_d256", "ials_msd_d512",
                                                      "safer2_2m500k_d1024"]
    assert bench.WORKLOADS["safer2_2m500k_d1024"]["max_extra_steps"] == 2
    for n in (1, 8):
        plan = _plan(_run(["--gpus", str(n), "--print-launch"]))
        assert plan["n_gpus"] == n and plan["workload"] == "ials_ml20m_d256"
        assert plan["extras"] == ["safer2_ml20m_d256", "ials_msd_d512", "safer2_2m500k_d1024"]
        assert plan["cpu_baseline"] == (n == 1)  # the CPU baseline stays at N = 1
        assert (plan["launch"] is None) == (n == 1)
        if n == 8:
            assert "--nproc-per-node=8" in plan["launch"]
    # every default extra is a BASELINE config the bench knows
    assert all(w in bench.WORKLOADS for w in bench.DEFAULT_EXTRAS)
