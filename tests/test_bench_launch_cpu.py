"""bench.py's multi-rank contract on CPU: ``python bench.py --gpus N``
starts the N ranks itself when WORLD_SIZE is unset (torch.distributed.run as a child process,
before any GPU call), the driver's ``torch.distributed.run ... bench.py --gpus N`` form runs as
is, a --gpus / WORLD_SIZE disagreement fails loudly, and rank 0 prints one JSON line with the
whole-job value, n_gpus and the max-over-ranks time.  The step is the --standin CPU step (an
oracle tiny-BiGRU training step per rank over gloo with the flat-gradient all-reduce), so
this checks the launcher and the timing contract, not a GPU number."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", **extra)
    return env


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2])
def test_bench_gpus_n_launches_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--standin", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, env=_env(), timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == n and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["config"]["global_batch"] == 2 * n and rec["config"]["parallelism"] == f"dp{n}"
    assert rec["value"] > 0 and abs(rec["value"] - 2 * n * 3 / (rec["ms_per_step"] * 3e-3)) < 1e-6 * rec["value"]
    assert rec["replicas_in_sync"] is True  # one flat all-reduce per step keeps the replicas identical


def test_bench_under_torchrun_as_the_driver_launches_it():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "2", "--standin",
                        "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, env=_env(), timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["replicas_in_sync"] is True


def test_bench_gpus_world_size_mismatch_fails_loudly():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--standin"], capture_output=True, text=True,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), timeout=120, cwd=ROOT)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr


def test_bench_configs_table():
    sys.path.insert(0, ROOT)
    import bench

    assert set(bench.CONFIGS) == {"C1", "C2", "C4", "C5"}
    assert bench.CONFIGS["C1"]["kind"] == "cpu" and bench.CONFIGS["C1"]["B"] == 1
    assert bench.parse([]).config == "C2" and bench.parse([]).gpus == 1
    c4 = bench.CONFIGS["C4"]
    assert (c4["cell"], c4["L"], c4["K"], c4["adjust"], c4["B"]) == ("gru", 2, 3, False, 32)
    assert bench.CONFIGS["C5"]["kind"] == "recursive" and bench.CONFIGS["C5"]["B"] == 1


def test_bench_c1_cpu_reference_line():
    """--config C1 (BASELINE configs[0]): the reference's CPU path timed on the host cores, no GPU;
    one JSON line with the four SURVEY 8d variants (N 40000 / 32000, without / with the classifier)."""
    import json

    r = subprocess.run([sys.executable, BENCH, "--config", "C1", "--cpu-steps", "1"], capture_output=True, text=True,
                       env=_env(), timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 0 and line["value"] > 0 and line["dtype"] == "f32"
    v = line["cpu_reference_c1"]
    assert set(v) == {"N40000_mask_path", "N40000_with_classifier", "N32000_mask_path", "N32000_with_classifier"}
    assert all(x["cores"] >= 1 and x["value"] > 0 for x in v.values())
    assert v["N40000_mask_path"]["T"] == 313 and v["N32000_mask_path"]["T"] == 251
