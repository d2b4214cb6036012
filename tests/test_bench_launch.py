"""bench.py's own rank launcher (CPU): `python bench.py --gpus N` with WORLD_SIZE unset starts N fresh child processes
with the torch.distributed.run environment, passes their output through and fails when any rank fails."""
import os
import subprocess
import sys
from pathlib import Path

import bench

ROOT = Path(__file__).resolve().parents[1]


def test_rank_env_has_the_launcher_variables():
    env = bench.rank_env({"PATH": "/bin", "KEEP": "1"}, 4, 3, 29577)
    assert env["RANK"] == "3" and env["LOCAL_RANK"] == "3" and env["WORLD_SIZE"] == "4"
    assert env["LOCAL_WORLD_SIZE"] == "4" and env["GROUP_RANK"] == "0"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29577"
    assert env["KEEP"] == "1" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launch_ranks_every_rank_sees_its_environment(tmp_path):
    code = ("import os, pathlib; e = os.environ; "
            f"pathlib.Path(r'{tmp_path}', 'r' + e['RANK']).write_text("
            "','.join(e[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')))")
    assert bench.launch_ranks([sys.executable, "-c", code], 3, port=29601) == 0
    for r in range(3):
        assert (tmp_path / f"r{r}").read_text() == f"{r},{r},3,127.0.0.1,29601"


def test_launch_ranks_failure_is_nonzero_and_stops_the_others():
    # rank 1 fails at once; ranks 0 and 2 would sleep for a minute (a rank stuck in a barrier): they are taken down
    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(7) if r == 1 else time.sleep(60)"
    import time
    t0 = time.monotonic()
    assert bench.launch_ranks([sys.executable, "-c", code], 3) == 7
    assert time.monotonic() - t0 < 30


def test_launch_ranks_signal_and_timeout_codes():
    code = "import os, signal; os.kill(os.getpid(), signal.SIGTERM) if os.environ['RANK'] == '0' else None"
    assert bench.launch_ranks([sys.executable, "-c", code], 2) == 128 + 15
    assert bench.launch_ranks([sys.executable, "-c", "import time; time.sleep(60)"], 2, timeout_s=1.0) == 124


def test_bench_gpus_n_without_enough_gpus_fails_fast():
    """--gpus 8 over RCCL on a box without 8 GPUs (here: none) exits non-zero before any measurement."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--dist-backend", "nccl"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 2
    assert "needs 8 visible GPUs" in p.stderr
    assert p.stdout.strip() == ""
