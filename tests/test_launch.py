"""``parallel/launch.py`` + ``bench.py``'s launcher mode on CPU: N rank processes are started
with the rendezvous environment, rank 0's stdout is relayed, a failing rank fails the job (and
stops the others), and a bench run whose WORLD_SIZE disagrees with --gpus refuses to run."""
import io
import json
import os
import subprocess
import sys
import textwrap
import time

from mlmicroservicetemplate_amd.parallel.launch import spawn_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    import torch, torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and os.environ["LOCAL_RANK"] == str(rank)
    assert os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    fail = int(sys.argv[1]) if len(sys.argv) > 1 else -1
    dist.init_process_group("gloo")
    if rank == fail:
        sys.exit(3)
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)          # a dead peer leaves the survivors blocked here
    if rank == 0:
        print(json.dumps({"world": world, "sum": t.item()}))
    dist.destroy_process_group()
""")


def test_spawn_ranks_relays_rank0_and_runs_all(tmp_path):
    script = tmp_path / "r.py"
    script.write_text(RANK_SCRIPT)
    out = io.StringIO()
    rc = spawn_ranks([sys.executable, str(script)], 3, timeout_s=120, stdout=out)
    assert rc == 0
    lines = [ln for ln in out.getvalue().splitlines() if ln.startswith("{")]
    assert [json.loads(ln) for ln in lines] == [{"world": 3, "sum": 3.0}]


def test_spawn_ranks_failure_stops_the_others(tmp_path):
    script = tmp_path / "r.py"
    script.write_text(RANK_SCRIPT)
    t0 = time.monotonic()
    rc = spawn_ranks([sys.executable, str(script), "1"], 3, timeout_s=120, stdout=io.StringIO())
    assert rc == 3
    assert time.monotonic() - t0 < 60  # the blocked survivors were terminated, not waited out


def test_spawn_ranks_timeout(tmp_path):
    script = tmp_path / "sleep.py"
    script.write_text("import time; time.sleep(60)\n")
    t0 = time.monotonic()
    rc = spawn_ranks([sys.executable, str(script)], 2, timeout_s=1.0, stdout=io.StringIO())
    assert rc == 124 and time.monotonic() - t0 < 30


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr and r.stdout == ""
