"""`bench.py --gpus N` outside torch.distributed.run starts N ranks as a child launcher
(mgen_amd/launch.py).  Rehearsed on the CPU: a script shaped like bench.py's entry (parse
--gpus, relaunch when needed, else init the process group, all-reduce, rank 0 prints one
JSON line) run with --gpus 2 over gloo."""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import argparse, json, os, sys
    sys.path.insert(0, {root!r})
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    args = ap.parse_args()
    from mgen_amd import launch
    if launch.needs_launch(args.gpus):
        sys.exit(launch.relaunch(__file__, sys.argv[1:], args.gpus, check_gpus=False))
    import torch, torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([float(rank + 1) * args.steps])
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({{"n_gpus": world, "sum": float(t.item())}}), flush=True)
    if world > 1:
        dist.destroy_process_group()
""")


def test_relaunch_two_ranks(tmp_path):
    script = tmp_path / "entry.py"
    script.write_text(SCRIPT.format(root=ROOT))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, str(script), "--gpus", "2", "--steps", "3"],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    assert json.loads(lines[0]) == {"n_gpus": 2, "sum": 9.0}


def test_single_rank_runs_in_process(tmp_path):
    script = tmp_path / "entry.py"
    script.write_text(SCRIPT.format(root=ROOT))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, str(script), "--gpus", "1"], capture_output=True,
                         text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    assert json.loads(out.stdout.strip().splitlines()[-1]) == {"n_gpus": 1, "sum": 1.0}


def test_launcher_command_shape():
    from mgen_amd import launch
    cmd = launch.launcher_cmd("/x/bench.py", ["--gpus", "4", "--steps", "5"], 4, 29500)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-5:] == ["/x/bench.py", "--gpus", "4", "--steps", "5"]
