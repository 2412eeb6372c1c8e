"""bench.py's rank launcher (CPU only, no GPU call anywhere).

`python bench.py --gpus N` without WORLD_SIZE must start N rank processes
itself (the driver's SCALE run may invoke it that way), forward rank 0's
JSON line, and fail loudly -- non-zero status, no orphaned ranks -- when a
rank fails. The children here run the hidden --launch-selftest mode: a gloo
rendezvous over the launcher's MASTER_ADDR / MASTER_PORT and an all-gather
of every rank's (RANK, LOCAL_RANK, WORLD_SIZE).
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
  env = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT",
                      "MASTER_ADDR", "LOCAL_WORLD_SIZE")}
  env.update(extra)
  return env


def _run(args, env, timeout=240):
  t = time.time()
  p = subprocess.run([sys.executable, BENCH] + args, env=env,
                     capture_output=True, timeout=timeout)
  return p, time.time() - t


def test_launcher_starts_n_ranks():
  p, _ = _run(["--gpus", "3", "--launch-selftest", "ok"], _env())
  err = p.stderr.decode()
  assert p.returncode == 0, err
  lines = [l for l in p.stdout.decode().splitlines() if l.startswith("{")]
  assert len(lines) == 1, p.stdout
  out = json.loads(lines[0])
  assert out["ranks_seen"] == 3
  assert sorted(tuple(r) for r in out["ranks"]) == [(0, 0, 3), (1, 1, 3),
                                                    (2, 2, 3)]
  for r in range(3):
    assert f"[selftest] rank {r} of 3" in err


def test_launcher_fails_when_a_rank_fails():
  # the last rank exits 3 while rank 0 blocks: the launcher must stop rank 0
  # and exit non-zero well before its own timeout
  p, dt = _run(["--gpus", "2", "--launch-selftest", "fail",
                "--launch-timeout", "120"], _env())
  assert p.returncode == 3, p.stderr.decode()
  assert dt < 100, dt
  assert "rank 1 exited with status 3" in p.stderr.decode()
  assert not [l for l in p.stdout.decode().splitlines() if l.startswith("{")]


def test_launcher_timeout_kills_ranks():
  p, dt = _run(["--gpus", "2", "--launch-selftest", "fail",
                "--launch-timeout", "0.5"], _env())
  # rank 1 may fail first (3) or the timeout may fire first (124)
  assert p.returncode in (3, 124), p.stderr.decode()
  assert dt < 60


def test_gpus_must_match_world_size():
  p, _ = _run(["--gpus", "3", "--launch-selftest", "ok"],
              _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
  assert p.returncode == 2
  assert "disagrees with WORLD_SIZE=2" in p.stderr.decode()


def test_ranks_die_with_a_killed_launcher():
  """A launcher killed with SIGKILL (no chance to clean up) takes its ranks
  with it (PR_SET_PDEATHSIG): nothing is left holding a GPU."""
  import signal
  p = subprocess.Popen([sys.executable, BENCH, "--gpus", "2", "--launch-selftest",
                        "hang", "--launch-timeout", "300"], env=_env(),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE)
  # wait until both ranks announce themselves (then they block)
  seen = b""
  t = time.time()
  while seen.count(b"[selftest] rank") < 2 and time.time() - t < 60:
    seen += p.stderr.read1(4096)
  assert seen.count(b"[selftest] rank") == 2
  p.send_signal(signal.SIGKILL)
  p.wait()
  time.sleep(2)
  out = subprocess.run(["ps", "-eo", "pid,args"], capture_output=True).stdout
  left = [l for l in out.decode().splitlines()
          if "--launch-selftest hang" in l]
  assert not left, left
