"""Build libhgx.so (all csrc/*.hip) in-tree for gfx950 with hipcc.

The .so is written next to this file so it travels with the repo snapshot to
the GPU box (it is git-ignored, not gpurun-ignored). Cross-compiles without a
GPU. ``python -m hypergraphembedding_amd.build [--force]``.
"""

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libhgx.so")
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
ARCH = os.environ.get("HGX_OFFLOAD_ARCH", "gfx950")


def _sources():
  return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _deps():
  return (_sources() + glob.glob(os.path.join(CSRC, "*.h")) +
          [os.path.join(INCLUDE, "hgx.h")])


def up_to_date():
  if not os.path.exists(LIB):
    return False
  t = os.path.getmtime(LIB)
  return all(os.path.getmtime(p) <= t for p in _deps())


def build(force=False, verbose=False):
  if not force and up_to_date():
    return LIB
  hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
  objdir = os.path.join(HERE, "_build")
  os.makedirs(objdir, exist_ok=True)
  flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
           "-I" + INCLUDE, "-Wno-pass-failed"]
  objs, procs = [], []
  for src in _sources():
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    objs.append(obj)
    if not force and os.path.exists(obj) and all(
        os.path.getmtime(obj) >= os.path.getmtime(p)
        for p in [src] + glob.glob(os.path.join(CSRC, "*.h")) +
        [os.path.join(INCLUDE, "hgx.h")]):
      continue
    cmd = [hipcc] + flags + ["-c", src, "-o", obj]
    if verbose:
      print(" ".join(cmd), file=sys.stderr)
    procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE,
                                        stderr=subprocess.STDOUT)))
  for src, p in procs:
    out, _ = p.communicate()
    if p.returncode != 0:
      raise RuntimeError(f"hipcc failed on {src}:\n{out.decode()}")
  tmp = LIB + ".tmp"
  cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
  r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
  if r.returncode != 0:
    raise RuntimeError("link failed:\n" + r.stdout.decode())
  os.replace(tmp, LIB)
  return LIB


if __name__ == "__main__":
  print(build(force="--force" in sys.argv, verbose=True))
