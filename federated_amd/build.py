"""Build recipe for libfedcodec.so (hipcc, gfx950 only, in-tree)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "fedcodec.hip")
HDR = os.path.join(os.path.dirname(HERE), "include", "fedcodec.h")
OUT = os.path.join(HERE, "libfedcodec.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         # TF-CPU numerics: FTZ/DAZ on float32, no FMA contraction
         "-fgpu-flush-denormals-to-zero", "-ffp-contract=off",
         # no SLP packing into v_pk_* f32 ops: on gfx950 a v_pk_mul/add costs about two
         # scalar ops plus the register moves it needs (k_encode -2.6 % without it)
         "-fno-slp-vectorize",
         # no atomic optimizer: its expansion (mbcnt, readfirstlane of the result right
         # after the atomic) made k_encode wait for each ticket atomic -- and every
         # vector memory operation before it -- where it is issued instead of where
         # the ticket is used, a tile later
         "-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]


def build(force=False, verbose=False):
  if (not force and os.path.exists(OUT) and
      os.path.getmtime(OUT) >= max(os.path.getmtime(SRC), os.path.getmtime(HDR))):
    return OUT
  tmp = OUT + ".tmp.%d" % os.getpid()
  cmd = [HIPCC] + FLAGS + ["-o", tmp, SRC]
  if verbose:
    print(" ".join(cmd), flush=True)
  subprocess.check_call(cmd)
  os.replace(tmp, OUT)
  return OUT


if __name__ == "__main__":
  build(force="--force" in sys.argv, verbose=True)
