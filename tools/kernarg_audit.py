"""Audit: no function other than a kernel reads the kernel arguments through
__builtin_amdgcn_kernarg_segment_ptr() (llvm.amdgcn.kernarg.segment.ptr).

LLVM lowers that intrinsic to NULL in any function that is not an amdgpu_kernel, so
an out-of-line device function (a __noinline__ callee, or any function the inliner
leaves out of line) that used it would dereference address 0 -- the cause of the
round-5 and round-6 encoder faults (DESIGN.md §2 "Ticket streams and progress").
Compiles the library's device code to LLVM IR at -O0 (always_inline functions are
inlined there; the rest stay separate functions) and lists offending functions.
Usage: python tools/kernarg_audit.py [source.hip]  (exit 1 if any is found)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "federated_amd", "csrc", "fedcodec.hip")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
INTRINSIC = "llvm.amdgcn.kernarg.segment.ptr"


def device_ir(src=SRC):
  with tempfile.TemporaryDirectory() as d:
    out = os.path.join(d, "dev.ll")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O0", "-std=c++17", "--cuda-device-only",
                           "-emit-llvm", "-S", "-I", os.path.join(ROOT, "include"), "-o", out, src],
                          stderr=subprocess.DEVNULL)
    with open(out) as f:
      return f.read()


def offenders(ir):
  """Non-kernel, non-always_inline functions that call the kernarg intrinsic."""
  attrs = {}
  for m in re.finditer(r"^attributes #(\d+) = \{(.*)\}$", ir, re.M):
    attrs[m.group(1)] = m.group(2)
  bad = []
  for m in re.finditer(r"^define ([^\n]*?)@([\w.$]+)\(([^\n]*)\{$(.*?)^\}$", ir, re.M | re.S):
    head, name, tail, body = m.group(1), m.group(2), m.group(3), m.group(4)
    if "amdgpu_kernel" in head or INTRINSIC not in body:
      continue
    groups = re.findall(r"#(\d+)", tail)
    if any("alwaysinline" in attrs.get(g, "") for g in groups):
      continue  # inlined into its callers (kernels, or the functions checked here)
    bad.append(name)
  return bad


def main():
  src = sys.argv[1] if len(sys.argv) > 1 else SRC
  bad = offenders(device_ir(src))
  for name in bad:
    print("reads kernel arguments outside a kernel:", name)
  print("kernarg audit: %d offending function(s)" % len(bad))
  return 1 if bad else 0


if __name__ == "__main__":
  sys.exit(main())
