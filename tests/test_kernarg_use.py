"""CPU check of the compiled device code (no GPU): only kernels read the kernel
arguments through __builtin_amdgcn_kernarg_segment_ptr().  LLVM lowers it to NULL
in any other function, and an out-of-line look-back that did so dereferenced
address 0 -- the round-5 and round-6 encoder faults (tools/kernarg_audit.py,
DESIGN.md §2 "Ticket streams and progress")."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import kernarg_audit  # noqa: E402  pylint: disable=g-import-not-at-top,wrong-import-position


@pytest.mark.skipif(not os.path.exists(kernarg_audit.HIPCC) and not shutil.which("hipcc"), reason="no hipcc")
def test_no_kernarg_reads_outside_kernels():
  ir = kernarg_audit.device_ir()
  assert "amdgpu_kernel" in ir
  assert kernarg_audit.offenders(ir) == []


def test_audit_flags_an_out_of_line_reader():
  """The audit itself: a non-kernel, non-inlined function calling the intrinsic is
  reported; a kernel or an always_inline helper is not."""
  ir = "\n".join([
      "define internal void @helper() #0 {",
      "  %p = call ptr addrspace(4) @llvm.amdgcn.kernarg.segment.ptr()",
      "}",
      "define internal void @outofline() #1 {",
      "  %p = call ptr addrspace(4) @llvm.amdgcn.kernarg.segment.ptr()",
      "}",
      "define amdgpu_kernel void @k() #1 {",
      "  %p = call ptr addrspace(4) @llvm.amdgcn.kernarg.segment.ptr()",
      "}",
      "attributes #0 = { alwaysinline nounwind }",
      "attributes #1 = { noinline nounwind }",
  ])
  assert kernarg_audit.offenders(ir) == ["outofline"]
