"""Audit: no untracked (inline-asm) global load's destination registers are clobbered,
copied or handed to a call before a wait lands the load.

k_decode's batch-point loads are inline asm the compiler's wait-count pass does not
see (SegReaderT<true>); the compiler believes their destination tuple is written
at the asm statement, so if it reused those registers (e.g. for the next load's
address) before an `s_waitcnt vmcnt(0)`, the late data would clobber a live value
(a GPU fault: an index-rebuild kernel built on that reader faulted this way in
round 4; a long code's restart computed the next address into the pending tuple).
This walks the control flow of every kernel that issues such loads, from each load
through branches and back-edges up to the waits.  Path-insensitive: a flagged path
may be one the reader's flags never take.  usage: python tools/audit_async_loads.py [file.s]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def assemble(out):
  sys.path.insert(0, ROOT)
  from federated_amd import build  # pylint: disable=g-import-not-at-top
  flags = [f for f in build.FLAGS if f not in ("-fPIC", "-shared")]
  subprocess.check_call([build.HIPCC] + flags + ["--cuda-device-only", "-S", "-o", out, build.SRC],
                        stderr=subprocess.DEVNULL)


def _regs(op):
  r = re.match(r"v\[(\d+):(\d+)\]$|v(\d+)$", op.strip())
  if not r:
    return set()
  return {int(r.group(3))} if r.group(3) else set(range(int(r.group(1)), int(r.group(2)) + 1))


def _hazard(t, regs):
  """An instruction that, before the load has landed, would clobber its registers (writes
  one: a VALU or load destination) or carry its stale value elsewhere (a move reading one).
  Other reads are the reader's own, which its flags order after a wait."""
  mn, _, rest = t.partition(" ")
  ops = [o for o in rest.split(",")]
  if not ops or not mn:
    return False
  writes_first = (mn.startswith("v_") and not mn.startswith(("v_cmp", "v_readlane", "v_readfirstlane"))) or \
      mn.startswith(("ds_read", "global_load", "buffer_load", "scratch_load", "flat_load", "global_atomic"))
  if writes_first and _regs(ops[0]) & regs:
    return True
  if mn.startswith("v_mov") and any(_regs(o) & regs for o in ops[1:]):
    return True
  return False


def audit(path):
  """{kernel: (async loads, loads with a hazard on some path before a vmcnt(0) wait)}.

  Control-flow aware: from each untracked load, every instruction reachable without
  passing an `s_waitcnt vmcnt(0)` (the asm waits or the compiler's own) is checked --
  through branches and loop back-edges -- for a write of the load's registers, a move
  reading them, or a call (the callee's temporaries may be those registers)."""
  lines = open(path).read().split("\n")
  report = {}
  for st, l in enumerate(lines):
    if not re.match(r"^_Z\S*:", l):
      continue
    name = l.split(":")[0]
    end = next((i for i in range(st + 1, len(lines)) if re.match(r"^\.Lfunc_end", lines[i])), len(lines))
    ins, labels, asm_prev = [], {}, False
    for raw in lines[st + 1:end]:
      t = raw.strip()
      m = re.match(r"^(\.LBB[0-9_]+):", t)
      if m:
        labels[m.group(1)] = len(ins)
        continue
      if "ASMSTART" in t:
        asm_prev = True
        continue
      if not t or t.startswith((";", ".")):
        continue
      ins.append((t.split(";")[0].strip(), asm_prev))
      asm_prev = False
    nloads = touched = 0
    for i, (t, is_asm) in enumerate(ins):
      m = re.search(r"global_load_dwordx4 v\[(\d+):(\d+)\], v\[\d+:\d+\], off$", t)
      if not (m and is_asm):
        continue
      nloads += 1
      regs = set(range(int(m.group(1)), int(m.group(2)) + 1))
      seen, todo, hit = set(), [i + 1], False
      while todo and not hit:
        k = todo.pop()
        if k >= len(ins) or k in seen:
          continue
        seen.add(k)
        u = ins[k][0]
        if re.match(r"s_waitcnt\b.*vmcnt\(0\)", u):
          continue
        if ins[k][1] and u.startswith("global_load_dwordx4"):
          pass  # the reader's own re-issue into the tuple: loads land in order, the newer one last
        elif u.startswith(("s_swappc", "s_setpc", "s_call")) or _hazard(u, regs):
          hit = True
          break
        if u.startswith("s_endpgm"):
          continue
        mb = re.match(r"s_(c?branch)\w*\s+(\.LBB[0-9_]+)", u)
        if mb:
          todo.append(labels[mb.group(2)])
          if mb.group(1) == "cbranch":
            todo.append(k + 1)
          continue
        todo.append(k + 1)
      touched += hit
    if nloads:
      report[name] = (nloads, touched)
  return report


def main():
  path = sys.argv[1] if len(sys.argv) > 1 else None
  if path is None:
    path = os.path.join(tempfile.mkdtemp(), "fedcodec.s")
    assemble(path)
  rep = audit(path)
  bad = {k: v for k, v in rep.items() if v[1]}
  for k, (n, t) in sorted(rep.items()):
    print("%-80s async loads %3d  touched before their wait %d" % (k[:80], n, t))
  return 1 if bad else 0


if __name__ == "__main__":
  sys.exit(main())
