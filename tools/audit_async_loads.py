"""Audit: no untracked (inline-asm) global load's destination registers are touched
before the asm wait that lands it.

k_decode's batch-point loads are inline asm the compiler's wait-count pass does not
see (SegReaderT<true>); the compiler believes their destination tuple is written
at the asm statement, so if it moved or reused those registers before the asm
`s_waitcnt vmcnt(0)`, the late data would clobber a live value (a GPU fault: an
index-rebuild kernel built on that reader faulted this way in round 4).  This scans
the gfx950 assembly of every kernel that issues such loads, linearly from each load
to the next asm wait.  usage: python tools/audit_async_loads.py [file.s]
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


def audit(path):
  lines = open(path).read().split("\n")
  report = {}
  for st, l in enumerate(lines):
    if not re.match(r"^_Z\S*:", l):
      continue
    name = l.split(":")[0]
    end = next((i for i in range(st + 1, len(lines))
                if "s_endpgm" in lines[i] or re.match(r"^\.Lfunc_end", lines[i])), len(lines))
    body = lines[st:end]
    nloads = touches = 0
    for i, b in enumerate(body):
      m = re.search(r"global_load_dwordx4 v\[(\d+):(\d+)\], v\[\d+:\d+\], off$", b.strip())
      if not (m and i > 0 and "ASMSTART" in body[i - 1]):
        continue
      nloads += 1
      regs = set(range(int(m.group(1)), int(m.group(2)) + 1))
      for j in range(i + 1, len(body)):
        t = body[j].strip()
        if "s_waitcnt vmcnt(0)" in t and "ASMSTART" in body[j - 1]:
          break
        if not t or t.startswith((";", ".")):
          continue
        if any((({int(r[2])} if r[2] else set(range(int(r[0]), int(r[1]) + 1))) & regs)
               for r in re.findall(r"v\[(\d+):(\d+)\]|v(\d+)\b", t)):
          touches += 1
          break
    if nloads:
      report[name] = (nloads, touches)
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
