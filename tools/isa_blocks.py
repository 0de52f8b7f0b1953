"""Diagnostic: per-basic-block instruction mix of one kernel in a hipcc -S listing.

python tools/isa_blocks.py <file.s> <symbol-substring> [min_instrs]
"""
import re
import sys


def main():
  path, sym = sys.argv[1], sys.argv[2]
  minn = int(sys.argv[3]) if len(sys.argv) > 3 else 8
  lines = open(path).read().split("\n")
  start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(sym), l))
  end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.section") or
             re.match(r"^\.Lfunc_end", lines[i]))
  blocks, cur, name = [], [], "entry"
  for l in lines[start + 1:end]:
    s = l.strip()
    if re.match(r"^(\.LBB\S+:|; %bb\.\d+:)", s):
      blocks.append((name, cur))
      name, cur = s.split()[0] if s.startswith(".LBB") else s[2:], []
      continue
    if not s or s.startswith(";") or s.startswith("."):
      continue
    cur.append(s.split(";")[0].strip())
  blocks.append((name, cur))
  tot = {"v": 0, "s": 0, "ds": 0, "vm": 0, "mad64": 0}
  for name, ins in blocks:
    c = {"v": 0, "s": 0, "ds": 0, "vm": 0, "mad64": 0}
    for i in ins:
      op = i.split()[0]
      if op.startswith("ds_"):
        c["ds"] += 1
      elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        c["vm"] += 1
      elif op.startswith("v_"):
        c["v"] += 1
        if op.startswith(("v_mad_u64", "v_mad_i64", "v_mul_hi", "v_mul_lo", "v_lshlrev_b64",
                          "v_lshrrev_b64", "v_ashrrev_i64")):
          c["mad64"] += 1
      elif op.startswith("s_"):
        c["s"] += 1
    for k in tot:
      tot[k] += c[k]
    if len(ins) >= minn:
      print("%-14s n=%4d v=%4d s=%3d ds=%3d vm=%2d wide=%3d | %s" % (
          name, len(ins), c["v"], c["s"], c["ds"], c["vm"], c["mad64"], " ; ".join(ins[:3])[:90]))
  print("TOTAL", tot)


if __name__ == "__main__":
  main()
