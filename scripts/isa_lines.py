"""Attribute the instructions of one kernel in a -gline-tables-only .s file
to source lines (the last .loc before each instruction). Static counts only:
where the copies / selects / spills of the hot loop come from.

  python scripts/isa_lines.py kern_g.s <kernel-symbol> [--only v_mov,v_cndmask]
"""
import collections
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
only = None
if "--only" in sys.argv:
    only = sys.argv[sys.argv.index("--only") + 1].split(",")
files = {}
lines = open(path).read().splitlines()
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
    if m:
        files[int(m.group(1))] = m.group(3)
inside = False
cur = ("?", 0)
per_line = collections.Counter()
per_line_ops = collections.defaultdict(collections.Counter)
for l in lines:
    if l.startswith(sym + ":"):
        inside = True
        continue
    if inside and l.startswith(".Lfunc_end"):
        break
    if not inside:
        continue
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        cur = (files.get(int(m.group(1)), "?"), int(m.group(2)))
        continue
    m = re.match(r"\s+([vs]_[a-z0-9_]+)", l)
    if not m:
        continue
    op = m.group(1)
    if not op.startswith("v_"):
        continue
    if only and not any(op.startswith(o) for o in only):
        continue
    per_line[cur] += 1
    per_line_ops[cur][op] += 1
src = {}
for (f, n), c in per_line.most_common(60):
    if f not in src:
        try:
            src[f] = open(f if f.startswith("/") else "petershirleyraytracer_amd/csrc/" + f).read().splitlines()
        except OSError:
            src[f] = []
    text = src[f][n - 1].strip() if 0 < n <= len(src[f]) else ""
    top = ", ".join(f"{o}x{k}" for o, k in per_line_ops[(f, n)].most_common(4))
    print(f"{c:4d} {f}:{n:<5d} {text[:70]:70s} | {top}")
print("total", sum(per_line.values()))
