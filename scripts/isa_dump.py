"""Annotated ISA of one kernel from a -gline-tables-only .s file: every
instruction with the source line it comes from, in program order (static).

  python scripts/isa_dump.py kern_g.s <kernel-symbol> > dump.txt
"""
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
lines = open(path).read().splitlines()
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
    if m:
        files[int(m.group(1))] = m.group(3)
inside, cur = False, None
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
        cur = "%s:%s" % (files.get(int(m.group(1)), "?").split("/")[-1], m.group(2))
        continue
    if re.match(r"\s+(v|s|ds|global|buffer|scratch)_", l) or re.match(r"^\.LBB", l):
        print("%-24s %s" % (cur, l.strip()[:110]))
