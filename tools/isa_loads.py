"""Global-load batching in a kernel's ISA (compile with -S -gline-tables-only for source lines):
for every s_waitcnt vmcnt(N) that retires loads issued since the previous wait (N < loads issued since
it: an 'immediate' wait -- the loads were not left in flight across other work), the count of such
loads and their source lines.  Runs of 1-2 loads per immediate wait point at serialized, conditional
loads.   python tools/isa_loads.py <file.s> <kernel-symbol-substring>"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
files = {}
for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s):
    files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
for m in re.finditer(r"^(_Z\S+):", s, re.M):
    name = m.group(1)
    if pat not in name:
        continue
    end = s.index(".Lfunc_end", m.end())
    loc, since, retired = None, [], collections.Counter()
    hist = collections.Counter()
    for l in s[m.end():end].split("\n"):
        t = l.strip()
        if t.startswith(".loc"):
            p = t.split()
            loc = f"{files.get(p[1], p[1])}:{p[2]}"
        elif t.startswith(("global_load", "buffer_load", "scratch_load")):
            since.append(loc)
        elif t.startswith("s_waitcnt") and "vmcnt" in t:
            n = int(re.search(r"vmcnt\((\d+)\)", t).group(1))
            if n < len(since):
                k = len(since) - n
                hist[k] += 1
                if k <= 2:
                    for lc in since[:k]:
                        retired[lc] += 1
                since = since[k:]
    print(name[:90], "immediate waits by loads retired", dict(sorted(hist.items())))
    print("   1-2-load waits at", retired.most_common(12))
