"""Where a kernel's scratch (register spill) traffic sits: the loop nests of one function in a
hipcc -S listing, each with its instruction count, scratch stores / loads and the source lines its
code comes from, so a spill count can be weighed by how often its loop runs (VERDICT r03 item 1:
a static spill count is not the dynamic spill traffic).
    hipcc ... --cuda-device-only -S -o k.s csrc/kernels.hip
    python tools/spillmap.py k.s [mangled-name-substring, default the mesh DYN k_render]"""
import collections
import re
import sys

path = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "k_renderILb1ELb0ELb0ELb1ELb0E"
txt = open(path).read()
m = [x for x in re.finditer(r"^(_Z\S+):[ \t]*;", txt, re.M) if want in x.group(1)]
if not m:
    sys.exit(f"no function matching {want}")
start = m[0].end()
body = txt[start:txt.index(".Lfunc_end", start)].split("\n")
files = {int(k): v for k, v in re.findall(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', txt, re.M)}

loops = collections.OrderedDict()  # header -> stats
stack = []  # (header, depth)
cur = ("<top>", 0)
line = 0
for l in body:
    hm = re.match(r"^(\.LBB\d+_\d+):", l)
    if hm or l.startswith("; %bb."):
        lh = re.search(r"Loop Header: Depth=(\d+)", l)
        li = re.search(r"in Loop: Header=(\S+) Depth=(\d+)", l)
        if lh:
            cur = ((hm.group(1) if hm else l.split()[1]).lstrip("."), int(lh.group(1)))
        elif li:
            cur = (li.group(1).lstrip("."), int(li.group(2)))
        else:
            cur = ("<top>", 0)
        continue
    lm = re.match(r"^\s*\.loc\s+(\d+)\s+(\d+)", l)
    if lm:
        line = (int(lm.group(1)), int(lm.group(2)))
        continue
    if not l.startswith("\t") or l.startswith("\t.") or l.startswith("\t;") or not l.strip():
        continue
    op = l.split()[0]
    s = loops.setdefault(cur, {"n": 0, "st": 0, "ld": 0, "lanes": 0, "lines": collections.Counter()})
    s["n"] += 1
    s["st"] += op.startswith("scratch_store")
    s["ld"] += op.startswith("scratch_load")
    s["lanes"] += op in ("v_readlane_b32", "v_writelane_b32")
    if op.startswith("scratch_") and line:
        s["lines"][line] += 1
print(f"{'loop header':18s} depth  instrs  scr_st  scr_ld  rd/wrlane   spill sites (file:line x count)")
for (hdr, depth), s in loops.items():
    sites = ", ".join(f"{files.get(f, f).split('/')[-1]}:{ln}x{c}" for (f, ln), c in s["lines"].most_common(8))
    print(f"{hdr:18s} {depth:5d} {s['n']:7d} {s['st']:7d} {s['ld']:7d} {s['lanes']:9d}   {sites}")
