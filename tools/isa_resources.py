"""Per k_render instantiation: VGPRs, SGPRs, spills (the compiler's resource remarks) and, from the
-S listing, the v_readlane / v_writelane sites and scratch accesses inside the render (segment)
loop — the outermost loop of the kernel — and inside its deepest hot loops.
    python tools/isa_resources.py LISTING.s [kres.txt]"""
import re
import sys
from collections import OrderedDict

txt = open(sys.argv[1]).read()
res = {}
if len(sys.argv) > 2:
    for line in open(sys.argv[2]):
        m = re.match(r"(k_render<\S+) (\{.*\})", line.strip())
        if m:
            res[m.group(1)] = eval(m.group(2))
names = [m.group(1) for m in re.finditer(r"^(_ZN8yart_dev8k_render\S+):[ \t]*;", txt, re.M)]
print(f"{'instantiation <MESH,BVH,STATS,DYN,EXT[,DEEP]>':48s} {'VGPR':>5s} {'VGPR-spill':>10s} {'SGPR-spill':>10s} "
      f"{'loop instrs':>11s} {'loop rd/wr-lane':>15s} {'loop scratch':>12s}")
for name in names:
    start = txt.index(name + ":")
    body = txt[start:txt.index(".Lfunc_end", start)].split("\n")
    depth1 = None
    stats = OrderedDict()
    cur = None
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
                cur = None
            continue
        if cur is None or not l.startswith("\t") or l.startswith("\t.") or l.startswith("\t;") or not l.strip():
            continue
        op = l.split()[0]
        s = stats.setdefault(cur, [0, 0, 0])
        s[0] += 1
        s[1] += op in ("v_readlane_b32", "v_writelane_b32")
        s[2] += op.startswith("scratch_")
    # the render loop: depth-1 loop with the most instructions, plus everything nested in it
    d1 = [k for k in stats if k[1] == 1]
    if not d1:
        continue
    top = max(d1, key=lambda k: stats[k][0])
    tot = [0, 0, 0]
    # nested loops of the render loop are every deeper loop (the kernel has one outer loop)
    for k, v in stats.items():
        if k[1] >= 1:
            for i in range(3):
                tot[i] += v[i]
    short = "k_render<" + ",".join("1" if b == "1" else "0" for b in re.findall(r"Lb(\d)E", name)) + ">"
    key = [k for k in res if k.startswith("k_render<") and
           "".join(re.findall(r"Lb(\d)E", k)) == "".join(re.findall(r"Lb(\d)E", name))]
    r = res.get(key[0], {}) if key else {}
    print(f"{short:48s} {r.get('VGPRs', '?'):>5s} {r.get('VGPRs Spill', '?'):>10s} {r.get('SGPRs Spill', '?'):>10s} "
          f"{tot[0]:11d} {tot[1]:15d} {tot[2]:12d}")
