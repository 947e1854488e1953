"""Static instruction mix of one k_render instantiation in a hipcc -S listing:
    python tools/asmstat.py file.s [template-args, default Lb0ELb0ELb0ELb1ELb0E (cornell, DYN)]"""
import sys

txt = open(sys.argv[1]).read()
name = "_ZN8yart_dev8k_renderI" + (sys.argv[2] if len(sys.argv) > 2 else "Lb0ELb0ELb0ELb1ELb0E") + "EEvNS_8DevSceneENS_10RenderArgsE"
i = txt.index(name + ": ")
j = txt.index(".Lfunc_end", i)
ins = [l.strip() for l in txt[i:j].split("\n") if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;")]
op = [l.split()[0] for l in ins if l]
cnt = lambda f: sum(1 for o in op if f(o))
print(f"instrs {len(op)}  scratch {cnt(lambda o: o.startswith('scratch_'))}  v_readlane {cnt(lambda o: 'readlane' in o)}  "
      f"v_writelane {cnt(lambda o: 'writelane' in o)}  ds_ {cnt(lambda o: o.startswith('ds_'))}  "
      f"v_div_scale {cnt(lambda o: o.startswith('v_div_scale'))}  v_rsq {cnt(lambda o: o.startswith('v_rsq'))}")
