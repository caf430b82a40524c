"""Instruction mix per kernel of a gfx950 .s file: python3 tools/isa_mix.py FILE [regex]."""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
for m in re.finditer(r"^(_Z\w+):\s*(?:;.*)?$", s, re.M):
    name = m.group(1)
    if not pat.search(name):
        continue
    body = s[m.end():s.find(".Lfunc_end", m.end())]
    ins = [l.split()[0] for l in body.splitlines()
           if l.strip() and not l.strip().startswith((".", ";")) and not l.strip().endswith(":")]
    c = collections.Counter(ins)
    tot = lambda p: sum(n for k, n in c.items() if k.startswith(p))
    vg = re.search(r"\.vgpr_count:\s+(\d+)", s[m.end():]) 
    print(f"{name[:70]:70s} n={len(ins)} valu={tot('v_')} sqrt={c['v_sqrt_f32_e32']+c['v_sqrt_f32_e64']} "
          f"div_scale={c['v_div_scale_f32']} fma={tot('v_fma_f32')} mul={tot('v_mul_f32')} "
          f"add={tot('v_add_f32')} ds={tot('ds_')} glob={tot('global_')} s={tot('s_')}")
